/* Native patch renderer: precompiled merge-patch byte templates for fired objects
 * (SURVEY.md §8(f) rank 2).
 *
 * Replaces, per fired object, the reference's Next.Patches → computeMergePatch →
 * gotpl.Renderer.ToJSON (text/template + sprig, sigs.k8s.io/yaml.YAMLToJSON) →
 * wrapMergePatchData round trip (pkg/utils/lifecycle/next.go:73-160,
 * pkg/utils/gotpl/renderer.go:59-124).  The host compiles each Stage patch template once
 * (kwok_amd/host/patchtpl.py: TemplateCompiler) into a byte program — the template's YAML
 * structure resolved, mapping keys in encoding/json's sorted order, literals as their final
 * JSON bytes — and this library fills the slots from each object's JSON.
 *
 * A Go host binds it next to kwok_engine.h: after kwk_fired, it renders the
 * patches of the fired objects in one call and sends them; objects whose status is
 * KWK_PATCH_NEEDS_RENDER go through the existing gotpl renderer.
 */
#ifndef KWOK_PATCH_H
#define KWOK_PATCH_H

#include <stdint.h>

#include "kwok_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct kwk_patcher kwk_patcher;

#define KWK_PATCH_OK 0
/* the byte program cannot place a value exactly (a printed value YAML would re-type, a
 * character YAML treats specially) or the template's execution fails: render this object
 * with the host renderer (which also reports the reference's error) */
#define KWK_PATCH_NEEDS_RENDER 1

/* value kinds passed to caller functions */
#define KWK_PATCH_ARG_MISSING 0
#define KWK_PATCH_ARG_NIL 1
#define KWK_PATCH_ARG_BOOL 2
#define KWK_PATCH_ARG_NUM 3
#define KWK_PATCH_ARG_STR 4
#define KWK_PATCH_ARG_ARR 5
#define KWK_PATCH_ARG_OBJ 6

/* A template function provided by the controller (NodeIPWith, PodIPWith, ...;
 * pod_controller.go:563-600): argv[i] / argl[i] is argument i printed (fmt.Sprint; arrays and
 * objects as JSON), kinds[i] its KWK_PATCH_ARG_* kind.  Writes the result string into
 * out[0..cap) and its length into *out_len; returns 0, or 2 when cap is too small (the
 * renderer calls again with *out_len bytes), anything else = the function failed (the
 * object gets KWK_PATCH_NEEDS_RENDER).  Called from the rendering threads. */
typedef int32_t (*kwk_patch_fn)(void* user, uint32_t func_id, uint32_t argc, const char* const* argv,
                                const uint32_t* argl, const uint8_t* kinds, char* out, uint32_t cap,
                                uint32_t* out_len);

/* message of the last failing call on handle h (per handle); h = NULL: the calling thread's
 * last message (create) */
const char* kwk_patch_last_error(const kwk_patcher* h);

/* spec_json: {"templates": [...], "funcs": [{"name", "const" | "callback"}], "consts": [...]}
 * as written by kwok_amd/host/patchtpl.py:PatchProgram */
kwk_status kwk_patcher_create(const char* spec_json, kwk_patcher** out);
kwk_status kwk_patcher_destroy(kwk_patcher* p);

/* Render the patches of n objects: object i (JSON bytes objs[obj_offsets[i] ..
 * obj_offsets[i+1])) with template template_ids[i], Now() = now_ns (RFC3339Nano, UTC).
 * *out_data receives a buffer owned by the patcher (valid until the next render / destroy)
 * holding patch i at [out_offsets[i], out_offsets[i+1]) (empty when status[i] != OK).
 * n_threads > 1 renders disjoint ranges in parallel; one render at a time per patcher. */
kwk_status kwk_patch_render(kwk_patcher* p, uint32_t n, const uint16_t* template_ids, const char* objs,
                            const uint64_t* obj_offsets, int64_t now_ns, kwk_patch_fn fn, void* user,
                            uint32_t n_threads, const char** out_data, uint64_t* out_offsets, uint8_t* status);

/* ---- skeletons for device emission (kwok_emit.h)
 *
 * The skeleton of template `tid` over an object class: the template rendered over the class's
 * representative `obj` with every per-object input kept out — the object's status and identity
 * (what the compiler's class key drops: status, metadata identity keys and ownerReferences,
 * spec.nodeName / hostname) are not read, Now and each call of a callback function become slots.
 * Eligible only when those inputs reach the patch solely as slot text, as call arguments
 * (identity, not status: a call's value is fixed per object) or through the Stages' status guard
 * `index $root.status.<list> $i` in `range $i, ... := <class-level list>` (its one effect is the
 * error when the status list is shorter; the device checks a per-object bit instead).
 * *out_json (owned by the patcher until its next skeleton call):
 *   {"eligible": true, "text": <the patch with slot markers>, "lits": [n_slots + 1 literal runs],
 *    "slots": [slot ids: 0 = Now, 1 + c = call site c], "calls": n_call_sites,
 *    "guards": [[<status list path>, <range list path>], ...]}
 *   or {"eligible": false, "reason": "..."}.
 * Objects of the class render (kwk_patch_render) to the literal runs with the slots filled in —
 * Now as RFC3339Nano, call c as its value — when kwk_patch_object_values accepts them. */
kwk_status kwk_patch_skeleton(kwk_patcher* p, uint32_t tid, const char* obj, uint64_t len, const char** out_json,
                              uint64_t* out_len);

/* Per object i (the objects of one class): renders template tid in skeleton mode with the call
 * sites evaluated for real (fn), ok[i] = 1 when the result equals `skeleton` (the class's "text")
 * and every call value fits stride - 1 bytes of characters JSON and YAML carry unchanged
 * (printable ASCII without " \ ' < > &).  values[(i * n_calls + c) * stride] = [length][bytes] of
 * call site c (length 0xFF: unusable). */
kwk_status kwk_patch_object_values(kwk_patcher* p, uint32_t tid, uint32_t n, const char* objs, const uint64_t* obj_offsets,
                                   const char* skeleton, uint64_t skeleton_len, kwk_patch_fn fn, void* user,
                                   uint32_t n_threads, uint32_t n_calls, uint32_t stride, uint8_t* values, uint8_t* ok);

#ifdef __cplusplus
}
#endif

#endif
