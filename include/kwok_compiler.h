/*
 * kwok_compiler.h — native Stage compiler (host C++, no GPU): one resourceRef's Stage list ->
 * the device stage table, (class, stage) next-state deltas, harness masks and the specs of the
 * encoder (kwok_encoder.h) and patch renderer (kwok_patch.h).  It is the drop-in for the
 * reference's Lifecycle construction, called from Go through cgo:
 *
 *   reference (Go)                                              replaced by
 *   ----------------------------------------------------------  -----------------------------------
 *   lifecycle.NewLifecycle(stages)  pkg/utils/lifecycle/         kwk_compile_stages (+ kwk_program_
 *     lifecycle.go:33-46; NewStage :194-267 (selectors,            explore for the delta classes) ->
 *     gojq queries, weight / delay / jitter getters, next)         kwk_program_table / _deltas /
 *   expression.NewRequirement / NewQuery selector.go:37-57,        _harness -> kwk_load_stages
 *     query.go:33-45; conversion.go:395-425 (statusTemplate)     (kwok_engine.h)
 *   StagesManager rebuilding the Lifecycle when Stage CRs       a new kwk_compile_stages with the new
 *     change  pkg/kwok/controllers/stages_manager.go:72-122        list, then kwk_load_stages
 *   per-resourceRef grouping  pkg/kwok/cmd/root.go:152           one program per resourceRef
 *
 * The host's Python compiler (kwok_amd/host/compiler.py KindProgram) is its CPU cross-check: the
 * table, deltas, harness, encoder spec and patch spec are byte-equal on every shipped stage set
 * (tests/test_native_compiler.py).  Selector queries must be of the step form the encoder runs
 * (.a.b, .["k"], .[], select(.x == literal), joined by |): anything else is a compile error here.
 *
 * Threading: a program is used by one thread at a time; programs are independent.
 */
#ifndef KWOK_COMPILER_H
#define KWOK_COMPILER_H

#include <stdint.h>

#include "kwok_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct kwk_program kwk_program;

/* message of the last failing call on program p (per program); p = NULL: the calling thread's
 * last message (kwk_compile_stages) */
const char* kwk_program_last_error(const kwk_program* p);

/* stages_json: a JSON array of v1alpha1 Stage objects of ONE resourceRef, in the Lifecycle's
 * order (the order is explicit: CRD-backed lists are unordered in the reference); stages with a
 * nil selector are dropped (lifecycle.go:199-201).  options_json (may be NULL): {"harness":
 * {"terminal_query": ".status.phase", "terminal_values": ["Succeeded", "Failed"],
 * "deletion_query": ".metadata.deletionTimestamp"}} enables the bench / parity churn harness
 * (the defaults apply to missing keys; "harness": true takes all defaults). */
kwk_status kwk_compile_stages(const char* stages_json, const char* options_json, kwk_program** out);
kwk_status kwk_program_destroy(kwk_program* p);

/* Derive the (class, stage) deltas from representative objects (JSON bytes objs[offsets[i],
 * offsets[i+1]), n + 1 offsets): each new (class, feature bits) root is explored through every
 * stage that can fire (KindProgram.explore).  Re-callable: only new roots re-run it.  A stage whose
 * patch can leave the object unchanged gets a "patch already applied" feature bit. */
kwk_status kwk_program_explore(kwk_program* p, uint32_t n, const char* objs, const uint64_t* offsets);

/* the delta class of one object (JSON bytes); register != 0 adds an unknown class (its deltas are
 * KWK_DELTA_UNKNOWN until explored), else an unknown class gives *cls = 0xFFFFFFFF */
kwk_status kwk_program_class(kwk_program* p, const char* obj, uint64_t len, int32_t reg, uint32_t* cls);

/* the device stage table (version as given) */
kwk_status kwk_program_table(const kwk_program* p, uint32_t version, kwk_stage_table* out);
/* n_classes x n_stages kwk_delta, row-major by class; out = NULL queries the sizes */
kwk_status kwk_program_deltas(const kwk_program* p, kwk_delta* out, uint64_t cap, uint32_t* n_classes,
                              uint32_t* n_stages);
kwk_status kwk_program_harness(const kwk_program* p, kwk_harness* out);
/* number of value slots (kwk_engine_desc.value_slots is max(1, this)) */
kwk_status kwk_program_value_slots(const kwk_program* p, uint32_t* n);

/* JSON strings owned by the program, valid until the next call on it:
 *  - describe: {"stages", "bits", "features", "applied_bits", "finalizers", "finalizer_other_bit",
 *    "value_slots", "classes", "uses_deletion_column"} (KindProgram.describe());
 *  - class keys: {class key: id} in registration order;
 *  - encoder spec: the spec kwk_encoder_create takes (kwok_amd/host/encoder.py encoder_spec; a
 *    program with "patch already applied" bits adds {"applied": [{"bit", "patches"}]}, which the
 *    native encoder evaluates with its template renderer — the host's encoder_spec rejects those);
 *  - patch spec: funcs_json = [{"name": ..., "const": "..."} | {"name": ..., "callback": true}] (the
 *    controller's template functions, kwk_patch_fn ids in name order) -> the spec
 *    kwk_patcher_create takes; *template_of (n_stages x KWK_MAX_PATCHES int32, -1 = the patch is
 *    not compiled: render it on the host) maps (stage, patch) to template ids. */
#define KWK_MAX_PATCHES 8
kwk_status kwk_program_describe(kwk_program* p, const char** json);
kwk_status kwk_program_class_keys(kwk_program* p, const char** json);
kwk_status kwk_program_encoder_spec(kwk_program* p, const char** json);
kwk_status kwk_program_patch_spec(kwk_program* p, const char* funcs_json, const char* version, const char** json,
                                  int32_t* template_of, uint32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* KWOK_COMPILER_H */
