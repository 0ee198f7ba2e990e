/* Device patch emission: the merge-patch bytes of fired objects written by the GPU
 * (the device form of kwok_patch.h).
 *
 * Replaces, per fired object, the reference's Next.Patches → computeMergePatch →
 * gotpl.Renderer.ToJSON round trip (pkg/utils/lifecycle/next.go:73-160,
 * pkg/utils/gotpl/renderer.go:59-124) for the templates whose bytes are fixed by the object's
 * class up to Now and the values of the controller's functions: the host builds each
 * (class, template) skeleton once with kwk_patch_skeleton (literal runs + slots), checks every
 * object once with kwk_patch_object_values (its render equals the skeleton; its call values,
 * e.g. funcPodIPWith / funcNodeIPWith of pod_controller.go:563-600, are fixed for the object's
 * life) and uploads per-slot words and value columns.  Each step, kwk_emit expands the engine's
 * fired list into the patches on the device: byte-equal to kwk_patch_render of the same object,
 * or KWK_EMIT_HOST for the items the host renders itself (ineligible template, object not
 * accepted, status guard not met, unusable value).
 *
 * Status guards: the Stages' `index $root.status.<list> $i` inside `range $i := <spec list>`
 * fails the render when the status list is shorter than the spec list.  Guard bit k of a slot's
 * word says the guard holds for the object's current status; the host sets it at ingest, the
 * emitter keeps it through every record it emits (a template's patch leaves it, or sets it to
 * the value its status list gives), an emitted delete resets it to the class's fresh value (the
 * harness re-creates from spec).  A record with an item left to the host keeps its word: the host
 * sets it (kwk_emit_set_words) once it has rendered and applied that object's patches, as it
 * does after any kwk_replace / kwk_upsert.
 */
#ifndef KWOK_EMIT_H
#define KWOK_EMIT_H

#include <stdint.h>

#include "kwok_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct kwk_emitter kwk_emitter;

#define KWK_EMIT_NO_SLOT 0xFFFFu
/* a literal run of the skeleton followed by a slot: KWK_EMIT_NO_SLOT, 0 = Now (RFC3339Nano, UTC),
 * 1 + c = value column c */
typedef struct {
  uint32_t lit_off;
  uint16_t lit_len;
  uint16_t slot;
} kwk_emit_piece;

typedef struct {
  uint32_t first_piece, n_pieces;
  uint8_t need;  /* guard bits the template's render requires */
  uint8_t keep;  /* guard bits its patch leaves as they are ... */
  uint8_t set;   /* ... and the values of the others after it */
  uint8_t reserved;
} kwk_emit_skel;

typedef struct {
  uint32_t n_classes, n_templates, n_stages, n_skels, n_pieces, n_columns;
  uint64_t n_lit_bytes;
  const uint32_t* stage_tpl_ptr;  /* n_stages + 1: stage s's templates are stage_tpl[ptr[s] .. ptr[s + 1]) */
  const uint16_t* stage_tpl;      /* template ids (< 32) in patch order */
  const uint8_t* stage_delete;    /* n_stages: the stage deletes the object (KWK_NEXT_DELETE) */
  const int32_t* skel_of;         /* n_classes * n_templates: skeleton index, -1 = the host renders */
  const kwk_emit_skel* skels;
  const kwk_emit_piece* pieces;
  const char* lits;
  const uint8_t* fresh_guards;    /* n_classes: guard bits of an object created from its spec */
  const uint32_t* column_stride;  /* n_columns: bytes per slot, a multiple of 4 in 4..256: [length][text]
                                   (length 0xFF = unusable) */
} kwk_emit_program;

/* per slot: bits 0-15 class, 16-23 guard bits, 32-63 template accepted (bit tid); bits 24-31 are
 * reserved (the device caches the slot's value lengths there: kwk_emit_get_words returns them 0) */
#define KWK_EMIT_WORD(cls, guards, accepted) \
  ((uint64_t)(uint16_t)(cls) | (uint64_t)(uint8_t)(guards) << 16 | (uint64_t)(uint32_t)(accepted) << 32)

#define KWK_EMIT_OK 0
#define KWK_EMIT_HOST 1 /* render this item with kwk_patch_render / the host renderer */
typedef struct {
  uint32_t rec;     /* index in the fired list */
  uint16_t tid;     /* template id */
  uint8_t status;   /* KWK_EMIT_* */
  uint8_t reserved;
} kwk_emit_item;

#define KWK_EMIT_FROM_RECORDS 0u /* kwk_fired_device's list (kwk_fired_compact) */
#define KWK_EMIT_FROM_PACKED 1u  /* kwk_fired_packed_device's list (kwk_fired_compact_packed) */
/* (round 5: the wave-per-record writers selected by bits 8 / 9 are retired — measured slower than
 * the lane-per-record writer; any other bit of source is KWK_EINVAL) */

const char* kwk_emit_last_error(const kwk_emitter* em);
/* an emitter for `eng`'s fired lists over slots [0, capacity), on the engine's stream */
kwk_status kwk_emitter_create(kwk_engine* eng, uint32_t capacity, const kwk_emit_program* prog, kwk_emitter** out);
kwk_status kwk_emitter_destroy(kwk_emitter* em);
kwk_status kwk_emit_set_words(kwk_emitter* em, uint32_t first, uint32_t n, const uint64_t* words);
kwk_status kwk_emit_get_words(kwk_emitter* em, uint32_t first, uint32_t n, uint64_t* words);
/* rows [first, first + n) of value column c: n * column_stride[c] bytes */
kwk_status kwk_emit_set_column(kwk_emitter* em, uint32_t c, uint32_t first, uint32_t n, const uint8_t* data);
/* output room: items and patch bytes one kwk_emit may produce */
kwk_status kwk_emit_reserve(kwk_emitter* em, uint32_t max_items, uint64_t max_bytes);
/* enqueue the emission of the engine's last compacted fired list (source: KWK_EMIT_FROM_*) */
kwk_status kwk_emit(kwk_emitter* em, int64_t now_ns, uint32_t source);
/* synchronise; the last emission's totals.  KWK_ECAP when they exceed the reservation: nothing was
 * written (words unchanged) — reserve more and emit the same list again */
kwk_status kwk_emit_result(kwk_emitter* em, uint32_t* n_items, uint64_t* n_bytes);
/* kwk_emit_result plus the number of items emitted on the device (status KWK_EMIT_OK) */
kwk_status kwk_emit_stats(kwk_emitter* em, uint32_t* n_items, uint32_t* n_emitted, uint64_t* n_bytes);
/* device outputs of the last emission: items, n_items + 1 byte offsets, the bytes */
kwk_status kwk_emit_device(kwk_emitter* em, const kwk_emit_item** items, const uint64_t** offsets, const char** bytes);
/* copy them to host memory (sizes from kwk_emit_result; offsets holds n_items + 1 entries) */
kwk_status kwk_emit_copy(kwk_emitter* em, kwk_emit_item* items, uint64_t* offsets, char* bytes);
/* HIP events around the last kwk_emit's kernels (bench timing): milliseconds between them */
kwk_status kwk_emit_elapsed(kwk_emitter* em, float* ms);

#ifdef __cplusplus
}
#endif

#endif
