/*
 * kwok_encoder.h — native ingestion encoder (host C++, no GPU): informer objects as JSON
 * -> the kwk_hot rows, deletion column, value records and delta classes kwk_load / kwk_upsert
 * take (kwok_engine.h).  It replaces, per informer event, the reference's ToJSONStandard +
 * gojq runs of the Stage selectors and *From getters:
 *
 *   reference (Go)                                          replaced by
 *   ------------------------------------------------------  ------------------------------
 *   PodController.watchResources / preprocess               kwk_encode (one parse per object;
 *     pkg/kwok/controllers/pod_controller.go:196-254,412-478  feature queries as compiled
 *   expression.ToJSONStandard query.go:72-88                  step programs; Go ParseInt /
 *   Requirement.Matches selector.go:65-120                    ParseDuration / RFC3339 for the
 *   int64From / durationFrom .Get value_*_from.go:53-81       *From getters)
 *
 * The encoder is built from the stage compiler's spec (kwok_amd/host/encoder.py encoder_spec:
 * feature queries, literal / finalizer bits, value slots, known delta classes).  A Go host
 * passes the apiserver's JSON bytes as they arrive; threads encode disjoint ranges.
 */
#ifndef KWOK_ENCODER_H
#define KWOK_ENCODER_H

#include <stdint.h>

#include "kwok_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct kwk_encoder kwk_encoder;

/* cls of an object whose delta class the compiler has not registered: the host registers it
 * (and reloads the stage table) before the row is loaded; its fires then round-trip
 * (KWK_FIRED_DELTA_UNKNOWN) */
#define KWK_ENCODE_CLASS_UNKNOWN 0xFFFFFFFFu

/* message of the last failing call on handle h (per handle); h = NULL: the calling thread's
 * last message (create) */
const char* kwk_encoder_last_error(const kwk_encoder* h);
kwk_status kwk_encoder_create(const char* spec_json, kwk_encoder** out);
kwk_status kwk_encoder_destroy(kwk_encoder* enc);
/* objects i = buf[offsets[i], offsets[i+1]) (n + 1 offsets); rows as Ingest.columns gives them
 * (sched = ALIVE | MANAGED | DIRTY [| HASREC] | KWK_STAGE_NONE; cls 0xFFFF for an unknown class,
 * counted in *n_unknown_class); value records are interned across calls, in object order */
kwk_status kwk_encode(kwk_encoder* enc, uint32_t n, const char* buf, const uint64_t* offsets, uint32_t n_threads,
                      kwk_hot* hot, int64_t* deletion_s, uint32_t* rec_idx, uint16_t* cls, uint32_t* n_unknown_class);
/* classes_json: {class key: id} of classes the stage compiler registered after this encoder was
 * created (a class first seen at run time, KWK_ENCODE_CLASS_UNKNOWN): later kwk_encode calls give
 * their objects that id.  The record table is kept (ids already loaded stay valid); a known key
 * must keep its id */
kwk_status kwk_encoder_add_classes(kwk_encoder* enc, const char* classes_json);
/* the interned records so far: n_records x (slots) kwk_value, for kwk_load / kwk_set_records */
kwk_status kwk_encoder_records(kwk_encoder* enc, kwk_value* out, uint32_t cap, uint32_t* n_records);

/* expression.NewQuery + Query.Execute (pkg/utils/expression/query.go:33-69) of one jq query on one
 * JSON document (taken as ToJSONStandard would hand it over: no presence rewriting), with the
 * native jq subset the encoder runs for Stage selector keys and *From getters (kwok_amd/csrc/jqc.hpp:
 * paths, pipes, comma, `//`, and / or / not, comparisons, arithmetic, literals, [..], {..}, if, try,
 * assignments, length / has / keys / select / map / ... ).  out <- the outputs as a JSON array
 * (nulls dropped; gojq ints as integers, float64 numbers as gojq encodes them) or `null` for the nil
 * result of a runtime error; NUL-terminated, *n_out = its length (KWK_ECAP: cap too small).
 * KWK_EINVAL: the query is outside the subset (the message names the construct) — the Go host then
 * keeps the reference lifecycle for that resourceRef. */
kwk_status kwk_jq_eval(const char* query, const char* json, char* out, uint32_t cap, uint32_t* n_out);

#ifdef __cplusplus
}
#endif
#endif /* KWOK_ENCODER_H */
