/*
 * kwok_engine.h — C ABI of the MI355X Stage-lifecycle engine.
 *
 * This is the device boundary a Go host binds through cgo.  It replaces,
 * for one resource kind, the per-object work the reference does between the informer event
 * and the client-go PATCH:
 *
 *   reference seam (Go)                                   replaced by
 *   ----------------------------------------------------  --------------------------------
 *   lifecycle.NewLifecycle / NewStage                     kwk_load_stages (host-compiled
 *     pkg/utils/lifecycle/lifecycle.go:33-46,194-267        table; explicit stage order)
 *   PodController.preprocess -> Lifecycle.Match,          kwk_step (fused sweep kernel:
 *     Stage.Delay, addStageJob                              match, weighted pick, delay +
 *     pkg/kwok/controllers/pod_controller.go:196-254        jitter, schedule, fire, delta)
 *     pkg/utils/lifecycle/lifecycle.go:125-191,313-341
 *     pkg/utils/queue/weight_delaying_queue.go:73-174
 *   (node: node_controller.go:262-319; generic: stage_controller.go:174-232)
 *   playStage's state change (finalizers, delete,         applied on device as delta ops;
 *     patches) pod_controller.go:290-360,                   the fired list (kwk_fired) is
 *     pkg/utils/lifecycle/next.go:43-88,                    what Go renders text patches for
 *     pkg/utils/lifecycle/finalizers.go:83-111
 *   informer Added/Modified events -> preprocessChan      kwk_load / kwk_upsert (pre-interned
 *     pod_controller.go:412-478                             SoA columns; marks objects dirty)
 *   Deleted events                                        kwk_delete
 *   server/metrics_resource_usage.go:170-224              kwk_usage (per-node segmented sums)
 *     (podResourceUsage / nodeResourceUsage and the
 *      *CumulativeUsage integrators :36-109)
 *
 * Conventions: every function returns kwk_status (0 = ok, < 0 = error; message via
 * kwk_last_error(eng), kept per engine).  No exceptions or panics cross the boundary.  Strings never cross it:
 * the host interns labels / annotations / phases / finalizers into feature bits and
 * pre-parses *From values.  All calls for one engine come from one thread (the reference
 * runs all matching for a kind on a single preprocess goroutine, pod_controller.go:150).
 * kwk_step and kwk_usage only enqueue work on the engine's HIP stream; the read functions
 * synchronise that stream.
 */
#ifndef KWOK_ENGINE_H
#define KWOK_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t kwk_status;
#define KWK_OK 0
#define KWK_EINVAL (-1)   /* bad argument / shape mismatch */
#define KWK_ECAP (-2)     /* capacity exceeded */
#define KWK_EHIP (-3)     /* HIP runtime error */
#define KWK_ESTATE (-4)   /* call order (e.g. step before load_stages) */

typedef struct kwk_engine kwk_engine;

/* ------------------------------------------------------------------ object hot record */
/* sched word layout */
#define KWK_STAGE_NONE 0xFFu          /* bits 0..7: pending stage index */
#define KWK_F_ALIVE (1u << 8)         /* object exists */
#define KWK_F_DIRTY (1u << 9)         /* changed since last match: re-match this step */
#define KWK_F_MANAGED (1u << 10)      /* pod on a managed node / node managed by this kwok */
#define KWK_F_HASREC (1u << 11)       /* has a value record (pre-parsed *From results) */
#define KWK_F_MATCHERR (1u << 12)     /* last match hit a Go panic path (Int63n(<0)) */
#define KWK_CLASS_SHIFT 16            /* bits 16..31: the object's delta class (spec shape) */
#define KWK_CLASS_MASK 0xFFFF0000u

/* Interchange row for loads / upserts / reads.  On the device the row is split:
 * an 8-byte {pred, sched} state stream that every step reads, and a due column read only
 * for objects with a pending stage.  due is meaningful only while a stage is pending. */
typedef struct {
  uint32_t pred;   /* feature bits (host-compiled predicate summary) */
  uint32_t sched;  /* pending stage | flags | delta class */
  int64_t due;     /* unix ns at which the pending stage fires */
} kwk_hot;         /* 16 bytes */

/* value record entry (one per value slot of a record) */
#define KWK_V_DEFAULT 0  /* query produced no output: use the stage's default value */
#define KWK_V_OK 1       /* value = int64 (weight) or duration ns */
#define KWK_V_NOTOK 2    /* getter returns (0, false) */
#define KWK_V_ABSTIME 3  /* RFC3339 time: value = unix seconds, nsec = nanoseconds; result = t - now */
typedef struct {
  int64_t value;
  int32_t nsec;
  int32_t kind;
} kwk_value; /* 16 bytes */

#define KWK_DEL_ABSENT INT64_MIN   /* deletion_s column: no deletionTimestamp */

/* ------------------------------------------------------------------ stage table */
#define KWK_MAX_STAGES 32
#define KWK_MAX_ANY 4
#define KWK_SLOT_NONE (-1)         /* getter has no *From query: constant default */
#define KWK_SLOT_DELETION (-2)     /* duration getter on .metadata.deletionTimestamp (column) */

#define KWK_NEXT_DELETE (1u << 0)
#define KWK_NEXT_IMMEDIATE (1u << 1)
#define KWK_NEXT_PATCHES (1u << 2)     /* has rendered patches */
#define KWK_NEXT_FIN (1u << 3)         /* has a finalizers op */
#define KWK_NEXT_FIN_EMPTY (1u << 4)   /* finalizers.empty */
#define KWK_NEXT_FIN_REMOVE (1u << 5)  /* finalizers.remove non-empty */
#define KWK_NEXT_PATCH_STATIC (1u << 6) /* patches do not depend on Now: re-applying them to an object
                                         * whose `applied_mask` bit is set changes nothing, so (as in
                                         * the reference: no watch event) the object is not re-matched */

typedef struct {
  /* selector: ((pred ^ eq_val) & eq_mask) == 0  AND  for k < n_any:
   *           ((pred & any_mask[k]) != 0) == ((any_want >> k) & 1) */
  uint32_t eq_mask, eq_val;
  uint32_t n_any, any_want;
  uint32_t any_mask[KWK_MAX_ANY];
  /* weight getter: IntFrom(&Spec.Weight, weightFrom) — always has a default */
  int64_t weight_default;
  int32_t weight_slot;
  /* delay getters (Stage.Delay) */
  int32_t has_delay;
  int64_t delay_default;       /* durationMilliseconds (or 0) in ns; always ok when has_delay */
  int32_t delay_slot;
  int32_t has_jitter;
  int64_t jitter_default;
  int32_t jitter_default_ok;   /* jitterDurationMilliseconds present */
  int32_t jitter_slot;
  /* next */
  uint32_t flags;              /* KWK_NEXT_* */
  uint32_t fin_add, fin_remove;/* bits inside the table's fin_group_mask */
  uint32_t applied_mask;       /* KWK_NEXT_PATCH_STATIC: feature bit "patch already applied" */
} kwk_stage_desc;

typedef struct {
  uint32_t n_stages;
  uint32_t fin_group_mask;     /* pred bits forming the object's finalizer set */
  uint32_t n_classes;          /* delta table is [n_classes][n_stages] */
  uint32_t version;
  uint32_t pred_bits;          /* feature bits in use: pred < 2^pred_bits (0 = all 32).  With the class
                                * and stage counts this picks the device state format */
  uint32_t disregard_mask;     /* need() (pod_controller.go:392-409, node_controller.go:153-166): a changed
                                * object with a pred bit in this mask is not re-matched (its watch event
                                * is skipped: disregardStatusWith{Annotation,Label}Selector); a queued
                                * stage stays queued.  0 = no disregard selectors */
  uint32_t reserved[2];
  kwk_stage_desc stages[KWK_MAX_STAGES];
} kwk_stage_table;

typedef struct {               /* next-state delta of (object class, stage) */
  uint32_t and_mask, or_mask;  /* pred' = (pred & and_mask) | or_mask (outside fin group) */
} kwk_delta;
#define KWK_DELTA_UNKNOWN_AND 0u  /* and_mask 0 with or_mask 0xFFFFFFFF: not derivable -> host */
#define KWK_DELTA_UNKNOWN_OR 0xFFFFFFFFu

/* ------------------------------------------------------------------ workload harness */
/* Optional device-side churn (simulates the user/apiserver side of a steady-state
 * cluster; bench and parity tests only):
 *   dead object            -> re-created: pred = pred & keep_mask, gen+1, dirty
 *   alive, (pred & terminal_mask) != 0, deletion bit clear
 *                          -> deletionTimestamp = now (second precision), dirty      */
typedef struct {
  uint32_t enable;
  uint32_t keep_mask;
  uint32_t terminal_mask;
  uint32_t deletion_bit;
  uint32_t track_deletion;     /* maintain the deletion_s column (only if a stage reads it) */
  uint32_t reserved[3];
} kwk_harness;

/* ------------------------------------------------------------------ fired records */
#define KWK_FIRED_DELETED (1u << 0)
#define KWK_FIRED_REMATCH (1u << 1)
#define KWK_FIRED_DELTA_UNKNOWN (1u << 2)
typedef struct {
  uint32_t slot;   /* local object slot */
  uint16_t stage;  /* stage index in the loaded table */
  uint16_t flags;  /* KWK_FIRED_* */
} kwk_fired_rec;

typedef struct {
  uint64_t steps;
  uint64_t matched;       /* objects (re)scheduled by a match */
  uint64_t fired;         /* stage transitions */
  uint64_t bytes;         /* algorithmic bytes moved by the sweep */
  uint64_t fired_per_stage[KWK_MAX_STAGES];
  uint64_t state_bytes;   /* bytes per object of the device state stream: 1 (dictionary id), 2 or 4 (packed),
                           * 8 (wide, or a packed word fused with its relative due time) */
  uint64_t line_bytes;    /* `bytes` with state writes counted as the whole 128-byte lines the 2-byte
                           * sweep stores (= bytes for the word-granular 4/8-byte sweeps) */
} kwk_step_stats;

/* ------------------------------------------------------------------ engine */
typedef struct {
  int32_t device;             /* HIP device ordinal */
  uint32_t capacity;          /* object slots */
  uint32_t value_slots;       /* kwk_value entries per value record */
  uint32_t max_records;       /* value records */
  uint64_t slot_base;         /* global id of local slot 0 (RNG counter; shard invariant) */
  uint32_t kind_salt;         /* mixed into the RNG key: separate streams per kind */
  uint32_t flags;             /* KWK_ENGINE_* */
} kwk_engine_desc;
#define KWK_ENGINE_WIDE_STATE (1u << 0) /* always use the 8-byte state format (never a packed one) */
#define KWK_ENGINE_STATE32 (1u << 1)    /* never the 2-byte packed format (4-byte packed or wide only) */
#define KWK_ENGINE_STATE16 (1u << 2)    /* never the 1-byte dictionary format (2-byte words at most narrow) */
#define KWK_ENGINE_SPLIT_DUE (1u << 3)  /* never the fused 8-byte record {packed word, relative due}: 4-byte
                                         * words and the separate 8-byte due column */

/* message of the last failing call on `eng` (kept per engine, so a caller that moves between OS
 * threads between the failing call and this one — a Go goroutine — still reads its own message);
 * eng = NULL: the calling thread's last message (kwk_engine_create, kwk_alloc_host / free_host) */
const char* kwk_last_error(const kwk_engine* eng);
kwk_status kwk_engine_create(const kwk_engine_desc* desc, kwk_engine** out);
kwk_status kwk_engine_destroy(kwk_engine* eng);

/* Explicit kernel choices (defaults = the measured best; tests use them to check
 * that every kernel shape gives the same results).  Nothing is read from the environment. */
/* 1, 2, 3, 5 (round 6: merged into KWK_TUNE_SWEEP16), 4, 7, 12 (round 5: experiment knobs; tools/variants.py
 * patches the constants for such measurements), 6, 13 (round 6: merged into KWK_TUNE_USAGE), 11 (the
 * one-pass look-back hand-back, measured slower: 73 vs 27 us at C5), 16 (round 6: the folded hand-back,
 * superseded by fused steps): retired */
#define KWK_TUNE_SWEEP16 18   /* the table-driven sweeps' shape, KWK_SWEEP16_SHAPE(q, persistent, kernel, table):
                                 q = 16-byte chunks per lane of the 2-byte sweep (4 default, 2 or 1), persistent = a
                                 persistent grid for large engines (1 default), kernel = the table-only kernel with 2
                                 (default) or 1 tiles prefetched (the 2-byte and the 1-byte sweeps), or 0 = the general
                                 sweep16_kernel; table = the precomputed transition table (1 default) or 0 */
#define KWK_SWEEP16_SHAPE(q, persistent, kernel, table) \
  ((uint32_t)(q) | (uint32_t)(persistent) << 4 | (uint32_t)(kernel) << 8 | (uint32_t)(table) << 12)
#define KWK_SWEEP16_DEFAULT KWK_SWEEP16_SHAPE(4, 1, 2, 1)
#define KWK_TUNE_USAGE 19     /* the usage path: KWK_USAGE_KEY8 (the 1-byte usage-key column when at most 256
                                 distinct keys occur) | KWK_USAGE_AGG_FUSED (kwk_aggregate with KWK_AGG_USAGE on 1-byte
                                 ids: the <= 4 mask counts inside the usage kernel's pass); default both */
#define KWK_USAGE_KEY8 1u
#define KWK_USAGE_AGG_FUSED 2u
#define KWK_TUNE_COMPACT_SMALL 8 /* fired hand-back: the most segments compacted in one launch (each block sums
                                   the counts before its own), 0..8192 (default 8192); more use the scan +
                                   expansion pair; 0 = always the pair */
#define KWK_TUNE_TAIL_HANDBACK 20 /* kwk_step_n / _pair / kwk_tick on 2-byte table-only engines swept one tile per
                                     workgroup (node kinds, the strong-scaling shards' node engines), at most a
                                     quarter as many workgroups as the device has CUs: 1 (default) = the sweep writes the step's
                                     list itself (each workgroup adds the counts of the ones before it, then copies
                                     its records: no compaction launch), 0 = a compaction launch after the sweep.
                                     The lists are identical */
#define KWK_TUNE_BYTE_STATE 9 /* the 1-byte dictionary format for table-only programs, 1 (default) or 0 (the
                                 2-byte words): DESIGN.md §3 */
#define KWK_TUNE_STREAM_PRIORITY 15 /* the engine's stream: 0 (default priority), 1 (the device's greatest) or 2 (its
                                       least); re-created after a synchronise, so set it between steps */
#define KWK_TUNE_WORD_TILES 10 /* word sweep (4-byte, fused and wide formats): tiles per workgroup, 1..16
                                  (exactly), or 0 (default: 8 fused, 4 otherwise, but at least 5 workgroups
                                  per CU) */
#define KWK_TUNE_FUSE_STEPS 17 /* kwk_step_n / _pair on 1-byte engines with <= 4 stages and no delayed stage: up to
                                  4 (default) or 2 steps per sweep launch (each id read once, stepped in LDS,
                                  written once; each step's fired records and hand-back kept apart), or 0 / 1 (one step
                                  per launch).  Results are bit-identical; kwk_step_stats.bytes / line_bytes count
                                  the fused launch's own reads and writes */
kwk_status kwk_set_tuning(kwk_engine* eng, uint32_t key, uint32_t value);

/* stage table + per-(class, stage) deltas; replaces the previous table (version bump) */
kwk_status kwk_load_stages(kwk_engine* eng, const kwk_stage_table* table, const kwk_delta* deltas);
kwk_status kwk_set_harness(kwk_engine* eng, const kwk_harness* h);

/* bulk column load of slots [0, n) from host arrays (initial list / informer Sync);
 * cls[i] is stored in the upper half of hot[i].sched */
kwk_status kwk_load(kwk_engine* eng, uint32_t n, const kwk_hot* hot, const int64_t* deletion_s,
                    const uint32_t* rec_idx, const uint16_t* cls, uint32_t n_records, const kwk_value* records);
/* per-object upsert (Added / Modified events): scatter into the given slots, marks dirty */
kwk_status kwk_upsert(kwk_engine* eng, uint32_t n, const uint32_t* slots, const kwk_hot* hot,
                      const int64_t* deletion_s, const uint32_t* rec_idx, const uint16_t* cls);
/* the same scatter with the rows taken as given (DIRTY only if the row carries it): the host's
 * re-encoded object after a fire whose next state the device could not derive
 * (KWK_FIRED_DELTA_UNKNOWN) — the watch event the reference would receive
 * (pod_controller.go:336-351, 412-478) re-matches it only if the object changed */
kwk_status kwk_replace(kwk_engine* eng, uint32_t n, const uint32_t* slots, const kwk_hot* hot, const int64_t* deletion_s,
                       const uint32_t* rec_idx, const uint16_t* cls);
kwk_status kwk_set_records(kwk_engine* eng, uint32_t first, uint32_t n, const kwk_value* records);
/* Deleted events: clear ALIVE (cancels any pending stage) */
kwk_status kwk_delete(kwk_engine* eng, uint32_t n, const uint32_t* slots);

/* Failed playStage with a retryable error (shouldRetry, pkg/kwok/controllers/utils.go:146-160):
 * the object did not change in the apiserver, so the device state the fire produced is replaced
 * by the host's unchanged row (`hot`, `cls`: what kwk_upsert would take, without a re-match) and
 * the same stage is queued again after backoffDelayByStep(retry_count, backoff)
 * (utils.go:138-143: min(duration * factor^steps, cap), then wait.Jitter(d, jitter) with
 * rand.Float64 from the Philox hook, site 4), as playStageWorker does
 * (pod_controller.go:257-285, node_controller.go / stage_controller.go alike; the retry's
 * queue weight 1 only orders jobs due at the same instant, which one device step fires
 * together).  retry_count[j] = the job's RetryCount before the increment (0 on the first
 * retry).  Go's math.Pow is restated for integer exponents (exact). */
typedef struct {
  int64_t duration_ns;   /* wait.Backoff.Duration (defaultBackoff, utils.go:133-135: 1 s) */
  double factor;         /* Factor (2.0) */
  double jitter;         /* Jitter (0.2; <= 0 means 1.0, as wait.Jitter) */
  int64_t cap_ns;        /* Cap (32 min) */
} kwk_backoff;
kwk_status kwk_retry(kwk_engine* eng, int64_t now_ns, uint64_t seed, uint64_t step, uint32_t n, const uint32_t* slots,
                     const kwk_hot* hot, const uint16_t* cls, const uint16_t* stages, const uint32_t* retry_count,
                     const kwk_backoff* backoff);

/* one reconciliation step at time now_ns over slots [0, n_active):
 * harness -> match dirty objects -> fire due objects -> apply deltas.
 * Random draws use Philox4x32-10(key = seed ^ ((uint64_t)kind_salt << 32),
 * ctr = (slot_base+slot, step lo, step hi, site)).  Enqueue only. */
kwk_status kwk_step(kwk_engine* eng, int64_t now_ns, uint64_t seed, uint64_t step);

/* match only: Lifecycle.Match + Stage.Delay for the dirty objects (lifecycle.go:125-191,
 * 313-341) without firing anything and without harness churn; the picked stage and its due
 * time are then readable with kwk_read (the reference-interface mirror's Match). */
kwk_status kwk_match(kwk_engine* eng, int64_t now_ns, uint64_t seed, uint64_t step);

/* Fired hand-back (the objects Go renders patches for, pod_controller.go:290-360).  The sweep
 * leaves per-(tile, wave) segments; kwk_fired_compact enqueues their scan + compaction into one
 * dense device list (enqueue only: call it after kwk_step to keep the list on the device, e.g.
 * for an in-process consumer through kwk_fired_device).  kwk_fired copies the LAST step's list
 * (compacting first if needed) into host memory — a kwk_alloc_host buffer makes the copy a
 * direct DMA — and synchronises.  Records are grouped by sweep region (ascending regions: a
 * wave's 512-2048 slots in the 2-byte sweeps, a tile's 2048 / 4096 slots in the 8- / 4-byte word
 * sweep), unordered within a region; each fired slot appears once.  A step that swept nothing
 * (no active slots) leaves an empty list.
 * Every compaction writes a list of its own in a ring of device lists tagged with the step it
 * compacted (DESIGN.md §5 "Hand-back"): the last one is the engine's list the readers below
 * return, and the lists of the last kwk_fired_keep() compactions stay readable by step number
 * through kwk_fired_fetch_step — every step of a kwk_step_n / _pair call, fused or not. */
kwk_status kwk_fired_compact(kwk_engine* eng);
/* n steps (now0 + k * dt, step0 + k for k < n), each with its hand-back in the given format when
 * compact != 0 (enqueue only): the per-tick loop of kwk_step / kwk_fired_compact in one call.
 * On 1-byte engines with <= 4 stages and no delayed stage (KWK_TUNE_FUSE_STEPS) the steps are swept
 * in launches of up to 4 steps (each id read and written once per launch) and the launch's
 * hand-backs run as one launch: results are those of the per-step calls, and every step's list is
 * compacted into its own ring slot (tag step0 + k), so kwk_fired_fetch_step(eng, step0 + k, ...)
 * reads it while the ring holds it.  The engine's readers (kwk_fired*, kwk_fired_fetch_async) return
 * the call's last step.  With ev_every > 0, events 2i / 2i + 1 (kwk_event_record) bracket the sweep
 * LAUNCH containing the first step j = ev_j0 + k that is a multiple of ev_every (i = j / ev_every):
 * that launch sweeps kwk_last_sweep().steps steps (1, 2 or 4; ev_every 2 or 3 caps launches at 2
 * steps, 1 disables the fusion), so a caller turning an event pair into per-step time divides by
 * the steps of that launch. */
kwk_status kwk_step_n(kwk_engine* eng, uint32_t n, int64_t now0_ns, int64_t dt_ns, uint64_t seed, uint64_t step0,
                      uint32_t compact, uint32_t ev_every, uint32_t ev_j0);
/* kwk_step_n over two engines of one shard (the pod and node kinds), enqueued launch by launch in
 * turn — eng's sweep launch (+ events) and hand-back, then as many of other's steps — so that
 * neither stream waits for the host to finish enqueuing the other's n steps; events go on eng's
 * stream only, as in kwk_step_n.  Both engines' steps are tagged step0 + k in their rings.
 * Messages: eng's handle. */
kwk_status kwk_step_n_pair(kwk_engine* eng, kwk_engine* other, uint32_t n, int64_t now0_ns, int64_t dt_ns, uint64_t seed,
                           uint64_t step0, uint32_t compact, uint32_t ev_every, uint32_t ev_j0);
kwk_status kwk_fired(kwk_engine* eng, kwk_fired_rec* out, uint32_t cap, uint32_t* n_out);
/* device pointers of the compacted list and of its u32 count (valid until the next kwk_step) */
kwk_status kwk_fired_device(kwk_engine* eng, const kwk_fired_rec** recs, const uint32_t** count);
/* The same hand-back as 4-byte packed records, half the bytes over HBM and PCIe:
 * KWK_FIRED_PACKED_STAGE(r) = r >> 27 (stage index), KWK_FIRED_PACKED_SLOT(r) = r & (2^27 - 1); same
 * order as kwk_fired.  The flags of kwk_fired_rec are not carried: DELETED is the stage's
 * KWK_NEXT_DELETE, DELTA_UNKNOWN the (class, stage) delta the host loaded, REMATCH is the device's
 * own business (kwk_fired still returns all three).  Engines of at most 2^27 slots (KWK_ECAP
 * otherwise).  kwk_step_n(..., compact = KWK_COMPACT_PACKED, ...) / KWK_TICK_COMPACT_PACKED enqueue
 * it per step. */
#define KWK_COMPACT_PACKED 2u
#define KWK_FIRED_PACKED_STAGE(r) ((uint32_t)(r) >> 27)
#define KWK_FIRED_PACKED_SLOT(r) ((uint32_t)(r) & 0x7FFFFFFu)
kwk_status kwk_fired_compact_packed(kwk_engine* eng);
/* The hand-back at 2 bytes per transition, for engines on the 1-byte dictionary sweep with at most 4
 * stages (the C1 / C5 pod-fast shape; KWK_ESTATE otherwise: use kwk_fired_packed): the sweep's
 * own records {offset: 11, stage: 2, flags: 3} copied into one dense list, grouped by segment, plus
 * the records per segment.  Segment s (in order) covers slots [s * region_slots, (s + 1) *
 * region_slots); a record r of it is slot s * region_slots + KWK_FIRED16_SLOT(r), stage
 * KWK_FIRED16_STAGE(r), flags KWK_FIRED16_FLAGS(r) (the KWK_FIRED_* bits).  Same (slot, stage)
 * sequence as kwk_fired.  kwk_step_n(..., KWK_COMPACT_PACKED16, ...) enqueues it per step (an engine
 * without 2-byte records then leaves the 4-byte packed list). */
#define KWK_COMPACT_PACKED16 3u
#define KWK_FIRED16_STAGE(r) (((uint32_t)(r) >> 11) & 3u)
#define KWK_FIRED16_FLAGS(r) (((uint32_t)(r) >> 13) & 7u)
#define KWK_FIRED16_SLOT(r)                                                                                   \
  (((((uint32_t)(r) & 0x7FFu) >> 8) >> 2) * 1024u + (((((uint32_t)(r) & 0x7FFu) >> 2) & 63u) ^ (((uint32_t)(r) & 0x7FFu) >> 8)) * 16u + \
   ((((uint32_t)(r) & 0x7FFu) >> 8) & 3u) * 4u + ((uint32_t)(r) & 3u))
kwk_status kwk_fired_compact_packed16(kwk_engine* eng);
kwk_status kwk_fired_packed16(kwk_engine* eng, uint16_t* out, uint32_t cap, uint32_t* n_out, uint32_t* seg_counts,
                              uint32_t seg_cap, uint32_t* n_segs, uint32_t* region_slots);
/* The hand-back at ~1.1 bytes per transition (C5's 10 % firing), for the same engines as the 2-byte
 * records: per segment s of n (slots [s * region_slots, (s + 1) * region_slots)) a 2048-bit fired
 * map, bit i set when the object of KWK_BITS_SLOT(i) fired, kept byte-sparse, and the 2-bit stage
 * codes of its set bits in bit order.  Words:
 *   s < n                 segment s: records c (bits 0-15), nonzero map bytes z (bits 16-31)
 *   n + P(s) ...          segment s: 8 summary words (bit t of word w: map byte 32 w + t is
 *                         nonzero), its z nonzero map bytes in order (padded to a word), its c
 *                         codes, 16 per word (code j at bits 2 (j % 16) of word j / 16; padded)
 * with P(s) = sum over t < s of (8 + ceil(z_t / 4) + ceil(c_t / 16)).  Same (slot, stage) sequence
 * as kwk_fired; the flags are not carried (as KWK_COMPACT_PACKED).  n_words: the list's words,
 * n_records: its transitions.  kwk_step_n(..., KWK_COMPACT_BITS, ...) enqueues it per step (an
 * engine without 2-byte records then leaves the 4-byte packed list). */
#define KWK_COMPACT_BITS 4u
#define KWK_BITS_SLOT(i) KWK_FIRED16_SLOT(((((uint32_t)(i) & 7u) << 8) | ((((uint32_t)(i) >> 5) & 63u) << 2 ^ (((uint32_t)(i) & 7u) << 2)) | (((uint32_t)(i) >> 3) & 3u)))
kwk_status kwk_fired_compact_bits(kwk_engine* eng);
kwk_status kwk_fired_bits(kwk_engine* eng, uint32_t* out, uint64_t cap_words, uint64_t* n_words, uint32_t* n_records,
                          uint32_t* n_segs, uint32_t* region_slots);
kwk_status kwk_fired_packed(kwk_engine* eng, uint32_t* out, uint32_t cap, uint32_t* n_out);
kwk_status kwk_fired_packed_device(kwk_engine* eng, const uint32_t** recs, const uint32_t** count);
/* Overlapped hand-back to the host (the playStage workers' input, pod_controller.go:257-290): the
 * last step's compacted list (whatever kwk_fired_compact* / kwk_step_n left: 2-, 4- or 8-byte
 * records) and, for the 2-byte records, the records per segment, copied by the engine's copy
 * stream while the device goes on.  The call waits for the list's length only (the compaction of
 * that step), enqueues the copies and returns: call it after enqueuing the NEXT step's sweep and
 * the copy overlaps that sweep.  The engine's next compaction waits for the copy on the device
 * (the list is rewritten in place); the host buffers hold the copy after kwk_fired_fetch_wait (or
 * the engine's next fetch).  Buffers from kwk_alloc_host make the copies DMA; double-buffer them
 * to read one step's records while the next step's copy runs.  seg_counts may be NULL. */
typedef struct {
  uint32_t n_records;      /* transitions in the list (records; the bitmap hand-back: its set bits) */
  uint32_t record_bytes;   /* 2 (KWK_COMPACT_PACKED16), 4 (KWK_COMPACT_PACKED), 8 (kwk_fired_rec), 0 (KWK_COMPACT_BITS) */
  uint32_t n_segs;         /* 2-byte records / bitmap hand-back: segments (seg_counts entries copied), else 0 */
  uint32_t region_slots;   /* 2-byte records / bitmap hand-back: slots per segment, else 0 */
  uint32_t format;         /* KWK_COMPACT_PACKED16, _PACKED, _BITS or 1 (kwk_fired_rec) */
  uint32_t reserved;
  uint64_t bytes;          /* bytes copied into out */
  uint64_t step;           /* the step whose list was copied */
} kwk_fetch_info;
kwk_status kwk_fired_fetch_async(kwk_engine* eng, void* out, uint64_t cap_bytes, uint32_t* seg_counts, uint32_t seg_cap,
                                 kwk_fetch_info* info);
kwk_status kwk_fired_fetch_wait(kwk_engine* eng);

/* Every step's hand-back to the host, fused steps included (the playStage workers' input for each
 * step, pod_controller.go:257-290).  kwk_fired_keep(eng, depth) keeps the lists of the last `depth`
 * compactions (1..64, at least 4: a fused launch's steps; 0 = the default: the last 4, no per-step
 * completion signal) in the device
 * ring and makes every compaction signal its own completion and write its length to pinned host
 * memory.  kwk_fired_fetch_step(eng, step, ...) is kwk_fired_fetch_async for the list of step
 * `step` (the step argument of kwk_step / kwk_step_n's step0 + k): it waits for THAT step's
 * compaction only (later steps go on running), enqueues the copies on the copy stream and returns;
 * the ring slot is rewritten only after its copy (the compaction waits on the device).  So a host
 * calls kwk_step_n(eng, n, ...) and then kwk_fired_fetch_step for step0 .. step0 + n - 1, each copy
 * overlapping the later steps' sweeps, and reads the buffers after kwk_fired_fetch_wait.  KWK_ESTATE
 * when the ring no longer holds that step. */
kwk_status kwk_fired_keep(kwk_engine* eng, uint32_t depth);
kwk_status kwk_fired_fetch_step(kwk_engine* eng, uint64_t step, void* out, uint64_t cap_bytes, uint32_t* seg_counts,
                                uint32_t seg_cap, kwk_fetch_info* info);
/* pinned (page-locked) host buffers for kwk_fired / kwk_read / usage outputs, reused across steps */
kwk_status kwk_alloc_host(uint64_t bytes, void** out);
kwk_status kwk_free_host(void* p);
/* cumulative counters (synchronises) */
kwk_status kwk_stats(kwk_engine* eng, kwk_step_stats* out);
/* read back columns of slots [first, first+n) (synchronises) */
kwk_status kwk_read(kwk_engine* eng, uint32_t first, uint32_t n, kwk_hot* hot, int64_t* deletion_s);
kwk_status kwk_sync(kwk_engine* eng);

/* ------------------------------------------------------------------ resource usage */
/* Pods must be loaded node-sorted: node j owns slots [node_ptr[j], node_ptr[j+1]).
 * usage_key per pod: bits 0..13 cpu value id, 14..27 memory value id, 28..31 containers
 * (each container of the pod evaluates to the pod's value, as usage-from-annotation does). */
kwk_status kwk_usage_config(kwk_engine* eng, uint32_t n_nodes, const uint32_t* node_ptr, const uint32_t* usage_key,
                            uint32_t n_cpu, const double* cpu_values, uint32_t n_mem, const double* mem_values);
/* per-node cpu / memory sums and cumulative integrators at now_ns (enqueue only) */
kwk_status kwk_usage(kwk_engine* eng, int64_t now_ns);
/* node_out: n_nodes x {cpu, mem, cpu_cumulative, mem_cumulative}; cluster_out: {cpu, mem} */
kwk_status kwk_usage_read(kwk_engine* eng, double* node_out, double* cluster_out);
/* per-pod outputs of kwk_usage (podResourceUsage / podResourceCumulativeUsage,
 * metrics_resource_usage.go:36-65,170-193): enable allocates 56 bytes per slot */
kwk_status kwk_usage_pods(kwk_engine* eng, uint32_t enable);
/* pod_out: n x {cpu, mem, cpu_cumulative, mem_cumulative} for slots [first, first+n) */
kwk_status kwk_usage_read_pods(kwk_engine* eng, uint32_t first, uint32_t n, double* pod_out);

/* Pods whose containers evaluate to different usages (metrics_resource_usage.go:136-168 per
 * container): usage_key = m with a 0 container count (bits 28..31), m indexing
 * mixed[2m] = first, mixed[2m+1] = count into ckeys (per container: cpu id | memory id << 14,
 * in spec.containers order).  Pods may share a mixed entry (their containers evaluate alike);
 * the cumulative integrators are still per pod and container.  Call after kwk_usage_config. */
kwk_status kwk_usage_mixed(kwk_engine* eng, uint32_t n_mixed, const uint32_t* mixed, uint32_t n_ckeys,
                           const uint32_t* ckeys);
/* per-container outputs of kwk_usage (containerResourceUsage / containerResourceCumulativeUsage,
 * metrics_resource_usage.go:36-52,111-134) for the containers of pods [first, first+n), in pod
 * then spec order: {cpu, mem, cpu_cumulative, mem_cumulative} each (0 for dead pods);
 * *n_out = the number of containers (synchronises; needs kwk_usage_pods(eng, 1)) */
kwk_status kwk_usage_read_containers(kwk_engine* eng, uint32_t first, uint32_t n, double* out, uint32_t cap,
                                     uint32_t* n_out);

/* ------------------------------------------------------------------ Metric CRD values */
/* A Metric CR's value expressions (kustomize/metrics/resource/metrics-resource.yaml; CEL,
 * pkg/kwok/metrics/evaluator.go) lowered by the host to postfix programs over doubles:
 * KWK_MOP_LOAD pushes one of the per-series inputs KWK_MIN_* (the engine's usage outputs of the
 * last kwk_usage, creation times, the scrape clock).  One program per metric, evaluated for
 * every series of a scrape by kwk_metrics_eval (one GPU thread per series). */
#define KWK_METRIC_DIM_NODE 0
#define KWK_METRIC_DIM_POD 1
#define KWK_METRIC_DIM_CONTAINER 2
#define KWK_MOP_CONST 1
#define KWK_MOP_LOAD 2
#define KWK_MOP_ADD 3
#define KWK_MOP_SUB 4
#define KWK_MOP_MUL 5
#define KWK_MOP_DIV 6
#define KWK_MOP_NEG 7
#define KWK_MIN_NOW_S 0               /* Now().UnixSecond() */
#define KWK_MIN_CONTAINER_CPU 1       /* pod.Usage("cpu", container.name) */
#define KWK_MIN_CONTAINER_MEM 2
#define KWK_MIN_CONTAINER_CUM_CPU 3   /* pod.CumulativeUsage("cpu", container.name) */
#define KWK_MIN_CONTAINER_CUM_MEM 4
#define KWK_MIN_POD_CPU 5             /* pod.Usage("cpu") */
#define KWK_MIN_POD_MEM 6
#define KWK_MIN_POD_CUM_CPU 7
#define KWK_MIN_POD_CUM_MEM 8
#define KWK_MIN_NODE_CPU 9            /* node.Usage("cpu") */
#define KWK_MIN_NODE_MEM 10
#define KWK_MIN_NODE_CUM_CPU 11
#define KWK_MIN_NODE_CUM_MEM 12
#define KWK_MIN_POD_SINCE 13          /* pod.SinceSecond() */
#define KWK_MIN_NODE_SINCE 14
#define KWK_MIN_POD_CREATED 15        /* pod.metadata.creationTimestamp.UnixSecond() */
#define KWK_MIN_NODE_CREATED 16
#define KWK_MIN_STARTED_CONTAINERS 17 /* node.StartedContainersTotal() */
typedef struct {
  uint32_t op;     /* KWK_MOP_* */
  uint32_t arg;    /* KWK_MIN_* for KWK_MOP_LOAD */
  double value;    /* KWK_MOP_CONST */
} kwk_metric_op;   /* 16 bytes */
typedef struct {
  uint32_t dimension;  /* KWK_METRIC_DIM_* */
  uint32_t first_op, n_ops;
  uint32_t reserved;
} kwk_metric_desc;
/* programs (replaces earlier ones); at most 64 ops per metric, stack depth 8 */
kwk_status kwk_metrics_load(kwk_engine* pods, uint32_t n_metrics, const kwk_metric_desc* metrics, uint32_t n_ops,
                            const kwk_metric_op* ops);
/* per-object inputs: creation times (unix ns, INT64_MIN = unset: the Go zero time) of the
 * engine's pods and of the n_nodes nodes of kwk_usage_config, and StartedContainersTotal per
 * node (controller.go:602-611); zero_time_unix_s = what UnixSecond() gives for the zero time */
kwk_status kwk_metrics_inputs(kwk_engine* pods, const int64_t* pod_created_ns, const int64_t* node_created_ns,
                              const double* node_started, double zero_time_unix_s);
/* every metric's series for the scrape of nodes [node_first, node_first + n_nodes) at now_ns
 * (after kwk_usage(now_ns)): metric by metric, node series per node, pod series per pod slot,
 * container series per container (kwk_usage_read_containers order); NaN for dead pods.
 * *n_out = values written (synchronises) */
kwk_status kwk_metrics_eval(kwk_engine* pods, int64_t now_ns, uint32_t node_first, uint32_t n_nodes, double* out,
                            uint64_t cap, uint64_t* n_out);
/* the same values left on the device (enqueue only): *out = the engine's device buffer of *n_out
 * doubles, valid until the next kwk_metrics_eval* call — for an in-process consumer (an exposition
 * writer on the GPU, an all-reduce) and for timing the evaluation without the copy */
kwk_status kwk_metrics_eval_device(kwk_engine* pods, int64_t now_ns, uint32_t node_first, uint32_t n_nodes,
                                   const double** out, uint64_t* n_out);

/* Histogram Metric CRs (kind: histogram; pkg/kwok/metrics/metrics.go:133-160,356-462,
 * histogram.go:81-164): per series every bucket's value program runs (a lowered CEL value, as
 * above), uint64(value) — Go's float64 -> uint64 conversion on amd64 — is stored at the bucket's
 * le (a later bucket with an equal le overwrites), and the exposition's bucket counts are
 * computed as histogram.Write does.  One record of n_visible + 3 uint64 words per series:
 *   [0, n_visible)   cumulative counts of the visible buckets, ascending le
 *   n_visible        the +Inf bucket's cumulative count (histogram.Write: only keys above the last
 *                    visible bound land there)
 *   n_visible + 1    sample count;  n_visible + 2: sample sum (float64 bits)
 * A dead pod's record is all ones (no series: ListPods skips it).  Series order as
 * kwk_metrics_eval, histogram by histogram. */
typedef struct {
  double le;          /* MetricBucket.Le */
  uint32_t hidden;    /* MetricBucket.Hidden: evaluated and stored, not a visible bucket */
  uint32_t first_op;  /* the bucket's value program */
  uint32_t n_ops;
  uint32_t reserved;
} kwk_metric_bucket;  /* 24 bytes */
typedef struct {
  uint32_t dimension;   /* KWK_METRIC_DIM_* */
  uint32_t first_bucket, n_buckets;  /* 1..64 buckets */
  uint32_t reserved;
} kwk_histogram_desc;
kwk_status kwk_histograms_load(kwk_engine* pods, uint32_t n_hist, const kwk_histogram_desc* hists, uint32_t n_buckets,
                               const kwk_metric_bucket* buckets, uint32_t n_ops, const kwk_metric_op* ops);
kwk_status kwk_histograms_eval(kwk_engine* pods, int64_t now_ns, uint32_t node_first, uint32_t n_nodes, uint64_t* out,
                               uint64_t cap, uint64_t* n_out);
kwk_status kwk_histograms_eval_device(kwk_engine* pods, int64_t now_ns, uint32_t node_first, uint32_t n_nodes,
                                      const uint64_t** out, uint64_t* n_out);

/* ------------------------------------------------------------------ node leases */
/* NodeLeaseController (pkg/kwok/controllers/node_lease_controller.go) on a NODE engine: one
 * lease record per node slot — the informer's cached coordination/v1 Lease plus the
 * controller's queue entry — advanced on the device by kwk_lease_step. */
#define KWK_LEASE_EXISTS (1u << 0)    /* the Lease object exists (getLease ok) */
#define KWK_LEASE_HOLDER (1u << 1)    /* spec.holderIdentity != nil */
#define KWK_LEASE_DURATION (1u << 2)  /* spec.leaseDurationSeconds != nil */
#define KWK_LEASE_RENEW (1u << 3)     /* spec.renewTime != nil */
#define KWK_LEASE_HOLD (1u << 4)      /* node in holdLeaseSet (TryHold; ReleaseHold clears it) */
#define KWK_LEASE_QUEUED (1u << 5)    /* a sync is queued at next_try_ns (TryHold queues one at once) */
typedef struct {
  int64_t renew_ns;      /* spec.renewTime, unix ns (a MicroTime: microsecond precision) */
  int64_t next_try_ns;   /* delay-queue due time of the node's next sync */
  uint32_t holder;       /* spec.holderIdentity, interned by the host */
  int32_t duration_s;    /* spec.leaseDurationSeconds */
  int32_t transitions;   /* spec.leaseTransitions */
  uint32_t flags;        /* KWK_LEASE_* */
} kwk_lease;             /* 32 bytes */

typedef struct {
  uint32_t holder_id;          /* this kwok's HolderIdentity (controller.go:275), interned */
  int32_t lease_duration_s;    /* NodeLeaseDurationSeconds */
  int64_t renew_interval_ns;   /* leaseDuration / 4 (controller.go:247) */
  double renew_jitter;         /* RenewIntervalJitter: 0.04 (controller.go:249) */
  uint32_t manage_nodes;       /* 1: the node's MANAGED bit follows Held() (readOnlyFunc,
                                * controller.go:285-288) and a successful sync re-matches it */
  uint32_t reserved;
} kwk_lease_params;

/* API writes of the last kwk_lease_step, as kwk_fired_rec {slot, op, 0} (unordered) */
#define KWK_LEASE_OP_CREATE 1   /* ensureLease (node_lease_controller.go:225-249) */
#define KWK_LEASE_OP_RENEW 2    /* renewLease by the holder (:252-275) */
#define KWK_LEASE_OP_ACQUIRE 3  /* renewLease taking over an absent or expired holder (transitions + 1) */
#define KWK_LEASE_OP_BUSY 4     /* held by another holder: no write, retried after interval() */
#define KWK_LEASE_OP_FAILED 5   /* set by kwk_lease_fail: the write was rejected, retried after interval() */

typedef struct {
  uint64_t steps, creates, renews, acquires, busy;
} kwk_lease_counters;

kwk_status kwk_lease_config(kwk_engine* nodes, const kwk_lease_params* cfg);
/* lease informer events / TryHold / ReleaseHold: overwrite records [first, first+n) */
kwk_status kwk_lease_set(kwk_engine* nodes, uint32_t first, uint32_t n, const kwk_lease* leases);
/* one pass of syncWorker over every held node whose sync is due (enqueue only).
 * interval() jitter uses Philox (key = seed ^ ((uint64_t)kind_salt << 32), ctr = (slot_base+slot, step, 3)) */
kwk_status kwk_lease_step(kwk_engine* nodes, int64_t now_ns, uint64_t seed, uint64_t step);
kwk_status kwk_lease_ops(kwk_engine* nodes, kwk_fired_rec* out, uint32_t cap, uint32_t* n_out);
kwk_status kwk_lease_read(kwk_engine* nodes, uint32_t first, uint32_t n, kwk_lease* out);
/* Lease writes of the last kwk_lease_step that the apiserver rejected (syncWorker's err
 * branch, node_lease_controller.go:121-128): `old` = the lease the informer still holds; the
 * device restores it (keeping HOLD / QUEUED), queues the retry after the same interval() draw
 * (AddWeightAfter(node, 1, dur)), sets the node's MANAGED bit from Held() of the restored lease
 * and drops the re-match the write would have caused; kwk_lease_sync_pods then applies
 * MANAGED to the node's pods without a resync.  Call before kwk_lease_sync_pods / kwk_step. */
kwk_status kwk_lease_fail(kwk_engine* nodes, int64_t now_ns, uint64_t seed, uint64_t step, uint32_t n,
                          const uint32_t* slots, const kwk_lease* old);
kwk_status kwk_lease_stats(kwk_engine* nodes, kwk_lease_counters* out);
/* pods of the nodes synced by the last lease step (node j owns pod slots [node_ptr[j],
 * node_ptr[j+1])): MANAGED follows Held(), a successful sync re-matches pods with no queued
 * stage (podsOnNodeSyncWorker, controller.go:559-573) */
kwk_status kwk_lease_sync_pods(kwk_engine* pods, const kwk_engine* nodes, uint32_t n_nodes, const uint32_t* node_ptr);

/* The fused reconciliation tick (C3 and any node + pod deployment): the per-tick sequence of
 *   kwk_lease_step(nodes) -> kwk_lease_sync_pods(pods, nodes, node_ptr) -> kwk_step(nodes) ->
 *   kwk_step(pods)   (+ kwk_fired_compact on both with KWK_TICK_COMPACT)
 * enqueued by one call, with the two engines' streams ordered by HIP events instead of host
 * synchronisations (kwk_lease_sync_pods synchronises the node stream each call).  Results are
 * those of the separate calls.  Lease ops / fired lists / stats are read as after the separate
 * calls (kwk_lease_ops, kwk_fired on either engine).  kwk_tick_bind registers the pods' node_ptr
 * (node-sorted pods, as kwk_lease_sync_pods) once; pods = NULL runs the node engine alone (its
 * lease step only if kwk_lease_config was called).  kwk_tick_n: n ticks at now0 + k * dt,
 * step0 + k (enqueue only; the last tick's lease ops / fired lists are readable). */
#define KWK_TICK_COMPACT (1u << 0)
#define KWK_TICK_COMPACT_PACKED (1u << 1) /* the hand-back as packed 4-byte records (kwk_fired_compact_packed) */
kwk_status kwk_tick_bind(kwk_engine* pods, const kwk_engine* nodes, uint32_t n_nodes, const uint32_t* node_ptr);
kwk_status kwk_tick(kwk_engine* nodes, kwk_engine* pods, int64_t now_ns, uint64_t seed, uint64_t step, uint32_t flags);
kwk_status kwk_tick_n(kwk_engine* nodes, kwk_engine* pods, uint32_t n, int64_t now0_ns, int64_t dt_ns, uint64_t seed,
                      uint64_t step0, uint32_t flags);

/* cluster aggregates: counts[k] = alive objects with (pred & masks[k]) != 0 (mask 0 = all
 * alive objects), k < 16 — e.g. the phase histogram all-reduced across GPUs (synchronises) */
kwk_status kwk_count(kwk_engine* eng, uint32_t n_masks, const uint32_t* masks, uint64_t* counts);

/* The whole reporting-interval aggregate of one engine, computed on the device without a host
 * round trip (SURVEY §8(b) kwk_aggregates; the C5 all-reduce reads it in place): enqueues the
 * per-stage transition totals (as kwk_stats), kwk_count of `masks` and, with KWK_AGG_USAGE, a
 * kwk_usage evaluation at now_ns, and writes float64
 *   out[0 .. n_stages)                       cumulative transitions per stage
 *   out[n_stages .. n_stages + n_masks)      counts per mask
 *   out[n_stages + n_masks + {0, 1}]         cluster cpu / memory usage (KWK_AGG_USAGE only)
 * `out` is DEVICE memory on the engine's device (e.g. the RCCL buffer; counts stay exact up to
 * 2^53), or NULL for the engine's own buffer, read back with kwk_aggregate_read.  Stream-ordered:
 * kwk_sync (or kwk_aggregate_read) before another stream reads `out`.  Returns the number of
 * doubles written in *n_out.  Reference: metrics_resource_usage.go:195-224 (cluster usage). */
#define KWK_AGG_USAGE (1u << 0)
kwk_status kwk_aggregate(kwk_engine* eng, uint32_t n_masks, const uint32_t* masks, int64_t now_ns, uint32_t flags,
                         double* out, uint32_t* n_out);
/* copies the engine-owned aggregate buffer (the last kwk_aggregate with out = NULL) to host memory
 * (synchronises): n doubles */
kwk_status kwk_aggregate_read(kwk_engine* eng, double* host_out, uint32_t n);

/* raw device pointers for in-process consumers (RCCL aggregates, profiling): state = the
 * state stream (kwk_step_stats.state_bytes per slot); fired / wave_counts = the sweep's
 * internal fired segments and per-segment counts (valid after kwk_fired) */
kwk_status kwk_device_ptrs(kwk_engine* eng, void** state, void** fired, void** wave_counts);

/* the engine's HIP stream (hipStream_t): in-process consumers order their own work after the
 * engine's (e.g. an RCCL all-reduce of kwk_aggregate's output) with stream waits, no host sync */
kwk_status kwk_stream(kwk_engine* eng, void** stream);
/* HIP events recorded on the engine's stream (live kernel timing in bench.py); timing-only
 * events without a system-scope fence: not a memory-visibility point for the host */
kwk_status kwk_event_record(kwk_engine* eng, uint32_t idx);
kwk_status kwk_event_elapsed(kwk_engine* eng, uint32_t a, uint32_t b, float* ms);
/* which sweep kernel the last kwk_step / kwk_match launched (tests pin the benchmarked shape) */
#define KWK_SWEEP_NONE 0     /* nothing swept (no active slots) */
#define KWK_SWEEP_16 1       /* sweep16_kernel: 2-byte words, general phase 2 */
#define KWK_SWEEP_16_FSM 2   /* sweep16_fsm_kernel: 2-byte words, transition table */
#define KWK_SWEEP_W4 3       /* sweepw_kernel<4>: 4-byte packed words */
#define KWK_SWEEP_W8 4       /* sweepw_kernel<8>: 8-byte wide words */
#define KWK_SWEEP_8 5        /* sweep8_kernel: 1-byte dictionary ids, id transition table in LDS */
#define KWK_SWEEP_WD 6       /* sweepw_kernel<8, fused>: 8-byte records {packed word, 36-bit relative due} */
typedef struct {
  uint32_t kernel;       /* KWK_SWEEP_* */
  uint32_t q;            /* 16-byte chunks per lane */
  uint32_t persistent;   /* 1: persistent grid (grid < tiles) */
  uint32_t depth;        /* tiles in flight per wave (table-only sweep) */
  uint32_t grid;         /* workgroups launched */
  uint32_t tiles;        /* tiles swept */
  uint32_t harness;      /* 1: the harness variant */
  uint32_t steps;        /* steps the launch swept: 2 or 4 when fused (KWK_TUNE_FUSE_STEPS), else 1 (0: unset) */
} kwk_sweep_info;
kwk_status kwk_last_sweep(kwk_engine* eng, kwk_sweep_info* out);
/* 2 since round 6: the hand-back ring (kwk_fired_keep / kwk_fired_fetch_step, kwk_fetch_info.step),
 * KWK_TUNE_FOLD_HB and kwk_fired_fold16 retired, kwk_sweep_info.steps (was reserved) */
#define KWK_ABI_VERSION 2u
uint32_t kwk_abi_version(void);
uint32_t kwk_tile_objects(void); /* objects per sweep workgroup */

#ifdef __cplusplus
}
#endif
#endif /* KWOK_ENGINE_H */
