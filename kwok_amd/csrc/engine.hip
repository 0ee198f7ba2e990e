// MI355X (gfx950) Stage-lifecycle engine: HIP kernels + the C ABI of include/kwok_engine.h.
//
// One fused, memory-bound sweep per step over the SoA object table (16-byte hot record per
// object).  Per object it does, in this order, what the reference does
// per informer event / per delay-queue pop:
//   harness churn (bench/parity only)
//   match      Lifecycle.match  pkg/utils/lifecycle/lifecycle.go:51-63, Stage.match :285-309
//   pick       Lifecycle.Match  lifecycle.go:125-191 (Philox hook at :157,:163,:175,:180)
//   delay      Stage.Delay      lifecycle.go:313-341 (Philox hook at :338); getters
//              expression/value_int_from.go:53-81, value_duration_from.go:53-79
//   schedule   addStageJob      pod_controller.go:660-671 (one pending job per object; a new
//              match replaces it; no match leaves the old job queued, pod_controller.go:222-229)
//   fire       delay queue pop  weight_delaying_queue.go:97-174 (due <= now)
//   next       playStage        pod_controller.go:290-360: finalizersModify
//              (finalizers.go:83-111) as bit-set algebra, delete, patches as a per-(class,
//              stage) delta precompiled on the host.
// No MFMA: nothing here is a contraction.  The stage table is wave-uniform and is read
// through the scalar cache (s_load), the per-object record streams through VGPRs with
// 16-byte loads; fired records are compacted per wave with a ballot into a private
// per-wave segment (no global atomics in the sweep).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <set>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../include/kwok_engine.h"

static void engine_set_error(kwk_engine* e, const std::string& msg);

namespace {

constexpr int kBlock = 256;              // 4 waves of 64
constexpr int kMinObjPerThread = 8;      // smallest sweep tile (2048 objects): sizes the per-tile arrays
constexpr int kMaxObjPerThread = 32;     // largest sweep tile (8192 objects): pads the state allocation
constexpr int kWavesPerBlock = kBlock / 64;
// matched, fired, algorithmic bytes, fired per stage, line bytes (algorithmic with state writes
// counted as the whole lines / chunks the sweep stores)
constexpr int kStatWords = 4 + KWK_MAX_STAGES;
constexpr int kStatLine = 3 + KWK_MAX_STAGES;

// Error messages: every failing call stores its message in the engine it was called on
// (kwk_last_error(eng)), so a caller that moves between OS threads (a cgo goroutine) reads the
// message of its own engine's call; calls without an engine (kwk_engine_create, pinned host
// buffers) leave it in the calling thread's slot (kwk_last_error(NULL)).
thread_local std::string g_err;
thread_local kwk_engine* tl_eng = nullptr;  // the engine of the API call running on this thread

struct ErrScope {  // marks the engine an API call works on, for fail()
  kwk_engine* prev;
  explicit ErrScope(const kwk_engine* e) : prev(tl_eng) { tl_eng = const_cast<kwk_engine*>(e); }
  ~ErrScope() { tl_eng = prev; }
};

kwk_status fail(kwk_status code, const std::string& msg) {
  g_err = msg;
  if (tl_eng) engine_set_error(tl_eng, msg);
  return code;
}

#define HIP_TRY(x)                                                                    \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) return fail(KWK_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

// ------------------------------------------------------------------ Philox4x32-10
__device__ __forceinline__ void philox10(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                                         uint32_t k1) {
  // the round keys are wave-uniform (a kernel argument): the empty asm re-defines the key here so
  // that the round keys are scalar adds at the call instead of 20 values hoisted out of the word
  // sweep's loops into SGPRs it does not have (spilled to VGPR lanes, reloaded lane by lane; r5)
  k0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)k0);
  k1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)k1);
  asm volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32 x 32 -> 64-bit multiply per product (v_mad_u64_u32) instead of separate lo / hi
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    const uint32_t n0 = hi1 ^ c1 ^ k0;
    const uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__device__ __forceinline__ uint64_t philox_u64(uint64_t gslot, uint64_t step, uint32_t site, uint64_t key) {
  uint32_t c0 = (uint32_t)gslot, c1 = (uint32_t)step, c2 = (uint32_t)(step >> 32), c3 = site;
  philox10(c0, c1, c2, c3, (uint32_t)key, (uint32_t)(key >> 32));
  return (uint64_t)c0 | ((uint64_t)c1 << 32);
}

// rand.Intn / rand.Int63n replacement: floor(u64 * n / 2^64), n > 0
__device__ __forceinline__ int64_t below_u64(uint64_t u, int64_t n) { return (int64_t)__umul64hi(u, (uint64_t)n); }

// rand.Float64 replacement: (u64 >> 11) * 2^-53, in [0, 1)
__device__ __forceinline__ double rng_float64(uint64_t gslot, uint64_t step, uint32_t site, uint64_t key) {
  return (double)(philox_u64(gslot, step, site, key) >> 11) * 0x1.0p-53;
}

// site 1's block carries both draws of a matched object: words 0-1 the pick, words 2-3 the Delay
// jitter ("site 2"), so an object that needs both runs one Philox (r5: C2 phase 2 is VALU-bound)
constexpr uint32_t kSitePick = 1, kSiteLeaseJitter = 3, kSiteRetryJitter = 4;

__device__ __forceinline__ int64_t sat_add(int64_t a, int64_t b) {
  int64_t r;
  if (__builtin_add_overflow(a, b, &r)) return b > 0 ? INT64_MAX : INT64_MIN;
  return r;
}

// time.Time.Sub for an RFC3339 time (sec, nsec) against now (ns), saturating like Go
__device__ __forceinline__ int64_t abs_time_sub(int64_t sec, int32_t nsec, int64_t now) {
  int64_t now_sec = now / 1000000000;
  int64_t now_ns = now % 1000000000;
  if (now_ns < 0) { now_ns += 1000000000; now_sec -= 1; }
  int64_t ds = sec - now_sec;
  int64_t dn = (int64_t)nsec - now_ns;  // (-1e9, 1e9)
  if (ds == 0) return dn;
  // move one second into dn so that ds' and dn' share a sign: overflow of ds'*1e9 then implies
  // overflow of the total
  if (ds > 0) { ds -= 1; dn += 1000000000; } else { ds += 1; dn -= 1000000000; }
  // ds * 1e9 overflows int64 iff |ds| > 9223372036 (a range test, not a 64 x 64 overflow multiply)
  if (ds > 9223372036ll || ds < -9223372036ll) return ds > 0 ? INT64_MAX : INT64_MIN;
  const int64_t p = ds * 1000000000ll;
  int64_t d;
  if (__builtin_add_overflow(p, dn, &d)) return dn > 0 ? INT64_MAX : INT64_MIN;
  return d;
}

struct Getter {   // result of an IntFrom / DurationFrom evaluation
  int64_t v;
  bool ok;
};

// value of a *From getter for one object.  slot: KWK_SLOT_NONE (constant default),
// KWK_SLOT_DELETION (deletionTimestamp column), or an index into the object's record.
__device__ __forceinline__ Getter eval_getter(int32_t slot, int64_t def, bool def_ok, uint32_t sched,
                                              const kwk_value* __restrict__ rec, int64_t del_s, int64_t now,
                                              bool is_duration) {
  if (slot == KWK_SLOT_NONE) return {def, def_ok};
  if (slot == KWK_SLOT_DELETION) {
    if (del_s == KWK_DEL_ABSENT) return {def, def_ok};
    return {abs_time_sub(del_s, 0, now), true};
  }
  if (!(sched & KWK_F_HASREC)) return {def, def_ok};
  const kwk_value e = rec[slot];
  switch (e.kind) {
    case KWK_V_OK: return {e.value, true};
    case KWK_V_NOTOK: return {0, false};
    case KWK_V_ABSTIME: return {is_duration ? abs_time_sub(e.value, e.nsec, now) : 0, is_duration};
    default: return {def, def_ok};
  }
}

// ------------------------------------------------------------------ object state formats
// wide   : uint2 {pred, sched} per slot (any compiled program);
// narrow : one u32 per slot when the program fits 32 bits:
//          [pred: pred_bits][class: cbits][stage code: sbits][flags: 5]
//          flags = sched bits 8..12 (ALIVE DIRTY MANAGED HASREC MATCHERR); stage code n_stages = none.
// half   : the same packing in one u16 per slot when it fits 16 bits (narrow = half = 1).
// byte   : one id byte per slot indexing a dictionary of the half words that can occur (a table-
//          only program; narrow = half = byte = 1): id2w / w2id on the device.
// fused  : one 8-byte record per slot, uint2 {x: packed word (bits 0..27) | due bits 32..35 at
//          28..31, y: due bits 0..31} when the packed word fits 28 bits (narrow = dw = 1): the
//          due time D relative to the engine's epoch rides with the word, so the word sweep reads
//          one stream; D = kDwFar means "in the side column" (the due column, for due times outside
//          [epoch, epoch + 2^36 - 1) ns, ~68.7 s; written and read only for those).
struct StateFmt {
  uint32_t narrow;
  uint32_t half;
  uint32_t byte;
  uint32_t dw;
  int64_t epoch;         // dw: the due times' origin (ns)
  uint32_t pmask;
  uint32_t cshift, cmask;
  uint32_t sshift, smask, none_code;
  uint32_t fshift;
  const uint16_t* id2w;  // byte: the word of each id
  const uint8_t* w2id;   // byte: the id of each half word (0xFF: none)
};

__host__ __device__ __forceinline__ uint2 fmt_unpack(uint32_t w, const StateFmt& f) {
  const uint32_t cls = (w >> f.cshift) & f.cmask;
  const uint32_t sc = (w >> f.sshift) & f.smask;
  const uint32_t stage = sc == f.none_code ? KWK_STAGE_NONE : sc;
  const uint32_t fl = (w >> f.fshift) & 0x1Fu;
  return make_uint2(w & f.pmask, stage | (fl << 8) | (cls << KWK_CLASS_SHIFT));
}

__host__ __device__ __forceinline__ uint32_t fmt_pack(uint32_t pred, uint32_t sched, const StateFmt& f) {
  const uint32_t stage = sched & 0xFFu;
  const uint32_t sc = stage == KWK_STAGE_NONE ? f.none_code : stage;
  return (pred & f.pmask) | (((sched >> KWK_CLASS_SHIFT) & f.cmask) << f.cshift) | ((sc & f.smask) << f.sshift) |
         (((sched >> 8) & 0x1Fu) << f.fshift);
}

// the fused record's relative due (StateFmt.dw)
constexpr uint32_t kDwShift = 28;                     // due bits 32..35 sit at word bits 28..31
constexpr uint32_t kDwWordMask = (1u << kDwShift) - 1u;
constexpr uint64_t kDwFar = (1ull << 36) - 1ull;      // "the due time is in the side column"
constexpr uint64_t kDwRebase = 1ull << 34;            // the epoch moves when now is this far past it
__host__ __device__ __forceinline__ uint64_t dw_get(uint2 r) {
  return ((uint64_t)(r.x >> kDwShift) << 32) | r.y;
}
__host__ __device__ __forceinline__ uint2 dw_put(uint2 r, uint64_t d) {
  return make_uint2((r.x & kDwWordMask) | ((uint32_t)(d >> 32) << kDwShift), (uint32_t)d);
}
// D of an absolute due time (kDwFar: outside the window, the side column holds it)
__host__ __device__ __forceinline__ uint64_t dw_enc(int64_t due, int64_t epoch) {
  if (due < epoch) return kDwFar;
  const uint64_t d = (uint64_t)due - (uint64_t)epoch;  // exact: due >= epoch
  return d < kDwFar ? d : kDwFar;
}
__host__ __device__ __forceinline__ int64_t dw_abs(uint64_t d, int64_t epoch) {
  return (int64_t)((uint64_t)epoch + d);
}

// small kernels (scatter / delete / usage / count) branch on the format at run time
__device__ __forceinline__ uint2 load_state(const void* st, uint64_t i, const StateFmt& f) {
  if (f.byte) return fmt_unpack(f.id2w[reinterpret_cast<const uint8_t*>(st)[i]], f);
  if (f.half) return fmt_unpack(reinterpret_cast<const uint16_t*>(st)[i], f);
  if (f.dw) return fmt_unpack(reinterpret_cast<const uint32_t*>(st)[2 * i], f);  // fmt_unpack ignores the due bits
  return f.narrow ? fmt_unpack(reinterpret_cast<const uint32_t*>(st)[i], f) : reinterpret_cast<const uint2*>(st)[i];
}
// the word only: a fused record keeps its due bits
__device__ __forceinline__ void store_state(void* st, uint64_t i, uint2 v, const StateFmt& f) {
  if (f.byte) {
    reinterpret_cast<uint8_t*>(st)[i] = f.w2id[fmt_pack(v.x, v.y, f) & 0xFFFFu];
  } else if (f.half) {
    reinterpret_cast<uint16_t*>(st)[i] = (uint16_t)fmt_pack(v.x, v.y, f);
  } else if (f.dw) {
    uint32_t* p = reinterpret_cast<uint32_t*>(st) + 2 * i;
    *p = (*p & ~kDwWordMask) | fmt_pack(v.x, v.y, f);
  } else if (f.narrow) {
    reinterpret_cast<uint32_t*>(st)[i] = fmt_pack(v.x, v.y, f);
  } else {
    reinterpret_cast<uint2*>(st)[i] = v;
  }
}
// word and due time together (scatter, retry)
__device__ __forceinline__ void store_state_due(void* st, int64_t* due_col, uint64_t i, uint2 v, int64_t due,
                                                const StateFmt& f) {
  if (f.dw) {
    const uint64_t d = dw_enc(due, f.epoch);
    reinterpret_cast<uint2*>(st)[i] = dw_put(make_uint2(fmt_pack(v.x, v.y, f), 0u), d);
    if (d == kDwFar) due_col[i] = due;
  } else {
    store_state(st, i, v, f);
    due_col[i] = due;
  }
}

// the word sweep is specialised per format
__device__ __forceinline__ uint2 sw_decode(uint2 w, const StateFmt&) { return w; }
__device__ __forceinline__ uint2 sw_decode(uint32_t w, const StateFmt& f) { return fmt_unpack(w, f); }
__device__ __forceinline__ void sw_encode(uint2& out, uint2 v, const StateFmt&) { out = v; }
__device__ __forceinline__ void sw_encode(uint32_t& out, uint2 v, const StateFmt& f) { out = fmt_pack(v.x, v.y, f); }

// the phase-1 idle test on raw state words: bit masks of the word holding flags + stage
// (fw: sched in the wide format, the packed word in the narrow one) and of the word holding
// pred (pw), computed on the host per launch
struct RawTest {
  uint32_t managed, dirty, alive;
  uint32_t sshift, smask, none_code;
  uint32_t term, del;  // harness: terminal phase bits / deletionTimestamp bit (pred)
};

constexpr uint32_t kMaxFuseSteps = 4;  // steps per 1-byte sweep launch (KWK_TUNE_FUSE_STEPS; 8 measured slower: r6x)
constexpr uint32_t kHbMin = kMaxFuseSteps;  // hand-back ring slots: at least a fused launch's steps (kwk_fired_keep)
constexpr uint32_t kHbMax = 64;
struct SweepArgs {
  void* __restrict__ st;         // per object state word (StateFmt: uint2 {pred, sched} or packed u32)
  int64_t* __restrict__ due;     // per object due time (read only for objects with a pending stage)
  int64_t* __restrict__ del_s;
  const uint32_t* __restrict__ rec_idx;
  const kwk_value* __restrict__ values;
  const kwk_stage_table* __restrict__ table;
  const kwk_delta* __restrict__ deltas;
  const uint32_t* __restrict__ lut;  // match-mask tables (lut_bytes x 256 entries, or 2^pred_bits), see match_mask
  kwk_fired_rec* __restrict__ fired;
  uint32_t* __restrict__ wave_counts;
  unsigned long long* __restrict__ cum;  // [n_blocks][kStatWords]
  uint32_t n;
  uint32_t lut_n;                    // table entries (0: no table)
  uint32_t lut_bytes;                // pred bytes with a table (1..4)
  uint32_t lut_rest;                 // stages the tables do not decide (clause loop)
  uint32_t value_slots;
  uint64_t slot_base;
  uint64_t key;
  uint64_t step;
  int64_t now;
  uint32_t fire;                 // 0: match only (kwk_match: Lifecycle.Match + Stage.Delay, no playStage)
  StateFmt fmt;
  RawTest raw;
  kwk_harness harness;
  const uint32_t* __restrict__ fsm;  // 2-byte sweep: per-(due ready, word) transition entries (or null)
  const int64_t* __restrict__ fsm_due;
  uint32_t fsm_bits;
  int64_t dw_epoch_old;          // fused format: the epoch the records hold (fmt.epoch: the one written)
  uint32_t dw_rebase;            // fused format: the epoch moves this sweep (every pending record re-encoded)
  // sweep8_kernel<..., kSteps>: steps 1 .. kSteps - 1 of the launch (their times, segments and counts)
  kwk_fired_rec* __restrict__ firedx[kMaxFuseSteps - 1];
  uint32_t* __restrict__ countsx[kMaxFuseSteps - 1];
  int64_t nowx[kMaxFuseSteps - 1];
  // the hand-back inside a one-tile-per-block 2-byte sweep (tail_handback; out == null: none)
  struct TailHb {
    void* out;                     // the ring slot's list: kwk_fired_rec, or packed 4-byte records
    uint32_t* offsets;             // [0] <- the list length
    uint32_t* host_len;            // kwk_fired_keep's pinned length word, or null
    unsigned long long* status;    // per block: seq << 32 | the block's records
    uint32_t seq;                  // this launch's tag (never 0)
    uint32_t packed;
  } tail;
};

__host__ __device__ __forceinline__ bool stage_matches(const kwk_stage_desc& s, uint32_t pred) {
  bool ok = ((pred ^ s.eq_val) & s.eq_mask) == 0;
  for (uint32_t k = 0; k < s.n_any; ++k) ok &= ((pred & s.any_mask[k]) != 0) == (((s.any_want >> k) & 1u) != 0);
  return ok;
}

// weight of matched stage s for this object (Stage.Weight)
__device__ __forceinline__ Getter stage_weight(const kwk_stage_desc& s, uint32_t sched,
                                               const kwk_value* __restrict__ rec) {
  return eval_getter(s.weight_slot, s.weight_default, true, sched, rec, KWK_DEL_ABSENT, 0, false);
}

// n-th (0-based) set bit of m
__device__ __forceinline__ int nth_bit(uint32_t m, int64_t n) {
  for (int64_t i = 0; i < n; ++i) m &= m - 1;
  return __ffs(m) - 1;
}

struct Fire {      // what one object's step produced
  bool fire;
  uint32_t stage;
  uint32_t flags;
  uint32_t bytes;  // algorithmic bytes beyond the 8-byte state read
};

// match + weighted pick + delay for one dirty object (preprocess, pod_controller.go:196-254).
// Updates sched (pending stage / MATCHERR) and due; returns true if a stage was scheduled.
// kProbe (fsm_build_kernel): evaluate for a state word alone; every step that needs more than
// the word (a value record, the deletion column, a Philox draw) sets `gen` instead.
// Matched-stage mask: the selector of a stage is a conjunction of per-bit tests (eq) and
// any-of clauses; when each clause lies within one byte of pred the stage is decided byte by
// byte, so the mask is the AND of one 256-entry table per pred byte (kwk_load_stages builds
// them; a program with <= 8 pred bits has one exact table).  Stages with a clause spanning
// bytes (lut_rest) run the clause loop.
__device__ __forceinline__ uint32_t match_mask(const kwk_stage_table* __restrict__ T, uint32_t n_stages,
                                               uint32_t pred, const uint32_t* lut, uint32_t lut_n,
                                               uint32_t lut_bytes, uint32_t lut_rest) {
  uint32_t m = 0;
  if (lut_n) {
    m = lut[pred & 0xFFu];
    if (lut_bytes > 1) m &= lut[256u | ((pred >> 8) & 0xFFu)];
    if (lut_bytes > 2) m &= lut[512u | ((pred >> 16) & 0xFFu)];
    if (lut_bytes > 3) m &= lut[768u | (pred >> 24)];
    for (uint32_t r = lut_rest; r; r &= r - 1) {
      const uint32_t s = (uint32_t)__ffs(r) - 1u;
      m |= (stage_matches(T->stages[s], pred) ? 1u : 0u) << s;
    }
  } else {
    for (uint32_t s = 0; s < n_stages; ++s) m |= (stage_matches(T->stages[s], pred) ? 1u : 0u) << s;
  }
  return m;
}

template <bool kProbe = false>
__device__ __forceinline__ bool match_object(const SweepArgs& a, const kwk_stage_table* __restrict__ T,
                                             uint32_t n_stages, uint64_t i, uint32_t pred, uint32_t& sched,
                                             int64_t& due, uint32_t& bytes, const uint32_t* lut, uint32_t lut_n,
                                             uint32_t& gen) {
  const uint32_t m = match_mask(T, n_stages, pred, lut, lut_n, a.lut_bytes, a.lut_rest);
  sched &= ~(KWK_F_DIRTY | KWK_F_MATCHERR);
  if (m == 0) return false;  // no match: a queued job stays queued (pod_controller.go:222-229)
  const kwk_value* __restrict__ rec = nullptr;
  if (sched & KWK_F_HASREC) {
    if constexpr (kProbe) { gen = 1; return false; }
    rec = a.values + (uint64_t)a.rec_idx[i] * a.value_slots;
    bytes += 4 + 16 * 3;  // record index + (at most) the picked stage's three entries
  }
  const uint64_t gslot = a.slot_base + i;
  int pick;
  const int cnt = __popc(m);
  // the object's draws: one Philox block when it may need the pick or a jitter (T->reserved[0]:
  // the stages with a Delay jitter, kwk_load_stages)
  uint64_t u_pick = 0, u_jit = 0;
  if (!kProbe && (cnt > 1 || (m & T->reserved[0]))) {
    uint32_t c0 = (uint32_t)gslot, c1 = (uint32_t)a.step, c2 = (uint32_t)(a.step >> 32), c3 = kSitePick;
    philox10(c0, c1, c2, c3, (uint32_t)a.key, (uint32_t)(a.key >> 32));
    u_pick = (uint64_t)c0 | ((uint64_t)c1 << 32);
    u_jit = (uint64_t)c2 | ((uint64_t)c3 << 32);
  }
  if (cnt == 1) {
    pick = __ffs(m) - 1;
  } else {
    if constexpr (kProbe) { gen = 1; return false; }  // weighted pick: a Philox draw (or a panic path)
    int64_t total = 0;
    int nerr = 0, nge0 = 0;
    for (uint32_t mm = m; mm; mm &= mm - 1) {
      const Getter w = stage_weight(T->stages[__ffs(mm) - 1], sched, rec);
      if (w.ok) {
        total = (int64_t)((uint64_t)total + (uint64_t)w.v);
        nge0 += w.v >= 0;
      } else {
        ++nerr;
      }
    }
    if (nerr == cnt || (total == 0 && nerr == 0)) {
      pick = nth_bit(m, below_u64(u_pick, cnt));                                    // lifecycle.go:157,163
    } else if (total == 0) {
      int64_t want = below_u64(u_pick, nge0);                                     // lifecycle.go:175
      pick = -1;
      for (uint32_t mm = m; mm; mm &= mm - 1) {
        const int s = __ffs(mm) - 1;
        const Getter w = stage_weight(T->stages[s], sched, rec);
        if (w.ok && w.v >= 0) {
          if (want == 0) { pick = s; break; }
          --want;
        }
      }
    } else if (total < 0) {
      sched |= KWK_F_MATCHERR;  // rand.Int63n panics on n <= 0 in the reference
      return false;
    } else {
      int64_t off = below_u64(u_pick, total);                                     // lifecycle.go:180
      pick = 31 - __clz(m);  // fallback: last matched stage (lifecycle.go:190)
      for (uint32_t mm = m; mm; mm &= mm - 1) {
        const int s = __ffs(mm) - 1;
        const Getter w = stage_weight(T->stages[s], sched, rec);
        const int64_t wv = w.ok ? w.v : -1;
        if (wv <= 0) continue;
        off -= wv;
        if (off < 0) { pick = s; break; }
      }
    }
  }
  // Stage.Delay (lifecycle.go:313-341); controllers ignore `ok` (pod_controller.go:234)
  const kwk_stage_desc& S = T->stages[pick];
  int64_t delay = 0;
  if (S.has_delay) {
    const bool need_del = S.delay_slot == KWK_SLOT_DELETION || S.jitter_slot == KWK_SLOT_DELETION;
    if constexpr (kProbe) {
      if (need_del) { gen = 1; return false; }
    }
    const int64_t dels = need_del ? a.del_s[i] : KWK_DEL_ABSENT;
    if (need_del) bytes += 8;
    const Getter d = eval_getter(S.delay_slot, S.delay_default, true, sched, rec, dels, a.now, true);
    if (d.ok) {
      delay = d.v;
      if (S.has_jitter) {
        const Getter j = eval_getter(S.jitter_slot, S.jitter_default, S.jitter_default_ok != 0, sched, rec, dels,
                                     a.now, true);
        if (j.ok) {
          if (j.v < delay) {
            delay = j.v;
          } else {
            const int64_t jit = (int64_t)((uint64_t)j.v - (uint64_t)delay);
            if constexpr (kProbe) {
              if (jit > 0) { gen = 1; return false; }
            }
            if (jit > 0)
              delay = (int64_t)((uint64_t)delay + (uint64_t)below_u64(u_jit, jit));
          }
        }
      }
    }
  }
  sched = (sched & ~0xFFu) | (uint32_t)pick;
  due = sat_add(a.now, delay);  // addStageJob / AddWeightAfter (weight_delaying_queue.go:73-95)
  return true;
}

// fire the pending stage (delay queue pop + playStage, pod_controller.go:257-360)
__device__ __forceinline__ void fire_object(const SweepArgs& a, const kwk_stage_table* __restrict__ T,
                                            const kwk_delta* __restrict__ deltas, uint32_t n_stages,
                                            uint32_t fin_group, uint32_t cls, uint32_t st, uint32_t& pred,
                                            uint32_t& sched, Fire& f) {
  const kwk_stage_desc& S = T->stages[st];
  f.fire = true;
  f.stage = st;
  const uint32_t pre = pred;
  // re-match iff the fire changed the object (its Modified watch event): always for
  // Now-dependent patches, for Now-independent ones only if not already applied
  bool rematch = (S.flags & KWK_NEXT_PATCHES) && (!(S.flags & KWK_NEXT_PATCH_STATIC) || !(pre & S.applied_mask));
  if (S.flags & KWK_NEXT_FIN) {  // finalizersModify (finalizers.go:83-111) as set algebra
    const uint32_t F = pre & fin_group;
    uint32_t F2;
    if ((S.flags & KWK_NEXT_FIN_EMPTY) || ((S.flags & KWK_NEXT_FIN_REMOVE) && (F & ~S.fin_remove) == 0))
      F2 = S.fin_add;
    else
      F2 = (F & ~S.fin_remove) | (S.fin_add & ~F);
    rematch |= F2 != F;
    pred = (pred & ~fin_group) | F2;
  }
  if (S.flags & KWK_NEXT_DELETE) {
    sched &= ~KWK_F_ALIVE;
    f.flags |= KWK_FIRED_DELETED;
    rematch = false;
  } else if (S.flags & KWK_NEXT_PATCHES) {
    const kwk_delta d = deltas[cls * n_stages + st];
    f.bytes += 2;
    if (d.and_mask == KWK_DELTA_UNKNOWN_AND && d.or_mask == KWK_DELTA_UNKNOWN_OR)
      f.flags |= KWK_FIRED_DELTA_UNKNOWN;
    else
      pred = (((pred & d.and_mask) | d.or_mask) & ~fin_group) | (pred & fin_group);
  }
  if (rematch) {
    sched |= KWK_F_DIRTY;
    f.flags |= KWK_FIRED_REMATCH;
  }
  sched |= KWK_STAGE_NONE;
}

// harness + match + fire for one object whose state needs work.  Returns the new state (the
// caller writes it back); writes the due column itself when a newly scheduled stage stays
// pending past this step (a stage that fires in the same step never needs its due stored).
// kProbe: see match_object; the due time a scheduled stage would store goes to due_w (gen and
// due_w are unused otherwise).  kDueOut (the fused format): the due time goes to due_w and gen = 1
// instead of the due column (the caller encodes it into the record)
template <bool kHarness, uint32_t kWordBytes, bool kProbe = false, bool kDueOut = false>
__device__ __forceinline__ uint2 process_object(const SweepArgs& a, const kwk_stage_table* __restrict__ T,
                                               const kwk_delta* __restrict__ deltas, uint32_t n_stages,
                                               uint32_t fin_group, uint64_t i, uint32_t pred, uint32_t sched,
                                               int64_t due, Fire& f, uint32_t& n_matched, const uint32_t* lut,
                                               uint32_t lut_n, uint32_t& gen, int64_t& due_w) {
  if (kHarness) {
    if (!(sched & KWK_F_ALIVE)) {  // re-create a deleted object from its spec
      pred &= a.harness.keep_mask;  // same spec: class bits and record flag stay
      sched = (sched & (KWK_F_MANAGED | KWK_F_HASREC | KWK_CLASS_MASK)) | KWK_F_ALIVE | KWK_F_DIRTY | KWK_STAGE_NONE;
      if (a.harness.track_deletion) {
        if constexpr (kProbe) gen = 1;
        else a.del_s[i] = KWK_DEL_ABSENT;
        f.bytes += 8;
      }
    } else if ((pred & a.harness.terminal_mask) && !(pred & a.harness.deletion_bit)) {
      pred |= a.harness.deletion_bit;  // the user deletes a finished pod
      int64_t sec = a.now / 1000000000;
      if (a.now % 1000000000 < 0) sec -= 1;
      if (a.harness.track_deletion) {
        if constexpr (kProbe) gen = 1;
        else a.del_s[i] = sec;
        f.bytes += 8;
      }
      sched |= KWK_F_DIRTY;
    }
  }
  bool scheduled = false;
  if (sched & KWK_F_ALIVE) {
    if (sched & KWK_F_DIRTY) {
      if (pred & T->disregard_mask) {
        // need() is false (disregardStatusWith{Annotation,Label}Selector, pod_controller.go:397-407,
        // node_controller.go:153-166): watchResources skips the event — no re-match, a queued job
        // stays queued (it still fires)
        sched &= ~KWK_F_DIRTY;
      } else {
        scheduled = match_object<kProbe>(a, T, n_stages, i, pred, sched, due, f.bytes, lut, lut_n, gen);
        n_matched += scheduled ? 1 : 0;
      }
    }
    const uint32_t st = sched & 0xFFu;
    if (a.fire && st < n_stages && due <= a.now) fire_object(a, T, deltas, n_stages, fin_group, sched >> KWK_CLASS_SHIFT, st,
                                                   pred, sched, f);
  }
  if (scheduled && (sched & 0xFFu) < n_stages) {
    if constexpr (kProbe) {
      due_w = due;
    } else if constexpr (kDueOut) {
      due_w = due;
      gen = 1;
    } else {
      a.due[i] = due;
    }
    if constexpr (!kDueOut) f.bytes += 8;  // fused: part of the record write below
  }
  f.bytes += kWordBytes;  // the state write-back (done by the caller)
  return make_uint2(pred, sched);
}

// wave-ballot compaction of the fired set into the wave's private segment + per-stage counts
// kPacked: 4-byte records {slot within the sweep region: 13 bits, stage: 5, flags: 3},
// expanded to kwk_fired_rec by compact_kernel (slot = region * region size + index; a region
// is a wave's words in sweep16_kernel, a tile's in sweepw_kernel)
template <bool kPacked = false>
__device__ __forceinline__ void emit_fired(const Fire& f, uint64_t i, uint32_t lane, kwk_fired_rec* __restrict__ seg,
                                           uint32_t& seg_n, unsigned int* s_stat, uint32_t& n_bytes) {
  const unsigned long long bal = __ballot(f.fire);
  if (!bal) return;
  if (f.fire) {
    const uint32_t pos = seg_n + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
    if constexpr (kPacked) {
      reinterpret_cast<uint32_t*>(seg)[pos] = (uint32_t)i | f.stage << 13 | f.flags << 18;
      n_bytes += 4;
    } else {
      seg[pos] = kwk_fired_rec{(uint32_t)i, (uint16_t)f.stage, (uint16_t)f.flags};
      n_bytes += 8;
    }
  }
  seg_n += (uint32_t)__popcll(bal);
  unsigned long long rest = bal;  // one LDS add per distinct fired stage
  while (rest) {
    const uint32_t s = __shfl(f.stage, __ffsll((long long)rest) - 1);
    const unsigned long long same = __ballot(f.fire && f.stage == s);
    if (lane == 0) atomicAdd(&s_stat[3 + s], (unsigned)__popcll(same));
    rest &= ~same;
  }
}

constexpr uint32_t kLutMax = 256;      // one match-mask table (programs with pred_bits <= 8)
constexpr uint32_t kLutTables = 1024;  // four byte tables (any pred width)
constexpr uint32_t kLutLdsW = 512;     // tables the word sweep stages in LDS (pred <= 16 bits)

// Streamed loads go through buffer resources (T8 in cdna_hip_programming.md): a load past the
// resource's byte size returns 0, so the tile tail and "load due only where a stage is
// pending" need no exec-mask branches (0 = MANAGED clear = never work).  Offsets are 32-bit:
// kwk_engine_create caps capacity so that capacity * 8 bytes fit.
constexpr uint32_t kOOB = 0xFFFFFFF0u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ int64_t buf_load_i64(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const auto t = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  return (int64_t)(((uint64_t)t[1] << 32) | t[0]);
}

// whole 128-byte line store of one lane's 16-byte chunk (8 lanes = one line), nontemporal:
// the state column is streamed once per step, keeping it out of L2 leaves room for the
// due / fired traffic (r1y: 122 -> 119 us)
__device__ __forceinline__ void store_chunk_nt(void* p, const uint4& v) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4*>(p));
}

// ------------------------------------------------------------------ 2-byte state transition table
// With 2-byte state words the compiled stage program is a finite state machine over at most
// 2^16 words: for every word (and whether its queued stage is due) fsm_build_kernel runs the
// same process_object as the sweep, in probe mode, once per stage-table / harness load.  An
// entry is marked general whenever the outcome needs more than the word (a Philox draw for a
// weighted pick or jitter, a value record, the deletion column); the sweep runs process_object
// for those and one table lookup for the rest.  Entry: [15:0] new word, [20:16] fired stage,
// [21] fired, [24:22] fired flags, [25] matched, [29:26] algorithmic bytes / 2, [30] writes
// due = now + fsm_due[entry], [31] general.
constexpr uint32_t kFsmDue = 1u << 30, kFsmGeneral = 1u << 31;

template <bool kHarness>
__global__ void fsm_build_kernel(SweepArgs a, uint32_t* __restrict__ tab, int64_t* __restrict__ dtab) {
  const uint32_t bits = a.fsm_bits;
  const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (2u << bits)) return;
  const uint32_t w = idx & ((1u << bits) - 1u), rdy = idx >> bits;
  const uint2 s = fmt_unpack(w, a.fmt);
  const kwk_stage_table* __restrict__ T = a.table;
  // probe clock: now = 0, a queued stage is due (0) or not yet (1)
  const int64_t due = ((s.y & 0xFFu) != KWK_STAGE_NONE) ? (rdy ? 0 : 1) : 0;
  Fire f{false, 0, 0, 0};
  uint32_t nm = 0, gen = 0;
  int64_t dw = INT64_MIN;  // set iff process_object stores a due time
  const uint2 nv = process_object<kHarness, 2, true>(a, T, a.deltas, T->n_stages, T->fin_group_mask, 0, s.x, s.y, due,
                                                     f, nm, a.lut, a.lut_n, gen, dw);
  uint32_t e = fmt_pack(nv.x, nv.y, a.fmt) & 0xFFFFu;
  e |= (f.stage & 31u) << 16 | (f.fire ? 1u : 0u) << 21 | (f.flags & 7u) << 22 | (nm & 1u) << 25;
  e |= ((f.bytes >> 1) & 15u) << 26;
  if (dw != INT64_MIN) e |= kFsmDue;
  if (gen || f.bytes > 30 || (f.bytes & 1u)) e = kFsmGeneral;
  tab[idx] = e;
  dtab[idx] = dw;
}

// ------------------------------------------------------------------ 2-byte state sweep
// Sweep over the 2-byte packed format (StateFmt.half: every shipped pod-fast / node stage set
// fits 16 bits).  At the steady-state churn of the C5 workload (~10 % of objects change per
// step) nearly every 128-byte line of the state column holds a changed word, so writing the
// changed words one by one costs a line fill plus a partial write per line once the line has
// left L2 (profiles/r1/README.md).  This kernel instead keeps the tile on chip and rewrites
// it as whole 128-byte lines:
//  phase 1  each lane streams Q 16-byte chunks (8 words each) of its wave's region (row q of
//           a wave = 1 KiB contiguous); due times only for lanes with a pending stage; the
//           idle test on the raw words; objects needing work are ballot-compacted into the
//           wave's LDS work list.  A wave with no work is done (no LDS, no stores);
//  phase 2  the chunks go to the wave's LDS tile; the heavy path runs over the dense work
//           list, reads and writes the word in LDS, emits fired records;
//  phase 3  every lane re-reads its chunks; each aligned group of 8 lanes (one 128-byte line)
//           with any changed word is stored whole from LDS (16 bytes per lane).
// Words past n are never work; chunks past n hold what was loaded (0 past the buffer range),
// so rewriting them is harmless inside the (tile-padded) allocation.
constexpr uint32_t kQ16 = 4;  // r1ao: Q = 4 at 4 blocks per CU 113.9 us / idle 42.8 us vs Q = 2 at 6: 116.6 / 47.8
constexpr int kWpe16 = 6;     // waves per SIMD the register allocation must allow (LDS allows 6 at Q = 2)
constexpr int kWpe16Q4 = 4;   // Q = 4: the LDS tile + work list allow 4 blocks per CU, so 128 VGPRs
constexpr int kLdsDeltas16 = 64;  // (class, stage) deltas staged in LDS by the 2-byte sweep (<= 11-bit programs)
constexpr uint32_t kStoreLanes = 8;  // phase-3 store group: 8 lanes x 16 bytes = one 128-byte line
// word offset (minus lane * 8) of bit b of a lane's phase-1 masks in the 2-byte sweep
__device__ __forceinline__ constexpr uint32_t bit_word(const uint32_t b) {
  return ((b & 15u) >> 2) * 512u + 2u * (b & 3u) + (b >> 4);
}
template <int Q>
constexpr uint32_t seg16_words() { return 64u * 8u * Q + 32u; }  // count + records + padding line
#define kSeg16 seg16_words<Q>()
template <bool kHarness, int Q, bool kPersist>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(Q >= 4 ? kWpe16Q4 : kWpe16))) void sweep16_kernel(SweepArgs a) {
  constexpr int K = 8 * Q;                 // words per lane
  constexpr uint32_t kWave = 64u * K;      // words per wave region
  constexpr uint32_t kTile = kBlock * K;   // words per block
  __shared__ unsigned int s_stat[kStatWords];
  __shared__ kwk_delta s_delta[kLdsDeltas16];
  __shared__ uint16_t s_work[kWavesPerBlock][kWave];
  __shared__ uint4 s_tile[kWavesPerBlock][64 * Q];
  __shared__ uint32_t s_lut[kLutMax];
  __shared__ kwk_stage_table s_tab;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = threadIdx.x >> 6;
  const uint32_t n_tiles = (uint32_t)(((uint64_t)a.n + kTile - 1) / kTile);
  // load range rounded to 16 bytes (the allocation is tile-padded): a chunk holding the last
  // words comes back whole
  const __amdgpu_buffer_rsrc_t st_rs = make_rsrc(a.st, ((a.n * 2u) + 15u) & ~15u);
  // one tile in flight per wave while the previous one is worked on (persistent grid): register
  // buffer va (a second buffer spilled VGPRs: 125-149 us, r1al)
  uint4 va[Q];
  auto issue_tile = [&](uint4 (&dst)[Q], const uint32_t t) {
    if (t >= n_tiles) return;
    const uint32_t wb = t * kTile + wave * kWave;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const auto c = __builtin_amdgcn_raw_buffer_load_b128(st_rs, (wb + (uint32_t)q * 512u + lane * 8u) * 2u, 0, 0);
      dst[q] = make_uint4(c[0], c[1], c[2], c[3]);
    }
  };
  uint32_t tile = blockIdx.x;
  issue_tile(va, tile);
  {  // LDS set-up overlaps the stream's latency
    const uint32_t nw = (offsetof(kwk_stage_table, stages) + a.table->n_stages * sizeof(kwk_stage_desc)) / 4;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(a.table);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&s_tab);
    for (uint32_t j = threadIdx.x; j < nw; j += kBlock) dst[j] = src[j];
  }
  const kwk_stage_table* __restrict__ T = &s_tab;
  const uint32_t n_stages = a.table->n_stages;
  const uint32_t fin_group = a.table->fin_group_mask;
  const uint32_t n_deltas = a.table->n_classes * n_stages;
  const uint32_t lut_n = a.lut_n;
  const uint32_t* __restrict__ lutp = lut_n <= kLutMax ? s_lut : a.lut;  // byte tables: read through L1
  if (lut_n <= kLutMax)
    for (uint32_t j = threadIdx.x; j < lut_n; j += kBlock) s_lut[j] = a.lut[j];
  if (threadIdx.x < kStatWords) s_stat[threadIdx.x] = 0;
  const kwk_delta* __restrict__ deltas = a.deltas;
  if (n_deltas <= kLdsDeltas16) {
    for (uint32_t j = threadIdx.x; j < n_deltas; j += kBlock) s_delta[j] = a.deltas[j];
    deltas = s_delta;
  }
  __syncthreads();

  const StateFmt fmt = a.fmt;
  const RawTest R = a.raw;
  // the idle test's masks doubled for both halves of a dword, and the shifts that move each
  // single-bit flag to bit 15 of its half (a zero mask yields a zero flag whatever the shift)
  struct {
    uint32_t m2, d2, a2, t2, l2, s2, n2;
    uint32_t sm, sd, sa, sl;
  } X;
  X.m2 = R.managed * 0x10001u; X.d2 = R.dirty * 0x10001u; X.a2 = R.alive * 0x10001u;
  X.t2 = R.term * 0x10001u; X.l2 = R.del * 0x10001u;
  // the stage field sits below the flags, so it never reaches bit 15: tested in place
  X.s2 = (R.smask << R.sshift) * 0x10001u; X.n2 = (R.none_code << R.sshift) * 0x10001u;
  X.sm = (uint32_t)(16 - __ffs(R.managed)) & 31u; X.sd = (uint32_t)(16 - __ffs(R.dirty)) & 31u;
  X.sa = (uint32_t)(16 - __ffs(R.alive)) & 31u; X.sl = (uint32_t)(16 - __ffs(R.del)) & 31u;
  uint32_t n_matched = 0, n_bytes = 0;  // per lane
  uint32_t n_line = 0;                  // per lane: line bytes - algorithmic bytes (mod 2^32)
  uint32_t wave_fired = 0;              // wave-uniform
  uint16_t* __restrict__ wl = s_work[wave];
  uint4* __restrict__ tq = s_tile[wave];
  uint16_t* __restrict__ tw = reinterpret_cast<uint16_t*>(tq);
  uint4* __restrict__ gq = reinterpret_cast<uint4*>(a.st);

  // one tile per block, or (kPersist) tiles blockIdx.x, +gridDim.x, ... with the next tile's
  // chunks in flight while this one runs phases 2 and 3
  auto tile_body = [&](uint4 (&v)[Q], const uint32_t tile) {
    const uint32_t wbase = tile * kTile + wave * kWave;  // the wave's first slot
    const bool full = (uint64_t)(tile + 1) * kTile <= a.n;
    uint32_t seg_n = 0;  // wave-uniform
    const uint64_t seg_id = (uint64_t)tile * kWavesPerBlock + wave;
    // the (tile, wave) segment: [count][packed 4-byte records ...], kSeg16 words apart; its
    // used part is padded to whole 128-byte lines (HBM3E has no write mask: a partial line
    // costs a read-modify-write), the count lives in the segment's first line
    uint32_t* __restrict__ seg32 = reinterpret_cast<uint32_t*>(a.fired) + seg_id * kSeg16;
    kwk_fired_rec* __restrict__ seg = reinterpret_cast<kwk_fired_rec*>(seg32 + 1);

    // the tile's words leave the prefetch buffer; the next tile's loads are issued before
    // phase 1, so they overlap this tile's idle test as well as phases 2-3 (r1as: 114.8 ->
    // 112.4 us against issuing them after phase 1)
    uint4 cur[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) cur[q] = v[q];
    if (kPersist) issue_tile(v, tile + gridDim.x);
    // ---- phase 1: idle test on the raw words.  bit k = q * 8 + h of a lane's masks
    // bit b of a lane's masks: dword (b & 15) of the lane's 4Q dwords (row (b & 15) / 4),
    // its low word for b < 16, its high word for b >= 16 (so the SWAR flags at bits 15 / 31
    // of each dword pack with one shift); word offset in the wave region: bit_word(b) + lane * 8
    constexpr uint32_t kHalfMask = (1u << (4 * Q)) - 1u;
    uint32_t in_range = kHalfMask | kHalfMask << 16;
    if (!full) {
      in_range = 0;
#pragma unroll
      for (int t = 0; t < K; ++t) {
        const int b = t < 4 * Q ? t : 16 + t - 4 * Q;
        in_range |= (wbase + bit_word((uint32_t)b) + lane * 8u < a.n ? 1u : 0u) << b;
      }
    }
    // two words per dword (SWAR): each test leaves its per-word flag at bit 15 / bit 31
    uint32_t pend = 0, need = 0, ready = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const uint32_t dw[4] = {cur[q].x, cur[q].y, cur[q].z, cur[q].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t d = dw[j];
        const uint32_t mg = (d & X.m2) << X.sm;
        const uint32_t pe = (((d & X.s2) ^ X.n2) + 0x7FFF7FFFu) & 0x80008000u;
        uint32_t nb = (d & X.d2) << X.sd;
        if (kHarness) {
          nb |= (~d & X.a2) << X.sa;
          nb |= (((d & X.t2) + 0x7FFF7FFFu) & 0x80008000u) & ~((d & X.l2) << X.sl);
        }
        const uint32_t n2 = mg & nb, p2 = mg & pe;
        const int jj = q * 4 + j;  // flags at bits 15 / 31 -> bits jj / 16 + jj
        need |= n2 >> (15 - jj);
        pend |= p2 >> (15 - jj);
      }
    }
    pend &= in_range;
    need &= in_range;
    if (__ballot(pend != 0)) {  // some object of the wave has a queued stage: is it due?
      const __amdgpu_buffer_rsrc_t due_rs = make_rsrc(a.due, a.n * 8u);
#pragma unroll 8
      for (int t = 0; t < K; ++t) {
        const int k = t < 4 * Q ? t : 16 + t - 4 * Q;
        const uint32_t p = (pend >> k) & 1u;
        const int64_t d = buf_load_i64(due_rs, p ? (wbase + bit_word((uint32_t)k) + lane * 8u) * 8u : kOOB);
        ready |= (p & (uint32_t)(d <= a.now)) << k;
      }
      need |= ready;
    }
    n_bytes += 2u * (uint32_t)__popc(in_range) + 8u * (uint32_t)__popc(pend);
    // work list in slot order: exclusive prefix of the per-lane counts (6 ballots, counts
    // <= 32), then each lane writes its own entries
    uint32_t n_work = 0, pos = 0;  // n_work wave-uniform
    {
      const uint32_t cnt = (uint32_t)__popc(need);
      const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
      for (int b = 0; b < 6; ++b) {
        const unsigned long long bal = __ballot((cnt >> b) & 1u);
        pos += (uint32_t)__popcll(bal & lt) << b;
        n_work += (uint32_t)__popcll(bal) << b;
      }
      for (uint32_t m = need; m; m &= m - 1u) {
        const uint32_t k = (uint32_t)__ffs(m) - 1u;
        wl[pos++] = (uint16_t)(bit_word(k) + lane * 8u + (((ready >> k) & 1u) << 15));
      }
    }

    if (n_work) {
      // ---- phase 2
#pragma unroll
      for (int q = 0; q < Q; ++q) tq[q * 64 + lane] = cur[q];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      // Software-pipelined passes of 64 work items: the next pass's work-list / tile reads and
      // table lookup are issued before this pass's stores (fired records, due), so waiting
      // for the lookup does not wait for those stores (vmcnt counts loads and stores in issue
      // order).
      auto fetch = [&](const uint32_t c, uint32_t& we, uint32_t& raw, uint32_t& ent) {
        we = (c + lane < n_work) ? (uint32_t)wl[c + lane] : 0xFFFFFFFFu;
        raw = we != 0xFFFFFFFFu ? (uint32_t)tw[we & 0x7FFFu] : 0u;
        ent = (we != 0xFFFFFFFFu && a.fsm) ? a.fsm[((we >> 15) << a.fsm_bits) | raw] : kFsmGeneral;
      };
      uint32_t we, raw, ent;
      fetch(0, we, raw, ent);
      for (uint32_t c = 0; c < n_work; c += 64u) {
        const uint32_t cwe = we, craw = raw, e = ent;
        if (c + 64u < n_work) fetch(c + 64u, we, raw, ent);  // wave-uniform
        Fire f{false, 0, 0, 0};
        uint64_t i = 0;
        if (cwe != 0xFFFFFFFFu) {
          const uint32_t w = cwe & 0x7FFFu, rdy = cwe >> 15;  // slot in the wave region, due ready
          i = wbase + w;
          if (!(e & kFsmGeneral)) {  // the word's transition, precomputed by fsm_build_kernel
            tw[w] = (uint16_t)e;
            if (e & kFsmDue) a.due[i] = sat_add(a.now, a.fsm_due[(rdy << a.fsm_bits) | craw]);
            f.fire = (e >> 21) & 1u;
            f.stage = (e >> 16) & 31u;
            f.flags = (e >> 22) & 7u;
            f.bytes = ((e >> 26) & 15u) * 2u;
            n_matched += (e >> 25) & 1u;
          } else {
            const uint2 s = fmt_unpack(craw, fmt);
            const int64_t due = ((s.y & 0xFFu) != KWK_STAGE_NONE) ? a.due[i] : 0;  // counted in phase 1
            uint32_t gen_unused = 0;
            int64_t due_unused = 0;
            const uint2 nv = process_object<kHarness, 2>(a, T, deltas, n_stages, fin_group, i, s.x, s.y, due, f,
                                                         n_matched, lutp, lut_n, gen_unused, due_unused);
            tw[w] = (uint16_t)fmt_pack(nv.x, nv.y, fmt);
          }
          n_line -= 2u;  // the word's own write is replaced by the line stores below
        }
        n_bytes += f.bytes;
        emit_fired<true>(f, i - wbase, lane, seg, seg_n, s_stat, n_bytes);
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      // ---- phase 3: whole 128-byte lines wherever a word changed
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const uint4 nv = tq[q * 64 + lane];
        const bool ch = (nv.x ^ cur[q].x) | (nv.y ^ cur[q].y) | (nv.z ^ cur[q].z) | (nv.w ^ cur[q].w);
        const unsigned long long bal = __ballot(ch);
        if ((bal >> (lane & ~(kStoreLanes - 1u))) & ((1ull << kStoreLanes) - 1ull)) {
          store_chunk_nt(&gq[(wbase + (uint32_t)q * 512u + lane * 8u) / 8u], nv);
          n_line += 16u;
        }
      }
      // the next tile reuses this wave's LDS lists and tile
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    {
      const uint32_t used = 1u + seg_n, end = (used + 31u) & ~31u;
      for (uint32_t x = used + lane; x < end; x += 64) seg32[x] = 0u;
      if (lane == 0) {
        seg32[0] = seg_n;
        a.wave_counts[seg_id] = seg_n;  // the hand-back's scan input
      }
      n_line += 4u * (uint32_t)__popc((uint32_t)(lane < end - used));  // padding: line bytes only
    }
    wave_fired += seg_n;
    n_bytes += lane == 0 ? 4u : 0u;  // the fired count word
  };
  if constexpr (!kPersist) {
    if (tile < n_tiles) tile_body(va, tile);
  } else {
    for (; tile < n_tiles; tile += gridDim.x) tile_body(va, tile);
  }

  // ---- block statistics
  for (int off = 32; off > 0; off >>= 1) {
    n_matched += __shfl_xor(n_matched, off);
    n_bytes += __shfl_xor(n_bytes, off);
    n_line += __shfl_xor(n_line, off);
  }
  if (lane == 0) {
    atomicAdd(&s_stat[0], n_matched);
    atomicAdd(&s_stat[1], wave_fired);
    atomicAdd(&s_stat[2], n_bytes);
    atomicAdd(&s_stat[kStatLine], n_bytes + n_line);
  }
  __syncthreads();
  if (threadIdx.x < 3 + n_stages || threadIdx.x == kStatLine) {
    const unsigned int val = s_stat[threadIdx.x];
    if (val) atomicAdd(&a.cum[(uint64_t)blockIdx.x * kStatWords + threadIdx.x], (unsigned long long)val);
  }
}

// ------------------------------------------------------------------ 2-byte sweep, transition table only
// sweep16_kernel with every object's step a lookup: chosen when the transition table holds no
// general entry (no Philox draw, value record or deletion column anywhere in the compiled
// program — pod-fast, node-fast), so process_object is not compiled in.  sweep16_kernel is
// VALU-bound at C5 (r1 SQ passes: ~1230 VALU per wave and tile, ~700 of them in phase 2, whose
// register pressure from the inlined general path spills SGPRs to VGPR lanes); here a 64-item
// pass is ~30 VALU.  Same phases, tiles, records, statistics and write-back as sweep16_kernel;
// the ordering differs where the memory counter is in order (gfx9 vmcnt):
//  * the table lookups of up to kFsmBatch passes are issued together, then the next tile's
//    loads (kDepth tiles ahead), so waiting for a lookup never waits for the HBM prefetch;
//  * the due loads of phase 1 come before the prefetch for the same reason;
//  * lookups, fired records and due times go through buffer resources (32-bit offsets; an
//    inactive lane's offset is out of range: loads return 0, stores are dropped).
// Cold path of sweep16_fsm_kernel: a word whose table entry is general (a Philox draw, a value
// record or the deletion column) runs process_object with the stage table, match masks and
// deltas read from global memory (L2).  Returns the entry the table would hold ({new word,
// fired stage / flag / flags, matched} without kFsmDue: the due time is already stored) and the
// algorithmic bytes.  (Inlined.  A round-2 build that made this a `noinline` function taking the
// kernel's SweepArgs by reference faulted twice — the one-block-per-tile Q = 1 node engine of
// test_node_fast_heartbeat and the C5 bench — and was reverted; DESIGN.md §5 records what its ISA
// shows and why the shared code it called is not the cause.)
template <bool kHarness>
__device__ __forceinline__ uint2 general16(uint32_t i, uint32_t raw) {
  // the kernel's SweepArgs (its only argument, at offset 0 of the kernarg segment) and the stage
  // table are read through a VGPR address: their values land in VGPRs, which the lookup loop
  // leaves free, instead of taking SGPRs from it (SGPR spills into VGPR lanes cost ~4 us)
  uint64_t ka = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+v"(ka));
  const SweepArgs& a = *reinterpret_cast<const SweepArgs*>(ka);
  uint64_t tp = (uint64_t)a.table;
  asm volatile("" : "+v"(tp));
  const kwk_stage_table* __restrict__ T = reinterpret_cast<const kwk_stage_table*>(tp);
  const uint2 s = fmt_unpack(raw, a.fmt);
  const int64_t due = ((s.y & 0xFFu) != KWK_STAGE_NONE) ? a.due[i] : 0;
  Fire f{false, 0, 0, 0};
  uint32_t nm = 0, gen_unused = 0;
  int64_t due_unused = 0;
  const uint2 nv = process_object<kHarness, 2>(a, T, a.deltas, T->n_stages, T->fin_group_mask, i, s.x, s.y, due, f, nm,
                                               a.lut, a.lut_n, gen_unused, due_unused);
  uint32_t e = fmt_pack(nv.x, nv.y, a.fmt) & 0xFFFFu;
  e |= (f.stage & 31u) << 16 | (f.fire ? 1u : 0u) << 21 | (f.flags & 7u) << 22 | (nm & 1u) << 25;
  return make_uint2(e, f.bytes);
}

// The prefix of a block's count over the blocks of one launch (status word per block, `stride`
// words apart: seq << 32 | count).  One wave: publishes the block's count, then loads the words of
// every block before it — 16 per lane in flight at once, so one memory round trip up to 1024
// blocks — re-reading (with back-off) only those not published yet: blocks are dispatched in index
// order, so each of them has started, and none waits on a later one.  Returns the exclusive
// prefix.
__device__ __forceinline__ uint32_t block_prefix(unsigned long long* status, uint32_t stride, uint32_t b, uint32_t bt,
                                                 uint32_t seq, uint32_t lane) {
  if (lane == 0)
    __hip_atomic_store(&status[(uint64_t)b * stride], (unsigned long long)seq << 32 | bt, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  constexpr uint32_t kIn = 16;  // loads in flight per lane
  uint32_t pre = 0;
  for (uint32_t j0 = lane; j0 < b; j0 += 64u * kIn) {  // wave-uniform trip count: ceil(b / 1024)
    unsigned long long v[kIn];
#pragma unroll
    for (uint32_t k = 0; k < kIn; ++k) {
      const uint32_t j = j0 + 64u * k;
      v[k] = j < b ? __hip_atomic_load(&status[(uint64_t)j * stride], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                   : (unsigned long long)seq << 32;
    }
#pragma unroll
    for (uint32_t k = 0; k < kIn; ++k) {
      const uint32_t j = j0 + 64u * k;
      while ((uint32_t)(v[k] >> 32) != seq) {  // a block before this one still sweeping: back off
        __builtin_amdgcn_s_sleep(2);
        v[k] = __hip_atomic_load(&status[(uint64_t)j * stride], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      pre += (uint32_t)v[k];
    }
  }
  for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o);
  return pre;
}

// The hand-back inside a one-tile-per-block sweep (small sweeps: the node kinds, the strong-scaling
// shards' node engines; the bench's N = 8 shard step was bound by the node engine's chain of two
// launches per step): each block finds its offset by block_prefix above and copies its waves'
// records to the dense list.  Only for grids resident in one dispatch round: no block exits before
// every block before it has finished its tile, so a second round would start only after the whole
// first one (the same hand-back inside the N = 8 shard's 1526-block pod sweep, more workgroups
// than its CUs hold at once: 51-59 vs 23 us per 4-step launch, r6q-r6t; not kept).  Taken for
// grids of at most a quarter as many workgroups as CUs: at the 125k-node shard (62) it shortens
// the node chain, at 250k / 500k (123 / 245) the step was 0.7-1.3 us slower with it (r6v)  The list (order, slots, record layout) is compact_small_kernel's:
// segments in order, each segment's records in order.
template <uint32_t kWaveSlots, uint32_t kSegWords>
__device__ __forceinline__ void tail_handback(const SweepArgs& a, uint32_t wave_n, uint32_t lane, uint32_t wave) {
  __shared__ uint32_t s_wn[kWavesPerBlock];
  __shared__ uint32_t s_pre;
  const SweepArgs::TailHb& t = a.tail;
  // the block's segments (buffer stores) complete before its waves read them back below (a
  // workgroup-scope fence: an agent-scope one writes the XCD's L2 back, r6h: the node step 7.6 ->
  // 18.4 us).  The status words need none: agent-scope atomics are coherent across the XCDs' L2s
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane == 0) s_wn[wave] = wave_n;
  __syncthreads();
  const uint32_t bt = s_wn[0] + s_wn[1] + s_wn[2] + s_wn[3];
  if (wave == 0) {
    const uint32_t pre = block_prefix(t.status, 1u, blockIdx.x, bt, t.seq, lane);
    if (lane == 0) s_pre = pre;
  }
  __syncthreads();
  uint32_t off = s_pre;
  for (uint32_t w = 0; w < wave; ++w) off += s_wn[w];
  const uint64_t seg_id = (uint64_t)blockIdx.x * kWavesPerBlock + wave;
  const uint32_t* __restrict__ sp = reinterpret_cast<const uint32_t*>(a.fired) + seg_id * kSegWords;
  const uint32_t base = (uint32_t)seg_id * kWaveSlots;
  for (uint32_t j = lane; j < wave_n; j += 64u) {
    const uint32_t x = sp[1u + j];
    const uint32_t slot = base + (x & 0x1FFFu);
    if (t.packed) {
      __builtin_nontemporal_store(((x >> 13) & 31u) << 27 | slot, reinterpret_cast<uint32_t*>(t.out) + off + j);
    } else {
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      __builtin_nontemporal_store(u32x2{slot, ((x >> 13) & 31u) | ((x >> 18) & 7u) << 16},
                                  reinterpret_cast<u32x2*>(reinterpret_cast<kwk_fired_rec*>(t.out) + off + j));
    }
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    t.offsets[0] = s_pre + bt;
    if (t.host_len) t.host_len[0] = s_pre + bt;
  }
}

constexpr int kFsmBatch = 4;  // passes (64 work items each) whose lookups are in flight together
constexpr uint32_t kFsmKernelDefault = 2;  // table-only sweep with its prefetch depth (0: never)
template <bool kHarness, int Q, bool kPersist, int kDepth>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(Q >= 4 ? 4 : 5))) void sweep16_fsm_kernel(SweepArgs a) {
  constexpr int K = 8 * Q;                 // words per lane
  constexpr uint32_t kWave = 64u * K;      // words per wave region
  constexpr uint32_t kTile = kBlock * K;   // words per block
  constexpr int B = kFsmBatch;
  static_assert(kDepth >= 1 && kDepth <= 2 && (kPersist || kDepth == 1), "prefetch depth");
  __shared__ unsigned int s_stat[kStatWords];
  __shared__ uint16_t s_work[kWavesPerBlock][kWave];
  __shared__ uint4 s_tile[kWavesPerBlock][64 * Q];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // scalar: segment resources stay in SGPRs
  const uint32_t n_tiles = (uint32_t)(((uint64_t)a.n + kTile - 1) / kTile);
  const __amdgpu_buffer_rsrc_t st_rs = make_rsrc(a.st, ((a.n * 2u) + 15u) & ~15u);
  const __amdgpu_buffer_rsrc_t due_rs = make_rsrc(a.due, a.n * 8u);
  const uint32_t fbits = a.fsm_bits;
  const __amdgpu_buffer_rsrc_t fsm_rs = make_rsrc(a.fsm, 4u << (fbits + 1));
  const __amdgpu_buffer_rsrc_t fdue_rs = make_rsrc(a.fsm_due, 8u << (fbits + 1));
  uint4 va[kDepth][Q];
  // always Q loads (out of range past the last tile: zeros), so that the compiler's in-order
  // wait counts are the same on every path
  auto issue_tile = [&](uint4 (&dst)[Q], const uint32_t t) __attribute__((always_inline)) {
    const uint32_t off = t < n_tiles ? (t * kTile + wave * kWave + lane * 8u) * 2u : kOOB - 4u * 1024u;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const auto c = __builtin_amdgcn_raw_buffer_load_b128(st_rs, off + (uint32_t)q * 1024u, 0, 0);
      dst[q] = make_uint4(c[0], c[1], c[2], c[3]);
    }
  };
  uint32_t tile = blockIdx.x;
  issue_tile(va[0], tile);
  if (kDepth > 1) issue_tile(va[1], tile + gridDim.x);
  const uint32_t n_stages = a.table->n_stages;
  if (threadIdx.x < kStatWords) s_stat[threadIdx.x] = 0;
  __syncthreads();

  const RawTest R = a.raw;
  struct {
    uint32_t m2, d2, a2, t2, l2, s2, n2;
    uint32_t sm, sd, sa, sl;
  } X;
  X.m2 = R.managed * 0x10001u; X.d2 = R.dirty * 0x10001u; X.a2 = R.alive * 0x10001u;
  X.t2 = R.term * 0x10001u; X.l2 = R.del * 0x10001u;
  X.s2 = (R.smask << R.sshift) * 0x10001u; X.n2 = (R.none_code << R.sshift) * 0x10001u;
  X.sm = (uint32_t)(16 - __ffs(R.managed)) & 31u; X.sd = (uint32_t)(16 - __ffs(R.dirty)) & 31u;
  X.sa = (uint32_t)(16 - __ffs(R.alive)) & 31u; X.sl = (uint32_t)(16 - __ffs(R.del)) & 31u;
  uint32_t stc01 = 0, stc23 = 0;        // per lane: fired records of stages 0 | 1 << 16, 2 | 3 << 16
  uint32_t n_matched = 0, n_bytes = 0;  // per lane: matches, algorithmic bytes
  uint32_t n_lline = 0;                 // per lane: bytes of the phase-3 line stores
  uint32_t w_bytes = 0, w_line = 0;     // wave-uniform: algorithmic bytes, line bytes - algorithmic bytes (mod 2^32)
  uint32_t wave_fired = 0;              // wave-uniform
  uint16_t* __restrict__ wl = s_work[wave];
  uint4* __restrict__ tq = s_tile[wave];
  uint16_t* __restrict__ tw = reinterpret_cast<uint16_t*>(tq);
  uint4* __restrict__ gq = reinterpret_cast<uint4*>(a.st);

  // kDepth 1: the tile's words are copied out of v and v receives the next tile's loads right
  // after this tile's lookups; kDepth 2 (ping-pong over va[0] / va[1]): the tile is worked on in
  // v itself, which receives the tile 2 grid strides ahead once this one is written back
  auto tile_body = [&](uint4 (&v)[Q], const uint32_t tile) __attribute__((always_inline)) {
    const uint32_t wbase = tile * kTile + wave * kWave;
    const bool full = (uint64_t)(tile + 1) * kTile <= a.n;
    uint32_t seg_n = 0;  // wave-uniform
    const uint64_t seg_id = (uint64_t)tile * kWavesPerBlock + wave;
    uint32_t* __restrict__ seg32 = reinterpret_cast<uint32_t*>(a.fired) + seg_id * kSeg16;
    const __amdgpu_buffer_rsrc_t seg_rs = make_rsrc(seg32, kSeg16 * 4u);
    uint4 cur_copy[Q];
    if (kDepth == 1) {
#pragma unroll
      for (int q = 0; q < Q; ++q) cur_copy[q] = v[q];
    }
    uint4 (&cur)[Q] = kDepth == 1 ? cur_copy : v;
    // ---- phase 1 (as sweep16_kernel); in a partial tile, row q of the lane holds
    // c = clamp(n - first word, 0, 8) words: its low words are bits q*4 + [0, (c+1)/2), its
    // high words bits 16 + q*4 + [0, c/2) (no per-bit constants: they would pin ~25 VGPRs)
    constexpr uint32_t kHalfMask = (1u << (4 * Q)) - 1u;
    uint32_t in_range = kHalfMask | kHalfMask << 16;
    if (!full) {
      in_range = 0;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int64_t left = (int64_t)a.n - (int64_t)(wbase + (uint32_t)q * 512u + lane * 8u);
        const uint32_t c = left <= 0 ? 0u : left >= 8 ? 8u : (uint32_t)left;
        in_range |= (((1u << ((c + 1u) >> 1)) - 1u) << (4 * q)) | (((1u << (c >> 1)) - 1u) << (16 + 4 * q));
      }
    }
    uint32_t pend = 0, need = 0, ready = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const uint32_t dw[4] = {cur[q].x, cur[q].y, cur[q].z, cur[q].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t d = dw[j];
        const uint32_t mg = (d & X.m2) << X.sm;
        const uint32_t pe = (((d & X.s2) ^ X.n2) + 0x7FFF7FFFu) & 0x80008000u;
        uint32_t nb = (d & X.d2) << X.sd;
        if (kHarness) {
          nb |= (~d & X.a2) << X.sa;
          nb |= (((d & X.t2) + 0x7FFF7FFFu) & 0x80008000u) & ~((d & X.l2) << X.sl);
        }
        const uint32_t n2 = mg & nb, p2 = mg & pe;
        const int jj = q * 4 + j;
        need |= n2 >> (15 - jj);
        pend |= p2 >> (15 - jj);
      }
    }
    pend &= in_range;
    need &= in_range;
    if (__ballot(pend != 0)) {
#pragma unroll 8
      for (int t = 0; t < K; ++t) {
        const int k = t < 4 * Q ? t : 16 + t - 4 * Q;
        const uint32_t p = (pend >> k) & 1u;
        const int64_t d = buf_load_i64(due_rs, p ? (wbase + bit_word((uint32_t)k) + lane * 8u) * 8u : kOOB);
        ready |= (p & (uint32_t)(d <= a.now)) << k;
      }
      need |= ready;
    }
    n_bytes += 2u * (uint32_t)__popc(in_range) + 8u * (uint32_t)__popc(pend);
    uint32_t n_work = 0, pos = 0;
    {
      const uint32_t cnt = (uint32_t)__popc(need);
      const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
      for (int b = 0; b < 6; ++b) {
        const unsigned long long bal = __ballot((cnt >> b) & 1u);
        pos += (uint32_t)__popcll(bal & lt) << b;
        n_work += (uint32_t)__popcll(bal) << b;
      }
      for (uint32_t m = need; m; m &= m - 1u) {
        const uint32_t k = (uint32_t)__ffs(m) - 1u;
        wl[pos++] = (uint16_t)(bit_word(k) + lane * 8u + (((ready >> k) & 1u) << 15));
      }
    }
    // ---- phase 2: lookups of the first kFsmBatch passes (straight-line code, so the
    // compiler's wait for a lookup counts the prefetch issued after it), then the prefetch
    uint32_t we[B], raw[B], ent[B];
    auto fetch = [&](const uint32_t c0) __attribute__((always_inline)) {
#pragma unroll
      for (int b = 0; b < B; ++b) {
        const uint32_t c = c0 + 64u * b + lane;
        const bool in = c < n_work;
        const uint32_t x0 = (uint32_t)wl[c & (kWave - 1u)];  // read unconditionally (no exec branch)
        const uint32_t x = in ? x0 : 0u;
        we[b] = in ? x : 0xFFFFFFFFu;
        raw[b] = (uint32_t)tw[x & 0x7FFFu];
        ent[b] = __builtin_amdgcn_raw_buffer_load_b32(fsm_rs, in ? ((((x >> 15) << fbits) | raw[b]) * 4u) : kOOB, 0, 0);
      }
    };
    // fired record + per-stage counts of one 64-item pass (e: the item's table entry)
    auto emit = [&](const bool fire, const uint32_t w, const uint32_t e) __attribute__((always_inline)) {
      const unsigned long long bal = __ballot(fire);
      if (bal) {
        const uint32_t pos = seg_n + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        const uint32_t rec = w | ((e >> 16) & 31u) << 13 | ((e >> 22) & 7u) << 18;
        __builtin_amdgcn_raw_buffer_store_b32(rec, seg_rs, fire ? (1u + pos) * 4u : kOOB, 0, 0);
        const uint32_t nf = (uint32_t)__popcll(bal);
        seg_n += nf;
        w_bytes += 4u * nf;
        const uint32_t code = fire ? ((e >> 16) & 31u) : 31u;
        if (n_stages <= 4) {  // per-lane 16-bit counters, stages 0-1 / 2-3 (reduced once per block)
          const uint32_t inc = 1u << (16u * (code & 1u));
          stc01 += code < 2u ? inc : 0u;
          stc23 += (code - 2u) < 2u ? inc : 0u;
        } else {
          for (uint32_t st = 0; st < n_stages; ++st) {  // one ballot per stage
            const unsigned long long same = __ballot(code == st);
            if (same && lane == 0) atomicAdd(&s_stat[3 + st], (unsigned)__popcll(same));
          }
        }
      }
    };
    // Items whose entry is general are deferred to one loop after the lookups (records are
    // unordered within a region): their slots are compacted to the front of the work list,
    // whose entries up to the current batch are already in registers; their words stay
    // unchanged in the LDS tile until then.
    uint32_t n_gen = 0;  // wave-uniform
    auto pass = [&](const int b) __attribute__((always_inline)) {
      const uint32_t cwe = we[b], e = ent[b];
      const bool act = cwe != 0xFFFFFFFFu;
      const uint32_t w = cwe & 0x7FFFu;
      const bool gen = act && (e & kFsmGeneral);
      const unsigned long long gb = __ballot(gen);
      if (gb) {
        if (gen) wl[n_gen + __builtin_amdgcn_mbcnt_hi((uint32_t)(gb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)gb, 0u))] = (uint16_t)w;
        n_gen += (uint32_t)__popcll(gb);
      }
      const bool tab = act && !gen;
      if (tab) {
        tw[w] = (uint16_t)e;
        n_matched += (e >> 25) & 1u;
        n_bytes += ((e >> 26) & 15u) * 2u;
      }
      const bool dw = tab && (e & kFsmDue);
      if (__ballot(dw)) {  // a delayed stage is scheduled (rare for table-only programs)
        const int64_t dd = buf_load_i64(fdue_rs, dw ? ((((cwe >> 15) << fbits) | raw[b]) * 8u) : kOOB);
        const int64_t v = sat_add(a.now, dd);
        const uint32_t off = dw ? (wbase + w) * 8u : kOOB;
        __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v, due_rs, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32((uint32_t)((uint64_t)v >> 32), due_rs, off + 4u, 0, 0);
      }
      emit(tab && ((e >> 21) & 1u), w, e);
    };
    if (n_work) {
#pragma unroll
      for (int q = 0; q < Q; ++q) tq[q * 64 + lane] = cur[q];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      fetch(0);
    }
    if (kPersist && kDepth == 1) issue_tile(v, tile + gridDim.x);
    if (n_work) {
#pragma unroll
      for (int b = 0; b < B; ++b)
        if (64u * b < n_work) pass(b);  // wave-uniform
      for (uint32_t c0 = 64u * B; c0 < n_work; c0 += 64u * B) {  // more than kFsmBatch passes
        fetch(c0);
#pragma unroll
        for (int b = 0; b < B; ++b)
          if (c0 + 64u * b < n_work) pass(b);
      }
      // cold: the general items (a Philox draw, a value record or the deletion column)
      for (uint32_t j = 0; j < n_gen; j += 64u) {
        const bool in = j + lane < n_gen;
        const uint32_t w = in ? (uint32_t)wl[j + lane] : 0u;
        uint32_t e = 0;
        if (in) {
          const uint2 r = general16<kHarness>(wbase + w, (uint32_t)tw[w]);
          e = r.x;
          tw[w] = (uint16_t)e;
          n_matched += (e >> 25) & 1u;
          n_bytes += r.y;
        }
        emit(in && ((e >> 21) & 1u), w, e);
      }
      w_line -= 2u * n_work;  // the words' own writes are replaced by the line stores below
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      // ---- phase 3: whole 128-byte lines wherever a word changed
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const uint4 nv = tq[q * 64 + lane];
        const bool ch = (nv.x ^ cur[q].x) | (nv.y ^ cur[q].y) | (nv.z ^ cur[q].z) | (nv.w ^ cur[q].w);
        const unsigned long long bal = __ballot(ch);
        if ((bal >> (lane & ~(kStoreLanes - 1u))) & ((1ull << kStoreLanes) - 1ull)) {
          store_chunk_nt(&gq[(wbase + (uint32_t)q * 512u + lane * 8u) / 8u], nv);
          n_lline += 16u;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    {
      const uint32_t used = 1u + seg_n, end = (used + 31u) & ~31u;
      for (uint32_t x = used + lane; x < end; x += 64) seg32[x] = 0u;
      if (lane == 0) {
        seg32[0] = seg_n;
        a.wave_counts[seg_id] = seg_n;
      }
      w_line += 4u * (end - used);  // padding: line bytes only
    }
    wave_fired += seg_n;
    w_bytes += 4u;  // the fired count word
    if (kPersist && kDepth == 2) issue_tile(v, tile + 2u * gridDim.x);
  };
  if constexpr (!kPersist) {
    if (tile < n_tiles) tile_body(va[0], tile);
  } else if constexpr (kDepth == 1) {
    for (; tile < n_tiles; tile += gridDim.x) tile_body(va[0], tile);
  } else {
    for (; tile < n_tiles; tile += 2u * gridDim.x) {
      tile_body(va[0], tile);
      if (tile + gridDim.x >= n_tiles) break;
      tile_body(va[1], tile + gridDim.x);
    }
  }

  // ---- block statistics
  for (int off = 32; off > 0; off >>= 1) {
    n_matched += __shfl_xor(n_matched, off);
    n_bytes += __shfl_xor(n_bytes, off);
    n_lline += __shfl_xor(n_lline, off);
  }
  uint32_t stn[4] = {stc01 & 0xFFFFu, stc01 >> 16, stc23 & 0xFFFFu, stc23 >> 16};
#pragma unroll
  for (int st = 0; st < 4; ++st)
    for (int off = 32; off > 0; off >>= 1) stn[st] += __shfl_xor(stn[st], off);
  if (lane == 0) {
#pragma unroll
    for (int st = 0; st < 4; ++st)
      if (stn[st]) atomicAdd(&s_stat[3 + st], stn[st]);
    atomicAdd(&s_stat[0], n_matched);
    atomicAdd(&s_stat[1], wave_fired);
    atomicAdd(&s_stat[2], n_bytes + w_bytes);
    atomicAdd(&s_stat[kStatLine], n_bytes + w_bytes + n_lline + w_line);
  }
  __syncthreads();
  if (threadIdx.x < 3 + n_stages || threadIdx.x == kStatLine) {
    const unsigned int val = s_stat[threadIdx.x];
    if (val) atomicAdd(&a.cum[(uint64_t)blockIdx.x * kStatWords + threadIdx.x], (unsigned long long)val);
  }
  if constexpr (!kPersist) {
    if (a.tail.out) tail_handback<kWave, kSeg16>(a, tile < n_tiles ? wave_fired : 0u, lane, wave);
  }
}

// ------------------------------------------------------------------ 1-byte state sweep
// When the compiled program is a finite state machine that needs nothing beyond the 2-byte word
// (pod-fast, node-fast: no Philox draw, value record or deletion column reachable) the words
// that can occur are few — the closure of the resident words under the transition table, delete,
// the lease MANAGED / DIRTY updates and upserts: 44 for pod-fast with the bench harness, 20 for
// node-fast + heartbeat — so the device keeps one byte per object, an index into a dictionary of
// at most 255 words.  The id's top bits carry what phase 1 tests:
//   bit 7  the word needs work whatever its due time (managed, and dirty or harness churn)
//   bit 6  a stage is queued on a managed object (work once its due time has passed)
//   bit 5  alive (usage / counts)        bits 0-4: index within that class
// so the idle test is two mask-and-shift ops per 4 objects, and the transition of a work item
// is one lookup in a 512-entry id table staged in LDS (no L2 gather).  The column halves: the
// C5 state stream is 100 MB instead of 200 MB, read once and rewritten as whole 128-byte lines.
constexpr uint32_t kIdNeed = 0x80u, kIdPend = 0x40u, kIdAlive = 0x20u, kIdIndex = 0x1Fu;
constexpr uint32_t kIdInvalid = 0xFFu;  // not in the dictionary (never stored: the host closes it)
constexpr int kQ8 = 2;                  // 16-byte chunks per lane: 32 ids per lane, 2048 per wave
// id transition entry (dict_upload): [7:0] new id, [15:11] the 2-byte fired record's high bits
// (stage 11-12 when the program has <= 4 stages, flags 13-15), [20:16] fired stage, [23:21]
// fired flags, [28:24] algorithmic bytes of the item beyond its 1-byte read, [29] writes due =
// now + fsm_due[entry], [30] matched, [31] fired.  Lookups the sweep never makes (and unused ids,
// kIdInvalid among them) hold the id itself: no change, nothing fires.
constexpr uint32_t kId8Rec16 = 0xF800u, kId8Due = 1u << 29, kId8Match = 1u << 30, kId8Fire = 1u << 31;
// SweepArgs::fsm_bits of the 1-byte sweep: the table holds a kId8Due entry
constexpr uint32_t kId8AnyDue = 1u;
// fired records of the 1-byte sweep: 2 bytes {LDS offset: 11, stage: 2, flags: 3} after a 16-byte
// header {count, 0, 0, 0} when the program has <= 4 stages (kStages4), else the 4-byte records
// {LDS offset: 13, stage: 5, flags: 3} after the count word as in the other sweeps
constexpr uint32_t kRec16Header = 16;

// A wave's 2048 ids sit in its 2 KiB LDS tile dword-major: dword jj (0-7) of every lane in one
// 256-byte row, lane L's at column L ^ jj, so that the items of one lane (consecutive in the work
// list) fall in different banks and a row's store / load by all lanes is a permutation.  Bit k
// of a lane's phase-1 masks is byte b = k >> 3 of its dword jj = k & 7 (dword j = jj & 3 of chunk
// q = jj >> 2): one mask-and-shift per dword and flag.  Fired records carry the LDS offset
// (11 bits); compaction maps it back to the slot (id8_slot).
__device__ __forceinline__ uint32_t lds_id8(const uint32_t k, const uint32_t lane4) {
  const uint32_t jj = k & 7u;
  return jj << 8 | (lane4 ^ jj << 2) | k >> 3;
}
__device__ __forceinline__ uint32_t lds_col8(const uint32_t jj, const uint32_t lane) { return jj * 64u + (lane ^ jj); }
// slot within the wave region of LDS offset x (row q of the region = 1 KiB, lane = 16 bytes of it)
__host__ __device__ __forceinline__ uint32_t id8_slot(const uint32_t x) {
  const uint32_t jj = x >> 8, lane = ((x >> 2) & 63u) ^ jj, b = x & 3u;
  return (jj >> 2) * 1024u + lane * 16u + (jj & 3u) * 4u + b;
}
__device__ __forceinline__ unsigned long long ballot(const bool b) { return __builtin_amdgcn_ballot_w64(b); }

// inclusive prefix sum over the wave's lanes on DPP lane moves: row_shr 1 / 2 / 4 / 8 within each
// row of 16, then row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3)
template <int C, int RM>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, C, RM, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v += dpp_u32<0x111, 0xF>(v);
  v += dpp_u32<0x112, 0xF>(v);
  v += dpp_u32<0x114, 0xF>(v);
  v += dpp_u32<0x118, 0xF>(v);
  v += dpp_u32<0x142, 0xA>(v);
  v += dpp_u32<0x143, 0xC>(v);
  return v;
}

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)p;
}

// One 64-item pass of the 1-byte sweep's phase 2.  Work-list entries are absolute LDS byte
// addresses of ids (tiles are 2 KiB aligned: the low 11 bits are the tile offset); an inactive
// lane's entry points at its own byte of a row of kIdInvalid, whose lookup is the identity.
// kSlow: entries carry "the queued stage is due" at bit 15, or the table schedules delayed
// stages.  kStages4: the fired records go to the wave's LDS work list (their positions lie
// behind the entries still to be read), 2 bytes each, and the per-stage counts to scalar
// registers; else 4-byte records straight to the segment and LDS counters.
template <bool kStages4>
__device__ __forceinline__ void id8_fire(const uint32_t addr, const uint32_t e, uint16_t* __restrict__ wl,
                                         const __amdgpu_buffer_rsrc_t seg_rs, uint32_t& seg_n, uint32_t (&stc)[4],
                                         unsigned int* s_stat, uint32_t n_stages, uint32_t lane);

template <bool kSlow, bool kStages4>
__device__ __forceinline__ void id8_pass(const uint32_t we, const uint32_t* __restrict__ s_fsm, uint16_t* __restrict__ wl,
                                         const __amdgpu_buffer_rsrc_t seg_rs, uint32_t& seg_n, uint32_t& n_bytes,
                                         uint32_t& n_matched, uint32_t (&stc)[4], unsigned int* s_stat, uint32_t n_stages,
                                         uint32_t lane, bool any_due, const __amdgpu_buffer_rsrc_t fdue_rs,
                                         const __amdgpu_buffer_rsrc_t due_rs, uint32_t wbase, int64_t now) {
  const uint32_t addr = kSlow ? (we & 0x7FFFu) : we;
  const uint32_t r = kSlow ? (we >> 7) & 0x100u : 0u;
  lds_u8* p = (lds_u8*)(size_t)addr;
  const uint32_t key = r | (uint32_t)*p;
  const uint32_t e = s_fsm[key];
  *p = (uint8_t)e;
  n_bytes += (e >> 24) & 31u;
  n_matched += (e >> 30) & 1u;
  if (kSlow && any_due && (e & kId8Due)) {  // a delayed stage is scheduled (rare for table-only programs)
    const int64_t dd = buf_load_i64(fdue_rs, key * 8u);
    const int64_t t = sat_add(now, dd);
    const uint32_t off = (wbase + id8_slot(addr & 0x7FFu)) * 8u;
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)t, due_rs, off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)((uint64_t)t >> 32), due_rs, off + 4u, 0, 0);
  }
  id8_fire<kStages4>(addr, e, wl, seg_rs, seg_n, stc, s_stat, n_stages, lane);
}

// kN passes whose LDS round trips overlap (table-only ids, no due path): every entry's byte, then
// every lookup, then every write — the passes touch distinct bytes (an inactive lane's entries
// are its kIdInvalid byte, whose lookup writes it back unchanged)
constexpr uint32_t kId8Batch = 4;  // passes per step of the id loop (vs 1: C5 step 93.7-95.1 -> 91.4-93.8 us,
                                   // sweep 50.9-51.6 -> 49.2-51.2 us, r3zc alternating)
template <bool kStages4, uint32_t kN>
__device__ __forceinline__ void id8_passn(const uint32_t (&we)[kN], const uint32_t* __restrict__ s_fsm,
                                          uint16_t* __restrict__ wl, const __amdgpu_buffer_rsrc_t seg_rs, uint32_t& seg_n,
                                          uint32_t& n_bytes, uint32_t& n_matched, uint32_t (&stc)[4],
                                          unsigned int* s_stat, uint32_t n_stages, uint32_t lane) {
  uint32_t k[kN], e[kN];
#pragma unroll
  for (uint32_t j = 0; j < kN; ++j) k[j] = (uint32_t)*(lds_u8*)(size_t)we[j];
#pragma unroll
  for (uint32_t j = 0; j < kN; ++j) e[j] = s_fsm[k[j]];
#pragma unroll
  for (uint32_t j = 0; j < kN; ++j) *(lds_u8*)(size_t)we[j] = (uint8_t)e[j];
#pragma unroll
  for (uint32_t j = 0; j < kN; ++j) {
    n_bytes += (e[j] >> 24) & 31u;
    n_matched += (e[j] >> 30) & 1u;
    id8_fire<kStages4>(we[j], e[j], wl, seg_rs, seg_n, stc, s_stat, n_stages, lane);
  }
}

// the fired ballot of one pass: records staged at the list's consumed front (<= 4 stages) or
// stored to the segment, per-stage counts
template <bool kStages4>
__device__ __forceinline__ void id8_fire(const uint32_t addr, const uint32_t e, uint16_t* __restrict__ wl,
                                         const __amdgpu_buffer_rsrc_t seg_rs, uint32_t& seg_n, uint32_t (&stc)[4],
                                         unsigned int* s_stat, uint32_t n_stages, uint32_t lane) {
  const bool fire = (int32_t)e < 0;
  const unsigned long long bal = ballot(fire);
  if (bal) {  // wave-uniform
    const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, seg_n));
    if constexpr (kStages4) {
      if (fire) wl[pos] = (uint16_t)((addr & 0x7FFu) | (e & kId8Rec16));
      // per-lane byte counters, one per stage code (bits 11-12): no ballot / SALU chain per stage
      stc[0] += (e >> 31) << ((e >> 8) & 0x18u);
    } else {
      __builtin_amdgcn_raw_buffer_store_b32((addr & 0x7FFu) | ((e >> 3) & 0x1FE000u), seg_rs, fire ? (1u + pos) * 4u : kOOB,
                                            0, 0);
      const uint32_t code = (e >> 16) & 31u;
      for (uint32_t st = 0; st < n_stages; ++st) {
        const unsigned long long same = ballot(code == st) & bal;
        if (same && lane == 0) atomicAdd(&s_stat[3 + st], (unsigned)__popcll(same));
      }
    }
    seg_n += (uint32_t)__popcll(bal);
  }
}

// one tile per workgroup (small engines, the strong-scaling shards): 6 workgroups per CU (<= 80
// VGPRs, 26.8 KB of LDS) so that a 12.5M-id shard's 1526 tiles are one dispatch round, not two
// kSteps > 1: fused steps (a.now, then a.nowx[s - 1] for step s) for tables without delayed
// stages — each id is read once, stepped kSteps times in LDS and written once; step 0's records go
// to a.fired / a.wave_counts, step s's to a.firedx / a.countsx[s - 1] (step_group)
template <bool kPersist, int kDepth, bool kStages4, int kSteps = 1>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kPersist ? 1 : 6))) void sweep8_kernel(SweepArgs a) {
  constexpr int Q = kQ8;
  constexpr int K = 16 * Q;                // ids per lane
  constexpr uint32_t kWave = 64u * K;      // ids per wave region
  constexpr uint32_t kTile = kBlock * K;   // ids per block
  constexpr uint32_t kSeg8 = 64u * K + 32u;
  static_assert(kDepth >= 1 && kDepth <= 2 && (kPersist || kDepth == 1), "prefetch depth");
  static_assert(kWave == 2048 && K == 32, "11-bit record offsets, 32-bit lane masks");
  static_assert((kSteps == 1 || kStages4) && kSteps >= 1 && kSteps <= (int)kMaxFuseSteps,
                "fused steps hand back 2-byte records");
  __shared__ __attribute__((aligned(2048))) uint32_t s_tile[kWavesPerBlock][4 * Q][64];
  __shared__ __attribute__((aligned(16))) uint16_t s_work[kWavesPerBlock][kWave];
  __shared__ uint32_t s_inv[64];  // kIdInvalid bytes: the inactive lanes' entries (shared by the waves:
                                  // they only ever write 0xFF back)
  __shared__ uint32_t s_fsm[512];
  __shared__ unsigned int s_stat[kStatWords];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t n_tiles = (uint32_t)(((uint64_t)a.n + kTile - 1) / kTile);
  const __amdgpu_buffer_rsrc_t st_rs = make_rsrc(a.st, (a.n + 15u) & ~15u);
  const __amdgpu_buffer_rsrc_t due_rs = make_rsrc(a.due, a.n * 8u);
  const __amdgpu_buffer_rsrc_t fdue_rs = make_rsrc(a.fsm_due, 8u * 512u);
  const __amdgpu_buffer_rsrc_t cnt_rs = make_rsrc(a.wave_counts, n_tiles * kWavesPerBlock * 4u);
  uint4 va[kDepth][Q];
  auto issue_tile = [&](uint4 (&dst)[Q], const uint32_t t) __attribute__((always_inline)) {
    const uint32_t off = t < n_tiles ? t * kTile + wave * kWave + lane * 16u : kOOB - 2048u;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const auto c = __builtin_amdgcn_raw_buffer_load_b128(st_rs, off + (uint32_t)q * 1024u, 0, 0);
      dst[q] = make_uint4(c[0], c[1], c[2], c[3]);
    }
  };
  uint32_t tile = blockIdx.x;
  issue_tile(va[0], tile);
  if (kDepth > 1) issue_tile(va[kDepth - 1], tile + gridDim.x);
  const uint32_t n_stages = a.table->n_stages;
  const bool any_due = (a.fsm_bits & kId8AnyDue) != 0;
  // two table entries per thread, no loop: the wait for them (which drains the tile loads issued
  // above) is on every path into the tile loop, so its waits count only the loop's own operations
  static_assert(kBlock * 2 == 512, "id table staging");
  {
    const uint32_t t0 = a.fsm[threadIdx.x], t1 = a.fsm[threadIdx.x + kBlock];
    s_fsm[threadIdx.x] = t0;
    s_fsm[threadIdx.x + kBlock] = t1;
  }
  if (threadIdx.x < kStatWords) s_stat[threadIdx.x] = 0;
  if (wave == 0) s_inv[lane] = 0xFFFFFFFFu;
  __syncthreads();

  // kStages4: stc[0] = this tile's fired records of stages 0-3 as byte counters (<= 32 items per lane
  // and tile), folded after each tile into 16-bit counters stc[1] (stages 0, 2) and stc[2] (1, 3)
  uint32_t stc[4] = {0u, 0u, 0u, 0u};
  uint32_t n_matched = 0, n_bytes = 0;  // per lane
  uint32_t n_lline = 0;                 // per lane: bytes of the phase-3 line stores
  uint32_t w_bytes = 0, w_line = 0;     // wave-uniform
  uint32_t wave_fired = 0;              // wave-uniform
  uint32_t* __restrict__ tw = &s_tile[wave][0][0];
  uint16_t* __restrict__ wl = s_work[wave];
  const __amdgpu_buffer_rsrc_t gq_rs = make_rsrc(a.st, (a.n + 2047u) & ~2047u);  // whole lines of the padded column
  const uint32_t tile_lds = lds_addr(tw);  // 2 KiB aligned
  const uint32_t lane4 = lane * 4u;
  const uint32_t inv_ent = lds_addr(&s_inv[lane]);

  // tile_body also runs for one tile past the last (the second half of the last pair of the
  // persistent loop, which has no exit in between: the in-order wait counts stay the same on
  // every path): its loads are out of range (zeros: no work) and so are its stores
  auto tile_body = [&](uint4 (&v)[Q], const uint32_t tile) __attribute__((always_inline)) {
    const bool real = tile < n_tiles;  // wave-uniform
    const uint32_t wbase = tile * kTile + wave * kWave;
    const bool full = (uint64_t)(tile + 1) * kTile <= a.n;
    const uint32_t seg_id = tile * kWavesPerBlock + wave;
    uint32_t* __restrict__ seg32 = reinterpret_cast<uint32_t*>(a.fired) + (uint64_t)seg_id * kSeg8;
    const __amdgpu_buffer_rsrc_t seg_rs = make_rsrc(seg32, kSeg8 * 4u);
    uint4 cur_copy[Q];
    if (kDepth == 1) {
#pragma unroll
      for (int q = 0; q < Q; ++q) cur_copy[q] = v[q];
    }
    uint4 (&cur)[Q] = kDepth == 1 ? cur_copy : v;
    if (kPersist && kDepth == 1) issue_tile(v, tile + gridDim.x);
    // ---- phase 1: the id's need / pend bits, one mask-and-shift per dword and flag
    uint32_t in_range = 0xFFFFFFFFu;
    if (!full) {
      in_range = 0;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int64_t left = (int64_t)a.n - (int64_t)(wbase + (uint32_t)q * 1024u + lane * 16u);
        const uint32_t c = left <= 0 ? 0u : left >= 16 ? 16u : (uint32_t)left;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
#pragma unroll
          for (uint32_t b = 0; b < 4; ++b) in_range |= (j * 4u + b < c ? 1u : 0u) << (b * 8u + (uint32_t)q * 4u + j);
      }
    }
    // phases 1 and 2 of one step over the wave's ids (registers): the need / pend bits, the due
    // test at `now`, the work list and the table passes; the step's records staged at the work
    // list's front (seg_n).  Returns the items worked: the tile is in LDS iff nonzero.  first: the
    // step that read the ids from HBM (a fused pair's second step adds no read bytes)
    auto phase12 = [&](const uint4 (&ids)[Q], const int64_t now, const bool first, const bool in_lds, uint32_t& seg_n)
                       __attribute__((always_inline)) -> uint32_t {
      uint32_t need = 0, pend = 0, ready = 0;
  #pragma unroll
      for (int q = 0; q < Q; ++q) {
        const uint32_t dw[4] = {ids[q].x, ids[q].y, ids[q].z, ids[q].w};
  #pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t jj = (uint32_t)(q * 4 + j);
          need |= (dw[j] & 0x80808080u) >> (7u - jj);
          pend |= ((dw[j] << 1) & 0x80808080u) >> (7u - jj);
        }
      }
      need &= in_range;
      pend &= in_range;
      if (ballot(pend != 0)) {  // a queued stage: is it due? (4 loads in flight: registers stay low)
  #pragma unroll 4
        for (int k = 0; k < K; ++k) {
          const uint32_t p = (pend >> k) & 1u;
          const uint32_t slot = id8_slot(lds_id8((uint32_t)k, lane4));
          const int64_t d = buf_load_i64(due_rs, p ? (wbase + slot) * 8u : kOOB);
          ready |= (p & (uint32_t)(d <= now)) << k;
        }
        need |= ready;
      }
      n_bytes += (first ? (uint32_t)__popc(in_range) : 0u) + 8u * (uint32_t)__popc(pend);
      uint32_t n_work = 0, pos = 0;
      {  // exclusive prefix of the lanes' item counts (DPP scan) and the wave's total
        const uint32_t cnt = (uint32_t)__popc(need);
        const uint32_t incl = wave_incl_scan(cnt);
        pos = incl - cnt;
        n_work = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      }
      if (n_work) {  // wave-uniform
        // ---- phase 2: the ids to the LDS tile, the work list (absolute LDS addresses of the ids in
        // slot order per lane), then one lookup in the id table per item, 64 items per pass
        if (!in_lds) {  // (a fused step after one with work: the tile is there already)
  #pragma unroll
          for (int q = 0; q < Q; ++q) {
            tw[lds_col8(q * 4 + 0, lane)] = ids[q].x;
            tw[lds_col8(q * 4 + 1, lane)] = ids[q].y;
            tw[lds_col8(q * 4 + 2, lane)] = ids[q].z;
            tw[lds_col8(q * 4 + 3, lane)] = ids[q].w;
          }
        }
        const bool rdy = ballot(ready != 0) != 0;  // wave-uniform: entries carry the ready bit
        const bool slow = rdy || any_due;          // ... or due times may be written
        {
          // entry = tile_lds | lds_id8(k, lane4) = ent0 ^ lds_id8(k, 0) (lane4 has no bits in
          // lds_id8's k fields): three ops per item on the per-lane loop, whose trip count is the
          // most items of any lane
          uint32_t m = need;
          uint16_t* wp = wl + pos;
          const uint32_t ent0 = tile_lds | lane4;
          if (rdy) {
            while (m) {
              const uint32_t k = (uint32_t)__builtin_ctz(m);
              m &= m - 1u;
              *wp++ = (uint16_t)((ent0 ^ ((k & 7u) * 0x104u | k >> 3)) | ((ready >> k) & 1u) << 15);
            }
          } else {
            while (m) {
              const uint32_t k = (uint32_t)__builtin_ctz(m);
              m &= m - 1u;
              *wp++ = (uint16_t)(ent0 ^ ((k & 7u) * 0x104u | k >> 3));
            }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        // the next pass's entries are read while this pass works (an entry past the list: the
        // lane's kIdInvalid byte)
        if (slow) {
          uint32_t nwe = lane < n_work ? (uint32_t)wl[lane] : inv_ent;
          for (uint32_t c = 0; c < n_work; c += 64u) {  // wave-uniform
            const uint32_t we = nwe;
            if (c + 64u < n_work) {
              const uint32_t x = (uint32_t)wl[(c + 64u + lane) & (kWave - 1u)];
              nwe = c + 64u + lane < n_work ? x : inv_ent;
            }
            id8_pass<true, kStages4>(we, s_fsm, wl, seg_rs, seg_n, n_bytes, n_matched, stc, s_stat, n_stages, lane, any_due,
                                     fdue_rs, due_rs, wbase, now);
          }
        } else {
          // kId8Batch passes per step (their LDS round trips overlap); the next step's entries are
          // read while these work (records of passes < c + 64 * kId8Batch land below it)
          constexpr uint32_t kB = kId8Batch;
          uint32_t nw[kB];
  #pragma unroll
          for (uint32_t j = 0; j < kB; ++j) nw[j] = 64u * j + lane < n_work ? (uint32_t)wl[64u * j + lane] : inv_ent;
          for (uint32_t c = 0; c < n_work; c += 64u * kB) {  // wave-uniform
            uint32_t we[kB];
  #pragma unroll
            for (uint32_t j = 0; j < kB; ++j) we[j] = nw[j];
            if (c + 64u * kB < n_work) {
  #pragma unroll
              for (uint32_t j = 0; j < kB; ++j) {
                const uint32_t i = c + 64u * (kB + j) + lane;
                const uint32_t x = (uint32_t)wl[i & (kWave - 1u)];
                nw[j] = i < n_work ? x : inv_ent;
              }
            }
            id8_passn<kStages4, kB>(we, s_fsm, wl, seg_rs, seg_n, n_bytes, n_matched, stc, s_stat, n_stages, lane);
          }
        }
        n_lline -= (uint32_t)__popc(need);  // the ids' own writes are replaced by the line stores below
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      }
      return n_work;
    };
    // the step's staged records to its segment (kStages4), the header and the count
    auto store_records = [&](const __amdgpu_buffer_rsrc_t seg_rs, const __amdgpu_buffer_rsrc_t cnt_rs,
                             const uint32_t seg_n) __attribute__((always_inline)) {
      if constexpr (kStages4) {
        // records: seg_n 2-byte records from the work list, as 16-byte chunks of whole 128-byte
        // lines (the tail of the last line is padding)
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        const uint32_t n_chunks = ((seg_n * 2u + 127u) & ~127u) / 16u;
        const uint4* wq = reinterpret_cast<const uint4*>(wl);
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  #pragma unroll
        for (uint32_t r = 0; r < 4; ++r) {
          const uint32_t ci = r * 64u + lane;
          const uint4 x = wq[ci];
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{x.x, x.y, x.z, x.w}, seg_rs,
                                                 ci < n_chunks ? kRec16Header + ci * 16u : kOOB, 0, 0);
        }
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{seg_n, 0u, 0u, 0u}, seg_rs, lane == 0 && real ? 0u : kOOB, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(seg_n, cnt_rs, lane == 0 && real ? seg_id * 4u : kOOB, 0, 0);
        if (real) {
          w_line += n_chunks * 16u - seg_n * 2u + kRec16Header - 4u;  // padding and header: line bytes only
          w_bytes += 2u * seg_n + 4u;
        }
        if constexpr (kSteps > 4) {  // a lane's byte counters hold <= 255 fires: fold them per step
          stc[1] += stc[0] & 0x00FF00FFu;
          stc[2] += (stc[0] >> 8) & 0x00FF00FFu;
          stc[0] = 0u;
        }
      } else if (real) {
        const uint32_t used = 1u + seg_n, end = (used + 31u) & ~31u;
        for (uint32_t x = used + lane; x < end; x += 64) seg32[x] = 0u;
        if (lane == 0) {
          seg32[0] = seg_n;
          a.wave_counts[seg_id] = seg_n;
        }
        w_line += 4u * (end - used);
        w_bytes += 4u * seg_n + 4u;
      }
      wave_fired += seg_n;
    };
    uint32_t seg_n = 0;  // wave-uniform
    const uint32_t n_work = phase12(cur, a.now, true, false, seg_n);
    uint32_t any_work = n_work;
    uint32_t seg_last = seg_n;
#pragma unroll
    for (int st = 1; st < kSteps; ++st) {
      // step st (a.nowx[st - 1]) on the ids the steps before left: the previous step's records go
      // to its segment first (they sit in the work list the next list overwrites)
      const uint32_t* px = reinterpret_cast<const uint32_t*>(st == 1 ? a.fired : a.firedx[st - 2]);
      store_records(make_rsrc(px + (uint64_t)seg_id * kSeg8, kSeg8 * 4u),
                    make_rsrc(st == 1 ? a.wave_counts : a.countsx[st - 2], n_tiles * kWavesPerBlock * 4u), seg_last);
      uint4 mid[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q)
        mid[q] = any_work ? make_uint4(tw[lds_col8(q * 4 + 0, lane)], tw[lds_col8(q * 4 + 1, lane)],
                                       tw[lds_col8(q * 4 + 2, lane)], tw[lds_col8(q * 4 + 3, lane)])
                          : cur[q];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      seg_last = 0;
      any_work |= phase12(mid, a.nowx[st - 1], false, any_work != 0, seg_last);
    }
    // ---- phase 3 and the hand-back segment: a fixed set of stores per tile (whole 128-byte lines
    // wherever an id changed, the staged records, the header), each lane's offset out of range
    // where it has nothing to store — no exec branch around a store, so that the compiler's
    // in-order wait for the next prefetched tile counts exactly the stores issued after it
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      // without work the tile is unchanged: nothing stored (the data is then never written)
      uint4 nv = make_uint4(0u, 0u, 0u, 0u);
      unsigned long long chm = 0;
      if (any_work) {
        nv = make_uint4(tw[lds_col8(q * 4 + 0, lane)], tw[lds_col8(q * 4 + 1, lane)], tw[lds_col8(q * 4 + 2, lane)],
                        tw[lds_col8(q * 4 + 3, lane)]);
        chm = ballot(nv.x != cur[q].x) | ballot(nv.y != cur[q].y) | ballot(nv.z != cur[q].z) | ballot(nv.w != cur[q].w);
      }
      const bool st = (chm >> (lane & ~(kStoreLanes - 1u))) & ((1ull << kStoreLanes) - 1ull);
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{nv.x, nv.y, nv.z, nv.w}, gq_rs,
                                             st ? wbase + (uint32_t)q * 1024u + lane * 16u : kOOB, 0, 2 /* nt */);
      n_lline += st ? 16u : 0u;
    }
    if constexpr (kSteps > 1)
      store_records(make_rsrc(reinterpret_cast<const uint32_t*>(a.firedx[kSteps - 2]) + (uint64_t)seg_id * kSeg8, kSeg8 * 4u),
                    make_rsrc(a.countsx[kSteps - 2], n_tiles * kWavesPerBlock * 4u), seg_last);
    else
      store_records(seg_rs, cnt_rs, seg_last);
    if constexpr (kStages4) {
      stc[1] += stc[0] & 0x00FF00FFu;
      stc[2] += (stc[0] >> 8) & 0x00FF00FFu;
      stc[0] = 0u;
    }
    if (kPersist && kDepth == 2) issue_tile(v, tile + 2u * gridDim.x);
  };
  if constexpr (!kPersist) {
    if (tile < n_tiles) tile_body(va[0], tile);
  } else if constexpr (kDepth == 1) {
    for (; tile < n_tiles; tile += gridDim.x) tile_body(va[0], tile);
  } else {
    for (; tile < n_tiles; tile += 2u * gridDim.x) {
      tile_body(va[0], tile);
      tile_body(va[kDepth - 1], tile + gridDim.x);
    }
  }

  uint32_t st4[4] = {0u, 0u, 0u, 0u};
  if constexpr (kStages4) {  // the lanes' 16-bit counters summed per stage (32-bit sums)
    st4[0] = stc[1] & 0xFFFFu;
    st4[1] = stc[2] & 0xFFFFu;
    st4[2] = stc[1] >> 16;
    st4[3] = stc[2] >> 16;
  }
  for (int off = 32; off > 0; off >>= 1) {
    n_matched += __shfl_xor(n_matched, off);
    n_bytes += __shfl_xor(n_bytes, off);
    n_lline += __shfl_xor(n_lline, off);
    if constexpr (kStages4) {
#pragma unroll
      for (int st = 0; st < 4; ++st) st4[st] += __shfl_xor(st4[st], off);
    }
  }
  if (lane == 0) {
    if constexpr (kStages4) {
#pragma unroll
      for (int st = 0; st < 4; ++st)
        if (st4[st]) atomicAdd(&s_stat[3 + st], st4[st]);
    }
    atomicAdd(&s_stat[0], n_matched);
    atomicAdd(&s_stat[1], wave_fired);
    atomicAdd(&s_stat[2], n_bytes + w_bytes);
    atomicAdd(&s_stat[kStatLine], n_bytes + w_bytes + n_lline + w_line);
  }
  __syncthreads();
  if (threadIdx.x < 3 + n_stages || threadIdx.x == kStatLine) {
    const unsigned int val = s_stat[threadIdx.x];
    if (val) atomicAdd(&a.cum[(uint64_t)blockIdx.x * kStatWords + threadIdx.x], (unsigned long long)val);
  }
}

// ------------------------------------------------------------------ 4- and 8-byte state sweep
// Sweep over the 4-byte packed and the 8-byte wide formats (pod-general / chaos and any
// program wider than 16 bits: no transition table, every work item runs process_object).
// Same three phases and the same whole-line write-back as sweep16_kernel — the word-granular
// write-back it replaces cost a line fill plus a partial-line write per scattered store
// (r1o: 1.09 GB of HBM traffic against 0.534 GB algorithmic at 100M pods):
//  phase 1  each lane streams Q 16-byte chunks (kC = 16 / word bytes words each) of its
//           wave's region, row q of a wave = 1 KiB contiguous; due times only for words with
//           a pending stage (and only if the wave has one); the idle test on the raw words;
//           the per-lane need masks become the wave's LDS work list in slot order, each entry
//           carrying "the queued stage is due" so phase 2 never re-reads the due column;
//  phase 2  the chunks go to the wave's LDS tile; process_object runs over the dense work
//           list, reading and writing the word in LDS (a due time is written only when a
//           newly scheduled stage stays pending), and emits packed fired records into the
//           (tile, wave) segment;
//  phase 3  aligned 8-lane groups (one 128-byte line) holding a changed word are stored whole.
constexpr int kQW = 4;                 // 16-byte chunks per lane: 16 (4-byte) / 8 (8-byte) words per lane
constexpr int kDwMinBlocks = 5;        // fused word sweep: resident workgroups per CU the VGPR cap allows
                                       // (96 VGPRs, no scratch: 470-482 vs 485-524 us at 6 on the same boxes,
                                       // r5t / r5v; at 6 the round-5 kernel spills 28-48 B of VGPRs, r3w had
                                       // 467-470 at 6 vs 477-479 at 5)
constexpr int kQWD = 4;                // fused records: 8 per lane, 2048-object tiles (16 per lane: 129 VGPRs,
                                       // 3 waves per SIMD, 630 vs 541 us at C2, r3p)
constexpr int kLdsDeltasW = 128;       // (class, stage) deltas staged in LDS by the word sweep

template <uint32_t kWB> struct WordOf { typedef uint32_t T; };
template <> struct WordOf<8> { typedef uint2 T; };

// word j of a 16-byte chunk
__device__ __forceinline__ uint32_t chunk_word(const uint4& c, int j, uint32_t*) {
  return j == 0 ? c.x : j == 1 ? c.y : j == 2 ? c.z : c.w;
}
__device__ __forceinline__ uint2 chunk_word(const uint4& c, int j, uint2*) {
  return j == 0 ? make_uint2(c.x, c.y) : make_uint2(c.z, c.w);
}
template <bool kDW> __device__ __forceinline__ uint32_t flag_word(uint32_t w) { return w; }  // word holding flags + stage
template <bool kDW> __device__ __forceinline__ uint32_t flag_word(uint2 w) { return kDW ? w.x : w.y; }
__device__ __forceinline__ bool same_word(uint32_t a, uint32_t b) { return a == b; }
__device__ __forceinline__ bool same_word(uint2 a, uint2 b) { return a.x == b.x && a.y == b.y; }
__device__ __forceinline__ void set_chunk_word(uint4& c, int j, uint2 w) {
  if (j == 0) { c.x = w.x; c.y = w.y; } else { c.z = w.x; c.w = w.y; }
}
__device__ __forceinline__ uint32_t pred_word(uint32_t w) { return w; }  // word holding pred
__device__ __forceinline__ uint32_t pred_word(uint2 w) { return w.x; }

// fused records: a VGPR cap (the next tile in flight pushed the kernel to 108 VGPRs / 4 waves:
// 528 -> 481 us at 5 waves, r3v; round 5: 5 waves per SIMD, kDwMinBlocks); the 4-byte words
// lose with a cap (522 -> 579 us at 5)
template <bool kHarness, uint32_t kWB, bool kDW = false>
__global__ __launch_bounds__(kBlock, kDW ? kDwMinBlocks : 1) void sweepw_kernel(SweepArgs a) {
  static_assert(!kDW || kWB == 8, "fused records are 8 bytes");
  typedef typename WordOf<kWB>::T W;
  constexpr int kQ = kDW ? kQWD : kQW;     // 16-byte chunks per lane
  constexpr int kC = 16 / (int)kWB;        // words per chunk
  constexpr int K = kC * kQ;              // words per lane
  constexpr uint32_t kWave = 64u * K;      // words per wave region
  constexpr uint32_t kTile = kBlock * K;   // words per tile (one block)
  static_assert(kTile <= 8192, "fired records carry a 13-bit slot within the tile");
  __shared__ unsigned int s_stat[kStatWords];
  __shared__ kwk_delta s_delta[kLdsDeltasW];
  __shared__ uint16_t s_work[kTile];
  __shared__ uint4 s_tile[kWavesPerBlock][64 * kQ];
  __shared__ uint32_t s_lut[kLutLdsW];
  __shared__ uint32_t s_cnt[kWavesPerBlock][2];
  __shared__ uint32_t s_dirty[kWavesPerBlock];  // per wave region: bit l = its 128-byte line l changed
  __shared__ kwk_stage_table s_tab;
  static_assert(kQ * 8 <= 32, "one dirty-line word per wave region");
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = threadIdx.x >> 6;
  const uint32_t n_tiles = (a.n + kTile - 1u) / kTile;
  uint32_t tile = blockIdx.x;  // tiles blockIdx.x, + gridDim.x, ... (one per block unless the grid is smaller)
  const __amdgpu_buffer_rsrc_t st_rs = make_rsrc(a.st, ((a.n * kWB) + 15u) & ~15u);
  uint4 cur[kQ];
  auto load_tile = [&](uint32_t t) {
    const uint32_t wb = t * kTile + wave * kWave;
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      const auto c = __builtin_amdgcn_raw_buffer_load_b128(st_rs, (wb + (uint32_t)q * 64u * kC + lane * kC) * kWB, 0, 0);
      cur[q] = make_uint4(c[0], c[1], c[2], c[3]);
    }
  };
  load_tile(tile);  // the first tile's stream is issued before the LDS set-up so its latency overlaps it
  {
    const uint32_t nw = (offsetof(kwk_stage_table, stages) + a.table->n_stages * sizeof(kwk_stage_desc)) / 4;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(a.table);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&s_tab);
    for (uint32_t j = threadIdx.x; j < nw; j += kBlock) dst[j] = src[j];
  }
  const kwk_stage_table* __restrict__ T = &s_tab;
  const uint32_t n_stages = a.table->n_stages;
  const uint32_t fin_group = a.table->fin_group_mask;
  const uint32_t n_deltas = a.table->n_classes * n_stages;
  const uint32_t lut_n = a.lut_n;
  const uint32_t* __restrict__ lutp = lut_n <= kLutLdsW ? s_lut : a.lut;  // wider programs: through L1
  if (lut_n <= kLutLdsW)
    for (uint32_t j = threadIdx.x; j < lut_n; j += kBlock) s_lut[j] = a.lut[j];
  if (threadIdx.x < kStatWords) s_stat[threadIdx.x] = 0;
  const kwk_delta* __restrict__ deltas = a.deltas;
  if (n_deltas <= (uint32_t)kLdsDeltasW) {
    for (uint32_t j = threadIdx.x; j < n_deltas; j += kBlock) s_delta[j] = a.deltas[j];
    deltas = s_delta;
  }

  const StateFmt fmt = a.fmt;
  const RawTest R = a.raw;
  uint32_t n_matched = 0, n_bytes = 0, n_line = 0;  // per lane
  uint32_t wave_fired = 0;
  uint4* __restrict__ tq = s_tile[wave];
  W* __restrict__ tw = reinterpret_cast<W*>(&s_tile[0][0]);  // the whole tile: slot t = wave * kWave + offset
  // LDS reuse across tiles needs no extra barrier: s_cnt / s_work of a tile are read before its
  // second / third barrier, and each wave rewrites only its own tq rows and dirty word.  The next
  // tile's stream is in flight (in `cur`, free once the tile is in LDS) while this one is worked.
  for (; tile < n_tiles; tile += gridDim.x) {
  const uint32_t tbase = tile * kTile;
  const uint32_t wbase = tbase + wave * kWave;
  const bool full = (uint64_t)(tile + 1) * kTile <= a.n;
  const uint64_t seg_id = (uint64_t)tile * kWavesPerBlock + wave;
  uint32_t* __restrict__ seg32 = reinterpret_cast<uint32_t*>(a.fired) + seg_id * (kWave + 32u);
  kwk_fired_rec* __restrict__ seg = reinterpret_cast<kwk_fired_rec*>(seg32 + 1);
  uint32_t seg_n = 0;  // wave-uniform

  // ---- phase 1: bit k = q * kC + j of a lane's masks <-> word q * 64 * kC + lane * kC + j
  uint32_t need = 0, heavy = 0, pend = 0, in_range = 0, pend_all = 0;
#pragma unroll
  for (int q = 0; q < kQ; ++q) {
#pragma unroll
    for (int j = 0; j < kC; ++j) {
      const W w = chunk_word(cur[q], j, (W*)nullptr);
      const uint32_t fw = flag_word<kDW>(w), pw = pred_word(w);
      const uint32_t off = (uint32_t)q * 64u * kC + lane * kC + (uint32_t)j;
      const uint32_t in = (full || wbase + off < a.n) ? 1u : 0u;
      const uint32_t mg = (fw & R.managed) ? in : 0u;
      const uint32_t pe = ((fw >> R.sshift) & R.smask) != R.none_code ? 1u : 0u;
      uint32_t nb = (fw & R.dirty) ? 1u : 0u;
      if (kHarness) nb |= ((~fw & R.alive) ? 1u : 0u) | (((pw & R.term) != 0 && (pw & R.del) == 0) ? 1u : 0u);
      const int k = q * kC + j;
      heavy |= (mg & nb) << k;
      pend |= (mg & pe) << k;
      in_range |= in << k;
      if constexpr (kDW) pend_all |= (in & pe) << k;
    }
  }
  need = heavy;
  uint32_t ready = 0;
  if constexpr (kDW) {
    // the due time rides in the record: D <= now - epoch, or the side column for D = kDwFar
    if (__ballot(pend != 0)) {
      const int64_t e0 = a.dw_epoch_old;
      const bool now_ok = a.now >= e0;
      const uint64_t thr = now_ok ? (uint64_t)a.now - (uint64_t)e0 : 0ull;
      uint32_t far = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const uint64_t d = dw_get(chunk_word(cur[k / kC], k % kC, (W*)nullptr));
        const uint32_t p = (pend >> k) & 1u;
        ready |= (p & (uint32_t)(d != kDwFar && now_ok && d <= thr)) << k;
        far |= (p & (uint32_t)(d == kDwFar)) << k;
      }
      if (__ballot(far != 0)) {  // cold: due times outside the window
        const __amdgpu_buffer_rsrc_t due_rs = make_rsrc(a.due, a.n * 8u);
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const uint32_t f = (far >> k) & 1u;
          const uint32_t off = (uint32_t)(k / kC) * 64u * kC + lane * kC + (uint32_t)(k % kC);
          const int64_t d = buf_load_i64(due_rs, f ? (wbase + off) * 8u : kOOB);
          ready |= (f & (uint32_t)(d <= a.now)) << k;
        }
        n_bytes += 8u * (uint32_t)__popc(far);
      }
      need |= ready;
    }
    if (a.dw_rebase && __ballot(pend_all != 0)) {
      // cold (every ~17 s of simulated time): every queued stage's due time re-encoded against
      // the new epoch; times leaving the window go to the side column
#pragma unroll
      for (int q = 0; q < kQ; ++q) {
#pragma unroll
        for (int j = 0; j < kC; ++j) {
          const int k = q * kC + j;
          if ((pend_all >> k) & 1u) {
            const uint64_t i = (uint64_t)wbase + (uint32_t)q * 64u * kC + lane * kC + (uint32_t)j;
            uint2 w = chunk_word(cur[q], j, (uint2*)nullptr);
            const uint64_t d = dw_get(w);
            const int64_t due = d != kDwFar ? dw_abs(d, a.dw_epoch_old) : a.due[i];
            const uint64_t d2 = dw_enc(due, a.fmt.epoch);
            if (d2 == kDwFar && d != kDwFar) a.due[i] = due;
            set_chunk_word(cur[q], j, dw_put(w, d2));
          }
        }
      }
    }
    n_bytes += kWB * (uint32_t)__popc(in_range);
  } else {
    if (__ballot(pend != 0)) {  // some object of the wave has a queued stage: is it due?
      const __amdgpu_buffer_rsrc_t due_rs = make_rsrc(a.due, a.n * 8u);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const uint32_t p = (pend >> k) & 1u;
        const uint32_t off = (uint32_t)(k / kC) * 64u * kC + lane * kC + (uint32_t)(k % kC);
        const int64_t d = buf_load_i64(due_rs, p ? (wbase + off) * 8u : kOOB);
        ready |= (p & (uint32_t)(d <= a.now)) << k;
      }
      need |= ready;
    }
    n_bytes += kWB * (uint32_t)__popc(in_range) + 8u * (uint32_t)__popc(pend);
  }
  // One work list per tile, sorted by kind: the fire-only items (a due stage, nothing to
  // match) of all four waves first, then the items that match (dirty / harness).  The waves
  // then take 64 consecutive items at a time: passes are full, and a pass runs the matcher
  // (weighted pick, jitter draws, getters) only if one of its items needs it.  (Sorting the items
  // with a value record last as a third kind measured slower: 584 vs 523 us fused, r3s.)
  const uint32_t light = need & ~heavy;
  const unsigned long long lt = (1ull << lane) - 1ull;
  uint32_t pos_l = 0, pos_h = 0, n_l = 0, n_h = 0;  // n_* wave-uniform
  {
    const uint32_t cl = (uint32_t)__popc(light), ch = (uint32_t)__popc(heavy);
#pragma unroll
    for (int b = 0; b < 5; ++b) {  // counts <= 16 (4-byte) / 8 (8-byte)
      const unsigned long long bl = __ballot((cl >> b) & 1u), bh = __ballot((ch >> b) & 1u);
      pos_l += (uint32_t)__popcll(bl & lt) << b;
      n_l += (uint32_t)__popcll(bl) << b;
      pos_h += (uint32_t)__popcll(bh & lt) << b;
      n_h += (uint32_t)__popcll(bh) << b;
    }
  }
  if (lane == 0) {
    s_cnt[wave][0] = n_l;
    s_cnt[wave][1] = n_h;
    s_dirty[wave] = 0u;
  }
#pragma unroll
  for (int q = 0; q < kQ; ++q) tq[q * 64 + lane] = cur[q];
  if (tile + gridDim.x < n_tiles) load_tile(tile + gridDim.x);  // block-uniform
  __syncthreads();
  uint32_t tot_l = 0, n_work = 0;  // block-uniform
#pragma unroll
  for (uint32_t w = 0; w < kWavesPerBlock; ++w) {
    const uint32_t xl = s_cnt[w][0], xh = s_cnt[w][1];
    if (w < wave) { pos_l += xl; pos_h += xh; }
    tot_l += xl;
    n_work += xl + xh;
  }
  pos_h += tot_l;
  for (uint32_t m = need; m; m &= m - 1u) {
    const uint32_t k = (uint32_t)__ffs(m) - 1u;
    const uint32_t off = wave * kWave + (k / kC) * 64u * kC + lane * kC + (k % kC);
    const uint16_t ent = (uint16_t)(off | (((ready >> k) & 1u) << 15));
    if ((heavy >> k) & 1u) s_work[pos_h++] = ent;
    else s_work[pos_l++] = ent;
  }
  __syncthreads();

  if (n_work) {
    // ---- phase 2: the tile's list, 64 items per wave pass
    for (uint32_t c = wave * 64u; c < n_work; c += kBlock) {
      const uint32_t jw = c + lane;
      Fire f{false, 0, 0, 0};
      uint32_t off = 0;
      if (jw < n_work) {
        const uint32_t we = s_work[jw];
        off = we & 0x7FFFu;
        const uint64_t i = tbase + off;
        const W r = tw[off];
        uint2 s;
        if constexpr (kDW) s = fmt_unpack(r.x, fmt);
        else s = sw_decode(r, fmt);
        // the queued stage's due time matters only as "due <= now" (a new match overwrites
        // it), which phase 1 already decided
        const int64_t due = (we >> 15) ? INT64_MIN : INT64_MAX;
        uint32_t due_set = 0;
        int64_t due_w = 0;
        const uint2 nv = process_object<kHarness, kWB, false, kDW>(a, T, deltas, n_stages, fin_group, i, s.x, s.y, due,
                                                                   f, n_matched, lutp, lut_n, due_set, due_w);
        W out;
        if constexpr (kDW) {  // the word, and D when a stage was scheduled (its due time leaves with the record)
          out = make_uint2((r.x & ~kDwWordMask) | fmt_pack(nv.x, nv.y, fmt), r.y);
          if (due_set) {
            const uint64_t d = dw_enc(due_w, a.fmt.epoch);
            out = dw_put(out, d);
            if (d == kDwFar) a.due[i] = due_w;
          }
        } else {
          sw_encode(out, nv, fmt);
        }
        tw[off] = out;
        if (!same_word(out, r)) atomicOr(&s_dirty[off / kWave], 1u << (((off % kWave) * kWB) >> 7));
        n_line -= kWB;  // the word's own write is replaced by the line stores below
      }
      n_bytes += f.bytes;
      emit_fired<true>(f, off, lane, seg, seg_n, s_stat, n_bytes);
    }
    __syncthreads();
  }
  const bool rebase = kDW && a.dw_rebase;  // block-uniform: every line is stored
  if (n_work || rebase) {
    // ---- phase 3: whole 128-byte lines of the wave's region wherever a word changed
    uint4* __restrict__ gq = reinterpret_cast<uint4*>(a.st);
    const uint32_t dirty = s_dirty[wave];
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      const uint4 nv = tq[q * 64 + lane];
      // lane's chunk lies in line q * 8 + lane / 8 of the wave region (8 lanes x 16 B per line)
      if (rebase || ((dirty >> (q * 8 + (lane >> 3))) & 1u)) {
        store_chunk_nt(&gq[(wbase + (uint32_t)q * 64u * kC + lane * kC) / kC], nv);
        n_line += 16u;
      }
    }
  }
  {  // segment: [count][records], padded to whole 128-byte lines
    const uint32_t used = 1u + seg_n, end = (used + 31u) & ~31u;
    for (uint32_t x = used + lane; x < end; x += 64) seg32[x] = 0u;
    if (lane == 0) {
      seg32[0] = seg_n;
      a.wave_counts[seg_id] = seg_n;  // the hand-back's scan input
    }
    n_line += 4u * (uint32_t)__popc((uint32_t)(lane < end - used));
  }
  n_bytes += lane == 0 ? 4u : 0u;  // the fired count word
  wave_fired += seg_n;
  }

  for (int o = 32; o > 0; o >>= 1) {
    n_matched += __shfl_xor(n_matched, o);
    n_bytes += __shfl_xor(n_bytes, o);
    n_line += __shfl_xor(n_line, o);
  }
  if (lane == 0) {
    atomicAdd(&s_stat[0], n_matched);
    atomicAdd(&s_stat[1], wave_fired);
    atomicAdd(&s_stat[2], n_bytes);
    atomicAdd(&s_stat[kStatLine], n_bytes + n_line);
  }
  __syncthreads();
  if (threadIdx.x < 3 + n_stages || threadIdx.x == kStatLine) {
    const unsigned int val = s_stat[threadIdx.x];
    if (val) atomicAdd(&a.cum[(uint64_t)blockIdx.x * kStatWords + threadIdx.x], (unsigned long long)val);
  }
}

// ------------------------------------------------------------------ fired hand-back
// Two launches over the sweep's per-(tile, wave) segments: seg_scan_kernel turns the segment
// counts (which the sweep writes into `counts`) into exclusive offsets within groups of
// kScanGroup segments plus one total per group (all groups in parallel: a single-workgroup scan
// over the ~50k counts of a 100M-object sweep was latency-bound, 18.5 us, r2b), then one wave
// per segment adds the totals of the groups before its own and expands its 4-byte records
// {slot within the region: bits 0-12, stage: bits 13-17, flags: bits 18-20; a region is a wave's
// words in the 2-byte sweeps (512-2048 slots), a tile's in the word sweep (2048 / 4096 slots)}
// into kwk_fired_rec at its offset of one
// dense list; the last segment's wave writes the list length.  (A single-pass decoupled
// look-back was measured slower here: with ~12k tiny blocks the look-back chains, not the bytes,
// set the time — 165 us vs the ~30 us the bytes need.)
constexpr uint32_t kPackedSlots = 1u << 27;                // packed fired records: 27-bit slots
constexpr uint32_t kScanPer = 4;                          // counts per thread (16: 4096-count groups, 12 workgroups
                                                          // at C5 for ~5 us; 4: 48 shorter ones)
constexpr uint32_t kScanGroup = kBlock * kScanPer;        // 1024 counts per group (one workgroup)
constexpr uint32_t kSegsPerBlock = kWavesPerBlock;        // one wave per segment

// offsets[1 + i] = records before segment i within its group, group_tot[g] = the group's records
__device__ __forceinline__ void seg_scan_block(const uint32_t* __restrict__ counts, uint32_t n,
                                               uint32_t* __restrict__ offsets, uint32_t* __restrict__ group_tot,
                                               const uint32_t block) {
  __shared__ uint32_t s_wave[kWavesPerBlock];
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint32_t i0 = block * kScanGroup + t * kScanPer;
  uint32_t v[kScanPer];
#pragma unroll
  for (uint32_t q = 0; q < kScanPer / 4; ++q) {
    const uint32_t i = i0 + 4u * q;
    uint4 c = make_uint4(0u, 0u, 0u, 0u);
    if (i + 3 < n) {
      c = *reinterpret_cast<const uint4*>(counts + i);  // counts is 16-byte aligned
    } else {
      if (i < n) c.x = counts[i];
      if (i + 1 < n) c.y = counts[i + 1];
      if (i + 2 < n) c.z = counts[i + 2];
    }
    v[4 * q] = c.x; v[4 * q + 1] = c.y; v[4 * q + 2] = c.z; v[4 * q + 3] = c.w;
  }
  uint32_t sum = 0;
#pragma unroll
  for (uint32_t j = 0; j < kScanPer; ++j) sum += v[j];
  uint32_t incl = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o);
    if (lane >= (uint32_t)o) incl += y;
  }
  if (lane == 63) s_wave[wave] = incl;
  __syncthreads();
  uint32_t before = 0;
#pragma unroll
  for (uint32_t w = 0; w < kWavesPerBlock; ++w) before += w < wave ? s_wave[w] : 0u;
  uint32_t run = before + incl - sum;
#pragma unroll
  for (uint32_t j = 0; j < kScanPer; ++j) {
    if (i0 + j < n) offsets[1 + i0 + j] = run;
    run += v[j];
  }
  if (t == kBlock - 1) group_tot[block] = run;
}
__global__ __launch_bounds__(kBlock) void seg_scan_kernel(const uint32_t* __restrict__ counts, uint32_t n,
                                                         uint32_t* __restrict__ offsets,
                                                         uint32_t* __restrict__ group_tot) {
  seg_scan_block(counts, n, offsets, group_tot, blockIdx.x);
}

struct CompactArgs {
  const uint32_t* __restrict__ fired32;   // segments, `stride` words apart: [count][records]
  const uint32_t* __restrict__ counts;    // records per segment
  uint32_t* __restrict__ offsets;         // seg_scan_kernel's output; [0] <- the list length
  const uint32_t* __restrict__ group_tot;
  kwk_fired_rec* __restrict__ out;
  uint32_t* __restrict__ counts_out;      // 2-byte / bitmap lists: the step's records per segment, kept with
                                          // the list (the next sweep rewrites `counts`), or null
  uint32_t* __restrict__ host_len;        // kwk_fired_keep: pinned host words <- the list length (bitmap:
                                          // {words, records}), or null
  uint32_t n_segs;
  uint32_t seg_region_shift;              // segments per sweep region = 1 << shift
  uint32_t region_slots;                  // object slots per region (wave / tile)
  uint32_t stride;
};
// the hand-backs of a fused launch's steps in one launch each (blockIdx.y = the step)
struct CompactArgs4 {
  CompactArgs a[kMaxFuseSteps];
};
__global__ __launch_bounds__(kBlock) void seg_scan_multi_kernel(CompactArgs4 m) {
  const CompactArgs& a = m.a[blockIdx.y];
  seg_scan_block(a.counts, a.n_segs, a.offsets, const_cast<uint32_t*>(a.group_tot), blockIdx.x);
}

// record kinds: 4-byte {slot within the region: 13, stage: 5, flags: 3} after the count word;
// the 1-byte sweep's 4-byte records with an LDS offset in the slot field (id8_slot); its 2-byte
// records {LDS offset: 11, stage: 2, flags: 3} after a 16-byte header
enum : int { kRecSlot = 0, kRecId8 = 1, kRecId8Half = 2 };

// record j of a segment as (slot within the region, 4-byte layout for the stage / flags)
template <int kRec>
__device__ __forceinline__ uint2 rec_at(const uint32_t* __restrict__ seg, uint32_t j) {
  if constexpr (kRec == kRecId8Half) {
    const uint32_t x = reinterpret_cast<const uint16_t*>(seg + kRec16Header / 4u)[j];
    return make_uint2(id8_slot(x & 0x7FFu), ((x >> 11) & 3u) << 13 | ((x >> 13) & 7u) << 18);
  } else {
    const uint32_t x = seg[1u + j];
    return make_uint2(kRec == kRecId8 ? id8_slot(x & 0x7FFu) : x & 0x1FFFu, x);
  }
}

// one kwk_fired_rec {slot, stage, flags} from a packed record, nontemporal (the dense list is
// written once per step and read by the consumer later: keeping it out of L2 leaves room for
// the segments being read)
__device__ __forceinline__ void store_rec_nt(kwk_fired_rec* p, uint32_t slot, uint32_t x) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  __builtin_nontemporal_store(u32x2{slot, ((x >> 13) & 31u) | ((x >> 18) & 7u) << 16}, reinterpret_cast<u32x2*>(p));
}

// the packed 4-byte record {stage: 31..27, slot: 26..0} (kwk_fired_packed), nontemporal
__device__ __forceinline__ void store_packed_nt(uint32_t* p, uint32_t slot, uint32_t x) {
  __builtin_nontemporal_store(((x >> 13) & 31u) << 27 | slot, p);
}

template <bool kPacked>
__device__ __forceinline__ void store_out(const CompactArgs& a, uint32_t at, uint32_t slot, uint32_t x) {
  if constexpr (kPacked) store_packed_nt(reinterpret_cast<uint32_t*>(a.out) + at, slot, x);
  else store_rec_nt(&a.out[at], slot, x);
}

// kSpw segments per wave; each segment's first 256 records are loaded together with its count
// and offset (a segment holds at least 64 * 16 + 31 words, so the loads stay inside it), all the
// wave's segments' loads in flight at once: at C5 (48k segments) one segment per wave ran six
// dispatch rounds of a ~3.5 us load chain (21 us); four per wave keep every wave resident.
// kPacked: 4-byte records (kwk_fired_packed) instead of kwk_fired_rec — half the bytes written
constexpr uint32_t kCompactSpw = 4;
constexpr uint32_t kCompact16Spw = 8;  // segments per wave of the 2-byte compaction (4 before round 6: C5 1.83 -> 1.90-1.92e11, r6af)
template <int kRec, bool kPacked = false, uint32_t kSpw = 1>
__global__ __launch_bounds__(kBlock) void compact_kernel(CompactArgs a) {
  constexpr int kPre = 4;
  static_assert(kScanGroup % (kSpw * kWavesPerBlock) == 0, "a wave's segments lie in one scan group");
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t seg0 = (blockIdx.x * kWavesPerBlock + wave) * kSpw;
  if (seg0 >= a.n_segs) return;
  uint2 r[kSpw][kPre];
  uint32_t c[kSpw], o1[kSpw];
#pragma unroll
  for (uint32_t s = 0; s < kSpw; ++s) {
    const uint32_t seg = seg0 + s < a.n_segs ? seg0 + s : seg0;
    const uint32_t* __restrict__ sp = a.fired32 + (uint64_t)seg * a.stride;
#pragma unroll
    for (int k = 0; k < kPre; ++k) r[s][k] = rec_at<kRec>(sp, lane + 64u * k);
    c[s] = seg0 + s < a.n_segs ? a.counts[seg] : 0u;
    o1[s] = a.offsets[1 + seg];
  }
  uint32_t gp = 0;  // records of the groups before the wave's segments' group
  for (uint32_t g = lane; g < seg0 / kScanGroup; g += 64) gp += a.group_tot[g];
  for (int o = 32; o > 0; o >>= 1) gp += __shfl_xor(gp, o);
#pragma unroll
  for (uint32_t s = 0; s < kSpw; ++s) {
    const uint32_t seg = seg0 + s;
    if (seg >= a.n_segs) break;
    const uint32_t off = gp + o1[s];
    if (seg == a.n_segs - 1 && lane == 0) {
      a.offsets[0] = off + c[s];
      if (a.host_len) a.host_len[0] = off + c[s];
    }
    const uint32_t base = (seg >> a.seg_region_shift) * a.region_slots;
#pragma unroll
    for (int k = 0; k < kPre; ++k) {
      const uint32_t j = lane + 64u * k;
      if (j < c[s]) store_out<kPacked>(a, off + j, base + r[s][k].x, r[s][k].y);
    }
    const uint32_t* __restrict__ sp = a.fired32 + (uint64_t)seg * a.stride;
    for (uint32_t j = lane + 64u * kPre; j < c[s]; j += 64) {
      const uint2 x = rec_at<kRec>(sp, j);
      store_out<kPacked>(a, off + j, base + x.x, x.y);
    }
  }
}

// The 2-byte hand-back (kwk_fired_compact_packed16): the 1-byte sweep's <= 4-stage records
// {LDS offset: 11, stage: 2, flags: 3} copied as they are into one dense list at their segment's
// offset; the host maps a record to its slot with its segment's region (KWK_FIRED16_SLOT)
template <uint32_t kSpw>
__device__ __forceinline__ void compact16_block(const CompactArgs& a, const uint32_t block) {
  static_assert(kScanGroup % (kSpw * kWavesPerBlock) == 0, "a wave's segments lie in one scan group");
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t seg0 = (block * kWavesPerBlock + wave) * kSpw;
  if (seg0 >= a.n_segs) return;
  uint32_t c[kSpw], o1[kSpw];
  uint16_t r[kSpw][4];
#pragma unroll
  for (uint32_t s = 0; s < kSpw; ++s) {
    const uint32_t seg = seg0 + s < a.n_segs ? seg0 + s : seg0;
    const uint16_t* sp = reinterpret_cast<const uint16_t*>(a.fired32 + (uint64_t)seg * a.stride + kRec16Header / 4u);
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) r[s][k] = sp[lane + 64u * k];
    c[s] = seg0 + s < a.n_segs ? a.counts[seg] : 0u;
    o1[s] = a.offsets[1 + seg];
  }
  if (a.counts_out) {
#pragma unroll
    for (uint32_t s = 0; s < kSpw; ++s)
      if (lane == s && seg0 + s < a.n_segs) a.counts_out[seg0 + s] = c[s];
  }
  uint32_t gp = 0;
  for (uint32_t g = lane; g < seg0 / kScanGroup; g += 64) gp += a.group_tot[g];
  for (int o = 32; o > 0; o >>= 1) gp += __shfl_xor(gp, o);
  uint16_t* out = reinterpret_cast<uint16_t*>(a.out);
#pragma unroll
  for (uint32_t s = 0; s < kSpw; ++s) {
    const uint32_t seg = seg0 + s;
    if (seg >= a.n_segs) break;
    const uint32_t off = gp + o1[s];
    if (seg == a.n_segs - 1 && lane == 0) {
      a.offsets[0] = off + c[s];
      if (a.host_len) a.host_len[0] = off + c[s];
    }
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k)
      if (lane + 64u * k < c[s]) __builtin_nontemporal_store(r[s][k], out + off + lane + 64u * k);
    const uint16_t* sp = reinterpret_cast<const uint16_t*>(a.fired32 + (uint64_t)seg * a.stride + kRec16Header / 4u);
    for (uint32_t j = lane + 256u; j < c[s]; j += 64) __builtin_nontemporal_store(sp[j], out + off + j);
  }
}
template <uint32_t kSpw>
__global__ __launch_bounds__(kBlock) void compact16_kernel(CompactArgs a) {
  compact16_block<kSpw>(a, blockIdx.x);
}
template <uint32_t kSpw>
__global__ __launch_bounds__(kBlock) void compact16_multi_kernel(CompactArgs4 m) {
  compact16_block<kSpw>(m.a[blockIdx.y], blockIdx.x);
}

// the 2-byte hand-back in one launch for small sweeps (as compact_small_kernel below), kSpw
// segments per wave: each block sums the counts of every segment before its first (16-byte loads),
// then each wave copies its segments' records, the first 256 of all kSpw segments loaded together.
// (One segment per wave made the 125k-node shard's group of four steps 6104 blocks re-reading the
// counts: 15-19 us per group, r6j.)
constexpr uint32_t kSmall16Spw = 4;
constexpr uint32_t kSmall16Spb = kSmall16Spw * kWavesPerBlock;  // segments per block
template <uint32_t kSpw>
__device__ __forceinline__ void compact16_small_block(const CompactArgs& a, const uint32_t block) {
  constexpr uint32_t kSpb = kSpw * kWavesPerBlock;
  static_assert(kSpb % 4 == 0, "prefix loads assume whole uint4s before the block");
  __shared__ uint32_t s_part[kWavesPerBlock];
  __shared__ uint32_t s_seg[kSpb];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t first = block * kSpb;
  const uint4* __restrict__ c4 = reinterpret_cast<const uint4*>(a.counts);
  uint32_t sum = 0;
#pragma unroll 8
  for (uint32_t q = threadIdx.x; q < first / 4u; q += kBlock) {
    const uint4 v = c4[q];
    sum += (v.x + v.y) + (v.z + v.w);
  }
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  if (lane == 0) s_part[wave] = sum;
  if (threadIdx.x < kSpb) {
    const uint32_t c = first + threadIdx.x < a.n_segs ? a.counts[first + threadIdx.x] : 0u;
    s_seg[threadIdx.x] = c;
    if (a.counts_out && first + threadIdx.x < a.n_segs) a.counts_out[first + threadIdx.x] = c;
  }
  __syncthreads();
  const uint32_t seg0 = first + wave * kSpw;
  if (seg0 >= a.n_segs) return;
  uint32_t off = s_part[0] + s_part[1] + s_part[2] + s_part[3];
  for (uint32_t w = 0; w < wave * kSpw; ++w) off += s_seg[w];
  uint32_t c[kSpw];
  uint16_t r[kSpw][4];
#pragma unroll
  for (uint32_t s = 0; s < kSpw; ++s) {  // (a segment holds room for >= 256 records: in bounds)
    const uint32_t seg = seg0 + s < a.n_segs ? seg0 + s : seg0;
    const uint16_t* sp = reinterpret_cast<const uint16_t*>(a.fired32 + (uint64_t)seg * a.stride + kRec16Header / 4u);
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) r[s][k] = sp[lane + 64u * k];
    c[s] = seg0 + s < a.n_segs ? s_seg[wave * kSpw + s] : 0u;
  }
  uint16_t* out = reinterpret_cast<uint16_t*>(a.out);
#pragma unroll
  for (uint32_t s = 0; s < kSpw; ++s) {
    const uint32_t seg = seg0 + s;
    if (seg >= a.n_segs) break;
    if (seg == a.n_segs - 1 && lane == 0) {
      a.offsets[0] = off + c[s];
      if (a.host_len) a.host_len[0] = off + c[s];
    }
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k)
      if (lane + 64u * k < c[s]) __builtin_nontemporal_store(r[s][k], out + off + lane + 64u * k);
    const uint16_t* sp = reinterpret_cast<const uint16_t*>(a.fired32 + (uint64_t)seg * a.stride + kRec16Header / 4u);
    for (uint32_t j = lane + 256u; j < c[s]; j += 64) __builtin_nontemporal_store(sp[j], out + off + j);
    off += c[s];
  }
}
__global__ __launch_bounds__(kBlock) void compact16_small_kernel(CompactArgs a) {
  compact16_small_block<kSmall16Spw>(a, blockIdx.x);
}
__global__ __launch_bounds__(kBlock) void compact16_small_multi_kernel(CompactArgs4 m) {
  compact16_small_block<kSmall16Spw>(m.a[blockIdx.y], blockIdx.x);
}

// The bitmap hand-back (kwk_fired_compact_bits): the 1-byte sweep's <= 4-stage records as one
// 2048-bit map per segment — bit i = lane * 32 + k for the id at lds_id8(k, lane * 4), the order
// the sweep's work list (lane-major, k ascending) writes its records in — kept byte-sparse, plus
// the records' 2-bit stage codes in that same order.  For n segments:
//   word s < n                {records c: 16, nonzero map bytes z: 16} of segment s
//   from word n + P(s)        segment s: 8 summary words (bit t of word w: map byte 32 w + t is
//                             nonzero), its z nonzero map bytes in order (padded to a word), its c
//                             codes, 16 per word (code j at bits 2 (j % 16) of word j / 16)
// with P(s) = sum over t < s of (8 + ceil(z_t / 4) + ceil(c_t / 16)).  ~1.1 bytes per transition at
// C5's 10 % firing (43 % of the map bytes are zero), against 2 (+ 4 per segment) for the 2-byte
// records.  Two kernels over one wave per segment: bits_size_kernel (the map in LDS -> {c, z}, the
// segment's words, its workgroup's records) and, after the prefix of those words (in-kernel up to
// compact_small segments, else seg_scan_kernel), bits_write_kernel (the map again -> the words at
// P(s)); tot <- {words, records}.
__device__ __forceinline__ void bits_map(const CompactArgs& a, uint32_t seg, uint32_t c, uint32_t* __restrict__ map,
                                         uint32_t lane) {
  const uint16_t* __restrict__ rp =
      reinterpret_cast<const uint16_t*>(a.fired32 + (uint64_t)seg * a.stride + kRec16Header / 4u);
  map[lane] = 0u;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  for (uint32_t j = lane; j < c; j += 64u) {
    const uint32_t x = rp[j] & 0x7FFu, jj = x >> 8;
    atomicOr(&map[((x >> 2) & 63u) ^ jj], 1u << ((x & 3u) * 8u + jj));
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t nz_bytes(uint32_t d) {
  return (uint32_t)((d & 0xFFu) != 0) + (uint32_t)((d & 0xFF00u) != 0) + (uint32_t)((d & 0xFF0000u) != 0) +
         (uint32_t)((d >> 24) != 0);
}

__global__ __launch_bounds__(kBlock) void bits_size_kernel(CompactArgs a, uint32_t* __restrict__ wc,
                                                           uint32_t* __restrict__ bsum) {
  __shared__ uint32_t s_map[kWavesPerBlock][64];
  __shared__ uint32_t s_c[kWavesPerBlock];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t seg = blockIdx.x * kSegsPerBlock + wave;
  uint32_t c = 0;
  if (seg < a.n_segs) {
    c = a.counts[seg];
    bits_map(a, seg, c, s_map[wave], lane);
    uint32_t z = nz_bytes(s_map[wave][lane]);
    for (int o = 32; o > 0; o >>= 1) z += __shfl_xor(z, o);
    if (lane == 0) {
      reinterpret_cast<uint32_t*>(a.out)[seg] = c | z << 16;
      wc[seg] = 8u + ((z + 3u) >> 2) + ((c + 15u) >> 4);
    }
  }
  if (lane == 0) s_c[wave] = c;
  __syncthreads();
  if (threadIdx.x == 0) bsum[blockIdx.x] = s_c[0] + s_c[1] + s_c[2] + s_c[3];
}

template <bool kSmall>
__global__ __launch_bounds__(kBlock) void bits_write_kernel(CompactArgs a, const uint32_t* __restrict__ wc,
                                                            const uint32_t* __restrict__ bsum, uint32_t* __restrict__ tot) {
  __shared__ uint32_t s_map[kWavesPerBlock][64];
  __shared__ uint32_t s_stage[kWavesPerBlock][64];  // the nonzero map bytes, in order
  __shared__ uint32_t s_sum[kWavesPerBlock][8];
  __shared__ uint32_t s_part[kWavesPerBlock];
  __shared__ uint32_t s_seg[kWavesPerBlock];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t first = blockIdx.x * kSegsPerBlock;
  const uint32_t seg = first + wave;
  const uint32_t n = a.n_segs;
  uint32_t pre = 0;  // P(seg)
  if constexpr (kSmall) {
    const uint4* __restrict__ w4 = reinterpret_cast<const uint4*>(wc);
    uint32_t ws = 0;
#pragma unroll 8
    for (uint32_t q = threadIdx.x; q < first / 4u; q += kBlock) {
      const uint4 v = w4[q];
      ws += (v.x + v.y) + (v.z + v.w);
    }
    for (int o = 32; o > 0; o >>= 1) ws += __shfl_xor(ws, o);
    if (lane == 0) s_part[wave] = ws;
    if (threadIdx.x < kSegsPerBlock) s_seg[threadIdx.x] = first + threadIdx.x < n ? wc[first + threadIdx.x] : 0u;
    __syncthreads();
    if (seg >= n) return;
    pre = s_part[0] + s_part[1] + s_part[2] + s_part[3];
    for (uint32_t w = 0; w < wave; ++w) pre += s_seg[w];
  } else {
    if (seg >= n) return;
    for (uint32_t x = lane; x < seg / kScanGroup; x += 64) pre += a.group_tot[x];
    for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o);
    pre += a.offsets[1 + seg];
  }
  uint32_t* __restrict__ out = reinterpret_cast<uint32_t*>(a.out);
  const uint32_t cz = out[seg];  // bits_size_kernel's {c, z}
  const uint32_t c = cz & 0xFFFFu, z = cz >> 16;
  uint32_t* __restrict__ map = s_map[wave];
  bits_map(a, seg, c, map, lane);
  uint32_t* __restrict__ dst = out + n + pre;
  // summary: lane L's four map bytes are bits 4 (L % 8) .. + 3 of word L / 8; the nonzero bytes
  // staged in LDS at their rank
  const uint32_t d = map[lane];
  const uint32_t f4 = (uint32_t)((d & 0xFFu) != 0) | (uint32_t)((d & 0xFF00u) != 0) << 1 |
                      (uint32_t)((d & 0xFF0000u) != 0) << 2 | (uint32_t)((d >> 24) != 0) << 3;
  uint32_t* __restrict__ sm = s_sum[wave];
  uint32_t* __restrict__ st = s_stage[wave];
  if (lane < 8) sm[lane] = 0u;
  st[lane] = 0u;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (f4) atomicOr(&sm[lane >> 3], f4 << (4u * (lane & 7u)));
  const uint32_t cnt = (uint32_t)__popc(f4);
  const uint32_t incl = wave_incl_scan(cnt);
  uint32_t pb = incl - cnt;
  uint8_t* __restrict__ sb = reinterpret_cast<uint8_t*>(st);
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j)
    if ((f4 >> j) & 1u) sb[pb++] = (uint8_t)(d >> (8u * j));
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (lane < 8) __builtin_nontemporal_store(sm[lane], dst + lane);
  const uint32_t zw = (z + 3u) >> 2;
  if (lane < zw) __builtin_nontemporal_store(st[lane], dst + 8u + lane);
  uint32_t* __restrict__ codes = dst + 8u + zw;
  const uint16_t* __restrict__ rp =
      reinterpret_cast<const uint16_t*>(a.fired32 + (uint64_t)seg * a.stride + kRec16Header / 4u);
  for (uint32_t base = 0; base < c; base += 1024u) {  // 16 records (two 16-byte loads) per lane and word
    const uint32_t i = base + 16u * lane;
    if (i < c) {
      const uint4* q = reinterpret_cast<const uint4*>(rp + i);
      const uint4 r0 = q[0], r1 = q[1];
      const uint32_t dd[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
      uint32_t w = 0;
#pragma unroll
      for (uint32_t t = 0; t < 8; ++t) {
        w |= ((dd[t] >> 11) & 3u) << (4u * t);
        w |= ((dd[t] >> 27) & 3u) << (4u * t + 2u);
      }
      const uint32_t left = c - i;  // codes past the segment's records: zero
      if (left < 16u) w &= (1u << (2u * left)) - 1u;
      __builtin_nontemporal_store(w, codes + i / 16u);
    }
  }
  if (seg == n - 1) {  // the list's words and records
    const uint32_t nb = (n + kSegsPerBlock - 1) / kSegsPerBlock;
    uint32_t r = 0;
    for (uint32_t x = lane; x < nb; x += 64) r += bsum[x];
    for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o);
    if (lane == 0) {
      tot[0] = n + pre + 8u + zw + ((c + 15u) >> 4);
      tot[1] = r;
      a.offsets[0] = tot[0];
      if (a.host_len) {
        a.host_len[0] = tot[0];
        a.host_len[1] = r;
      }
    }
  }
}

// Hand-back in one launch for small sweeps (at most kwk_engine::compact_small segments, 8192 by default: the node kinds, the
// strong-scaling shards): each block sums the counts of every segment before its own (at most
// 32 KB, L2-resident) instead of waiting for seg_scan_kernel, then expands its four segments as
// compact_kernel does.  Saves one launch and its gap per step.
template <int kRec, bool kPacked = false>
__global__ __launch_bounds__(kBlock) void compact_small_kernel(CompactArgs a) {
  __shared__ uint32_t s_part[kWavesPerBlock];
  __shared__ uint32_t s_seg[kWavesPerBlock];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t first = blockIdx.x * kSegsPerBlock;  // the block's first segment
  // the prefix as 16-byte loads (counts is 16-byte aligned, `first` a multiple of 4), eight in
  // flight per thread: one memory round trip up to 8192 segments instead of one per 256
  static_assert(kSegsPerBlock % 4 == 0, "prefix loads assume whole uint4s before the block");
  const uint4* __restrict__ c4 = reinterpret_cast<const uint4*>(a.counts);
  const uint32_t nq = first / 4u;
  uint32_t sum = 0;
#pragma unroll 8
  for (uint32_t q = threadIdx.x; q < nq; q += kBlock) {
    const uint4 v = c4[q];
    sum += (v.x + v.y) + (v.z + v.w);
  }
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  if (lane == 0) s_part[wave] = sum;
  if (threadIdx.x < kSegsPerBlock) s_seg[threadIdx.x] = first + threadIdx.x < a.n_segs ? a.counts[first + threadIdx.x] : 0u;
  __syncthreads();
  const uint32_t seg = first + wave;
  if (seg >= a.n_segs) return;
  uint32_t off = s_part[0] + s_part[1] + s_part[2] + s_part[3];
  for (uint32_t w = 0; w < wave; ++w) off += s_seg[w];
  const uint32_t c = s_seg[wave];
  if (seg == a.n_segs - 1 && lane == 0) {
    a.offsets[0] = off + c;
    if (a.host_len) a.host_len[0] = off + c;
  }
  const uint32_t* __restrict__ sp = a.fired32 + (uint64_t)seg * a.stride;
  const uint32_t base = (seg >> a.seg_region_shift) * a.region_slots;
  for (uint32_t j = lane; j < c; j += 64) {
    const uint2 x = rec_at<kRec>(sp, j);
    store_out<kPacked>(a, off + j, base + x.x, x.y);
  }
}

// sums the per-block statistics rows [0, n_blocks) (the rows any sweep grid has used)
__global__ void reduce_stats_kernel(const unsigned long long* __restrict__ cum, uint32_t n_blocks,
                                    unsigned long long* __restrict__ out) {
  const uint32_t word = blockIdx.x;  // one workgroup per statistic word
  unsigned long long s = 0;
  for (uint32_t b = threadIdx.x; b < n_blocks; b += blockDim.x) s += cum[(uint64_t)b * kStatWords + word];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  __shared__ unsigned long long part[kBlock / 64];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int i = 0; i < kBlock / 64; ++i) t += part[i];
    out[word] = t;
  }
}

struct ScatterArgs {
  void* st;
  StateFmt fmt;
  int64_t* due;
  int64_t* del_s;
  uint32_t* rec_idx;
  const uint32_t* slots;
  const kwk_hot* s_hot;
  const int64_t* s_del;
  const uint32_t* s_rec;
  const uint16_t* s_cls;
  uint32_t n;
  uint32_t mark_dirty;
};

__global__ void scatter_kernel(ScatterArgs a) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= a.n) return;
  const uint32_t i = a.slots[j];
  kwk_hot h = a.s_hot[j];
  h.sched = (h.sched & ~KWK_CLASS_MASK) | ((uint32_t)a.s_cls[j] << KWK_CLASS_SHIFT);
  if (a.mark_dirty) h.sched |= KWK_F_DIRTY;
  store_state_due(a.st, a.due, i, make_uint2(h.pred, h.sched), h.due, a.fmt);
  a.del_s[i] = a.s_del[j];
  a.rec_idx[i] = a.s_rec[j];
}

// Go's math.Pow(x, y) for a non-negative integer y (src/math/pow.go: frexp, then repeated
// squaring of the mantissa with a separate binary exponent, Ldexp at the end), so the
// backoff matches the reference bit for bit
__device__ __forceinline__ double go_pow_int(double x, uint64_t n) {
  if (n == 0 || x == 1.0) return 1.0;
  if (n == 1) return x;
  if (x == 0.0 || isinf(x) || isnan(x)) return pow(x, (double)n);
  double a1 = 1.0;
  int ae = 0;
  int xe;
  double x1 = frexp(x, &xe);
  for (uint64_t i = n; i != 0; i >>= 1) {
    if (xe < -(1 << 12) || (1 << 12) < xe) {  // catastrophic overflow: let Ldexp handle it
      ae += xe;
      break;
    }
    if (i & 1) {
      a1 *= x1;
      ae += xe;
    }
    x1 *= x1;
    xe <<= 1;
    if (x1 < 0.5) {
      x1 += x1;
      xe--;
    }
  }
  return ldexp(a1, ae);
}

// float64 -> time.Duration (int64) as Go converts it on amd64: truncation, out of range ->
// INT64_MIN
__device__ __forceinline__ int64_t go_duration(double d) {
  if (!(d > -9223372036854775808.0 && d < 9223372036854775808.0)) return INT64_MIN;
  return (int64_t)d;
}

struct RetryArgs {
  void* st;
  StateFmt fmt;
  int64_t* due;
  const uint32_t* slots;
  const kwk_hot* hot;
  const uint16_t* cls;
  const uint16_t* stages;
  const uint32_t* retry_count;
  kwk_backoff b;
  uint32_t n;
  uint64_t slot_base;
  uint64_t key;
  uint64_t step;
  int64_t now;
};

// kwk_retry: playStageWorker's retry branch (pod_controller.go:273-284) for each failed job
__global__ void retry_kernel(RetryArgs a) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= a.n) return;
  const uint32_t i = a.slots[j];
  // backoffDelayByStep (utils.go:138-143)
  const double d = fmin((double)a.b.duration_ns * go_pow_int(a.b.factor, a.retry_count[j]), (double)a.b.cap_ns);
  const int64_t base = go_duration(d);
  const double mf = a.b.jitter <= 0.0 ? 1.0 : a.b.jitter;
  const double u = rng_float64(a.slot_base + i, a.step, kSiteRetryJitter, a.key);
  const int64_t delay = base + go_duration(u * mf * (double)base);
  // the unchanged object, its job queued again (no event: not dirty)
  const uint32_t sched = (a.hot[j].sched & ~(KWK_CLASS_MASK | 0xFFu | KWK_F_DIRTY)) |
                         ((uint32_t)a.cls[j] << KWK_CLASS_SHIFT) | (uint32_t)a.stages[j];
  // addStageJob -> AddWeightAfter(job, 1, retryDelay)
  store_state_due(a.st, a.due, i, make_uint2(a.hot[j].pred, sched), sat_add(a.now, delay), a.fmt);
}

__global__ void delete_kernel(void* st, StateFmt fmt, const uint32_t* slots, uint32_t n) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t i = slots[j];
  uint2 v = load_state(st, i, fmt);
  v.y = (v.y & ~(KWK_F_ALIVE | KWK_F_DIRTY | 0xFFu)) | KWK_STAGE_NONE;
  store_state(st, i, v, fmt);
}

// the fused format's due times <-> the due column.  fold: every record's D from the column
// (kDwFar where the time is outside the window: the column already holds it); unfold: the column
// from every record whose D is in the window (the column is then exact for every slot)
// (grid-stride over a bounded grid.  At 100M slots either shape takes 110-140 ms per call in the
// kernel trace (r3ze one workgroup per 256 slots, r3zf grid-stride) for 2.4 GB of traffic: not
// dispatch-bound, cause not found; load-time only)
__global__ void dw_fold_kernel(uint2* __restrict__ st, const int64_t* __restrict__ due, uint32_t first, uint32_t n,
                               int64_t epoch) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    const uint32_t i = first + j;
    st[i] = dw_put(st[i], dw_enc(due[i], epoch));
  }
}
__global__ void dw_unfold_kernel(const uint2* __restrict__ st, int64_t* __restrict__ due, uint32_t first, uint32_t n,
                                 int64_t epoch) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    const uint32_t i = first + j;
    const uint64_t d = dw_get(st[i]);
    if (d != kDwFar) due[i] = dw_abs(d, epoch);
  }
}

// ------------------------------------------------------------------ resource usage
// server/metrics_resource_usage.go:170-224 (pod / node sums), :36-109 (cumulative integrators).
// The pods are node-sorted (node_ptr CSR).  kwk_usage_config cuts the node list into chunks of
// whole nodes holding at most kUChunkPods pods (and kUChunkNodes nodes); one wave per chunk.
// Each lane owns kURun consecutive pods (the wave's row of 64 x kURun slots starts at the
// chunk's first pod rounded down to 8, so every lane's state / usage-key bytes are whole
// 16-byte loads) and adds them up in order, closing a node where its pods end:
//  * a node whose first pod lies in the lane is complete in the lane: finalised there;
//  * the lane's first node may have started in earlier lanes (its "head"), its last may go on
//    in later lanes (its open "tail"): one segmented scan over the lanes' tails (keyed by node,
//    pods of a node are contiguous) gives the earlier lanes' share, which the lane that closes
//    the node adds to its head.  Nodes larger than a row carry their sum into the next row.
// So a node sum costs one cross-lane scan per 64 x kURun pods instead of one per 64, and the
// stream is read with wide loads.  A pod contributes containers x its interned cpu / memory
// value (dead pods — not in the pod cache — nothing), containers added in spec order (:170-193).
// The reference adds pods in SyncMap order (unordered, utils/maps/sync.go:93-100), so sums agree
// with it to floating-point reassociation: the tests hold them to 1e-6 relative (north_star);
// the order here is fixed, so results are reproducible run to run.
// With per-pod outputs enabled (kwk_usage_pods) every pod also gets its Usage (podResourceUsage,
// :170-193) and its cumulative usage (podResourceCumulativeUsage, :54-65: the sum of its
// containers' integrators, each advanced by (now - last) * value, :36-52); a dead pod reads 0
// and keeps its integrators (Go keys them by name, so a re-created pod continues them).
constexpr uint32_t kURun = 16;                  // consecutive pods per lane
constexpr uint32_t kURow = 64u * kURun;         // slots per wave row
constexpr uint32_t kUChunkRows = 4;            // rows per chunk: the per-chunk costs
                                                // (descriptor, node boundaries, integrators, node stores) spread
                                                // over up to 4 rows, whose loads run one row ahead
constexpr uint32_t kUChunkPods = kURow - 8u;    // pods of a one-row chunk: it fits one row even after rounding its
                                                // start down to 8; an R-row chunk holds R * kURow - 8
constexpr uint32_t kUChunkNodes = 128;          // nodes per chunk: the wave's LDS copy of node_ptr
constexpr uint32_t kULdsValues = 512;           // cpu + mem dictionary entries staged in LDS (else read via L1)
constexpr int kMaxCountMasks = 16;  // kwk_count / kwk_aggregate masks per call
struct UsageArgs {
  const void* __restrict__ st;
  StateFmt fmt;
  const uint32_t* __restrict__ node_ptr;
  const uint32_t* __restrict__ ukey;
  const double* __restrict__ cpu_v;
  const double* __restrict__ mem_v;
  uint32_t n_cpu, n_mem;
  const uint4* __restrict__ chunks;  // {first pod, end pod, first node, end node}
  uint32_t n_chunks;
  uint32_t n_pods;
  double* __restrict__ node_out;   // n_nodes x {cpu, mem, cpu_cum, mem_cum}
  double* __restrict__ cum;        // n_nodes x {cpu, mem}
  int64_t* __restrict__ last_t;
  int64_t now;
  double* __restrict__ block_part;  // per block {cpu, mem}
  double* __restrict__ pod_out;     // optional per pod outputs
  double* __restrict__ pod_cum;     // per pod: one container's integrators (uniform pods)
  int64_t* __restrict__ pod_last;
  const uint2* __restrict__ mixed;  // pods whose containers differ: {first, count} into ckeys
  const uint32_t* __restrict__ ckeys;
  const uint32_t* __restrict__ mbase;  // per pod: its containers' first integrator in ccum (mixed pods)
  double* __restrict__ ccum;        // per container of a mixed pod: {cpu, mem} integrators
  const double* __restrict__ podv;  // usage_fast_kernel: pod values per (containers, value id), see kwk_usage_config
  uint32_t podv_n;                  // entries of podv
  const uint8_t* __restrict__ ukey8;  // usage_fast_kernel<WB, true>: per pod, an index into kv
  const double2* __restrict__ kv;     // {cpu, mem} value of each distinct usage key (<= kUKeyDict)
  uint32_t kv_n;
  // usage_fast_kernel<1, true> with kwk_aggregate's mask counts folded in (n_cmasks 1..4, 0: none):
  // count8_kernel's per-id table over the same id rows, partial rows per block into cpart
  const uint32_t* __restrict__ cmasks;
  uint32_t n_cmasks;
  uint32_t* __restrict__ cpart;       // [grid][kMaxCountMasks]
};
constexpr uint32_t kUKeyDict = 256;  // entries of the 1-byte key column's value table
constexpr uint32_t kUKeyZero = 255;  // its entry {0, 0}: the key a dead / out-of-range pod reads, so at
                                     // most 255 distinct keys take the 1-byte column
constexpr uint32_t kUSeqKeys = 16;   // keys whose in-order sums of 0..16 pods usage_fast_kernel keeps in LDS

// a pod's usage_key: containers (bits 28..31) x one interned value each, or 0 containers =
// a pod whose containers differ: bits 0..27 index its {first, count} entry of the mixed table
constexpr uint32_t kUKeyMixedIndex = 0x0FFFFFFFu;

// time.Duration.Seconds() of now - last
__device__ __forceinline__ double dur_seconds(int64_t d) {
  return (double)(d / 1000000000) + (double)(d % 1000000000) / 1e9;
}

// alive flag of pod j of a lane's run (kURun words of WB bytes in WB 16-byte chunks)
template <uint32_t WB>
__device__ __forceinline__ bool run_alive(const uint4 (&sv)[WB], int j, uint32_t abit, bool px) {
  if constexpr (WB == 1) {  // 1-byte ids: the alive bit is an id bit (kIdAlive)
    const uint4 c = sv[0];
    const int d = j >> 2;
    const uint32_t w = d == 0 ? c.x : d == 1 ? c.y : d == 2 ? c.z : c.w;
    return ((w >> (8 * (j & 3))) & abit) != 0;
  } else if constexpr (WB == 2) {
    const uint4 c = sv[j >> 3];
    const int d = (j >> 1) & 3;
    const uint32_t w = d == 0 ? c.x : d == 1 ? c.y : d == 2 ? c.z : c.w;
    return ((w >> (16 * (j & 1))) & abit) != 0;
  } else if constexpr (WB == 4) {
    const uint4 c = sv[j >> 2];
    const int d = j & 3;
    return ((d == 0 ? c.x : d == 1 ? c.y : d == 2 ? c.z : c.w) & abit) != 0;
  } else {
    const uint4 c = sv[j >> 1];
    // the sched word of {pred, sched}; px: the packed word of a fused record
    return ((px ? ((j & 1) ? c.z : c.x) : ((j & 1) ? c.w : c.y)) & abit) != 0;
  }
}

// the alive bits (kIdAlive) of a lane's 16 1-byte ids as a 16-bit mask, bit j = pod j of the run:
// per dword the four bits at 0 / 8 / 16 / 24 meet at bits 21-24 of one multiply (no carries)
__device__ __forceinline__ uint32_t alive16_ids(const uint4 c) {
  const uint32_t dw[4] = {c.x, c.y, c.z, c.w};
  uint32_t m = 0;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t a = (dw[d] >> 5) & 0x01010101u;
    m |= (((a * 0x204081u) >> 21) & 15u) << (4 * d);
  }
  return m;
}

// DPP helpers of the usage kernels' lane scans (GFX9 DPP: row_shr, row_bcast15/31, wave_shr);
// a lane whose source is outside its row or the row mask keeps `old` (0.0 / the no-node key)
template <int C, int RM>
__device__ __forceinline__ double dpp_f64(double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, C, RM, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), C, RM, 0xF, false);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
template <int C, int RM>
__device__ __forceinline__ uint32_t dpp_key(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFFu, (int)v, C, RM, 0xF, false);
}
template <int C, int RM>
__device__ __forceinline__ void dpp_seg_step(double& sc, double& sm, const uint32_t key) {
  const double uc = dpp_f64<C, RM>(sc), um = dpp_f64<C, RM>(sm);
  const uint32_t uk = dpp_key<C, RM>(key);
  if (uk == key) { sc += uc; sm += um; }
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// persistent grid: wave w takes chunks w, w + W, ... (W = waves in the grid); the next chunk's
// descriptor and first row are requested before the current chunk is worked on, so each
// wave keeps one chunk's loads in flight (one block per chunk paid 3 memory latencies per
// chunk back to back: 236-255 us for 100M pods, r2c-r2e)
template <uint32_t WB>
__global__ __launch_bounds__(kBlock) void usage_kernel(UsageArgs a) {
  __shared__ uint32_t s_ptr[kWavesPerBlock][kUChunkNodes + 1];
  __shared__ double2 s_sum[kWavesPerBlock][kUChunkNodes];  // node sums, each written once where the node closes
  __shared__ double s_val[kULdsValues];
  __shared__ double s_c[kWavesPerBlock], s_m[kWavesPerBlock];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t n_waves = gridDim.x * kWavesPerBlock;
  uint32_t chunk = blockIdx.x * kWavesPerBlock + wave;
  // range-checked per dword: a size that ends inside a dword would zero the last pods' bytes of
  // it (ids of 1-2 bytes), so the size is rounded up to whole 16-byte loads (the columns are
  // padded; pods past the chunk's end are masked out by the lanes' ranges)
  const __amdgpu_buffer_rsrc_t st_rs = make_rsrc(a.st, (a.n_pods * WB + 15u) & ~15u);
  const __amdgpu_buffer_rsrc_t uk_rs = make_rsrc(a.ukey, a.n_pods * 4u);
  // the next chunk: descriptor and first row in flight
  uint4 nch = make_uint4(0u, 0u, 0u, 0u);
  uint4 nsv[WB], nkv[4];
  auto load_row = [&](uint4 (&dsv)[WB], uint4 (&dkv)[4], uint32_t r0, uint32_t c0, uint32_t c1) {
    const uint32_t lf = r0 + lane * kURun;
    const bool has = max(lf, c0) < min(lf + kURun, c1);
#pragma unroll
    for (uint32_t q = 0; q < WB; ++q) {
      const auto c = __builtin_amdgcn_raw_buffer_load_b128(st_rs, has ? lf * WB + q * 16u : kOOB, 0, 0);
      dsv[q] = make_uint4(c[0], c[1], c[2], c[3]);
    }
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
      const auto c = __builtin_amdgcn_raw_buffer_load_b128(uk_rs, has ? lf * 4u + q * 16u : kOOB, 0, 0);
      dkv[q] = make_uint4(c[0], c[1], c[2], c[3]);
    }
  };
  if (chunk < a.n_chunks) {
    nch = a.chunks[chunk];
    load_row(nsv, nkv, nch.x & ~7u, nch.x, nch.y);
  }
  const bool lds_vals = a.n_cpu + a.n_mem <= kULdsValues;
  if (lds_vals) {
    for (uint32_t j = threadIdx.x; j < a.n_cpu + a.n_mem; j += kBlock)
      s_val[j] = j < a.n_cpu ? a.cpu_v[j] : a.mem_v[j - a.n_cpu];
  }
  __syncthreads();
  const double* __restrict__ cpu_v = lds_vals ? s_val : a.cpu_v;
  const double* __restrict__ mem_v = lds_vals ? s_val + a.n_cpu : a.mem_v;
  // the alive flag in the raw word (packed: at fshift; wide: in sched)
  const uint32_t abit = WB == 1 ? kIdAlive : (WB == 8 && !a.fmt.dw) ? (uint32_t)KWK_F_ALIVE
                                                                   : (uint32_t)(KWK_F_ALIVE >> 8) << a.fmt.fshift;
  double tot_c = 0.0, tot_m = 0.0;  // per lane: the nodes it finalised
  uint32_t* __restrict__ sp = s_ptr[wave];
  double2* __restrict__ ss = s_sum[wave];
  for (; chunk < a.n_chunks; chunk += n_waves) {  // wave-uniform
    const uint4 ch = nch;
    const uint32_t c0 = ch.x, c1 = ch.y, na = ch.z, nk = ch.w - ch.z;  // pods [c0, c1), nodes na + [0, nk)
    const uint32_t r_first = c0 & ~7u;
    uint4 sv[WB], kv[4];
#pragma unroll
    for (uint32_t q = 0; q < WB; ++q) sv[q] = nsv[q];
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) kv[q] = nkv[q];
    const uint32_t nxt = chunk + n_waves;
    if (nxt < a.n_chunks) nch = a.chunks[nxt];
    // the first 64 nodes' integrators and the node boundaries
    double2 pre_cum = make_double2(0.0, 0.0);
    int64_t pre_last = INT64_MIN;
    if (lane < nk) {
      pre_cum = reinterpret_cast<const double2*>(a.cum)[na + lane];
      pre_last = a.last_t[na + lane];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the previous chunk is done with sp / ss
    for (uint32_t j = lane; j <= nk; j += 64) sp[j] = a.node_ptr[na + j];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // a node's sum is final where it closes (in LDS); the integrators and outputs are written
    // after the rows, all lanes at once
    auto finalize = [&](uint32_t k, double c, double m) { ss[k] = make_double2(c, m); };
    if (c0 == c1) {  // nodes without pods
      for (uint32_t k = lane; k < nk; k += 64) finalize(k, 0.0, 0.0);
    }
    double carry_c = 0.0, carry_m = 0.0;  // the open node's sum from earlier rows
    uint32_t carry_k = 0xFFFFFFFFu;
    if (r_first >= c1)  // no rows (a chunk of empty nodes): the next chunk's first row
      load_row(nsv, nkv, nch.x & ~7u, nch.x, nxt < a.n_chunks ? nch.y : 0u);
    for (uint32_t r0 = r_first; r0 < c1; r0 += kURow) {  // wave-uniform
      if (r0 != r_first) {  // the row loaded during the previous one
#pragma unroll
        for (uint32_t q = 0; q < WB; ++q) sv[q] = nsv[q];
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) kv[q] = nkv[q];
      }
      {  // one row ahead: the chunk's next row, or after its last the next chunk's first
        const bool more = r0 + kURow < c1;
        load_row(nsv, nkv, more ? r0 + kURow : nch.x & ~7u, more ? c0 : nch.x, more ? c1 : nxt < a.n_chunks ? nch.y : 0u);
      }
      const uint32_t lf = r0 + lane * kURun;
      const uint32_t p_lo = max(lf, c0), p_hi = min(lf + kURun, c1);
      const bool has = p_lo < p_hi;
      // the node holding the lane's pod before its first (the chunk's first lane: node 0)
      uint32_t k = 0;
      if (has && p_lo > c0) {
        uint32_t lo = 0, hi = nk;
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (sp[mid] <= p_lo - 1u) lo = mid; else hi = mid;
        }
        k = lo;
      }
      double acc_c = 0.0, acc_m = 0.0, head_c = 0.0, head_m = 0.0;
      bool head = false;
      uint32_t head_k = 0;
      uint32_t bnd = sp[k + 1];  // end of node k
      auto close = [&]() {
        if (!head && sp[k] < p_lo) {  // started in an earlier lane: the head
          head = true;
          head_k = k;
          head_c = acc_c;
          head_m = acc_m;
        } else {
          finalize(k, acc_c, acc_m);
        }
        acc_c = 0.0;
        acc_m = 0.0;
        ++k;
        bnd = k < nk ? sp[k + 1] : 0xFFFFFFFFu;
      };
#pragma unroll
      for (int j = 0; j < (int)kURun; ++j) {
        const uint32_t p = lf + (uint32_t)j;
        if (p < p_lo || p >= p_hi) continue;
        while (p >= bnd) close();
        const uint4 kq = kv[j >> 2];
        const uint32_t key = (j & 3) == 0 ? kq.x : (j & 3) == 1 ? kq.y : (j & 3) == 2 ? kq.z : kq.w;
        const bool alive = run_alive<WB>(sv, j, abit, a.fmt.dw != 0);
        const uint32_t nc = key >> 28;
        double vc = 0.0, vm = 0.0, c1v = 0.0, m1v = 0.0;
        uint2 fc = make_uint2(0u, 0u);
        if (alive) {
          if (nc) {
            c1v = cpu_v[key & 0x3FFFu];
            m1v = mem_v[(key >> 14) & 0x3FFFu];
            for (uint32_t c = 0; c < nc; ++c) { vc += c1v; vm += m1v; }
          } else {
            fc = a.mixed[key & kUKeyMixedIndex];
            for (uint32_t c = 0; c < fc.y; ++c) {
              const uint32_t ck = a.ckeys[fc.x + c];
              vc += cpu_v[ck & 0x3FFFu];
              vm += mem_v[(ck >> 14) & 0x3FFFu];
            }
          }
        }
        if (a.pod_out) {
          if (alive) {
            // containerResourceCumulativeUsage (:36-52): one integrator per container, advanced
            // by (now - last) * value; the pod's is their sum (:54-65)
            const int64_t lt = a.pod_last[p];
            const double dt = lt != INT64_MIN ? dur_seconds(a.now - lt) : 0.0;
            double cc = 0.0, cm = 0.0;
            if (nc) {  // equal containers share one integrator
              double2 unit = reinterpret_cast<double2*>(a.pod_cum)[p];
              if (lt != INT64_MIN) {
                unit.x += dt * c1v;
                unit.y += dt * m1v;
                reinterpret_cast<double2*>(a.pod_cum)[p] = unit;
              }
              for (uint32_t c = 0; c < nc; ++c) { cc += unit.x; cm += unit.y; }
            } else {
              const uint32_t mb = a.mbase[p];
              for (uint32_t c = 0; c < fc.y; ++c) {
                const uint32_t ck = a.ckeys[fc.x + c];
                double2 cu = reinterpret_cast<double2*>(a.ccum)[mb + c];
                if (lt != INT64_MIN) {
                  cu.x += dt * cpu_v[ck & 0x3FFFu];
                  cu.y += dt * mem_v[(ck >> 14) & 0x3FFFu];
                  reinterpret_cast<double2*>(a.ccum)[mb + c] = cu;
                }
                cc += cu.x;
                cm += cu.y;
              }
            }
            a.pod_last[p] = a.now;
            reinterpret_cast<double4*>(a.pod_out)[p] = make_double4(vc, vm, cc, cm);
          } else {
            reinterpret_cast<double4*>(a.pod_out)[p] = make_double4(0.0, 0.0, 0.0, 0.0);
          }
        }
        acc_c += vc;
        acc_m += vm;
      }
      // the chunk's last pod: close every node left (trailing nodes without pods too)
      const bool last = has && p_hi == c1;
      if (last)
        while (k < nk) close();
      // segmented inclusive scan of the open tails (keys ascend over the lanes with pods)
      const uint32_t key = (has && !last) ? k : 0xFFFFFFFFu;
      double sc = (has && !last) ? acc_c : 0.0, sm = (has && !last) ? acc_m : 0.0;
      if (lane == 0 && key == carry_k) { sc += carry_c; sm += carry_m; }
      dpp_seg_step<0x111, 0xF>(sc, sm, key);  // on DPP lane moves (dpp_seg_step)
      dpp_seg_step<0x112, 0xF>(sc, sm, key);
      dpp_seg_step<0x114, 0xF>(sc, sm, key);
      dpp_seg_step<0x118, 0xF>(sc, sm, key);
      dpp_seg_step<0x142, 0xA>(sc, sm, key);
      dpp_seg_step<0x143, 0xC>(sc, sm, key);
      // the lane before a head ends with that node open: its scan value is the earlier share
      double pc = dpp_f64<0x138, 0xF>(sc), pm = dpp_f64<0x138, 0xF>(sm);  // wave_shr:1
      if (lane == 0) { pc = carry_c; pm = carry_m; }
      if (head) finalize(head_k, head_c + pc, head_m + pm);
      carry_c = readlane_f64(sc, 63);
      carry_m = readlane_f64(sm, 63);
      carry_k = (uint32_t)__builtin_amdgcn_readlane((int)key, 63);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // NodeResourceUsage (:195-224) and its integrator (nodeResourceCumulativeUsage, :67-109)
    for (uint32_t k = lane; k < nk; k += 64) {
      const double2 v = ss[k];
      const uint64_t node = na + k;
      double2 cm = k == lane ? pre_cum : reinterpret_cast<double2*>(a.cum)[node];
      const int64_t lt = k == lane ? pre_last : a.last_t[node];
      if (lt != INT64_MIN) {  // now.Sub(c.time).Seconds()
        const double dt = dur_seconds(a.now - lt);
        cm.x += dt * v.x;
        cm.y += dt * v.y;
        reinterpret_cast<double2*>(a.cum)[node] = cm;
      }
      a.last_t[node] = a.now;
      reinterpret_cast<double4*>(a.node_out)[node] = make_double4(v.x, v.y, cm.x, cm.y);
      tot_c += v.x;
      tot_m += v.y;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    tot_c += __shfl_xor(tot_c, o);
    tot_m += __shfl_xor(tot_m, o);
  }
  if (lane == 0) { s_c[wave] = tot_c; s_m[wave] = tot_m; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double tc = 0, tm = 0;
    for (int i = 0; i < kWavesPerBlock; ++i) { tc += s_c[i]; tm += s_m[i]; }
    a.block_part[blockIdx.x * 2 + 0] = tc;
    a.block_part[blockIdx.x * 2 + 1] = tm;
  }
}

// The common configuration — every pod's containers evaluate alike (no mixed table) and no
// per-pod outputs — takes usage_fast_kernel: the same chunks, lanes and scan, but a pod's value
// is one LDS lookup in `podv` (containers x value, summed on the host in spec order exactly as
// the device loop would), and a node boundary inside a lane is a short masked branch.  Empty
// nodes are written separately, so closing a node never loops.
constexpr uint32_t kUFastVals = 2048;  // podv entries staged in LDS
// kKey8: the pods' usage keys as one byte each (an index into the distinct keys' {cpu, mem}
// values, kwk_usage_config builds it when at most kUKeyDict keys occur): 16 bytes per lane's run
// instead of 64, one LDS read per pod instead of two and no key decode
template <uint32_t WB, bool kKey8 = false>
__global__ __launch_bounds__(kBlock) void usage_fast_kernel(UsageArgs a) {
  constexpr uint32_t KQ = kKey8 ? 1u : 4u;  // 16-byte key chunks per lane's run
  __shared__ uint32_t s_ptr[kWavesPerBlock][kUChunkNodes + 1];
  __shared__ double2 s_sum[kWavesPerBlock][kUChunkNodes];
  __shared__ double s_pv[kKey8 ? 1 : kUFastVals];
  __shared__ double2 s_kv[kKey8 ? kUKeyDict : 1];
  __shared__ uint32_t s_nib[16];
  // s_seq[k][n]: the in-order sum of n pods of key k (0.0 + v + v + ..., n adds), keys < kUSeqKeys:
  // a lane's run whose 16 keys are one key sums to the entry of its live-pod count, bit for bit
  // the per-pod sums below (a masked pod adds the zero entry, and s + 0.0 == s)
  __shared__ double2 s_seq[kKey8 && WB == 1 ? kUSeqKeys : 1][kURun + 1];
  constexpr bool kCnt = kKey8 && WB == 1;  // mask counts can ride along (a.n_cmasks)
  __shared__ uint32_t s_clut[kCnt ? 256 : 1];
  __shared__ unsigned int s_ccnt[kCnt ? 4 : 1];
  __shared__ double s_c[kWavesPerBlock], s_m[kWavesPerBlock];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t n_waves = gridDim.x * kWavesPerBlock;
  uint32_t chunk = blockIdx.x * kWavesPerBlock + wave;
  // range-checked per dword: a size that ends inside a dword would zero the last pods' bytes of
  // it (ids of 1-2 bytes), so the size is rounded up to whole 16-byte loads (the columns are
  // padded; pods past the chunk's end are masked out by the lanes' ranges)
  const __amdgpu_buffer_rsrc_t st_rs = make_rsrc(a.st, (a.n_pods * WB + 15u) & ~15u);
  const __amdgpu_buffer_rsrc_t uk_rs = kKey8 ? make_rsrc(a.ukey8, (a.n_pods + 15u) & ~15u) : make_rsrc(a.ukey, a.n_pods * 4u);
  uint4 nch = make_uint4(0u, 0u, 0u, 0u);
  uint4 nsv[WB], nkv[KQ];
  auto load_row = [&](uint4 (&dsv)[WB], uint4 (&dkv)[KQ], uint32_t r0, uint32_t c0, uint32_t c1) {
    const uint32_t lf = r0 + lane * kURun;
    const bool has = max(lf, c0) < min(lf + kURun, c1);
#pragma unroll
    for (uint32_t q = 0; q < WB; ++q) {
      const auto c = __builtin_amdgcn_raw_buffer_load_b128(st_rs, has ? lf * WB + q * 16u : kOOB, 0, 0);
      dsv[q] = make_uint4(c[0], c[1], c[2], c[3]);
    }
#pragma unroll
    for (uint32_t q = 0; q < KQ; ++q) {
      const auto c = __builtin_amdgcn_raw_buffer_load_b128(uk_rs, has ? lf * (kKey8 ? 1u : 4u) + q * 16u : kOOB, 0, 0);
      dkv[q] = make_uint4(c[0], c[1], c[2], c[3]);
    }
  };
  // a chunk's node boundaries and its nodes' integrators, loaded one chunk ahead like its row
  // (they were the first thing each chunk waited for: one global round trip per chunk)
  uint32_t nnp[3];
  double2 npc = make_double2(0.0, 0.0);
  int64_t npl = INT64_MIN;
  auto load_meta = [&](const uint4 c, uint32_t (&np)[3], double2& pc, int64_t& pl) {
    const uint32_t na_ = c.z, nk_ = c.w - c.z;  // nk_ <= kUChunkNodes = 128: entries 0..128
#pragma unroll
    for (uint32_t t = 0; t < 3; ++t) {
      const uint32_t j = lane + 64u * t;
      np[t] = j <= nk_ ? a.node_ptr[na_ + j] : 0u;
    }
    pc = make_double2(0.0, 0.0);
    pl = INT64_MIN;
    if (lane < nk_) {
      pc = reinterpret_cast<const double2*>(a.cum)[na_ + lane];
      pl = a.last_t[na_ + lane];
    }
  };
  uint4 nch2 = make_uint4(0u, 0u, 0u, 0u);  // descriptor two chunks ahead
  if (chunk < a.n_chunks) {
    nch = a.chunks[chunk];
    load_row(nsv, nkv, nch.x & ~7u, nch.x, nch.y);
    load_meta(nch, nnp, npc, npl);
  }
  if (chunk + n_waves < a.n_chunks) nch2 = a.chunks[chunk + n_waves];
  if (kKey8) {
    for (uint32_t j = threadIdx.x; j < kUKeyDict; j += kBlock) s_kv[j] = j < a.kv_n ? a.kv[j] : make_double2(0.0, 0.0);
    if (threadIdx.x < 16) {  // s_nib[x]: byte i = 0xFF where bit i of x is clear (that pod reads kUKeyZero)
      uint32_t m = 0;
      for (uint32_t i = 0; i < 4; ++i) m |= ((threadIdx.x >> i) & 1u) ? 0u : 0xFFu << (8 * i);
      s_nib[threadIdx.x] = m;
    }
    if constexpr (kCnt) {
      if (a.n_cmasks) {  // count8_kernel's table: byte m of entry id = 1 if the id counts for mask m
        const uint2 v = fmt_unpack(a.fmt.id2w[threadIdx.x], a.fmt);
        const uint32_t al = (v.y & KWK_F_ALIVE) ? 1u : 0u;
        uint32_t x = 0;
        for (uint32_t m = 0; m < a.n_cmasks; ++m) {
          const uint32_t mk = a.cmasks[m];
          x |= (al & ((mk == 0u || (v.x & mk) != 0u) ? 1u : 0u)) << (8 * m);
        }
        s_clut[threadIdx.x] = x;  // kBlock = 256 threads: one entry each
        if (threadIdx.x < 4) s_ccnt[threadIdx.x] = 0;
      }
    }
  } else {
    for (uint32_t j = threadIdx.x; j < a.podv_n; j += kBlock) s_pv[j] = a.podv[j];
  }
  __syncthreads();
  if constexpr (kKey8 && WB == 1) {  // s_seq: one thread per (key, cpu | memory), n = 0..kURun in order
    if (threadIdx.x < 2 * kUSeqKeys) {
      const uint32_t k = threadIdx.x >> 1;
      const double v = (threadIdx.x & 1) ? s_kv[k].y : s_kv[k].x;
      double* col = reinterpret_cast<double*>(&s_seq[k][0]) + (threadIdx.x & 1);
      double s = 0.0;
      col[0] = s;
      for (uint32_t n = 1; n <= kURun; ++n) {
        s += v;
        col[2 * n] = s;
      }
    }
    __syncthreads();
  }
  const uint32_t nv = a.n_cpu + a.n_mem;  // podv row: cpu values then memory values
  const uint32_t abit = WB == 1 ? kIdAlive : (WB == 8 && !a.fmt.dw) ? (uint32_t)KWK_F_ALIVE
                                                                   : (uint32_t)(KWK_F_ALIVE >> 8) << a.fmt.fshift;
  double tot_c = 0.0, tot_m = 0.0;
  uint32_t* __restrict__ sp = s_ptr[wave];
  double2* __restrict__ ss = s_sum[wave];
  const bool cnt_on = kCnt && a.n_cmasks != 0;  // uniform
  uint32_t ccnt[4] = {0u, 0u, 0u, 0u};          // per lane: pods counted for masks 0..3
  for (; chunk < a.n_chunks; chunk += n_waves) {  // wave-uniform
    const uint4 ch = nch;
    const uint32_t c0 = ch.x, c1 = ch.y, na = ch.z, nk = ch.w - ch.z;
    const uint32_t r_first = c0 & ~7u;
    uint4 sv[WB], kv[KQ];
#pragma unroll
    for (uint32_t q = 0; q < WB; ++q) sv[q] = nsv[q];
#pragma unroll
    for (uint32_t q = 0; q < KQ; ++q) kv[q] = nkv[q];
    uint32_t cnp[3];
#pragma unroll
    for (uint32_t t = 0; t < 3; ++t) cnp[t] = nnp[t];
    const double2 pre_cum = npc;
    const int64_t pre_last = npl;
    const uint32_t nxt = chunk + n_waves;
    nch = nch2;  // the next chunk's descriptor, loaded one chunk ago
    if (nxt + n_waves < a.n_chunks) nch2 = a.chunks[nxt + n_waves];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the previous chunk is done with sp / ss
#pragma unroll
    for (uint32_t t = 0; t < 3; ++t)
      if (lane + 64u * t <= nk) sp[lane + 64u * t] = cnp[t];
    if (nxt < a.n_chunks) load_meta(nch, nnp, npc, npl);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (uint32_t k = lane; k < nk; k += 64)  // nodes without pods
      if (sp[k] == sp[k + 1]) ss[k] = make_double2(0.0, 0.0);
    double carry_c = 0.0, carry_m = 0.0;
    uint32_t carry_k = 0xFFFFFFFFu;
    if (r_first >= c1)  // no rows (a chunk of empty nodes): the next chunk's first row
      load_row(nsv, nkv, nch.x & ~7u, nch.x, nxt < a.n_chunks ? nch.y : 0u);
    for (uint32_t r0 = r_first; r0 < c1; r0 += kURow) {  // wave-uniform
      if (r0 != r_first) {  // the row loaded during the previous one
#pragma unroll
        for (uint32_t q = 0; q < WB; ++q) sv[q] = nsv[q];
#pragma unroll
        for (uint32_t q = 0; q < KQ; ++q) kv[q] = nkv[q];
      }
      {  // one row ahead: the chunk's next row, or after its last the next chunk's first
        const bool more = r0 + kURow < c1;
        load_row(nsv, nkv, more ? r0 + kURow : nch.x & ~7u, more ? c0 : nch.x, more ? c1 : nxt < a.n_chunks ? nch.y : 0u);
      }
      const uint32_t lf = r0 + lane * kURun;
      const uint32_t p_lo = max(lf, c0), p_hi = min(lf + kURun, c1);
      const bool has = p_lo < p_hi;
      // the non-empty node holding the lane's first pod (the last k with sp[k] <= p_lo): from the
      // chunk's mean node size: the guess's own bounds decide it for equal-sized nodes, else a
      // binary search over the side of the guess that holds it
      uint32_t k = 0;
      if (has) {
        const float f = (float)(p_lo - c0) * ((float)nk / (float)(c1 - c0));
        const uint32_t g = min((uint32_t)f, nk - 1u);
        uint32_t lo = 0, hi = nk;  // the node is in [lo, hi)
        if (sp[g] > p_lo) hi = g;
        else if (sp[g + 1u] <= p_lo) lo = g + 1u;
        else { lo = g; hi = g + 1u; }
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (sp[mid] <= p_lo) lo = mid; else hi = mid;
        }
        k = lo;
      }
      // its start decides whether the lane's first segment is a head (continues earlier lanes)
      const bool cont = has && sp[k] < p_lo;
      bool head = false;
      uint32_t head_k = 0;
      double acc_c = 0.0, acc_m = 0.0, head_c = 0.0, head_m = 0.0;
      uint32_t bnd = sp[k + 1];
      bool done = false;  // the row's pods summed by the branch-free path below
      if constexpr (kKey8 && WB == 1) {
        // every lane's run crosses at most one node boundary (nodes of >= 16 pods, C5's 100): its
        // pods before the boundary and from it are summed separately without branches — a pod
        // that is dead, out of range or on the other side reads the zero entry kUKeyZero, so each
        // sum is the in-order sum of its pods exactly as the per-pod loop adds them
        uint32_t k2 = k, nb2 = bnd;
        const bool has_b = has && bnd < p_hi;
        if (has_b) {  // the node holding pod bnd (past nodes without pods)
          k2 = k + 1;
          while (sp[k2 + 1] <= bnd) ++k2;
          nb2 = sp[k2 + 1];
        }
        if (!ballot(has_b && nb2 < p_hi)) {  // wave-uniform: no run crosses two boundaries
          done = true;
          const uint32_t lo = has ? p_lo - lf : 0u, hi = has ? p_hi - lf : 0u, jb = has_b ? bnd - lf : hi;
          const uint32_t alive = alive16_ids(sv[0]);
          if constexpr (kCnt) {
            if (cnt_on) {  // the row's pods [lo, hi) by id (an out-of-range pod reads id 0: counts nothing)
              const uint32_t rng = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
              const uint32_t ids[4] = {sv[0].x, sv[0].y, sv[0].z, sv[0].w};
              uint32_t acc = 0;  // four byte counters (<= 16 each)
#pragma unroll
              for (int d = 0; d < 4; ++d) {
                const uint32_t q = ids[d] & ~s_nib[(rng >> (4 * d)) & 15u];
#pragma unroll
                for (int b = 0; b < 4; ++b) acc += s_clut[(q >> (8 * b)) & 0xFFu];
              }
#pragma unroll
              for (int m = 0; m < 4; ++m) ccnt[m] += (acc >> (8 * m)) & 0xFFu;
            }
          }
          const uint32_t m_a = alive & ((1u << jb) - 1u) & ~((1u << lo) - 1u);  // pods [lo, jb)
          const uint32_t m_b = alive & ((1u << hi) - 1u) & ~((1u << jb) - 1u);  // pods [jb, hi)
          uint4 kq = kv[0];  // one key dword (4 pods) per step, rotated: 8 values in flight, not 32
          uint32_t qa = m_a, qb = m_b;
          double ac = 0.0, am = 0.0, bc = 0.0, bm = 0.0;
          // one key over the lane's 16 pods (a lane without pods reads the n = 0 entries): the sums
          // are s_seq entries; the wave takes the per-pod loop if any lane's keys differ
          const uint32_t k0 = kq.x & 0xFFu, rep = k0 * 0x01010101u;
          const bool one = !has || (kq.x == rep && kq.y == rep && kq.z == rep && kq.w == rep && k0 < kUSeqKeys);
          const int d_end = ballot(!one) ? 4 : 0;  // wave-uniform
          if (d_end == 0) {
            const uint32_t ks = has ? k0 : 0u;
            const double2 sa = s_seq[ks][__popc(m_a)], sb = s_seq[ks][__popc(m_b)];
            ac = sa.x;
            am = sa.y;
            bc = sb.x;
            bm = sb.y;
          }
#pragma unroll 1
          for (int d = 0; d < d_end; ++d) {
            const uint32_t ka = kq.x | s_nib[qa & 15u], kb = kq.x | s_nib[qb & 15u];
            kq = make_uint4(kq.y, kq.z, kq.w, 0u);
            qa >>= 4;
            qb >>= 4;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
              const double2 va = s_kv[(ka >> (8 * b)) & 0xFFu], vb = s_kv[(kb >> (8 * b)) & 0xFFu];
              ac += va.x;
              am += va.y;
              bc += vb.x;
              bm += vb.y;
            }
          }
          if (has_b) {  // node k closes at the boundary, node k2 goes on to the run's end
            if (cont && !head) {
              head = true; head_k = k; head_c = ac; head_m = am;
            } else {
              ss[k] = make_double2(ac, am);
            }
            k = k2;
            bnd = nb2;
            acc_c = bc;
            acc_m = bm;
          } else {
            acc_c = ac;
            acc_m = am;
          }
        }
      }
      if (!done) {
#pragma unroll
      for (int j = 0; j < (int)kURun; ++j) {
        const uint32_t p = lf + (uint32_t)j;
        const bool in = p >= p_lo && p < p_hi;
        if (in && p >= bnd) {  // node k ends before pod p: close it, move to the node holding p
          if (cont && !head) {
            head = true; head_k = k; head_c = acc_c; head_m = acc_m;
          } else {
            ss[k] = make_double2(acc_c, acc_m);
          }
          acc_c = 0.0;
          acc_m = 0.0;
          do { ++k; } while (sp[k + 1] <= p);  // past nodes without pods
          bnd = sp[k + 1];
        }
        const bool live = in && run_alive<WB>(sv, j, abit, a.fmt.dw != 0);
        if constexpr (kCnt) {
          if (cnt_on && in) {
            const uint32_t e = s_clut[(((j >> 2) == 0 ? sv[0].x : (j >> 2) == 1 ? sv[0].y : (j >> 2) == 2 ? sv[0].z : sv[0].w) >>
                                       (8 * (j & 3))) & 0xFFu];
#pragma unroll
            for (int m = 0; m < 4; ++m) ccnt[m] += (e >> (8 * m)) & 0xFFu;
          }
        }
        double vc, vm;
        if constexpr (kKey8) {
          const uint4 kq = kv[0];
          const uint32_t d = (j >> 2) == 0 ? kq.x : (j >> 2) == 1 ? kq.y : (j >> 2) == 2 ? kq.z : kq.w;
          const double2 v = s_kv[(d >> (8 * (j & 3))) & 0xFFu];
          vc = v.x;
          vm = v.y;
        } else {
          const uint4 kq = kv[j >> 2];
          const uint32_t key = (j & 3) == 0 ? kq.x : (j & 3) == 1 ? kq.y : (j & 3) == 2 ? kq.z : kq.w;
          const uint32_t row = (key >> 28) * nv;
          vc = s_pv[row + (key & 0x3FFFu)];
          vm = s_pv[row + a.n_cpu + ((key >> 14) & 0x3FFFu)];
        }
        acc_c += live ? vc : 0.0;
        acc_m += live ? vm : 0.0;
      }
      }
      // a node ending with the lane's last pod is closed here (the next lane starts a new
      // node); so is the chunk's last node
      const bool last = has && bnd == p_hi;
      if (last) {
        if (cont && !head) {
          head = true; head_k = k; head_c = acc_c; head_m = acc_m;
        } else {
          ss[k] = make_double2(acc_c, acc_m);
        }
      }
      const uint32_t key = (has && !last) ? k : 0xFFFFFFFFu;
      // the open tail: a lane that closed nothing carries all its pods in it
      double sc = (has && !last) ? acc_c : 0.0, sm = (has && !last) ? acc_m : 0.0;
      if (lane == 0 && key == carry_k) { sc += carry_c; sm += carry_m; }
      // segmented inclusive scan by node over the lanes on DPP (VALU) instead of LDS
      // permutes: within rows of 16 (row_shr 1, 2, 4, 8), then row 0 / 2's last lane into rows
      // 1 / 3 (row_bcast15) and lane 31 into rows 2-3 (row_bcast31); a lane adds what it reads
      // only when the source is in its node (keys are monotonic over the lanes, so equal keys
      // are contiguous; a source outside the row / mask reads the no-node key)
      dpp_seg_step<0x111, 0xF>(sc, sm, key);
      dpp_seg_step<0x112, 0xF>(sc, sm, key);
      dpp_seg_step<0x114, 0xF>(sc, sm, key);
      dpp_seg_step<0x118, 0xF>(sc, sm, key);
      dpp_seg_step<0x142, 0xA>(sc, sm, key);
      dpp_seg_step<0x143, 0xC>(sc, sm, key);
      double pc = dpp_f64<0x138, 0xF>(sc), pm = dpp_f64<0x138, 0xF>(sm);  // wave_shr:1
      if (lane == 0) { pc = carry_c; pm = carry_m; }
      if (head) ss[head_k] = make_double2(head_c + pc, head_m + pm);
      carry_c = readlane_f64(sc, 63);
      carry_m = readlane_f64(sm, 63);
      carry_k = (uint32_t)__builtin_amdgcn_readlane((int)key, 63);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (uint32_t k = lane; k < nk; k += 64) {
      const double2 v = ss[k];
      const uint64_t node = na + k;
      double2 cm = k == lane ? pre_cum : reinterpret_cast<double2*>(a.cum)[node];
      const int64_t lt = k == lane ? pre_last : a.last_t[node];
      if (lt != INT64_MIN) {
        const double dt = dur_seconds(a.now - lt);
        cm.x += dt * v.x;
        cm.y += dt * v.y;
        reinterpret_cast<double2*>(a.cum)[node] = cm;
      }
      a.last_t[node] = a.now;
      reinterpret_cast<double4*>(a.node_out)[node] = make_double4(v.x, v.y, cm.x, cm.y);
      tot_c += v.x;
      tot_m += v.y;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    tot_c += __shfl_xor(tot_c, o);
    tot_m += __shfl_xor(tot_m, o);
  }
  if (lane == 0) { s_c[wave] = tot_c; s_m[wave] = tot_m; }
  if constexpr (kCnt) {
    if (cnt_on) {  // the block's partial row of mask counts (summed by agg_final_kernel)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        uint32_t c = ccnt[m];
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
        if (lane == 0 && c) atomicAdd(&s_ccnt[m], c);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double tc = 0, tm = 0;
    for (int i = 0; i < kWavesPerBlock; ++i) { tc += s_c[i]; tm += s_m[i]; }
    a.block_part[blockIdx.x * 2 + 0] = tc;
    a.block_part[blockIdx.x * 2 + 1] = tm;
  }
  if constexpr (kCnt) {
    if (cnt_on && threadIdx.x < kMaxCountMasks)
      a.cpart[(uint64_t)blockIdx.x * kMaxCountMasks + threadIdx.x] = threadIdx.x < 4u ? s_ccnt[threadIdx.x] : 0u;
  }
}

// cluster totals: the per-block partials summed in a fixed order (1024 threads); thread 0 writes
// out[0..1] and returns true
__device__ __forceinline__ bool usage_total_block(const double* __restrict__ part, uint32_t n_blocks,
                                                  double* __restrict__ out) {
  double c = 0, m = 0;
  for (uint32_t b = threadIdx.x; b < n_blocks; b += blockDim.x) { c += part[b * 2]; m += part[b * 2 + 1]; }
  for (int o = 32; o > 0; o >>= 1) { c += __shfl_xor(c, o); m += __shfl_xor(m, o); }
  __shared__ double sc[16], sm[16];
  if ((threadIdx.x & 63) == 0) { sc[threadIdx.x >> 6] = c; sm[threadIdx.x >> 6] = m; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double tc = 0, tm = 0;
    for (uint32_t i = 0; i < blockDim.x / 64; ++i) { tc += sc[i]; tm += sm[i]; }
    out[0] = tc;
    out[1] = tm;
    return true;
  }
  return false;
}
__global__ __launch_bounds__(1024) void usage_total_kernel(const double* __restrict__ part, uint32_t n_blocks,
                                                           double* __restrict__ out) {
  usage_total_block(part, n_blocks, out);
}

// ------------------------------------------------------------------ Metric CRD values
// kwok's Metric CRs (pkg/kwok/metrics/metrics.go:168-571) evaluate one CEL value per series:
// per node, per pod of the node or per container of its pods.  The host lowers each value to a
// postfix program over doubles (kwok_amd/host/cel.py lower()); one thread per series runs it
// over the quantities the engine keeps: the last kwk_usage's pod / node outputs, the
// per-container values and integrators, creation times and the scrape's clock.  Dead pods
// (not in the pod cache, so not listed by ListPods) yield NaN, which the host skips.
struct MetricArgs {
  const kwk_metric_op* __restrict__ ops;
  uint32_t n_ops;
  uint32_t dim;          // KWK_METRIC_DIM_*
  uint32_t n0, n1;       // nodes [n0, n1) of the scrape, their pods [p0, p1)
  uint32_t p0, p1, c0;   // and the containers from c0 on
  uint32_t n_series;
  const void* __restrict__ st;
  StateFmt fmt;
  const uint32_t* __restrict__ node_ptr;
  const uint32_t* __restrict__ cptr;      // per pod: first container (n_pods + 1)
  const uint32_t* __restrict__ ukey;
  const uint2* __restrict__ mixed;
  const uint32_t* __restrict__ ckeys;
  const uint32_t* __restrict__ mbase;
  const double* __restrict__ cpu_v;
  const double* __restrict__ mem_v;
  const double* __restrict__ pod_out;
  const double* __restrict__ pod_cum;
  const double* __restrict__ ccum;
  const double* __restrict__ node_out;
  const int64_t* __restrict__ pod_created;   // ns, INT64_MIN = the Go zero time
  const int64_t* __restrict__ node_created;
  const double* __restrict__ node_started;   // StartedContainersTotal per node
  int64_t now;
  double zero_time_unix_s;                   // UnixSecond of the Go zero time
  double* __restrict__ out;
};

// first index i in [lo, hi) with a[i] > x, minus one (the segment holding x)
__device__ __forceinline__ uint32_t seg_of(const uint32_t* __restrict__ a, uint32_t lo, uint32_t hi, uint32_t x) {
  while (hi - lo > 1) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (a[mid] <= x) lo = mid; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ double since_seconds(int64_t now, int64_t created) {
  if (created == INT64_MIN) return 9223372036.854775807;  // time.Since(zero time) saturates
  int64_t d;
  if (__builtin_sub_overflow(now, created, &d)) d = now > created ? INT64_MAX : INT64_MIN;
  return dur_seconds(d);
}

// the series s of a metric: its node, pod and container index (false: a dead pod, no series)
__device__ __forceinline__ bool metric_series(const MetricArgs& a, uint32_t s, uint32_t& node, uint32_t& pod,
                                              uint32_t& j) {
  node = 0; pod = 0; j = 0;
  if (a.dim == KWK_METRIC_DIM_NODE) {
    node = a.n0 + s;
    return true;
  }
  if (a.dim == KWK_METRIC_DIM_CONTAINER) {
    const uint32_t c = a.c0 + s;
    pod = seg_of(a.cptr, a.p0, a.p1, c);
    j = c - a.cptr[pod];
  } else {
    pod = a.p0 + s;
  }
  if (!(load_state(a.st, pod, a.fmt).y & KWK_F_ALIVE)) return false;
  node = seg_of(a.node_ptr, a.n0, a.n1, pod);
  return true;
}

// one lowered CEL value program for one series
__device__ double run_metric_program(const MetricArgs& a, const kwk_metric_op* __restrict__ ops, uint32_t n_ops,
                                     uint32_t node, uint32_t pod, uint32_t j) {
  double stk[8];
  int sp = 0;
  for (uint32_t i = 0; i < n_ops; ++i) {
    const kwk_metric_op op = ops[i];
    switch (op.op) {
      case KWK_MOP_CONST: stk[sp++] = op.value; break;
      case KWK_MOP_LOAD: {
        double v = 0.0;
        const uint32_t in = op.arg;
        if (in == KWK_MIN_NOW_S) {
          v = (double)a.now / 1e9;
        } else if (in >= KWK_MIN_CONTAINER_CPU && in <= KWK_MIN_CONTAINER_CUM_MEM) {
          const uint32_t k = a.ukey[pod];
          const bool cum = in >= KWK_MIN_CONTAINER_CUM_CPU;
          const uint32_t r = (in - KWK_MIN_CONTAINER_CPU) & 1u;
          if (k >> 28) {
            v = cum ? a.pod_cum[2 * (uint64_t)pod + r] : (r ? a.mem_v[(k >> 14) & 0x3FFFu] : a.cpu_v[k & 0x3FFFu]);
          } else {
            const uint2 fc = a.mixed[k & kUKeyMixedIndex];
            const uint32_t ck = a.ckeys[fc.x + j];
            v = cum ? a.ccum[2 * (uint64_t)(a.mbase[pod] + j) + r] : (r ? a.mem_v[(ck >> 14) & 0x3FFFu] : a.cpu_v[ck & 0x3FFFu]);
          }
        } else if (in >= KWK_MIN_POD_CPU && in <= KWK_MIN_POD_CUM_MEM) {
          v = a.pod_out[4 * (uint64_t)pod + (in - KWK_MIN_POD_CPU)];
        } else if (in >= KWK_MIN_NODE_CPU && in <= KWK_MIN_NODE_CUM_MEM) {
          v = a.node_out[4 * (uint64_t)node + (in - KWK_MIN_NODE_CPU)];
        } else if (in == KWK_MIN_POD_SINCE) {
          v = since_seconds(a.now, a.pod_created[pod]);
        } else if (in == KWK_MIN_NODE_SINCE) {
          v = since_seconds(a.now, a.node_created[node]);
        } else if (in == KWK_MIN_POD_CREATED || in == KWK_MIN_NODE_CREATED) {
          const int64_t c = in == KWK_MIN_POD_CREATED ? a.pod_created[pod] : a.node_created[node];
          v = c == INT64_MIN ? a.zero_time_unix_s : (double)c / 1e9;
        } else if (in == KWK_MIN_STARTED_CONTAINERS) {
          v = a.node_started[node];
        }
        stk[sp++] = v;
        break;
      }
      case KWK_MOP_ADD: --sp; stk[sp - 1] = stk[sp - 1] + stk[sp]; break;
      case KWK_MOP_SUB: --sp; stk[sp - 1] = stk[sp - 1] - stk[sp]; break;
      case KWK_MOP_MUL: --sp; stk[sp - 1] = stk[sp - 1] * stk[sp]; break;
      case KWK_MOP_DIV: --sp; stk[sp - 1] = stk[sp - 1] / stk[sp]; break;
      case KWK_MOP_NEG: stk[sp - 1] = -stk[sp - 1]; break;
      default: break;
    }
  }
  return sp > 0 ? stk[sp - 1] : 0.0;
}

__global__ __launch_bounds__(kBlock) void metrics_kernel(MetricArgs a) {
  const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
  if (s >= a.n_series) return;
  uint32_t node, pod, j;
  if (!metric_series(a, s, node, pod, j)) {
    a.out[s] = __builtin_nan("");
    return;
  }
  a.out[s] = run_metric_program(a, a.ops, a.n_ops, node, pod, j);
}

// Pod-major evaluation of every pod / container metric of a scrape in one launch: one thread per
// pod of [p0, p1) finds its node once (a guess from the pods' mean per node, then a local walk:
// no binary search over 100M entries per series), reads its state once and writes its series of
// each metric at the metric's offset (metric-major output, as metrics_kernel: pod series at
// pod - p0, container series at cptr[pod] - c0 + j; NaN for a dead pod).  Adjacent lanes write
// adjacent pods' / containers' values, so the stores coalesce.  The node metrics keep
// metrics_kernel (one thread per node).
constexpr uint32_t kMaxPodMetrics = 16;
struct PodMetric {
  uint32_t dim, first_op, n_ops, pad;
  uint64_t off;  // the metric's first value in the scrape's output
};
struct PodMetricList {
  uint32_t n;
  PodMetric m[kMaxPodMetrics];
};
__global__ __launch_bounds__(kBlock) void metrics_pod_kernel(MetricArgs a, PodMetricList L, double* __restrict__ out) {
  const uint32_t pod = a.p0 + blockIdx.x * kBlock + threadIdx.x;
  if (pod >= a.p1) return;
  // node: the guess node_ptr would give for equal-sized nodes, corrected by walking (nodes of the
  // scrape are consecutive; equal-sized nodes need no step)
  uint32_t node = a.n0 + (uint32_t)((uint64_t)(pod - a.p0) * (a.n1 - a.n0) / (uint64_t)(a.p1 - a.p0));
  if (node >= a.n1) node = a.n1 - 1;
  while (node > a.n0 && a.node_ptr[node] > pod) --node;
  while (node + 1 < a.n1 && a.node_ptr[node + 1] <= pod) ++node;
  const bool alive = (load_state(a.st, pod, a.fmt).y & KWK_F_ALIVE) != 0;
  const uint32_t cl = a.cptr[pod], ch = a.cptr[pod + 1];
  for (uint32_t k = 0; k < L.n; ++k) {
    const PodMetric m = L.m[k];
    const kwk_metric_op* ops = a.ops + m.first_op;
    if (m.dim == KWK_METRIC_DIM_POD) {
      out[m.off + (pod - a.p0)] = alive ? run_metric_program(a, ops, m.n_ops, node, pod, 0) : __builtin_nan("");
    } else {
      double* o = out + m.off + (cl - a.c0);
      for (uint32_t j = 0; j < ch - cl; ++j)
        o[j] = alive ? run_metric_program(a, ops, m.n_ops, node, pod, j) : __builtin_nan("");
    }
  }
}

// Go's uint64(float64) on amd64 (the compiler's float64ToUint64 lowering): x < 2^63 ->
// CVTTSD2SQ (truncation; -Inf, NaN-free values <= -2^63 give the "integer indefinite"
// 0x8000000000000000), else CVTTSD2SQ(x - 2^63) | 1 << 63 (NaN and x >= 2^64: 1 << 63)
__device__ __forceinline__ uint64_t go_f64_to_u64(double x) {
  constexpr uint64_t kInd = 0x8000000000000000ull;
  auto cvtt = [](double v) -> uint64_t {
    if (!(v > -9223372036854775808.0 && v < 9223372036854775808.0)) return kInd;
    return (uint64_t)(int64_t)v;
  };
  if (x < 9223372036854775808.0) return cvtt(x);
  return cvtt(x - 9223372036854775808.0) | kInd;
}

// Histogram metrics (metrics.go:356-462 updateHistogram; histogram.go:81-164 Set / Write): per
// series every bucket's value program runs, uint64(value) is Set at the bucket's le (a later
// bucket with the same le overwrites), and Write turns the stored (le, count) pairs — ascending
// le — into the cumulative counts of the visible upper bounds (ascending) plus +Inf, the sample
// count and the sample sum (sum += le * count in key order), exactly as histogram.Write does
// (note: +Inf only collects keys above the last visible bound).  The host orders the keys and
// bounds (Go's sort.Float64s order) per histogram.
struct HistDesc {
  uint32_t first_bucket, n_buckets;  // buckets [first, first + n) of the bucket table
  uint32_t first_key, n_keys;        // bucket indices (relative) of the distinct le, ascending
  uint32_t first_bound, n_bounds;    // visible upper bounds, ascending
  uint32_t out_words;                // n_bounds + 3
  uint32_t dim;
};
constexpr uint32_t kMaxHistBuckets = 64;
__global__ __launch_bounds__(kBlock) void histogram_kernel(MetricArgs a, HistDesc h,
                                                           const kwk_metric_bucket* __restrict__ buckets,
                                                           const uint32_t* __restrict__ keys,
                                                           const double* __restrict__ bounds,
                                                           uint64_t* __restrict__ out) {
  const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
  if (s >= a.n_series) return;
  uint64_t* o = out + (uint64_t)s * h.out_words;
  uint32_t node, pod, j;
  if (!metric_series(a, s, node, pod, j)) {  // a dead pod: no series (count slot = all ones)
    for (uint32_t w = 0; w < h.out_words; ++w) o[w] = ~0ull;
    return;
  }
  uint64_t val[kMaxHistBuckets];
  for (uint32_t b = 0; b < h.n_buckets; ++b) {
    const kwk_metric_bucket B = buckets[h.first_bucket + b];
    val[b] = go_f64_to_u64(run_metric_program(a, a.ops + B.first_op, B.n_ops, node, pod, j));
  }
  const uint32_t nb = h.n_bounds + 1;  // + the +Inf bucket
  for (uint32_t w = 0; w < nb; ++w) o[w] = 0;
  uint32_t bi = 0;
  uint64_t count = 0;
  double sum = 0.0;
  for (uint32_t k = 0; k < h.n_keys; ++k) {
    const uint32_t b = keys[h.first_key + k];
    const double le = buckets[h.first_bucket + b].le;
    // cumulative count of previous buckets (histogram.go:128-133): the bound past the last
    // visible one is +Inf, which no le exceeds
    while (bi < nb && bi < h.n_bounds && le > bounds[h.first_bound + bi]) {
      ++bi;
      o[bi] += count;
    }
    o[bi] += val[b];
    count += val[b];
    sum += le * (double)val[b];
  }
  o[nb] = count;
  o[nb + 1] = (uint64_t)__double_as_longlong(sum);
}

// count alive objects with (pred & mask[k]) != 0 for each k (mask 0: every alive object):
// phase histograms and other cluster aggregates.  Each lane streams 16-byte chunks of the
// state column (8, 4 or 2 words) and tests the raw words (pred bits, alive flag) against the
// masks — only the n_masks masks asked for (a wave-uniform loop bound) — with per-lane
// counters in registers, one 64-bit atomic per block and mask.
template <uint32_t WB, int NM>  // NM >= n_masks masks tested (compile time); the rest count nothing used
__global__ __launch_bounds__(kBlock) void count_kernel(const void* __restrict__ st, uint32_t n, uint32_t abit,
                                                       uint32_t pmask, const uint32_t* __restrict__ masks,
                                                       uint32_t n_masks, uint32_t* __restrict__ part, uint32_t px) {
  __shared__ unsigned int s_cnt[NM];
  if (threadIdx.x < NM) s_cnt[threadIdx.x] = 0;
  uint32_t cnt[NM];
  uint32_t mk[NM];     // wave-uniform: the mask's pred bits
  uint32_t every[NM];  // 1: mask 0 = every alive object
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    cnt[m] = 0;
    const uint32_t x = (uint32_t)m < n_masks ? masks[m] : 0u;
    mk[m] = x & pmask;
    every[m] = x == 0u ? 1u : 0u;
  }
  __syncthreads();
  constexpr uint32_t kWpc = 16u / WB;  // words per chunk
  // the 2-byte format's masks for both halves of a dword
  const uint32_t a2 = (abit & 0xFFFFu) * 0x10001u;
  uint32_t m2[NM], every2[NM];
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    m2[m] = (mk[m] & 0xFFFFu) * 0x10001u;
    every2[m] = every[m] ? 0x80008000u : 0u;
  }
  const uint64_t n_chunks = ((uint64_t)n * WB + 15u) / 16u;
  const uint4* __restrict__ q = reinterpret_cast<const uint4*>(st);
  auto tally = [&](uint32_t pred, uint32_t flags, bool in) {
    const uint32_t al = (in && (flags & abit)) ? 1u : 0u;
#pragma unroll
    for (int m = 0; m < NM; ++m) cnt[m] += (((pred & mk[m]) != 0u ? 1u : 0u) | every[m]) & al;
  };
  auto tally_chunk = [&](const uint4 v, uint64_t c) {
    const uint32_t dw[4] = {v.x, v.y, v.z, v.w};
    const uint64_t i0 = c * kWpc;
    const uint32_t lim = i0 + kWpc <= n ? kWpc : (uint32_t)(n - i0);  // words of the chunk below n
    if constexpr (WB == 2) {
      // two words per dword (SWAR): a half is nonzero iff bit 15 of
      // ((h & 0x7FFF) + 0x7FFF) | h is set; hits = alive & (every | pred & mask), popcounted
      const uint32_t lim_m = lim >= 8u ? 0xFFFFFFFFu : 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t d = dw[q];
        const uint32_t in = lim_m | ((2u * q < lim ? 0x8000u : 0u) | (2u * q + 1u < lim ? 0x80000000u : 0u));
        const uint32_t al = ((((d & a2) & 0x7FFF7FFFu) + 0x7FFF7FFFu) | (d & a2)) & 0x80008000u & in;
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          const uint32_t x = d & m2[m];
          const uint32_t hit = ((((x & 0x7FFF7FFFu) + 0x7FFF7FFFu) | x) & 0x80008000u) | every2[m];
          cnt[m] += (uint32_t)__popc(hit & al);
        }
      }
    } else if constexpr (WB == 4) {
#pragma unroll
      for (int j = 0; j < 4; ++j) tally(dw[j], dw[j], (uint32_t)j < lim);
    } else {
      tally(v.x, px ? v.x : v.y, true);  // px: flags in the packed word of a fused record
      tally(v.z, px ? v.z : v.w, lim > 1);
    }
  };
  // kCountU chunks per lane in flight together, kBlock chunks apart (coalesced)
  constexpr uint32_t kCountU = 4;
  for (uint64_t c0 = (uint64_t)blockIdx.x * kBlock * kCountU + threadIdx.x; c0 < n_chunks;
       c0 += (uint64_t)gridDim.x * kBlock * kCountU) {
    uint4 vs[kCountU];
#pragma unroll
    for (uint32_t u = 0; u < kCountU; ++u) {
      const uint64_t c = c0 + u * kBlock;
      vs[u] = c < n_chunks ? q[c] : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (uint32_t u = 0; u < kCountU; ++u)
      if (c0 + u * kBlock < n_chunks) tally_chunk(vs[u], c0 + u * kBlock);
  }
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    uint32_t c = cnt[m];
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(&s_cnt[m], c);
  }
  __syncthreads();
  // one row of partial counts per block (same-address atomics from thousands of blocks
  // serialise at the L2: 111 us for a 100M-object count, r2d); count_total_kernel sums them
  if (threadIdx.x < kMaxCountMasks)
    part[(uint64_t)blockIdx.x * kMaxCountMasks + threadIdx.x] = threadIdx.x < (uint32_t)NM ? s_cnt[threadIdx.x] : 0u;
}

// 2-byte words, at most 4 masks and 11 pred bits (pod-fast, node kinds): one LDS lookup per word
// instead of the SWAR mask tests (~36 VALU per dword at 4 masks, r2zd).  Entry (pred bits |
// alive << pred_bits) holds, in byte m, 1 if the word counts for mask m; the lane adds entries into
// one packed counter and unpacks it every 32 words.  Same partial rows as count_kernel.
constexpr uint32_t kCountLutBits = 12;
__global__ __launch_bounds__(kBlock) void count16_lut_kernel(const void* __restrict__ st, uint32_t n, uint32_t abit,
                                                             uint32_t pmask, const uint32_t* __restrict__ masks,
                                                             uint32_t n_masks, uint32_t* __restrict__ part) {
  __shared__ uint32_t s_lut[1u << kCountLutBits];
  __shared__ unsigned int s_cnt[4];
  const uint32_t pb = 32u - (uint32_t)__clz(pmask);  // pmask = 2^pb - 1
  const uint32_t apos = (uint32_t)__ffs(abit) - 1u;
  uint32_t mk[4], every[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const uint32_t x = (uint32_t)m < n_masks ? masks[m] : 0u;
    mk[m] = (uint32_t)m < n_masks ? x & pmask : 0u;
    every[m] = ((uint32_t)m < n_masks && x == 0u) ? 1u : 0u;
  }
  for (uint32_t e = threadIdx.x; e < (2u << pb); e += kBlock) {
    const uint32_t pred = e & pmask, al = e >> pb;
    uint32_t v = 0;
#pragma unroll
    for (int m = 0; m < 4; ++m) v |= (al & ((every[m] | ((pred & mk[m]) != 0u ? 1u : 0u)))) << (8 * m);
    s_lut[e] = v;
  }
  if (threadIdx.x < 4) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  uint32_t cnt[4] = {0u, 0u, 0u, 0u};
  const uint64_t n_chunks = ((uint64_t)n * 2u + 15u) / 16u;
  const uint4* __restrict__ q = reinterpret_cast<const uint4*>(st);
  constexpr uint32_t kCountU = 4;
  for (uint64_t c0 = (uint64_t)blockIdx.x * kBlock * kCountU + threadIdx.x; c0 < n_chunks;
       c0 += (uint64_t)gridDim.x * kBlock * kCountU) {
    uint4 vs[kCountU];
#pragma unroll
    for (uint32_t u = 0; u < kCountU; ++u) {
      const uint64_t c = c0 + u * kBlock;
      vs[u] = c < n_chunks ? q[c] : make_uint4(0u, 0u, 0u, 0u);
    }
    uint32_t acc = 0;  // byte m: words counted for mask m (at most 32 per group)
#pragma unroll
    for (uint32_t u = 0; u < kCountU; ++u) {
      const uint64_t i0 = (c0 + u * kBlock) * 8u;
      const bool whole = i0 + 8u <= n;
      const uint32_t dw[4] = {vs[u].x, vs[u].y, vs[u].z, vs[u].w};
#pragma unroll
      for (int h = 0; h < 8; ++h) {
        const uint32_t w = (h & 1) ? dw[h >> 1] >> 16 : dw[h >> 1] & 0xFFFFu;
        uint32_t idx = (w & pmask) | (((w >> apos) & 1u) << pb);
        if (!whole && i0 + (uint64_t)h >= n) idx = 0u;  // entry 0: not alive, counts nothing
        acc += s_lut[idx];
      }
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) cnt[m] += (acc >> (8 * m)) & 0xFFu;
  }
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    uint32_t c = cnt[m];
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(&s_cnt[m], c);
  }
  __syncthreads();
  if (threadIdx.x < kMaxCountMasks)
    part[(uint64_t)blockIdx.x * kMaxCountMasks + threadIdx.x] = threadIdx.x < 4u ? s_cnt[threadIdx.x] : 0u;
}

// 1-byte ids: one LDS lookup per id and group of four masks — entry [g][id] holds, in byte m, 1 if
// the id's word counts for mask 4g + m (alive and, unless the mask is 0, (pred & mask) != 0); each
// block builds its table from the dictionary.  Same partial rows as count_kernel.
template <int NG>  // mask groups of four (n_masks <= 4 * NG)
__global__ __launch_bounds__(kBlock) void count8_kernel(const void* __restrict__ st, uint32_t n, StateFmt fmt,
                                                        const uint32_t* __restrict__ masks, uint32_t n_masks,
                                                        uint32_t* __restrict__ part) {
  __shared__ uint32_t s_lut[NG][256];
  __shared__ unsigned int s_cnt[4 * NG];
  for (uint32_t e = threadIdx.x; e < 256u * NG; e += kBlock) {
    const uint32_t g = e >> 8, id = e & 255u;
    const uint2 v = fmt_unpack(fmt.id2w[id], fmt);
    const uint32_t al = (v.y & KWK_F_ALIVE) ? 1u : 0u;
    uint32_t x = 0;
#pragma unroll
    for (uint32_t m = 0; m < 4; ++m) {
      const uint32_t k = 4u * g + m;
      if (k < n_masks) {
        const uint32_t mk = masks[k];
        x |= (al & ((mk == 0u || (v.x & mk) != 0u) ? 1u : 0u)) << (8 * m);
      }
    }
    s_lut[g][id] = x;
  }
  if (threadIdx.x < 4 * NG) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  uint32_t cnt[4 * NG];
#pragma unroll
  for (int m = 0; m < 4 * NG; ++m) cnt[m] = 0;
  const uint64_t n_chunks = ((uint64_t)n + 15u) / 16u;
  const uint4* __restrict__ q = reinterpret_cast<const uint4*>(st);
  constexpr uint32_t kCountU = 4;  // 64 ids per lane and round: byte counters stay below 256
  for (uint64_t c0 = (uint64_t)blockIdx.x * kBlock * kCountU + threadIdx.x; c0 < n_chunks;
       c0 += (uint64_t)gridDim.x * kBlock * kCountU) {
    uint4 vs[kCountU];
#pragma unroll
    for (uint32_t u = 0; u < kCountU; ++u) {
      const uint64_t c = c0 + u * kBlock;
      vs[u] = c < n_chunks ? q[c] : make_uint4(0u, 0u, 0u, 0u);  // id 0: not alive
    }
    uint32_t acc[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) acc[g] = 0;
#pragma unroll
    for (uint32_t u = 0; u < kCountU; ++u) {
      const uint64_t i0 = (c0 + u * kBlock) * 16u;
      const bool whole = i0 + 16u <= n;
      const uint32_t dw[4] = {vs[u].x, vs[u].y, vs[u].z, vs[u].w};
#pragma unroll
      for (int h = 0; h < 16; ++h) {
        uint32_t id = (dw[h >> 2] >> (8 * (h & 3))) & 0xFFu;
        if (!whole && i0 + (uint64_t)h >= n) id = 0u;
#pragma unroll
        for (int g = 0; g < NG; ++g) acc[g] += s_lut[g][id];
      }
    }
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int m = 0; m < 4; ++m) cnt[4 * g + m] += (acc[g] >> (8 * m)) & 0xFFu;
  }
#pragma unroll
  for (int m = 0; m < 4 * NG; ++m) {
    uint32_t c = cnt[m];
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(&s_cnt[m], c);
  }
  __syncthreads();
  if (threadIdx.x < kMaxCountMasks)
    part[(uint64_t)blockIdx.x * kMaxCountMasks + threadIdx.x] = threadIdx.x < 4u * NG ? s_cnt[threadIdx.x] : 0u;
}

// out[m] = sum over the blocks' partial rows (1024 threads: 16 masks x 64 block strides); s[m]
// holds the sum afterwards
__device__ __forceinline__ void count_total_block(const uint32_t* __restrict__ part, uint32_t n_blocks,
                                                  uint32_t n_masks, unsigned long long* __restrict__ out,
                                                  unsigned long long* s) {
  const uint32_t m = threadIdx.x & (kMaxCountMasks - 1), r = threadIdx.x / kMaxCountMasks;
  unsigned long long c = 0;
  constexpr uint32_t kRows = 1024 / kMaxCountMasks;  // rows summed in parallel
  for (uint32_t b = r; b < n_blocks; b += 8 * kRows) {  // 8 loads in flight per thread (was one at a time: 9.6 us)
    uint32_t v[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
      const uint32_t bb = b + j * kRows;
      v[j] = bb < n_blocks ? part[(uint64_t)bb * kMaxCountMasks + m] : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) c += v[j];
  }
  s[threadIdx.x] = c;
  __syncthreads();
  for (uint32_t h = 512; h >= kMaxCountMasks; h >>= 1) {
    if (threadIdx.x < h) s[threadIdx.x] += s[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x < n_masks) out[threadIdx.x] = s[threadIdx.x];
}
__global__ __launch_bounds__(1024) void count_total_kernel(const uint32_t* __restrict__ part, uint32_t n_blocks,
                                                           uint32_t n_masks, unsigned long long* __restrict__ out) {
  __shared__ unsigned long long s[1024];
  count_total_block(part, n_blocks, n_masks, out, s);
}

// out = nullptr: the partial rows only (kwk_aggregate sums them in agg_final_kernel)
static void launch_count8(uint32_t n_masks, dim3 g, hipStream_t s, const void* st, uint32_t n, const StateFmt& fmt,
                          const uint32_t* masks, uint32_t* part, unsigned long long* out) {
  if (n_masks <= 4) hipLaunchKernelGGL((count8_kernel<1>), g, dim3(kBlock), 0, s, st, n, fmt, masks, n_masks, part);
  else if (n_masks <= 8) hipLaunchKernelGGL((count8_kernel<2>), g, dim3(kBlock), 0, s, st, n, fmt, masks, n_masks, part);
  else hipLaunchKernelGGL((count8_kernel<4>), g, dim3(kBlock), 0, s, st, n, fmt, masks, n_masks, part);
  if (out) hipLaunchKernelGGL(count_total_kernel, dim3(1), dim3(1024), 0, s, part, g.x, n_masks, out);
}

template <uint32_t WB>
static void launch_count(uint32_t n_masks, dim3 g, hipStream_t s, const void* st, uint32_t n, uint32_t abit,
                         uint32_t pmask, const uint32_t* masks, uint32_t* part, unsigned long long* out,
                         uint32_t px = 0) {
  if (WB == 2 && n_masks <= 4 && pmask < (1u << (kCountLutBits - 1)) && abit > pmask)
    hipLaunchKernelGGL(count16_lut_kernel, g, dim3(kBlock), 0, s, st, n, abit, pmask, masks, n_masks, part);
  else if (n_masks <= 2) hipLaunchKernelGGL((count_kernel<WB, 2>), g, dim3(kBlock), 0, s, st, n, abit, pmask, masks, n_masks, part, px);
  else if (n_masks <= 4) hipLaunchKernelGGL((count_kernel<WB, 4>), g, dim3(kBlock), 0, s, st, n, abit, pmask, masks, n_masks, part, px);
  else if (n_masks <= 8) hipLaunchKernelGGL((count_kernel<WB, 8>), g, dim3(kBlock), 0, s, st, n, abit, pmask, masks, n_masks, part, px);
  else hipLaunchKernelGGL((count_kernel<WB, 16>), g, dim3(kBlock), 0, s, st, n, abit, pmask, masks, n_masks, part, px);
  if (out) hipLaunchKernelGGL(count_total_kernel, dim3(1), dim3(1024), 0, s, part, g.x, n_masks, out);
}

// kwk_aggregate's tail in one launch (was count_total + usage_total + agg_pack: two launch gaps
// fewer per report): the sweeps' per-stage statistics rows, the mask counts' partial rows
// (n_cblocks = 0: counts already final) and the usage kernel's block partials (usage 1; 2: no usage
// kernel ran, the cluster sums are packed as they stand), then the packed output.  The three sums
// run side by side on their own waves (0-3 statistics, 4-11 counts, 12-15 usage), each with its
// loads in flight together, then one barrier (round 6: the three one after the other, each a load
// round trip and a barrier tree, took 10.1 us per launch at the 125k-node shard, r6ab — on the
// pod chain once per report)
__global__ __launch_bounds__(1024) void agg_final_kernel(const uint32_t* __restrict__ cpart, uint32_t n_cblocks,
                                                         uint32_t n_masks, unsigned long long* __restrict__ counts,
                                                         const double* __restrict__ upart, uint32_t n_ublocks,
                                                         double* __restrict__ cluster, uint32_t usage,
                                                         const unsigned long long* __restrict__ cum, uint32_t cum_rows,
                                                         uint32_t n_stages, double* __restrict__ out) {
  constexpr uint32_t kCW = 8, kUW = 4;   // count / usage waves
  constexpr uint32_t kRows = kCW * 64 / kMaxCountMasks;  // count rows summed in parallel
  __shared__ unsigned long long s_st[KWK_MAX_STAGES];
  __shared__ unsigned long long s_cnt[kCW][kMaxCountMasks];
  __shared__ double s_u[kUW][2];
  const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
  if (t < KWK_MAX_STAGES) s_st[t] = 0;
  __syncthreads();
  if (wave < 4) {
    // per-stage transitions: rows u, u + 256, ... of 8 stage words at a time, 4 rows in flight
    const uint32_t u = t;
    for (uint32_t s0 = 0; s0 < n_stages; s0 += 8) {  // uniform
      unsigned long long v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (uint32_t r0 = u; r0 < cum_rows; r0 += 4 * 256u) {
        unsigned long long x[4][8];
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
          const uint32_t r = r0 + q * 256u;
          const unsigned long long* __restrict__ row = cum + (uint64_t)r * kStatWords + 3 + s0;
#pragma unroll
          for (uint32_t j = 0; j < 8; ++j) x[q][j] = (r < cum_rows && s0 + j < n_stages) ? row[j] : 0ull;
        }
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q)
#pragma unroll
          for (uint32_t j = 0; j < 8; ++j) v[j] += x[q][j];
      }
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) {
        if (s0 + j >= n_stages) break;
        for (int o = 32; o > 0; o >>= 1) v[j] += __shfl_xor(v[j], o);
        if (lane == 0 && v[j]) atomicAdd(&s_st[s0 + j], v[j]);
      }
    }
  } else if (wave < 4 + kCW) {
    // the mask counts' partial rows: lane m = mask, 16 rows in flight per thread
    const uint32_t u = t - 256u, m = u & (kMaxCountMasks - 1u), cr = u / kMaxCountMasks;
    unsigned long long c = 0;
    for (uint32_t b = cr; b < n_cblocks; b += 16 * kRows) {
      uint32_t cv[16];
#pragma unroll
      for (uint32_t q = 0; q < 16; ++q) {
        const uint32_t bb = b + q * kRows;
        cv[q] = bb < n_cblocks ? cpart[(uint64_t)bb * kMaxCountMasks + m] : 0u;
      }
#pragma unroll
      for (uint32_t q = 0; q < 16; ++q) c += cv[q];
    }
    c += __shfl_xor(c, 16);  // lanes 16 apart hold the same mask
    c += __shfl_xor(c, 32);
    if (lane < kMaxCountMasks) s_cnt[wave - 4][lane] = c;
  } else if (usage == 1) {
    // the usage kernel's block partials, 8 in flight per thread
    const uint32_t u = t - 768u;
    double uc = 0, um = 0;
    for (uint32_t b0 = u; b0 < n_ublocks; b0 += 8 * 256u) {
      double2 x[8];
#pragma unroll
      for (uint32_t q = 0; q < 8; ++q) {
        const uint32_t b = b0 + q * 256u;
        x[q] = b < n_ublocks ? make_double2(upart[b * 2], upart[b * 2 + 1]) : make_double2(0.0, 0.0);
      }
#pragma unroll
      for (uint32_t q = 0; q < 8; ++q) {
        uc += x[q].x;
        um += x[q].y;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      uc += __shfl_xor(uc, o);
      um += __shfl_xor(um, o);
    }
    if (lane == 0) {
      s_u[wave - 12][0] = uc;
      s_u[wave - 12][1] = um;
    }
  }
  __syncthreads();
  if (t < n_stages) {
    out[t] = (double)s_st[t];
  } else if (t < n_stages + n_masks) {
    const uint32_t k = t - n_stages;
    if (n_cblocks) {
      unsigned long long sum = 0;
      for (uint32_t w = 0; w < kCW; ++w) sum += s_cnt[w][k];
      counts[k] = sum;
      out[t] = (double)sum;
    } else {
      out[t] = (double)counts[k];
    }
  } else if (usage && t < n_stages + n_masks + 2) {
    const uint32_t k = t - n_stages - n_masks;
    double x;
    if (usage == 1) {
      x = 0;
      for (uint32_t w = 0; w < kUW; ++w) x += s_u[w][k];
      cluster[k] = x;
    } else {
      x = cluster[k];
    }
    out[t] = x;
  }
}

// ------------------------------------------------------------------ node leases
// NodeLeaseController.syncWorker (pkg/kwok/controllers/node_lease_controller.go:108-143) for
// every held node whose queued sync is due, one lane per lease:
//   dur  = interval() = wait.Jitter(renewInterval, jitter)          :145-147 (Philox site 3)
//   sync: lease exists ? (tryAcquireOrRenew ? renewLease : "held by another")
//                      : ensureLease                                :174-275
//   next = lease ok ? nextTryDuration(dur, expireTime - now, hold) : dur   :131-141, 309-338
//   AddWeightAfter(node, next)                                       (<= 0: runnable now)
// The API writes are applied to the device copy of the lease (what the informer cache shows
// the next Held()); renewTime is a MicroTime, so it keeps microseconds.  With manage_nodes,
// the node's MANAGED bit follows Held() (readOnlyFunc, controller.go:285-288) and a
// successful sync re-matches a node with no queued stage (onNodeManaged -> ManageNode,
// controller.go:276-279, 307-329; preprocess skips nodes whose queued job is current).
constexpr uint32_t kLeaseOpSetDirty = 0x80u;  // per-node op byte: this sync set the node's DIRTY bit

struct LeaseArgs {
  kwk_lease* __restrict__ lease;
  uint8_t* __restrict__ op;          // per node: KWK_LEASE_OP_* of this step (0 = no sync)
  void* __restrict__ st;             // node engine state words
  kwk_fired_rec* __restrict__ ops;   // API writes (slot, op) of this step
  uint32_t* __restrict__ n_ops;
  unsigned long long* __restrict__ stats;  // [5]: steps, creates, renews, acquires, busy
  StateFmt fmt;
  uint32_t n;
  uint64_t slot_base;
  uint64_t key;
  uint64_t step;
  int64_t now;
  kwk_lease_params cfg;
};

__device__ __forceinline__ bool lease_try_acquire_or_renew(const kwk_lease& L, uint32_t me, int64_t now) {
  if (!(L.flags & KWK_LEASE_HOLDER) || L.holder == me) return true;
  if (!(L.flags & KWK_LEASE_RENEW) || !(L.flags & KWK_LEASE_DURATION)) return true;
  return sat_add(L.renew_ns, (int64_t)L.duration_s * 1000000000) < now;  // expireTime.Before(now)
}

__device__ __forceinline__ int64_t lease_next_try(int64_t renew_interval, int64_t expire, bool hold) {
  if (!hold) return renew_interval;
  if (renew_interval < expire) return renew_interval;
  if (expire < 1000000000) return 1000000000;
  return expire;
}

__global__ __launch_bounds__(kBlock) void lease_kernel(LeaseArgs a, uint32_t* __restrict__ next_n_ops) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63;
  // the API-write count of the NEXT lease step starts at 0 (no memset launch per tick)
  if (i == 0) *next_n_ops = 0u;
  uint32_t op = 0;
  if (i < a.n) {
    kwk_lease L = a.lease[i];
    if ((L.flags & (KWK_LEASE_HOLD | KWK_LEASE_QUEUED)) == (KWK_LEASE_HOLD | KWK_LEASE_QUEUED) &&
        L.next_try_ns <= a.now) {
      const uint32_t me = a.cfg.holder_id;
      const double factor = a.cfg.renew_jitter <= 0.0 ? 1.0 : a.cfg.renew_jitter;
      const double u = rng_float64(a.slot_base + i, a.step, kSiteLeaseJitter, a.key);
      const int64_t dur = a.cfg.renew_interval_ns + (int64_t)(u * factor * (double)a.cfg.renew_interval_ns);
      const int64_t now_us = a.now - a.now % 1000;  // metav1.MicroTime
      bool ok = false;
      if (L.flags & KWK_LEASE_EXISTS) {
        if (lease_try_acquire_or_renew(L, me, a.now)) {
          op = KWK_LEASE_OP_RENEW;
          if (!(L.flags & KWK_LEASE_HOLDER) || L.holder != me) {  // renewLease transitions (:255-260)
            L.holder = me;
            L.duration_s = a.cfg.lease_duration_s;
            L.transitions += 1;
            L.flags |= KWK_LEASE_HOLDER | KWK_LEASE_DURATION;
            op = KWK_LEASE_OP_ACQUIRE;
          }
          L.renew_ns = now_us;
          L.flags |= KWK_LEASE_RENEW;
          ok = true;
        } else {
          op = KWK_LEASE_OP_BUSY;  // sync returns (nil, nil): expireTime not ok
        }
      } else {  // ensureLease
        L.flags |= KWK_LEASE_EXISTS | KWK_LEASE_HOLDER | KWK_LEASE_DURATION | KWK_LEASE_RENEW;
        L.holder = me;
        L.duration_s = a.cfg.lease_duration_s;
        L.renew_ns = now_us;
        L.transitions = 0;
        op = KWK_LEASE_OP_CREATE;
        ok = true;
      }
      int64_t next = dur;
      if (ok) {
        const int64_t expire = sat_add(L.renew_ns, (int64_t)L.duration_s * 1000000000);
        next = lease_next_try(dur, expire - a.now, lease_try_acquire_or_renew(L, me, a.now));
      }
      L.next_try_ns = next <= 0 ? a.now : sat_add(a.now, next);
      a.lease[i] = L;
      uint32_t set_dirty = 0;  // kwk_lease_fail undoes exactly this re-match
      if (a.cfg.manage_nodes) {
        uint2 s = load_state(a.st, i, a.fmt);
        const bool held = (L.flags & KWK_LEASE_EXISTS) && (L.flags & KWK_LEASE_HOLDER) && L.holder == me;
        if (held) {
          s.y |= KWK_F_MANAGED;
          if (ok && (s.y & KWK_F_ALIVE) && (s.y & 0xFFu) == KWK_STAGE_NONE && !(s.y & KWK_F_DIRTY)) {
            s.y |= KWK_F_DIRTY;
            set_dirty = kLeaseOpSetDirty;
          }
        } else {
          s.y &= ~KWK_F_MANAGED;
        }
        store_state(a.st, i, s, a.fmt);
      }
      a.op[i] = (uint8_t)(op | set_dirty);
    } else {
      a.op[i] = 0;
    }
  }
  // API writes of this step, compacted per wave (one atomic per wave), and counters
  const unsigned long long bal = __ballot(op != 0);
  if (bal) {
    uint32_t base = 0;
    if (lane == __ffsll((long long)bal) - 1) base = atomicAdd(a.n_ops, (uint32_t)__popcll(bal));
    base = __shfl(base, __ffsll((long long)bal) - 1);
    if (op) a.ops[base + __popcll(bal & ((1ull << lane) - 1ull))] = kwk_fired_rec{i, (uint16_t)op, 0};
    for (uint32_t k = 1; k <= 4; ++k) {
      const unsigned long long m = __ballot(op == k);
      if (m && lane == 0) atomicAdd(&a.stats[k], (unsigned long long)__popcll(m));
    }
  }
}

// pods on nodes whose lease sync ran this step: MANAGED follows Held(); a successful sync
// re-matches the pods with no queued stage (podsOnNodeSyncWorker, controller.go:559-573).
// One wave per node over its node-sorted pods.
__global__ __launch_bounds__(kBlock) void lease_pods_kernel(void* __restrict__ st, StateFmt fmt,
                                                            const uint32_t* __restrict__ node_ptr,
                                                            const uint8_t* __restrict__ op,
                                                            const kwk_lease* __restrict__ lease, uint32_t me,
                                                            uint32_t n_nodes) {
  const uint32_t node = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (node >= n_nodes) return;
  const uint32_t o = op[node] & 0x7Fu;
  if (o == 0) return;
  const kwk_lease L = lease[node];
  const bool held = (L.flags & KWK_LEASE_EXISTS) && (L.flags & KWK_LEASE_HOLDER) && L.holder == me;
  const bool ok = o != KWK_LEASE_OP_BUSY && o != KWK_LEASE_OP_FAILED;
  for (uint32_t p = node_ptr[node] + (threadIdx.x & 63); p < node_ptr[node + 1]; p += 64) {
    uint2 s = load_state(st, p, fmt);
    if (held) {
      s.y |= KWK_F_MANAGED;
      if (ok && (s.y & KWK_F_ALIVE) && (s.y & 0xFFu) == KWK_STAGE_NONE) s.y |= KWK_F_DIRTY;
    } else {
      s.y &= ~KWK_F_MANAGED;
    }
    store_state(st, p, s, fmt);
  }
}

// kwk_lease_fail: syncWorker's error branch (node_lease_controller.go:121-128) for lease writes
// the apiserver rejected: the informer still shows the old lease (the controller flags HOLD /
// QUEUED stay), the sync is retried after the same interval() draw, and the node's MANAGED bit
// follows Held() of the restored lease without the re-match the write would have caused.
__global__ void lease_fail_kernel(LeaseArgs a, const uint32_t* __restrict__ slots, const kwk_lease* __restrict__ old,
                                  uint32_t n) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t i = slots[j];
  const uint32_t ctl = a.lease[i].flags & (KWK_LEASE_HOLD | KWK_LEASE_QUEUED);
  kwk_lease L = old[j];
  L.flags = (L.flags & ~(KWK_LEASE_HOLD | KWK_LEASE_QUEUED)) | ctl;
  const double factor = a.cfg.renew_jitter <= 0.0 ? 1.0 : a.cfg.renew_jitter;
  const double u = rng_float64(a.slot_base + i, a.step, kSiteLeaseJitter, a.key);
  const int64_t dur = a.cfg.renew_interval_ns + (int64_t)(u * factor * (double)a.cfg.renew_interval_ns);
  L.next_try_ns = sat_add(a.now, dur);  // AddWeightAfter(nodeName, 1, dur)
  a.lease[i] = L;
  const uint32_t prev = a.op[i];
  a.op[i] = (uint8_t)KWK_LEASE_OP_FAILED;
  if (a.cfg.manage_nodes) {
    uint2 s = load_state(a.st, i, a.fmt);
    if (prev & kLeaseOpSetDirty) s.y &= ~KWK_F_DIRTY;
    const bool held = (L.flags & KWK_LEASE_EXISTS) && (L.flags & KWK_LEASE_HOLDER) && L.holder == a.cfg.holder_id;
    s.y = held ? (s.y | KWK_F_MANAGED) : (s.y & ~KWK_F_MANAGED);
    store_state(a.st, i, s, a.fmt);
  }
}

}  // namespace

// ------------------------------------------------------------------ engine object
struct kwk_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  uint32_t capacity = 0, n_active = 0, value_slots = 0, max_records = 0;
  uint64_t slot_base = 0;
  uint32_t kind_salt = 0;
  uint32_t n_blocks_cap = 0, last_blocks = 0, last_grid = 0;
  uint32_t cum_rows = 0;      // statistics rows any sweep grid has written (<= n_blocks_cap)
  uint32_t last_objs = 16;    // words per lane of the last sweep (fired segment stride = 64 * last_objs + 32)
  uint32_t last_region_shift = 0;  // fired segments per record region = 1 << shift (wave: 0, tile: 2)
  int last_rec = 0;                // record kind of the last sweep's segments (kRecSlot / kRecId8 / kRecId8Half)
  bool compacted = false;     // the last sweep's fired list is compacted on the device
  bool compacted_packed = false;  // ... as 4-byte packed records (kwk_fired_compact_packed)
  bool compacted_16 = false;      // ... as the 1-byte sweep's 2-byte records (kwk_fired_compact_packed16)
  bool compacted_bits = false;    // ... as its per-segment maps + stage codes (kwk_fired_compact_bits)
  // The hand-back ring (DESIGN.md §5 "Hand-back"): every compaction writes a slot of its own, in
  // turn — the step's dense list, its scan offsets ([0] = the length) and group totals, the bitmap
  // hand-back's {words, records} and, for 2-byte / bitmap lists, the step's records per segment
  // (the next sweep rewrites d_wave_counts) — tagged with the step it compacted.  So the lists of
  // the last hb.size() compactions stay readable by step (kwk_fired_fetch_step: every step of a
  // kwk_step_n call, fused or not), hb[hb_cur] is the engine's last list (kwk_fired*), and a
  // compaction waits on the device only for the copy of the slot it rewrites.
  struct HbSlot {
    void* list = nullptr;
    size_t list_bytes = 0;
    uint32_t* offsets = nullptr;
    uint32_t* groups = nullptr;
    uint32_t* tot = nullptr;
    uint32_t* counts = nullptr;
    hipEvent_t ev_copied = nullptr;  // the copy stream's last copy out of this slot
    hipEvent_t ev_done = nullptr;    // kwk_fired_keep: recorded after the compaction that wrote the slot
    int done_slot = -1;              // ... the slot whose ev_done marks it (a fused group's last step)
    bool copy_pending = false;       // ev_copied recorded and not yet waited for by a compaction
    bool valid = false;
    uint64_t step = 0;               // the step whose list the slot holds
    int mode = 0;                    // enqueue_compact's mode
    uint32_t n_segs = 0, region_slots = 0;
  };
  std::vector<HbSlot> hb = std::vector<HbSlot>(kHbMin);
  uint32_t hb_cur = 0;
  bool hb_track = false;       // kwk_fired_keep: compactions record ev_done and write their length to h_len
  uint32_t* h_len = nullptr;   // pinned, 2 words per slot (the kernels write them: host_len)
  uint32_t* h_len_dev = nullptr;
  uint64_t last_step_no = 0;   // the step number of the last sweep's (last) step
  hipStream_t copy_stream = nullptr;
  hipEvent_t ev_count = nullptr;  // kwk_fired_fetch_async without kwk_fired_keep: the length's copy
  uint32_t* h_count = nullptr;
  bool copy_recorded = false;  // a copy was enqueued (kwk_fired_fetch_wait)
  kwk_sweep_info last_sweep{};  // kwk_last_sweep
  bool loaded_table = false;
  uint32_t n_stages = 0, n_classes = 0;
  kwk_harness harness{};

  void* d_st = nullptr;       // state word per slot (8-byte capacity; format in fmt)
  StateFmt fmt{};             // current state format (wide until a table allows narrow)
  bool force_wide = false;
  bool allow_half = true;     // KWK_ENGINE_STATE32: never the 2-byte format
  // kernel choices (kwk_set_tuning; defaults = the measured best)
  uint32_t q16 = kQ16;        // 2-byte sweep: 16-byte chunks per lane (1 | 2 | 4)
  bool persist16 = true;      // 2-byte sweep: persistent grid for large engines
  bool use_fsm = true;        // 2-byte sweep: transition table
  bool usage_key8 = true;     // usage fast path: the 1-byte key column when it exists
  bool agg_fused = true;      // KWK_TUNE_USAGE & KWK_USAGE_AGG_FUSED: kwk_aggregate's mask counts inside the usage kernel
  int n_cus = 256;
  std::vector<std::pair<const void*, int>> occupancy;  // blocks per CU per kernel (this engine's device)
  uint32_t* d_fsm = nullptr;  // transition table of the 2-byte format (fsm_build_kernel)
  int64_t* d_fsm_due = nullptr;
  uint32_t fsm_bits = 0;
  int fsm_harness = -1;       // harness enable the table was built for (-1: no table)
  uint32_t fsm_kernel = kFsmKernelDefault;  // KWK_TUNE_SWEEP16 kernel: 0 never, else its prefetch depth
  // the 1-byte format (StateFmt.byte): a dictionary of the half words that can occur
  bool allow_byte = true;     // KWK_ENGINE_STATE16 clears it
  bool allow_dw = true;       // KWK_ENGINE_SPLIT_DUE clears it: never the fused record
  uint32_t word_tpb = 0;      // KWK_TUNE_WORD_TILES: tiles per workgroup of the word sweep (0: per format)
  bool byte_tune = true;      // KWK_TUNE_BYTE_STATE
  bool byte_ok = false;       // the transition table exists for the loaded program and harness
  std::vector<uint32_t> h_fsm;    // host copy of the 2-byte transition table (closure, id table)
  std::vector<int64_t> h_fsm_due;
  std::vector<uint16_t> h_id2w;   // [256] word of each id
  std::vector<uint8_t> h_w2id;    // [65536] id of each half word (kIdInvalid: none)
  uint32_t id_fill[8] = {};       // ids used per class (need, pend, alive)
  uint16_t* d_id2w = nullptr;
  uint8_t* d_w2id = nullptr;
  uint32_t* d_fsm8 = nullptr;     // [2][256] id transition table of sweep8_kernel
  int64_t* d_fsm8_due = nullptr;
  bool fsm8_due_any = false;      // some d_fsm8 entry schedules a delayed stage (kId8Due)
  int64_t* d_due = nullptr;   // due time per slot
  int64_t* d_del = nullptr;
  uint32_t* d_rec = nullptr;
  kwk_value* d_values = nullptr;
  kwk_stage_table* d_table = nullptr;
  uint32_t* d_lut = nullptr;  // kLutTables match masks (valid for lut_n entries)
  uint32_t lut_n = 0, lut_bytes = 0, lut_rest = 0;
  kwk_delta* d_deltas = nullptr;
  kwk_fired_rec* d_fired = nullptr;
  // up to fuse_steps steps per 1-byte sweep launch (KWK_TUNE_FUSE_STEPS, sweep8_kernel<..., kSteps>):
  // steps 1.. segments and counts, rotated with d_fired / d_wave_counts by the steps' hand-backs
  uint32_t fuse_steps = kMaxFuseSteps;
  kwk_fired_rec* d_firedx[kMaxFuseSteps - 1] = {};
  uint32_t* d_countsx[kMaxFuseSteps - 1] = {};
  uint32_t* d_wave_counts = nullptr;
  // the hand-back inside one-tile-per-block 2-byte sweeps (tail_handback, KWK_TUNE_TAIL_HANDBACK):
  // per block the launch's tag and fired count; the tag of the last such launch
  unsigned long long* d_tail_status = nullptr;
  uint32_t tail_seq = 0;
  bool tail_hb = true;
  uint32_t* d_bits_wc = nullptr;      // ... its words per segment
  uint32_t* d_bits_bsum = nullptr;    // ... its records per workgroup of bits_size_kernel
  unsigned long long* d_cum = nullptr;
  unsigned long long* d_stats = nullptr;
  uint64_t steps = 0;

  // usage
  uint32_t n_nodes = 0, n_usage_pods = 0;
  uint32_t* d_node_ptr = nullptr;
  uint32_t* d_ukey = nullptr;
  uint8_t* d_ukey8 = nullptr;   // usage_fast_kernel<WB, true>: 1-byte key column (<= kUKeyDict distinct keys)
  double2* d_kv = nullptr;      // {cpu, mem} per distinct key
  uint32_t kv_n = 0;
  double* d_cpu = nullptr;
  double* d_mem = nullptr;
  double* d_node_out = nullptr;
  double* d_node_cum = nullptr;
  int64_t* d_node_last = nullptr;
  double* d_pod_out = nullptr;   // per pod {cpu, mem, cpu_cumulative, mem_cumulative} (kwk_usage_pods)
  double* d_pod_cum = nullptr;
  int64_t* d_pod_last = nullptr;
  double* d_usage_part = nullptr;
  double* d_cluster = nullptr;
  double* d_agg = nullptr;        // kwk_aggregate's own output buffer
  uint32_t* d_count_part = nullptr;  // count_kernel's per-block partial counts
  unsigned long long* d_agg_counts = nullptr;
  uint32_t agg_masks[16] = {};    // the masks last copied to d_agg_masks (kMaxCountMasks)
  uint32_t agg_n_masks = 0;
  uint32_t* d_agg_masks = nullptr;
  double* d_podv = nullptr;       // usage_fast_kernel's pod values per (containers, value id)
  uint32_t podv_n = 0;
  uint32_t compact_small = 8192;  // KWK_TUNE_COMPACT_SMALL (kSmallSegs)
  uint4* d_uchunk = nullptr;      // usage_kernel's chunks of whole nodes {first pod, end pod, first node, end node}
  uint32_t n_uchunks = 0;
  // host copies of the usage configuration (per-container reads, metric scrapes)
  std::vector<uint32_t> h_node_ptr, h_ukey, h_mixed, h_ckeys, h_cptr;
  std::vector<double> h_cpu, h_mem;
  bool has_mixed_keys = false;
  uint2* d_mixed = nullptr;       // {first, count} per mixed pod
  uint32_t* d_ckeys = nullptr;
  double* d_ccum = nullptr;       // per container of a mixed pod: {cpu, mem} integrators
  uint32_t* d_mbase = nullptr;    // per pod: first integrator of its containers in d_ccum (mixed pods)
  std::vector<uint32_t> h_mbase;
  uint32_t* d_cptr = nullptr;     // per pod: first container (metric scrapes)
  // Metric CRD programs
  kwk_metric_op* d_mops = nullptr;
  std::vector<kwk_metric_desc> metrics;
  uint32_t metric_inputs_needed = 0;  // 1: some program reads creation times / started containers
  int64_t* d_pod_created = nullptr;
  int64_t* d_node_created = nullptr;
  double* d_node_started = nullptr;
  double zero_time_unix_s = 0.0;
  double* d_mout = nullptr;
  size_t mout_cap = 0;
  // histogram Metric programs (kwk_histograms_load)
  kwk_metric_op* d_hops = nullptr;
  kwk_metric_bucket* d_hbuckets = nullptr;
  uint32_t* d_hkeys = nullptr;
  double* d_hbounds = nullptr;
  std::vector<HistDesc> hists;
  uint32_t hist_inputs_needed = 0;
  uint64_t* d_hout = nullptr;
  size_t hout_cap = 0;

  // staging for upserts
  void* d_stage_buf = nullptr;
  size_t stage_bytes = 0;

  // node leases (node engines only)
  bool lease_on = false;
  kwk_lease_params lease_cfg{};
  kwk_lease* d_lease = nullptr;
  uint8_t* d_lease_op = nullptr;
  kwk_fired_rec* d_lease_ops = nullptr;
  uint32_t* d_lease_nops = nullptr;   // [2]: API writes of the last lease step / zeroed for the next one
  uint32_t lease_par = 0;               // d_lease_nops entry the next lease step counts into
  uint32_t lease_last = 0;              // entry of the last lease step (kwk_lease_ops)
  // kwk_tick_bind (pod engines): the node engine whose lease results the fused tick applies
  const kwk_engine* tick_nodes = nullptr;
  uint32_t tick_n_nodes = 0;
  uint32_t* d_tick_ptr = nullptr;       // node_ptr on the device
  hipEvent_t ev_lease = nullptr;        // node stream: the tick's lease step is done
  hipEvent_t ev_podsync = nullptr;      // pod stream: the tick's pod sync has read the lease results
  bool tick_pending = false;            // ev_podsync recorded by an earlier tick
  kwk_engine* tick_pods = nullptr;      // node engines: the pod engine of the last fused tick
  unsigned long long* d_lease_stats = nullptr;
  uint64_t lease_steps = 0;

  std::vector<hipEvent_t> events;
  std::string err;            // message of the last failing call on this engine (kwk_last_error)
};

static void engine_set_error(kwk_engine* e, const std::string& msg) { e->err = msg; }

// live engines: a fused tick links a pod engine and a node engine; destroying either unlinks it
static std::mutex g_live_mu;
static std::set<kwk_engine*> g_live;


// narrow iff pred + class + stage code + 5 flag bits fit 32 bits, half iff they fit 16, fused
// (dw) iff they fit 28 and not 16
static StateFmt make_fmt(uint32_t pred_bits, uint32_t n_classes, uint32_t n_stages, bool allow_narrow, bool allow_half,
                         bool allow_dw) {
  auto bitlen = [](uint32_t x) {
    uint32_t b = 0;
    while (x) { ++b; x >>= 1; }
    return b;
  };
  const uint32_t pb = pred_bits == 0 ? 32u : pred_bits;
  const uint32_t cb = bitlen(n_classes ? n_classes - 1 : 0);
  const uint32_t sb = bitlen(n_stages);  // codes 0..n_stages, n_stages = none
  StateFmt f{};
  if (!allow_narrow || pb + cb + sb + 5 > 32) return f;
  f.narrow = 1;
  f.half = (allow_half && pb + cb + sb + 5 <= 16) ? 1u : 0u;
  f.dw = (allow_dw && !f.half && pb + cb + sb + 5 <= kDwShift) ? 1u : 0u;
  f.pmask = (1u << pb) - 1u;
  f.cshift = pb;
  f.cmask = cb ? ((1u << cb) - 1u) : 0u;
  f.sshift = pb + cb;
  f.smask = sb ? ((1u << sb) - 1u) : 0u;
  f.none_code = n_stages;
  f.fshift = pb + cb + sb;
  return f;
}

static kwk_status build_fsm(kwk_engine* e);

static size_t word_bytes(const StateFmt& f) { return f.byte ? 1 : f.half ? 2 : f.dw ? 8 : f.narrow ? 4 : 8; }

// the layout only (the fused format's epoch moves with time)
static bool same_fmt(const StateFmt& a, const StateFmt& b) {
  StateFmt x = a, y = b;
  x.epoch = y.epoch = 0;
  return memcmp(&x, &y, sizeof(StateFmt)) == 0;
}

// host-side conversion of device state words <-> (pred, sched); the 1-byte format through the
// engine's dictionary
static std::vector<uint2> unpack_words(const kwk_engine* e, const std::vector<uint8_t>& raw, const StateFmt& f, uint32_t n) {
  std::vector<uint2> out(n);
  if (f.byte) {
    for (uint32_t i = 0; i < n; ++i) out[i] = fmt_unpack(e->h_id2w[raw[i]], f);
  } else if (f.half) {
    const uint16_t* w = reinterpret_cast<const uint16_t*>(raw.data());
    for (uint32_t i = 0; i < n; ++i) out[i] = fmt_unpack(w[i], f);
  } else if (f.dw) {  // the word of each record (due times: dw_unfold + the due column)
    const uint32_t* w = reinterpret_cast<const uint32_t*>(raw.data());
    for (uint32_t i = 0; i < n; ++i) out[i] = fmt_unpack(w[2 * (size_t)i], f);
  } else if (f.narrow) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(raw.data());
    for (uint32_t i = 0; i < n; ++i) out[i] = fmt_unpack(w[i], f);
  } else {
    memcpy(out.data(), raw.data(), sizeof(uint2) * (size_t)n);
  }
  return out;
}

static std::vector<uint8_t> pack_words(const kwk_engine* e, const std::vector<uint2>& v, const StateFmt& f) {
  std::vector<uint8_t> raw(word_bytes(f) * v.size());
  if (f.byte) {
    for (size_t i = 0; i < v.size(); ++i) raw[i] = e->h_w2id[fmt_pack(v[i].x, v[i].y, f) & 0xFFFFu];
  } else if (f.half) {
    uint16_t* w = reinterpret_cast<uint16_t*>(raw.data());
    for (size_t i = 0; i < v.size(); ++i) w[i] = (uint16_t)fmt_pack(v[i].x, v[i].y, f);
  } else if (f.dw) {  // records with D = 0 (dw_fold sets it from the due column)
    uint32_t* w = reinterpret_cast<uint32_t*>(raw.data());
    for (size_t i = 0; i < v.size(); ++i) w[2 * i] = fmt_pack(v[i].x, v[i].y, f);
  } else if (f.narrow) {
    uint32_t* w = reinterpret_cast<uint32_t*>(raw.data());
    for (size_t i = 0; i < v.size(); ++i) w[i] = fmt_pack(v[i].x, v[i].y, f);
  } else {
    memcpy(raw.data(), v.data(), sizeof(uint2) * v.size());
  }
  return raw;
}

// the narrow format holds only pred bits < pred_bits and stage indices < n_stages
static bool fits_fmt(const StateFmt& f, uint32_t n_stages, uint32_t pred, uint32_t sched) {
  if (!f.narrow) return true;
  const uint32_t st = sched & 0xFFu;
  return (pred & ~f.pmask) == 0 && (st == KWK_STAGE_NONE || st < n_stages);
}

static kwk_status set_dev(kwk_engine* e) {
  HIP_TRY(hipSetDevice(e->device));
  return KWK_OK;
}

// host -> device on the engine's stream, complete on return.  A pageable hipMemcpy on the null
// stream may return with its DMA still in flight, and the engine's stream is non-blocking: a
// kernel enqueued next on it ran concurrently with the upload (dw_fold_kernel after a 100M-object
// kwk_load: 110-140 ms, overlapping the copy, vs 0.48 ms ordered after it, r3zf / r3zg)
static hipError_t upload(const kwk_engine* e, void* dst, const void* src, size_t bytes) {
  const hipError_t r = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, e->stream);
  return r != hipSuccess ? r : hipStreamSynchronize(e->stream);
}

static kwk_status ensure_stage_buf(kwk_engine* e, size_t bytes) {
  if (bytes <= e->stage_bytes) return KWK_OK;
  if (e->d_stage_buf) HIP_TRY(hipFree(e->d_stage_buf));
  e->d_stage_buf = nullptr;
  HIP_TRY(hipMalloc(&e->d_stage_buf, bytes));
  e->stage_bytes = bytes;
  return KWK_OK;
}

// ---- the 1-byte format's dictionary
// class of a half word: bit 2 needs work whatever its due (managed, and dirty or the harness
// churns it), bit 1 a queued stage (managed), bit 0 alive — the id's top three bits
static uint32_t word_class(const kwk_engine* e, uint32_t w) {
  const StateFmt& f = e->fmt;
  const uint32_t fl = (w >> f.fshift) & 0x1Fu;  // sched bits 8..12
  const bool alive = fl & (KWK_F_ALIVE >> 8), dirty = fl & (KWK_F_DIRTY >> 8), managed = fl & (KWK_F_MANAGED >> 8);
  const uint32_t pred = w & f.pmask;
  const bool pend = managed && ((w >> f.sshift) & f.smask) != f.none_code;
  bool need = false;
  if (managed) {
    need = dirty;
    if (e->harness.enable) {
      const uint32_t term = e->harness.terminal_mask & f.pmask, del = e->harness.deletion_bit & f.pmask;
      need = need || !alive || ((pred & term) != 0 && (pred & del) == 0);
    }
  }
  return (need ? 4u : 0u) | (pend ? 2u : 0u) | (alive ? 1u : 0u);
}

// the words a half word can become on the device: the transition table for the lookups the sweep
// makes (need -> not ready, queued -> ready), kwk_delete, and the lease updates of MANAGED /
// DIRTY; false if a reachable lookup is general (a Philox draw, a record or the deletion column)
static bool word_successors(const kwk_engine* e, uint32_t w, std::vector<uint32_t>& out) {
  const uint32_t cls = word_class(e, w);
  const uint32_t bits = e->fsm_bits;
  if (cls & 4u) {
    const uint32_t t = e->h_fsm[w];
    if (t & kFsmGeneral) return false;
    out.push_back(t & 0xFFFFu);
  }
  if (cls & 2u) {
    const uint32_t t = e->h_fsm[(1u << bits) | w];
    if (t & kFsmGeneral) return false;
    out.push_back(t & 0xFFFFu);
  }
  const uint2 v = fmt_unpack(w, e->fmt);
  auto add = [&](uint32_t sched) { out.push_back(fmt_pack(v.x, sched, e->fmt) & 0xFFFFu); };
  add((v.y & ~(KWK_F_ALIVE | KWK_F_DIRTY | 0xFFu)) | KWK_STAGE_NONE);  // kwk_delete
  add(v.y | KWK_F_MANAGED);   // lease_kernel / lease_pods_kernel: Held()
  add(v.y & ~KWK_F_MANAGED);
  add(v.y | KWK_F_DIRTY);     // a successful lease sync re-matches
  add(v.y & ~KWK_F_DIRTY);    // kwk_lease_fail undoes it
  return true;
}

// index within class c of its j-th id: classes start 4 banks apart (class 7 at 0, so that its
// last index, 0xFF = kIdInvalid, is never reached), so the id-table entries that the
// 1-byte sweep's lanes look up together rarely share an LDS bank
static uint32_t id8_index(uint32_t c, uint32_t j) { return c == 7u ? j : (j + 4u * c) & kIdIndex; }
static uint32_t id8_rank(uint32_t id) {
  const uint32_t c = id >> 5;
  return c == 7u ? (id & kIdIndex) : ((id & kIdIndex) - 4u * c) & kIdIndex;
}

static void dict_reset(kwk_engine* e) {
  e->h_id2w.assign(256, 0);
  e->h_w2id.assign(65536, (uint8_t)kIdInvalid);
  for (uint32_t& c : e->id_fill) c = 0;
  e->h_w2id[0] = 0;  // id 0 = word 0 (padding, never-loaded slots): not alive, not managed
  e->id_fill[0] = 1;
}

// adds the closure of `seeds` to the dictionary; false (dictionary unchanged) if a class runs out
// of ids or a general transition is reachable
static bool dict_extend(kwk_engine* e, const std::vector<uint32_t>& seeds, bool& changed) {
  changed = false;
  std::vector<uint32_t> added, frontier, next;
  std::vector<uint8_t> seen(65536, 0);
  for (uint32_t w : seeds) {
    w &= 0xFFFFu;
    if (e->h_w2id[w] == kIdInvalid && !seen[w]) {
      seen[w] = 1;
      frontier.push_back(w);
    }
  }
  uint32_t fill[8];
  memcpy(fill, e->id_fill, sizeof(fill));
  while (!frontier.empty()) {
    next.clear();
    for (uint32_t w : frontier) {
      const uint32_t c = word_class(e, w);
      if (fill[c] >= (c == 7u ? kIdIndex : kIdIndex + 1u)) return false;  // 0xFF stays invalid
      ++fill[c];
      added.push_back(w);
      std::vector<uint32_t> succ;
      if (!word_successors(e, w, succ)) return false;
      for (uint32_t x : succ)
        if (e->h_w2id[x] == kIdInvalid && !seen[x]) {
          seen[x] = 1;
          next.push_back(x);
        }
    }
    frontier.swap(next);
  }
  for (uint32_t w : added) {
    const uint32_t c = word_class(e, w);
    const uint32_t id = (c << 5) | id8_index(c, e->id_fill[c]++);
    e->h_id2w[id] = (uint16_t)w;
    e->h_w2id[w] = (uint8_t)id;
  }
  changed = !added.empty();
  return true;
}

// the dictionary and the id transition table on the device (synchronous)
static kwk_status dict_upload(kwk_engine* e) {
  std::vector<uint32_t> t8(512);
  e->fsm8_due_any = false;
  std::vector<int64_t> d8(512, 0);
  const uint32_t bits = e->fsm_bits;
  for (uint32_t id = 0; id < 256; ++id) {
    const uint32_t w = e->h_id2w[id];
    const bool used = id == 0 || (id != kIdInvalid && id8_rank(id) < e->id_fill[id >> 5]);
    for (uint32_t rdy = 0; rdy < 2; ++rdy) {
      const uint32_t t = e->h_fsm[(rdy << bits) | w];
      uint32_t x = id;  // unused ids and lookups the sweep never makes: no change, nothing fires
      if (used && !(t & kFsmGeneral) && e->h_w2id[t & 0xFFFFu] != kIdInvalid) {
        // the 2-byte entry ([20:16] stage, [21] fired, [24:22] flags, [25] matched, [29:26]
        // bytes / 2 counting a 2-byte word write, [30] due) in the id layout (kId8*)
        const uint32_t bytes8 = ((t >> 26) & 15u) * 2u - 1u, stage = (t >> 16) & 31u, flags = (t >> 22) & 7u;
        x = e->h_w2id[t & 0xFFFFu] | (stage & 3u) << 11 | flags << 13 | stage << 16 | flags << 21 | bytes8 << 24 |
            ((t & kFsmDue) ? kId8Due : 0u) | ((t >> 25) & 1u) * kId8Match | ((t >> 21) & 1u) * kId8Fire;
        if (t & kFsmDue) e->fsm8_due_any = true;
        d8[(rdy << 8) | id] = e->h_fsm_due[(rdy << bits) | w];
      }
      t8[(rdy << 8) | id] = x;
    }
  }
  HIP_TRY(upload(e, e->d_id2w, e->h_id2w.data(), sizeof(uint16_t) * 256));
  HIP_TRY(upload(e, e->d_w2id, e->h_w2id.data(), 65536));
  HIP_TRY(upload(e, e->d_fsm8, t8.data(), sizeof(uint32_t) * 512));
  HIP_TRY(upload(e, e->d_fsm8_due, d8.data(), sizeof(int64_t) * 512));
  return KWK_OK;
}

// the fused format: records' D from the due column / the due column made exact (stream-ordered)
static kwk_status dw_fold(kwk_engine* e, uint32_t first, uint32_t n) {
  if (!e->fmt.dw || n == 0) return KWK_OK;
  const uint32_t g = std::min((n + kBlock - 1) / kBlock, (uint32_t)e->n_cus * 32u);
  hipLaunchKernelGGL(dw_fold_kernel, dim3(g), dim3(kBlock), 0, e->stream,
                     reinterpret_cast<uint2*>(e->d_st), e->d_due, first, n, e->fmt.epoch);
  HIP_TRY(hipGetLastError());
  return KWK_OK;
}
static kwk_status dw_unfold(kwk_engine* e, uint32_t first, uint32_t n) {
  if (!e->fmt.dw || n == 0) return KWK_OK;
  const uint32_t g = std::min((n + kBlock - 1) / kBlock, (uint32_t)e->n_cus * 32u);
  hipLaunchKernelGGL(dw_unfold_kernel, dim3(g), dim3(kBlock), 0, e->stream,
                     reinterpret_cast<const uint2*>(e->d_st), e->d_due, first, n, e->fmt.epoch);
  HIP_TRY(hipGetLastError());
  return KWK_OK;
}

// resident rows [0, n_active) as (pred, sched) (synchronises; the due column is left exact)
static kwk_status read_rows(kwk_engine* e, std::vector<uint2>& rows) {
  const uint32_t n = e->n_active;
  if (kwk_status st = dw_unfold(e, 0, n)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  std::vector<uint8_t> raw(word_bytes(e->fmt) * (size_t)n);
  if (n) HIP_TRY(hipMemcpy(raw.data(), e->d_st, raw.size(), hipMemcpyDeviceToHost));
  rows = unpack_words(e, raw, e->fmt, n);
  return KWK_OK;
}

// writes rows [0, n) in format nf and makes nf current (the dictionary must hold their words)
static kwk_status write_rows(kwk_engine* e, const std::vector<uint2>& rows, const StateFmt& nf) {
  const std::vector<uint8_t> out = pack_words(e, rows, nf);
  if (!out.empty()) HIP_TRY(hipMemcpyAsync(e->d_st, out.data(), out.size(), hipMemcpyHostToDevice, e->stream));
  e->fmt = nf;
  if (kwk_status st = dw_fold(e, 0, (uint32_t)rows.size())) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));  // `out` goes with this frame
  return KWK_OK;
}

// the format without the dictionary (2-byte words when the program fits 16 bits)
static StateFmt base_fmt(const StateFmt& f) {
  StateFmt b = f;
  b.byte = 0;
  b.id2w = nullptr;
  b.w2id = nullptr;
  return b;
}

static bool byte_allowed(const kwk_engine* e) {
  return e->fmt.half && e->byte_ok && e->allow_byte && e->byte_tune && e->use_fsm && e->fsm_kernel != 0 &&
         e->fsm_harness >= 0;
}

// the 1-byte format when the program allows it and the dictionary closes over `rows`, else the
// base format; sets e->fmt (and uploads the dictionary) without writing the state column
static kwk_status pick_format(kwk_engine* e, const std::vector<uint2>& rows, StateFmt& nf) {
  nf = base_fmt(e->fmt);
  if (!(nf.half && byte_allowed(e))) return KWK_OK;
  const StateFmt saved = e->fmt;
  e->fmt = nf;  // word_class reads the half layout
  dict_reset(e);
  std::vector<uint32_t> seeds;
  seeds.reserve(rows.size() + 1);
  std::vector<uint8_t> seen(65536, 0);
  for (const uint2& r : rows) {
    const uint32_t w = fmt_pack(r.x, r.y, nf) & 0xFFFFu;
    if (!seen[w]) { seen[w] = 1; seeds.push_back(w); }
  }
  bool changed = false;
  const bool ok = dict_extend(e, seeds, changed);
  e->fmt = saved;
  if (!ok) return KWK_OK;
  if (kwk_status st = dict_upload(e)) return st;
  nf.byte = 1;
  nf.id2w = e->d_id2w;
  nf.w2id = e->d_w2id;
  return KWK_OK;
}

// re-decides the format for the resident objects (after a table / harness / tuning change)
static kwk_status refresh_format(kwk_engine* e) {
  std::vector<uint2> rows;
  if (kwk_status st = read_rows(e, rows)) return st;
  StateFmt nf;
  if (kwk_status st = pick_format(e, rows, nf)) return st;
  return write_rows(e, rows, nf);
}

// rows about to be written by an upsert / replace / retry: in the 1-byte format their words join
// the dictionary, or the engine returns to the 2-byte words
static kwk_status admit_rows(kwk_engine* e, const std::vector<uint2>& incoming) {
  if (!e->fmt.byte) return KWK_OK;
  std::vector<uint32_t> seeds;
  for (const uint2& r : incoming) seeds.push_back(fmt_pack(r.x, r.y, e->fmt) & 0xFFFFu);
  bool changed = false;
  if (dict_extend(e, seeds, changed)) return changed ? dict_upload(e) : KWK_OK;
  std::vector<uint2> rows;
  if (kwk_status st = read_rows(e, rows)) return st;
  return write_rows(e, rows, base_fmt(e->fmt));
}

// leaves the 1-byte format (a call the table-only sweep does not cover, e.g. kwk_match)
static kwk_status leave_byte(kwk_engine* e) {
  if (!e->fmt.byte) return KWK_OK;
  std::vector<uint2> rows;
  if (kwk_status st = read_rows(e, rows)) return st;
  return write_rows(e, rows, base_fmt(e->fmt));
}

extern "C" {

const char* kwk_last_error(const kwk_engine* e) { return e ? e->err.c_str() : g_err.c_str(); }

// ------------------------------------------------------------------ hand-back ring
static void hb_free(kwk_engine::HbSlot& h) {
  for (void* p : {h.list, (void*)h.offsets, (void*)h.groups, (void*)h.tot, (void*)h.counts})
    if (p) hipFree(p);
  for (hipEvent_t ev : {h.ev_copied, h.ev_done})
    if (ev) hipEventDestroy(ev);
  h = kwk_engine::HbSlot{};
}

kwk_status kwk_engine_create(const kwk_engine_desc* d, kwk_engine** out) {
  if (!d || !out) return fail(KWK_EINVAL, "null argument");
  if (d->capacity == 0) return fail(KWK_EINVAL, "capacity must be > 0");
  if ((uint64_t)d->capacity * 8u >= kOOB)  // 32-bit buffer offsets of the due column (sweep phase 1)
    return fail(KWK_ECAP, "capacity above 536870909 slots per engine: shard the kind over more engines");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (d->device < 0 || d->device >= ndev) return fail(KWK_EINVAL, "device ordinal out of range");
  auto* e = new kwk_engine();
  e->device = d->device;
  e->capacity = d->capacity;
  e->value_slots = d->value_slots ? d->value_slots : 1;
  e->max_records = d->max_records ? d->max_records : 1;
  e->slot_base = d->slot_base;
  e->kind_salt = d->kind_salt;
  e->n_blocks_cap = (d->capacity + kBlock * kMinObjPerThread - 1) / (kBlock * kMinObjPerThread);
  e->force_wide = (d->flags & KWK_ENGINE_WIDE_STATE) != 0;
  e->allow_half = (d->flags & KWK_ENGINE_STATE32) == 0;
  e->allow_byte = (d->flags & (KWK_ENGINE_STATE32 | KWK_ENGINE_STATE16 | KWK_ENGINE_WIDE_STATE)) == 0;
  e->allow_dw = (d->flags & KWK_ENGINE_SPLIT_DUE) == 0;
  kwk_status st = set_dev(e);
  if (st) { delete e; return st; }
  if (hipDeviceGetAttribute(&e->n_cus, hipDeviceAttributeMultiprocessorCount, e->device) != hipSuccess || e->n_cus <= 0)
    e->n_cus = 256;
  const size_t n_waves = (size_t)e->n_blocks_cap * kWavesPerBlock;
#define ALLOC(p, bytes)                                                          \
  do {                                                                           \
    hipError_t er = hipMalloc((void**)&(p), (bytes));                            \
    if (er != hipSuccess) {                                                      \
      kwk_engine_destroy(e);                                                     \
      return fail(KWK_EHIP, std::string("hipMalloc: ") + hipGetErrorString(er)); \
    }                                                                            \
  } while (0)
  // state words: 8 bytes per slot (wide), slots padded to the largest sweep tile so that whole
  // chunks / lines of the last tile stay inside the allocation
  const size_t st_slots = ((size_t)e->capacity + kBlock * kMaxObjPerThread - 1) / (kBlock * kMaxObjPerThread) *
                          (kBlock * kMaxObjPerThread);
  ALLOC(e->d_st, sizeof(uint2) * st_slots);
  ALLOC(e->d_due, sizeof(int64_t) * (size_t)e->capacity);
  ALLOC(e->d_del, sizeof(int64_t) * (size_t)e->capacity);
  ALLOC(e->d_rec, sizeof(uint32_t) * (size_t)e->capacity);
  ALLOC(e->d_values, sizeof(kwk_value) * (size_t)e->max_records * e->value_slots);
  ALLOC(e->d_table, sizeof(kwk_stage_table));
  ALLOC(e->d_lut, sizeof(uint32_t) * kLutTables);
  ALLOC(e->d_fired, sizeof(kwk_fired_rec) * ((size_t)e->n_blocks_cap * kBlock * kMinObjPerThread +
                                              (size_t)kBlock * kMaxObjPerThread));
  ALLOC(e->d_wave_counts, sizeof(uint32_t) * (n_waves + 1));
  ALLOC(e->d_tail_status, sizeof(unsigned long long) * ((size_t)e->n_blocks_cap + 1));
  ALLOC(e->d_bits_wc, sizeof(uint32_t) * (n_waves + 4));
  ALLOC(e->d_bits_bsum, sizeof(uint32_t) * (n_waves / kSegsPerBlock + 4));
  ALLOC(e->d_cum, sizeof(unsigned long long) * (size_t)e->n_blocks_cap * kStatWords);
  ALLOC(e->d_stats, sizeof(unsigned long long) * kStatWords);
  ALLOC(e->d_id2w, sizeof(uint16_t) * 256);
  ALLOC(e->d_w2id, 65536);
  ALLOC(e->d_fsm8, sizeof(uint32_t) * 512);
  ALLOC(e->d_fsm8_due, sizeof(int64_t) * 512);
  hipError_t er = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
  if (er != hipSuccess) { kwk_engine_destroy(e); return fail(KWK_EHIP, "hipStreamCreate"); }
  hipMemsetAsync(e->d_st, 0, sizeof(uint2) * st_slots, e->stream);
  hipMemsetAsync(e->d_due, 0, sizeof(int64_t) * (size_t)e->capacity, e->stream);
  hipMemsetAsync(e->d_cum, 0, sizeof(unsigned long long) * (size_t)e->n_blocks_cap * kStatWords, e->stream);
  hipMemsetAsync(e->d_wave_counts, 0, sizeof(uint32_t) * (n_waves + 1), e->stream);
  hipMemsetAsync(e->d_tail_status, 0, sizeof(unsigned long long) * ((size_t)e->n_blocks_cap + 1), e->stream);
#undef ALLOC
  er = hipStreamSynchronize(e->stream);
  if (er != hipSuccess) { kwk_engine_destroy(e); return fail(KWK_EHIP, hipGetErrorString(er)); }
  {
    std::lock_guard<std::mutex> lk(g_live_mu);
    g_live.insert(e);
  }
  *out = e;
  return KWK_OK;
}

kwk_status kwk_engine_destroy(kwk_engine* e) {
  if (!e) return KWK_OK;
  {
    std::lock_guard<std::mutex> lk(g_live_mu);
    g_live.erase(e);
    kwk_engine* tn = const_cast<kwk_engine*>(e->tick_nodes);
    if (tn && g_live.count(tn) && tn->tick_pods == e) tn->tick_pods = nullptr;
    if (e->tick_pods && g_live.count(e->tick_pods) && e->tick_pods->tick_nodes == e) {
      e->tick_pods->tick_nodes = nullptr;
      e->tick_pods->tick_n_nodes = 0;
    }
  }
  hipSetDevice(e->device);
  if (e->stream) hipStreamSynchronize(e->stream);
  if (e->copy_stream) hipStreamSynchronize(e->copy_stream);
  for (kwk_engine::HbSlot& h : e->hb) hb_free(h);
  for (uint32_t i = 0; i + 1 < kMaxFuseSteps; ++i) {
    if (e->d_firedx[i]) hipFree(e->d_firedx[i]);
    if (e->d_countsx[i]) hipFree(e->d_countsx[i]);
  }
  void* ptrs[] = {                  e->d_bits_wc, e->d_bits_bsum, e->d_st, e->d_due, e->d_del, e->d_rec, e->d_values, e->d_table, e->d_lut, e->d_deltas, e->d_fired,
                  e->d_wave_counts, e->d_tail_status, e->d_cum, e->d_stats,
                  e->d_node_ptr, e->d_ukey, e->d_cpu, e->d_mem, e->d_node_out, e->d_node_cum, e->d_node_last,
                  e->d_usage_part, e->d_cluster, e->d_uchunk, e->d_podv, e->d_agg, e->d_agg_counts, e->d_agg_masks, e->d_count_part, e->d_stage_buf, e->d_pod_out, e->d_pod_cum, e->d_pod_last,
                  e->d_lease, e->d_lease_op, e->d_lease_ops, e->d_fsm, e->d_fsm_due, e->d_mixed, e->d_ckeys, e->d_ccum,
                  e->d_mbase, e->d_cptr, e->d_mops, e->d_pod_created, e->d_node_created, e->d_node_started, e->d_mout,
                  e->d_lease_nops, e->d_lease_stats, e->d_ukey8, e->d_kv, e->d_hops, e->d_hbuckets, e->d_hkeys,
                  e->d_hbounds, e->d_hout, e->d_id2w, e->d_w2id, e->d_fsm8, e->d_fsm8_due};
  for (void* p : ptrs) if (p) hipFree(p);
  if (e->d_tick_ptr) hipFree(e->d_tick_ptr);
  if (e->ev_lease) hipEventDestroy(e->ev_lease);
  if (e->ev_podsync) hipEventDestroy(e->ev_podsync);
  if (e->ev_count) hipEventDestroy(e->ev_count);
  if (e->h_count) hipHostFree(e->h_count);
  if (e->h_len) hipHostFree(e->h_len);
  if (e->copy_stream) hipStreamDestroy(e->copy_stream);
  for (auto ev : e->events) hipEventDestroy(ev);
  if (e->stream) hipStreamDestroy(e->stream);
  delete e;
  return KWK_OK;
}

kwk_status kwk_load_stages(kwk_engine* e, const kwk_stage_table* t, const kwk_delta* deltas) {
  ErrScope es_(e);
  if (!e || !t) return fail(KWK_EINVAL, "null argument");
  if (t->n_stages > KWK_MAX_STAGES) return fail(KWK_EINVAL, "too many stages");
  if (t->n_classes == 0 && t->n_stages) return fail(KWK_EINVAL, "n_classes must be > 0");
  for (uint32_t s = 0; s < t->n_stages; ++s) {
    const kwk_stage_desc& S = t->stages[s];
    if (S.n_any > KWK_MAX_ANY) return fail(KWK_EINVAL, "stage " + std::to_string(s) + ": n_any > KWK_MAX_ANY");
    const int32_t slots[3] = {S.weight_slot, S.delay_slot, S.jitter_slot};
    for (int32_t sl : slots)
      if (sl < KWK_SLOT_DELETION || sl >= (int32_t)e->value_slots)
        return fail(KWK_EINVAL, "stage " + std::to_string(s) + ": value slot out of range");
    if (S.weight_slot == KWK_SLOT_DELETION) return fail(KWK_EINVAL, "weight cannot use the deletion column");
  }
  if (t->pred_bits > 32) return fail(KWK_EINVAL, "pred_bits > 32");
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  StateFmt nf = make_fmt(t->pred_bits, t->n_classes, t->n_stages, !e->force_wide, e->allow_half, e->allow_dw);
  nf.epoch = e->fmt.epoch;
  if (!same_fmt(nf, e->fmt)) {
    if (e->n_active) {  // repack the resident objects into the new format
      const uint32_t n = e->n_active;
      if (kwk_status st = dw_unfold(e, 0, n)) return st;  // the due column exact before leaving the fused format
      HIP_TRY(hipStreamSynchronize(e->stream));
      std::vector<uint8_t> raw(word_bytes(e->fmt) * (size_t)n);
      HIP_TRY(hipMemcpy(raw.data(), e->d_st, raw.size(), hipMemcpyDeviceToHost));
      std::vector<uint2> v = unpack_words(e, raw, e->fmt, n);
      for (uint32_t i = 0; i < n; ++i)
        if (!fits_fmt(nf, t->n_stages, v[i].x, v[i].y) || (v[i].y >> KWK_CLASS_SHIFT) >= (t->n_classes ? t->n_classes : 1))
          return fail(KWK_EINVAL, "resident object " + std::to_string(i) + " does not fit the new stage table");
      std::vector<uint8_t> out = pack_words(e, v, nf);
      HIP_TRY(hipMemcpyAsync(e->d_st, out.data(), out.size(), hipMemcpyHostToDevice, e->stream));
      e->fmt = nf;
      if (kwk_status st = dw_fold(e, 0, n)) return st;
      HIP_TRY(hipStreamSynchronize(e->stream));
    }
    e->fmt = nf;
  }
  {  // the device copy carries the stages with a Delay jitter in reserved[0] (match_object's draw test)
    kwk_stage_table dt = *t;
    dt.reserved[0] = 0;
    for (uint32_t s = 0; s < t->n_stages; ++s)
      if (t->stages[s].has_delay && t->stages[s].has_jitter) dt.reserved[0] |= 1u << s;
    HIP_TRY(upload(e, e->d_table, &dt, sizeof(kwk_stage_table)));
  }
  // the match set of every pred value, when pred_bits is small (Lifecycle.match, lifecycle.go:51-63)
  // match-mask tables (match_mask): one exact table up to 8 pred bits, else one per pred byte
  // for the stages whose clauses each lie within one byte
  e->lut_n = e->lut_bytes = e->lut_rest = 0;
  if (t->pred_bits != 0 && t->pred_bits <= 8) {
    e->lut_n = 1u << t->pred_bits;
    e->lut_bytes = 1;
  } else if (t->pred_bits > 8) {
    e->lut_bytes = (t->pred_bits + 7) / 8;
    e->lut_n = 256u * e->lut_bytes;
  }
  if (e->lut_n) {
    std::vector<uint32_t> lut(e->lut_n, 0u);
    if (e->lut_bytes == 1 && e->lut_n <= 256) {
      for (uint32_t p = 0; p < e->lut_n; ++p)
        for (uint32_t s = 0; s < t->n_stages; ++s) lut[p] |= (stage_matches(t->stages[s], p) ? 1u : 0u) << s;
    } else {
      for (uint32_t s = 0; s < t->n_stages; ++s) {
        const kwk_stage_desc& S = t->stages[s];
        bool sep = true;
        for (uint32_t k = 0; k < S.n_any; ++k) {
          const uint32_t am = S.any_mask[k];
          bool one = false;
          for (uint32_t b = 0; b < 4; ++b) one |= am != 0 && (am & ~(0xFFu << (8 * b))) == 0;
          sep &= one || am == 0;
        }
        if (!sep) { e->lut_rest |= 1u << s; continue; }
        for (uint32_t b = 0; b < e->lut_bytes; ++b)
          for (uint32_t v = 0; v < 256; ++v) {
            const uint32_t x = v << (8 * b), bm = 0xFFu << (8 * b);
            bool ok = ((x ^ S.eq_val) & S.eq_mask & bm) == 0;
            for (uint32_t k = 0; k < S.n_any; ++k)
              if ((S.any_mask[k] & ~bm) == 0 && S.any_mask[k])
                ok &= ((x & S.any_mask[k]) != 0) == (((S.any_want >> k) & 1u) != 0);
              else if (S.any_mask[k] == 0 && b == 0)
                ok &= ((S.any_want >> k) & 1u) == 0;  // an empty clause is never satisfied
            lut[256 * b + v] |= (ok ? 1u : 0u) << s;
          }
      }
    }
    HIP_TRY(upload(e, e->d_lut, lut.data(), sizeof(uint32_t) * e->lut_n));
  }
  if (e->d_deltas) HIP_TRY(hipFree(e->d_deltas));
  e->d_deltas = nullptr;
  const size_t nd = (size_t)(t->n_classes ? t->n_classes : 1) * (t->n_stages ? t->n_stages : 1);
  HIP_TRY(hipMalloc(&e->d_deltas, sizeof(kwk_delta) * nd));
  if (deltas && t->n_stages) HIP_TRY(upload(e, e->d_deltas, deltas, sizeof(kwk_delta) * nd));
  else HIP_TRY(hipMemsetAsync(e->d_deltas, 0xFF, sizeof(kwk_delta) * nd, e->stream));
  e->n_stages = t->n_stages;
  e->n_classes = t->n_classes;
  e->loaded_table = true;
  if (kwk_status st = build_fsm(e)) return st;
  return refresh_format(e);
}

kwk_status kwk_set_tuning(kwk_engine* e, uint32_t key, uint32_t value) {
  ErrScope es_(e);
  if (!e) return fail(KWK_EINVAL, "null engine");
  if (kwk_status st = set_dev(e)) return st;
  switch (key) {
    case KWK_TUNE_SWEEP16: {  // KWK_SWEEP16_SHAPE(q, persistent, kernel, table)
      const uint32_t q = value & 0xFu, persist = (value >> 4) & 0xFu, kernel = (value >> 8) & 0xFu,
                     table = (value >> 12) & 0xFu;
      if ((q != 1 && q != 2 && q != 4) || persist > 1 || kernel > 2 || table > 1 || (value >> 16))
        return fail(KWK_EINVAL, "KWK_TUNE_SWEEP16: KWK_SWEEP16_SHAPE(q 1|2|4, persistent 0|1, kernel 0|1|2, table 0|1)");
      e->q16 = q;
      e->persist16 = persist != 0;
      e->fsm_kernel = kernel;
      if ((table != 0) != e->use_fsm) {
        e->use_fsm = table != 0;
        HIP_TRY(hipStreamSynchronize(e->stream));
        if (kwk_status st = build_fsm(e)) return st;
      }
      return refresh_format(e);
    }
    case KWK_TUNE_BYTE_STATE:
      if (value > 1) return fail(KWK_EINVAL, "KWK_TUNE_BYTE_STATE: 0 or 1");
      e->byte_tune = value != 0;
      return refresh_format(e);
    case KWK_TUNE_USAGE:
      if (value > 3) return fail(KWK_EINVAL, "KWK_TUNE_USAGE: KWK_USAGE_KEY8 | KWK_USAGE_AGG_FUSED bits");
      e->usage_key8 = (value & KWK_USAGE_KEY8) != 0;
      e->agg_fused = (value & KWK_USAGE_AGG_FUSED) != 0;
      return KWK_OK;
    case KWK_TUNE_STREAM_PRIORITY: {  // the engine's stream re-created at the HIP priority asked for
      if (value > 2) return fail(KWK_EINVAL, "KWK_TUNE_STREAM_PRIORITY: 0 (default), 1 (greatest) or 2 (least)");
      if (kwk_status st = set_dev(e)) return st;
      int least = 0, greatest = 0;
      HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
      HIP_TRY(hipStreamSynchronize(e->stream));
      hipStream_t ns = nullptr;
      HIP_TRY(hipStreamCreateWithPriority(&ns, hipStreamNonBlocking, value == 1 ? greatest : value == 2 ? least : 0));
      HIP_TRY(hipStreamDestroy(e->stream));
      e->stream = ns;
      return KWK_OK;
    }
    case KWK_TUNE_WORD_TILES:
      if (value > 16) return fail(KWK_EINVAL, "KWK_TUNE_WORD_TILES: 0 (per format) or 1..16");
      e->word_tpb = value;
      return KWK_OK;
    case KWK_TUNE_COMPACT_SMALL:
      // each block of the one-launch compaction re-sums every count before its segments: the
      // prefix reads grow with the square of the segments, so the knob stops at 8192 (32 KB of counts)
      if (value > 8192) return fail(KWK_EINVAL, "KWK_TUNE_COMPACT_SMALL: 0..8192");
      e->compact_small = value;
      return KWK_OK;
    case KWK_TUNE_TAIL_HANDBACK:
      if (value > 1) return fail(KWK_EINVAL, "KWK_TUNE_TAIL_HANDBACK: 0 or 1");
      e->tail_hb = value != 0;
      return KWK_OK;
    case KWK_TUNE_FUSE_STEPS:
      if (value > kMaxFuseSteps || (value > 2 && (value & (value - 1u))))
        return fail(KWK_EINVAL, "KWK_TUNE_FUSE_STEPS: 0 / 1 (off), 2 or 4");
      e->fuse_steps = value < 2 ? 1u : value;
      return KWK_OK;
    default:
      return fail(KWK_EINVAL, "unknown tuning key " + std::to_string(key));
  }
}

kwk_status kwk_set_harness(kwk_engine* e, const kwk_harness* h) {
  ErrScope es_(e);
  if (!e || !h) return fail(KWK_EINVAL, "null argument");
  if (kwk_status st = set_dev(e)) return st;
  // the 1-byte ids encode what the harness makes "work": re-read the rows before it changes
  std::vector<uint2> rows;
  if (kwk_status st = read_rows(e, rows)) return st;
  e->harness = *h;
  if (kwk_status st = build_fsm(e)) return st;
  StateFmt nf;
  if (kwk_status st = pick_format(e, rows, nf)) return st;
  return write_rows(e, rows, nf);
}

kwk_status kwk_load(kwk_engine* e, uint32_t n, const kwk_hot* hot, const int64_t* del, const uint32_t* rec,
                    const uint16_t* cls, uint32_t n_records, const kwk_value* records) {
  ErrScope es_(e);
  if (!e || (n && (!hot || !del || !rec || !cls))) return fail(KWK_EINVAL, "null argument");
  if (n > e->capacity) return fail(KWK_ECAP, "n exceeds capacity");
  if (n_records > e->max_records) return fail(KWK_ECAP, "n_records exceeds max_records");
  for (uint32_t i = 0; i < n; ++i) {
    if ((hot[i].sched & KWK_F_HASREC) && rec[i] >= n_records)
      return fail(KWK_EINVAL, "object " + std::to_string(i) + ": record index out of range");
    if (e->loaded_table && cls[i] >= e->n_classes)
      return fail(KWK_EINVAL, "object " + std::to_string(i) + ": class out of range");
  }
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  {  // AoS interchange rows -> device SoA; the delta class lives in the upper half of sched
    std::vector<uint2> st(n);
    std::vector<int64_t> due(n);
    for (uint32_t i = 0; i < n; ++i) {
      st[i] = make_uint2(hot[i].pred, (hot[i].sched & ~KWK_CLASS_MASK) | ((uint32_t)cls[i] << KWK_CLASS_SHIFT));
      if (!fits_fmt(e->fmt, e->n_stages, st[i].x, st[i].y))
        return fail(KWK_EINVAL, "object " + std::to_string(i) + ": pred bits / stage beyond the loaded stage table");
      due[i] = hot[i].due;
    }
    // the loaded objects replace the resident ones: the format follows their words
    StateFmt nf;
    if (kwk_status s2 = pick_format(e, st, nf)) return s2;
    e->fmt = nf;
    const std::vector<uint8_t> raw = pack_words(e, st, e->fmt);
    // on the engine's stream, so that the fold (and every later kernel) is ordered after the
    // uploads whatever a pageable hipMemcpy's return means for its DMA; synchronised before the
    // host buffers go
    HIP_TRY(hipMemcpyAsync(e->d_st, raw.data(), raw.size(), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->d_due, due.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, e->stream));
    if (kwk_status s2 = dw_fold(e, 0, n)) return s2;
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  HIP_TRY(upload(e, e->d_del, del, sizeof(int64_t) * n));
  HIP_TRY(upload(e, e->d_rec, rec, sizeof(uint32_t) * n));
  if (n_records)
    HIP_TRY(upload(e, e->d_values, records, sizeof(kwk_value) * (size_t)n_records * e->value_slots));
  if (n < e->n_active)
    HIP_TRY(hipMemsetAsync((char*)e->d_st + word_bytes(e->fmt) * n, 0, word_bytes(e->fmt) * (size_t)(e->n_active - n), e->stream));
  e->n_active = n;
  return KWK_OK;
}

kwk_status kwk_set_records(kwk_engine* e, uint32_t first, uint32_t n, const kwk_value* records) {
  ErrScope es_(e);
  if (!e || (n && !records)) return fail(KWK_EINVAL, "null argument");
  if ((uint64_t)first + n > e->max_records) return fail(KWK_ECAP, "records exceed max_records");
  if (kwk_status st = set_dev(e)) return st;
  // on the engine's stream (ordered after every enqueued sweep, complete on return): a pageable
  // null-stream copy could still be in flight when the next sweep reads the records
  HIP_TRY(upload(e, e->d_values + (size_t)first * e->value_slots, records, sizeof(kwk_value) * (size_t)n * e->value_slots));
  return KWK_OK;
}

static kwk_status scatter_rows(kwk_engine* e, uint32_t n, const uint32_t* slots, const kwk_hot* hot, const int64_t* del,
                               const uint32_t* rec, const uint16_t* cls, uint32_t mark_dirty);

kwk_status kwk_upsert(kwk_engine* e, uint32_t n, const uint32_t* slots, const kwk_hot* hot, const int64_t* del,
                      const uint32_t* rec, const uint16_t* cls) {
  ErrScope es_(e);
  return scatter_rows(e, n, slots, hot, del, rec, cls, 1u);
}

kwk_status kwk_replace(kwk_engine* e, uint32_t n, const uint32_t* slots, const kwk_hot* hot, const int64_t* del,
                       const uint32_t* rec, const uint16_t* cls) {
  ErrScope es_(e);
  return scatter_rows(e, n, slots, hot, del, rec, cls, 0u);
}

static kwk_status scatter_rows(kwk_engine* e, uint32_t n, const uint32_t* slots, const kwk_hot* hot, const int64_t* del,
                               const uint32_t* rec, const uint16_t* cls, uint32_t mark_dirty) {
  if (!e || (n && (!slots || !hot || !del || !rec || !cls))) return fail(KWK_EINVAL, "null argument");
  if (n == 0) return KWK_OK;
  uint32_t max_slot = 0;
  for (uint32_t j = 0; j < n; ++j) {
    if (slots[j] >= e->capacity) return fail(KWK_ECAP, "slot beyond capacity");
    if (e->loaded_table && cls[j] >= e->n_classes) return fail(KWK_EINVAL, "class out of range");
    if ((hot[j].sched & KWK_F_HASREC) && rec[j] >= e->max_records) return fail(KWK_EINVAL, "record out of range");
    if (!fits_fmt(e->fmt, e->n_stages, hot[j].pred, hot[j].sched))
      return fail(KWK_EINVAL, "pred bits / stage beyond the loaded stage table");
    max_slot = slots[j] > max_slot ? slots[j] : max_slot;
  }
  if (kwk_status st = set_dev(e)) return st;
  {  // the words the scatter writes (1-byte format: they join the dictionary first)
    std::vector<uint2> rows(n);
    for (uint32_t j = 0; j < n; ++j)
      rows[j] = make_uint2(hot[j].pred, (hot[j].sched & ~KWK_CLASS_MASK) | ((uint32_t)cls[j] << KWK_CLASS_SHIFT) |
                                            (mark_dirty ? KWK_F_DIRTY : 0u));
    if (kwk_status st = admit_rows(e, rows)) return st;
  }
  const size_t bytes = (size_t)n * (4 + sizeof(kwk_hot) + 8 + 4 + 2) + 64;
  if (kwk_status st = ensure_stage_buf(e, bytes)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  char* p = (char*)e->d_stage_buf;
  kwk_hot* s_hot = (kwk_hot*)p; p += sizeof(kwk_hot) * n;
  int64_t* s_del = (int64_t*)p; p += 8 * (size_t)n;
  uint32_t* s_slots = (uint32_t*)p; p += 4 * (size_t)n;
  uint32_t* s_rec = (uint32_t*)p; p += 4 * (size_t)n;
  uint16_t* s_cls = (uint16_t*)p;
  HIP_TRY(upload(e, s_hot, hot, sizeof(kwk_hot) * n));
  HIP_TRY(upload(e, s_del, del, 8 * (size_t)n));
  HIP_TRY(upload(e, s_slots, slots, 4 * (size_t)n));
  HIP_TRY(upload(e, s_rec, rec, 4 * (size_t)n));
  HIP_TRY(upload(e, s_cls, cls, 2 * (size_t)n));
  if (max_slot + 1 > e->n_active) {
    HIP_TRY(hipMemsetAsync((char*)e->d_st + word_bytes(e->fmt) * e->n_active, 0,
                           word_bytes(e->fmt) * (size_t)(max_slot + 1 - e->n_active), e->stream));
    e->n_active = max_slot + 1;
  }
  ScatterArgs a{e->d_st, e->fmt, e->d_due, e->d_del, e->d_rec, s_slots, s_hot, s_del, s_rec, s_cls, n, mark_dirty};
  hipLaunchKernelGGL(scatter_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, e->stream, a);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(e->stream));
  return KWK_OK;
}

kwk_status kwk_delete(kwk_engine* e, uint32_t n, const uint32_t* slots) {
  ErrScope es_(e);
  if (!e || (n && !slots)) return fail(KWK_EINVAL, "null argument");
  if (n == 0) return KWK_OK;
  for (uint32_t j = 0; j < n; ++j)
    if (slots[j] >= e->n_active) return fail(KWK_EINVAL, "slot not active");
  if (kwk_status st = set_dev(e)) return st;
  if (kwk_status st = ensure_stage_buf(e, 4 * (size_t)n)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  HIP_TRY(upload(e, e->d_stage_buf, slots, 4 * (size_t)n));
  hipLaunchKernelGGL(delete_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, e->stream, e->d_st,
                     e->fmt, (const uint32_t*)e->d_stage_buf, n);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(e->stream));
  return KWK_OK;
}

kwk_status kwk_retry(kwk_engine* e, int64_t now_ns, uint64_t seed, uint64_t step, uint32_t n, const uint32_t* slots,
                     const kwk_hot* hot, const uint16_t* cls, const uint16_t* stages, const uint32_t* retry_count,
                     const kwk_backoff* backoff) {
  ErrScope es_(e);
  if (!e || !backoff || (n && (!slots || !hot || !cls || !stages || !retry_count)))
    return fail(KWK_EINVAL, "null argument");
  if (n == 0) return KWK_OK;
  for (uint32_t j = 0; j < n; ++j) {
    if (slots[j] >= e->n_active) return fail(KWK_EINVAL, "slot not active");
    if (stages[j] >= e->n_stages) return fail(KWK_EINVAL, "stage out of range");
    if (e->loaded_table && cls[j] >= e->n_classes) return fail(KWK_EINVAL, "class out of range");
    if (!(hot[j].sched & KWK_F_ALIVE)) return fail(KWK_EINVAL, "retried object must be alive");
    if (!fits_fmt(e->fmt, e->n_stages, hot[j].pred, stages[j])) return fail(KWK_EINVAL, "pred bits beyond the stage table");
  }
  if (kwk_status st = set_dev(e)) return st;
  {  // the rows the retry writes (retry_kernel)
    std::vector<uint2> rows(n);
    for (uint32_t j = 0; j < n; ++j)
      rows[j] = make_uint2(hot[j].pred, (hot[j].sched & ~(KWK_CLASS_MASK | 0xFFu | KWK_F_DIRTY)) |
                                            ((uint32_t)cls[j] << KWK_CLASS_SHIFT) | (uint32_t)stages[j]);
    if (kwk_status st = admit_rows(e, rows)) return st;
  }
  const size_t bytes = (size_t)n * (4 + sizeof(kwk_hot) + 2 + 2 + 4) + 64;
  if (kwk_status st = ensure_stage_buf(e, bytes)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  char* p = (char*)e->d_stage_buf;
  kwk_hot* s_hot = (kwk_hot*)p; p += sizeof(kwk_hot) * n;
  uint32_t* s_slots = (uint32_t*)p; p += 4 * (size_t)n;
  uint32_t* s_rc = (uint32_t*)p; p += 4 * (size_t)n;
  uint16_t* s_cls = (uint16_t*)p; p += 2 * (size_t)n;
  uint16_t* s_stg = (uint16_t*)p;
  HIP_TRY(upload(e, s_hot, hot, sizeof(kwk_hot) * n));
  HIP_TRY(upload(e, s_slots, slots, 4 * (size_t)n));
  HIP_TRY(upload(e, s_rc, retry_count, 4 * (size_t)n));
  HIP_TRY(upload(e, s_cls, cls, 2 * (size_t)n));
  HIP_TRY(upload(e, s_stg, stages, 2 * (size_t)n));
  RetryArgs a{e->d_st, e->fmt, e->d_due, s_slots, s_hot, s_cls, s_stg, s_rc, *backoff, n, e->slot_base,
              seed ^ ((uint64_t)e->kind_salt << 32), step, now_ns};
  hipLaunchKernelGGL(retry_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, e->stream, a);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(e->stream));
  return KWK_OK;
}

// persistent grid of the 2-byte sweep: every block slot the occupancy allows on every CU
// (occupancy cached per engine and kernel: engines on different devices or threads never share it)
static uint32_t persist_grid(kwk_engine* e, const void* kernel, uint32_t tiles) {
  int per_cu = 0;
  for (const auto& kv : e->occupancy)
    if (kv.first == kernel) per_cu = kv.second;
  if (per_cu == 0) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, 0) != hipSuccess || per_cu <= 0) per_cu = 1;
    e->occupancy.emplace_back(kernel, per_cu);
  }
  const uint32_t g = (uint32_t)e->n_cus * (uint32_t)per_cu;
  return tiles < g ? tiles : g;
}

static SweepArgs sweep_args(kwk_engine* e, int64_t now_ns, uint64_t seed, uint64_t step, bool fire) {
  SweepArgs a;
  a.st = e->d_st;
  a.due = e->d_due;
  a.del_s = e->d_del;
  a.rec_idx = e->d_rec;
  a.values = e->d_values;
  a.table = e->d_table;
  a.deltas = e->d_deltas;
  a.lut = e->d_lut;
  a.lut_n = e->lut_n;
  a.lut_bytes = e->lut_bytes;
  a.lut_rest = e->lut_rest;
  a.fired = e->d_fired;
  a.wave_counts = e->d_wave_counts;
  a.cum = e->d_cum;
  a.n = e->n_active;
  a.value_slots = e->value_slots;
  a.slot_base = e->slot_base;
  a.key = seed ^ ((uint64_t)e->kind_salt << 32);
  a.step = step;
  a.now = now_ns;
  a.fire = fire ? 1u : 0u;
  a.fmt = e->fmt;
  if (e->fmt.narrow) {  // flag bits sit at fshift in the packed word (sched bits 8..12 there)
    const uint32_t fs = e->fmt.fshift;
    a.raw = RawTest{(KWK_F_MANAGED >> 8) << fs, (KWK_F_DIRTY >> 8) << fs, (KWK_F_ALIVE >> 8) << fs, e->fmt.sshift,
                    e->fmt.smask, e->fmt.none_code, e->harness.terminal_mask & e->fmt.pmask,
                    e->harness.deletion_bit & e->fmt.pmask};
  } else {
    a.raw = RawTest{KWK_F_MANAGED, KWK_F_DIRTY, KWK_F_ALIVE, 0, 0xFFu, KWK_STAGE_NONE, e->harness.terminal_mask,
                    e->harness.deletion_bit};
  }
  a.harness = e->harness;
  if (!fire) a.harness.enable = 0;
  a.fsm = nullptr;
  a.fsm_due = nullptr;
  a.fsm_bits = 0;
  a.dw_epoch_old = e->fmt.epoch;
  a.dw_rebase = 0;
  a.tail = SweepArgs::TailHb{nullptr, nullptr, nullptr, nullptr, 0u, 0u};
  return a;
}

// (re)build the 2-byte format's transition table for the loaded stage table and harness
static kwk_status build_fsm(kwk_engine* e) {
  e->fsm_harness = -1;
  e->byte_ok = false;
  if (!e->fmt.half || !e->loaded_table || !e->use_fsm) return KWK_OK;
  const uint32_t bits = e->fmt.fshift + 5;
  if (bits > 16) return KWK_OK;
  if (e->fsm_bits != bits || !e->d_fsm) {
    if (e->d_fsm) HIP_TRY(hipFree(e->d_fsm));
    if (e->d_fsm_due) HIP_TRY(hipFree(e->d_fsm_due));
    e->d_fsm = nullptr;
    e->d_fsm_due = nullptr;
    HIP_TRY(hipMalloc(&e->d_fsm, sizeof(uint32_t) * (2u << bits)));
    HIP_TRY(hipMalloc(&e->d_fsm_due, sizeof(int64_t) * (2u << bits)));
    e->fsm_bits = bits;
  }
  SweepArgs a = sweep_args(e, 0, 0, 0, true);
  a.fsm_bits = bits;
  const uint32_t n = 2u << bits;
  if (a.harness.enable)
    hipLaunchKernelGGL(fsm_build_kernel<true>, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, e->stream, a, e->d_fsm,
                       e->d_fsm_due);
  else
    hipLaunchKernelGGL(fsm_build_kernel<false>, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, e->stream, a, e->d_fsm,
                       e->d_fsm_due);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->fsm_harness = a.harness.enable ? 1 : 0;
  // host copy: the 1-byte format's closure and id table are derived from it
  e->h_fsm.resize(n);
  e->h_fsm_due.resize(n);
  HIP_TRY(hipMemcpy(e->h_fsm.data(), e->d_fsm, sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(e->h_fsm_due.data(), e->d_fsm_due, sizeof(int64_t) * n, hipMemcpyDeviceToHost));
  e->byte_ok = true;
  return KWK_OK;
}

// a hand-back the sweep may do itself (tail_handback): ring slot `slot` in `mode` (0 / 1); `done`
// tells the caller whether it did (a one-tile-per-block 2-byte table-only sweep) or the caller
// still has to compact
struct TailReq {
  uint32_t slot;
  int mode;
  bool done;
};
static void hb_tail_args(kwk_engine* e, const TailReq& t, SweepArgs& a);

// steps > 1: the 1-byte sweep takes that many steps (now_ns + s * dt_ns) in one launch (step_group;
// step s's segments and counts go to d_firedx / d_countsx[s - 1])
static kwk_status launch_sweep(kwk_engine* e, int64_t now_ns, uint64_t seed, uint64_t step, bool fire,
                               uint32_t steps = 1, int64_t dt_ns = 0, TailReq* tail = nullptr) {
  const bool fuse = steps > 1;
  if (!e) return fail(KWK_EINVAL, "null engine");
  if (!e->loaded_table) return fail(KWK_ESTATE, "kwk_load_stages must be called before kwk_step");
  e->compacted = false;
  e->last_sweep = kwk_sweep_info{};
  e->last_step_no = step + (steps ? steps - 1 : 0);
  if (e->n_active == 0) { e->last_blocks = 0; e->steps += steps; return KWK_OK; }
  SweepArgs a = sweep_args(e, now_ns, seed, step, fire);
  const bool nar = e->fmt.narrow != 0;
  const bool h = a.harness.enable != 0;
  // every sweep emits packed fired segments of 64 * K + 32 words per (tile, wave) and counts one
  // statistics row per block: the per-tile arrays are sized for the smallest tile
  if (e->fmt.half && fire && e->fsm_harness == (h ? 1 : 0)) {
    a.fsm = e->d_fsm;
    a.fsm_due = e->d_fsm_due;
    a.fsm_bits = e->fsm_bits;
  }

  if (e->fmt.byte) {  // 1-byte ids: the table-only id sweep (fire only: kwk_match leaves the format)
    if (!fire) return fail(KWK_ESTATE, "the 1-byte format sweeps with fire only");
    a.fsm = e->d_fsm8;
    a.fsm_due = e->d_fsm8_due;
    a.fsm_bits = e->fsm8_due_any ? kId8AnyDue : 0u;
    constexpr uint32_t tile = kBlock * 16 * kQ8;
    const uint32_t tiles = (e->n_active + tile - 1) / tile;
    const bool s4 = e->n_stages <= 4;  // per-stage counts in scalar registers

    if (fuse) {
      if (!s4 || (steps != 2 && steps != 4)) return fail(KWK_ESTATE, "fused steps: 2 or 4, 1-byte sweep with <= 4 stages");
      for (uint32_t i = 0; i + 1 < steps; ++i) {
        if (!e->d_firedx[i]) return fail(KWK_ESTATE, "fused steps: buffers not allocated");
        a.firedx[i] = e->d_firedx[i];
        a.countsx[i] = e->d_countsx[i];
        a.nowx[i] = now_ns + (int64_t)(i + 1) * dt_ns;
      }
    }
#define K8(P, D)                                                                                        \
  (steps == 4   ? (const void*)sweep8_kernel<P, D, true, 4>                                            \
   : steps == 2 ? (const void*)sweep8_kernel<P, D, true, 2>                                            \
   : s4         ? (const void*)sweep8_kernel<P, D, true> : (const void*)sweep8_kernel<P, D, false>)
    const void* pk = e->fsm_kernel == 2 ? K8(true, 2) : K8(true, 1);
    uint32_t pg = e->persist16 ? persist_grid(e, pk, tiles) : tiles;

    uint32_t blocks = tiles;
    e->last_sweep = kwk_sweep_info{KWK_SWEEP_8, (uint32_t)kQ8, 0, 1, tiles, tiles, a.harness.enable ? 1u : 0u, 0};
    const void* kern = K8(false, 1);
    if (2 * pg <= tiles) {  // else the persistent loop would run about once: one block per tile
      blocks = pg;
      e->last_sweep.persistent = 1;
      e->last_sweep.grid = pg;
      e->last_sweep.depth = e->fsm_kernel;
      kern = pk;
    }
#undef K8
    void* args[] = {&a};
    HIP_TRY(hipLaunchKernel(kern, dim3(blocks), dim3(kBlock), args, 0, e->stream));
    HIP_TRY(hipGetLastError());
    e->last_objs = 16 * kQ8;
    e->last_region_shift = 0;
    e->last_rec = s4 ? kRecId8Half : kRecId8;
    e->last_blocks = tiles;
    e->last_grid = blocks;
    e->cum_rows = blocks > e->cum_rows ? blocks : e->cum_rows;
    e->last_sweep.steps = steps;
    e->steps += steps;
    return KWK_OK;
  }
  if (e->fmt.half) {  // 2-byte words: whole-line write-back sweep
    // small engines (a node kind, the cache-resident configs) take 2048-word tiles so that
    // the grid still spreads over every CU
    uint32_t q16 = e->q16;
    if (q16 > 1 && (e->n_active + kBlock * 8 * q16 - 1) / (kBlock * 8 * q16) < 4u * (uint32_t)e->n_cus) q16 = 1;
    const uint32_t K = 8 * q16, tile = kBlock * K;
    const uint32_t tiles = (e->n_active + tile - 1) / tile;
    uint32_t blocks = tiles;
    const bool lean = a.fsm && e->fsm_kernel;
#define LAUNCH16(HV, QV)                                                                                        \
  do {                                                                                                          \
    const void* pk = lean ? (e->fsm_kernel == 2 ? (const void*)sweep16_fsm_kernel<HV, QV, true, 2>              \
                                                : (const void*)sweep16_fsm_kernel<HV, QV, true, 1>)             \
                          : (const void*)sweep16_kernel<HV, QV, true>;                                          \
    uint32_t pg = e->persist16 ? persist_grid(e, pk, tiles) : tiles;                                            \
    e->last_sweep = kwk_sweep_info{lean ? (uint32_t)KWK_SWEEP_16_FSM : (uint32_t)KWK_SWEEP_16, QV, 0, 1, tiles,    \
                                   tiles, HV ? 1u : 0u, 0};                                                     \
    if (2 * pg > tiles) { /* the persistent loop would run about once: one block per tile */                   \
      if (lean && tail && tiles * 4u <= (uint32_t)e->n_cus && tiles * kWavesPerBlock <= e->compact_small) {    \
        hb_tail_args(e, *tail, a);                                                                              \
        tail->done = true;                                                                                      \
      }                                                                                                         \
      if (lean)                                                                                                 \
        hipLaunchKernelGGL((sweep16_fsm_kernel<HV, QV, false, 1>), dim3(blocks), dim3(kBlock), 0, e->stream, a); \
      else                                                                                                      \
        hipLaunchKernelGGL((sweep16_kernel<HV, QV, false>), dim3(blocks), dim3(kBlock), 0, e->stream, a);     \
    } else {                                                                                                    \
      blocks = pg;                                                                                              \
      e->last_sweep.persistent = 1;                                                                             \
      e->last_sweep.grid = pg;                                                                                  \
      e->last_sweep.depth = lean ? e->fsm_kernel : 1;                                                           \
      if (lean && e->fsm_kernel == 2)                                                                           \
        hipLaunchKernelGGL((sweep16_fsm_kernel<HV, QV, true, 2>), dim3(blocks), dim3(kBlock), 0, e->stream, a); \
      else if (lean)                                                                                            \
        hipLaunchKernelGGL((sweep16_fsm_kernel<HV, QV, true, 1>), dim3(blocks), dim3(kBlock), 0, e->stream, a); \
      else                                                                                                      \
        hipLaunchKernelGGL((sweep16_kernel<HV, QV, true>), dim3(blocks), dim3(kBlock), 0, e->stream, a);      \
    }                                                                                                           \
  } while (0)
    if (q16 == 4) {
      if (h) LAUNCH16(true, 4); else LAUNCH16(false, 4);
    } else if (q16 == 1) {
      if (h) LAUNCH16(true, 1); else LAUNCH16(false, 1);
    } else {
      if (h) LAUNCH16(true, 2); else LAUNCH16(false, 2);
    }
#undef LAUNCH16
    e->last_objs = K;
    e->last_region_shift = 0;
    e->last_rec = kRecSlot;
    HIP_TRY(hipGetLastError());
    e->last_blocks = tiles;  // fired segments / wave counts are per (tile, wave)
    e->last_grid = blocks;
    e->cum_rows = blocks > e->cum_rows ? blocks : e->cum_rows;
    ++e->steps;
    return KWK_OK;
  }
  // 4- / 8-byte words: whole-line write-back word sweep, one block per tile
  const bool dw = e->fmt.dw != 0;
  const uint32_t K = dw ? (uint32_t)kQWD * 2u : (uint32_t)kQW * (nar ? 4u : 2u);
  const uint32_t tile = kBlock * K;
  const uint32_t tiles = (e->n_active + tile - 1) / tile;
  // tiles per workgroup (the next tile's stream in flight while one is worked: 8 for the fused
  // records, 4 for the 4-byte words, r3r), but at least ~5 workgroups per CU
  // (an explicit KWK_TUNE_WORD_TILES is taken as it is: the parity tests loop small engines)
  const uint32_t tpb = e->word_tpb ? e->word_tpb : dw ? 8u : 4u;
  const uint32_t blocks = e->word_tpb ? (tiles + tpb - 1) / tpb
                                      : std::min(tiles, std::max((tiles + tpb - 1) / tpb, (uint32_t)e->n_cus * 5u));
  if (dw) {
    // the fused records' epoch follows the clock: re-encoded (inside this sweep) once now is
    // more than 2^34 ns (~17 s) past it or before it, so that due times up to ~51 s ahead of now
    // stay in the 2^36 ns window
    // (the host's epoch moves only once the re-encoding sweep is enqueued, below)
    const int64_t e0 = e->fmt.epoch;
    if (now_ns < e0 || (uint64_t)now_ns - (uint64_t)e0 > kDwRebase) {
      a.fmt.epoch = now_ns;
      a.dw_rebase = 1;
    }
    if (h) hipLaunchKernelGGL((sweepw_kernel<true, 8, true>), dim3(blocks), dim3(kBlock), 0, e->stream, a);
    else hipLaunchKernelGGL((sweepw_kernel<false, 8, true>), dim3(blocks), dim3(kBlock), 0, e->stream, a);
  } else if (nar) {
    if (h) hipLaunchKernelGGL((sweepw_kernel<true, 4>), dim3(blocks), dim3(kBlock), 0, e->stream, a);
    else hipLaunchKernelGGL((sweepw_kernel<false, 4>), dim3(blocks), dim3(kBlock), 0, e->stream, a);
  } else {
    if (h) hipLaunchKernelGGL((sweepw_kernel<true, 8>), dim3(blocks), dim3(kBlock), 0, e->stream, a);
    else hipLaunchKernelGGL((sweepw_kernel<false, 8>), dim3(blocks), dim3(kBlock), 0, e->stream, a);
  }
  e->last_sweep = kwk_sweep_info{dw ? (uint32_t)KWK_SWEEP_WD : nar ? (uint32_t)KWK_SWEEP_W4 : (uint32_t)KWK_SWEEP_W8,
                                 (uint32_t)(dw ? kQWD : kQW), blocks < tiles ? 1u : 0u,
                                 blocks < tiles ? 2u : 1u /* the next tile in flight */, blocks, tiles, h ? 1u : 0u, 0};
  e->last_objs = K;
  e->last_region_shift = 2;  // log2(kWavesPerBlock): records carry tile-relative slots
  e->last_rec = kRecSlot;
  static_assert(kWavesPerBlock == 4, "region shift");
  HIP_TRY(hipGetLastError());
  if (dw) e->fmt.epoch = a.fmt.epoch;  // the records now hold due times relative to it
  e->last_blocks = tiles;  // fired segments / wave counts are per (tile, wave)
  e->last_grid = blocks;
  e->cum_rows = blocks > e->cum_rows ? blocks : e->cum_rows;
  ++e->steps;
  return KWK_OK;
}

kwk_status kwk_step(kwk_engine* e, int64_t now_ns, uint64_t seed, uint64_t step) {
  ErrScope es_(e);
  return launch_sweep(e, now_ns, seed, step, true);
}

kwk_status kwk_match(kwk_engine* e, int64_t now_ns, uint64_t seed, uint64_t step) {
  ErrScope es_(e);
  if (!e) return fail(KWK_EINVAL, "null engine");
  if (kwk_status st = set_dev(e)) return st;
  if (kwk_status st = leave_byte(e)) return st;  // match-only runs the general word sweep
  return launch_sweep(e, now_ns, seed, step, false);
}

kwk_status kwk_sync(kwk_engine* e) {
  ErrScope es_(e);
  if (!e) return fail(KWK_EINVAL, "null engine");
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  return KWK_OK;
}

// fired hand-back on the device: per-(tile, wave) counts -> exclusive scan -> dense list in the
// next ring slot, its length at the slot's offsets[0] (enqueue only)
// mode: 0 kwk_fired_rec, 1 packed 4-byte records, 2 the 2-byte records where the sweep wrote them
// (else the 4-byte packed ones), 3 the bitmap hand-back (likewise)

// the ring slot `k` compactions after the engine's last list
static uint32_t hb_next(const kwk_engine* e, uint32_t k = 1) { return (e->hb_cur + k) % (uint32_t)e->hb.size(); }

// bytes of a slot's list in `mode` at the engine's capacity (the bitmap hand-back: at most
// 1 + 8 + 64 + 128 words per 2048-slot segment)
static size_t hb_list_bytes(const kwk_engine* e, int mode) {
  if (mode == 3) return 4u * ((size_t)e->n_blocks_cap * kWavesPerBlock * 201u + 64u);
  const size_t rb = mode == 2 ? 2u : mode == 1 ? 4u : sizeof(kwk_fired_rec);
  return rb * (size_t)e->capacity + 64u;
}

// slot i made ready for a compaction in `mode` on `stream`: the copy stream's last copy out of it
// waited for on the device, its buffers (re)sized
static kwk_status hb_prepare(kwk_engine* e, uint32_t i, int mode, hipStream_t stream) {
  kwk_engine::HbSlot& h = e->hb[i];
  if (h.copy_pending) {
    HIP_TRY(hipStreamWaitEvent(stream, h.ev_copied, 0));
    h.copy_pending = false;
  }
  const size_t need = hb_list_bytes(e, mode);
  if (h.list_bytes < need) {
    if (h.list) HIP_TRY(hipFree(h.list));  // (synchronises the device: no copy or kernel still reads it)
    h.list = nullptr;
    h.list_bytes = 0;
    HIP_TRY(hipMalloc(&h.list, need));
    h.list_bytes = need;
  }
  if (!h.offsets) {
    const size_t n_waves = (size_t)e->n_blocks_cap * kWavesPerBlock;
    HIP_TRY(hipMalloc((void**)&h.offsets, sizeof(uint32_t) * (n_waves + 4)));
    HIP_TRY(hipMalloc((void**)&h.groups, sizeof(uint32_t) * (n_waves / kScanGroup + 4)));
    HIP_TRY(hipMalloc((void**)&h.tot, 64));
    HIP_TRY(hipMalloc((void**)&h.counts, sizeof(uint32_t) * (n_waves + 4)));
  }
  if (e->hb_track && !h.ev_done) HIP_TRY(hipEventCreateWithFlags(&h.ev_done, hipEventDisableTiming));
  return KWK_OK;
}

// slot i now holds step `step`'s list (written by the compaction just enqueued on `stream`)
static kwk_status hb_commit(kwk_engine* e, uint32_t i, uint64_t step, int mode, uint32_t n_segs, int done_slot,
                            hipStream_t stream, bool record) {
  kwk_engine::HbSlot& h = e->hb[i];
  h.valid = true;
  h.step = step;
  h.mode = mode;
  h.n_segs = n_segs;
  h.region_slots = n_segs ? 64u * e->last_objs << e->last_region_shift : 0u;
  h.done_slot = done_slot;
  e->hb_cur = i;
  if (e->hb_track && record) HIP_TRY(hipEventRecord(h.ev_done, stream));
  return KWK_OK;
}

static void hb_args(const kwk_engine* e, uint32_t i, int mode, CompactArgs& a) {
  const kwk_engine::HbSlot& h = e->hb[i];
  a.out = reinterpret_cast<kwk_fired_rec*>(h.list);
  a.offsets = h.offsets;
  a.group_tot = h.groups;
  a.counts_out = mode == 2 ? h.counts : nullptr;
  a.host_len = e->hb_track ? e->h_len_dev + 2u * i : nullptr;
  a.n_segs = e->last_blocks * kWavesPerBlock;
  a.seg_region_shift = e->last_region_shift;
  a.region_slots = 64u * e->last_objs << e->last_region_shift;
  a.stride = 64u * e->last_objs + 32u;
}

static void hb_tail_args(kwk_engine* e, const TailReq& t, SweepArgs& a) {
  const kwk_engine::HbSlot& h = e->hb[t.slot];
  if (++e->tail_seq == 0) e->tail_seq = 1;  // 0 never tags a launch (the status words start at 0)
  a.tail = SweepArgs::TailHb{h.list, h.offsets, e->hb_track ? e->h_len_dev + 2u * t.slot : nullptr, e->d_tail_status,
                             e->tail_seq, t.mode == 1 ? 1u : 0u};
}

static kwk_status enqueue_compact(kwk_engine* e, int mode = 0, hipStream_t stream = nullptr) {
  if (!stream) stream = e->stream;
  const uint32_t n_waves = e->last_blocks * kWavesPerBlock;
  if ((mode == 2 || mode == 3) && e->last_rec != kRecId8Half) mode = 1;
  const bool packed = mode == 1;
  const uint32_t i = hb_next(e);
  if (kwk_status st = hb_prepare(e, i, mode, stream)) return st;
  kwk_engine::HbSlot& h = e->hb[i];
  e->compacted = true;
  e->compacted_packed = packed;
  e->compacted_16 = mode == 2;
  e->compacted_bits = mode == 3;
  if (n_waves == 0) {  // nothing swept: the device list is empty (never the previous step's count)
    HIP_TRY(hipMemsetAsync(h.offsets, 0, sizeof(uint32_t), stream));
    HIP_TRY(hipMemsetAsync(h.tot, 0, 2 * sizeof(uint32_t), stream));
    if (e->hb_track) HIP_TRY(hipMemsetAsync(e->h_len_dev + 2u * i, 0, 2 * sizeof(uint32_t), stream));
    return hb_commit(e, i, e->last_step_no, mode, 0, (int)i, stream, true);
  }
  const uint32_t blocks = (n_waves + kSegsPerBlock - 1) / kSegsPerBlock;
  CompactArgs a;
  a.fired32 = reinterpret_cast<const uint32_t*>(e->d_fired);
  a.counts = e->d_wave_counts;
  hb_args(e, i, mode, a);
  const int rk = e->last_rec;
  void* args[] = {&a};
  const uint32_t groups = (n_waves + kScanGroup - 1) / kScanGroup;
  if (mode == 2 && n_waves <= e->compact_small) {
    hipLaunchKernelGGL(compact16_small_kernel, dim3((n_waves + kSmall16Spb - 1) / kSmall16Spb), dim3(kBlock), 0, stream, a);
  } else if (mode == 3 && n_waves <= e->compact_small) {
    hipLaunchKernelGGL(bits_size_kernel, dim3(blocks), dim3(kBlock), 0, stream, a, e->d_bits_wc, e->d_bits_bsum);
    hipLaunchKernelGGL(bits_write_kernel<true>, dim3(blocks), dim3(kBlock), 0, stream, a, e->d_bits_wc, e->d_bits_bsum,
                       h.tot);
  } else if (mode != 2 && mode != 3 && n_waves <= e->compact_small) {  // one launch: prefix sums inside the expansion
    const void* k = packed ? (rk == kRecId8Half ? (const void*)compact_small_kernel<kRecId8Half, true>
                              : rk == kRecId8   ? (const void*)compact_small_kernel<kRecId8, true>
                                                : (const void*)compact_small_kernel<kRecSlot, true>)
                           : (rk == kRecId8Half ? (const void*)compact_small_kernel<kRecId8Half>
                              : rk == kRecId8   ? (const void*)compact_small_kernel<kRecId8>
                                                : (const void*)compact_small_kernel<kRecSlot>);
    HIP_TRY(hipLaunchKernel(k, dim3(blocks), dim3(kBlock), args, 0, stream));
  } else if (mode == 3) {
    hipLaunchKernelGGL(bits_size_kernel, dim3(blocks), dim3(kBlock), 0, stream, a, e->d_bits_wc, e->d_bits_bsum);
    hipLaunchKernelGGL(seg_scan_kernel, dim3(groups), dim3(kBlock), 0, stream, e->d_bits_wc, n_waves, h.offsets, h.groups);
    hipLaunchKernelGGL(bits_write_kernel<false>, dim3(blocks), dim3(kBlock), 0, stream, a, e->d_bits_wc, e->d_bits_bsum,
                       h.tot);
  } else {
    hipLaunchKernelGGL(seg_scan_kernel, dim3(groups), dim3(kBlock), 0, stream, e->d_wave_counts, n_waves, h.offsets,
                       h.groups);
    if (mode == 2) {
      constexpr uint32_t W16 = kCompact16Spw;
      hipLaunchKernelGGL(compact16_kernel<W16>, dim3((n_waves + W16 * kWavesPerBlock - 1) / (W16 * kWavesPerBlock)),
                         dim3(kBlock), 0, stream, a);
    } else {
      constexpr uint32_t W = kCompactSpw;
      const void* k = packed ? (rk == kRecId8Half ? (const void*)compact_kernel<kRecId8Half, true, W>
                                : rk == kRecId8   ? (const void*)compact_kernel<kRecId8, true, W>
                                                  : (const void*)compact_kernel<kRecSlot, true, W>)
                             : (rk == kRecId8Half ? (const void*)compact_kernel<kRecId8Half, false, W>
                                : rk == kRecId8   ? (const void*)compact_kernel<kRecId8, false, W>
                                                  : (const void*)compact_kernel<kRecSlot, false, W>);
      const uint32_t eblocks = (n_waves + W * kWavesPerBlock - 1) / (W * kWavesPerBlock);
      HIP_TRY(hipLaunchKernel(k, dim3(eblocks), dim3(kBlock), args, 0, stream));
    }
  }
  HIP_TRY(hipGetLastError());
  return hb_commit(e, i, e->last_step_no, mode, n_waves, (int)i, stream, true);
}

kwk_status kwk_fired_compact(kwk_engine* e) {
  ErrScope es_(e);
  if (!e) return fail(KWK_EINVAL, "null engine");
  if (kwk_status st = set_dev(e)) return st;
  return enqueue_compact(e);
}

static kwk_status packed_ok(const kwk_engine* e) {
  if (e->capacity > kPackedSlots) return fail(KWK_ECAP, "packed fired records hold 27-bit slots: engine capacity > 2^27");
  return KWK_OK;
}

kwk_status kwk_fired_compact_packed(kwk_engine* e) {
  ErrScope es_(e);
  if (!e) return fail(KWK_EINVAL, "null engine");
  if (kwk_status st = packed_ok(e)) return st;
  if (kwk_status st = set_dev(e)) return st;
  return enqueue_compact(e, 1);
}

kwk_status kwk_fired_packed_device(kwk_engine* e, const uint32_t** recs, const uint32_t** count) {
  ErrScope es_(e);
  if (!e || !recs || !count) return fail(KWK_EINVAL, "null argument");
  if (!e->compacted || !e->compacted_packed) return fail(KWK_ESTATE, "kwk_fired_compact_packed must follow kwk_step");
  *recs = reinterpret_cast<const uint32_t*>(e->hb[e->hb_cur].list);
  *count = e->hb[e->hb_cur].offsets;
  return KWK_OK;
}

// the length (or the bitmap hand-back's {words, records}) of the engine's last list (synchronises)
static kwk_status hb_len(kwk_engine* e, uint32_t* t) {
  const kwk_engine::HbSlot& h = e->hb[e->hb_cur];
  HIP_TRY(hipMemcpyAsync(t, h.mode == 3 ? h.tot : h.offsets, h.mode == 3 ? 2 * sizeof(uint32_t) : sizeof(uint32_t),
                         hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return KWK_OK;
}

kwk_status kwk_fired_packed(kwk_engine* e, uint32_t* out, uint32_t cap, uint32_t* n_out) {
  ErrScope es_(e);
  if (!e || !n_out) return fail(KWK_EINVAL, "null argument");
  if (kwk_status st = packed_ok(e)) return st;
  if (kwk_status st = set_dev(e)) return st;
  const uint32_t n_waves = e->last_blocks * kWavesPerBlock;
  if (n_waves == 0) { *n_out = 0; return KWK_OK; }
  if (!e->compacted || !e->compacted_packed)
    if (kwk_status st = enqueue_compact(e, 1)) return st;
  uint32_t total = 0;
  if (kwk_status st = hb_len(e, &total)) return st;
  *n_out = total;
  if (!out || total == 0) return KWK_OK;
  if (total > cap) return fail(KWK_ECAP, "fired buffer too small: need " + std::to_string(total));
  HIP_TRY(hipMemcpyAsync(out, e->hb[e->hb_cur].list, sizeof(uint32_t) * total, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return KWK_OK;
}

static int compact_mode(uint32_t compact) {
  return compact == KWK_COMPACT_BITS ? 3 : compact == KWK_COMPACT_PACKED16 ? 2 : compact == KWK_COMPACT_PACKED ? 1 : 0;
}

kwk_status kwk_fired_compact_bits(kwk_engine* e) {
  ErrScope es_(e);
  if (!e) return fail(KWK_EINVAL, "null engine");
  if (kwk_status st = set_dev(e)) return st;
  return enqueue_compact(e, 3);
}

kwk_status kwk_fired_bits(kwk_engine* e, uint32_t* out, uint64_t cap_words, uint64_t* n_words, uint32_t* n_records,
                          uint32_t* n_segs, uint32_t* region_slots) {
  ErrScope es_(e);
  if (!e || !n_words || !n_records || !n_segs || !region_slots) return fail(KWK_EINVAL, "null argument");
  if (kwk_status st = set_dev(e)) return st;
  const uint32_t n_waves = e->last_blocks * kWavesPerBlock;
  *n_segs = n_waves;
  *region_slots = 64u * e->last_objs << e->last_region_shift;
  *n_words = 0;
  *n_records = 0;
  if (n_waves == 0) return KWK_OK;
  if (!e->compacted || !e->compacted_bits) {
    if (e->last_rec != kRecId8Half)
      return fail(KWK_ESTATE, "the bitmap hand-back is the 1-byte sweep's with at most 4 stages: use kwk_fired_packed");
    if (kwk_status st = enqueue_compact(e, 3)) return st;
  }
  uint32_t t[2] = {0, 0};
  if (kwk_status st = hb_len(e, t)) return st;
  *n_words = t[0];
  *n_records = t[1];
  if (!out) return KWK_OK;
  if (t[0] > cap_words) return fail(KWK_ECAP, "fired buffer too small: need " + std::to_string(t[0]) + " words");
  HIP_TRY(hipMemcpyAsync(out, e->hb[e->hb_cur].list, sizeof(uint32_t) * (size_t)t[0], hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return KWK_OK;
}

kwk_status kwk_fired_compact_packed16(kwk_engine* e) {
  ErrScope es_(e);
  if (!e) return fail(KWK_EINVAL, "null engine");
  if (kwk_status st = set_dev(e)) return st;
  return enqueue_compact(e, 2);
}

kwk_status kwk_fired_packed16(kwk_engine* e, uint16_t* out, uint32_t cap, uint32_t* n_out, uint32_t* seg_counts,
                              uint32_t seg_cap, uint32_t* n_segs, uint32_t* region_slots) {
  ErrScope es_(e);
  if (!e || !n_out || !n_segs || !region_slots) return fail(KWK_EINVAL, "null argument");
  if (kwk_status st = set_dev(e)) return st;
  const uint32_t n_waves = e->last_blocks * kWavesPerBlock;
  *n_segs = n_waves;
  *region_slots = 64u * e->last_objs << e->last_region_shift;
  if (n_waves == 0) { *n_out = 0; return KWK_OK; }
  if (!e->compacted || !e->compacted_16) {
    if (e->last_rec != kRecId8Half)
      return fail(KWK_ESTATE, "2-byte records are the 1-byte sweep's with at most 4 stages: use kwk_fired_packed");
    if (kwk_status st = enqueue_compact(e, 2)) return st;
  }
  uint32_t total = 0;
  if (kwk_status st = hb_len(e, &total)) return st;
  *n_out = total;
  if (!out && !seg_counts) return KWK_OK;
  if (out && total > cap) return fail(KWK_ECAP, "fired buffer too small: need " + std::to_string(total));
  if (seg_counts && n_waves > seg_cap) return fail(KWK_ECAP, "segment buffer too small: need " + std::to_string(n_waves));
  const kwk_engine::HbSlot& h = e->hb[e->hb_cur];
  if (out && total) HIP_TRY(hipMemcpyAsync(out, h.list, sizeof(uint16_t) * total, hipMemcpyDeviceToHost, e->stream));
  if (seg_counts)
    HIP_TRY(hipMemcpyAsync(seg_counts, h.counts, sizeof(uint32_t) * n_waves, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return KWK_OK;
}

// one step of kwk_step_n / _pair: the sweep (bracketed by events ev_a, ev_a + 1 when ev_a >= 0),
// then the hand-back into the next ring slot.  (The hand-back of step k on a side stream
// overlapping the sweep of step k + 1, segments double-buffered, measured slower: 80.1-80.8 vs
// 78.4-78.7 us per C5 step, the persistent sweep holding the CUs the two latency-bound launches
// then wait for; r5p / r5r.  Round 5's folded hand-back — the next sweep copying a step's 2-byte
// list — is superseded by fused steps at the shard size and was removed in round 6.)
// the sweep of one step and its hand-back in `mode` (< 0: none) into the next ring slot — inside
// the sweep (tail_handback) when it is a one-tile-per-block 2-byte table-only sweep, else by
// enqueue_compact.  ev_a >= 0: events ev_a, ev_a + 1 bracket the sweep launch
static kwk_status sweep_compact(kwk_engine* e, int64_t now, uint64_t seed, uint64_t step, int mode, int ev_a = -1) {
  TailReq tr{0u, mode == 0 ? 0 : 1, false};  // a 2-byte sweep's records: the 2-byte / bitmap modes fall to packed
  const bool try_tail = mode >= 0 && e->tail_hb && e->fmt.half && !e->fmt.byte && e->loaded_table;
  if (try_tail) {
    tr.slot = hb_next(e);
    if (kwk_status st = hb_prepare(e, tr.slot, tr.mode, e->stream)) return st;
  }
  if (ev_a >= 0)
    if (kwk_status st = kwk_event_record(e, (uint32_t)ev_a)) return st;
  if (kwk_status st = launch_sweep(e, now, seed, step, true, 1, 0, try_tail ? &tr : nullptr)) return st;
  if (ev_a >= 0)
    if (kwk_status st = kwk_event_record(e, (uint32_t)ev_a + 1u)) return st;
  if (mode < 0) return KWK_OK;
  if (tr.done) {
    e->compacted = true;
    e->compacted_packed = tr.mode == 1;
    e->compacted_16 = false;
    e->compacted_bits = false;
    return hb_commit(e, tr.slot, e->last_step_no, tr.mode, e->last_blocks * kWavesPerBlock, (int)tr.slot, e->stream,
                     true);
  }
  return enqueue_compact(e, mode);
}

static kwk_status step_one(kwk_engine* e, int64_t now, uint64_t seed, uint64_t step, uint32_t compact, int ev_a = -1) {
  return sweep_compact(e, now, seed, step, compact ? compact_mode(compact) : -1, ev_a);
}

// several steps in one sweep launch (KWK_TUNE_FUSE_STEPS): a 1-byte engine whose table writes no
// due time (objects then step independently of the clock except through due times already
// queued, which each step tests at its own now) and whose records are the 2-byte ones.  The steps
// a launch takes: 4, 2 or 1, at most the tuning's and the call's steps left, and at most one event
// sample per launch (ev_every 2 or 3: pairs; 1: none fused)
static uint32_t fuse_group(const kwk_engine* e, uint32_t left, uint32_t ev_every) {
  if (e->fuse_steps < 2 || !e->fmt.byte || e->n_stages > 4 || e->fsm8_due_any || !e->loaded_table || ev_every == 1)
    return 1;
  uint32_t m = e->fuse_steps;
  while (ev_every && m > 2 && m > ev_every) m >>= 1;  // at most one event sample per launch
  while (m > left) m >>= 1;
  return m ? m : 1;
}

// steps k .. k + m - 1 of kwk_step_n / _pair (now, now + dt, ...) in one launch, then every step's
// hand-back into a ring slot of its own (the next m slots, in step order, so each step's list stays
// readable by kwk_fired_fetch_step): step 0's segments in d_fired, step s's in d_firedx[s - 1],
// rotated so that the last step's stay in d_fired / d_wave_counts (the engine's last step); ev_a
// brackets the launch (the sample of whichever step it is)
static kwk_status step_group(kwk_engine* e, uint32_t m, int64_t now, int64_t dt, uint64_t seed, uint64_t step,
                             uint32_t compact, int ev_a) {
  for (uint32_t i = 0; i + 1 < m; ++i) {
    if (e->d_firedx[i]) continue;
    const size_t n_waves = (size_t)e->n_blocks_cap * kWavesPerBlock;
    HIP_TRY(hipMalloc((void**)&e->d_firedx[i], sizeof(kwk_fired_rec) * ((size_t)e->n_blocks_cap * kBlock * kMinObjPerThread +
                                                                         (size_t)kBlock * kMaxObjPerThread)));
    HIP_TRY(hipMalloc((void**)&e->d_countsx[i], sizeof(uint32_t) * (n_waves + 4)));
  }
  if (ev_a >= 0)
    if (kwk_status st = kwk_event_record(e, (uint32_t)ev_a)) return st;
  if (kwk_status st = launch_sweep(e, now, seed, step, true, m, dt)) return st;
  if (ev_a >= 0)
    if (kwk_status st = kwk_event_record(e, (uint32_t)ev_a + 1u)) return st;
  const uint32_t n_waves = e->last_blocks * kWavesPerBlock;
  if (compact == KWK_COMPACT_PACKED16 && e->last_rec == kRecId8Half && n_waves) {
    // the steps' 2-byte hand-backs in one launch (two: scan + expansion, past compact_small
    // segments), blockIdx.y = the step, step i's list into ring slot hb_next(i + 1)
    CompactArgs4 c4;
    for (uint32_t i = 0; i < m; ++i)
      if (kwk_status st = hb_prepare(e, hb_next(e, i + 1), 2, e->stream)) return st;
    for (uint32_t i = 0; i < m; ++i) {
      CompactArgs& a = c4.a[i];
      a.fired32 = reinterpret_cast<const uint32_t*>(i ? e->d_firedx[i - 1] : e->d_fired);
      a.counts = i ? e->d_countsx[i - 1] : e->d_wave_counts;
      hb_args(e, hb_next(e, i + 1), 2, a);
    }
    const uint32_t blocks = (n_waves + kSegsPerBlock - 1) / kSegsPerBlock;
    if (n_waves <= e->compact_small) {
      hipLaunchKernelGGL(compact16_small_multi_kernel, dim3((n_waves + kSmall16Spb - 1) / kSmall16Spb, m), dim3(kBlock), 0,
                         e->stream, c4);
    } else {
      constexpr uint32_t W16 = kCompact16Spw;
      hipLaunchKernelGGL(seg_scan_multi_kernel, dim3((n_waves + kScanGroup - 1) / kScanGroup, m), dim3(kBlock), 0,
                         e->stream, c4);
      hipLaunchKernelGGL(compact16_multi_kernel<W16>, dim3((n_waves + W16 * kWavesPerBlock - 1) / (W16 * kWavesPerBlock), m),
                         dim3(kBlock), 0, e->stream, c4);
    }
    HIP_TRY(hipGetLastError());
    for (uint32_t i = 1; i < m; ++i) {  // the last step's segments and counts where the engine reads them
      std::swap(e->d_fired, e->d_firedx[i - 1]);
      std::swap(e->d_wave_counts, e->d_countsx[i - 1]);
    }
    const uint32_t last = hb_next(e, m);
    for (uint32_t i = 0; i < m; ++i) {
      const uint32_t slot = hb_next(e, 1);  // hb_commit advances hb_cur: slots in step order
      if (kwk_status st = hb_commit(e, slot, step + i, 2, n_waves, (int)last, e->stream, i + 1 == m)) return st;
    }
    e->compacted = true;
    e->compacted_packed = false;
    e->compacted_16 = true;
    e->compacted_bits = false;
    return KWK_OK;
  }
  for (uint32_t i = 0; i < m; ++i) {
    if (i) {
      std::swap(e->d_fired, e->d_firedx[i - 1]);
      std::swap(e->d_wave_counts, e->d_countsx[i - 1]);
      e->compacted = false;
    }
    if (compact) {
      e->last_step_no = step + i;  // the tag of this step's list
      if (kwk_status st = enqueue_compact(e, compact_mode(compact))) return st;
    }
  }
  e->last_step_no = step + m - 1;
  return KWK_OK;
}

// the event sample of step j (ev_every > 0), or -1; of a launch of steps j .. j + m - 1: the first
static int ev_of(uint32_t ev_every, uint32_t j) {
  return ev_every && j % ev_every == 0 ? (int)(2u * (j / ev_every)) : -1;
}
static int ev_of_group(uint32_t ev_every, uint32_t j, uint32_t m) {
  for (uint32_t i = 0; i < m; ++i)
    if (ev_of(ev_every, j + i) >= 0) return ev_of(ev_every, j + i);
  return -1;
}

kwk_status kwk_step_n(kwk_engine* e, uint32_t n, int64_t now0_ns, int64_t dt_ns, uint64_t seed, uint64_t step0,
                      uint32_t compact, uint32_t ev_every, uint32_t ev_j0) {
  ErrScope es_(e);
  if (!e) return fail(KWK_EINVAL, "null engine");
  if (compact == KWK_COMPACT_PACKED || compact == KWK_COMPACT_PACKED16)
    if (kwk_status st = packed_ok(e)) return st;
  if (kwk_status st = set_dev(e)) return st;
  for (uint32_t k = 0; k < n;) {
    const uint32_t j = ev_j0 + k;
    const uint32_t m = fuse_group(e, n - k, ev_every);
    if (m > 1) {
      if (kwk_status st = step_group(e, m, now0_ns + (int64_t)k * dt_ns, dt_ns, seed, step0 + k, compact,
                                     ev_of_group(ev_every, j, m)))
        return st;
      k += m;
      continue;
    }
    if (kwk_status st = step_one(e, now0_ns + (int64_t)k * dt_ns, seed, step0 + k, compact, ev_of(ev_every, j)))
      return st;
    ++k;
  }
  return KWK_OK;
}

kwk_status kwk_step_n_pair(kwk_engine* e, kwk_engine* other, uint32_t n, int64_t now0_ns, int64_t dt_ns, uint64_t seed,
                           uint64_t step0, uint32_t compact, uint32_t ev_every, uint32_t ev_j0) {
  ErrScope es_(e);
  if (!e || !other) return fail(KWK_EINVAL, "null engine");
  if (e == other) return fail(KWK_EINVAL, "the two engines must differ");
  if (e->device != other->device) return fail(KWK_EINVAL, "the two engines are on different devices");
  if (compact == KWK_COMPACT_PACKED || compact == KWK_COMPACT_PACKED16) {
    if (kwk_status st = packed_ok(e)) return st;
    if (other->capacity > kPackedSlots) return fail(KWK_ECAP, "packed fired records hold 27-bit slots: other engine > 2^27");
  }
  if (kwk_status st = set_dev(e)) return st;
  for (uint32_t k = 0; k < n;) {
    const uint32_t j = ev_j0 + k;
    const int64_t now = now0_ns + (int64_t)k * dt_ns;
    // the first engine's fused steps (or one), the other's as many right behind (its own stream)
    const uint32_t m = fuse_group(e, n - k, ev_every);
    if (m > 1) {
      if (kwk_status st = step_group(e, m, now, dt_ns, seed, step0 + k, compact, ev_of_group(ev_every, j, m))) return st;
    } else if (kwk_status st = step_one(e, now, seed, step0 + k, compact, ev_of(ev_every, j))) {
      return st;
    }
    // the other engine's step(s) right behind (its own stream): both chains start together
    for (uint32_t i = 0; i < m; ++i)
      if (kwk_status st = step_one(other, now + (int64_t)i * dt_ns, seed, step0 + k + i, compact, -1)) return st;
    k += m;
  }
  return KWK_OK;
}

kwk_status kwk_fired_device(kwk_engine* e, const kwk_fired_rec** recs, const uint32_t** count) {
  ErrScope es_(e);
  if (!e || !recs || !count) return fail(KWK_EINVAL, "null argument");
  if (!e->compacted || e->compacted_packed || e->compacted_16 || e->compacted_bits)
    return fail(KWK_ESTATE, "kwk_fired_compact must follow kwk_step");
  *recs = reinterpret_cast<const kwk_fired_rec*>(e->hb[e->hb_cur].list);
  *count = e->hb[e->hb_cur].offsets;
  return KWK_OK;
}

kwk_status kwk_fired(kwk_engine* e, kwk_fired_rec* out, uint32_t cap, uint32_t* n_out) {
  ErrScope es_(e);
  if (!e || !n_out) return fail(KWK_EINVAL, "null argument");
  if (kwk_status st = set_dev(e)) return st;
  const uint32_t n_waves = e->last_blocks * kWavesPerBlock;
  if (n_waves == 0) { *n_out = 0; return KWK_OK; }
  if (!e->compacted || e->compacted_packed || e->compacted_16 || e->compacted_bits)  // the segments are intact: expand them
    if (kwk_status st = enqueue_compact(e)) return st;
  uint32_t total = 0;
  if (kwk_status st = hb_len(e, &total)) return st;
  *n_out = total;
  if (!out || total == 0) return KWK_OK;
  if (total > cap) return fail(KWK_ECAP, "fired buffer too small: need " + std::to_string(total));
  HIP_TRY(hipMemcpyAsync(out, e->hb[e->hb_cur].list, sizeof(kwk_fired_rec) * total, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return KWK_OK;
}

kwk_status kwk_fired_keep(kwk_engine* e, uint32_t depth) {
  ErrScope es_(e);
  if (!e) return fail(KWK_EINVAL, "null engine");
  if (depth > kHbMax) return fail(KWK_EINVAL, "kwk_fired_keep: depth 0.." + std::to_string(kHbMax));
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (e->copy_stream) HIP_TRY(hipStreamSynchronize(e->copy_stream));
  const uint32_t slots = depth > kHbMin ? depth : kHbMin;
  // the engine's last list stays the last (moved to slot 0 of the new ring)
  kwk_engine::HbSlot cur = e->hb[e->hb_cur];
  e->hb[e->hb_cur] = kwk_engine::HbSlot{};
  for (kwk_engine::HbSlot& h : e->hb) hb_free(h);
  e->hb.assign(slots, kwk_engine::HbSlot{});
  cur.copy_pending = false;
  e->hb[0] = cur;
  e->hb_cur = 0;
  e->hb_track = depth > 0;
  if (e->hb_track && !e->h_len) {
    HIP_TRY(hipHostMalloc((void**)&e->h_len, 2 * sizeof(uint32_t) * kHbMax, hipHostMallocDefault));
    memset(e->h_len, 0, 2 * sizeof(uint32_t) * kHbMax);
    HIP_TRY(hipHostGetDevicePointer((void**)&e->h_len_dev, e->h_len, 0));
  }
  e->hb[0].done_slot = 0;
  if (e->hb_track && e->hb[0].offsets) {  // the current list's length where a fetch reads it
    if (!e->hb[0].ev_done) HIP_TRY(hipEventCreateWithFlags(&e->hb[0].ev_done, hipEventDisableTiming));
    const bool bits = e->hb[0].mode == 3;
    e->h_len[1] = 0u;
    HIP_TRY(hipMemcpy(e->h_len, bits ? e->hb[0].tot : e->hb[0].offsets, (bits ? 2 : 1) * sizeof(uint32_t),
                      hipMemcpyDeviceToHost));
    HIP_TRY(hipEventRecord(e->hb[0].ev_done, e->stream));
  }
  return KWK_OK;
}

// slot i's list to host memory on the copy stream (kwk_fired_fetch_async / _step)
static kwk_status hb_fetch(kwk_engine* e, uint32_t i, void* out, uint64_t cap_bytes, uint32_t* seg_counts,
                           uint32_t seg_cap, kwk_fetch_info* info) {
  kwk_engine::HbSlot& h = e->hb[i];
  if (!e->copy_stream) {
    int prio = 0;
    HIP_TRY(hipStreamGetPriority(e->stream, &prio));
    HIP_TRY(hipStreamCreateWithPriority(&e->copy_stream, hipStreamNonBlocking, prio));
    HIP_TRY(hipEventCreateWithFlags(&e->ev_count, hipEventDisableTiming));
    HIP_TRY(hipHostMalloc((void**)&e->h_count, 64, hipHostMallocDefault));
  }
  if (!h.ev_copied) HIP_TRY(hipEventCreateWithFlags(&h.ev_copied, hipEventDisableTiming));
  const bool bits = h.mode == 3, b16 = h.mode == 2;
  const uint32_t rb = bits ? 4u : b16 ? 2u : h.mode == 1 ? 4u : (uint32_t)sizeof(kwk_fired_rec);
  const bool segs = b16 && seg_counts && h.n_segs;
  if (segs && h.n_segs > seg_cap) return fail(KWK_ECAP, "segment buffer too small: need " + std::to_string(h.n_segs));
  uint32_t t[2] = {0u, 0u};
  hipEvent_t done = nullptr;
  if (e->hb_track && h.done_slot >= 0 && e->hb[h.done_slot].ev_done) {
    // the compaction that wrote the slot signals its own end; its kernels wrote the length here
    done = e->hb[h.done_slot].ev_done;
    HIP_TRY(hipEventSynchronize(done));
    t[0] = e->h_len[2u * i];
    t[1] = e->h_len[2u * i + 1u];
  } else {
    // the length behind everything enqueued on the engine's stream so far
    HIP_TRY(hipMemcpyAsync(e->h_count, bits ? h.tot : h.offsets, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipEventRecord(e->ev_count, e->stream));
    HIP_TRY(hipEventSynchronize(e->ev_count));
    done = e->ev_count;
    t[0] = e->h_count[0];
    t[1] = e->h_count[1];
  }
  if (!h.n_segs) t[0] = t[1] = 0u;
  const uint32_t total = t[0];  // records, or the bitmap hand-back's 32-bit words
  info->n_records = bits ? t[1] : total;
  info->record_bytes = bits ? 0u : rb;
  info->format = bits ? KWK_COMPACT_BITS : b16 ? KWK_COMPACT_PACKED16 : h.mode == 1 ? KWK_COMPACT_PACKED : 1u;
  info->bytes = (uint64_t)total * rb;
  info->step = h.step;
  if (b16 || bits) {
    info->n_segs = h.n_segs;
    info->region_slots = h.region_slots;
  }
  if (out && (uint64_t)total * rb > cap_bytes)
    return fail(KWK_ECAP, "fired buffer too small: need " + std::to_string((uint64_t)total * rb) + " bytes");
  HIP_TRY(hipStreamWaitEvent(e->copy_stream, done, 0));
  if (out && total) HIP_TRY(hipMemcpyAsync(out, h.list, (size_t)total * rb, hipMemcpyDeviceToHost, e->copy_stream));
  if (segs)
    HIP_TRY(hipMemcpyAsync(seg_counts, h.counts, sizeof(uint32_t) * h.n_segs, hipMemcpyDeviceToHost, e->copy_stream));
  HIP_TRY(hipEventRecord(h.ev_copied, e->copy_stream));
  h.copy_pending = true;
  e->copy_recorded = true;
  return KWK_OK;
}

kwk_status kwk_fired_fetch_async(kwk_engine* e, void* out, uint64_t cap_bytes, uint32_t* seg_counts, uint32_t seg_cap,
                                 kwk_fetch_info* info) {
  ErrScope es_(e);
  if (!e || !info) return fail(KWK_EINVAL, "null argument");
  if (kwk_status st = set_dev(e)) return st;
  memset(info, 0, sizeof(*info));
  const uint32_t n_waves = e->last_blocks * kWavesPerBlock;
  if (n_waves == 0) return KWK_OK;
  if (!e->compacted) return fail(KWK_ESTATE, "kwk_fired_fetch_async needs the step's list compacted (kwk_fired_compact*)");
  return hb_fetch(e, e->hb_cur, out, cap_bytes, seg_counts, seg_cap, info);
}

kwk_status kwk_fired_fetch_step(kwk_engine* e, uint64_t step, void* out, uint64_t cap_bytes, uint32_t* seg_counts,
                                uint32_t seg_cap, kwk_fetch_info* info) {
  ErrScope es_(e);
  if (!e || !info) return fail(KWK_EINVAL, "null argument");
  if (kwk_status st = set_dev(e)) return st;
  memset(info, 0, sizeof(*info));
  const uint32_t n = (uint32_t)e->hb.size();
  for (uint32_t k = 0; k < n; ++k) {  // newest first
    const uint32_t i = (e->hb_cur + n - k) % n;
    if (e->hb[i].valid && e->hb[i].step == step) return hb_fetch(e, i, out, cap_bytes, seg_counts, seg_cap, info);
  }
  return fail(KWK_ESTATE, "no kept list of step " + std::to_string(step) + " (the ring holds the last " +
                              std::to_string(n) + " compactions: kwk_fired_keep)");
}

kwk_status kwk_fired_fetch_wait(kwk_engine* e) {
  ErrScope es_(e);
  if (!e) return fail(KWK_EINVAL, "null engine");
  if (kwk_status st = set_dev(e)) return st;
  if (e->copy_recorded) HIP_TRY(hipStreamSynchronize(e->copy_stream));  // every slot's copies
  return KWK_OK;
}

kwk_status kwk_alloc_host(uint64_t bytes, void** out) {
  if (!out) return fail(KWK_EINVAL, "null argument");
  *out = nullptr;
  if (bytes == 0) return KWK_OK;
  HIP_TRY(hipHostMalloc(out, bytes, hipHostMallocDefault));
  return KWK_OK;
}

kwk_status kwk_free_host(void* p) {
  if (p) HIP_TRY(hipHostFree(p));
  return KWK_OK;
}

kwk_status kwk_stats(kwk_engine* e, kwk_step_stats* out) {
  ErrScope es_(e);
  if (!e || !out) return fail(KWK_EINVAL, "null argument");
  if (kwk_status st = set_dev(e)) return st;
  hipLaunchKernelGGL(reduce_stats_kernel, dim3(kStatWords), dim3(kBlock), 0, e->stream, e->d_cum, e->cum_rows,
                     e->d_stats);
  HIP_TRY(hipGetLastError());
  unsigned long long h[kStatWords];
  HIP_TRY(hipMemcpyAsync(h, e->d_stats, sizeof(h), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  memset(out, 0, sizeof(*out));
  out->steps = e->steps;
  out->matched = h[0];
  out->fired = h[1];
  out->bytes = h[2];
  for (int s = 0; s < KWK_MAX_STAGES; ++s) out->fired_per_stage[s] = h[3 + s];
  out->line_bytes = h[kStatLine];
  out->state_bytes = word_bytes(e->fmt);
  return KWK_OK;
}

kwk_status kwk_read(kwk_engine* e, uint32_t first, uint32_t n, kwk_hot* hot, int64_t* del) {
  ErrScope es_(e);
  if (!e) return fail(KWK_EINVAL, "null engine");
  if ((uint64_t)first + n > e->capacity) return fail(KWK_EINVAL, "range beyond capacity");
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (hot) {  // device SoA -> AoS interchange rows
    std::vector<uint8_t> raw(word_bytes(e->fmt) * (size_t)n);
    std::vector<int64_t> due(n);
    HIP_TRY(hipMemcpy(raw.data(), (const char*)e->d_st + word_bytes(e->fmt) * first, raw.size(), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(due.data(), e->d_due + first, sizeof(int64_t) * n, hipMemcpyDeviceToHost));
    const std::vector<uint2> st = unpack_words(e, raw, e->fmt, n);
    if (e->fmt.dw) {  // D in the window, else the due column's value
      const uint2* r = reinterpret_cast<const uint2*>(raw.data());
      for (uint32_t i = 0; i < n; ++i) {
        const uint64_t d = dw_get(r[i]);
        if (d != kDwFar) due[i] = dw_abs(d, e->fmt.epoch);
      }
    }
    for (uint32_t i = 0; i < n; ++i) hot[i] = kwk_hot{st[i].x, st[i].y, due[i]};
  }
  if (del) HIP_TRY(hipMemcpy(del, e->d_del + first, sizeof(int64_t) * n, hipMemcpyDeviceToHost));
  return KWK_OK;
}

kwk_status kwk_usage_config(kwk_engine* e, uint32_t n_nodes, const uint32_t* node_ptr, const uint32_t* ukey,
                            uint32_t n_cpu, const double* cpu_values, uint32_t n_mem, const double* mem_values) {
  ErrScope es_(e);
  if (!e || !node_ptr || !ukey || !cpu_values || !mem_values) return fail(KWK_EINVAL, "null argument");
  if (n_cpu == 0 || n_mem == 0 || n_cpu > 0x4000 || n_mem > 0x4000) return fail(KWK_EINVAL, "dictionary size");
  if (node_ptr[0] != 0) return fail(KWK_EINVAL, "node_ptr[0] must be 0");
  for (uint32_t j = 0; j < n_nodes; ++j)
    if (node_ptr[j + 1] < node_ptr[j]) return fail(KWK_EINVAL, "node_ptr must be non-decreasing");
  const uint32_t n_pods = node_ptr[n_nodes];
  if (n_pods > e->capacity) return fail(KWK_ECAP, "node_ptr covers more pods than capacity");
  bool mixed_keys = false;
  for (uint32_t p = 0; p < n_pods; ++p) {
    if ((ukey[p] >> 28) == 0) {  // containers differ: index into kwk_usage_mixed's table
      mixed_keys = true;
      continue;
    }
    if ((ukey[p] & 0x3FFFu) >= n_cpu || ((ukey[p] >> 14) & 0x3FFFu) >= n_mem)
      return fail(KWK_EINVAL, "usage_key value id out of range");
  }
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  void* olds[] = {e->d_node_ptr, e->d_ukey, e->d_cpu, e->d_mem, e->d_node_out, e->d_node_cum, e->d_node_last,
                  e->d_usage_part, e->d_cluster, e->d_uchunk};
  for (void* p : olds) if (p) hipFree(p);
  // the usage kernels' chunks: whole nodes, at most kUChunkRows wave rows of pods (less the 8 of the
  // rounded start) and kUChunkNodes nodes each; a node with more pods than that gets a chunk of its
  // own (the wave carries its sum from row to row)
  std::vector<uint4> chunks;
  const uint32_t chunk_pods = kUChunkRows * kURow - 8u;
  for (uint32_t n = 0; n < n_nodes;) {
    const uint32_t c0 = node_ptr[n];
    uint32_t nb = n + 1;
    while (nb < n_nodes && nb - n < kUChunkNodes && node_ptr[nb + 1] - c0 <= chunk_pods) ++nb;
    chunks.push_back(make_uint4(c0, node_ptr[nb], n, nb));
    n = nb;
  }
  const uint32_t ublocks = ((uint32_t)chunks.size() + kWavesPerBlock - 1) / kWavesPerBlock;
  HIP_TRY(hipMalloc(&e->d_uchunk, sizeof(uint4) * (chunks.size() + 1)));
  if (!chunks.empty())
    HIP_TRY(upload(e, e->d_uchunk, chunks.data(), sizeof(uint4) * chunks.size()));
  e->n_uchunks = (uint32_t)chunks.size();
  // usage_fast_kernel's table: row nc = the value of a pod with nc alike containers, summed
  // container by container (podResourceUsage's order, :170-193) — what usage_kernel's loop adds
  uint32_t max_nc = 0;
  for (uint32_t p = 0; p < n_pods; ++p) max_nc = (ukey[p] >> 28) > max_nc ? (ukey[p] >> 28) : max_nc;
  if (e->d_podv) HIP_TRY(hipFree(e->d_podv));
  if (e->d_ukey8) HIP_TRY(hipFree(e->d_ukey8));
  if (e->d_kv) HIP_TRY(hipFree(e->d_kv));
  e->d_podv = nullptr;
  e->d_ukey8 = nullptr;
  e->d_kv = nullptr;
  e->podv_n = 0;
  e->kv_n = 0;
  const size_t nv = (size_t)n_cpu + n_mem;
  if ((max_nc + 1) * nv <= kUFastVals) {
    std::vector<double> podv((max_nc + 1) * nv, 0.0);
    for (uint32_t nc = 1; nc <= max_nc; ++nc) {
      for (uint32_t i = 0; i < n_cpu; ++i) {
        double v = 0.0;
        for (uint32_t c = 0; c < nc; ++c) v += cpu_values[i];
        podv[nc * nv + i] = v;
      }
      for (uint32_t i = 0; i < n_mem; ++i) {
        double v = 0.0;
        for (uint32_t c = 0; c < nc; ++c) v += mem_values[i];
        podv[nc * nv + n_cpu + i] = v;
      }
    }
    HIP_TRY(hipMalloc(&e->d_podv, sizeof(double) * podv.size()));
    HIP_TRY(upload(e, e->d_podv, podv.data(), sizeof(double) * podv.size()));
    e->podv_n = (uint32_t)podv.size();
    // distinct keys -> 1-byte column + {cpu, mem} values (the same podv entries, so the sums are
    // bit-identical to the 4-byte-key kernel's)
    std::vector<uint32_t> dict;
    std::vector<uint8_t> k8(n_pods);
    bool fits = true;
    for (uint32_t p = 0; p < n_pods && fits; ++p) {
      uint32_t d = 0;
      while (d < dict.size() && dict[d] != ukey[p]) ++d;  // few distinct keys: linear search
      if (d == dict.size()) {
        if (dict.size() == kUKeyZero) { fits = false; break; }
        dict.push_back(ukey[p]);
      }
      k8[p] = (uint8_t)d;
    }
    if (fits && n_pods) {
      std::vector<double2> kv(dict.size());
      for (size_t d = 0; d < dict.size(); ++d) {
        const uint32_t k = dict[d], row = (k >> 28) * (uint32_t)nv;
        kv[d] = make_double2(podv[row + (k & 0x3FFFu)], podv[row + n_cpu + ((k >> 14) & 0x3FFFu)]);
      }
      HIP_TRY(hipMalloc(&e->d_ukey8, (size_t)n_pods + 16));
      HIP_TRY(hipMalloc(&e->d_kv, sizeof(double2) * kv.size()));
      HIP_TRY(upload(e, e->d_ukey8, k8.data(), n_pods));
      HIP_TRY(upload(e, e->d_kv, kv.data(), sizeof(double2) * kv.size()));
      e->kv_n = (uint32_t)kv.size();
    }
  }
  HIP_TRY(hipMalloc(&e->d_node_ptr, 4 * ((size_t)n_nodes + 1)));
  HIP_TRY(hipMalloc(&e->d_ukey, 4 * ((size_t)n_pods + 1)));
  HIP_TRY(hipMalloc(&e->d_cpu, 8 * (size_t)n_cpu));
  HIP_TRY(hipMalloc(&e->d_mem, 8 * (size_t)n_mem));
  HIP_TRY(hipMalloc(&e->d_node_out, 32 * ((size_t)n_nodes + 1)));
  HIP_TRY(hipMalloc(&e->d_node_cum, 16 * ((size_t)n_nodes + 1)));
  HIP_TRY(hipMalloc(&e->d_node_last, 8 * ((size_t)n_nodes + 1)));
  HIP_TRY(hipMalloc(&e->d_usage_part, 16 * ((size_t)ublocks + 1)));
  HIP_TRY(hipMalloc(&e->d_cluster, 16));
  HIP_TRY(upload(e, e->d_node_ptr, node_ptr, 4 * ((size_t)n_nodes + 1)));
  HIP_TRY(upload(e, e->d_ukey, ukey, 4 * (size_t)n_pods));
  HIP_TRY(upload(e, e->d_cpu, cpu_values, 8 * (size_t)n_cpu));
  HIP_TRY(upload(e, e->d_mem, mem_values, 8 * (size_t)n_mem));
  HIP_TRY(hipMemsetAsync(e->d_node_cum, 0, 16 * ((size_t)n_nodes + 1), e->stream));
  HIP_TRY(hipMemsetAsync(e->d_cluster, 0, 16, e->stream));  // totals of a configuration without nodes stay 0
  HIP_TRY(hipMemsetAsync(e->d_node_last, 0x80, 8 * ((size_t)n_nodes + 1), e->stream));  // INT64_MIN-ish sentinel below
  std::vector<int64_t> lasts((size_t)n_nodes + 1, INT64_MIN);
  HIP_TRY(upload(e, e->d_node_last, lasts.data(), 8 * lasts.size()));
  e->n_nodes = n_nodes;
  e->n_usage_pods = n_pods;
  e->has_mixed_keys = mixed_keys;
  e->h_node_ptr.assign(node_ptr, node_ptr + n_nodes + 1);
  e->h_ukey.assign(ukey, ukey + n_pods);
  e->h_cpu.assign(cpu_values, cpu_values + n_cpu);
  e->h_mem.assign(mem_values, mem_values + n_mem);
  e->h_mixed.clear();
  e->h_ckeys.clear();
  e->h_cptr.clear();
  for (void* q : {(void*)e->d_mixed, (void*)e->d_ckeys, (void*)e->d_ccum, (void*)e->d_cptr, (void*)e->d_mbase})
    if (q) HIP_TRY(hipFree(q));
  e->d_mixed = nullptr;
  e->d_ckeys = nullptr;
  e->d_ccum = nullptr;
  e->d_cptr = nullptr;
  e->d_mbase = nullptr;
  e->h_mbase.clear();
  if (e->d_pod_cum) HIP_TRY(hipMemsetAsync(e->d_pod_cum, 0, 16 * (size_t)e->capacity, e->stream));
  return KWK_OK;
}

kwk_status kwk_usage_mixed(kwk_engine* e, uint32_t n_mixed, const uint32_t* mixed, uint32_t n_ckeys, const uint32_t* ckeys) {
  ErrScope es_(e);
  if (!e || (n_mixed && !mixed) || (n_ckeys && !ckeys)) return fail(KWK_EINVAL, "null argument");
  if (!e->d_node_ptr) return fail(KWK_ESTATE, "kwk_usage_config must be called first");
  if (n_mixed > kUKeyMixedIndex) return fail(KWK_ECAP, "too many mixed pods");
  for (uint32_t m = 0; m < n_mixed; ++m)
    if ((uint64_t)mixed[2 * m] + mixed[2 * m + 1] > n_ckeys) return fail(KWK_EINVAL, "mixed entry beyond ckeys");
  for (uint32_t c = 0; c < n_ckeys; ++c)
    if ((ckeys[c] & 0x3FFFu) >= e->h_cpu.size() || ((ckeys[c] >> 14) & 0x3FFFu) >= e->h_mem.size())
      return fail(KWK_EINVAL, "ckeys value id out of range");
  for (uint32_t p = 0; p < e->n_usage_pods; ++p)
    if ((e->h_ukey[p] >> 28) == 0 && (e->h_ukey[p] & kUKeyMixedIndex) >= n_mixed)
      return fail(KWK_EINVAL, "usage_key mixed index out of range");
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  for (void* q : {(void*)e->d_mixed, (void*)e->d_ckeys, (void*)e->d_ccum, (void*)e->d_cptr, (void*)e->d_mbase})
    if (q) HIP_TRY(hipFree(q));
  e->d_cptr = nullptr;
  e->h_cptr.clear();
  // integrators are per pod and container (mixed entries may be shared by pods whose containers
  // evaluate alike): each mixed pod's containers get their own range of ccum
  e->h_mbase.assign(e->n_usage_pods, 0u);
  uint64_t nint = 0;
  for (uint32_t p = 0; p < e->n_usage_pods; ++p)
    if ((e->h_ukey[p] >> 28) == 0) {
      e->h_mbase[p] = (uint32_t)nint;
      nint += mixed[2 * (size_t)(e->h_ukey[p] & kUKeyMixedIndex) + 1];
      if (nint > 0xFFFFFFFFull) return fail(KWK_ECAP, "more than 2^32 containers of mixed pods");
    }
  HIP_TRY(hipMalloc(&e->d_mixed, 8 * ((size_t)n_mixed + 1)));
  HIP_TRY(hipMalloc(&e->d_ckeys, 4 * ((size_t)n_ckeys + 1)));
  HIP_TRY(hipMalloc(&e->d_ccum, 16 * ((size_t)nint + 1)));
  HIP_TRY(hipMalloc(&e->d_mbase, 4 * ((size_t)e->n_usage_pods + 1)));
  if (n_mixed) HIP_TRY(upload(e, e->d_mixed, mixed, 8 * (size_t)n_mixed));
  if (n_ckeys) HIP_TRY(upload(e, e->d_ckeys, ckeys, 4 * (size_t)n_ckeys));
  if (e->n_usage_pods) HIP_TRY(upload(e, e->d_mbase, e->h_mbase.data(), 4 * (size_t)e->n_usage_pods));
  HIP_TRY(hipMemsetAsync(e->d_ccum, 0, 16 * ((size_t)nint + 1), e->stream));
  e->h_mixed.assign(mixed, mixed + 2 * (size_t)n_mixed);
  e->h_ckeys.assign(ckeys, ckeys + n_ckeys);
  return KWK_OK;
}

// containers per pod of the usage configuration
static uint32_t pod_containers(const kwk_engine* e, uint32_t p) {
  const uint32_t k = e->h_ukey[p];
  return (k >> 28) ? (k >> 28) : e->h_mixed[2 * (size_t)(k & kUKeyMixedIndex) + 1];
}

static kwk_status ensure_cptr(kwk_engine* e) {
  if (e->d_cptr) return KWK_OK;
  e->h_cptr.resize((size_t)e->n_usage_pods + 1);
  uint64_t c = 0;
  for (uint32_t p = 0; p < e->n_usage_pods; ++p) {
    e->h_cptr[p] = (uint32_t)c;
    c += pod_containers(e, p);
    if (c > 0xFFFFFFFFull) return fail(KWK_ECAP, "more than 2^32 containers");
  }
  e->h_cptr[e->n_usage_pods] = (uint32_t)c;
  HIP_TRY(hipMalloc(&e->d_cptr, 4 * e->h_cptr.size()));
  HIP_TRY(upload(e, e->d_cptr, e->h_cptr.data(), 4 * e->h_cptr.size()));
  return KWK_OK;
}

kwk_status kwk_usage_read_containers(kwk_engine* e, uint32_t first, uint32_t n, double* out, uint32_t cap, uint32_t* n_out) {
  ErrScope es_(e);
  if (!e || !n_out || (n && cap && !out)) return fail(KWK_EINVAL, "null argument");
  if (!e->d_pod_out) return fail(KWK_ESTATE, "kwk_usage_pods(eng, 1) must be called first");
  if ((uint64_t)first + n > e->n_usage_pods) return fail(KWK_EINVAL, "pods beyond the usage configuration");
  if (e->has_mixed_keys && !e->d_mixed) return fail(KWK_ESTATE, "kwk_usage_mixed must be called first");
  uint64_t total = 0;
  uint32_t cmin = 0xFFFFFFFFu, cmax = 0;
  for (uint32_t p = first; p < first + n; ++p) {
    total += pod_containers(e, p);
    const uint32_t k = e->h_ukey[p];
    if (!(k >> 28)) {
      const uint32_t f = e->h_mbase[p], c = e->h_mixed[2 * (size_t)(k & kUKeyMixedIndex) + 1];
      if (c) { cmin = f < cmin ? f : cmin; cmax = f + c > cmax ? f + c : cmax; }
    }
  }
  *n_out = (uint32_t)total;
  if (!out || total == 0) return KWK_OK;
  if (total > cap) return fail(KWK_ECAP, "container buffer too small: need " + std::to_string(total));
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  std::vector<uint8_t> raw(word_bytes(e->fmt) * (size_t)n);
  HIP_TRY(hipMemcpy(raw.data(), (const char*)e->d_st + word_bytes(e->fmt) * first, raw.size(), hipMemcpyDeviceToHost));
  const std::vector<uint2> st = unpack_words(e, raw, e->fmt, n);
  std::vector<double> unit(2 * (size_t)n);
  HIP_TRY(hipMemcpy(unit.data(), e->d_pod_cum + 2 * (size_t)first, 16 * (size_t)n, hipMemcpyDeviceToHost));
  std::vector<double> cc;
  if (cmin < cmax) {
    cc.resize(2 * (size_t)(cmax - cmin));
    HIP_TRY(hipMemcpy(cc.data(), e->d_ccum + 2 * (size_t)cmin, 16 * (size_t)(cmax - cmin), hipMemcpyDeviceToHost));
  }
  size_t o = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t p = first + i, k = e->h_ukey[p];
    const bool alive = (st[i].y & KWK_F_ALIVE) != 0;
    if (k >> 28) {
      for (uint32_t j = 0; j < (k >> 28); ++j, o += 4) {
        out[o] = alive ? e->h_cpu[k & 0x3FFFu] : 0.0;
        out[o + 1] = alive ? e->h_mem[(k >> 14) & 0x3FFFu] : 0.0;
        out[o + 2] = alive ? unit[2 * (size_t)i] : 0.0;
        out[o + 3] = alive ? unit[2 * (size_t)i + 1] : 0.0;
      }
    } else {
      const uint32_t f = e->h_mixed[2 * (size_t)(k & kUKeyMixedIndex)], c = e->h_mixed[2 * (size_t)(k & kUKeyMixedIndex) + 1];
      const uint32_t mb = e->h_mbase[p];
      for (uint32_t j = 0; j < c; ++j, o += 4) {
        const uint32_t ck = e->h_ckeys[f + j];
        out[o] = alive ? e->h_cpu[ck & 0x3FFFu] : 0.0;
        out[o + 1] = alive ? e->h_mem[(ck >> 14) & 0x3FFFu] : 0.0;
        out[o + 2] = alive ? cc[2 * (size_t)(mb + j - cmin)] : 0.0;
        out[o + 3] = alive ? cc[2 * (size_t)(mb + j - cmin) + 1] : 0.0;
      }
    }
  }
  return KWK_OK;
}

// the series inputs of one metric over nodes [n0, n1) (pods [p0, p1), containers from c0)
static MetricArgs metric_args(kwk_engine* e, uint32_t dim, int64_t now_ns, uint32_t n0, uint32_t n1, uint32_t p0,
                              uint32_t p1, uint32_t c0, uint32_t n_nodes) {
  MetricArgs a{};
  a.dim = dim;
  a.n0 = n0; a.n1 = n1; a.p0 = p0; a.p1 = p1; a.c0 = c0;
  const uint32_t c1 = e->h_cptr[p1];
  a.n_series = dim == KWK_METRIC_DIM_NODE ? n_nodes : dim == KWK_METRIC_DIM_POD ? (p1 - p0) : (c1 - c0);
  a.st = e->d_st;
  a.fmt = e->fmt;
  a.node_ptr = e->d_node_ptr;
  a.cptr = e->d_cptr;
  a.ukey = e->d_ukey;
  a.mixed = e->d_mixed;
  a.ckeys = e->d_ckeys;
  a.mbase = e->d_mbase;
  a.cpu_v = e->d_cpu;
  a.mem_v = e->d_mem;
  a.pod_out = e->d_pod_out;
  a.pod_cum = e->d_pod_cum;
  a.ccum = e->d_ccum;
  a.node_out = e->d_node_out;
  a.pod_created = e->d_pod_created;
  a.node_created = e->d_node_created;
  a.node_started = e->d_node_started;
  a.now = now_ns;
  a.zero_time_unix_s = e->zero_time_unix_s;
  return a;
}

// validates one lowered value program of `dimension` (kwk_metrics_load / kwk_histograms_load)
static kwk_status check_metric_program(const kwk_metric_op* ops, uint32_t first, uint32_t n, uint32_t n_ops,
                                       uint32_t dimension, uint32_t& needs) {
  if (dimension > KWK_METRIC_DIM_CONTAINER) return fail(KWK_EINVAL, "metric dimension");
  if (n == 0 || n > 64 || (uint64_t)first + n > n_ops) return fail(KWK_EINVAL, "metric ops range");
  int depth = 0;
  for (uint32_t i = first; i < first + n; ++i) {
    const kwk_metric_op& op = ops[i];
    if (op.op == KWK_MOP_CONST || op.op == KWK_MOP_LOAD) {
      if (++depth > 8) return fail(KWK_EINVAL, "metric program deeper than 8");
      if (op.op == KWK_MOP_LOAD) {
        if (op.arg > KWK_MIN_STARTED_CONTAINERS) return fail(KWK_EINVAL, "metric input");
        if (op.arg >= KWK_MIN_POD_SINCE) needs = 1;
        if (dimension == KWK_METRIC_DIM_NODE && op.arg >= KWK_MIN_CONTAINER_CPU && op.arg <= KWK_MIN_POD_CUM_MEM)
          return fail(KWK_EINVAL, "a node metric cannot read pod / container inputs");
        if (dimension == KWK_METRIC_DIM_NODE && (op.arg == KWK_MIN_POD_SINCE || op.arg == KWK_MIN_POD_CREATED))
          return fail(KWK_EINVAL, "a node metric cannot read pod inputs");
        if (dimension == KWK_METRIC_DIM_POD && op.arg >= KWK_MIN_CONTAINER_CPU && op.arg <= KWK_MIN_CONTAINER_CUM_MEM)
          return fail(KWK_EINVAL, "a pod metric cannot read container inputs");
      }
    } else if (op.op == KWK_MOP_NEG) {
      if (depth < 1) return fail(KWK_EINVAL, "metric program underflow");
    } else if (op.op >= KWK_MOP_ADD && op.op <= KWK_MOP_DIV) {
      if (depth < 2) return fail(KWK_EINVAL, "metric program underflow");
      --depth;
    } else {
      return fail(KWK_EINVAL, "metric op");
    }
  }
  if (depth != 1) return fail(KWK_EINVAL, "a metric program leaves one value");
  return KWK_OK;
}

kwk_status kwk_metrics_load(kwk_engine* e, uint32_t n_metrics, const kwk_metric_desc* metrics, uint32_t n_ops,
                            const kwk_metric_op* ops) {
  ErrScope es_(e);
  if (!e || (n_metrics && !metrics) || (n_ops && !ops)) return fail(KWK_EINVAL, "null argument");
  uint32_t needs = 0;
  for (uint32_t m = 0; m < n_metrics; ++m)
    if (kwk_status st = check_metric_program(ops, metrics[m].first_op, metrics[m].n_ops, n_ops, metrics[m].dimension, needs))
      return st;
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (e->d_mops) HIP_TRY(hipFree(e->d_mops));
  e->d_mops = nullptr;
  HIP_TRY(hipMalloc(&e->d_mops, sizeof(kwk_metric_op) * ((size_t)n_ops + 1)));
  if (n_ops) HIP_TRY(upload(e, e->d_mops, ops, sizeof(kwk_metric_op) * n_ops));
  e->metrics.assign(metrics, metrics + n_metrics);
  e->metric_inputs_needed = needs;
  return KWK_OK;
}

kwk_status kwk_metrics_inputs(kwk_engine* e, const int64_t* pod_created, const int64_t* node_created, const double* started,
                              double zero_time_unix_s) {
  ErrScope es_(e);
  if (!e || !pod_created || !node_created || !started) return fail(KWK_EINVAL, "null argument");
  if (!e->d_node_ptr) return fail(KWK_ESTATE, "kwk_usage_config must be called first");
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  for (void* q : {(void*)e->d_pod_created, (void*)e->d_node_created, (void*)e->d_node_started})
    if (q) HIP_TRY(hipFree(q));
  HIP_TRY(hipMalloc(&e->d_pod_created, 8 * ((size_t)e->n_usage_pods + 1)));
  HIP_TRY(hipMalloc(&e->d_node_created, 8 * ((size_t)e->n_nodes + 1)));
  HIP_TRY(hipMalloc(&e->d_node_started, 8 * ((size_t)e->n_nodes + 1)));
  if (e->n_usage_pods)
    HIP_TRY(upload(e, e->d_pod_created, pod_created, 8 * (size_t)e->n_usage_pods));
  if (e->n_nodes) {
    HIP_TRY(upload(e, e->d_node_created, node_created, 8 * (size_t)e->n_nodes));
    HIP_TRY(upload(e, e->d_node_started, started, 8 * (size_t)e->n_nodes));
  }
  e->zero_time_unix_s = zero_time_unix_s;
  return KWK_OK;
}

// the metric kernels of a scrape into d_mout (enqueue only); *n_out = the values
static kwk_status enqueue_metrics(kwk_engine* e, int64_t now_ns, uint32_t node_first, uint32_t n_nodes, bool run,
                                  uint64_t* n_out) {
  if (!e->d_node_ptr) return fail(KWK_ESTATE, "kwk_usage_config must be called first");
  if (!e->d_pod_out) return fail(KWK_ESTATE, "kwk_usage_pods(eng, 1) must be called first");
  if (e->has_mixed_keys && !e->d_mixed) return fail(KWK_ESTATE, "kwk_usage_mixed must be called first");
  if (e->metric_inputs_needed && !e->d_pod_created) return fail(KWK_ESTATE, "kwk_metrics_inputs must be called first");
  if ((uint64_t)node_first + n_nodes > e->n_nodes) return fail(KWK_EINVAL, "nodes beyond the usage configuration");
  if (kwk_status st = set_dev(e)) return st;
  if (kwk_status st = ensure_cptr(e)) return st;
  const uint32_t n0 = node_first, n1 = node_first + n_nodes;
  const uint32_t p0 = e->h_node_ptr[n0], p1 = e->h_node_ptr[n1];
  const uint32_t c0 = e->h_cptr[p0], c1 = e->h_cptr[p1];
  uint64_t total = 0;
  for (const auto& m : e->metrics)
    total += m.dimension == KWK_METRIC_DIM_NODE ? n_nodes : m.dimension == KWK_METRIC_DIM_POD ? (p1 - p0) : (c1 - c0);
  *n_out = total;
  if (!run || total == 0) return KWK_OK;
  if (total > e->mout_cap) {
    if (e->d_mout) HIP_TRY(hipFree(e->d_mout));
    e->d_mout = nullptr;
    HIP_TRY(hipMalloc(&e->d_mout, 8 * total));
    e->mout_cap = total;
  }
  uint64_t off = 0;
  PodMetricList pl{};
  for (const auto& m : e->metrics) {
    MetricArgs a = metric_args(e, m.dimension, now_ns, n0, n1, p0, p1, c0, n_nodes);
    if (m.dimension != KWK_METRIC_DIM_NODE && pl.n < kMaxPodMetrics) {  // pod-major launch below
      pl.m[pl.n++] = PodMetric{m.dimension, m.first_op, m.n_ops, 0u, off};
    } else {
      a.ops = e->d_mops + m.first_op;
      a.n_ops = m.n_ops;
      a.out = e->d_mout + off;
      if (a.n_series)
        hipLaunchKernelGGL(metrics_kernel, dim3((a.n_series + kBlock - 1) / kBlock), dim3(kBlock), 0, e->stream, a);
      HIP_TRY(hipGetLastError());
    }
    off += a.n_series;
  }
  if (pl.n && p1 > p0) {
    MetricArgs a = metric_args(e, KWK_METRIC_DIM_POD, now_ns, n0, n1, p0, p1, c0, n_nodes);
    a.ops = e->d_mops;
    hipLaunchKernelGGL(metrics_pod_kernel, dim3((p1 - p0 + kBlock - 1) / kBlock), dim3(kBlock), 0, e->stream, a, pl,
                       e->d_mout);
    HIP_TRY(hipGetLastError());
  }
  return KWK_OK;
}

kwk_status kwk_metrics_eval(kwk_engine* e, int64_t now_ns, uint32_t node_first, uint32_t n_nodes, double* out, uint64_t cap,
                            uint64_t* n_out) {
  ErrScope es_(e);
  if (!e || !n_out) return fail(KWK_EINVAL, "null argument");
  uint64_t total = 0;
  if (kwk_status st = enqueue_metrics(e, now_ns, node_first, n_nodes, false, &total)) return st;
  *n_out = total;
  if (!out || total == 0) return KWK_OK;
  if (total > cap) return fail(KWK_ECAP, "metric buffer too small: need " + std::to_string(total));
  if (kwk_status st = enqueue_metrics(e, now_ns, node_first, n_nodes, true, &total)) return st;
  HIP_TRY(hipMemcpyAsync(out, e->d_mout, 8 * total, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return KWK_OK;
}

kwk_status kwk_metrics_eval_device(kwk_engine* e, int64_t now_ns, uint32_t node_first, uint32_t n_nodes,
                                   const double** out, uint64_t* n_out) {
  ErrScope es_(e);
  if (!e || !out || !n_out) return fail(KWK_EINVAL, "null argument");
  *out = nullptr;
  if (kwk_status st = enqueue_metrics(e, now_ns, node_first, n_nodes, true, n_out)) return st;
  *out = e->d_mout;
  return KWK_OK;
}

// Go's sort.Float64s order (NaN first, then ascending)
static bool go_float_less(double x, double y) { return x < y || (std::isnan(x) && !std::isnan(y)); }

kwk_status kwk_histograms_load(kwk_engine* e, uint32_t n_hist, const kwk_histogram_desc* hists, uint32_t n_buckets,
                               const kwk_metric_bucket* buckets, uint32_t n_ops, const kwk_metric_op* ops) {
  ErrScope es_(e);
  if (!e || (n_hist && !hists) || (n_buckets && !buckets) || (n_ops && !ops)) return fail(KWK_EINVAL, "null argument");
  uint32_t needs = 0;
  std::vector<HistDesc> hd(n_hist);
  std::vector<uint32_t> keys;
  std::vector<double> bounds;
  for (uint32_t h = 0; h < n_hist; ++h) {
    const kwk_histogram_desc& d = hists[h];
    if (d.n_buckets == 0 || d.n_buckets > kMaxHistBuckets || (uint64_t)d.first_bucket + d.n_buckets > n_buckets)
      return fail(KWK_EINVAL, "histogram " + std::to_string(h) + ": buckets range (1..64 buckets)");
    for (uint32_t b = d.first_bucket; b < d.first_bucket + d.n_buckets; ++b)
      if (kwk_status st = check_metric_program(ops, buckets[b].first_op, buckets[b].n_ops, n_ops, d.dimension, needs))
        return st;
    HistDesc x{};
    x.dim = d.dimension;
    x.first_bucket = d.first_bucket;
    x.n_buckets = d.n_buckets;
    // stored keys: one per distinct le, the last bucket setting it wins (histogram.Set); ascending
    std::vector<uint32_t> k;
    for (uint32_t b = 0; b < d.n_buckets; ++b) {
      const double le = buckets[d.first_bucket + b].le;
      bool dup = false;
      for (uint32_t& q : k)
        if (buckets[d.first_bucket + q].le == le || (std::isnan(le) && std::isnan(buckets[d.first_bucket + q].le))) {
          q = b;
          dup = true;
        }
      if (!dup) k.push_back(b);
    }
    std::stable_sort(k.begin(), k.end(), [&](uint32_t p, uint32_t q) {
      return go_float_less(buckets[d.first_bucket + p].le, buckets[d.first_bucket + q].le);
    });
    std::vector<double> vb;  // the visible upper bounds (getOrRegisterHistogram skips hidden ones), sorted
    for (uint32_t b = 0; b < d.n_buckets; ++b)
      if (!buckets[d.first_bucket + b].hidden) vb.push_back(buckets[d.first_bucket + b].le);
    std::stable_sort(vb.begin(), vb.end(), go_float_less);
    x.first_key = (uint32_t)keys.size();
    x.n_keys = (uint32_t)k.size();
    x.first_bound = (uint32_t)bounds.size();
    x.n_bounds = (uint32_t)vb.size();
    x.out_words = x.n_bounds + 3;
    keys.insert(keys.end(), k.begin(), k.end());
    bounds.insert(bounds.end(), vb.begin(), vb.end());
    hd[h] = x;
  }
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  for (void** q : {(void**)&e->d_hops, (void**)&e->d_hbuckets, (void**)&e->d_hkeys, (void**)&e->d_hbounds}) {
    if (*q) HIP_TRY(hipFree(*q));
    *q = nullptr;
  }
  HIP_TRY(hipMalloc(&e->d_hops, sizeof(kwk_metric_op) * ((size_t)n_ops + 1)));
  HIP_TRY(hipMalloc(&e->d_hbuckets, sizeof(kwk_metric_bucket) * ((size_t)n_buckets + 1)));
  HIP_TRY(hipMalloc(&e->d_hkeys, sizeof(uint32_t) * (keys.size() + 1)));
  HIP_TRY(hipMalloc(&e->d_hbounds, sizeof(double) * (bounds.size() + 1)));
  if (n_ops) HIP_TRY(upload(e, e->d_hops, ops, sizeof(kwk_metric_op) * n_ops));
  if (n_buckets) HIP_TRY(upload(e, e->d_hbuckets, buckets, sizeof(kwk_metric_bucket) * n_buckets));
  if (!keys.empty()) HIP_TRY(upload(e, e->d_hkeys, keys.data(), sizeof(uint32_t) * keys.size()));
  if (!bounds.empty())
    HIP_TRY(upload(e, e->d_hbounds, bounds.data(), sizeof(double) * bounds.size()));
  e->hists = hd;
  e->hist_inputs_needed = needs;
  return KWK_OK;
}

static kwk_status enqueue_histograms(kwk_engine* e, int64_t now_ns, uint32_t node_first, uint32_t n_nodes, bool run,
                                     uint64_t* n_out) {
  if (!e->d_node_ptr) return fail(KWK_ESTATE, "kwk_usage_config must be called first");
  if (!e->d_pod_out) return fail(KWK_ESTATE, "kwk_usage_pods(eng, 1) must be called first");
  if (e->has_mixed_keys && !e->d_mixed) return fail(KWK_ESTATE, "kwk_usage_mixed must be called first");
  if (e->hist_inputs_needed && !e->d_pod_created) return fail(KWK_ESTATE, "kwk_metrics_inputs must be called first");
  if ((uint64_t)node_first + n_nodes > e->n_nodes) return fail(KWK_EINVAL, "nodes beyond the usage configuration");
  if (kwk_status st = set_dev(e)) return st;
  if (kwk_status st = ensure_cptr(e)) return st;
  const uint32_t n0 = node_first, n1 = node_first + n_nodes;
  const uint32_t p0 = e->h_node_ptr[n0], p1 = e->h_node_ptr[n1];
  const uint32_t c0 = e->h_cptr[p0];
  uint64_t total = 0;
  for (const auto& h : e->hists)
    total += (uint64_t)metric_args(e, h.dim, now_ns, n0, n1, p0, p1, c0, n_nodes).n_series * h.out_words;
  *n_out = total;
  if (!run || total == 0) return KWK_OK;
  if (total > e->hout_cap) {
    if (e->d_hout) HIP_TRY(hipFree(e->d_hout));
    e->d_hout = nullptr;
    HIP_TRY(hipMalloc(&e->d_hout, 8 * total));
    e->hout_cap = total;
  }
  uint64_t off = 0;
  for (const auto& h : e->hists) {
    MetricArgs a = metric_args(e, h.dim, now_ns, n0, n1, p0, p1, c0, n_nodes);
    a.ops = e->d_hops;
    if (a.n_series)
      hipLaunchKernelGGL(histogram_kernel, dim3((a.n_series + kBlock - 1) / kBlock), dim3(kBlock), 0, e->stream, a, h,
                         (const kwk_metric_bucket*)e->d_hbuckets, (const uint32_t*)e->d_hkeys,
                         (const double*)e->d_hbounds, e->d_hout + off);
    HIP_TRY(hipGetLastError());
    off += (uint64_t)a.n_series * h.out_words;
  }
  return KWK_OK;
}

kwk_status kwk_histograms_eval(kwk_engine* e, int64_t now_ns, uint32_t node_first, uint32_t n_nodes, uint64_t* out,
                               uint64_t cap, uint64_t* n_out) {
  ErrScope es_(e);
  if (!e || !n_out) return fail(KWK_EINVAL, "null argument");
  uint64_t total = 0;
  if (kwk_status st = enqueue_histograms(e, now_ns, node_first, n_nodes, false, &total)) return st;
  *n_out = total;
  if (!out || total == 0) return KWK_OK;
  if (total > cap) return fail(KWK_ECAP, "histogram buffer too small: need " + std::to_string(total));
  if (kwk_status st = enqueue_histograms(e, now_ns, node_first, n_nodes, true, &total)) return st;
  HIP_TRY(hipMemcpyAsync(out, e->d_hout, 8 * total, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return KWK_OK;
}

kwk_status kwk_histograms_eval_device(kwk_engine* e, int64_t now_ns, uint32_t node_first, uint32_t n_nodes,
                                      const uint64_t** out, uint64_t* n_out) {
  ErrScope es_(e);
  if (!e || !out || !n_out) return fail(KWK_EINVAL, "null argument");
  *out = nullptr;
  if (kwk_status st = enqueue_histograms(e, now_ns, node_first, n_nodes, true, n_out)) return st;
  *out = e->d_hout;
  return KWK_OK;
}

// whether usage_fast_kernel<1, true> runs for this engine and covers every active slot, so that
// kwk_aggregate's mask counts (<= 4) can ride along in it instead of a count8_kernel pass
static bool usage_counts(const kwk_engine* e, uint32_t n_masks) {
  return e->agg_fused && n_masks >= 1 && n_masks <= 4 && word_bytes(e->fmt) == 1 && !e->has_mixed_keys &&
         !e->d_pod_out && e->podv_n && e->d_ukey8 && e->usage_key8 && e->n_nodes && e->n_usage_pods == e->n_active;
}

// the usage kernel alone (its block partials in d_usage_part, *n_blocks of them); cmasks: the
// mask counts folded in (usage_counts), their partial rows in d_count_part
static kwk_status enqueue_usage(kwk_engine* e, int64_t now_ns, uint32_t* n_blocks, const uint32_t* cmasks = nullptr,
                                uint32_t n_cmasks = 0) {
  *n_blocks = 0;
  const uint32_t ublocks = (e->n_uchunks + kWavesPerBlock - 1) / kWavesPerBlock;
  UsageArgs ua{e->d_st, e->fmt, e->d_node_ptr, e->d_ukey, e->d_cpu, e->d_mem, (uint32_t)e->h_cpu.size(),
               (uint32_t)e->h_mem.size(), e->d_uchunk, e->n_uchunks, e->n_usage_pods, e->d_node_out, e->d_node_cum,
               e->d_node_last, now_ns, e->d_usage_part, e->d_pod_out, e->d_pod_cum, e->d_pod_last, e->d_mixed,
               e->d_ckeys, e->d_mbase, e->d_ccum, e->d_podv, e->podv_n, e->d_ukey8, e->d_kv, e->kv_n,
               cmasks, n_cmasks, e->d_count_part};
  const uint32_t wb = word_bytes(e->fmt);
  // the kernels are specialised on the state word's bytes (1: dictionary ids, 2, 4, 8)
#define USAGE_KERNEL(K, ...) (wb == 1 ? (const void*)K<1 __VA_ARGS__> : wb == 2 ? (const void*)K<2 __VA_ARGS__>   \
                              : wb == 4 ? (const void*)K<4 __VA_ARGS__> : (const void*)K<8 __VA_ARGS__>)
  if (!e->has_mixed_keys && !e->d_pod_out && e->podv_n) {  // usage_fast_kernel
    const bool k8 = e->d_ukey8 != nullptr && e->usage_key8;
    const void* fk = k8 ? USAGE_KERNEL(usage_fast_kernel, , true) : USAGE_KERNEL(usage_fast_kernel);
    // 8 workgroups per CU by default, twice what is resident: the last chunks start as the first
    // workgroups finish, so the tail is shorter (C5: 91-93 vs 97-99 us with the occupancy grid, r4 agg)
    const uint32_t per_cu = 8u;
    const uint32_t grid = std::min(ublocks, (uint32_t)e->n_cus * per_cu);
    if (grid) {
      void* args[] = {&ua};
      HIP_TRY(hipLaunchKernel(fk, dim3(grid), dim3(kBlock), args, 0, e->stream));
    }
    *n_blocks = grid;
    return KWK_OK;
  }
  // persistent grid (every block slot the occupancy allows), at most one chunk per wave
  const void* kern = USAGE_KERNEL(usage_kernel);
#undef USAGE_KERNEL
  const uint32_t grid = persist_grid(e, kern, ublocks);
  if (grid) {
    void* args[] = {&ua};
    HIP_TRY(hipLaunchKernel(kern, dim3(grid), dim3(kBlock), args, 0, e->stream));
  }
  *n_blocks = grid;
  return KWK_OK;
}

kwk_status kwk_usage(kwk_engine* e, int64_t now_ns) {
  ErrScope es_(e);
  if (!e) return fail(KWK_EINVAL, "null engine");
  if (!e->d_node_ptr) return fail(KWK_ESTATE, "kwk_usage_config must be called first");
  if (e->n_nodes == 0) return KWK_OK;
  if (e->has_mixed_keys && !e->d_mixed) return fail(KWK_ESTATE, "kwk_usage_mixed must be called first");
  uint32_t grid = 0;
  if (kwk_status st = enqueue_usage(e, now_ns, &grid)) return st;
  hipLaunchKernelGGL(usage_total_kernel, dim3(1), dim3(1024), 0, e->stream, e->d_usage_part, grid, e->d_cluster);
  HIP_TRY(hipGetLastError());
  return KWK_OK;
}

kwk_status kwk_usage_pods(kwk_engine* e, uint32_t enable) {
  ErrScope es_(e);
  if (!e) return fail(KWK_EINVAL, "null engine");
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  void* olds[] = {e->d_pod_out, e->d_pod_cum, e->d_pod_last};
  for (void* p : olds) if (p) HIP_TRY(hipFree(p));
  e->d_pod_out = nullptr;
  e->d_pod_cum = nullptr;
  e->d_pod_last = nullptr;
  if (!enable) return KWK_OK;
  const size_t n = e->capacity;
  HIP_TRY(hipMalloc(&e->d_pod_out, 32 * n));
  HIP_TRY(hipMalloc(&e->d_pod_cum, 16 * n));
  HIP_TRY(hipMalloc(&e->d_pod_last, 8 * n));
  HIP_TRY(hipMemsetAsync(e->d_pod_out, 0, 32 * n, e->stream));
  HIP_TRY(hipMemsetAsync(e->d_pod_cum, 0, 16 * n, e->stream));
  std::vector<int64_t> lasts(n, INT64_MIN);
  HIP_TRY(upload(e, e->d_pod_last, lasts.data(), 8 * n));
  return KWK_OK;
}

kwk_status kwk_usage_read_pods(kwk_engine* e, uint32_t first, uint32_t n, double* pod_out) {
  ErrScope es_(e);
  if (!e || (n && !pod_out)) return fail(KWK_EINVAL, "null argument");
  if (!e->d_pod_out) return fail(KWK_ESTATE, "kwk_usage_pods(eng, 1) must be called first");
  if ((uint64_t)first + n > e->capacity) return fail(KWK_EINVAL, "range beyond capacity");
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (n) HIP_TRY(hipMemcpy(pod_out, e->d_pod_out + 4 * (size_t)first, 32 * (size_t)n, hipMemcpyDeviceToHost));
  return KWK_OK;
}

kwk_status kwk_usage_read(kwk_engine* e, double* node_out, double* cluster_out) {
  ErrScope es_(e);
  if (!e) return fail(KWK_EINVAL, "null engine");
  if (!e->d_node_ptr) return fail(KWK_ESTATE, "kwk_usage_config must be called first");
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (node_out && e->n_nodes) HIP_TRY(hipMemcpy(node_out, e->d_node_out, 32 * (size_t)e->n_nodes, hipMemcpyDeviceToHost));
  if (cluster_out) HIP_TRY(hipMemcpy(cluster_out, e->d_cluster, 16, hipMemcpyDeviceToHost));
  return KWK_OK;
}

// count_kernel's partial rows: at most n_cus * 32 blocks
static kwk_status ensure_count_part(kwk_engine* e) {
  if (!e->d_count_part)
    HIP_TRY(hipMalloc(&e->d_count_part, sizeof(uint32_t) * kMaxCountMasks * ((size_t)e->n_cus * 32u + 1)));
  return KWK_OK;
}

kwk_status kwk_count(kwk_engine* e, uint32_t n_masks, const uint32_t* masks, uint64_t* counts) {
  ErrScope es_(e);
  if (!e || (n_masks && (!masks || !counts))) return fail(KWK_EINVAL, "null argument");
  if (n_masks > kMaxCountMasks) return fail(KWK_EINVAL, "at most 16 masks");
  if (n_masks == 0) return KWK_OK;
  if (kwk_status st = set_dev(e)) return st;
  if (kwk_status st = ensure_stage_buf(e, 4 * kMaxCountMasks + 8 * kMaxCountMasks)) return st;
  uint32_t* d_masks = (uint32_t*)e->d_stage_buf;
  unsigned long long* d_out = (unsigned long long*)((char*)e->d_stage_buf + 4 * kMaxCountMasks);
  HIP_TRY(hipMemcpyAsync(d_masks, masks, 4 * (size_t)n_masks, hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemsetAsync(d_out, 0, 8 * kMaxCountMasks, e->stream));
  if (e->n_active) {
    const uint32_t wb = (uint32_t)word_bytes(e->fmt);
    const uint64_t chunks = ((uint64_t)e->n_active * wb + 15u) / 16u;
    uint64_t blocks = (chunks + kBlock * 4 - 1) / (kBlock * 4);  // 4 chunks per lane, loaded together
    blocks = blocks < (uint64_t)e->n_cus * 8u ? blocks : (uint64_t)e->n_cus * 8u;
    // the alive flag and the pred bits in the raw word (packed: flags at fshift; wide: {pred, sched})
    const bool wide = wb == 8 && !e->fmt.dw;
    const uint32_t abit = wide ? (uint32_t)KWK_F_ALIVE : (uint32_t)(KWK_F_ALIVE >> 8) << e->fmt.fshift;
    const uint32_t pmask = wide ? 0xFFFFFFFFu : e->fmt.pmask;
    const dim3 g((uint32_t)blocks);
    if (kwk_status st = ensure_count_part(e)) return st;
    if (wb == 1) launch_count8(n_masks, g, e->stream, e->d_st, e->n_active, e->fmt, d_masks, e->d_count_part, d_out);
    else if (wb == 2) launch_count<2>(n_masks, g, e->stream, e->d_st, e->n_active, abit, pmask, d_masks, e->d_count_part, d_out);
    else if (wb == 4) launch_count<4>(n_masks, g, e->stream, e->d_st, e->n_active, abit, pmask, d_masks, e->d_count_part, d_out);
    else launch_count<8>(n_masks, g, e->stream, e->d_st, e->n_active, abit, pmask, d_masks, e->d_count_part, d_out,
                         e->fmt.dw);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipMemcpyAsync(counts, d_out, 8 * (size_t)n_masks, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return KWK_OK;
}

kwk_status kwk_aggregate(kwk_engine* e, uint32_t n_masks, const uint32_t* masks, int64_t now_ns, uint32_t flags,
                         double* out, uint32_t* n_out) {
  ErrScope es_(e);
  if (!e || !n_out || (n_masks && !masks)) return fail(KWK_EINVAL, "null argument");
  if (n_masks > kMaxCountMasks) return fail(KWK_EINVAL, "at most 16 masks");
  const bool usage = (flags & KWK_AGG_USAGE) != 0;
  if (usage && !e->d_node_ptr) return fail(KWK_ESTATE, "kwk_usage_config must be called first");
  if (kwk_status st = set_dev(e)) return st;
  const uint32_t n_stages = e->loaded_table ? e->n_stages : 0u;
  if (!e->d_agg) {
    HIP_TRY(hipMalloc(&e->d_agg, sizeof(double) * (KWK_MAX_STAGES + kMaxCountMasks + 2)));
    HIP_TRY(hipMalloc(&e->d_agg_counts, sizeof(unsigned long long) * kMaxCountMasks));
    HIP_TRY(hipMalloc(&e->d_agg_masks, sizeof(uint32_t) * kMaxCountMasks));
  }
  double* dst = out ? out : e->d_agg;
  // count_total_kernel overwrites the counts it produces: zeroed only when no count runs.  The
  // masks go to the device only when they change (a pageable copy would stall the host, r3 trace)
  if (!(n_masks && e->n_active))
    HIP_TRY(hipMemsetAsync(e->d_agg_counts, 0, sizeof(unsigned long long) * kMaxCountMasks, e->stream));
  uint32_t n_cblocks = 0;  // count blocks whose partial rows agg_final_kernel sums
  // the counts ride along in the usage kernel (one pass over the id column instead of two)
  const bool fused = usage && e->d_node_ptr && usage_counts(e, n_masks);
  if (fused)
    if (kwk_status st = ensure_count_part(e)) return st;
  if (n_masks) {
    if (n_masks != e->agg_n_masks || memcmp(masks, e->agg_masks, 4 * (size_t)n_masks) != 0) {
      // the previous masks' copy may still be queued on the stream (it reads e->agg_masks when
      // it runs): drain it before the array is overwritten (masks change rarely)
      HIP_TRY(hipStreamSynchronize(e->stream));
      memcpy(e->agg_masks, masks, 4 * (size_t)n_masks);
      e->agg_n_masks = n_masks;
      HIP_TRY(hipMemcpyAsync(e->d_agg_masks, e->agg_masks, 4 * (size_t)n_masks, hipMemcpyHostToDevice, e->stream));
    }
    if (e->n_active && !fused) {
      const uint32_t wb = (uint32_t)word_bytes(e->fmt);
      const uint64_t chunks = ((uint64_t)e->n_active * wb + 15u) / 16u;
      uint64_t blocks = (chunks + kBlock * 4 - 1) / (kBlock * 4);
      blocks = blocks < (uint64_t)e->n_cus * 8u ? blocks : (uint64_t)e->n_cus * 8u;
      const bool wide = wb == 8 && !e->fmt.dw;
      const uint32_t abit = wide ? (uint32_t)KWK_F_ALIVE : (uint32_t)(KWK_F_ALIVE >> 8) << e->fmt.fshift;
      const uint32_t pmask = wide ? 0xFFFFFFFFu : e->fmt.pmask;
      const dim3 g((uint32_t)blocks);
      if (kwk_status st = ensure_count_part(e)) return st;
      uint32_t* pp = e->d_count_part;
      // partial rows only: agg_final_kernel sums them
      if (wb == 1) launch_count8(n_masks, g, e->stream, e->d_st, e->n_active, e->fmt, e->d_agg_masks, pp, nullptr);
      else if (wb == 2) launch_count<2>(n_masks, g, e->stream, e->d_st, e->n_active, abit, pmask, e->d_agg_masks, pp, nullptr);
      else if (wb == 4) launch_count<4>(n_masks, g, e->stream, e->d_st, e->n_active, abit, pmask, e->d_agg_masks, pp, nullptr);
      else launch_count<8>(n_masks, g, e->stream, e->d_st, e->n_active, abit, pmask, e->d_agg_masks, pp, nullptr,
                           e->fmt.dw);
      HIP_TRY(hipGetLastError());
      n_cblocks = g.x;
    }
  }
  uint32_t n_ublocks = 0;
  const bool run_usage = usage && e->n_nodes;
  if (run_usage) {
    if (e->has_mixed_keys && !e->d_mixed) return fail(KWK_ESTATE, "kwk_usage_mixed must be called first");
    if (kwk_status st = enqueue_usage(e, now_ns, &n_ublocks, fused ? e->d_agg_masks : nullptr, fused ? n_masks : 0u))
      return st;
    if (fused) n_cblocks = n_ublocks;
  }
  // usage with no nodes: the cluster sums stay what the last kwk_usage left (as before)
  hipLaunchKernelGGL(agg_final_kernel, dim3(1), dim3(1024), 0, e->stream, e->d_count_part, n_cblocks, n_masks,
                     e->d_agg_counts, e->d_usage_part, n_ublocks, e->d_cluster, usage ? (run_usage ? 1u : 2u) : 0u,
                     e->d_cum, e->cum_rows, n_stages, dst);
  HIP_TRY(hipGetLastError());
  *n_out = n_stages + n_masks + (usage ? 2u : 0u);
  return KWK_OK;
}

kwk_status kwk_aggregate_read(kwk_engine* e, double* host_out, uint32_t n) {
  ErrScope es_(e);
  if (!e || (n && !host_out)) return fail(KWK_EINVAL, "null argument");
  if (n > KWK_MAX_STAGES + kMaxCountMasks + 2) return fail(KWK_EINVAL, "more doubles than kwk_aggregate writes");
  if (!e->d_agg) return fail(KWK_ESTATE, "kwk_aggregate must be called first");
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (n) HIP_TRY(hipMemcpy(host_out, e->d_agg, sizeof(double) * n, hipMemcpyDeviceToHost));
  return KWK_OK;
}

// ---- node leases
kwk_status kwk_lease_config(kwk_engine* e, const kwk_lease_params* cfg) {
  ErrScope es_(e);
  if (!e || !cfg) return fail(KWK_EINVAL, "null argument");
  if (cfg->renew_interval_ns <= 0) return fail(KWK_EINVAL, "renew_interval_ns must be > 0");
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (!e->d_lease) {
    HIP_TRY(hipMalloc(&e->d_lease, sizeof(kwk_lease) * (size_t)e->capacity));
    HIP_TRY(hipMalloc(&e->d_lease_op, (size_t)e->capacity));
    HIP_TRY(hipMalloc(&e->d_lease_ops, sizeof(kwk_fired_rec) * (size_t)e->capacity));
    HIP_TRY(hipMalloc(&e->d_lease_nops, 2 * sizeof(uint32_t)));
    HIP_TRY(hipMalloc(&e->d_lease_stats, sizeof(unsigned long long) * 5));
    HIP_TRY(hipMemsetAsync(e->d_lease, 0, sizeof(kwk_lease) * (size_t)e->capacity, e->stream));
    HIP_TRY(hipMemsetAsync(e->d_lease_op, 0, (size_t)e->capacity, e->stream));
    HIP_TRY(hipMemsetAsync(e->d_lease_nops, 0, 2 * sizeof(uint32_t), e->stream));
    HIP_TRY(hipMemsetAsync(e->d_lease_stats, 0, sizeof(unsigned long long) * 5, e->stream));
  }
  e->lease_cfg = *cfg;
  e->lease_on = true;
  return KWK_OK;
}

kwk_status kwk_lease_set(kwk_engine* e, uint32_t first, uint32_t n, const kwk_lease* leases) {
  ErrScope es_(e);
  if (!e || (n && !leases)) return fail(KWK_EINVAL, "null argument");
  if (!e->lease_on) return fail(KWK_ESTATE, "kwk_lease_config must be called first");
  if ((uint64_t)first + n > e->capacity) return fail(KWK_ECAP, "lease range beyond capacity");
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (n) HIP_TRY(upload(e, e->d_lease + first, leases, sizeof(kwk_lease) * n));
  return KWK_OK;
}

// one lease step (enqueue only): the count it writes was zeroed by the previous step's kernel
// (or at kwk_lease_config), and it zeroes the other entry for the next step
static kwk_status enqueue_lease_step(kwk_engine* e, int64_t now_ns, uint64_t seed, uint64_t step) {
  // a fused tick's pod sync (pod stream) may still be reading the previous step's lease results
  if (e->tick_pods && e->tick_pods->tick_pending) HIP_TRY(hipStreamWaitEvent(e->stream, e->tick_pods->ev_podsync, 0));
  ++e->lease_steps;
  const uint32_t cur = e->lease_par;
  e->lease_last = cur;
  if (e->n_active == 0) {
    HIP_TRY(hipMemsetAsync(e->d_lease_nops + cur, 0, sizeof(uint32_t), e->stream));
    return KWK_OK;
  }
  e->lease_par ^= 1u;
  LeaseArgs a;
  a.lease = e->d_lease;
  a.op = e->d_lease_op;
  a.st = e->d_st;
  a.ops = e->d_lease_ops;
  a.n_ops = e->d_lease_nops + cur;
  a.stats = e->d_lease_stats;
  a.fmt = e->fmt;
  a.n = e->n_active;
  a.slot_base = e->slot_base;
  a.key = seed ^ ((uint64_t)e->kind_salt << 32);
  a.step = step;
  a.now = now_ns;
  a.cfg = e->lease_cfg;
  hipLaunchKernelGGL(lease_kernel, dim3((e->n_active + kBlock - 1) / kBlock), dim3(kBlock), 0, e->stream, a,
                     e->d_lease_nops + (cur ^ 1u));
  HIP_TRY(hipGetLastError());
  return KWK_OK;
}

kwk_status kwk_lease_step(kwk_engine* e, int64_t now_ns, uint64_t seed, uint64_t step) {
  ErrScope es_(e);
  if (!e) return fail(KWK_EINVAL, "null engine");
  if (!e->lease_on) return fail(KWK_ESTATE, "kwk_lease_config must be called first");
  if (kwk_status st = set_dev(e)) return st;
  return enqueue_lease_step(e, now_ns, seed, step);
}

kwk_status kwk_lease_fail(kwk_engine* e, int64_t now_ns, uint64_t seed, uint64_t step, uint32_t n, const uint32_t* slots,
                          const kwk_lease* old) {
  ErrScope es_(e);
  if (!e || (n && (!slots || !old))) return fail(KWK_EINVAL, "null argument");
  if (!e->lease_on) return fail(KWK_ESTATE, "kwk_lease_config must be called first");
  if (n == 0) return KWK_OK;
  for (uint32_t j = 0; j < n; ++j)
    if (slots[j] >= e->n_active) return fail(KWK_EINVAL, "slot not active");
  if (kwk_status st = set_dev(e)) return st;
  if (kwk_status st = ensure_stage_buf(e, (size_t)n * (4 + sizeof(kwk_lease)) + 64)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  kwk_lease* s_old = (kwk_lease*)e->d_stage_buf;
  uint32_t* s_slots = (uint32_t*)((char*)e->d_stage_buf + sizeof(kwk_lease) * n);
  HIP_TRY(upload(e, s_old, old, sizeof(kwk_lease) * n));
  HIP_TRY(upload(e, s_slots, slots, 4 * (size_t)n));
  LeaseArgs a;
  a.lease = e->d_lease;
  a.op = e->d_lease_op;
  a.st = e->d_st;
  a.ops = e->d_lease_ops;
  a.n_ops = e->d_lease_nops;
  a.stats = e->d_lease_stats;
  a.fmt = e->fmt;
  a.n = e->n_active;
  a.slot_base = e->slot_base;
  a.key = seed ^ ((uint64_t)e->kind_salt << 32);
  a.step = step;
  a.now = now_ns;
  a.cfg = e->lease_cfg;
  a.n_ops = e->d_lease_nops + e->lease_last;
  hipLaunchKernelGGL(lease_fail_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, e->stream, a, s_slots, s_old, n);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(e->stream));
  return KWK_OK;
}

kwk_status kwk_lease_ops(kwk_engine* e, kwk_fired_rec* out, uint32_t cap, uint32_t* n_out) {
  ErrScope es_(e);
  if (!e || !n_out) return fail(KWK_EINVAL, "null argument");
  if (!e->lease_on) return fail(KWK_ESTATE, "kwk_lease_config must be called first");
  if (kwk_status st = set_dev(e)) return st;
  uint32_t n = 0;
  HIP_TRY(hipMemcpyAsync(&n, e->d_lease_nops + e->lease_last, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  *n_out = n;
  if (!out || n == 0) return KWK_OK;
  if (n > cap) return fail(KWK_ECAP, "lease ops buffer too small: need " + std::to_string(n));
  HIP_TRY(hipMemcpy(out, e->d_lease_ops, sizeof(kwk_fired_rec) * n, hipMemcpyDeviceToHost));
  return KWK_OK;
}

kwk_status kwk_lease_read(kwk_engine* e, uint32_t first, uint32_t n, kwk_lease* out) {
  ErrScope es_(e);
  if (!e || (n && !out)) return fail(KWK_EINVAL, "null argument");
  if (!e->lease_on) return fail(KWK_ESTATE, "kwk_lease_config must be called first");
  if ((uint64_t)first + n > e->capacity) return fail(KWK_EINVAL, "range beyond capacity");
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (n) HIP_TRY(hipMemcpy(out, e->d_lease + first, sizeof(kwk_lease) * n, hipMemcpyDeviceToHost));
  return KWK_OK;
}

kwk_status kwk_lease_stats(kwk_engine* e, kwk_lease_counters* out) {
  ErrScope es_(e);
  if (!e || !out) return fail(KWK_EINVAL, "null argument");
  if (!e->lease_on) return fail(KWK_ESTATE, "kwk_lease_config must be called first");
  if (kwk_status st = set_dev(e)) return st;
  unsigned long long h[5];
  HIP_TRY(hipMemcpyAsync(h, e->d_lease_stats, sizeof(h), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  out->steps = e->lease_steps;
  out->creates = h[1];
  out->renews = h[2];
  out->acquires = h[3];
  out->busy = h[4];
  return KWK_OK;
}

kwk_status kwk_lease_sync_pods(kwk_engine* pods, const kwk_engine* nodes, uint32_t n_nodes, const uint32_t* node_ptr) {
  ErrScope es_(pods);
  if (!pods || !nodes || !node_ptr) return fail(KWK_EINVAL, "null argument");
  if (!nodes->lease_on) return fail(KWK_ESTATE, "node engine has no lease configuration");
  if (n_nodes > nodes->n_active) return fail(KWK_EINVAL, "n_nodes beyond the node engine's objects");
  if (pods->device != nodes->device) return fail(KWK_EINVAL, "pod and node engines on different devices");
  if (node_ptr[0] != 0 || node_ptr[n_nodes] > pods->n_active) return fail(KWK_EINVAL, "node_ptr out of range");
  for (uint32_t j = 0; j < n_nodes; ++j)
    if (node_ptr[j + 1] < node_ptr[j]) return fail(KWK_EINVAL, "node_ptr must be non-decreasing");
  if (kwk_status st = set_dev(pods)) return st;
  if (n_nodes == 0) return KWK_OK;
  if (kwk_status st = ensure_stage_buf(pods, 4 * ((size_t)n_nodes + 1))) return st;
  // the node engine's lease step must be complete before the pods read its results
  HIP_TRY(hipStreamSynchronize(nodes->stream));
  HIP_TRY(hipMemcpyAsync(pods->d_stage_buf, node_ptr, 4 * ((size_t)n_nodes + 1), hipMemcpyHostToDevice, pods->stream));
  hipLaunchKernelGGL(lease_pods_kernel, dim3((n_nodes + kWavesPerBlock - 1) / kWavesPerBlock), dim3(kBlock), 0,
                     pods->stream, pods->d_st, pods->fmt, (const uint32_t*)pods->d_stage_buf, nodes->d_lease_op,
                     nodes->d_lease, nodes->lease_cfg.holder_id, n_nodes);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(pods->stream));
  return KWK_OK;
}

// ---- the fused reconciliation tick (C3): lease step -> pod sync -> node step -> pod step
kwk_status kwk_tick_bind(kwk_engine* pods, const kwk_engine* nodes, uint32_t n_nodes, const uint32_t* node_ptr) {
  ErrScope es_(pods);
  if (!pods || !nodes || !node_ptr) return fail(KWK_EINVAL, "null argument");
  if (pods == nodes) return fail(KWK_EINVAL, "pod and node engines must differ");
  if (!nodes->lease_on) return fail(KWK_ESTATE, "node engine has no lease configuration");
  if (n_nodes > nodes->capacity) return fail(KWK_EINVAL, "n_nodes beyond the node engine's capacity");
  if (pods->device != nodes->device) return fail(KWK_EINVAL, "pod and node engines on different devices");
  if (node_ptr[0] != 0 || node_ptr[n_nodes] > pods->capacity) return fail(KWK_EINVAL, "node_ptr out of range");
  for (uint32_t j = 0; j < n_nodes; ++j)
    if (node_ptr[j + 1] < node_ptr[j]) return fail(KWK_EINVAL, "node_ptr must be non-decreasing");
  if (kwk_status st = set_dev(pods)) return st;
  HIP_TRY(hipStreamSynchronize(pods->stream));
  if (pods->d_tick_ptr) HIP_TRY(hipFree(pods->d_tick_ptr));
  pods->d_tick_ptr = nullptr;
  HIP_TRY(hipMalloc(&pods->d_tick_ptr, 4 * ((size_t)n_nodes + 1)));
  HIP_TRY(upload(pods, pods->d_tick_ptr, node_ptr, 4 * ((size_t)n_nodes + 1)));
  if (!pods->ev_lease) HIP_TRY(hipEventCreateWithFlags(&pods->ev_lease, hipEventDisableTiming));
  if (!pods->ev_podsync) HIP_TRY(hipEventCreateWithFlags(&pods->ev_podsync, hipEventDisableTiming));
  pods->tick_nodes = nodes;
  pods->tick_n_nodes = n_nodes;
  pods->tick_pending = false;
  return KWK_OK;
}

static kwk_status enqueue_tick(kwk_engine* nodes, kwk_engine* pods, int64_t now_ns, uint64_t seed, uint64_t step,
                               uint32_t flags) {
  const bool compact = (flags & (KWK_TICK_COMPACT | KWK_TICK_COMPACT_PACKED)) != 0;
  const bool packed = (flags & KWK_TICK_COMPACT_PACKED) != 0;
  // the previous tick's pod sync must have read the lease results before this lease step
  // rewrites them (cross-stream order by events: no host synchronisation)
  if (pods) nodes->tick_pods = pods;
  if (nodes->lease_on)
    if (kwk_status st = enqueue_lease_step(nodes, now_ns, seed, step)) return st;
  if (pods && pods->tick_n_nodes && nodes->n_active) {
    HIP_TRY(hipEventRecord(pods->ev_lease, nodes->stream));
    HIP_TRY(hipStreamWaitEvent(pods->stream, pods->ev_lease, 0));
    const uint32_t nn = std::min(pods->tick_n_nodes, nodes->n_active);
    hipLaunchKernelGGL(lease_pods_kernel, dim3((nn + kWavesPerBlock - 1) / kWavesPerBlock), dim3(kBlock), 0,
                       pods->stream, pods->d_st, pods->fmt, (const uint32_t*)pods->d_tick_ptr, nodes->d_lease_op,
                       nodes->d_lease, nodes->lease_cfg.holder_id, nn);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(pods->ev_podsync, pods->stream));
    pods->tick_pending = true;
  }
  if (kwk_status st = sweep_compact(nodes, now_ns, seed, step, compact ? (packed ? 1 : 0) : -1)) return st;
  if (pods)
    if (kwk_status st = sweep_compact(pods, now_ns, seed, step, compact ? (packed ? 1 : 0) : -1)) return st;
  return KWK_OK;
}

static kwk_status tick_check(kwk_engine* nodes, kwk_engine* pods) {
  if (!nodes) return fail(KWK_EINVAL, "null node engine");
  if (pods && pods->tick_nodes != nodes) return fail(KWK_ESTATE, "kwk_tick_bind(pods, nodes, ...) must come first");
  return set_dev(nodes);
}

kwk_status kwk_tick(kwk_engine* nodes, kwk_engine* pods, int64_t now_ns, uint64_t seed, uint64_t step, uint32_t flags) {
  ErrScope es_(nodes);
  if (kwk_status st = tick_check(nodes, pods)) return st;
  return enqueue_tick(nodes, pods, now_ns, seed, step, flags);
}

kwk_status kwk_tick_n(kwk_engine* nodes, kwk_engine* pods, uint32_t n, int64_t now0_ns, int64_t dt_ns, uint64_t seed,
                      uint64_t step0, uint32_t flags) {
  ErrScope es_(nodes);
  if (kwk_status st = tick_check(nodes, pods)) return st;
  for (uint32_t k = 0; k < n; ++k)
    if (kwk_status st = enqueue_tick(nodes, pods, now0_ns + (int64_t)k * dt_ns, seed, step0 + k, flags)) return st;
  return KWK_OK;
}

kwk_status kwk_device_ptrs(kwk_engine* e, void** hot, void** fired, void** wave_counts) {
  ErrScope es_(e);
  if (!e) return fail(KWK_EINVAL, "null engine");
  if (hot) *hot = e->d_st;
  if (fired) *fired = e->d_fired;
  if (wave_counts) *wave_counts = e->d_wave_counts;
  return KWK_OK;
}

// ---- timing helpers (HIP events on the engine's own stream; bench.py)
kwk_status kwk_last_sweep(kwk_engine* e, kwk_sweep_info* out) {
  ErrScope es_(e);
  if (!e || !out) return fail(KWK_EINVAL, "null argument");
  *out = e->last_sweep;
  return KWK_OK;
}

kwk_status kwk_stream(kwk_engine* e, void** stream) {
  ErrScope es_(e);
  if (!e || !stream) return fail(KWK_EINVAL, "null argument");
  *stream = (void*)e->stream;
  return KWK_OK;
}

kwk_status kwk_event_record(kwk_engine* e, uint32_t idx) {
  ErrScope es_(e);
  if (!e) return fail(KWK_EINVAL, "null engine");
  if (kwk_status st = set_dev(e)) return st;
  while (e->events.size() <= idx) {
    hipEvent_t ev;
    // timing only: no system-scope release (its L2 write-back idled the stream ~5 us per marker)
    HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableSystemFence));
    e->events.push_back(ev);
  }
  HIP_TRY(hipEventRecord(e->events[idx], e->stream));
  return KWK_OK;
}

kwk_status kwk_event_elapsed(kwk_engine* e, uint32_t a, uint32_t b, float* ms) {
  ErrScope es_(e);
  if (!e || !ms || a >= e->events.size() || b >= e->events.size()) return fail(KWK_EINVAL, "bad event index");
  if (kwk_status st = set_dev(e)) return st;
  HIP_TRY(hipEventSynchronize(e->events[b]));
  HIP_TRY(hipEventElapsedTime(ms, e->events[a], e->events[b]));
  return KWK_OK;
}

uint32_t kwk_abi_version(void) { return KWK_ABI_VERSION; }
uint32_t kwk_tile_objects(void) { return (uint32_t)(kBlock * kMinObjPerThread); }

}  // extern "C"
