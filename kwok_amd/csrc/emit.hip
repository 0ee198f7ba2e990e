// Device patch emission (include/kwok_emit.h): the merge-patch bytes of a step's fired objects,
// expanded from per-(class, template) skeletons on the engine's stream.
//
// Reference: playStage renders each fired object's Stage patches (pkg/utils/lifecycle/
// next.go:73-160, pkg/utils/gotpl/renderer.go:59-124) — here the host's one-time skeleton build
// (patch.cpp: kwk_patch_skeleton / kwk_patch_object_values) leaves only Now and the objects' call
// values (funcPodIPWith / funcNodeIPWith, pod_controller.go:563-600) to fill per fire.
//
// Three launches per list, sized by the device-resident record count (no host round trip):
//   emit_size_kernel   per 256-record tile (one per thread): items and bytes (a gather of one 8-byte
//                      word per record)
//   emit_scan_kernel   one workgroup: exclusive bases of the tiles, the totals
//   emit_write_kernel  per tile again: each record's items / offsets, its guard word, then each wave
//                      writes its 64 records' bytes (one contiguous span), 64 lanes over every literal
//                      run and value, through an LDS window that leaves as 16-byte stores
// The skeleton pieces and literal runs are staged in LDS when they fit (12 KiB of literals).
// Roofline: HBM-bound on the patch bytes written (plus 8 bytes read per record and the literal
// runs, L2-resident); the byte copy is 1-byte stores coalesced per wave.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/kwok_emit.h"
#include "timefmt.hpp"

namespace {

thread_local std::string g_err;
thread_local std::string* tl_err = nullptr;
struct ErrScope {
  std::string* prev;
  explicit ErrScope(std::string* target) : prev(tl_err) { tl_err = target; }
  ~ErrScope() { tl_err = prev; }
};
kwk_status fail(kwk_status code, const std::string& msg) {
  g_err = msg;
  if (tl_err) *tl_err = msg;
  return code;
}
#define HIP_TRY(x)                                                                                \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) return fail(KWK_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

constexpr uint32_t kBlock = 256, kTile = kBlock;  // records per tile: one per thread, 64 per wave
constexpr uint32_t kWaves = kBlock / 64, kWaveRecs = kTile / kWaves;
constexpr uint32_t kMaxStageTpl = 16;  // templates of one stage (an item mask per record)
constexpr uint32_t kScanBlock = 1024;
constexpr uint32_t kNowWords = 10;      // Now() text (< 40 bytes) as dwords in LDS
constexpr uint32_t kLdsPieces = 256;    // skeleton tables staged in LDS when they fit
constexpr uint32_t kLdsLits = 8192;
constexpr uint32_t kLdsSkels = 64;
constexpr uint32_t kRecSk = 4;          // skeletons of a record's emitted items kept in LDS (more: looked up)

struct Prog {
  const uint32_t* stage_tpl_ptr;
  const uint16_t* stage_tpl;
  const uint8_t* stage_delete;
  const int32_t* skel_of;
  const kwk_emit_skel* skels;
  const kwk_emit_piece* pieces;
  const char* lits;
  const uint8_t* fresh;
  uint8_t* const* cols;
  const uint32_t* stride;
  uint32_t n_classes, n_templates, n_stages, n_pieces;
  uint32_t n_lits, n_cols, n_skels;
};

struct EmitArgs {
  Prog p;
  const kwk_fired_rec* recs;  // or
  const uint32_t* packed;
  const uint32_t* count;
  uint64_t* words;
  uint32_t capacity;
  uint32_t max_recs;                 // records the tile arrays cover (capacity rounded up)
  uint32_t* tile_items;              // per tile: items, then (emit_scan_kernel) the exclusive base
  unsigned long long* tile_bytes;    // per tile: bytes, then the base
  unsigned long long* totals;        // [0] items, [1] bytes, [2] the list is longer than max_recs, [3] items emitted
  kwk_emit_item* items;
  uint64_t* offsets;
  char* out;
  unsigned long long cap_items, cap_bytes;
  uint32_t now_len;
  char now[40];
  uint32_t lencache;                 // words' bits 24-31 cache the value lengths (emit_lens_kernel)
};

// per skeleton (LDS, built per block for this call's Now length): x = its fixed bytes (literal runs
// and Now) | value slots << 24 (kSkszPieces: more than 4, count them piece by piece), y = the slots'
// value columns, a byte each
constexpr uint32_t kSkszPieces = 0xFFu;
__device__ __forceinline__ void build_sksz(const EmitArgs& a, const kwk_emit_piece* pieces, uint2* sksz) {
  for (uint32_t k = threadIdx.x; k < a.p.n_skels && k < kLdsSkels; k += blockDim.x) {
    const kwk_emit_skel S = a.p.skels[k];
    uint32_t fixed = 0, nv = 0, cols = 0;
    for (uint32_t q = 0; q < S.n_pieces; ++q) {
      const kwk_emit_piece P = pieces[S.first_piece + q];
      fixed += P.lit_len + (P.slot == 0 ? a.now_len : 0u);
      if (P.slot != 0 && P.slot != KWK_EMIT_NO_SLOT) {
        if (nv < 4u) cols |= (uint32_t)(P.slot - 1u) << (8u * nv);
        ++nv;
      }
    }
    sksz[k] = make_uint2(nv > 4u || fixed >= (1u << 24) ? kSkszPieces << 24 : fixed | nv << 24, cols);
  }
}

// the skeleton pieces and literal runs a kernel reads: LDS copies when the program's fit
struct Tables {
  const kwk_emit_piece* pieces;
  const char* lits;
  const uint2* sksz = nullptr;  // per-skeleton sizes (build_sksz), when staged
};

template <bool kLds, bool kLits = true>
__device__ __forceinline__ Tables stage_tables(const EmitArgs& a, kwk_emit_piece* s_pieces, uint32_t* s_lits,
                                               uint2* s_sksz) {
  if constexpr (kLds) {
    for (uint32_t j = threadIdx.x; j < a.p.n_pieces; j += blockDim.x) s_pieces[j] = a.p.pieces[j];
    build_sksz(a, a.p.pieces, s_sksz);
    if constexpr (!kLits) {  // the literal runs stay in global memory
      __syncthreads();
      return Tables{s_pieces, a.p.lits, s_sksz};
    }
    const uint32_t nw = (a.p.n_lits + 3u) / 4u;
    for (uint32_t j = threadIdx.x; j < nw; j += blockDim.x) {
      uint32_t w = 0;
      for (uint32_t b = 0; b < 4u; ++b)
        if (4u * j + b < a.p.n_lits) w |= (uint32_t)(uint8_t)a.p.lits[4u * j + b] << (8u * b);
      s_lits[j] = w;
    }
    __syncthreads();
    return Tables{s_pieces, reinterpret_cast<const char*>(s_lits), s_sksz};
  } else {
    return Tables{a.p.pieces, a.p.lits, nullptr};
  }
}

struct Rec {
  uint32_t slot, stage;
  bool valid;
};

__device__ __forceinline__ Rec fetch(const EmitArgs& a, uint32_t r) {
  Rec x;
  if (a.packed) {
    const uint32_t v = a.packed[r];
    x.slot = v & 0x7FFFFFFu;
    x.stage = v >> 27;
  } else {
    const kwk_fired_rec f = a.recs[r];
    x.slot = f.slot;
    x.stage = f.stage;
  }
  x.valid = x.slot < a.capacity;
  return x;
}

// where a record's call values are read: the value columns in global memory, or the rows the
// write kernel staged in LDS for the tile (kLdsCols columns of 16 bytes)
constexpr uint32_t kLdsCols = 2;
struct Vals {
  const uint8_t* lds;  // [kLdsCols][kTile][16] or null
  uint32_t lr;         // the record's index in the tile
  uint32_t lens = 0xFFu;  // the word's cached value lengths (kLenCache): column 0 | column 1 << 4; 0xFF: none
  __device__ __forceinline__ const uint8_t* row(const EmitArgs& a, uint32_t c, uint32_t slot) const {
    if (lds) return lds + ((uint64_t)c * kTile + lr) * 16u;
    return a.p.cols[c] + (uint64_t)slot * a.p.stride[c];
  }
  // a value's length byte (0xFF: unusable), from the cache when the word holds it
  __device__ __forceinline__ uint32_t len(const EmitArgs& a, uint32_t c, uint32_t slot) const {
    if (lens != 0xFFu && c < 2u) return c ? lens >> 4 : lens & 15u;
    return row(a, c, slot)[0];
  }
};

// Cached value lengths: with at most two value columns of 16-byte rows, a slot's word keeps both
// rows' text lengths in bits 24-31 (column 0 | column 1 << 4; 0xFF when either is unusable or both
// are 15, i.e. "read the rows"), refreshed by the host entry points that write words or rows, so
// that the size kernel gathers one word per record instead of the word and two rows
__global__ void emit_lens_kernel(uint64_t* __restrict__ words, uint8_t* const* __restrict__ cols, uint32_t n_cols,
                                 uint32_t first, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t s = (uint64_t)first + i;
    const uint32_t l0 = n_cols > 0 ? cols[0][s * 16u] : 0u, l1 = n_cols > 1 ? cols[1][s * 16u] : 0u;
    const uint32_t code = (l0 <= 15u && l1 <= 15u) ? (l0 | l1 << 4) : 0xFFu;
    words[s] = (words[s] & ~(0xFFull << 24)) | (uint64_t)code << 24;
  }
}

// bytes of skeleton k for this slot, or -1 when a value is unusable
__device__ __forceinline__ long long skel_bytes(const EmitArgs& a, const Tables& T, uint32_t k, uint32_t slot,
                                                const Vals& V = Vals{nullptr, 0}) {
  if (T.sksz) {
    const uint2 z = T.sksz[k];
    const uint32_t nv = z.x >> 24;
    if (nv != kSkszPieces) {
      long long b = z.x & 0xFFFFFFu;
      for (uint32_t i = 0; i < nv; ++i) {
        const uint32_t len = V.len(a, (z.y >> (8u * i)) & 0xFFu, slot);
        if (len == 0xFFu) return -1;
        b += len;
      }
      return b;
    }
  }
  const kwk_emit_skel S = a.p.skels[k];
  long long b = 0;
  for (uint32_t q = 0; q < S.n_pieces; ++q) {
    const kwk_emit_piece P = T.pieces[S.first_piece + q];
    b += P.lit_len;
    if (P.slot == 0) {
      b += a.now_len;
    } else if (P.slot != KWK_EMIT_NO_SLOT) {
      const uint32_t len = V.len(a, P.slot - 1u, slot);
      if (len == 0xFFu) return -1;
      b += len;
    }
  }
  return b;
}

__device__ __forceinline__ int skel_index(const EmitArgs& a, uint64_t w, uint32_t tid) {
  const uint32_t cls = (uint32_t)(w & 0xFFFFu), g = (uint32_t)(w >> 16) & 0xFFu;
  if (cls >= a.p.n_classes || tid >= 32u || !((w >> (32u + tid)) & 1u)) return -1;
  const int k = a.p.skel_of[cls * a.p.n_templates + tid];
  if (k < 0) return -1;
  const uint32_t need = a.p.skels[k].need;
  return (g & need) == need ? k : -1;
}

struct Size {
  uint32_t items, ok;  // ok: bit j = the stage's j-th template is emitted here
  unsigned long long bytes;
};

__device__ __forceinline__ Size rec_size(const EmitArgs& a, const Tables& T, const Rec& x, uint64_t w,
                                         const Vals& V = Vals{nullptr, 0}) {
  Size s{0u, 0u, 0ull};
  if (x.stage >= a.p.n_stages) return s;
  const uint32_t t0 = a.p.stage_tpl_ptr[x.stage], t1 = a.p.stage_tpl_ptr[x.stage + 1];
  for (uint32_t j = t0; j < t1; ++j) {
    ++s.items;
    const int k = x.valid ? skel_index(a, w, a.p.stage_tpl[j]) : -1;
    if (k < 0) continue;
    const long long b = skel_bytes(a, T, (uint32_t)k, x.slot, V);
    if (b < 0) continue;
    s.ok |= 1u << (j - t0);
    s.bytes += (unsigned long long)b;
  }
  return s;
}

// One lane's output stream (a record written by the thread that sized it), assembled four bytes
// at a time in a 16-byte register window {lo, hi}: every append is one shifted OR at the window's
// byte position (no per-byte work), a full window leaves as one 16-byte store.  The stream starts
// at global byte g0: the window starts with g0 & 15 phantom bytes, so that every store is 16-byte
// aligned; the first window (it shares its 16 bytes with the record before) and the last one (the
// record after) are written with dword and byte stores covering exactly the record's bytes.
struct Acc {
  char* out;
  unsigned long long w0;  // global position of the window's byte 0 (16-byte aligned)
  uint64_t lo, hi;
  uint32_t n;             // bytes in the window (incl. the phantom head)
  uint32_t head;          // phantom bytes of the first window (0 once it has left)
  __device__ __forceinline__ Acc(char* o, unsigned long long g0)
      : out(o), w0(g0 & ~15ull), lo(0), hi(0), n((uint32_t)(g0 & 15u)), head((uint32_t)(g0 & 15u)) {}
  // bytes [b0, b1) of the window at w0, for a window shared with a neighbouring record
  __device__ __forceinline__ void partial(uint32_t b0, uint32_t b1) const {
    for (uint32_t b = b0; b < b1;) {
      const uint64_t v = b < 8u ? lo : hi;
      const uint32_t sh = 8u * (b & 7u);
      if ((b & 3u) == 0u && b + 4u <= b1) {
        *reinterpret_cast<uint32_t*>(out + w0 + b) = (uint32_t)(v >> sh);
        b += 4u;
      } else {
        out[w0 + b] = (char)((v >> sh) & 0xFFu);
        ++b;
      }
    }
  }
  __device__ __forceinline__ void flush_full() {
    if (head) {
      partial(head, 16u);
      head = 0;
    } else {
      *reinterpret_cast<uint4*>(out + w0) = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
    }
  }
  // `cnt` (1..4) bytes, low byte first; w's bytes above cnt are zero
  __device__ __forceinline__ void put(uint32_t w, uint32_t cnt) {
    const uint64_t x = (uint64_t)w;
    const uint32_t sh = 8u * n;  // 0..120
    if (sh < 64u) {
      lo |= x << sh;
      hi |= sh > 32u ? x >> (64u - sh) : 0ull;
    } else {
      hi |= x << (sh - 64u);
    }
    const uint64_t spill = sh > 96u ? x >> (128u - sh) : 0ull;  // bytes past the window
    n += cnt;
    if (n >= 16u) {
      flush_full();
      w0 += 16u;
      lo = spill;
      hi = 0;
      n -= 16u;
    }
  }
  __device__ __forceinline__ void finish() const { partial(head, n); }
};

__device__ __forceinline__ uint32_t low_bytes(uint32_t w, uint32_t cnt) {
  return cnt >= 4u ? w : w & ((1u << (8u * cnt)) - 1u);
}

// `len` bytes starting at byte `off` of a dword array (aligned dword reads, one per step, joined by
// alignbyte): the literal runs (LDS or global, 16 bytes of zero padding after them), Now (LDS) and
// a value row's text (byte 1 on)
__device__ __forceinline__ void put_run(Acc& o, const uint32_t* __restrict__ src, uint32_t off, uint32_t len) {
  if (!len) return;
  uint32_t d = off >> 2;
  const uint32_t sh = off & 3u;
  uint32_t cur = src[d];
  for (uint32_t k = 0; k < len; k += 4u) {
    const uint32_t nxt = src[d + 1u];
    const uint32_t w = sh ? __builtin_amdgcn_alignbyte(nxt, cur, sh) : cur;
    const uint32_t cnt = min(4u, len - k);
    o.put(low_bytes(w, cnt), cnt);
    cur = nxt;
    ++d;
  }
}

// one emitted item by one lane
__device__ __forceinline__ void lane_skel(const EmitArgs& a, const Tables& T, const kwk_emit_skel& S, uint32_t slot,
                                          const uint32_t* s_now, const Vals& V, Acc& o) {
  const uint32_t* L = reinterpret_cast<const uint32_t*>(T.lits);
  for (uint32_t q = 0; q < S.n_pieces; ++q) {
    const kwk_emit_piece P = T.pieces[S.first_piece + q];
    put_run(o, L, P.lit_off, P.lit_len);
    if (P.slot == 0) {
      put_run(o, s_now, 0u, a.now_len);
    } else if (P.slot != KWK_EMIT_NO_SLOT) {
      const uint8_t* v = V.row(a, P.slot - 1u, slot);  // [length][text]: rows 16-byte aligned in LDS, 4 in global
      const uint32_t* v32 = reinterpret_cast<const uint32_t*>(v);
      put_run(o, v32, 1u, (uint32_t)(v32[0] & 0xFFu));
    }
  }
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_incl(T v, uint32_t lane) {
  for (int o = 1; o < 64; o <<= 1) {
    const T y = __shfl_up(v, o);
    if (lane >= (uint32_t)o) v += y;
  }
  return v;
}

template <bool kLds>
__global__ __launch_bounds__(kBlock) void emit_size_kernel(EmitArgs a) {
  __shared__ kwk_emit_piece s_pieces[kLds ? kLdsPieces : 1];
  __shared__ uint32_t s_lits[kLds ? kLdsLits / 4 : 1];
  __shared__ uint2 s_sksz[kLds ? kLdsSkels : 1];
  __shared__ uint32_t s_i[kWaves];
  __shared__ unsigned long long s_b[kWaves];
  const Tables T = stage_tables<kLds>(a, s_pieces, s_lits, s_sksz);
  const uint32_t n = min(*a.count, a.max_recs), n_tiles = (n + kTile - 1) / kTile;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  for (uint32_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    uint32_t it = 0;
    unsigned long long by = 0;
    const uint32_t r = t * kTile + threadIdx.x;
    if (r < n) {
      const Rec x = fetch(a, r);
      const uint64_t w = x.valid ? a.words[x.slot] : 0ull;
      const Size s = rec_size(a, T, x, w, Vals{nullptr, 0u, a.lencache ? (uint32_t)(w >> 24) & 0xFFu : 0xFFu});
      it = s.items;
      by = s.bytes;
    }
    it = wave_sum(it);
    by = wave_sum(by);
    if (lane == 0) {
      s_i[wave] = it;
      s_b[wave] = by;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t ti = 0;
      unsigned long long tb = 0;
      for (uint32_t w = 0; w < kWaves; ++w) {
        ti += s_i[w];
        tb += s_b[w];
      }
      a.tile_items[t] = ti;
      a.tile_bytes[t] = tb;
    }
    __syncthreads();
  }
}

// 8 consecutive tiles per thread: 8192 tiles per pass of the one workgroup
constexpr uint32_t kScanPer = 8;
__global__ __launch_bounds__(kScanBlock) void emit_scan_kernel(EmitArgs a) {
  __shared__ uint32_t s_i[kScanBlock / 64];
  __shared__ unsigned long long s_b[kScanBlock / 64];
  const uint32_t n = min(*a.count, a.max_recs), n_tiles = (n + kTile - 1) / kTile;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t run_i = 0;
  unsigned long long run_b = 0;
  for (uint32_t base = 0; base < n_tiles; base += kScanBlock * kScanPer) {
    const uint32_t t0 = base + threadIdx.x * kScanPer;
    uint32_t vi[kScanPer];
    unsigned long long vb[kScanPer];
    uint32_t si = 0;
    unsigned long long sb = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) {
      vi[k] = t0 + k < n_tiles ? a.tile_items[t0 + k] : 0u;
      vb[k] = t0 + k < n_tiles ? a.tile_bytes[t0 + k] : 0ull;
      si += vi[k];
      sb += vb[k];
    }
    const uint32_t ii = wave_incl(si, lane);
    const unsigned long long ib = wave_incl(sb, lane);
    if (lane == 63) {
      s_i[wave] = ii;
      s_b[wave] = ib;
    }
    __syncthreads();
    uint32_t pi = 0, ti = 0;
    unsigned long long pb = 0, tb = 0;
    for (uint32_t w = 0; w < kScanBlock / 64; ++w) {
      if (w < wave) {
        pi += s_i[w];
        pb += s_b[w];
      }
      ti += s_i[w];
      tb += s_b[w];
    }
    uint32_t ei = run_i + pi + ii - si;
    unsigned long long eb = run_b + pb + ib - sb;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) {
      if (t0 + k < n_tiles) {
        a.tile_items[t0 + k] = ei;
        a.tile_bytes[t0 + k] = eb;
      }
      ei += vi[k];
      eb += vb[k];
    }
    run_i += ti;
    run_b += tb;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    a.totals[0] = run_i;
    a.totals[1] = run_b;
    a.totals[2] = *a.count > a.max_recs ? 1ull : 0ull;
    a.totals[3] = 0;
  }
}

// ---- the chunk writer (the default when the program's tables fit in LDS) ----
// Per call, every block renders each skeleton once into an LDS template with Now filled in:
// consecutive literal runs and Now slots merge into one template run, so a skeleton is a short
// list of segments (template run | value column c).  A record's bytes are the concatenation of its
// items' segments; the thread that sized the record writes it as aligned 16-byte chunks: each chunk
// gathers the bytes of the segments overlapping it (16 unaligned bytes from LDS: five aligned dword
// reads joined by alignbyte, merged under a byte mask), and leaves as one 16-byte store.  The first
// and the last chunk of a record share their 16 bytes with the neighbouring records: they are
// written at the end with dword / byte stores covering exactly the record's bytes.  Every store
// goes through a buffer resource with the offset out of range where a lane has nothing to store,
// so no store sits under a divergent branch.
constexpr uint32_t kTplBytes = 8192;                     // rendered templates in LDS
constexpr uint32_t kMaxSegs = 2 * kLdsPieces + kLdsSkels;  // segments of every skeleton
constexpr uint32_t kSegValue = 1u << 24;                 // segment kind: value column (y >> 24) - 1
constexpr uint32_t kOOB = 0x80000000u;                   // buffer offset past the resource: no store

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint8_t lds_u8;
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)p;
}
__device__ __forceinline__ uint32_t lds_rd(uint32_t a) { return *(const lds_u32*)(size_t)a; }

// the 16 bytes at LDS byte address A (any alignment; bytes outside the arrays are don't-care)
__device__ __forceinline__ void lds_load16(uint32_t A, uint32_t (&y)[4]) {
  const uint32_t d = A & ~3u, sh = A & 3u;
  const uint32_t w0 = lds_rd(d), w1 = lds_rd(d + 4u), w2 = lds_rd(d + 8u), w3 = lds_rd(d + 12u), w4 = lds_rd(d + 16u);
  y[0] = __builtin_amdgcn_alignbyte(w1, w0, sh);
  y[1] = __builtin_amdgcn_alignbyte(w2, w1, sh);
  y[2] = __builtin_amdgcn_alignbyte(w3, w2, sh);
  y[3] = __builtin_amdgcn_alignbyte(w4, w3, sh);
}

// a if bit is 0, b if 1 (bit: 0 or 1)
__device__ __forceinline__ uint32_t blend(uint32_t a, uint32_t b, uint32_t bit) { return a ^ ((a ^ b) & (0u - bit)); }

// byte mask of [lo, hi) (0 <= lo <= hi <= 16) as two 64-bit halves
__device__ __forceinline__ uint64_t ones_bytes(uint32_t n) { return n >= 8u ? ~0ull : (1ull << (8u * n)) - 1ull; }
__device__ __forceinline__ void merge16(uint32_t (&x)[4], const uint32_t (&y)[4], uint32_t lo, uint32_t hi) {
  const uint64_t ml = ones_bytes(min(hi, 8u)) & ~ones_bytes(min(lo, 8u));
  const uint64_t mh = ones_bytes(hi > 8u ? hi - 8u : 0u) & ~ones_bytes(lo > 8u ? lo - 8u : 0u);
  x[0] = (y[0] & (uint32_t)ml) | (x[0] & ~(uint32_t)ml);
  x[1] = (y[1] & (uint32_t)(ml >> 32)) | (x[1] & ~(uint32_t)(ml >> 32));
  x[2] = (y[2] & (uint32_t)mh) | (x[2] & ~(uint32_t)mh);
  x[3] = (y[3] & (uint32_t)(mh >> 32)) | (x[3] & ~(uint32_t)(mh >> 32));
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// bytes [b0, b1) of the chunk x stored at offset `at` of the resource (dword stores where whole
// dwords lie inside, byte stores for the rest; all with out-of-range offsets where not needed)
__device__ __forceinline__ void store_part(const __amdgpu_buffer_rsrc_t r, uint32_t at, const uint32_t (&x)[4], uint32_t b0,
                                           uint32_t b1, bool live) {
#pragma unroll
  for (uint32_t k = 0; k < 4u; ++k) {
    const bool whole = live && 4u * k >= b0 && 4u * k + 4u <= b1;
    __builtin_amdgcn_raw_buffer_store_b32(x[k], r, whole ? at + 4u * k : kOOB, 0, 0);
  }
  // the partial dword at the front (bytes b0 .. its dword's end) and at the back (its dword's start .. b1)
  const uint32_t f0 = b0, f1 = min(b1, (b0 + 3u) & ~3u);
  const uint32_t e0 = max(b0, b1 & ~3u), e1 = b1;
  const uint32_t x0 = x[0], x1 = x[1], x2 = x[2], x3 = x[3];
  auto byte_at = [=](uint32_t b) __attribute__((always_inline)) {  // mask blends, not an indexed register array
    const uint32_t d = blend(blend(x0, x1, (b >> 2) & 1u), blend(x2, x3, (b >> 2) & 1u), (b >> 3) & 1u);
    return (d >> (8u * (b & 3u))) & 0xFFu;
  };
#pragma unroll
  for (uint32_t j = 0; j < 3u; ++j) {
    const uint32_t bf = f0 + j, be = e0 + j;
    const uint32_t vf = byte_at(bf), ve = byte_at(be);
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)vf, r, live && bf < f1 ? at + bf : kOOB, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)ve, r, live && be < e1 && (be & 3u) < (e1 & 3u) ? at + be : kOOB, 0, 0);
  }
}

// chunk idx (0..7, per lane) of a 128-byte line buffer: mask blends (a select of two array elements
// would be folded into an indexed load, and the buffer would leave the registers for scratch)
constexpr uint32_t kLine = 128;            // bytes per burst of the line writer: one L2 line (64-byte bursts
constexpr uint32_t kLineChunks = kLine / 16;  // left the L2 writing half lines back: r5h, 1.35x the bytes)
__device__ __forceinline__ void pick_chunk(const uint32_t (&buf)[kLineChunks][4], uint32_t idx, uint32_t (&x)[4]) {
  static_assert(kLineChunks == 8, "a three-level blend tree");
  const uint32_t b0 = idx & 1u, b1 = (idx >> 1) & 1u, b2 = (idx >> 2) & 1u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t t0 = blend(buf[0][k], buf[1][k], b0), t1 = blend(buf[2][k], buf[3][k], b0);
    const uint32_t t2 = blend(buf[4][k], buf[5][k], b0), t3 = blend(buf[6][k], buf[7][k], b0);
    x[k] = blend(blend(t0, t1, b1), blend(t2, t3, b1), b2);
  }
}

// bytes [lo, hi) (0 <= lo < hi <= kLine) of a line buffer at resource offset L: whole chunks
// as 16-byte stores, the (at most two) chunks cut by lo / hi with dword and byte stores
__device__ __forceinline__ void store_line_part(const __amdgpu_buffer_rsrc_t r, uint32_t L, const uint32_t (&buf)[kLineChunks][4],
                                                uint32_t lo, uint32_t hi, bool live) {
#pragma unroll
  for (uint32_t i = 0; i < kLineChunks; ++i) {
    const bool whole = live && 16u * i >= lo && 16u * i + 16u <= hi;
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{buf[i][0], buf[i][1], buf[i][2], buf[i][3]}, r, whole ? L + 16u * i : kOOB,
                                           0, 0);
  }
  const uint32_t il = lo >> 4, ih = (hi - 1u) >> 4;
  uint32_t x[4];
  pick_chunk(buf, il, x);
  const bool cut_lo = (lo & 15u) || (il == ih && (hi & 15u));
  store_part(r, L + 16u * il, x, lo - 16u * il, min(hi - 16u * il, 16u), live && cut_lo);
  pick_chunk(buf, ih, x);
  const bool cut_hi = (hi & 15u) && ih != il;
  store_part(r, L + 16u * ih, x, 0u, hi - 16u * ih, live && cut_hi);
}


// the tile's bytes from record `rec` on, segment by segment in output order: each record's items'
// skeleton segment lists (template runs in LDS; value column c of record r at vals0 + (c * kTile +
// r) * 16), records of no bytes skipped
struct SegIter {
  const uint2* skseg;
  const uint2* seg;
  const int16_t* sk;       // per record: its skeleton ids (kRecSk each)
  const uint8_t* nsk;      // per record: its items
  uint32_t vals0;
  uint32_t rec, n_sk, j, q, n, f;
  uint32_t sa, sb;         // the current segment's output range [sa, sb) ...
  uint32_t src;            // ... and the LDS address of its first byte
  __device__ __forceinline__ void next() {  // the next non-empty segment (sa = ~0 past the tile's last)
    uint32_t a0 = sb, b0 = 0xFFFFFFFFu, s0 = src;
    bool found = false;
    while (!found) {
      if (q < n) {
        const uint2 sg = seg[f + q];
        ++q;
        uint32_t so = sg.x, len = sg.y;
        if (sg.y >= kSegValue) {
          const uint32_t row = vals0 + (sg.x * kTile + rec) * 16u;
          so = row + 1u;
          len = lds_rd(row) & 0xFFu;
        }
        if (len) {
          b0 = a0 + len;
          s0 = so;
          found = true;
        }
      } else if (j < n_sk) {
        const uint2 ss = skseg[sk[rec * kRecSk + j]];
        f = ss.x;
        n = ss.y;
        q = 0;
        ++j;
      } else if (rec + 1u < kTile) {  // the next record: its bytes follow these
        ++rec;
        n_sk = nsk[rec];
        j = q = n = 0;
      } else {
        break;
      }
    }
    sa = found ? a0 : 0xFFFFFFFFu;
    sb = b0;
    src = s0;
  }
};

// merge16 with the byte masks from two LDS tables: bytes >= lo (mlo[lo]) and bytes < hi (mhi[hi])
__device__ __forceinline__ void merge16_lut(uint32_t (&x)[4], const uint32_t (&y)[4], uint32_t lo, uint32_t hi,
                                            uint32_t mlo, uint32_t mhi) {
  const u32x4 a = *(const __attribute__((address_space(3))) u32x4*)(size_t)(mlo + 16u * lo);
  const u32x4 b = *(const __attribute__((address_space(3))) u32x4*)(size_t)(mhi + 16u * hi);
  const uint32_t m0 = a.x & b.x, m1 = a.y & b.y, m2 = a.z & b.z, m3 = a.w & b.w;
  x[0] = __builtin_amdgcn_bitop3_b32(y[0], x[0], m0, 0xe4);  // m ? y : x, bit by bit
  x[1] = __builtin_amdgcn_bitop3_b32(y[1], x[1], m1, 0xe4);
  x[2] = __builtin_amdgcn_bitop3_b32(y[2], x[2], m2, 0xe4);
  x[3] = __builtin_amdgcn_bitop3_b32(y[3], x[3], m3, 0xe4);
}

// the 16-byte chunks of the line at L, gathered from the segments overlapping them
__device__ __forceinline__ void produce_line(SegIter& it, uint32_t L, uint32_t (&buf)[kLineChunks][4], uint32_t mlo,
                                             uint32_t mhi) {
#pragma unroll
  for (uint32_t i = 0; i < kLineChunks; ++i) {
    const uint32_t P = L + 16u * i;
    uint32_t x0 = 0u, x1 = 0u, x2 = 0u, x3 = 0u;
    while (it.sa < P + 16u) {
      if (it.sb > P) {
        uint32_t y[4], x[4] = {x0, x1, x2, x3};
        lds_load16(it.src + P - it.sa, y);  // (bytes before the segment are masked out)
        merge16_lut(x, y, it.sa > P ? it.sa - P : 0u, min(it.sb - P, 16u), mlo, mhi);
        x0 = x[0];
        x1 = x[1];
        x2 = x[2];
        x3 = x[3];
      }
      if (it.sb > P + 16u) break;  // the segment continues into the next chunk
      it.next();
    }
    buf[i][0] = x0;
    buf[i][1] = x1;
    buf[i][2] = x2;
    buf[i][3] = x3;
  }
}

// Each thread writes the record it sized.  kChunk (the default when the program's tables fit in
// LDS): the line writer above — the record's bytes gathered 16 at a time from its items' segments
// (the skeletons' rendered templates and its value rows, all in LDS) and stored kLine bytes at a
// time.  (The first version, 16-byte stores as each chunk filled, left the L2 writing half-filled
// lines back and refilling them: r5e, 2x the patch bytes written; a wave writing its records'
// span together, lane L taking chunks L, L + 64, ..., stored whole lines but spent ~4x the VALU
// finding each chunk's record and segment: r5f, 3.1 vs 2.4 ms.)  Records of more than kRecSk items
// and !kChunk: Acc, four bytes per append.  kLds: the skeleton tables and the records' call-value
// rows (at most kLdsCols columns of 16 bytes) staged in LDS
template <bool kLds, bool kChunk>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kChunk ? 5 : 1))) void emit_write_kernel(EmitArgs a) {
  static_assert(kLds || !kChunk, "the chunk writer reads its tables from LDS");
  __shared__ __attribute__((aligned(16))) uint32_t s_tpl[kChunk ? kTplBytes / 4 + 8 : 1];
  __shared__ uint2 s_seg[kChunk ? kMaxSegs : 1];
  __shared__ uint2 s_skseg[kChunk ? kLdsSkels : 1];
  __shared__ uint16_t s_pofs[kChunk ? kLdsPieces : 1];
  __shared__ uint2 s_tsz[kChunk ? kLdsSkels : 1];
  __shared__ __attribute__((aligned(16))) uint4 s_vals[kLds ? kLdsCols * kTile : 1];
  __shared__ kwk_emit_skel s_skels[kLds ? kLdsSkels : 1];
  __shared__ int16_t s_sk[kTile * kRecSk];
  __shared__ uint8_t s_nsk[kChunk ? kTile : 1];  // items per record (the line writer's iterator)
  __shared__ uint32_t s_tend;                    // the tile's bytes end (relative to its 16-byte aligned base)
  __shared__ kwk_emit_piece s_pieces[kLds ? kLdsPieces : 1];
  __shared__ uint32_t s_lits[kLds && !kChunk ? kLdsLits / 4 : 1];
  __shared__ uint2 s_sksz[kLds ? kLdsSkels : 1];
  __shared__ uint32_t s_wi[kWaves];
  __shared__ unsigned long long s_wb[kWaves];
  __shared__ uint32_t s_now[kNowWords];
  __shared__ uint4 s_mlo[kChunk ? 17 : 1], s_mhi[kChunk ? 17 : 1];  // merge16_lut's byte masks
  const uint32_t n = min(*a.count, a.max_recs), n_tiles = (n + kTile - 1) / kTile;
  const unsigned long long tot_i = a.totals[0], tot_b = a.totals[1];
  if (tot_i > a.cap_items || tot_b > a.cap_bytes || a.totals[2]) return;  // KWK_ECAP: nothing is written
  if constexpr (kLds)
    for (uint32_t j = threadIdx.x; j < a.p.n_skels; j += blockDim.x) s_skels[j] = a.p.skels[j];
  if (threadIdx.x < kNowWords) {
    uint32_t w = 0;
    for (uint32_t b = 0; b < 4u; ++b) w |= (uint32_t)(uint8_t)a.now[4u * threadIdx.x + b] << (8u * b);
    s_now[threadIdx.x] = w;
  }
  const Tables T = stage_tables<kLds, !kChunk>(a, s_pieces, s_lits, s_sksz);
  __syncthreads();  // s_skels, s_now
  const kwk_emit_skel* skels = kLds ? s_skels : a.p.skels;
  if constexpr (kChunk) {
    if (threadIdx.x < 34u) {  // mlo[t]: bytes >= t; mhi[t]: bytes < t
      const uint32_t t = threadIdx.x % 17u;
      uint32_t m[4];
      for (uint32_t k = 0; k < 4u; ++k) {
        m[k] = 0;
        for (uint32_t b = 0; b < 4u; ++b) {
          const uint32_t byte = 4u * k + b;
          if (threadIdx.x < 17u ? byte >= t : byte < t) m[k] |= 0xFFu << (8u * b);
        }
      }
      (threadIdx.x < 17u ? s_mlo : s_mhi)[t] = make_uint4(m[0], m[1], m[2], m[3]);
    }
  }
  if constexpr (kChunk) {  // render every skeleton into its template (Now filled in) and its segment list
    const uint32_t ns = a.p.n_skels;
    for (uint32_t q = threadIdx.x; q < a.p.n_pieces; q += kBlock) s_pofs[q] = 0xFFFFu;  // pieces of no skeleton
    if (threadIdx.x < ns) {
      const kwk_emit_skel S = s_skels[threadIdx.x];
      uint32_t sz = 0;
      for (uint32_t q = 0; q < S.n_pieces; ++q) {
        const kwk_emit_piece P = s_pieces[S.first_piece + q];
        sz += P.lit_len + (P.slot == 0 ? a.now_len : 0u);
      }
      s_tsz[threadIdx.x] = make_uint2(sz, 2u * S.n_pieces + 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // exclusive bases: template bytes, segment slots
      uint32_t tb = 0, sb = 0;
      for (uint32_t k = 0; k < ns; ++k) {
        const uint2 v = s_tsz[k];
        s_tsz[k] = make_uint2(tb, sb);
        tb += v.x;
        sb += v.y;
      }
    }
    __syncthreads();
    if (threadIdx.x < ns) {
      const kwk_emit_skel S = s_skels[threadIdx.x];
      const uint32_t tpl = lds_addr(s_tpl);
      uint32_t pos = s_tsz[threadIdx.x].x, run = pos, sb = s_tsz[threadIdx.x].y, n = 0;
      for (uint32_t q = 0; q < S.n_pieces; ++q) {
        const kwk_emit_piece P = s_pieces[S.first_piece + q];
        s_pofs[S.first_piece + q] = (uint16_t)pos;
        pos += P.lit_len;
        if (P.slot == 0) {
          pos += a.now_len;
        } else if (P.slot != KWK_EMIT_NO_SLOT) {
          if (pos > run) s_seg[sb + n++] = make_uint2(tpl + run, pos - run);
          s_seg[sb + n++] = make_uint2(P.slot - 1u, (uint32_t)P.slot * kSegValue);
          run = pos;
        }
      }
      if (pos > run) s_seg[sb + n++] = make_uint2(tpl + run, pos - run);
      s_skseg[threadIdx.x] = make_uint2(sb, n);
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < a.p.n_pieces; q += kBlock) {  // the bytes: one piece per thread
      if (s_pofs[q] == 0xFFFFu) continue;
      const kwk_emit_piece P = s_pieces[q];
      lds_u8* d = (lds_u8*)(size_t)(lds_addr(s_tpl) + s_pofs[q]);
      const char* src = T.lits + P.lit_off;
      for (uint32_t k = 0; k < P.lit_len; ++k) d[k] = (uint8_t)src[k];
      if (P.slot == 0)
        for (uint32_t k = 0; k < a.now_len; ++k) d[P.lit_len + k] = (uint8_t)(s_now[k >> 2] >> (8u * (k & 3u)));
    }
    __syncthreads();
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) a.offsets[tot_i] = tot_b;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t n_ok = 0;
  for (uint32_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    const uint32_t lr = threadIdx.x, r = t * kTile + lr;
    Rec x{0u, 0xFFFFFFFFu, false};
    uint64_t w = 0;
    Size sz{0u, 0u, 0ull};
    Vals V{nullptr, lr};
    if constexpr (kLds) V.lds = reinterpret_cast<const uint8_t*>(s_vals);
    if (r < n) {
      x = fetch(a, r);
      w = x.valid ? a.words[x.slot] : 0ull;
      if constexpr (kLds) {  // the record's value rows, one 16-byte gather per column (stages with patches only)
        const bool any = x.valid && x.stage < a.p.n_stages && a.p.stage_tpl_ptr[x.stage + 1] > a.p.stage_tpl_ptr[x.stage];
        for (uint32_t c = 0; c < kLdsCols; ++c)
          s_vals[c * kTile + lr] = c < a.p.n_cols && any
                                       ? *reinterpret_cast<const uint4*>(a.p.cols[c] + (uint64_t)x.slot * 16u)
                                       : make_uint4(0xFFu, 0u, 0u, 0u);
      }
      sz = rec_size(a, T, x, w, V);
    }
    n_ok += (uint32_t)__popc(sz.ok);
    // block-exclusive prefix of the records' items / bytes, plus the tile's base
    const uint32_t ii = wave_incl(sz.items, lane);
    const unsigned long long ib = wave_incl(sz.bytes, lane);
    if (lane == 63) {
      s_wi[wave] = ii;
      s_wb[wave] = ib;
    }
    __syncthreads();
    uint32_t item = a.tile_items[t] + ii - sz.items;
    unsigned long long pos = a.tile_bytes[t] + ib - sz.bytes;
    for (uint32_t v = 0; v < wave; ++v) {
      item += s_wi[v];
      pos += s_wb[v];
    }
    const unsigned long long rec_base = pos;
    uint32_t n_sk = 0, t0 = 0, t1 = 0;
    if (r < n && x.stage < a.p.n_stages) {
      t0 = a.p.stage_tpl_ptr[x.stage];
      t1 = a.p.stage_tpl_ptr[x.stage + 1];
      uint32_t g = (uint32_t)(w >> 16) & 0xFFu;
      for (uint32_t j = t0; j < t1; ++j, ++item) {
        const uint32_t tid = a.p.stage_tpl[j];
        const bool ok = (sz.ok >> (j - t0)) & 1u;
        a.items[item] = kwk_emit_item{r, (uint16_t)tid, (uint8_t)(ok ? KWK_EMIT_OK : KWK_EMIT_HOST), 0};
        a.offsets[item] = pos;
        if (ok) {
          const int k = skel_index(a, w, tid);
          const kwk_emit_skel& S = skels[k];
          pos += (unsigned long long)skel_bytes(a, T, (uint32_t)k, x.slot, V);
          g = (g & S.keep) | S.set;
          if (n_sk < kRecSk) s_sk[lr * kRecSk + n_sk] = (int16_t)k;
          ++n_sk;
        }
      }
      // the object's guard bits after the patches (all items emitted here; else the host sets them)
      const uint32_t all = t1 - t0 >= 32 ? 0xFFFFFFFFu : (1u << (t1 - t0)) - 1u;
      if (x.valid && sz.ok == all) {
        const uint32_t cls = (uint32_t)(w & 0xFFFFu);
        if (a.p.stage_delete[x.stage] && cls < a.p.n_classes) g = a.p.fresh[cls];
        const uint64_t nw = (w & ~(0xFFull << 16)) | (uint64_t)g << 16;
        if (nw != w) a.words[x.slot] = nw;
      }
    }
    // ---- the bytes
    bool lane_writes = n_sk != 0;  // this lane writes its own record with Acc
    if constexpr (kChunk) {
      const unsigned long long tb = a.tile_bytes[t] & ~15ull;  // the tile's bytes: < 2 GiB past tb
      const uint32_t g0 = (uint32_t)(rec_base - tb), g1 = (uint32_t)(pos - tb);
      s_nsk[lr] = (uint8_t)min(n_sk, kRecSk);
      if (lr == kTile - 1u) s_tend = g1;
      // a record of more than kRecSk items: the whole tile per lane (Acc)
      if (!__syncthreads_or(n_sk > kRecSk)) {
        lane_writes = false;
        // lane r writes the 128-byte lines that start inside its record, their bytes past it
        // from the records after it: every line of the tile leaves whole, once (lane 0 also
        // writes its part of the line the tile shares with the tile before, and the tile's last
        // line is cut at its end)
        const uint32_t tend = s_tend;
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(a.out + tb, 0x7FFFFFFFu);
        const uint32_t L0 = g0 & ~(kLine - 1u), L1 = (g0 + kLine - 1u) & ~(kLine - 1u);
        const bool head = lr == 0 && L0 != g0 && tend > g0;  // the tile's head line
        SegIter it{s_skseg, s_seg, s_sk, s_nsk, lds_addr(s_vals), lr, s_nsk[lr], 0u, 0u, 0u, 0u, g0, g0, 0u};
        if (head || L1 < g1) it.next();  // (a lane with no line to write never walks the records after it)
        uint32_t buf[kLineChunks][4];
        if (head) {
          produce_line(it, L0, buf, lds_addr(s_mlo), lds_addr(s_mhi));
          store_line_part(rs, L0, buf, g0 - L0, min(tend - L0, kLine), true);
        }
        for (uint32_t L = L1; L < g1; L += kLine) {
          produce_line(it, L, buf, lds_addr(s_mlo), lds_addr(s_mhi));
          const bool whole = L + kLine <= tend;
#pragma unroll
          for (uint32_t i = 0; i < kLineChunks; ++i)
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{buf[i][0], buf[i][1], buf[i][2], buf[i][3]}, rs,
                                                   whole ? L + 16u * i : kOOB, 0, 0);
          if (!whole) store_line_part(rs, L, buf, 0u, min(tend - L, kLine), true);  // the tile's last line
        }
      }
    }
    if (lane_writes) {  // per lane, Acc (four bytes per append)
      Acc o(a.out, rec_base);
      if (n_sk <= kRecSk) {
        for (uint32_t j = 0; j < n_sk; ++j) lane_skel(a, T, skels[s_sk[lr * kRecSk + j]], x.slot, s_now, V, o);
      } else {
        for (uint32_t j = t0; j < t1; ++j)
          if ((sz.ok >> (j - t0)) & 1u) lane_skel(a, T, skels[skel_index(a, w, a.p.stage_tpl[j])], x.slot, s_now, V, o);
      }
      o.finish();
    }
    __syncthreads();  // s_wi / s_wb and the tables are rewritten by the next tile
  }
  n_ok = wave_sum(n_ok);
  if (lane == 0 && n_ok) atomicAdd(&a.totals[3], (unsigned long long)n_ok);
}

}  // namespace

struct kwk_emitter {
  std::string err;
  kwk_engine* eng = nullptr;  // must outlive the emitter
  hipStream_t stream = nullptr;  // the engine's stream as of the current call (kwk_stream at every entry:
                                 // KWK_TUNE_STREAM_PRIORITY re-creates it, so it is never cached across calls)
  int device = 0;
  uint32_t capacity = 0, n_columns = 0, max_tiles = 0, grid = 0, cus = 1;
  int write_occ[3] = {0, 0, 0};   // resident blocks per CU of each write kernel variant (0: not asked yet)
  Prog p{};
  std::vector<void*> allocs;
  std::vector<uint32_t> stride;
  std::vector<uint8_t*> cols;
  uint64_t* d_words = nullptr;
  uint32_t* d_tile_items = nullptr;
  unsigned long long* d_tile_bytes = nullptr;
  unsigned long long* d_totals = nullptr;
  kwk_emit_item* d_items = nullptr;
  uint64_t* d_offsets = nullptr;
  char* d_out = nullptr;
  uint64_t cap_items = 0, cap_bytes = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool emitted = false;
  bool chunk_ok = false;          // skeletons own consecutive, disjoint piece ranges (the chunk writer's templates)
  bool lencache = false;          // words' bits 24-31 cache the value lengths (emit_lens_kernel)
  uint64_t tpl_lits = 0;          // literal bytes of every skeleton's pieces
  uint32_t tpl_now_slots = 0;     // Now slots of every skeleton's pieces

  ~kwk_emitter() {
    hipSetDevice(device);
    void* s = nullptr;
    if (eng && kwk_stream(eng, &s) == KWK_OK && s) hipStreamSynchronize(static_cast<hipStream_t>(s));
    for (void* x : allocs) hipFree(x);
    if (d_items) hipFree(d_items);
    if (d_offsets) hipFree(d_offsets);
    if (d_out) hipFree(d_out);
    if (ev0) hipEventDestroy(ev0);
    if (ev1) hipEventDestroy(ev1);
  }
};

namespace {

// the engine's current stream and device (every entry point: the stream may have been re-created)
kwk_status bind(kwk_emitter* em) {
  void* s = nullptr;
  if (kwk_stream(em->eng, &s) != KWK_OK || !s)
    return fail(KWK_ESTATE, std::string("kwk_stream: ") + kwk_last_error(em->eng));
  em->stream = static_cast<hipStream_t>(s);
  HIP_TRY(hipSetDevice(em->device));
  return KWK_OK;
}

// host -> device copy ordered on the engine's stream (a pageable hipMemcpy on the null stream can
// return with its DMA in flight, and the engine's non-blocking stream would not wait for it)
kwk_status copy_in(kwk_emitter* em, void* dst, const void* src, size_t bytes) {
  if (!bytes) return KWK_OK;
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, em->stream));
  HIP_TRY(hipStreamSynchronize(em->stream));
  return KWK_OK;
}

kwk_status copy_out(kwk_emitter* em, void* dst, const void* src, size_t bytes) {
  if (!bytes) return KWK_OK;
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, em->stream));
  HIP_TRY(hipStreamSynchronize(em->stream));
  return KWK_OK;
}

kwk_status fill(kwk_emitter* em, void* dst, int v, size_t bytes) {
  HIP_TRY(hipMemsetAsync(dst, v, bytes, em->stream));
  HIP_TRY(hipStreamSynchronize(em->stream));
  return KWK_OK;
}

template <typename T>
kwk_status upload(kwk_emitter* em, T** dst, const T* src, size_t n) {
  void* d = nullptr;
  HIP_TRY(hipMalloc(&d, std::max<size_t>(1, n) * sizeof(T)));
  em->allocs.push_back(d);
  if (kwk_status st = copy_in(em, d, src, n * sizeof(T))) return st;
  *dst = static_cast<T*>(d);
  return KWK_OK;
}

kwk_status check_program(const kwk_emit_program* g) {
  if (!g->stage_tpl_ptr || !g->stage_delete || (g->n_classes && !g->fresh_guards) ||
      (g->n_classes * g->n_templates && !g->skel_of))
    return fail(KWK_EINVAL, "emit program: null array");
  if (g->n_templates > 32) return fail(KWK_EINVAL, "emit program: more than 32 templates");
  if ((uint64_t)g->n_classes * g->n_templates > (1u << 26)) return fail(KWK_EINVAL, "emit program: too many skeletons");
  if (g->stage_tpl_ptr[0] != 0) return fail(KWK_EINVAL, "emit program: stage_tpl_ptr[0] != 0");
  for (uint32_t s = 0; s < g->n_stages; ++s) {
    const uint32_t a = g->stage_tpl_ptr[s], b = g->stage_tpl_ptr[s + 1];
    if (b < a || b - a > kMaxStageTpl) return fail(KWK_EINVAL, "emit program: stage template ranges");
  }
  const uint32_t n_st = g->stage_tpl_ptr[g->n_stages];
  if (n_st && !g->stage_tpl) return fail(KWK_EINVAL, "emit program: null stage_tpl");
  for (uint32_t j = 0; j < n_st; ++j)
    if (g->stage_tpl[j] >= g->n_templates) return fail(KWK_EINVAL, "emit program: template id out of range");
  for (uint64_t i = 0; i < (uint64_t)g->n_classes * g->n_templates; ++i)
    if (g->skel_of[i] < -1 || g->skel_of[i] >= (int64_t)g->n_skels) return fail(KWK_EINVAL, "emit program: skeleton index");
  if ((g->n_skels && !g->skels) || (g->n_pieces && !g->pieces) || (g->n_lit_bytes && !g->lits) ||
      (g->n_columns && !g->column_stride))
    return fail(KWK_EINVAL, "emit program: null array");
  for (uint32_t k = 0; k < g->n_skels; ++k) {
    const kwk_emit_skel& S = g->skels[k];
    if ((uint64_t)S.first_piece + S.n_pieces > g->n_pieces) return fail(KWK_EINVAL, "emit program: piece range");
  }
  for (uint32_t q = 0; q < g->n_pieces; ++q) {
    const kwk_emit_piece& P = g->pieces[q];
    if ((uint64_t)P.lit_off + P.lit_len > g->n_lit_bytes) return fail(KWK_EINVAL, "emit program: literal range");
    if (P.slot != KWK_EMIT_NO_SLOT && P.slot > g->n_columns) return fail(KWK_EINVAL, "emit program: slot out of range");
  }
  for (uint32_t c = 0; c < g->n_columns; ++c)
    if (g->column_stride[c] < 4 || g->column_stride[c] > 256 || (g->column_stride[c] & 3u))
      return fail(KWK_EINVAL, "emit program: column stride 4..256, a multiple of 4");
  return KWK_OK;
}

// the words' cached value lengths for slots [first, first + n) (after any write of words or rows)
kwk_status refresh_lens(kwk_emitter* em, uint32_t first, uint32_t n) {
  if (!em->lencache || !n) return KWK_OK;
  const uint32_t blocks = std::min<uint32_t>((n + 255u) / 256u, em->cus * 16u);
  hipLaunchKernelGGL(emit_lens_kernel, dim3(blocks), dim3(256), 0, em->stream, em->d_words, em->p.cols, em->n_columns,
                     first, n);
  HIP_TRY(hipGetLastError());
  return KWK_OK;
}

kwk_status emitter_init(kwk_emitter* em, const kwk_emit_program* g) {
  em->p.n_classes = g->n_classes;
  em->p.n_templates = g->n_templates;
  em->p.n_stages = g->n_stages;
  em->p.n_pieces = g->n_pieces;
  em->p.n_lits = (uint32_t)std::min<uint64_t>(g->n_lit_bytes, 0xFFFFFFFFu);
  em->p.n_cols = g->n_columns;
  em->p.n_skels = g->n_skels;
  {  // the chunk writer's templates: pieces owned by one skeleton each, in skeleton order
    bool ok = true;
    uint32_t next = 0;
    for (uint32_t k = 0; k < g->n_skels && ok; ++k) {
      const kwk_emit_skel& S = g->skels[k];
      ok = S.first_piece >= next;
      next = S.first_piece + S.n_pieces;
      for (uint32_t q = 0; q < S.n_pieces; ++q) {
        const kwk_emit_piece& P = g->pieces[S.first_piece + q];
        em->tpl_lits += P.lit_len;
        em->tpl_now_slots += P.slot == 0 ? 1u : 0u;
      }
    }
    em->chunk_ok = ok;
  }
  const uint32_t n_st = g->stage_tpl_ptr[g->n_stages];
  if (kwk_status st = upload(em, const_cast<uint32_t**>(&em->p.stage_tpl_ptr), g->stage_tpl_ptr, g->n_stages + 1)) return st;
  if (kwk_status st = upload(em, const_cast<uint16_t**>(&em->p.stage_tpl), g->stage_tpl, n_st)) return st;
  if (kwk_status st = upload(em, const_cast<uint8_t**>(&em->p.stage_delete), g->stage_delete, g->n_stages)) return st;
  if (kwk_status st = upload(em, const_cast<int32_t**>(&em->p.skel_of), g->skel_of, (size_t)g->n_classes * g->n_templates))
    return st;
  if (kwk_status st = upload(em, const_cast<kwk_emit_skel**>(&em->p.skels), g->skels, g->n_skels)) return st;
  if (kwk_status st = upload(em, const_cast<kwk_emit_piece**>(&em->p.pieces), g->pieces, g->n_pieces)) return st;
  {  // the literal runs with 16 bytes of zero padding (the writers read aligned dword pairs)
    std::vector<char> lits(g->lits, g->lits + g->n_lit_bytes);
    lits.resize(lits.size() + 16, 0);
    if (kwk_status st = upload(em, const_cast<char**>(&em->p.lits), lits.data(), lits.size())) return st;
  }
  if (kwk_status st = upload(em, const_cast<uint8_t**>(&em->p.fresh), g->fresh_guards, g->n_classes)) return st;
  em->n_columns = g->n_columns;
  em->stride.assign(g->column_stride, g->column_stride + g->n_columns);
  for (uint32_t c = 0; c < g->n_columns; ++c) {
    void* d = nullptr;
    HIP_TRY(hipMalloc(&d, (size_t)em->capacity * em->stride[c] + 16));  // + the dword a row's last read may touch
    em->allocs.push_back(d);
    if (kwk_status st = fill(em, d, 0xFF, (size_t)em->capacity * em->stride[c] + 16)) return st;  // unusable until set
    em->cols.push_back(static_cast<uint8_t*>(d));
  }
  if (kwk_status st = upload(em, const_cast<uint8_t***>(&em->p.cols), em->cols.data(), em->cols.size())) return st;
  if (kwk_status st = upload(em, const_cast<uint32_t**>(&em->p.stride), em->stride.data(), em->stride.size())) return st;
  void* d = nullptr;
  HIP_TRY(hipMalloc(&d, (size_t)std::max(1u, em->capacity) * 8));
  em->allocs.push_back(d);
  if (kwk_status st = fill(em, d, 0, (size_t)std::max(1u, em->capacity) * 8)) return st;  // class 0, nothing accepted: all to the host
  em->d_words = static_cast<uint64_t*>(d);
  em->lencache = g->n_columns <= 2;
  for (uint32_t c = 0; c < g->n_columns; ++c) em->lencache = em->lencache && g->column_stride[c] == 16u;
  em->max_tiles = (em->capacity + kTile - 1) / kTile + 1;
  HIP_TRY(hipMalloc(&d, (size_t)em->max_tiles * 4));
  em->allocs.push_back(d);
  em->d_tile_items = static_cast<uint32_t*>(d);
  HIP_TRY(hipMalloc(&d, (size_t)em->max_tiles * 8));
  em->allocs.push_back(d);
  em->d_tile_bytes = static_cast<unsigned long long*>(d);
  HIP_TRY(hipMalloc(&d, 4 * 8));
  em->allocs.push_back(d);
  em->d_totals = static_cast<unsigned long long*>(d);
  if (kwk_status st = fill(em, d, 0, 4 * 8)) return st;
  int cus = 0;
  HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, em->device));
  em->grid = std::max(1u, std::min(em->max_tiles, (uint32_t)std::max(1, cus) * 8u));
  em->cus = (uint32_t)std::max(1, cus);
  if (kwk_status st = refresh_lens(em, 0, em->capacity)) return st;
  HIP_TRY(hipEventCreate(&em->ev0));
  HIP_TRY(hipEventCreate(&em->ev1));
  return KWK_OK;
}

}  // namespace

extern "C" {

const char* kwk_emit_last_error(const kwk_emitter* em) { return em ? em->err.c_str() : g_err.c_str(); }

kwk_status kwk_emitter_create(kwk_engine* eng, uint32_t capacity, const kwk_emit_program* prog, kwk_emitter** out) {
  ErrScope es_(nullptr);
  if (!eng || !prog || !out) return fail(KWK_EINVAL, "null argument");
  if (capacity > (1u << 27)) return fail(KWK_EINVAL, "capacity above 2^27 slots");
  if (kwk_status st = check_program(prog)) return st;
  void* s = nullptr;
  if (kwk_stream(eng, &s) != KWK_OK) return fail(KWK_EINVAL, std::string("kwk_stream: ") + kwk_last_error(eng));
  auto* em = new kwk_emitter();
  em->eng = eng;
  em->stream = static_cast<hipStream_t>(s);
  em->capacity = capacity;
  hipError_t e = hipStreamGetDevice(em->stream, &em->device);
  if (e != hipSuccess) {
    delete em;
    return fail(KWK_EHIP, std::string("hipStreamGetDevice: ") + hipGetErrorString(e));
  }
  kwk_status st = bind(em);
  if (!st) st = emitter_init(em, prog);
  if (st) {
    delete em;
    return st;
  }
  *out = em;
  return KWK_OK;
}

kwk_status kwk_emitter_destroy(kwk_emitter* em) {
  delete em;
  return KWK_OK;
}

kwk_status kwk_emit_set_words(kwk_emitter* em, uint32_t first, uint32_t n, const uint64_t* words) {
  ErrScope es_(em ? &em->err : nullptr);
  if (!em || (n && !words)) return fail(KWK_EINVAL, "null argument");
  if ((uint64_t)first + n > em->capacity) return fail(KWK_EINVAL, "rows beyond the capacity");
  if (kwk_status st = bind(em)) return st;
  if (kwk_status st = copy_in(em, em->d_words + first, words, (size_t)n * 8)) return st;
  return refresh_lens(em, first, n);
}

kwk_status kwk_emit_get_words(kwk_emitter* em, uint32_t first, uint32_t n, uint64_t* words) {
  ErrScope es_(em ? &em->err : nullptr);
  if (!em || (n && !words)) return fail(KWK_EINVAL, "null argument");
  if ((uint64_t)first + n > em->capacity) return fail(KWK_EINVAL, "rows beyond the capacity");
  if (kwk_status st = bind(em)) return st;
  if (kwk_status st = copy_out(em, words, em->d_words + first, (size_t)n * 8)) return st;
  for (uint32_t i = 0; i < n; ++i) words[i] &= ~(0xFFull << 24);  // (the device's length cache)
  return KWK_OK;
}

kwk_status kwk_emit_set_column(kwk_emitter* em, uint32_t c, uint32_t first, uint32_t n, const uint8_t* data) {
  ErrScope es_(em ? &em->err : nullptr);
  if (!em || (n && !data)) return fail(KWK_EINVAL, "null argument");
  if (c >= em->n_columns) return fail(KWK_EINVAL, "column out of range");
  if ((uint64_t)first + n > em->capacity) return fail(KWK_EINVAL, "rows beyond the capacity");
  if (kwk_status st = bind(em)) return st;
  if (kwk_status st = copy_in(em, em->cols[c] + (size_t)first * em->stride[c], data, (size_t)n * em->stride[c])) return st;
  return refresh_lens(em, first, n);
}

kwk_status kwk_emit_reserve(kwk_emitter* em, uint32_t max_items, uint64_t max_bytes) {
  ErrScope es_(em ? &em->err : nullptr);
  if (!em) return fail(KWK_EINVAL, "null emitter");
  if (kwk_status st = bind(em)) return st;
  HIP_TRY(hipStreamSynchronize(em->stream));
  if (max_items > em->cap_items) {
    if (em->d_items) HIP_TRY(hipFree(em->d_items));
    if (em->d_offsets) HIP_TRY(hipFree(em->d_offsets));
    em->d_items = nullptr;
    em->d_offsets = nullptr;
    em->cap_items = 0;
    HIP_TRY(hipMalloc(&em->d_items, (size_t)max_items * sizeof(kwk_emit_item)));
    HIP_TRY(hipMalloc(&em->d_offsets, ((size_t)max_items + 1) * 8));
    em->cap_items = max_items;
  }
  if (max_bytes > em->cap_bytes) {
    if (em->d_out) HIP_TRY(hipFree(em->d_out));
    em->d_out = nullptr;
    em->cap_bytes = 0;
    HIP_TRY(hipMalloc(&em->d_out, (size_t)max_bytes));
    em->cap_bytes = max_bytes;
  }
  return KWK_OK;
}

kwk_status kwk_emit(kwk_emitter* em, int64_t now_ns, uint32_t source) {
  ErrScope es_(em ? &em->err : nullptr);
  if (!em) return fail(KWK_EINVAL, "null emitter");
  EmitArgs a{};
  a.p = em->p;
  const uint32_t from = source & 0xFFu;
  if (from == KWK_EMIT_FROM_RECORDS) {
    if (kwk_fired_device(em->eng, &a.recs, &a.count) != KWK_OK)
      return fail(KWK_ESTATE, std::string("kwk_fired_device: ") + kwk_last_error(em->eng));
  } else if (from == KWK_EMIT_FROM_PACKED) {
    if (kwk_fired_packed_device(em->eng, &a.packed, &a.count) != KWK_OK)
      return fail(KWK_ESTATE, std::string("kwk_fired_packed_device: ") + kwk_last_error(em->eng));
  } else {
    return fail(KWK_EINVAL, "source must be KWK_EMIT_FROM_RECORDS or KWK_EMIT_FROM_PACKED");
  }
  if (source & ~0xFFu) return fail(KWK_EINVAL, "unknown source flags");
  if (kwk_status st = bind(em)) return st;
  if (!em->d_offsets)
    if (kwk_status st = kwk_emit_reserve(em, 1, 1)) return st;
  a.words = em->d_words;
  a.capacity = em->capacity;
  a.max_recs = (em->max_tiles - 1) * kTile;
  a.tile_items = em->d_tile_items;
  a.tile_bytes = em->d_tile_bytes;
  a.totals = em->d_totals;
  a.items = em->d_items;
  a.offsets = em->d_offsets;
  a.out = em->d_out;
  a.cap_items = em->cap_items;
  a.cap_bytes = em->cap_bytes;
  a.lencache = em->lencache ? 1u : 0u;
  const std::string now = kwkfmt::rfc3339nano(now_ns);
  if (now.size() >= sizeof a.now) return fail(KWK_EINVAL, "Now() text too long");
  memcpy(a.now, now.data(), now.size());
  a.now_len = (uint32_t)now.size();
  // the list's count lives on the device: every tile loop reads it; the grid covers the capacity
  HIP_TRY(hipEventRecord(em->ev0, em->stream));
  bool lds = em->p.n_pieces <= kLdsPieces && em->p.n_lits + 8u <= kLdsLits && em->p.n_skels <= kLdsSkels;
  bool vals16 = em->n_columns <= kLdsCols;
  for (uint32_t c = 0; c < em->n_columns; ++c) vals16 = vals16 && em->stride[c] == 16u;
  if (lds)
    hipLaunchKernelGGL(emit_size_kernel<true>, dim3(em->grid), dim3(kBlock), 0, em->stream, a);
  else
    hipLaunchKernelGGL(emit_size_kernel<false>, dim3(em->grid), dim3(kBlock), 0, em->stream, a);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(emit_scan_kernel, dim3(1), dim3(kScanBlock), 0, em->stream, a);
  HIP_TRY(hipGetLastError());
  const bool wl = lds && vals16;  // the write kernel's LDS path also stages the value rows
  // the chunk writer: templates (literals + Now per slot) within kTplBytes, pieces in skeleton order
  const bool chunk = wl && em->chunk_ok && em->tpl_lits + (uint64_t)em->tpl_now_slots * a.now_len + 16u <= kTplBytes;
  const void* wk = chunk ? (const void*)emit_write_kernel<true, true>
                   : wl  ? (const void*)emit_write_kernel<true, false>
                         : (const void*)emit_write_kernel<false, false>;
  void* wargs[] = {&a};
  // the write kernel's grid: every block resident at once (one round; its tile loop does the rest)
  const int vi = chunk ? 0 : wl ? 1 : 2;
  if (!em->write_occ[vi]) {
    int occ = 0;
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, wk, kBlock, 0));
    em->write_occ[vi] = std::max(1, occ);
  }
  const uint32_t wgrid = std::max(1u, std::min(em->max_tiles, em->cus * (uint32_t)em->write_occ[vi]));
  HIP_TRY(hipLaunchKernel(wk, dim3(wgrid), dim3(kBlock), wargs, 0, em->stream));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(em->ev1, em->stream));
  em->emitted = true;
  return KWK_OK;
}

kwk_status kwk_emit_result(kwk_emitter* em, uint32_t* n_items, uint64_t* n_bytes) {
  ErrScope es_(em ? &em->err : nullptr);
  if (!em || !n_items || !n_bytes) return fail(KWK_EINVAL, "null argument");
  if (!em->emitted) return fail(KWK_ESTATE, "kwk_emit must come first");
  if (kwk_status st = bind(em)) return st;
  unsigned long long t[3];
  if (kwk_status st = copy_out(em, t, em->d_totals, sizeof t)) return st;
  *n_items = (uint32_t)t[0];
  *n_bytes = t[1];
  if (t[2]) return fail(KWK_ECAP, "the fired list is longer than the emitter's capacity");
  if (t[0] > em->cap_items || t[1] > em->cap_bytes)
    return fail(KWK_ECAP, "emission exceeds the reservation: kwk_emit_reserve(" + std::to_string(t[0]) + ", " +
                              std::to_string(t[1]) + ") and emit again");
  return KWK_OK;
}

kwk_status kwk_emit_stats(kwk_emitter* em, uint32_t* n_items, uint32_t* n_emitted, uint64_t* n_bytes) {
  ErrScope es_(em ? &em->err : nullptr);
  if (!em || !n_items || !n_emitted || !n_bytes) return fail(KWK_EINVAL, "null argument");
  if (kwk_status st = kwk_emit_result(em, n_items, n_bytes)) return st;
  unsigned long long t = 0;
  if (kwk_status st = copy_out(em, &t, em->d_totals + 3, 8)) return st;
  *n_emitted = (uint32_t)t;
  return KWK_OK;
}

kwk_status kwk_emit_device(kwk_emitter* em, const kwk_emit_item** items, const uint64_t** offsets, const char** bytes) {
  ErrScope es_(em ? &em->err : nullptr);
  if (!em) return fail(KWK_EINVAL, "null emitter");
  if (items) *items = em->d_items;
  if (offsets) *offsets = em->d_offsets;
  if (bytes) *bytes = em->d_out;
  return KWK_OK;
}

kwk_status kwk_emit_copy(kwk_emitter* em, kwk_emit_item* items, uint64_t* offsets, char* bytes) {
  ErrScope es_(em ? &em->err : nullptr);
  uint32_t ni = 0;
  uint64_t nb = 0;
  if (kwk_status st = kwk_emit_result(em, &ni, &nb)) return st;
  if ((ni && (!items || !offsets)) || (nb && !bytes) || !offsets) return fail(KWK_EINVAL, "null argument");
  if (ni) {
    if (kwk_status st = copy_out(em, items, em->d_items, (size_t)ni * sizeof(kwk_emit_item))) return st;
    if (kwk_status st = copy_out(em, offsets, em->d_offsets, ((size_t)ni + 1) * 8)) return st;
  } else {
    offsets[0] = 0;
  }
  if (kwk_status st = copy_out(em, bytes, em->d_out, (size_t)nb)) return st;
  return KWK_OK;
}

kwk_status kwk_emit_elapsed(kwk_emitter* em, float* ms) {
  ErrScope es_(em ? &em->err : nullptr);
  if (!em || !ms) return fail(KWK_EINVAL, "null argument");
  if (!em->emitted) return fail(KWK_ESTATE, "kwk_emit must come first");
  if (kwk_status st = bind(em)) return st;
  HIP_TRY(hipEventSynchronize(em->ev1));
  HIP_TRY(hipEventElapsedTime(ms, em->ev0, em->ev1));
  return KWK_OK;
}

}  // extern "C"
