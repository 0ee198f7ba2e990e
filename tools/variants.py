"""Cost-isolation builds of the engine (tools only: never loaded by the package, the tests or
bench.py).  Each variant is engine.hip with a few source replacements — most of them give
WRONG results on purpose (a phase skipped, a draw replaced) and exist only to time what the
removed work costs on the C2-mix HBM working set.

    python tools/variants.py build [names...]      # -> tools/build/libkwok_engine_<name>.so ("a+b": b applied to a)
    python tools/variants.py run [names...]        # one child process per variant, JSON lines
    python tools/variants.py snap                  # HEAD's engine.hip -> tools/ab/ (the "head" variant on the box)
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "kwok_amd", "csrc", "engine.hip")
OUT = os.path.join(ROOT, "tools", "build")

_P2 = ("const uint2 nv = process_object<kHarness, kWB, false, kDW>(a, T, deltas, n_stages, fin_group, i, s.x, s.y, due,\n"
       "                                                                   f, n_matched, lutp, lut_n, due_set, due_w);")

_PF_EARLY = ("  if (tile + gridDim.x < n_tiles) load_tile(tile + gridDim.x);  // block-uniform\n", "")
_PF_LATE = ("  const bool rebase = kDW && a.dw_rebase;",
            "  if (tile + gridDim.x < n_tiles) load_tile(tile + gridDim.x);\n  const bool rebase = kDW && a.dw_rebase;")

_S8_INV = [("  __shared__ uint32_t s_inv[kWavesPerBlock][64];", "  __shared__ uint32_t s_inv[64];"),
           ("  s_inv[wave][lane] = 0xFFFFFFFFu;", "  s_inv[lane] = 0xFFFFFFFFu;"),
           ("lds_addr(&s_inv[wave][lane])", "lds_addr(&s_inv[lane])")]

_FORCE = ("const bool lean = a.fsm && e->fsm_kernel;", "const bool lean = a.fsm && e->fsm_kernel;")

_NOCALL = ("          const uint2 r = general16<kHarness>(wbase + w, (uint32_t)tw[w]);",
           "          const uint2 r = make_uint2(0u, 0u);")

VARIANTS = {
    "base": [],
    "head": [],
    # phase 2 of the word sweep does nothing (no state change, no fires)
    "w_nophase2": [(_P2, "const uint2 nv = s; (void)due; (void)i;")],
    # jitter without its Philox draw
    "nojitter": [("delay = (int64_t)((uint64_t)delay + (uint64_t)below_u64(u_jit, jit));",
                  "delay = (int64_t)((uint64_t)delay + (uint64_t)(jit >> 1));")],
    # the word sweep's fired records / per-stage counts are not written
    "w_noemit": [("      emit_fired<true>(f, off, lane, seg, seg_n, s_stat, n_bytes);\n", "      (void)f;\n")],
    # scheduled stages do not store their due time (the due column is only read)
    "nodue_w": [("    else a.due[i] = due;\n", "    else (void)due;\n")],
    # table-only 2-byte sweep (sweep16_fsm_kernel) even when some table entry is general (pod-fast at
    # C5 reaches none of them: results stay correct there, not in general)
    "f_force": [_FORCE],
    # the general 2-byte sweep (sweep16_kernel) for every program
    "g_old": [("constexpr uint32_t kFsmKernelDefault = 2;", "constexpr uint32_t kFsmKernelDefault = 0;")],
    "f_force_d1": [_FORCE, ("constexpr uint32_t kFsmKernelDefault = 2;", "constexpr uint32_t kFsmKernelDefault = 1;")],
    # ... without the out-of-line general path (wrong results if a general entry is reached)
    "f_nocall_d1": [_FORCE, _NOCALL, ("constexpr uint32_t kFsmKernelDefault = 2;", "constexpr uint32_t kFsmKernelDefault = 1;")],
    "f_nocall_d2": [_FORCE, _NOCALL],
    # table-only 2-byte sweep (sweep16_fsm_kernel), C5 cost isolation (run with --c5):
    # phase 3 stores no lines
    "f_nop3": [_FORCE, ("          store_chunk_nt(&gq[(wbase + (uint32_t)q * 512u + lane * 8u) / 8u], nv);\n          n_lline += 16u;",
                "          (void)gq;\n          n_lline += 16u;")],
    # no fired records stored
    "f_norec": [_FORCE, ("__builtin_amdgcn_raw_buffer_store_b32(rec, seg_rs, fire ? (1u + pos) * 4u : kOOB, 0, 0);",
                 "(void)rec; (void)pos;")],
    # phase 2 does nothing (the words never change: every later step is the same read + work list)
    "f_nop2": [_FORCE, ("        if (64u * b < n_work) pass(b);  // wave-uniform", "        (void)b;")],
    # phase 2 does nothing and phase 3 rewrites every line: the kernel's own read + rewrite stream
    "f_nop2_all": [_FORCE, ("        if (64u * b < n_work) pass(b);  // wave-uniform", "        (void)b;"),
                   ("        if ((bal >> (lane & ~(kStoreLanes - 1u))) & ((1ull << kStoreLanes) - 1ull)) {\n"
                    "          store_chunk_nt(&gq[(wbase + (uint32_t)q * 512u + lane * 8u) / 8u], nv);\n          n_lline",
                    "        if (bal || true) {\n"
                    "          store_chunk_nt(&gq[(wbase + (uint32_t)q * 512u + lane * 8u) / 8u], nv);\n          n_lline")],
    # no value-record loads: objects with a record take the stage defaults (C2 cost isolation of
    # the dependent rec_idx -> record round trips of phase 2)
    "w_norec": [("  if (!(sched & KWK_F_HASREC)) return {def, def_ok};", "  return {def, def_ok};"),
                ("  if (sched & KWK_F_HASREC) {\n    if constexpr (kProbe) { gen = 1; return false; }",
                 "  if (false) {\n    if constexpr (kProbe) { gen = 1; return false; }")],
    # no deletion-column loads (pod-delete's jitterDurationFrom)
    "w_nodel": [("    const int64_t dels = need_del ? a.del_s[i] : KWK_DEL_ABSENT;",
                 "    const int64_t dels = KWK_DEL_ABSENT;")],
    # 1-byte sweep (run with --c5): no phase 2, every line of the column rewritten — the kernel's
    # own read + rewrite stream (wrong results: the ids never change)
    "s8_stream": [("    if (n_work) {  // wave-uniform\n      // ---- phase 2: the ids to the LDS tile",
                   "    if (false) {  // wave-uniform\n      // ---- phase 2: the ids to the LDS tile"),
                  ("      const bool st = (ballot(ch) >> (lane & ~(kStoreLanes - 1u))) & ((1ull << kStoreLanes) - 1ull);",
                   "      const bool st = real || ch;")],
    # ... and no line stores: the read stream alone
    "s8_read": [("    if (n_work) {  // wave-uniform\n      // ---- phase 2: the ids to the LDS tile",
                 "    if (false) {  // wave-uniform\n      // ---- phase 2: the ids to the LDS tile"),
                ("      const bool st = (ballot(ch) >> (lane & ~(kStoreLanes - 1u))) & ((1ull << kStoreLanes) - 1ull);",
                 "      const bool st = !real && ch;")],
    # sweep8: one kIdInvalid row shared by the block's waves (LDS 27.8 -> 27.0 KB: 6 workgroups per CU
    # fit) / and a VGPR cap for 6 waves per SIMD (run with --c5; r3x: 52.5-53.6 / 53.6-53.9 vs
    # 52.7-52.8 us, not kept)
    "s8_inv": _S8_INV,
    "s8_lb6": _S8_INV + [("__global__ __launch_bounds__(kBlock) void sweep8_kernel(SweepArgs a) {",
                          "__global__ __launch_bounds__(kBlock, 6) void sweep8_kernel(SweepArgs a) {")],
    # sweep8: 1 / 2 id passes per loop step instead of 4 (run with --c5)
    "id8b1": [("constexpr uint32_t kId8Batch = 4;", "constexpr uint32_t kId8Batch = 1;")],
    "id8b2": [("constexpr uint32_t kId8Batch = 4;", "constexpr uint32_t kId8Batch = 2;")],
    # fused word sweep capped at 6 waves per SIMD instead of 5 (the round-4 default)
    "lb6": [("constexpr int kDwMinBlocks = 5;", "constexpr int kDwMinBlocks = 6;")],
    # sweep8 cost isolation (the shard-size step, --c5 --c5-nodes 125000): no phase 2 (no LDS passes,
    # no fires) / no statistics atomics at the end / no phase-3 line stores / an empty kernel
    "s8_nop2": [("    if (n_work) {  // wave-uniform\n      // ---- phase 2: the ids to the LDS tile",
                 "    if (n_work && a.n == 0u) {  // wave-uniform\n      // ---- phase 2: the ids to the LDS tile")],
    "s8_nostat": [("    if (val) atomicAdd(&a.cum[(uint64_t)blockIdx.x * kStatWords + threadIdx.x], (unsigned long long)val);\n"
                   "  }\n}\n\n// ------------------------------------------------------------------ 4- and 8-byte state sweep",
                   "    if (val && a.n == 0u) atomicAdd(&a.cum[(uint64_t)blockIdx.x * kStatWords + threadIdx.x], "
                   "(unsigned long long)val);\n  }\n}\n\n// ------------------------------------------------------------------ 4- and 8-byte state sweep")],
    "s8_nop3": [("st ? wbase + (uint32_t)q * 1024u + lane * 16u : kOOB, 0, 2 /* nt */);", "kOOB, 0, 2 /* nt */);")],
    "s8_empty": [("  __shared__ unsigned int s_stat[kStatWords];\n  const uint32_t lane = threadIdx.x & 63;\n"
                  "  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n  const uint32_t n_tiles = (uint32_t)(((uint64_t)a.n + kTile - 1) / kTile);",
                  "  __shared__ unsigned int s_stat[kStatWords];\n  if (a.n != 0xFFFFFFFFu) return;\n  const uint32_t lane = threadIdx.x & 63;\n"
                  "  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n  const uint32_t n_tiles = (uint32_t)(((uint64_t)a.n + kTile - 1) / kTile);")],
    # word sweep: one workgroup per tile / 2 / 4 / 8 tiles per workgroup (a loop over tiles, the LDS
    # set-up once, the next tile's stream in flight)
    "tpb1": [("  uint32_t word_tpb = 0;", "  uint32_t word_tpb = 1;")],
    "tpb2": [("  uint32_t word_tpb = 0;", "  uint32_t word_tpb = 2;")],
    "tpb4": [("  uint32_t word_tpb = 0;", "  uint32_t word_tpb = 4;")],
    "tpb8": [("  uint32_t word_tpb = 0;", "  uint32_t word_tpb = 8;")],
    "tpb16": [("  uint32_t word_tpb = 0;", "  uint32_t word_tpb = 16;")],
    # ... the next tile's stream issued after phase 2 (its registers not live across process_object)
    "tpb4_late": [("  uint32_t word_tpb = 0;", "  uint32_t word_tpb = 4;"), _PF_EARLY, _PF_LATE],
    "tpb8_late": [("  uint32_t word_tpb = 0;", "  uint32_t word_tpb = 8;"), _PF_EARLY, _PF_LATE],
    # the word sweep's per-stage fired counts are not kept (the fired records still are)
    "w_nostat": [("  unsigned long long rest = bal;  // one LDS add per distinct fired stage\n  while (rest) {",
                  "  unsigned long long rest = 0;  // one LDS add per distinct fired stage\n  while (rest) {")],
    # a multi-match takes its first matched stage: no weight getters, no pick draw
    "w_nopick": [("  if (cnt == 1) {\n    pick = __ffs(m) - 1;\n  } else {",
                  "  if (cnt >= 1) {\n    pick = __ffs(m) - 1;\n  } else {")],
    # the matcher's Philox block replaced by a few multiplies (the pick and jitter draws)
    "w_nophilox": [("    philox10(c0, c1, c2, c3, (uint32_t)a.key, (uint32_t)(a.key >> 32));",
                    "    c0 ^= c1 * 0x9E3779B9u; c1 ^= c0 * 0x85EBCA6Bu; c2 ^= c1 * 0xC2B2AE35u; c3 ^= c2 * 0x27D4EB2Fu;")],
    # fused: fired records stored per phase-2 pass (not staged in LDS)
    "w_nolds": [("constexpr bool kDwLdsRecs = true;", "constexpr bool kDwLdsRecs = false;")],
    # fused word sweep: each wave touches the 32 lines of its region of the tile after next (one dword
    # load per line, into L2), so the next tile's prefetch issued before phase 2 — which phase 2's
    # loads wait behind in the in-order vmcnt queue — hits L2
    "w_touch": [("  const uint32_t tbase = tile * kTile;\n",
                 "  const uint32_t tbase = tile * kTile;\n"
                 "  if (kDW && tile + 2u * gridDim.x < n_tiles)\n"
                 "    touch_sink ^= __builtin_amdgcn_raw_buffer_load_b32(st_rs, lane < 32u ? ((tile + 2u * gridDim.x) * kTile + "
                 "wave * kWave) * kWB + lane * 128u : kOOB, 0, 0);\n"),
                ("  load_tile(tile);  // the first tile's stream is issued before the LDS set-up so its latency overlaps it\n",
                 "  load_tile(tile);  // the first tile's stream is issued before the LDS set-up so its latency overlaps it\n"
                 "  uint32_t touch_sink = 0;\n"),
                ("  for (int o = 32; o > 0; o >>= 1) {\n    n_matched += __shfl_xor(n_matched, o);\n    n_bytes += __shfl_xor(n_bytes, o);\n    n_line += __shfl_xor(n_line, o);\n  }\n  if (lane == 0) {\n    atomicAdd(&s_stat[0], n_matched);",
                 "  for (int o = 32; o > 0; o >>= 1) {\n    n_matched += __shfl_xor(n_matched, o);\n    n_bytes += __shfl_xor(n_bytes, o);\n    n_line += __shfl_xor(n_line, o);\n  }\n  if (touch_sink == 0x9E3779B9u && a.n == 1u) n_line += 1u;\n  if (lane == 0) {\n    atomicAdd(&s_stat[0], n_matched);")],
    # the one-launch 2-byte hand-back with one segment per wave (round 5's) instead of four
    "c16spw1": [("constexpr uint32_t kSmall16Spw = 4;", "constexpr uint32_t kSmall16Spw = 1;")],
    # no hand-back inside the one-tile 2-byte sweep (KWK_TUNE_TAIL_HANDBACK 0 by default)
    "notail": [("  bool tail_hb = true;", "  bool tail_hb = false;")],
    # sweep8: the work list built k-major (ballot per id position: a pass's items are the same id position
    # of many lanes, LDS bank-spread; contiguous list writes) instead of lane-major (records' order changes:
    # the bitmap hand-back would need its codes ranked; C5 cost isolation only)
    "s8_kmajor": [('          if (rdy) {\n            while (m) {\n              const uint32_t k = (uint32_t)__builtin_ctz(m);\n              m &= m - 1u;\n              *wp++ = (uint16_t)((ent0 ^ ((k & 7u) * 0x104u | k >> 3)) | ((ready >> k) & 1u) << 15);\n            }\n          } else {\n            while (m) {\n              const uint32_t k = (uint32_t)__builtin_ctz(m);\n              m &= m - 1u;\n              *wp++ = (uint16_t)(ent0 ^ ((k & 7u) * 0x104u | k >> 3));\n            }\n          }', "          (void)m; (void)wp;\n          uint32_t kbase = 0;\n#pragma unroll\n          for (uint32_t k = 0; k < 32u; ++k) {  // k-major: a pass's items are one k of many lanes\n            const bool b = (need >> k) & 1u;\n            const unsigned long long bal = ballot(b);\n            const uint32_t p = kbase + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));\n            if (b) wl[p] = (uint16_t)((ent0 ^ ((k & 7u) * 0x104u | k >> 3)) | ((ready >> k) & 1u) << 15);\n            kbase += (uint32_t)__popcll(bal);\n          }")],
    # the 2-byte scan + expansion hand-back (C5) with 4 (round 5) / 16 segments per wave instead of 8
    "dwmb4": [("constexpr int kDwMinBlocks = 5; ", "constexpr int kDwMinBlocks = 4; ")],
    "dwmb6": [("constexpr int kDwMinBlocks = 5; ", "constexpr int kDwMinBlocks = 6; ")],
    "ucu16": [("    const uint32_t per_cu = 8u;", "    const uint32_t per_cu = 16u;")],
    "ucu32": [("    const uint32_t per_cu = 8u;", "    const uint32_t per_cu = 32u;")],
    "ur2": [("constexpr uint32_t kUChunkRows = 4; ", "constexpr uint32_t kUChunkRows = 2; ")],
    "ur1": [("constexpr uint32_t kUChunkRows = 4; ", "constexpr uint32_t kUChunkRows = 1; ")],
    "c16s8": [("constexpr uint32_t kSmall16Spw = 4;", "constexpr uint32_t kSmall16Spw = 8;")],
    "c16s2": [("constexpr uint32_t kSmall16Spw = 4;", "constexpr uint32_t kSmall16Spw = 2;")],
    "c16x4": [("constexpr uint32_t kCompact16Spw = 8;", "constexpr uint32_t kCompact16Spw = 4;")],
    "c16x16": [("constexpr uint32_t kCompact16Spw = 8;", "constexpr uint32_t kCompact16Spw = 16;")],
    # the word sweep's phase 3 stores no state lines
    "w_nophase3": [("        store_chunk_nt(&gq[(wbase + (uint32_t)q * 64u * kC + lane * kC) / kC], nv);\n",
                    "        (void)gq;\n")],
}


def build(names):
    os.makedirs(OUT, exist_ok=True)
    src = open(SRC).read()

    def one(name):
        s = src
        parts = name.split("+")  # "a+b": variant b's replacements applied to variant a's source
        if parts[0] == "head":  # the committed engine.hip: same-box A/B against the working tree ("base");
            # the GPU box has no .git: `variants.py snap` leaves HEAD's source in tools/ab/ first
            snap = os.path.join(ROOT, "tools", "ab", "engine_head.hip")
            if os.path.exists(snap):
                s = open(snap).read()
            else:
                s = subprocess.run(["git", "show", "HEAD:kwok_amd/csrc/engine.hip"], cwd=ROOT, check=True,
                                   capture_output=True, text=True).stdout
        for part in parts:
            for old, new in VARIANTS[part]:
                if old not in s:
                    raise SystemExit(f"variant {name}: pattern not found: {old[:60]!r}")
                s = s.replace(old, new)
        path = os.path.join(OUT, f"engine_{name}.hip")
        open(path, "w").write(s)
        so = os.path.join(OUT, f"libkwok_engine_{name}.so")
        cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-unused-result",
               "-Wno-unused-value", "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "kwok_amd", "csrc"),
               "-o", so, path]
        subprocess.run(cmd, check=True)
        return so

    with ThreadPoolExecutor(8) as ex:
        for so in ex.map(one, list(dict.fromkeys(names))):  # "run a b a b" alternates; each is built once
            print(so, flush=True)


def child(name, hbm_nodes, steps, state="auto"):
    sys.path.insert(0, ROOT)
    from kwok_amd.host import abi
    abi.LIB_PATH = os.path.join(OUT, f"libkwok_engine_{name}.so")
    import bench
    args = argparse.Namespace(hbm_nodes=hbm_nodes, pods_per_node=100, seed=0x6B776F6B, job_frac=0.1,
                              hbm_steps=steps, hbm_warmup=12, hbm_state=state)
    r = bench.measure_hbm_working_set(args, 0)
    print(json.dumps({"variant": name, "state": state, **r}), flush=True)


def child_c5(name, steps, nodes=0):
    """The C5 bench line (pod sweep timing) with the variant library (nodes > 0: that many nodes, e.g.
    the N = 8 shard's 125000)."""
    sys.path.insert(0, ROOT)
    from kwok_amd.host import abi
    abi.LIB_PATH = os.path.join(OUT, f"libkwok_engine_{name}.so")
    import bench
    sys.argv = ["bench.py", "--steps", str(steps), "--warmup", "5", "--no-pmc", "--no-cpu-baseline", "--hbm-nodes", "0",
                "--pcie-steps", "0", "--emit-steps", "0"] + (["--nodes", str(nodes)] if nodes else [])
    bench.main()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=("build", "run", "child", "snap"))
    ap.add_argument("names", nargs="*")
    ap.add_argument("--hbm-nodes", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--c5", action="store_true", help="time the C5 pod sweep instead of the C2 working set")
    ap.add_argument("--c5-nodes", type=int, default=0, help="with --c5: the bench's --nodes (0: the default 1M)")
    ap.add_argument("--state", default="auto", help="C2 pod state format (auto: fused records, u32: split due)")
    a = ap.parse_args()
    names = a.names or list(VARIANTS)
    if a.cmd == "snap":
        os.makedirs(os.path.join(ROOT, "tools", "ab"), exist_ok=True)
        src = subprocess.run(["git", "show", "HEAD:kwok_amd/csrc/engine.hip"], cwd=ROOT, check=True,
                             capture_output=True, text=True).stdout
        open(os.path.join(ROOT, "tools", "ab", "engine_head.hip"), "w").write(src)
    elif a.cmd == "build":
        build(names)
    elif a.cmd == "child":
        if a.c5:
            child_c5(names[0], a.steps, a.c5_nodes)
        else:
            child(names[0], a.hbm_nodes, a.steps, a.state)
    else:
        for n in names:
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "child", n, "--hbm-nodes", str(a.hbm_nodes),
                                "--steps", str(a.steps), "--state", a.state, "--c5-nodes", str(a.c5_nodes)] +
                               (["--c5"] if a.c5 else []), timeout=300)
            if r.returncode != 0:
                raise SystemExit(f"variant {n}: rc {r.returncode}")


if __name__ == "__main__":
    main()
