"""The benchmarked sweep kernels against the oracle at the sizes they run.

The small-cluster parity tests (test_gpu_parity.py) exercise the one-block-per-tile kernel
shapes; the bench's C5 pod sweep runs `sweep16_fsm_kernel<harness, 4, persistent, depth 2>`,
which only launches once the 8192-word tiles outnumber twice the resident blocks (~17M pods
on 256 CUs), and the C2 mix runs `sweepw_kernel<4>` over millions of pods.  Here both run at
those sizes and a deterministic sample of slots (every 997th / 4999th) is checked against
`OracleSim` at every step: the fired records of the sampled slots (slot, stage, flags), and
each sampled object's pending stage, due time, feature bits, deletion column and dirty flag.

Objects are independent within a step (a pod reads only its own fields) and the
Philox counter is the global slot, so simulating the sampled objects alone is
exact: reference `pkg/utils/lifecycle/lifecycle.go:125-191,313-341` (Match, Delay),
`pkg/kwok/controllers/pod_controller.go:196-360` (preprocess, playStage)."""
import numpy as np
import pytest

from tests.parity_util import compare_state

pytestmark = pytest.mark.gpu

NOW0 = 1_700_000_000 * 10**9
SEED = 0x6B776F6B


def _sampled_run(prog, eng, stage_files, variants, index, slots, steps, dt_ns, kernel, persistent, kind_salt=0,
                 harness=True):
    from kwok_amd.host import abi
    from oracle.next_ref import load_stage_docs
    from oracle.sim import OracleSim
    objs = [variants[int(index[s])] for s in slots]
    sim = OracleSim(load_stage_docs(*stage_files), objs, harness=harness, slots=slots, kind_salt=kind_salt)
    sample = np.asarray(slots, dtype=np.int64)
    total = 0
    for k in range(steps):
        now = NOW0 + k * dt_ns
        eng.step(now, SEED, k)
        info = eng.last_sweep()
        assert info["kernel"] == kernel and info["persistent"] == persistent and info["harness"] == int(harness), info
        if persistent:
            assert info["grid"] < info["tiles"] and info["depth"] == 2, info
        f = eng.fired()
        assert len(np.unique(f["slot"])) == len(f), f"step {k}: a slot fired twice"
        sel = f[np.isin(f["slot"].astype(np.int64), sample)]
        got = sorted((int(r["slot"]), int(r["stage"]), int(r["flags"])) for r in sel)
        exp = sorted(sim.step(now, SEED, k))
        assert got == exp, f"step {k}: device-only {sorted(set(got) - set(exp))[:6]} oracle-only " \
                           f"{sorted(set(exp) - set(got))[:6]}"
        total += len(exp)
        compare_state(prog, eng, sim, k, rows=_rows_at(eng, slots))
    return total


def _rows_at(eng, slots):
    """(hot, deletion_s) of the sampled slots only (kwk_read per slot: the sample is small)."""
    from kwok_amd.host import abi
    hot = np.zeros(len(slots), dtype=abi.HOT_DTYPE)
    dels = np.zeros(len(slots), dtype=np.int64)
    for j, s in enumerate(slots):
        h, d = eng.read(int(s), 1)
        hot[j], dels[j] = h[0], d[0]
    return hot, dels


@pytest.mark.parametrize("state", ["auto", "u16", "auto-shard"])
def test_c5_persistent_table_sweep_sampled_oracle(state):
    """C5 pod shape (pod-fast, 100 pods per node, 10 % Job-owned, harness churn) at the sizes
    where the sweeps run persistent with two tiles in flight (the shard: one tile per workgroup): the 1-byte dictionary-id sweep
    (auto: sweep8_kernel, the bench's kernel; 8192-id tiles, 40M pods) and the 2-byte table-only
    sweep (u16: sweep16_fsm_kernel, 20M pods), every ~10000th / 4999th slot checked each step;
    auto-shard: the 12.5M-pod shard of N = 8 (1526 one-tile workgroups)."""
    from bench import shard_pod_variants
    from kwok_amd import workload as W
    from kwok_amd.host import abi
    from kwok_amd.host.compiler import HarnessSpec, KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files
    n = {"auto": 40_000_000, "u16": 20_000_000, "auto-shard": 12_500_000}[state]
    persistent = 0 if state == "auto-shard" else 1  # the shard's tiles fit one resident grid
    state = "auto" if state == "auto-shard" else state
    files = W.stage_paths(W.POD_FAST)
    pvars = [W.pod_object("p", "n"), W.pod_object("p", "n", job=True)]
    prog = KindProgram(load_stage_files(*files), HarnessSpec())
    prog.explore(pvars)
    ing = Ingest(prog)
    idx = shard_pod_variants(0, n, SEED, 0.1)
    hot, dels, rec, cls = ing.variant_columns(pvars, idx)
    eng = Engine(prog, capacity=n, state=state)
    try:
        eng.load_stages()
        eng.set_harness(True)
        eng.load(hot, dels, rec, cls, ing.record_array())
        del hot, dels, rec, cls
        slots = list(range(3, n, 9973 if state == "auto" else 4999))
        assert int(np.sum(idx[slots])) > 100  # Job-owned pods (pod-complete) are in the sample
        kernel = abi.SWEEP_8 if state == "auto" else abi.SWEEP_16_FSM
        total = _sampled_run(prog, eng, files, pvars, idx, slots, 10, 10**9, kernel, persistent)
        assert total > len(slots)  # every pod became ready once, Job pods completed, deletions re-created
        assert eng.stats()["state_bytes"] == (1 if state == "auto" else 2)
    finally:
        eng.close()


@pytest.mark.parametrize("n", [40_000_000, 12_500_000])
def test_c5_fused_steps_every_step_sampled_oracle(n):
    """The headline kernel as the bench runs it: `sweep8_kernel<..., 4>`, four
    steps per launch over the C5 pod shape — 40M pods on the persistent grid, 12.5M (the N = 8
    shard) one tile per workgroup — stepped by kwk_step_n calls of 10 steps (launches of 4 + 4 + 2
    steps, each launch's 2-byte hand-backs in one launch), and EVERY step's list read by step
    through the hand-back ring (kwk_fired_keep + kwk_fired_fetch_step) and decoded on the host: the
    fired records of every ~9973rd slot must equal `OracleSim` stepped one step at a time, at each
    of the 20 steps; after each call the sampled objects' states equal the oracle's."""
    from bench import shard_pod_variants
    from kwok_amd import workload as W
    from kwok_amd.host import abi
    from kwok_amd.host.compiler import HarnessSpec, KindProgram
    from kwok_amd.host.engine import Engine, Ingest, PinnedBuffer
    from kwok_amd.host.stages import load_stage_files
    from oracle.next_ref import load_stage_docs
    from oracle.sim import OracleSim
    files = W.stage_paths(W.POD_FAST)
    pvars = [W.pod_object("p", "n"), W.pod_object("p", "n", job=True)]
    prog = KindProgram(load_stage_files(*files), HarnessSpec())
    prog.explore(pvars)
    ing = Ingest(prog)
    idx = shard_pod_variants(0, n, SEED, 0.1)
    hot, dels, rec, cls = ing.variant_columns(pvars, idx)
    eng = Engine(prog, capacity=n, state="auto")
    bufs = [(PinnedBuffer(2 * n + 64), PinnedBuffer(4 * (n // 2048 + 64))) for _ in range(10)]
    try:
        eng.load_stages()
        eng.set_harness(True)
        eng.load(hot, dels, rec, cls, ing.record_array())
        del hot, dels, rec, cls
        eng.fired_keep(10)
        slots = list(range(3, n, 9973))
        sample = np.asarray(slots, dtype=np.int64)
        sim = OracleSim(load_stage_docs(*files), [pvars[int(idx[s])] for s in slots], harness=True, slots=slots)
        total = 0
        for call in range(2):
            k0 = 10 * call
            eng.step_n(10, NOW0 + k0 * 10**9, 10**9, SEED, k0, "packed16")
            info = eng.last_sweep()
            assert info["kernel"] == abi.SWEEP_8 and info["steps"] == 2, info
            assert info["persistent"] == (1 if n == 40_000_000 else 0), info
            infos = [eng.fetch_step(k0 + j, *bufs[j]) for j in range(10)]
            eng.fetch_wait()
            for j, fi in enumerate(infos):
                k = k0 + j
                out, cnt = bufs[j]
                slot, stage, flags = abi.fired16_decode(out.array(np.uint16, fi["n_records"]),
                                                        cnt.array(np.uint32, fi["n_segs"]), fi["region_slots"])
                assert len(np.unique(slot)) == len(slot), f"step {k}: a slot fired twice"
                sel = np.isin(slot.astype(np.int64), sample)
                got = sorted(zip(slot[sel].tolist(), stage[sel].tolist(), flags[sel].tolist()))
                exp = sorted(sim.step(NOW0 + k * 10**9, SEED, k))
                assert got == exp, f"step {k}: device-only {sorted(set(got) - set(exp))[:6]} oracle-only " \
                                   f"{sorted(set(exp) - set(got))[:6]}"
                total += len(exp)
            compare_state(prog, eng, sim, k0 + 9, rows=_rows_at(eng, slots))
        assert total > len(slots)
    finally:
        eng.close()
        for x in bufs:
            for p in x:
                p.close()


@pytest.mark.parametrize("state", ["u32", "auto"])
def test_c2_word_sweep_sampled_oracle(state):
    """C2 stage mix (pod-general + chaos: weighted picks, jitter draws, value records, the
    deletion column) at 4M pods through `sweepw_kernel<4>` (u32: 4-byte words + the due column)
    and `sweepw_kernel<8, fused>` (auto: the 8-byte records with the relative due time, the
    benchmarked C2 kernel), every 997th slot each step."""
    from kwok_amd import workload as W
    from kwok_amd.host import abi
    from kwok_amd.host.compiler import HarnessSpec, KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files
    n = 4_000_000
    files = W.stage_paths(W.POD_GENERAL + W.POD_CHAOS)
    pvars, pidx = W.c2_pod_variants(0, n, seed=SEED, job_frac=0.1)
    prog = KindProgram(load_stage_files(*files), HarnessSpec())
    prog.explore(pvars)
    ing = Ingest(prog)
    hot, dels, rec, cls = ing.variant_columns(pvars, pidx)
    eng = Engine(prog, capacity=n, state=state, max_records=max(1, len(ing.records)) + 16)
    try:
        eng.load_stages()
        eng.set_harness(True)
        eng.load(hot, dels, rec, cls, ing.record_array())
        assert eng.stats()["state_bytes"] == (4 if state == "u32" else 8)
        slots = list(range(1, n, 997))
        kernel = abi.SWEEP_W4 if state == "u32" else abi.SWEEP_WD
        # fused: 1953 tiles over 5 workgroups per CU, each looping over its tiles; 4-byte: 977 tiles,
        # one workgroup each
        total = _sampled_run(prog, eng, files, pvars, pidx, slots, 24, 500 * 10**6, kernel, 1 if state == "auto" else 0)
        assert total > len(slots)
        fired = {k: v for k, v in eng.stats()["fired_per_stage"].items() if v}
        assert any("failed" in name for name in fired), fired  # weighted picks ran
    finally:
        eng.close()


def test_node_heartbeat_persistent_cold_path_sampled_oracle():
    """The cold path of the persistent table sweep: node-initialize +
    node-heartbeat (delay + Philox jitter: general table entries, run by `process_object` in
    the per-tile cold loop) over 20M nodes, so `sweep16_fsm_kernel<false, 4, persistent,
    depth 2>` runs on a persistent grid and every heartbeat goes through the cold loop;
    every 4999th slot checked against the oracle at each step.  The out-of-line variant of that
    loop faulted on the small engine of test_node_fast_heartbeat; this is the
    shared code it called, at the size where the grid strides."""
    from kwok_amd import workload as W
    from kwok_amd.host import abi
    from kwok_amd.host.compiler import KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files
    n = 20_000_000
    files = W.stage_paths(W.NODE_FAST + W.NODE_HEARTBEAT)
    nvars = [W.node_object("n"), W.node_object("n", annotations={"example.com/zone": "b"})]
    prog = KindProgram(load_stage_files(*files))
    prog.explore(nvars)
    ing = Ingest(prog)
    idx = (np.arange(n, dtype=np.int64) * 2654435761 >> 7) & 1
    hot, dels, rec, cls = ing.variant_columns(nvars, idx)
    eng = Engine(prog, capacity=n, kind_salt=1)
    try:
        eng.load_stages()
        eng.load(hot, dels, rec, cls, ing.record_array())
        del hot, dels, rec, cls
        assert eng.stats()["state_bytes"] == 2  # jitter: not table-only, so not the 1-byte ids
        slots = list(range(7, n, 4999))
        # 2 s per step: node-initialize, then heartbeats every 20 s + up to 5 s of jitter
        total = _sampled_run(prog, eng, files, nvars, idx, slots, 16, 2 * 10**9, abi.SWEEP_16_FSM, 1,
                             kind_salt=1, harness=False)
        per = eng.stats()["fired_per_stage"]
        assert per["node-initialize"] == n and per["node-heartbeat"] > n // 2, per
        assert total >= 2 * len(slots)
    finally:
        eng.close()
