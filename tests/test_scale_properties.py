"""Parity at scale through size-independent properties: the C5 pod shape (100 pods per node,
10 % Job-owned, pod-fast, harness churn) at 4M pods, stepped by the three sweep kernels —
the 2-byte whole-line sweep with its transition table, the 4-byte and the 8-byte
word-granular sweeps (each oracle-checked at small sizes in test_gpu_parity.py) — must fire
the same (slot, stage, flags) sets and leave identical object states, step after step.
Also: fired slots are unique per step, per-stage counts add up, and every pod that fires
pod-ready this step was not Running before (the stage order of the pod-fast program)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_NODES, PPN, STEPS = 40_000, 100, 20


def _pods(state, n_nodes=N_NODES, tuning=None):
    from bench import shard_pod_variants
    from kwok_amd import workload as W
    from kwok_amd.host.compiler import HarnessSpec, KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files
    pvars = [W.pod_object("p", "n"), W.pod_object("p", "n", job=True)]
    prog = KindProgram(load_stage_files(*W.stage_paths(W.POD_FAST)), HarnessSpec())
    prog.explore(pvars)
    ing = Ingest(prog)
    idx = shard_pod_variants(0, n_nodes * PPN, 0x6B776F6B, 0.1)
    hot, dels, rec, cls = ing.variant_columns(pvars, idx)
    eng = Engine(prog, capacity=n_nodes * PPN, state=state)
    for k, v in (tuning or {}).items():
        eng.set_tuning(k, v)
    eng.load_stages()
    eng.set_harness(True)
    eng.load(hot, dels, rec, cls, ing.record_array())
    return prog, eng


def _fired_key(f):
    return np.sort(f["slot"].astype(np.uint64) << np.uint64(32) | f["stage"].astype(np.uint64) << np.uint64(16) |
                   f["flags"].astype(np.uint64))


def test_three_sweeps_agree_at_4m_pods():
    engines = {s: _pods(s) for s in ("auto", "u16", "u32", "wide")}
    try:
        sb = {s: e.stats()["state_bytes"] for s, (_, e) in engines.items()}
        assert sb == {"auto": 1, "u16": 2, "u32": 4, "wide": 8}, sb
        now0 = 1_700_000_000 * 10**9
        for k in range(STEPS):
            keys = {}
            for s, (prog, e) in engines.items():
                e.step(now0 + k * 10**9, 0x6B776F6B, k)
                f = e.fired()
                assert len(np.unique(f["slot"])) == len(f), f"{s} step {k}: a slot fired twice"
                keys[s] = _fired_key(f)
            for s in ("u16", "u32", "wide"):
                assert np.array_equal(keys["auto"], keys[s]), f"step {k}: {s}"
            assert len(keys["auto"]) > 0
        states = {s: e.read() for s, (_, e) in engines.items()}
        for s in ("u16", "u32", "wide"):
            for col in ("pred", "sched"):
                assert np.array_equal(states["auto"][0][col], states[s][0][col]), (s, col)
            pend = (states["auto"][0]["sched"] & 0xFF) != 0xFF
            assert np.array_equal(states["auto"][0]["due"][pend], states[s][0]["due"][pend]), s
        st = {s: e.stats() for s, (_, e) in engines.items()}
        for s in ("u16", "u32", "wide"):
            assert st[s]["fired"] == st["auto"]["fired"] and st[s]["fired_per_stage"] == st["auto"]["fired_per_stage"]
        assert sum(st["auto"]["fired_per_stage"].values()) == st["auto"]["fired"]
    finally:
        for _, e in engines.values():
            e.close()


def test_sweep16_tile_shapes_agree_at_17m_pods():
    """The 2-byte sweep's kernels and tile shapes: the table-only sweep (pod-fast has no general
    table entry) with the next 2 or 1 tiles in flight and the general sweep16_kernel
    (KWK_TUNE_SWEEP16 kernel 0), at Q = 4 (8192-word tiles, persistent grid: at 17M pods the tiles
    outnumber twice the resident blocks), Q = 2 and Q = 1 (one block per tile) must fire the
    same sets, leave the same words and count the same statistics."""
    from kwok_amd.host import abi
    sh = lambda **k: {abi.TUNE_SWEEP16: abi.sweep16_shape(**k)}  # noqa: E731
    shapes = {"4": sh(q=4), "4-d1": sh(q=4, kernel=1), "4-gen": sh(q=4, kernel=0), "2": sh(q=2), "1": sh(q=1),
              "1-gen": sh(q=1, kernel=0)}
    byte_shapes = {"id8": {}, "id8-d1": sh(kernel=1)}  # the 1-byte id sweep, 2 / 1 tiles in flight
    engines = {}
    try:
        for q, tuning in shapes.items():
            engines[q] = _pods("u16", n_nodes=170_000, tuning=tuning)
        for q, tuning in byte_shapes.items():
            engines[q] = _pods("auto", n_nodes=170_000, tuning=tuning)
        assert all(e.stats()["state_bytes"] == (1 if q.startswith("id8") else 2) for q, (_, e) in engines.items())
        shapes.update(byte_shapes)
        now0 = 1_700_000_000 * 10**9
        for k in range(10):
            keys = {}
            for q, (_, e) in engines.items():
                e.step(now0 + k * 10**9, 0x6B776F6B, k)
                keys[q] = _fired_key(e.fired())
            assert len(keys["4"]) > 0
            for q in shapes:
                assert np.array_equal(keys["4"], keys[q]), f"step {k}: {q}"
        states = {q: e.read()[0] for q, (_, e) in engines.items()}
        for q in shapes:
            for col in ("pred", "sched"):
                assert np.array_equal(states["4"][col], states[q][col]), (q, col)
        st = {q: e.stats() for q, (_, e) in engines.items()}
        for q in shapes:
            assert st[q]["fired_per_stage"] == st["4"]["fired_per_stage"], q
            for key in ("fired", "matched"):
                assert st[q][key] == st["4"][key], (q, key)
        # byte counts include one fired-count word per (tile, wave) segment: equal per tile shape
        for q, ref in (("4-d1", "4"), ("4-gen", "4"), ("1-gen", "1"), ("id8-d1", "id8")):
            for key in ("bytes", "line_bytes"):
                assert st[q][key] == st[ref][key], (q, key)
    finally:
        for _, e in engines.values():
            e.close()


HANDBACK_PATHS = (8192, 0)  # KWK_TUNE_COMPACT_SMALL; [0] = default


def _handback_path(eng, path):
    from kwok_amd.host import abi
    eng.set_tuning(abi.TUNE_COMPACT_SMALL, path)


def test_handback_pair_equals_one_launch_at_4m_pods():
    """The fired hand-back's two paths over the same step's segments: the one-launch compaction
    that re-sums the counts (at most 8192 segments, the default here) and the scan + expansion pair
    (KWK_TUNE_COMPACT_SMALL 0) give the same dense list in the same order; every slot once."""
    prog, eng = _pods("auto")
    try:
        now0 = 1_700_000_000 * 10**9
        for k in range(4):
            eng.step(now0 + k * 10**9, 0x6B776F6B, k)
            lists = []
            for path in HANDBACK_PATHS:
                _handback_path(eng, path)
                eng.fired_compact()
                lists.append(eng.fired())
            one, pair = lists[0], lists[-1]
            assert len(one) > 0 and all(np.array_equal(one, x) for x in lists[1:]), f"step {k}"
            sl = np.sort(pair["slot"].astype(np.int64))
            assert np.all(np.diff(sl) > 0), f"step {k}: a slot fired twice"
    finally:
        eng.close()


@pytest.mark.parametrize("state", ["auto", "u16", "dw"])
def test_packed_handback_equals_records_at_4m_pods(state):
    """The packed hand-back (kwk_fired_compact_packed / kwk_fired_packed: 4-byte records, stage in
    bits 31-27, slot in 26-0) over the same step's segments as the 8-byte list, through both
    compaction paths (one launch at <= 8192 segments, the scan + expansion pair above): the same
    (slot, stage) sequence; kwk_fired after a packed compaction re-expands the full records
    (flags included); kwk_step_n with KWK_COMPACT_PACKED leaves the same packed list as the
    per-step calls.  1-byte ids (sweep8), 2-byte words, fused 8-byte records (C2 mix).  The 2-byte
    hand-back (kwk_fired_packed16) of the 1-byte sweep decodes to the same (slot, stage, flags); the
    other formats refuse it."""
    from kwok_amd.host import abi
    if state == "dw":
        from kwok_amd import workload as W
        from kwok_amd.host.compiler import HarnessSpec, KindProgram
        from kwok_amd.host.engine import Engine, Ingest
        from kwok_amd.host.stages import load_stage_files
        n = 4_000_000
        pvars, pidx = W.c2_pod_variants(0, n, seed=0x6B776F6B, job_frac=0.1)
        prog = KindProgram(load_stage_files(*W.stage_paths(W.POD_GENERAL + W.POD_CHAOS)), HarnessSpec())
        prog.explore(pvars)
        ing = Ingest(prog)
        hot, dels, rec, cls = ing.variant_columns(pvars, pidx)
        eng = Engine(prog, capacity=n, max_records=max(1, len(ing.records)) + 16)
        eng.load_stages()
        eng.set_harness(True)
        eng.load(hot, dels, rec, cls, ing.record_array())
        dt = 500 * 10**6
    else:
        prog, eng = _pods(state)
        dt = 10**9
    try:
        now0 = 1_700_000_000 * 10**9
        for k in range(4):
            eng.step(now0 + k * dt, 0x6B776F6B, k)
            for small in HANDBACK_PATHS:
                _handback_path(eng, small)
                eng.fired_compact(packed=True)
                pk = eng.fired_packed()
                full = eng.fired()  # re-expanded from the same segments
                assert len(pk) == len(full) > 0, (k, small)
                assert np.array_equal(pk & np.uint32(0x7FFFFFF), full["slot"]), (k, small)
                assert np.array_equal(pk >> np.uint32(27), full["stage"].astype(np.uint32)), (k, small)
            # the 2-byte records (1-byte sweep, <= 4 stages): same slots, stages and flags
            if state == "auto":
                eng.fired_compact("16")
                recs, cnt, rs = eng.fired_packed16()
                full = eng.fired()
                sl, sg, fl = abi.fired16_decode(recs, cnt, rs)
                assert len(recs) == len(full) and int(cnt.sum()) == len(full), k
                assert np.array_equal(sl, full["slot"].astype(np.int64)), k
                assert np.array_equal(sg, full["stage"].astype(np.uint32)), k
                assert np.array_equal(fl, full["flags"].astype(np.uint32)), k
                # the bitmap hand-back (maps + 2-bit codes), both paths: same (slot, stage) sequence
                for small in HANDBACK_PATHS:
                    _handback_path(eng, small)
                    eng.fired_compact("bits")
                    words, n_tr, ns, rs2 = eng.fired_bits()
                    assert n_tr == len(full) and ns == len(cnt) and rs2 == rs, (k, small)
                    bsl, bsg = abi.bits_decode(words, ns, rs2)
                    assert int((words[:ns] & np.uint32(0xFFFF)).astype(np.int64).sum()) == n_tr, (k, small)
                    assert np.array_equal(bsl, full["slot"].astype(np.int64)), (k, small)
                    assert np.array_equal(bsg, full["stage"].astype(np.uint32)), (k, small)
                _handback_path(eng, HANDBACK_PATHS[0])
            else:
                with pytest.raises(abi.EngineError):
                    eng.fired_packed16()
                with pytest.raises(abi.EngineError):
                    eng.fired_bits()
        _handback_path(eng, HANDBACK_PATHS[0])
        ref = eng.fired_packed()
        eng.step_n(1, now0 + 4 * dt, dt, 0x6B776F6B, 4, "packed")
        a = eng.fired_packed()
        eng2_full = eng.fired()
        assert np.array_equal(a & np.uint32(0x7FFFFFF), eng2_full["slot"]) and len(a) > 0 and len(ref) > 0
        if state == "auto":  # kwk_step_n leaves the 2-byte list itself
            eng.step_n(1, now0 + 5 * dt, dt, 0x6B776F6B, 5, "packed16")
            recs, cnt, rs = eng.fired_packed16()
            full = eng.fired()
            sl, sg, _ = abi.fired16_decode(recs, cnt, rs)
            assert len(recs) > 0 and np.array_equal(sl, full["slot"].astype(np.int64))
            eng.step_n(1, now0 + 6 * dt, dt, 0x6B776F6B, 6, "bits")
            words, n_tr, ns, rs = eng.fired_bits()
            full = eng.fired()
            bsl, bsg = abi.bits_decode(words, ns, rs)
            assert n_tr == len(full) > 0 and np.array_equal(bsl, full["slot"].astype(np.int64))
            assert np.array_equal(bsg, full["stage"].astype(np.uint32))
    finally:
        eng.close()


def test_aggregates_and_handback_at_17m_pods():
    """At 17M pods (the 2-byte sweep's persistent grid): kwk_count and kwk_usage against the
    state read back through kwk_read (numpy), and the device-compacted fired list (one
    look-back pass): every slot once, as many records as the step's transition count."""
    from kwok_amd.host import abi
    from kwok_amd.host.cluster import phase_masks
    n_nodes = 170_000
    prog, eng = _pods("auto", n_nodes=n_nodes)
    try:
        n = n_nodes * PPN
        rng = np.random.default_rng(5)
        cpu = rng.random(37) * 4
        mem = rng.random(41) * 2**32
        ci, mi, nc = rng.integers(0, 37, n), rng.integers(0, 41, n), rng.integers(1, 5, n)
        keys = (ci | (mi << 14) | (nc << 28)).astype(np.uint32)
        ptr = np.concatenate([[0], np.cumsum(rng.integers(0, 2 * PPN, n_nodes))]).astype(np.int64)
        ptr = (ptr * (n / ptr[-1])).astype(np.uint32)
        ptr[-1] = n
        eng.usage_config(ptr, keys, cpu, mem)
        pm = phase_masks(prog, values=("Running", "Succeeded"))
        masks = [0, pm["Running"], pm["Succeeded"], pm["Running"] | pm["Succeeded"]]
        now0 = 1_700_000_000 * 10**9
        prev = eng.stats()["fired"]
        for k in range(6):
            eng.step(now0 + k * 10**9, 0x6B776F6B, k)
            eng.fired_compact()
            f = eng.fired()
            st = eng.stats()["fired"]
            assert len(f) == st - prev and len(f) > 0
            prev = st
            sl = np.sort(f["slot"].astype(np.int64))
            assert np.all(np.diff(sl) > 0) and sl[-1] < n, f"step {k}: a slot fired twice / out of range"
            got = eng.count(masks)
            hot, _ = eng.read()
            alive = (hot["sched"] & abi.F_ALIVE) != 0
            want = [int(alive.sum())] + [int((alive & ((hot["pred"] & m) != 0)).sum()) for m in masks[1:]]
            assert got.tolist() == want, f"step {k}"
            eng.usage(now0 + k * 10**9)
            node, total = eng.usage_read()
            vc = np.where(alive, nc * cpu[ci], 0.0)
            vm = np.where(alive, nc * mem[mi], 0.0)
            seg_c = np.add.reduceat(np.append(vc, 0.0), ptr[:-1].astype(np.int64))
            seg_m = np.add.reduceat(np.append(vm, 0.0), ptr[:-1].astype(np.int64))
            empty = ptr[1:] == ptr[:-1]
            seg_c[empty] = 0.0
            seg_m[empty] = 0.0
            np.testing.assert_allclose(node[:, 0], seg_c, rtol=1e-9, atol=1e-9)
            np.testing.assert_allclose(node[:, 1], seg_m, rtol=1e-9, atol=1e-3)
            np.testing.assert_allclose(total, [vc.sum(), vm.sum()], rtol=1e-9)
    finally:
        eng.close()


def _c2_program(n):
    from kwok_amd import workload as W
    from kwok_amd.host.compiler import HarnessSpec, KindProgram
    from kwok_amd.host.stages import load_stage_files
    pvars, _ = W.c2_pod_variants(0, n, seed=0x6B776F6B, job_frac=0.1)
    prog = KindProgram(load_stage_files(*W.stage_paths(W.POD_GENERAL + W.POD_CHAOS)), HarnessSpec())
    prog.explore(pvars)  # one program for every shard (same classes / features)
    return prog


def _c2_pods(prog, lo, hi, state):
    """Pods [lo, hi) of the C2 mix (pod-general + pod-chaos: weighted picks, jitter draws, value
    records, deletion-timestamp getters) as one engine with slot_base = lo."""
    from kwok_amd import workload as W
    from kwok_amd.host.engine import Engine, Ingest
    pvars, pidx = W.c2_pod_variants(lo, hi, seed=0x6B776F6B, job_frac=0.1)
    ing = Ingest(prog)
    hot, dels, rec, cls = ing.variant_columns(pvars, pidx)
    eng = Engine(prog, capacity=hi - lo, state=state, slot_base=lo, max_records=max(1, len(ing.records)) + 16)
    eng.load_stages()
    eng.set_harness(True)
    eng.load(hot, dels, rec, cls, ing.record_array())
    return prog, eng


def test_c2_mix_formats_and_shards_agree_at_4m_pods():
    """The word sweep on the C2 stage mix at 4M pods: the 4-byte, fused 8-byte and wide 8-byte
    formats and two half-cluster shards (global-slot RNG keys) fire the same (slot, stage, flags)
    sets and leave the same objects, step after step; the weighted-pick / jitter / record paths
    all run."""
    n = 4_000_000
    prog = _c2_program(n)
    eng = {"u32": _c2_pods(prog, 0, n, "u32"), "wide": _c2_pods(prog, 0, n, "wide"), "dw": _c2_pods(prog, 0, n, "auto"),
           "s0": _c2_pods(prog, 0, n // 2, "u32"), "s1": _c2_pods(prog, n // 2, n, "u32")}
    try:
        assert eng["u32"][1].stats()["state_bytes"] == 4 and eng["wide"][1].stats()["state_bytes"] == 8
        assert eng["dw"][1].stats()["state_bytes"] == 8
        now0 = 1_700_000_000 * 10**9
        total = 0
        for k in range(24):
            keys = {}
            for s, (_, e) in eng.items():
                e.step(now0 + k * 500 * 10**6, 0x6B776F6B, k)
                f = e.fired()
                assert len(np.unique(f["slot"])) == len(f), f"{s} step {k}: a slot fired twice"
                if s == "s1":
                    f = f.copy()
                    f["slot"] += n // 2
                keys[s] = _fired_key(f)
            shards = np.sort(np.concatenate([keys["s0"], keys["s1"]]))
            assert np.array_equal(keys["u32"], keys["wide"]), f"step {k}: formats differ"
            assert np.array_equal(keys["u32"], keys["dw"]), f"step {k}: fused format differs"
            assert np.array_equal(keys["u32"], shards), f"step {k}: shards differ"
            total += len(keys["u32"])
        assert total > n // 2
        a = eng["u32"][1].read()[0]
        w = eng["wide"][1].read()[0]
        d = eng["dw"][1].read()[0]
        s0, s1 = eng["s0"][1].read()[0], eng["s1"][1].read()[0]
        for col in ("pred", "sched"):
            assert np.array_equal(a[col], w[col]), col
            assert np.array_equal(a[col], d[col]), col
            assert np.array_equal(a[col], np.concatenate([s0[col], s1[col]])), col
        pend = (a["sched"] & 0xFF) != 0xFF
        assert np.array_equal(a["due"][pend], w["due"][pend])
        assert np.array_equal(a["due"][pend], d["due"][pend])
        st = eng["u32"][1].stats()
        fired = {name: c for name, c in st["fired_per_stage"].items() if c}
        assert {"pod-create", "pod-ready", "pod-complete", "pod-delete"} <= set(fired), fired
        assert any("failed" in name for name in fired), fired  # the chaos stages (weighted picks)
    finally:
        for _, e in eng.values():
            e.close()


def test_step_n_equals_per_step_calls():
    """kwk_step_n (the bench's per-interval call) enqueues exactly the per-tick kwk_step +
    kwk_fired_compact sequence: same states, statistics and last fired list, with and without
    the event samples."""
    from kwok_amd.host import abi
    unfused = {abi.TUNE_FUSE_STEPS: 0}  # one step per launch (the fused pairs: the test below)
    engines = {name: _pods("auto", n_nodes=20_000, tuning=None if name == "calls" else unfused)[1]
               for name in ("calls", "n", "n_ev")}
    try:
        now0, dt, seed = 1_700_000_000 * 10**9, 10**9, 0x6B776F6B
        for k in range(7):
            engines["calls"].step(now0 + k * dt, seed, k)
            engines["calls"].fired_compact()
        engines["n"].step_n(3, now0, dt, seed, 0)
        engines["n"].step_n(4, now0 + 3 * dt, dt, seed, 3)
        engines["n_ev"].step_n(7, now0, dt, seed, 0, True, 2, 0)
        ref = engines["calls"]
        r_hot, r_del = ref.read()
        r_fired = _fired_key(ref.fired())
        assert len(r_fired) > 0
        for name in ("n", "n_ev"):
            e = engines[name]
            hot, dels = e.read()
            for col in ("pred", "sched"):
                assert np.array_equal(hot[col], r_hot[col]), (name, col)
            assert np.array_equal(_fired_key(e.fired()), r_fired), name
            for key in ("fired", "matched", "bytes", "line_bytes", "steps"):
                assert e.stats()[key] == ref.stats()[key], (name, key)
        assert engines["n_ev"].event_elapsed_ms(4, 5) > 0.0  # sample 2 = step 4
    finally:
        for e in engines.values():
            e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n_nodes", [20_000, 250_000])
def test_fused_step_pairs_equal_per_step_calls(n_nodes):
    """KWK_TUNE_FUSE_STEPS (default 4): kwk_step_n sweeps the 1-byte ids up to four steps per launch
    (sweep8_kernel<..., kSteps>: each id read once, stepped in LDS, written once; each step's
    records to its own segments, each hand-back in turn).  States, the last fired list, the fired /
    matched / per-stage counts and the step count must equal the per-step kwk_step +
    kwk_fired_compact calls — one-tile grid (2M pods) and persistent grid (25M pods); groups of
    four, pairs (event samples every 2nd step cap a launch at two steps) and single steps; the
    fused launches read and write the ids once."""
    from kwok_amd.host import abi
    engines = {"calls": _pods("auto", n_nodes=n_nodes, tuning={abi.TUNE_FUSE_STEPS: 0})[1]}
    engines["fused"] = _pods("auto", n_nodes=n_nodes)[1]
    engines["fused_ev"] = _pods("auto", n_nodes=n_nodes)[1]
    try:
        now0, dt, seed = 1_700_000_000 * 10**9, 10**9, 0x6B776F6B
        ref = engines["calls"]
        for k in range(7):
            ref.step(now0 + k * dt, seed, k)
            ref.fired_compact()
        assert ref.last_sweep()["kernel"] == abi.SWEEP_8
        f = engines["fused"]
        f.step_n(3, now0, dt, seed, 0)
        f.step_n(4, now0 + 3 * dt, dt, seed, 3)
        assert f.last_sweep()["steps"] == 4  # the second call's four steps: one launch
        engines["fused_ev"].step_n(7, now0, dt, seed, 0, True, 2, 0)
        assert engines["fused_ev"].last_sweep()["steps"] == 1  # samples every 2nd step: 3 pairs, then step 6
        r_hot, _ = ref.read()
        r_fired = _fired_key(ref.fired())
        r_st = ref.stats()
        assert len(r_fired) > 0
        for name in ("fused", "fused_ev"):
            e = engines[name]
            hot, _ = e.read()
            for col in ("pred", "sched"):
                assert np.array_equal(hot[col], r_hot[col]), (name, col)
            assert np.array_equal(_fired_key(e.fired()), r_fired), name
            st = e.stats()
            for key in ("fired", "matched", "steps", "fired_per_stage"):
                assert st[key] == r_st[key], (name, key)
            assert st["bytes"] < r_st["bytes"]  # the pairs read and write each id once
        assert engines["fused_ev"].event_elapsed_ms(4, 5) > 0.0  # sample 2 = the launch of steps 4-5
    finally:
        for e in engines.values():
            e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("compact_small", [-1, 0])
def test_fused_step_n_pair_equals_per_step_calls(compact_small):
    """The bench's call, kwk_step_n_pair with 2-byte hand-backs: the pod engine's steps fused in
    groups of four and two, each group's hand-backs in one launch (one-launch prefix, or with
    KWK_TUNE_COMPACT_SMALL 0 the scan + expansion pair, blockIdx.y = the step), the node engine
    stepped one by one behind each group.  Both engines' states, last fired lists (2-byte pod
    records with their segment counts, 4-byte node records) and counts equal the per-step calls."""
    import bench
    from kwok_amd.host import abi
    now0, dt, seed = 1_700_000_000 * 10**9, 10**9, 0x6B776F6B
    runs = {}
    for mode in ("calls", "pair"):
        pods, nodes, _ = bench.build_engines(0, 20_000, PPN, 0, seed, 0.1)
        try:
            assert pods.stats()["state_bytes"] == 1
            if compact_small >= 0:
                pods.set_tuning(abi.TUNE_COMPACT_SMALL, compact_small)
            if mode == "calls":
                pods.set_tuning(abi.TUNE_FUSE_STEPS, 0)
                for k in range(10):
                    pods.step(now0 + k * dt, seed, k)
                    pods.fired_compact("16")
                    nodes.step(now0 + k * dt, seed, k)
                    nodes.fired_compact(True)
            else:
                pods.step_n_pair(nodes, 4, now0, dt, seed, 0, "packed16")
                pods.step_n_pair(nodes, 6, now0 + 4 * dt, dt, seed, 4, "packed16")
                assert pods.last_sweep()["steps"] == 2  # groups 4 | 4, 2
            recs, segc, _ = pods.fired_packed16()
            runs[mode] = (pods.read()[0], nodes.read()[0], recs, segc, nodes.fired_packed(), pods.stats(), nodes.stats())
        finally:
            pods.close()
            nodes.close()
    a, b = runs["calls"], runs["pair"]
    for i in (0, 1):
        for col in ("pred", "sched"):
            assert np.array_equal(a[i][col], b[i][col]), (i, col)
    assert np.array_equal(a[2], b[2]) and np.array_equal(a[3], b[3]) and len(a[2]) > 0
    assert np.array_equal(np.sort(a[4]), np.sort(b[4]))
    for i in (5, 6):
        for key in ("fired", "matched", "steps", "fired_per_stage"):
            assert a[i][key] == b[i][key], (i, key)


def test_fetch_async_equals_sync_readback():
    """kwk_fired_fetch_async (the overlapped host hand-back): each step's list copied on the copy
    stream while the next step is enqueued and compacted (the compaction waits for the copy on the
    device), buffers alternating, equals the synchronous kwk_fired_packed16 / kwk_fired_packed /
    kwk_fired of a twin engine stepped alike — the bitmap hand-back (maps + stage codes), 2-byte
    records with their per-segment counts, 4-byte packed and 8-byte records."""
    from kwok_amd.host import abi
    from kwok_amd.host.engine import PinnedBuffer
    now0, dt, seed = 1_700_000_000 * 10**9, 10**9, 0x6B776F6B
    for mode in ("bits", "16", True, False):
        (_, a), (_, b) = _pods("auto", n_nodes=20_000), _pods("auto", n_nodes=20_000)
        bufs = [(PinnedBuffer(8 * a.capacity), PinnedBuffer(4 * (a.capacity // 512 + 64))) for _ in range(2)]
        try:
            for k in range(6):
                for e in (a, b):
                    e.step(now0 + k * dt, seed, k)
                    e.fired_compact(mode)
                out, cnt = bufs[k % 2]
                info = b.fetch_async(out, cnt)
                if mode == "bits":
                    words, n_tr, ns, rs = a.fired_bits()
                    b.fetch_wait()
                    assert info["format"] == abi.COMPACT_BITS and info["record_bytes"] == 0
                    assert info["n_records"] == n_tr and info["n_segs"] == ns and info["bytes"] == 4 * len(words)
                    assert np.array_equal(out.array(np.uint32, len(words)), words), k
                elif mode == "16":
                    recs, segc, rs = a.fired_packed16()
                    b.fetch_wait()
                    assert info["record_bytes"] == 2 and info["n_segs"] == len(segc) and info["region_slots"] == rs
                    got = out.array(np.uint16, info["n_records"])
                    assert np.array_equal(got, recs), k
                    assert np.array_equal(cnt.array(np.uint32, info["n_segs"]), segc), k
                elif mode:
                    ref = a.fired_packed()
                    b.fetch_wait()
                    assert info["record_bytes"] == 4 and np.array_equal(out.array(np.uint32, info["n_records"]), ref), k
                else:
                    ref = a.fired()
                    b.fetch_wait()
                    got = out.array(abi.FIRED_DTYPE, info["n_records"])
                    assert info["record_bytes"] == 8 and np.array_equal(got, ref), k
                assert info["n_records"] > 0
            # an un-waited fetch, then a step: the engine's own compaction orders after the copy
            info = b.fetch_async(bufs[0][0], bufs[0][1])
            for e in (a, b):
                e.step(now0 + 6 * dt, seed, 6)
                e.fired_compact(mode)
            assert np.array_equal(_fired_key(a.fired()), _fired_key(b.fired()))
        finally:
            for e in (a, b):
                e.close()
            for x in bufs:
                for p in x:
                    p.close()


@pytest.mark.parametrize("n_nodes,mode", [(250_000, "16"), (250_000, "bits"), (20_000, "16")])
def test_fused_call_every_step_list_equals_per_step_calls(n_nodes, mode):
    """Every step's hand-back of a fused kwk_step_n call: 10 steps in one call
    sweep as launches of 4 + 4 + 2 steps, each launch's hand-backs in one launch, and every step's
    list lands in a ring slot of its own (kwk_fired_keep).  kwk_fired_fetch_step(k) for each of the
    10 steps — all fetched before one wait, the copies overlapping the later steps — must equal the
    list of the same step from per-step kwk_step + compaction calls of an unfused twin: the 2-byte
    records with their per-segment counts (25M pods: persistent grid, scan + expansion pair; 2M:
    one-tile grid, one-launch prefix) and the bitmap hand-back (25M).  The lists' transitions add up
    to the fired count (n_host == fired), a step the ring no longer holds is refused, and the
    call's last list is still the engine's (kwk_fired_packed16)."""
    from kwok_amd.host import abi
    from kwok_amd.host.engine import PinnedBuffer
    now0, dt, seed = 1_700_000_000 * 10**9, 10**9, 0x6B776F6B
    compact = "packed16" if mode == "16" else "bits"
    (_, ref), (_, f) = _pods("auto", n_nodes=n_nodes, tuning={abi.TUNE_FUSE_STEPS: 0}), _pods("auto", n_nodes=n_nodes)
    cap = f.capacity
    bufs = [(PinnedBuffer(2 * cap + 64), PinnedBuffer(4 * (cap // 2048 + 64))) for _ in range(10)]
    try:
        exp = []
        for k in range(10):
            ref.step(now0 + k * dt, seed, k)
            ref.fired_compact(mode)
            exp.append(ref.fired_packed16()[:2] if mode == "16" else ref.fired_bits())
        f.fired_keep(16)
        fired0 = f.stats()["fired"]
        f.step_n(10, now0, dt, seed, 0, compact)
        assert f.last_sweep()["steps"] == 2  # groups 4 | 4 | 2
        infos = [f.fetch_step(k, *bufs[k]) for k in range(10)]
        f.fetch_wait()
        n_host = 0
        for k, info in enumerate(infos):
            out, cnt = bufs[k]
            assert info["step"] == k
            if mode == "16":
                recs, segc = exp[k]
                assert info["format"] == abi.COMPACT_PACKED16 and info["n_records"] == len(recs), k
                assert np.array_equal(out.array(np.uint16, info["n_records"]), recs), k
                assert np.array_equal(cnt.array(np.uint32, info["n_segs"]), segc), k
            else:
                words, n_tr, ns, _ = exp[k]
                assert info["format"] == abi.COMPACT_BITS and info["n_records"] == n_tr and info["n_segs"] == ns, k
                assert np.array_equal(out.array(np.uint32, info["bytes"] // 4), words), k
            n_host += info["n_records"]
        assert n_host == f.stats()["fired"] - fired0 and n_host > 0
        assert f.stats()["fired"] == ref.stats()["fired"]
        if mode == "16":
            assert np.array_equal(f.fired_packed16()[0], exp[9][0])
        # a 4-deep ring holds the last 4 compactions only
        f.fired_keep(4)
        f.step_n(10, now0 + 10 * dt, dt, seed, 10, compact)
        for k in (16, 17, 18, 19):
            f.fetch_step(k, *bufs[k - 16])
        f.fetch_wait()
        with pytest.raises(abi.EngineError, match="no kept list of step 15"):
            f.fetch_step(15, *bufs[4])
    finally:
        for e in (ref, f):
            e.close()
        for x in bufs:
            for p in x:
                p.close()


@pytest.mark.parametrize("n_nodes", [125_000, 1_500])
def test_tail_handback_equals_compaction_launch(n_nodes):
    """KWK_TUNE_TAIL_HANDBACK (round 6): a 2-byte table-only node engine swept one tile per
    workgroup (the N = 8 shard's node engine at 125k nodes: 62 workgroups; 1.5k nodes: one) writes
    each step's list inside the sweep — every workgroup adds the counts of the workgroups before
    it, then copies its records.  Against a twin with the compaction launch: every step's list of
    a 10-step kwk_step_n (4-byte packed, then 8-byte records, fetched from the ring by step) is
    identical in content and order, the states and counts equal, and kwk_tick's node lists too."""
    import bench
    from kwok_amd.host import abi
    from kwok_amd.host.engine import PinnedBuffer
    now0, dt, seed = 1_700_000_000 * 10**9, 5 * 10**9, 0x6B776F6B  # 5 s steps: heartbeats fire in both calls
    engs = {}
    for tail in (1, 0):
        pods, nodes, _ = bench.build_engines(0, n_nodes, 1, 0, seed, 0.1)
        pods.close()
        nodes.set_tuning(abi.TUNE_TAIL_HANDBACK, tail)
        engs[tail] = nodes
    cap = engs[1].capacity
    bufs = [PinnedBuffer(8 * cap + 64) for _ in range(10)]
    try:
        assert engs[1].stats()["state_bytes"] == 2
        for e in engs.values():
            e.fired_keep(16)
        t = 0
        for compact, rec in (("packed", np.uint32), (True, abi.FIRED_DTYPE)):
            lists = {}
            for tail, e in engs.items():
                e.step_n(10, now0 + t * dt, dt, seed, t, compact)
                assert e.last_sweep()["kernel"] == abi.SWEEP_16_FSM and not e.last_sweep()["persistent"]
                infos = [e.fetch_step(t + k, bufs[k]) for k in range(10)]
                e.fetch_wait()
                lists[tail] = [bufs[k].array(rec, infos[k]["n_records"]).copy() for k in range(10)]
            total = 0
            for k in range(10):
                assert np.array_equal(lists[1][k], lists[0][k]), (compact, k)
                total += len(lists[1][k])
            assert total > 0, "no node transition in 10 steps"
            t += 10
        a, b = engs[1], engs[0]
        for col in ("pred", "sched"):
            assert np.array_equal(a.read()[0][col], b.read()[0][col]), col
        for key in ("fired", "matched", "fired_per_stage"):
            assert a.stats()[key] == b.stats()[key], key
        # kwk_tick (nodes alone): lease step + node sweep + hand-back
        for tail, e in engs.items():
            e.tick(None, now0 + t * dt, seed, t, "packed")
        assert np.array_equal(a.fired_packed(), b.fired_packed())
    finally:
        for e in engs.values():
            e.close()
        for x in bufs:
            x.close()


def test_fused_records_load_read_step_at_4m_pods():
    """The fused records' due times at scale: 4M C2 pods loaded with a queued stage on every third
    pod, its due time inside the 68.7 s window of the first step's epoch, years before it, or
    hours after it (the due column), read back exactly (fold on load, decode on read), then
    stepped with 20 s between steps (the epoch moves every step: re-encoded, far times to and
    from the column) — the fused engine leaves every row and fires every transition exactly as
    the 4-byte-word engine with its separate due column does."""
    from kwok_amd import workload as W
    from kwok_amd.host import abi
    from kwok_amd.host.engine import Engine, Ingest
    n = 4_000_000
    prog = _c2_program(n)
    pvars, pidx = W.c2_pod_variants(0, n, seed=0x6B776F6B, job_frac=0.1)
    ing = Ingest(prog)
    hot, dels, rec, cls = ing.variant_columns(pvars, pidx)
    rng = np.random.default_rng(77)
    now0 = 1_700_000_000 * 10**9
    sel = np.arange(0, n, 3)
    n_stages = len(prog.names)
    hot["sched"][sel] = (hot["sched"][sel] & ~np.uint32(0xFF)) | rng.integers(0, n_stages, len(sel)).astype(np.uint32)
    kind = rng.integers(0, 3, len(sel))
    hot["due"][sel] = np.where(kind == 0, now0 + rng.integers(0, 60 * 10**9, len(sel)),
                               np.where(kind == 1, now0 - 3 * 10**17, now0 + rng.integers(10**12, 10**13, len(sel))))
    engs = {}
    try:
        for st in ("u32", "auto"):
            eng = Engine(prog, capacity=n, state=st, max_records=max(1, len(ing.records)) + 16)
            eng.load_stages()
            eng.set_harness(True)
            eng.load(hot, dels, rec, cls, ing.record_array())
            engs[st] = eng
        assert engs["auto"].stats()["state_bytes"] == 8 and engs["u32"].stats()["state_bytes"] == 4

        def rows_equal(tag):
            a, _ = engs["u32"].read()
            b, _ = engs["auto"].read()
            assert np.array_equal(a["pred"], b["pred"]) and np.array_equal(a["sched"], b["sched"]), tag
            pend = (a["sched"] & 0xFF) != 0xFF
            assert np.array_equal(a["due"][pend], b["due"][pend]), tag
            return a, pend
        a, pend = rows_equal("load")
        assert np.array_equal(a["due"][sel], hot["due"][sel])  # read back exactly as loaded
        for k in range(4):
            now = now0 + k * 20 * 10**9
            keys = []
            for st in ("u32", "auto"):
                engs[st].step(now, 0x6B776F6B, k)
                f = engs[st].fired()
                keys.append(np.sort(f["slot"].astype(np.uint64) << 32 | f["stage"].astype(np.uint64) << 16
                                    | f["flags"].astype(np.uint64)))
            assert engs["auto"].last_sweep()["kernel"] == abi.SWEEP_WD
            assert np.array_equal(keys[0], keys[1]), f"step {k}: fired sets differ"
            rows_equal(f"step {k}")
    finally:
        for e in engs.values():
            e.close()
