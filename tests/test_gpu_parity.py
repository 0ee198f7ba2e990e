"""GPU parity: the HIP sweep kernel (through the C ABI) against the oracle simulation.

Matched-stage choice, stage indices, due times (delay + Philox jitter), fired sets, the
next-state feature bits, deletion timestamps and the dirty/re-match flag must be bit-exact
at every step (BASELINE.json north_star)."""
import numpy as np
import pytest

from kwok_amd import workload as W
from kwok_amd.host import abi
from tests.parity_util import run

pytestmark = pytest.mark.gpu


FORMATS = ["auto", "u16", "u32", "dw", "wide"]


@pytest.mark.parametrize("state", FORMATS + ["auto-nofsm", "auto-gen", "auto-pair", "u16-pair"])
def test_pod_fast_c1_mini(state):
    """C1 shape (pod-fast, 10% Job-owned, harness churn) at 40 nodes x 10 pods, in every
    device state format: auto = the 1-byte dictionary ids of sweep8_kernel (pod-fast is
    table-only), u16 = the 2-byte words (the table-only sweep16_fsm_kernel), the general
    sweep16_kernel with its transition table (auto-gen: leaves the 1-byte format) and without it
    (auto-nofsm); dw = the 8-byte records of a packed word fused with its relative due time;
    auto-pair hands the fired list back through the scan + expansion pair (KWK_TUNE_COMPACT_SMALL
    0), u16-pair the 2-byte words through the same pair, instead of the one-launch compaction."""
    tuning, kernel = {}, {"auto": abi.SWEEP_8, "u16": abi.SWEEP_16_FSM, "u32": abi.SWEEP_W4, "dw": abi.SWEEP_WD,
                          "wide": abi.SWEEP_W8}.get(state)
    if state == "auto-nofsm":
        tuning, kernel, state = {abi.TUNE_SWEEP16: abi.sweep16_shape(table=0)}, abi.SWEEP_16, "auto"
    elif state == "auto-gen":
        tuning, kernel, state = {abi.TUNE_SWEEP16: abi.sweep16_shape(kernel=0)}, abi.SWEEP_16, "auto"
    elif state == "auto-pair":
        tuning, kernel, state = {abi.TUNE_COMPACT_SMALL: 0}, abi.SWEEP_8, "auto"
    elif state == "u16-pair":
        tuning, kernel, state = {abi.TUNE_COMPACT_SMALL: 0}, abi.SWEEP_16_FSM, "u16"
    cl = W.make_cluster("C1", 40, 400, seed=11)
    objs = cl.pods.materialize()
    total, per = run(cl.pod_stage_files, objs, steps=12, dt_ns=10**9, harness=True, state=state, tuning=tuning,
                     expect_kernel=kernel)
    assert per["pod-ready"] >= 400 and per["pod-complete"] > 0 and per["pod-delete"] > 0


@pytest.mark.parametrize("state", ["auto", "u32", "wide"])
def test_pod_general_c2_mini(state):
    """C2 shape: pod-general + chaos, init containers, override annotations (valid and
    invalid ints / durations / RFC3339), chaos labels, deletionTimestamps; weighted picks
    and Philox jitter.  auto = the fused 8-byte records (28-bit words), u32 = 4-byte words and
    the separate due column, wide = 8-byte {pred, sched}."""
    cl = W.make_cluster("C2", 50, 600, seed=12)
    objs = cl.pods.materialize()
    kernel = {"auto": abi.SWEEP_WD, "u32": abi.SWEEP_W4, "wide": abi.SWEEP_W8}[state]
    total, per = run(cl.pod_stage_files, objs, steps=40, dt_ns=500 * 10**6, harness=True, state=state,
                     expect_kernel=kernel)
    assert per["pod-create"] > 0 and per["pod-ready"] > 0 and per["pod-delete"] > 0
    assert per["pod-container-running-failed"] + per["pod-init-container-running-failed"] > 0


@pytest.mark.parametrize("state", ["auto", "u32", "wide"])
def test_word_sweep_tile_loop(state):
    """The word sweep's workgroups looping over several tiles (KWK_TUNE_WORD_TILES 2: every
    second tile's stream in flight while the first is worked, the LDS dirty-line mask deciding
    the line stores) on a C2 cluster of several tiles, against the oracle at every step."""
    cl = W.make_cluster("C2", 120, 12000, seed=23)
    objs = cl.pods.materialize()
    kernel = {"auto": abi.SWEEP_WD, "u32": abi.SWEEP_W4, "wide": abi.SWEEP_W8}[state]
    run(cl.pod_stage_files, objs, steps=8, dt_ns=700 * 10**6, harness=True, state=state,
        tuning={abi.TUNE_WORD_TILES: 2}, expect_kernel=kernel)


@pytest.mark.parametrize("clock", ["jumps", "backwards", "from-zero"])
def test_fused_due_epoch(clock):
    """The fused records' due times against the oracle where the epoch moves: steps of 9-40 s
    (re-encoded every ~17 s, due times past the 68.7 s window in the side column: the C2
    deletion jitter reaches 30 s, RFC3339 overrides lie years back), a clock that runs backwards
    (the epoch follows it down), and a clock starting at 0 (objects loaded with due times
    relative to epoch 0)."""
    from tests.parity_util import NOW0
    cl = W.make_cluster("C2", 30, 400, seed=21)
    objs = cl.pods.materialize()
    if clock == "jumps":
        nows = [NOW0 + sum((9 + 31 * (k % 2)) * 10**9 for k in range(j)) for j in range(24)]
    elif clock == "backwards":
        nows = [NOW0 + (k if k < 10 else 20 - k) * 3 * 10**9 + (k % 3) * 10**8 for k in range(20)]
    else:
        nows = [k * 700 * 10**6 for k in range(30)]
    run(cl.pod_stage_files, objs, steps=len(nows), dt_ns=0, harness=True, state="auto", expect_kernel=abi.SWEEP_WD,
        nows=nows)


@pytest.mark.parametrize("state", ["auto", "u16", "auto-nofsm", "u32", "dw"])
def test_node_fast_heartbeat(state):
    tuning = {}
    if state == "auto-nofsm":
        tuning = {abi.TUNE_SWEEP16: abi.sweep16_shape(table=0)}
        state = "auto"
    cl = W.make_cluster("C1", 64, 64, seed=13)
    objs = cl.nodes.materialize()
    total, per = run(cl.node_stage_files, objs, steps=30, dt_ns=2 * 10**9, kind_salt=1, state=state, tuning=tuning)
    assert per["node-initialize"] == 64 and per["node-heartbeat"] > 0


@pytest.mark.parametrize("case", ["pod-fast", "pod-general", "node-heartbeat", "node-chaos"])
def test_native_compiler_tables_parity(case):
    """The engine loaded from the NATIVE Stage compiler (kwk_compile_stages / kwk_program_explore /
    kwk_program_table / _deltas / _harness) with rows from libkwok_encoder built from its spec —
    the Go host's path, no Python compiler — bit-exact against the oracle at every step: pod-fast
    (1-byte ids), pod-general + chaos (fused records, value records), node-fast + node-heartbeat
    ("patch already applied" bits evaluated by the native encoder) and node-chaos (weights)."""
    if case == "pod-fast":
        cl = W.make_cluster("C1", 30, 300, seed=71)
        run(cl.pod_stage_files, cl.pods.materialize(), steps=10, dt_ns=10**9, harness=True, compiler="native",
            expect_kernel=abi.SWEEP_8)
    elif case == "pod-general":
        cl = W.make_cluster("C2", 40, 500, seed=72)
        run(cl.pod_stage_files, cl.pods.materialize(), steps=36, dt_ns=500 * 10**6, harness=True, compiler="native",
            expect_kernel=abi.SWEEP_WD)
    elif case == "node-heartbeat":
        cl = W.make_cluster("C1", 64, 64, seed=73)
        _, per = run(cl.node_stage_files, cl.nodes.materialize(), steps=30, dt_ns=2 * 10**9, kind_salt=1,
                     compiler="native")
        assert per["node-initialize"] == 64 and per["node-heartbeat"] > 0
    else:
        objs = [W.node_object(f"node-{i}", labels={"node-not-ready.stage.kwok.x-k8s.io": "true"} if i % 3 == 0 else None,
                              annotations={"node-not-ready.stage.kwok.x-k8s.io/weight": str(i % 5)} if i % 2 else None)
                for i in range(90)]
        run(W.stage_paths(W.NODE_FAST + W.NODE_HEARTBEAT + W.NODE_CHAOS), objs, steps=25, dt_ns=3 * 10**9, kind_salt=1,
            compiler="native")


def test_node_chaos_weights():
    """node-not-ready (weight 10000) beside node-heartbeat (weight 0): weighted pick path."""
    objs = [W.node_object(f"node-{i}", labels={"node-not-ready.stage.kwok.x-k8s.io": "true"} if i % 3 == 0 else None,
                          annotations={"node-not-ready.stage.kwok.x-k8s.io/weight": str(i % 5)} if i % 2 else None)
            for i in range(90)]
    files = W.stage_paths(W.NODE_FAST + W.NODE_HEARTBEAT + W.NODE_CHAOS)
    run(files, objs, steps=25, dt_ns=3 * 10**9, kind_salt=1)


def test_empty_and_single():
    files = W.stage_paths(W.POD_FAST)
    run(files, [W.pod_object("p0", "node-0")], steps=3, dt_ns=10**9)


def test_weight_edge_cases():
    """All-error weights (Intn over all), zero total with errors (subset pick), negative
    total (Go panics: no schedule, KWK_F_MATCHERR)."""
    base = W.pod_object("p", "node-0")
    stages_yaml = []
    objs = []
    for i, (w1, w2) in enumerate([("abc", "xyz"), ("0", "bad"), ("-5", "2"), ("3", "4"), ("0", "0"), ("", "7")]):
        o = W.pod_object(f"p{i}", "node-0", annotations={"a.w": w1, "b.w": w2})
        objs.append(o)
    import os
    import tempfile
    import yaml
    d = tempfile.mkdtemp()
    paths = []
    for name, key in (("a", "a.w"), ("b", "b.w")):
        st = {"apiVersion": "kwok.x-k8s.io/v1alpha1", "kind": "Stage", "metadata": {"name": name},
              "spec": {"resourceRef": {"apiGroup": "v1", "kind": "Pod"},
                       "selector": {"matchExpressions": [{"key": ".metadata.deletionTimestamp",
                                                          "operator": "DoesNotExist"}]},
                       "weight": 1, "weightFrom": {"expressionFrom": f'.metadata.annotations["{key}"]'},
                       "delay": {"durationMilliseconds": 1000, "jitterDurationMilliseconds": 9000},
                       "next": {"statusTemplate": "phase: Running\n"}}}
        p = os.path.join(d, name + ".yaml")
        yaml.safe_dump(st, open(p, "w"))
        paths.append(p)
    run(paths, objs * 20, steps=6, dt_ns=2 * 10**9)


def test_shard_invariance_two_engines():
    """The cluster split into two engines (slot_base = global id of each shard's first pod)
    fires exactly what one engine over the whole cluster fires (RNG keyed by global slot),
    and both match the oracle."""
    from kwok_amd.host.cluster import node_block, pod_range
    from tests.parity_util import NOW0, build
    cl = W.make_cluster("C2", 12, 240, seed=14)
    objs = cl.pods.materialize()
    _, whole, sim = build(cl.pod_stage_files, objs, harness=True)
    shards = []
    for r in range(2):
        lo, hi = node_block(12, 2, r)
        plo, phi = pod_range(cl.node_ptr, lo, hi)
        _, eng, _ = build(cl.pod_stage_files, objs[plo:phi], harness=True, slot_base=plo)
        shards.append((plo, eng))
    try:
        for k in range(25):
            now = NOW0 + k * 700 * 10**6
            whole.step(now, 7, k)
            for _, e in shards:
                e.step(now, 7, k)
            exp = sorted((i, s, f) for i, s, f in sim.step(now, 7, k))
            w = sorted((int(r["slot"]), int(r["stage"]), int(r["flags"])) for r in whole.fired())
            sh = sorted((plo + int(r["slot"]), int(r["stage"]), int(r["flags"])) for plo, e in shards for r in e.fired())
            assert w == exp and sh == exp, f"step {k}"
    finally:
        whole.close()
        for _, e in shards:
            e.close()


@pytest.mark.parametrize("state", ["auto", "u16", "u32", "dw", "wide"])
def test_count_phase_histogram(state):
    """kwk_count and kwk_aggregate (cluster aggregates for the RCCL all-reduce) against the
    oracle's phases, in the 2-, 4- and 8-byte state formats; a ragged object count so the last
    16-byte chunk is partly past the end."""
    from kwok_amd.host.cluster import phase_masks
    from oracle import refcpu
    from tests.parity_util import NOW0, build
    cl = W.make_cluster("C1", 20, 403, seed=15)
    prog, eng, sim = build(cl.pod_stage_files, cl.pods.materialize(), harness=True, state=state)
    try:
        masks = phase_masks(prog, values=("Running", "Succeeded"))
        fired = np.zeros(len(prog.names), dtype=np.int64)
        for k in range(5):
            eng.step(NOW0 + k * 10**9, 3, k)
            for _, s, _ in sim.step(NOW0 + k * 10**9, 3, k):
                fired[s] += 1
            got = eng.count([masks["Running"], masks["Succeeded"], 0])
            alive = [o for o in sim.objs if o is not None]
            ph = [(refcpu.query(".status.phase", o) or [None])[0] for o in alive]
            want = [ph.count("Running"), ph.count("Succeeded"), len(alive)]
            assert got.tolist() == want
            n = eng.aggregate([masks["Running"], masks["Succeeded"], 0])
            agg = eng.aggregate_read(n)
            assert agg[:len(fired)].tolist() == fired.tolist() and agg[len(fired):].tolist() == want
    finally:
        eng.close()


def test_state_format_repack_on_table_reload():
    """kwk_load_stages with objects resident and a table that needs the other state format
    (pred_bits = 0 -> 32 bits -> wide, then back to 16 bits: the 1-byte dictionary ids) repacks them in place; the run
    stays bit-exact with the oracle."""
    import ctypes as C
    from kwok_amd.host import abi
    from tests.parity_util import NOW0, build, compare_state
    cl = W.make_cluster("C1", 10, 200, seed=16)
    prog, eng, sim = build(cl.pod_stage_files, cl.pods.materialize(), harness=True)
    try:
        for k in range(8):
            if k in (3, 6):
                t = prog.table(version=k)
                if k == 3:
                    t.pred_bits = 0
                deltas = np.ascontiguousarray(prog.delta_array())
                abi.check(abi.lib().kwk_load_stages(eng.h, C.byref(t), abi.ptr(deltas)), "kwk_load_stages", eng.h)
                assert eng.stats()["state_bytes"] == (8 if k == 3 else 1)  # back to 16 bits: the 1-byte ids
            now = NOW0 + k * 10**9
            eng.step(now, 9, k)
            got = sorted((int(r["slot"]), int(r["stage"]), int(r["flags"])) for r in eng.fired())
            assert got == sorted(sim.step(now, 9, k)), f"step {k}"
            compare_state(prog, eng, sim, k)
    finally:
        eng.close()


def test_device_list_empty_after_sweeping_nothing():
    """a step over no active slots must leave an EMPTY device-compacted list, not the
    previous step's count (an in-process consumer of kwk_fired_device would re-render patches
    for objects that fired a step earlier)."""
    import ctypes as C
    from kwok_amd.host import abi
    from tests.parity_util import build
    files = W.stage_paths(W.POD_FAST)
    prog, eng, _ = build(files, [W.pod_object(f"p{i}", "node-0") for i in range(300)], harness=False)
    try:
        L = abi.lib()

        hip = C.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]

        def device_count():
            recs, cnt = C.c_void_p(), C.c_void_p()
            abi.check(L.kwk_fired_device(eng.h, C.byref(recs), C.byref(cnt)), "kwk_fired_device", eng.h)
            eng.sync()
            out = C.c_uint32(0xFFFFFFFF)
            assert hip.hipMemcpy(C.byref(out), cnt, 4, 2) == 0  # hipMemcpyDeviceToHost
            return out.value
        eng.step(10**18, 1, 0)
        eng.fired_compact()
        assert device_count() == 300  # every pod matched pod-ready and fired
        eng.load(np.zeros(0, dtype=abi.HOT_DTYPE), [], [], [])
        eng.step(10**18 + 10**9, 1, 1)
        eng.fired_compact()
        assert device_count() == 0
        assert len(eng.fired()) == 0
    finally:
        eng.close()


def test_byte_format_dictionary_lifecycle():
    """The 1-byte dictionary format through the calls that bring new words: upserts
    of objects in other states join the dictionary (still 1 byte, bit-exact with the oracle); a
    harness change re-assigns the ids; an upsert whose words overflow an id class returns the
    engine to the 2-byte words in place; kwk_match leaves the 1-byte format.  Every step is checked
    against the oracle."""
    from kwok_amd.host import abi
    from tests.parity_util import NOW0, build, compare_state
    files = W.stage_paths(W.POD_FAST)
    objs = [W.pod_object(f"p{i}", "node-0", job=(i % 3 == 0)) for i in range(300)]
    prog, eng, sim = build(files, objs, harness=True)
    try:
        assert eng.stats()["state_bytes"] == 1
        seed = 0x51
        from kwok_amd.host.engine import Ingest

        def step(k):
            eng.step(NOW0 + k * 10**9, seed, k)
            got = sorted((int(r["slot"]), int(r["stage"]), int(r["flags"])) for r in eng.fired())
            assert got == sorted(sim.step(NOW0 + k * 10**9, seed, k)), k
            compare_state(prog, eng, sim, k)

        def upsert(slots, new_objs):
            import copy
            ing = Ingest(prog)
            hot, dels, rec, cls = ing.columns(new_objs)
            eng.upsert(np.array(slots), hot, dels, rec, cls)
            from oracle.next_ref import omitempty
            for s, o in zip(slots, new_objs):
                sim.objs[s] = omitempty(copy.deepcopy(o))
                sim.orig[s] = copy.deepcopy(sim.objs[s])
                sim.dirty[s] = True
                sim.pending[s] = None
        for k in range(3):
            step(k)
        # Running pods with a podIP and a finalizer: words outside the first closure
        run = []
        for i in range(10):
            o = W.pod_object(f"q{i}", "node-0")
            o["metadata"]["finalizers"] = ["kwok.x-k8s.io/fake"]
            o["status"] = {"phase": "Running", "podIP": "10.0.0.9"}
            run.append(o)
        upsert(list(range(10)), run)
        assert eng.stats()["state_bytes"] == 1
        for k in range(3, 6):
            step(k)
        eng.set_harness(False)  # the ids encode the harness's "needs work": re-assigned in place
        sim.harness = False
        assert eng.stats()["state_bytes"] == 1
        step(6)
        eng.set_harness(True)
        sim.harness = True
        step(7)
        # every combination of the program's feature bits at once: more words than an id class holds
        n_bits = prog.table().pred_bits
        many = []
        for i in range(2 ** min(n_bits, 7)):
            o = W.pod_object(f"m{i}", "node-0", job=bool(i & 1))
            if i & 2:
                o["metadata"]["deletionTimestamp"] = "2023-11-14T22:13:20Z"
            st = {}
            if i & 4:
                st["podIP"] = "10.0.0.7"
            st["phase"] = ["Pending", "Running", "Succeeded", "Failed"][(i >> 3) & 3]
            if st["phase"] == "Running":  # pod-complete's template indexes the container statuses
                st["containerStatuses"] = [{"name": "container-0", "image": "busybox", "ready": True, "restartCount": 0,
                                            "state": {"running": {"startedAt": "2023-11-14T22:13:20Z"}}}]
            o["status"] = st
            if i & 32:
                o["metadata"]["finalizers"] = ["kwok.x-k8s.io/fake"]
            many.append(o)
        hot, _, _, _ = Ingest(prog).columns(many)
        upsert(list(range(20, 20 + len(many))), many)
        if len(set(hot["pred"].tolist())) > 31:
            assert eng.stats()["state_bytes"] == 2, "an overflowing id class must return to the 2-byte words"
        for k in range(8, 11):
            step(k)
        eng.set_tuning(abi.TUNE_BYTE_STATE, 1)  # back to the ids if they fit (they may not)
        step(11)
        eng.match(NOW0 + 12 * 10**9, seed, 12)  # match-only: the general sweep on 2-byte words
        assert eng.stats()["state_bytes"] == 2
    finally:
        eng.close()
