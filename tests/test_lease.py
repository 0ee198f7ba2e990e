"""Node leases (NodeLeaseController, BASELINE C3): the oracle pinned by the reference's unit
vectors and its controller scenario test; the device lease step (kwk_lease_step) bit-exact
against the oracle, coupled to the node sweep (readOnlyFunc / ManageNode) and to the pods on
those nodes (podsOnNodeSyncWorker)."""
import json
import os

import numpy as np
import pytest

from kwok_amd import workload as W
from oracle import lease_ref as LR

VEC = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "lease_vectors.json")))
NOW = 1_700_000_000 * 10**9
IDS = {"test": 1, "test-new": 2, "lease1": 11, "lease2": 12, "lease3": 13}


def _lease(holder, duration_s, renew_rel_s, exists=True):
    f = LR.EXISTS if exists else 0
    L = LR.Lease(flags=f)
    if holder is not None:
        L.holder, L.flags = IDS[holder], L.flags | LR.HOLDER
    if duration_s is not None:
        L.duration_s, L.flags = duration_s, L.flags | LR.DURATION
    if renew_rel_s is not None:
        L.renew_ns, L.flags = NOW + renew_rel_s * 10**9, L.flags | LR.RENEW
    return L


@pytest.mark.parametrize("c", VEC["try_acquire_or_renew"], ids=lambda c: c["ref"])
def test_try_acquire_or_renew(c):
    L = _lease(c["holder"], c["duration_s"], c["renew_rel_s"])
    assert LR.try_acquire_or_renew(L, IDS[c["self"]], NOW) is c["want"]


@pytest.mark.parametrize("c", VEC["next_try_duration"], ids=lambda c: c["ref"])
def test_next_try_duration(c):
    ms = 10**6
    assert LR.next_try_duration(c["renew_interval_ms"] * ms, c["expire_ms"] * ms, c["hold"]) == c["want_ms"] * ms


@pytest.mark.parametrize("c", VEC["expire_time"], ids=lambda c: c["ref"])
def test_expire_time(c):
    L = _lease(c["holder"], c["duration_s"], c["renew_rel_s"])
    t, ok = LR.expire_time(L)
    assert ok is c["want_ok"]
    if ok:
        assert t == NOW + c["want_rel_s"] * 10**9


def test_jitter_hook_range():
    """wait.Jitter(10 s, 0.04) stays in [10 s, 10.4 s); maxFactor <= 0 means 1."""
    for slot in range(200):
        u = LR.float64_hook(7, slot, 3)
        assert 0.0 <= u < 1.0
        d = LR.jitter(10 * 10**9, 0.04, u)
        assert 10 * 10**9 <= d < 10.4 * 10**9
    assert LR.jitter(10, 0.0, 0.5) == 15


def _scenario_leases():
    sc = VEC["controller_scenario"]
    names = ["lease0", "lease1", "lease2", "lease3", "lease4"]
    leases = []
    for n in names:
        spec = sc["leases"].get(n)
        L = _lease(spec["holder"], spec["duration_s"], spec["renew_rel_s"]) if spec else LR.Lease()
        if n in sc["try_hold"]:  # TryHold: into holdLeaseSet, queued at once
            L.flags |= LR.HOLD | LR.QUEUED
            L.next_try_ns = NOW
        leases.append(L)
    return sc, names, leases


def test_controller_scenario_oracle():
    """TestNodeLeaseController (node_lease_controller_test.go:37-156) on the oracle."""
    sc, names, leases = _scenario_leases()
    sim = LR.LeaseSim(leases, IDS[sc["self"]], sc["lease_duration_s"], sc["renew_interval_s"] * 10**9, sc["jitter"])
    sim.step(NOW, 1, 0)
    for n, want in sc["after_1s_held"].items():
        assert LR.held(sim.leases[names.index(n)], IDS[sc["self"]]) is want, n
    # the apiserver deletes lease1: the informer cache no longer has it
    sim.leases[names.index(sc["delete"])].flags &= ~(LR.EXISTS | LR.HOLDER | LR.DURATION | LR.RENEW)
    sim.step(NOW + 2 * 10**9, 1, 1)
    for n, want in sc["after_delete_held"].items():
        assert LR.held(sim.leases[names.index(n)], IDS[sc["self"]]) is want, n


def to_array(leases):
    a = np.zeros(len(leases), dtype=[("renew_ns", "<i8"), ("next_try_ns", "<i8"), ("holder", "<u4"),
                                     ("duration_s", "<i4"), ("transitions", "<i4"), ("flags", "<u4")])
    for i, L in enumerate(leases):
        a[i] = (L.renew_ns, L.next_try_ns, L.holder, L.duration_s, L.transitions, L.flags)
    return a


def assert_leases_equal(got, sim_leases, step):
    want = to_array(sim_leases)
    for f in want.dtype.names:
        bad = np.nonzero(got[f] != want[f])[0]
        assert bad.size == 0, f"step {step}: lease field {f} differs at {bad[:8].tolist()}: " \
                              f"{got[f][bad[:4]].tolist()} vs {want[f][bad[:4]].tolist()}"


def c3_leases(n, now, rng):
    """C3 lease mix: 50% absent (created), 20% our own stale lease, 20% foreign and expiring
    during the run, 5% foreign and fresh, 5% not in the hold set."""
    leases = []
    for i in range(n):
        r = rng.random()
        if r < 0.5:
            L = LR.Lease()
        elif r < 0.7:
            L = LR.Lease(flags=LR.EXISTS | LR.HOLDER | LR.DURATION | LR.RENEW, holder=1, duration_s=40,
                         renew_ns=now - int(rng.integers(0, 60)) * 10**9, transitions=int(rng.integers(0, 3)))
        elif r < 0.95:
            L = LR.Lease(flags=LR.EXISTS | LR.HOLDER | LR.DURATION | LR.RENEW, holder=7, duration_s=40,
                         renew_ns=now - (40 - int(rng.integers(0, 30))) * 10**9 if r < 0.9 else now)
        else:
            L = LR.Lease(flags=LR.EXISTS | LR.HOLDER | LR.DURATION | LR.RENEW, holder=7, duration_s=40,
                         renew_ns=now - 100 * 10**9)
        if r < 0.95 or i % 2:
            L.flags |= LR.HOLD | LR.QUEUED
            L.next_try_ns = now
        leases.append(L)
    return leases


@pytest.mark.gpu
def test_controller_scenario_gpu():
    from kwok_amd.host.compiler import KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files
    sc, names, leases = _scenario_leases()
    objs = [W.node_object(n) for n in names]
    prog = KindProgram(load_stage_files(*W.stage_paths(W.NODE_FAST + W.NODE_HEARTBEAT)))
    prog.explore(objs)
    ing = Ingest(prog)
    eng = Engine(prog, capacity=len(objs), kind_salt=1)
    try:
        eng.load_stages()
        eng.load(*ing.columns(objs), ing.record_array())
        eng.lease_config(IDS[sc["self"]], sc["lease_duration_s"], sc["renew_interval_s"] * 10**9, sc["jitter"])
        eng.lease_set(to_array(leases))
        sim = LR.LeaseSim(leases, IDS[sc["self"]], sc["lease_duration_s"], sc["renew_interval_s"] * 10**9, sc["jitter"])
        eng.lease_step(NOW, 1, 0)
        want_ops = sorted(sim.step(NOW, 1, 0))
        assert sorted((int(r["slot"]), int(r["stage"])) for r in eng.lease_ops()) == want_ops
        got = eng.lease_read()
        assert_leases_equal(got, sim.leases, 0)
        me = IDS[sc["self"]]
        for n, want in sc["after_1s_held"].items():
            i = names.index(n)
            assert bool(got["flags"][i] & LR.EXISTS and got["flags"][i] & LR.HOLDER and got["holder"][i] == me) is want
        assert eng.lease_stats()["creates"] == 1 and eng.lease_stats()["acquires"] == 1
    finally:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("state,fused", [("auto", False), ("u32", False), ("wide", False), ("auto", True),
                                         ("u32", True), ("dw", False), ("dw", True)])
def test_c3_nodes_leases_pods_parity(state, fused):
    """C3 shape at 96 nodes (node-initialize + node-heartbeat 20 s / 25 s, leases 40 s with a
    10 s +- 4% renew, 250 ms tick for 50 s) with 4 pod-fast pods per node: lease step ->
    node MANAGED / resync -> node sweep -> pod resync -> pod sweep, every step bit-exact
    (lease records, lease API writes, fired sets, object states) against the oracle — as
    separate calls, and (fused) as one kwk_tick per step (HIP-event stream order)."""
    from tests.parity_util import NOW0, build, compare_state
    rng = np.random.default_rng(33)
    n_nodes, ppn = 96, 4
    nodes = [W.node_object(f"node-{i}") for i in range(n_nodes)]
    pods = [W.pod_object(f"pod-{i}", f"node-{i // ppn}", job=(i % 10 == 0)) for i in range(n_nodes * ppn)]
    node_ptr = np.arange(0, n_nodes * ppn + 1, ppn, dtype=np.uint32)
    leases = c3_leases(n_nodes, NOW0, rng)
    me = 1
    nprog, neng, nsim = build(W.stage_paths(W.NODE_FAST + W.NODE_HEARTBEAT), nodes, kind_salt=1, state=state)
    pprog, peng, psim = build(W.stage_paths(W.POD_FAST), pods, harness=True, state=state)
    try:
        # initial readOnly: only nodes whose cached lease is ours are managed (and their pods)
        init_held = [LR.held(L, me) for L in leases]
        hot, dels = neng.read()
        from kwok_amd.host import abi
        for i in range(n_nodes):
            if not init_held[i]:
                hot["sched"][i] &= ~np.uint32(abi.F_MANAGED)
                nsim.managed[i] = False
        neng.upsert(np.arange(n_nodes), hot, dels, np.zeros(n_nodes, np.uint32),
                    (hot["sched"] >> 16).astype(np.uint16))
        phot, pdels = peng.read()
        for i in range(len(pods)):
            if not init_held[i // ppn]:
                phot["sched"][i] &= ~np.uint32(abi.F_MANAGED)
                psim.managed[i] = False
        peng.upsert(np.arange(len(pods)), phot, pdels, np.zeros(len(pods), np.uint32),
                    (phot["sched"] >> 16).astype(np.uint16))
        neng.lease_config(me, 40, 10 * 10**9, 0.04)
        neng.lease_set(to_array(leases))
        lsim = LR.LeaseSim(leases, me, 40, 10 * 10**9, 0.04, kind_salt=1)
        seed = 0x77
        if fused:
            peng.tick_bind(neng, node_ptr)
        for k in range(200):
            now = NOW0 + k * 250 * 10**6
            if fused:
                neng.tick(peng, now, seed, k, compact=(k % 2 == 0))
            else:
                neng.lease_step(now, seed, k)
            ops = lsim.step(now, seed, k)
            assert sorted((int(r["slot"]), int(r["stage"])) for r in neng.lease_ops()) == sorted(ops), f"step {k}"
            assert_leases_equal(neng.lease_read(), lsim.leases, k)
            for i, op in ops:
                h = LR.held(lsim.leases[i], me)
                nsim.set_managed(i, h, op != LR.OP_BUSY)
                for p in range(node_ptr[i], node_ptr[i + 1]):
                    psim.set_managed(p, h, op != LR.OP_BUSY)
            if not fused:
                neng.lease_sync_pods(peng, node_ptr)
            for eng, sim, prog in ((neng, nsim, nprog), (peng, psim, pprog)):
                if not fused:
                    eng.step(now, seed, k)
                got = sorted((int(r["slot"]), int(r["stage"]), int(r["flags"])) for r in eng.fired())
                assert got == sorted(sim.step(now, seed, k)), f"step {k}"
                compare_state(prog, eng, sim, k)
                hot, _ = eng.read()
                assert [bool(x & abi.F_MANAGED) for x in hot["sched"]] == sim.managed, f"step {k}: managed"
        st = neng.lease_stats()
        assert st["creates"] > 0 and st["renews"] > 0 and st["acquires"] > 0 and st["busy"] > 0, st
    finally:
        neng.close()
        peng.close()


@pytest.mark.gpu
def test_c3_lease_write_failures_parity():
    """The C3 loop with every fourth lease write rejected by the apiserver (kwk_lease_fail,
    syncWorker's err branch node_lease_controller.go:121-128): restored lease, retry after the
    same interval() draw, MANAGED from Held() of the old lease, no re-match; bit-exact with
    the oracle at every step."""
    from dataclasses import replace
    from kwok_amd.host import abi
    from tests.parity_util import NOW0, build, compare_state
    rng = np.random.default_rng(34)
    n_nodes, ppn = 64, 3
    nodes = [W.node_object(f"node-{i}") for i in range(n_nodes)]
    pods = [W.pod_object(f"pod-{i}", f"node-{i // ppn}", job=(i % 10 == 0)) for i in range(n_nodes * ppn)]
    node_ptr = np.arange(0, n_nodes * ppn + 1, ppn, dtype=np.uint32)
    leases = c3_leases(n_nodes, NOW0, rng)
    me = 1
    nprog, neng, nsim = build(W.stage_paths(W.NODE_FAST + W.NODE_HEARTBEAT), nodes, kind_salt=1)
    pprog, peng, psim = build(W.stage_paths(W.POD_FAST), pods, harness=True)
    try:
        neng.lease_config(me, 40, 10 * 10**9, 0.04)
        neng.lease_set(to_array(leases))
        lsim = LR.LeaseSim(leases, me, 40, 10 * 10**9, 0.04, kind_salt=1)
        seed = 0x78
        n_failed = 0
        for k in range(160):
            now = NOW0 + k * 250 * 10**6
            before = [replace(L) for L in lsim.leases]
            neng.lease_step(now, seed, k)
            ops = lsim.step(now, seed, k)
            assert sorted((int(r["slot"]), int(r["stage"])) for r in neng.lease_ops()) == sorted(ops), f"step {k}"
            writes = sorted(i for i, op in ops if op != LR.OP_BUSY)
            failed = writes[k % 4::4]
            if failed:
                neng.lease_fail(now, seed, k, failed, to_array([before[i] for i in failed]))
                for i in failed:
                    lsim.fail(i, before[i], now, seed, k)
                n_failed += len(failed)
            assert_leases_equal(neng.lease_read(), lsim.leases, k)
            for i, op in ops:
                h = LR.held(lsim.leases[i], me)
                resync = op != LR.OP_BUSY and i not in failed
                nsim.set_managed(i, h, resync)
                for p in range(node_ptr[i], node_ptr[i + 1]):
                    psim.set_managed(p, h, resync)
            neng.lease_sync_pods(peng, node_ptr)
            for eng, sim, prog in ((neng, nsim, nprog), (peng, psim, pprog)):
                eng.step(now, seed, k)
                got = sorted((int(r["slot"]), int(r["stage"]), int(r["flags"])) for r in eng.fired())
                assert got == sorted(sim.step(now, seed, k)), f"step {k}"
                compare_state(prog, eng, sim, k)
                hot, _ = eng.read()
                assert [bool(x & abi.F_MANAGED) for x in hot["sched"]] == sim.managed, f"step {k}: managed"
        assert n_failed > 10
    finally:
        neng.close()
        peng.close()


@pytest.mark.gpu
def test_tick_n_equals_separate_calls():
    """kwk_tick_n (the C3 bench's per-interval call) enqueues exactly the per-tick sequence of
    separate calls: same leases, lease statistics, node / pod states, statistics and last fired
    lists / lease ops, for a node + pod pair and for a node engine alone."""
    from tests.parity_util import NOW0, build
    rng = np.random.default_rng(35)
    n_nodes, ppn = 300, 5
    nodes = [W.node_object(f"node-{i}") for i in range(n_nodes)]
    pods = [W.pod_object(f"pod-{i}", f"node-{i // ppn}", job=(i % 10 == 0)) for i in range(n_nodes * ppn)]
    node_ptr = np.arange(0, n_nodes * ppn + 1, ppn, dtype=np.uint32)
    leases = to_array(c3_leases(n_nodes, NOW0, rng))
    pairs = []
    try:
        for _ in range(3):
            _, ne, _ = build(W.stage_paths(W.NODE_FAST + W.NODE_HEARTBEAT), nodes, kind_salt=1)
            _, pe, _ = build(W.stage_paths(W.POD_FAST), pods, harness=True)
            ne.lease_config(1, 40, 10 * 10**9, 0.04)
            ne.lease_set(leases)
            pairs.append((ne, pe))
        seed, dt, n = 0x79, 100 * 10**6, 37
        (ne0, pe0), (ne1, pe1), (ne2, _) = pairs
        for k in range(n):  # separate calls
            ne0.lease_step(NOW0 + k * dt, seed, k)
            ne0.lease_sync_pods(pe0, node_ptr)
            ne0.step(NOW0 + k * dt, seed, k)
            ne0.fired_compact()
            pe0.step(NOW0 + k * dt, seed, k)
            pe0.fired_compact()
        pe1.tick_bind(ne1, node_ptr)
        ne1.tick_n(pe1, 20, NOW0, dt, seed, 0, compact=True)
        ne1.tick_n(pe1, n - 20, NOW0 + 20 * dt, dt, seed, 20, compact=True)
        ne2.tick_n(None, n, NOW0, dt, seed, 0, compact=True)  # the node engine alone (the C3 bench)
        for name, a, b in (("nodes", ne0, ne1), ("pods", pe0, pe1)):
            ha, hb = a.read()[0], b.read()[0]
            for col in ("pred", "sched"):
                assert np.array_equal(ha[col], hb[col]), (name, col)
            pend = (ha["sched"] & 0xFF) != 0xFF
            assert np.array_equal(ha["due"][pend], hb["due"][pend]), name
            fa, fb = a.fired(), b.fired()
            assert np.array_equal(np.sort(fa["slot"]), np.sort(fb["slot"])), name
            for key in ("fired", "matched", "steps", "bytes"):
                assert a.stats()[key] == b.stats()[key], (name, key)
        assert np.array_equal(ne0.lease_read(), ne1.lease_read())
        assert ne0.lease_stats() == ne1.lease_stats()
        oa, ob = ne0.lease_ops(), ne1.lease_ops()
        assert sorted(oa["slot"].tolist()) == sorted(ob["slot"].tolist())
        # node engine alone: its leases advance exactly as the pair's (pods only read them)
        assert np.array_equal(ne0.lease_read(), ne2.lease_read())
        assert ne0.stats()["fired"] > 0 and pe0.stats()["fired"] > 0
    finally:
        for ne, pe in pairs:
            ne.close()
            pe.close()


@pytest.mark.gpu
def test_c3_config_size_tick_n_sampled_oracle():
    """C3 at its configuration size: 100k nodes (node-initialize +
    node-heartbeat 20 s / 25 s, leases 40 s with a 10 s +- 4 % renew) and 2 pod-fast pods per
    node, driven by kwk_tick_n (lease step -> pod sync -> node step -> pod step per tick, the C3
    bench's call) in calls of 1 and 3 ticks of 250 ms for 60 s.  Every 997th node and its pods
    are simulated by the oracle (lease_ref.LeaseSim / OracleSim over the sampled slots: leases
    are independent and the Philox counter is the global slot); after every call the last tick's
    lease API writes, lease records, fired sets, object states and MANAGED flags of the sample
    are bit-exact.  Reference: node_lease_controller.go:108-338, controller.go:285-288."""
    from kwok_amd.host import abi
    from kwok_amd.host.compiler import HarnessSpec, KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files
    from oracle.next_ref import load_stage_docs
    from oracle.sim import OracleSim
    from tests.parity_util import NOW0, compare_state
    from tests.test_scale_oracle import _rows_at
    n_nodes, ppn, me = 100_000, 2, 1
    n_pods = n_nodes * ppn
    rng = np.random.default_rng(36)
    leases = c3_leases(n_nodes, NOW0, rng)
    nfiles, pfiles = W.stage_paths(W.NODE_FAST + W.NODE_HEARTBEAT), W.stage_paths(W.POD_FAST)
    nvars, pvars = [W.node_object("node")], [W.pod_object("p", "n"), W.pod_object("p", "n", job=True)]
    nidx = np.zeros(n_nodes, dtype=np.int32)
    pidx = (((np.arange(n_pods, dtype=np.int64) * 2654435761) >> 9) % 10 == 0).astype(np.int32)
    node_ptr = np.arange(0, n_pods + 1, ppn, dtype=np.uint32)
    held0 = np.array([LR.held(L, me) for L in leases])
    engines = []
    try:
        progs = []
        for files, variants, idx, harness, salt, cap in ((nfiles, nvars, nidx, False, 1, n_nodes),
                                                         (pfiles, pvars, pidx, True, 0, n_pods)):
            prog = KindProgram(load_stage_files(*files), HarnessSpec() if harness else None)
            prog.explore(variants)
            ing = Ingest(prog)
            hot, dels, rec, cls = ing.variant_columns(variants, idx)
            owner = np.arange(cap) if not harness else np.arange(cap) // ppn
            hot["sched"][~held0[owner]] &= ~np.uint32(abi.F_MANAGED)  # readOnly until the lease is held
            eng = Engine(prog, capacity=cap, kind_salt=salt)
            engines.append(eng)
            eng.load_stages()
            eng.set_harness(harness)
            eng.load(hot, dels, rec, cls, ing.record_array())
            progs.append(prog)
        neng, peng = engines
        nprog, pprog = progs
        neng.lease_config(me, 40, 10 * 10**9, 0.04)
        neng.lease_set(to_array(leases))
        peng.tick_bind(neng, node_ptr)
        nslots = list(range(5, n_nodes, 997))
        pslots = [p for i in nslots for p in range(int(node_ptr[i]), int(node_ptr[i + 1]))]
        lsim = LR.LeaseSim([leases[i] for i in nslots], me, 40, 10 * 10**9, 0.04, kind_salt=1, slots=nslots)
        nsim = OracleSim(load_stage_docs(*nfiles), [nvars[0]] * len(nslots), kind_salt=1, slots=nslots)
        psim = OracleSim(load_stage_docs(*pfiles), [pvars[int(pidx[p])] for p in pslots], harness=True, slots=pslots)
        for j, i in enumerate(nslots):
            nsim.managed[j] = bool(held0[i])
            for q in range(ppn):
                psim.managed[j * ppn + q] = bool(held0[i])
        nset, pset = np.asarray(nslots, dtype=np.int64), np.asarray(pslots, dtype=np.int64)
        seed, dt, k, call = 0x7A, 250 * 10**6, 0, 0
        counts = {"ops": 0, "node": 0, "pod": 0}
        while k < 240:
            n = 1 if call % 2 == 0 else 3
            neng.tick_n(peng, n, NOW0 + k * dt, dt, seed, k, compact=True)
            for t in range(k, k + n):
                now = NOW0 + t * dt
                ops = lsim.step(now, seed, t)
                for j, op in ops:
                    h = LR.held(lsim.leases[j], me)
                    nsim.set_managed(j, h, op != LR.OP_BUSY)
                    for q in range(ppn):
                        psim.set_managed(j * ppn + q, h, op != LR.OP_BUSY)
                nexp = nsim.step(now, seed, t)
                pexp = psim.step(now, seed, t)
            k += n
            call += 1
            got_ops = neng.lease_ops()
            sel = got_ops[np.isin(got_ops["slot"].astype(np.int64), nset)]
            assert sorted((int(r["slot"]), int(r["stage"])) for r in sel) == \
                sorted((nslots[j], op) for j, op in ops), f"tick {k - 1}: lease ops"
            got_leases = np.concatenate([neng.lease_read(i, 1) for i in nslots])
            assert_leases_equal(got_leases, lsim.leases, k - 1)
            for eng, sim, prog, sset, exp, name in ((neng, nsim, nprog, nset, nexp, "node"),
                                                    (peng, psim, pprog, pset, pexp, "pod")):
                f = eng.fired()
                f = f[np.isin(f["slot"].astype(np.int64), sset)]
                assert sorted((int(r["slot"]), int(r["stage"]), int(r["flags"])) for r in f) == sorted(exp), \
                    f"tick {k - 1}: {name} fired"
                rows = _rows_at(eng, sim.slots)
                compare_state(prog, eng, sim, k - 1, rows=rows)
                assert [bool(x & abi.F_MANAGED) for x in rows[0]["sched"]] == sim.managed, f"tick {k - 1}: {name} managed"
                counts[name] += len(exp)
            counts["ops"] += len(ops)
        st = neng.lease_stats()
        assert st["creates"] > 40_000 and st["renews"] > 0 and st["acquires"] > 0 and st["busy"] > 0, st
        assert counts["ops"] > 0 and counts["node"] > 0 and counts["pod"] > 0, counts
        per = neng.stats()["fired_per_stage"]
        assert per["node-heartbeat"] > 0, per
    finally:
        for e in engines:
            e.close()


@pytest.mark.gpu
def test_tick_disregarded_nodes_are_not_managed():
    """a node need() rejects (node_controller.go:186-200) never gets putNodeInfo /
    onNodeManagedFunc, so kwok never calls TryHold for its Lease and its pods are never managed
    (nodeGetFunc fails, pod_controller.go:393-395).  The host duty: such a node's
    lease record goes to kwk_lease_set without HOLD / QUEUED, and its pods are upserted with
    KWK_F_MANAGED clear.  A third of 3000 nodes carry pool=frozen (the disregard label selector);
    kwk_tick_n over 40 ticks: no lease write, fire or MANAGED bit ever touches them or their pods,
    while every other node's leases, nodes and pods stay bit-exact against the oracle
    (lease_ref.LeaseSim + OracleSim with the same filter)."""
    from kwok_amd.host import abi
    from kwok_amd.host.compiler import HarnessSpec, KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.labelsel import DisregardSpec
    from kwok_amd.host.stages import load_stage_files
    from oracle.next_ref import load_stage_docs
    from oracle.sim import OracleSim
    from tests.parity_util import NOW0, compare_state
    n_nodes, ppn, me = 3000, 2, 1
    n_pods = n_nodes * ppn
    rng = np.random.default_rng(37)
    frozen = np.arange(n_nodes) % 3 == 0
    leases = c3_leases(n_nodes, NOW0, rng)
    for i in np.flatnonzero(frozen):  # no TryHold: not in holdLeaseSet, nothing queued
        leases[i].flags &= ~(LR.HOLD | LR.QUEUED)
        leases[i].next_try_ns = 0
    nfiles, pfiles = W.stage_paths(W.NODE_FAST + W.NODE_HEARTBEAT), W.stage_paths(W.POD_FAST)
    nodes = [W.node_object(f"node-{i}", labels={"pool": "frozen"} if frozen[i] else None) for i in range(n_nodes)]
    pvars = [W.pod_object("p", "n"), W.pod_object("p", "n", job=True)]
    pidx = (np.arange(n_pods) % 10 == 3).astype(np.int32)
    pods = [pvars[int(k)] for k in pidx]
    node_ptr = np.arange(0, n_pods + 1, ppn, dtype=np.uint32)
    held0 = np.array([LR.held(L, me) for L in leases])
    dg = DisregardSpec(label_selector="pool=frozen")
    engines = []
    try:
        nprog = KindProgram(load_stage_files(*nfiles), None, disregard=dg)
        nprog.explore(nodes)
        ning = Ingest(nprog)
        nhot, ndels, nrec, ncls = ning.columns(nodes)
        nhot["sched"][~held0] &= ~np.uint32(abi.F_MANAGED)
        pprog = KindProgram(load_stage_files(*pfiles), HarnessSpec())
        pprog.explore(pvars)
        ping = Ingest(pprog)
        phot, pdels, prec, pcls = ping.variant_columns(pvars, pidx)
        pod_node = np.arange(n_pods) // ppn
        phot["sched"][~held0[pod_node] | frozen[pod_node]] &= ~np.uint32(abi.F_MANAGED)
        neng = Engine(nprog, capacity=n_nodes, kind_salt=1)
        engines.append(neng)
        peng = Engine(pprog, capacity=n_pods)
        engines.append(peng)
        neng.load_stages()
        neng.load(nhot, ndels, nrec, ncls, ning.record_array())
        peng.load_stages()
        peng.set_harness(True)
        peng.load(phot, pdels, prec, pcls, ping.record_array())
        neng.lease_config(me, 40, 10 * 10**9, 0.04)
        neng.lease_set(to_array(leases))
        peng.tick_bind(neng, node_ptr)
        lsim = LR.LeaseSim(leases, me, 40, 10 * 10**9, 0.04, kind_salt=1)
        nsim = OracleSim(load_stage_docs(*nfiles), nodes, kind_salt=1,
                         disregard=(dg.annotation_selector, dg.label_selector))
        psim = OracleSim(load_stage_docs(*pfiles), pods, harness=True)
        for i in range(n_nodes):
            nsim.managed[i] = bool(held0[i])
            for q in range(ppn):
                psim.managed[i * ppn + q] = bool(held0[i]) and not frozen[i]
        frozen_pods = set(np.flatnonzero(frozen[pod_node]).tolist())
        frozen_nodes = set(np.flatnonzero(frozen).tolist())
        seed, dt = 0x7B, 250 * 10**6
        counts = {"ops": 0, "node": 0, "pod": 0}
        for k in range(40):
            now = NOW0 + k * dt
            neng.tick_n(peng, 1, now, dt, seed, k, compact=True)
            ops = lsim.step(now, seed, k)
            for j, op in ops:
                h = LR.held(lsim.leases[j], me)
                nsim.set_managed(j, h, op != LR.OP_BUSY)
                for q in range(ppn):
                    psim.set_managed(j * ppn + q, h, op != LR.OP_BUSY)
            nexp, pexp = nsim.step(now, seed, k), psim.step(now, seed, k)
            got_ops = neng.lease_ops()
            assert sorted((int(r["slot"]), int(r["stage"])) for r in got_ops) == sorted(ops), f"tick {k}: lease ops"
            assert not {int(r["slot"]) for r in got_ops} & frozen_nodes, k
            assert_leases_equal(neng.lease_read(), lsim.leases, k)
            for eng, sim, prog, exp, name, frz in ((neng, nsim, nprog, nexp, "node", frozen_nodes),
                                                  (peng, psim, pprog, pexp, "pod", frozen_pods)):
                f = eng.fired()
                got = sorted((int(r["slot"]), int(r["stage"]), int(r["flags"])) for r in f)
                assert got == sorted(exp), f"tick {k}: {name} fired"
                assert not {g[0] for g in got} & frz, (k, name)
                compare_state(prog, eng, sim, k)
                hot, _ = eng.read()
                managed = (hot["sched"] & np.uint32(abi.F_MANAGED)) != 0
                assert managed.tolist() == list(sim.managed), f"tick {k}: {name} managed"
                if name == "pod":
                    assert not managed[sorted(frz)].any(), k
                counts[name] += len(exp)
            counts["ops"] += len(ops)
        assert counts["ops"] > 0 and counts["node"] > 0 and counts["pod"] > 0, counts
    finally:
        for e in engines:
            e.close()
