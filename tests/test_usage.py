"""Resource usage (BASELINE C4): per-node usage sums and cumulative integrators.

CPU: the host's compiled per-pod values equal the oracle's restatement of
evaluateContainerResourceUsage for every pod.  GPU: usage_kernel through the C ABI against
the oracle's nodeResourceUsage / nodeResourceCumulativeUsage within 1e-6 relative
(BASELINE.json north_star tolerance)."""
import copy
import os

import numpy as np
import pytest
import yaml

from kwok_amd import workload as W
from kwok_amd.host.usage import UsageProgram, load_usage_yaml, usage_columns
from oracle import usage_ref

GOLDEN = os.path.join(os.path.dirname(os.path.dirname(__file__)), "kwok_amd", "metrics", "usage-from-annotation.yaml")
REL_TOL = 1e-6

EXTRA = """
apiVersion: kwok.x-k8s.io/v1alpha1
kind: ResourceUsage
metadata:
  name: pod-3
  namespace: default
spec:
  usages:
  - containers: [container-0]
    usage:
      cpu: {value: 250m}
      memory: {value: 64Mi}
  - usage:
      cpu: {value: "2"}
"""


def _cluster(n_nodes=30, n_pods=600, seed=21):
    cl = W.make_cluster("C4", n_nodes, n_pods, seed=seed)
    pods = cl.pods.materialize()
    # invalid / odd annotation values: CEL Quantity() error -> 0 (metrics_resource_usage.go:155-160)
    for i, bad in ((5, "abc"), (6, "1.5Gi"), (7, ""), (8, "0.0000000001"), (9, "1e3")):
        pods[i].setdefault("metadata", {}).setdefault("annotations", {})["kwok.x-k8s.io/usage-cpu"] = bad
    return cl, pods


def _docs():
    return [d for d in yaml.safe_load_all(open(GOLDEN).read() + "\n---\n" + EXTRA) if d]


def _program():
    return UsageProgram(*load_usage_yaml(open(GOLDEN).read(), EXTRA))


def test_host_usage_values_match_oracle():
    cl, pods = _cluster()
    prog = _program()
    docs = _docs()
    for p in pods:
        for c in p["spec"]["containers"]:
            for r in ("cpu", "memory"):
                assert prog.container_value(p, c["name"], r) == usage_ref.container_usage(docs, p, c["name"], r)


@pytest.mark.gpu
def test_gpu_node_usage_and_cumulative():
    from kwok_amd.host.compiler import KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files

    cl, pods = _cluster()
    prog = _program()
    keys, cv, mv, mx, ck = usage_columns(prog, pods)
    kp = KindProgram(load_stage_files(*cl.pod_stage_files))
    kp.explore(pods)
    ing = Ingest(kp)
    hot, dels, rec, cls = ing.columns(pods)
    eng = Engine(kp, capacity=len(pods))
    try:
        eng.load_stages()
        eng.load(hot, dels, rec, cls, ing.record_array())
        eng.usage_config(cl.node_ptr, keys, cv, mv, mx, ck)
        docs = _docs()
        ptr = cl.node_ptr
        t0 = 1_700_000_000 * 10**9
        eng.usage(t0)
        node, total = eng.usage_read()

        def expect(alive):
            out = np.zeros((len(ptr) - 1, 2))
            for j in range(len(ptr) - 1):
                pn = [pods[k] for k in range(ptr[j], ptr[j + 1]) if alive[k]]
                out[j] = (usage_ref.node_usage(docs, pn, "cpu"), usage_ref.node_usage(docs, pn, "memory"))
            return out

        alive = np.ones(len(pods), dtype=bool)
        e0 = expect(alive)
        np.testing.assert_allclose(node[:, :2], e0, rtol=REL_TOL, atol=0)
        np.testing.assert_allclose(total, e0.sum(axis=0), rtol=REL_TOL)
        assert np.all(node[:, 2:] == 0)  # first evaluation: integrators start at 0
        # delete every 7th pod (Deleted events) and evaluate 2.5 s later
        gone = np.arange(0, len(pods), 7)
        eng.delete(gone)
        alive[gone] = False
        t1 = t0 + 2_500_000_123
        eng.usage(t1)
        node, total = eng.usage_read()
        e1 = expect(alive)
        np.testing.assert_allclose(node[:, :2], e1, rtol=REL_TOL, atol=0)
        np.testing.assert_allclose(node[:, 2:], usage_ref.seconds(t1 - t0) * e1, rtol=REL_TOL, atol=0)
        t2 = t1 + 10**9
        eng.usage(t2)
        node, _ = eng.usage_read()
        np.testing.assert_allclose(node[:, 2:], usage_ref.seconds(t1 - t0) * e1 + usage_ref.seconds(t2 - t1) * e1,
                                   rtol=REL_TOL, atol=0)
    finally:
        eng.close()


@pytest.mark.gpu
def test_gpu_pod_usage_and_cumulative():
    """Per-pod Usage / CumulativeUsage (the pod and container series of metrics-resource.yaml)
    against the oracle's per-container integrators, across deletions and re-creation."""
    from kwok_amd.host.compiler import KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files

    cl, pods = _cluster(n_nodes=12, n_pods=300, seed=5)
    prog = _program()
    keys, cv, mv, mx, ck = usage_columns(prog, pods)
    kp = KindProgram(load_stage_files(*cl.pod_stage_files))
    kp.explore(pods)
    ing = Ingest(kp)
    cols = ing.columns(pods)
    eng = Engine(kp, capacity=len(pods))
    try:
        eng.load_stages()
        eng.load(*cols, ing.record_array())
        eng.usage_config(cl.node_ptr, keys, cv, mv, mx, ck)
        eng.usage_pods(True)
        docs = _docs()
        cum = usage_ref.Cumulative()
        alive = np.ones(len(pods), dtype=bool)
        gone = np.arange(0, len(pods), 5)
        t = 1_700_000_000 * 10**9
        for k in range(6):
            if k == 2:
                eng.delete(gone)
                alive[gone] = False
            if k == 4:  # re-created under the same names: the integrators continue
                hot, dels, rec, cls = cols
                eng.upsert(gone, hot[gone], dels[gone], rec[gone], cls[gone])
                alive[gone] = True
            eng.usage(t)
            got = eng.usage_read_pods()
            want = np.zeros((len(pods), 4))
            for i, p in enumerate(pods):
                if alive[i]:
                    want[i] = (usage_ref.pod_usage(docs, p, "cpu"), usage_ref.pod_usage(docs, p, "memory"),
                               cum.pod(docs, p, "cpu", t), cum.pod(docs, p, "memory", t))
            np.testing.assert_allclose(got, want, rtol=REL_TOL, atol=1e-9, err_msg=f"evaluation {k}")
            t += 1_000_000_000 + 37_000_001 * k
        assert np.any(got[:, 2] > 0) and np.any(got[:, 3] > 0)
    finally:
        eng.close()


def test_oracle_cumulative_integrator():
    """The first evaluation of a key records the time only; later ones add seconds(dt) * value
    (metrics_resource_usage.go:36-52); pods sum their containers' integrators."""
    c = usage_ref.Cumulative()
    assert c.advance("k", 3.0, 10**9) == 0.0
    assert c.advance("k", 3.0, 3_500_000_000) == pytest.approx(7.5)
    assert c.advance("k", 1.0, 4_500_000_000) == pytest.approx(8.5)
    docs = _docs()
    _, pods = _cluster(n_nodes=2, n_pods=20, seed=3)
    p = max(pods, key=lambda q: len(q["spec"]["containers"]))
    assert c.pod(docs, p, "cpu", 0) == 0.0
    assert c.pod(docs, p, "cpu", 2 * 10**9) == pytest.approx(2 * usage_ref.pod_usage(docs, p, "cpu"))


def _irregular_node_ptr(n_pods):
    """Node sizes the chunking must get right: empty nodes (first, inner, trailing), 1-pod nodes
    (more of them than one chunk holds), a node larger than a wave row (its sum carried from row
    to row), chunk-sized runs, and an odd first pod of a chunk."""
    sizes = [0, 1, 2500, 0, 0] + [1] * 300 + [7, 0, 1016, 1017, 3]
    rest = n_pods - sum(sizes)
    assert rest > 0
    while rest > 0:
        sizes.append(min(37, rest))
        rest -= sizes[-1]
    sizes += [0, 0]
    return np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)


@pytest.mark.gpu
@pytest.mark.parametrize("state", ["auto", "u32", "dw", "wide"])
def test_gpu_usage_irregular_nodes(state):
    """usage_kernel's chunks of whole nodes (kwk_usage_config) against the oracle's
    nodeResourceUsage, per node and in total, for the 2-, 4- and 8-byte state formats, with
    per-pod outputs on."""
    from kwok_amd.host.compiler import KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files

    cl, pods = _cluster(n_nodes=40, n_pods=6000, seed=17)
    ptr = _irregular_node_ptr(len(pods))
    prog = _program()
    keys, cv, mv, mx, ck = usage_columns(prog, pods)
    kp = KindProgram(load_stage_files(*cl.pod_stage_files))
    kp.explore(pods)
    ing = Ingest(kp)
    cols = ing.columns(pods)
    eng = Engine(kp, capacity=len(pods), state=state)
    try:
        eng.load_stages()
        eng.load(*cols, ing.record_array())
        eng.usage_config(ptr, keys, cv, mv, mx, ck)
        eng.usage_pods(True)
        gone = np.arange(3, len(pods), 11)
        eng.delete(gone)
        alive = np.ones(len(pods), dtype=bool)
        alive[gone] = False
        docs = _docs()
        t0 = 1_700_000_000 * 10**9
        eng.usage(t0)
        eng.usage(t0 + 2 * 10**9)
        node, total = eng.usage_read()
        want = np.zeros((len(ptr) - 1, 2))
        for j in range(len(ptr) - 1):
            pn = [pods[k] for k in range(ptr[j], ptr[j + 1]) if alive[k]]
            want[j] = (usage_ref.node_usage(docs, pn, "cpu"), usage_ref.node_usage(docs, pn, "memory"))
        np.testing.assert_allclose(node[:, :2], want, rtol=REL_TOL, atol=0)
        np.testing.assert_allclose(node[:, 2:], 2.0 * want, rtol=REL_TOL, atol=0)
        np.testing.assert_allclose(total, want.sum(axis=0), rtol=REL_TOL)
        per_pod = eng.usage_read_pods()
        np.testing.assert_allclose(per_pod[~alive], 0.0)
        want_pod = [usage_ref.pod_usage(docs, p, "cpu") for p, a in zip(pods, alive) if a]
        np.testing.assert_allclose(per_pod[alive, 0], want_pod, rtol=REL_TOL, atol=0)
    finally:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n_pods", [6000, 5997])
@pytest.mark.parametrize("state", ["auto", "u32", "dw", "wide"])
def test_gpu_usage_fast_path_irregular_nodes(state, n_pods):
    """The uniform-container configuration (no mixed pods, no per-pod outputs) takes
    usage_fast_kernel: same irregular node layout, node sums and integrators vs the oracle.
    5997 pods: the state / key columns end inside a dword (the buffer resources' range check
    works per dword: round 4 found the last pods read as dead there)."""
    from kwok_amd.host.compiler import KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files

    cl, pods = _cluster(n_nodes=40, n_pods=n_pods, seed=23)
    ptr = _irregular_node_ptr(len(pods))
    text = open(GOLDEN).read()
    prog = UsageProgram(*load_usage_yaml(text))
    docs = [d for d in yaml.safe_load_all(text) if d]
    keys, cv, mv, mx, ck = usage_columns(prog, pods)
    assert mx is None or len(mx) == 0  # every pod's containers alike: the fast kernel's case
    kp = KindProgram(load_stage_files(*cl.pod_stage_files))
    kp.explore(pods)
    ing = Ingest(kp)
    cols = ing.columns(pods)
    eng = Engine(kp, capacity=len(pods), state=state)
    try:
        eng.load_stages()
        eng.load(*cols, ing.record_array())
        eng.usage_config(ptr, keys, cv, mv, mx, ck)
        gone = np.arange(5, len(pods), 13)
        eng.delete(gone)
        alive = np.ones(len(pods), dtype=bool)
        alive[gone] = False
        t0 = 1_700_000_000 * 10**9
        eng.usage(t0)
        eng.usage(t0 + 3 * 10**9)
        node, total = eng.usage_read()
        want = np.zeros((len(ptr) - 1, 2))
        for j in range(len(ptr) - 1):
            pn = [pods[k] for k in range(ptr[j], ptr[j + 1]) if alive[k]]
            want[j] = (usage_ref.node_usage(docs, pn, "cpu"), usage_ref.node_usage(docs, pn, "memory"))
        np.testing.assert_allclose(node[:, :2], want, rtol=REL_TOL, atol=0)
        np.testing.assert_allclose(node[:, 2:], 3.0 * want, rtol=REL_TOL, atol=0)
        np.testing.assert_allclose(total, want.sum(axis=0), rtol=REL_TOL)
        assert want[:, 0].min() == 0.0 and want[:, 0].max() > 0  # empty nodes and busy ones
    finally:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("state", ["auto", "u32", "dw"])
def test_gpu_usage_key8_column_matches_4byte_keys(state):
    """kwk_usage_config builds a 1-byte usage-key column when at most 256 distinct keys occur
    (the C5 pods have 2): usage_fast_kernel<WB, true> must give node sums and integrators
    bit-identical to the 4-byte-key kernel (KWK_TUNE_USAGE without KWK_USAGE_KEY8), and equal to numpy."""
    from kwok_amd.host import abi
    from kwok_amd.host.compiler import KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files

    cl, pods = _cluster(n_nodes=40, n_pods=6000, seed=29)
    ptr = _irregular_node_ptr(len(pods))
    rng = np.random.default_rng(3)
    cv, mv = rng.random(60) * 4, rng.random(70) * 2**32
    ci, mi, nc = rng.integers(0, 60, 200), rng.integers(0, 70, 200), rng.integers(1, 6, 200)
    dict_keys = (ci | (mi << 14) | (nc << 28)).astype(np.uint32)  # 200 distinct keys
    pick = rng.integers(0, 200, len(pods))
    keys = dict_keys[pick]
    kp = KindProgram(load_stage_files(*cl.pod_stage_files))
    kp.explore(pods)
    ing = Ingest(kp)
    cols = ing.columns(pods)
    gone = np.arange(7, len(pods), 11)
    alive = np.ones(len(pods), dtype=bool)
    alive[gone] = False
    t0 = 1_700_000_000 * 10**9
    got = {}
    for key8 in (1, 0):
        eng = Engine(kp, capacity=len(pods), state=state)
        try:
            eng.set_tuning(abi.TUNE_USAGE, key8 * abi.USAGE_KEY8 | abi.USAGE_AGG_FUSED)
            eng.load_stages()
            eng.load(*cols, ing.record_array())
            eng.usage_config(ptr, keys, cv, mv)
            eng.delete(gone)
            eng.usage(t0)
            eng.usage(t0 + 2 * 10**9)
            got[key8] = eng.usage_read()
        finally:
            eng.close()
    assert np.array_equal(got[1][0], got[0][0]) and np.array_equal(got[1][1], got[0][1])
    node, total = got[1]
    pod_c = np.where(alive, nc[pick] * cv[ci[pick]], 0.0)
    pod_m = np.where(alive, nc[pick] * mv[mi[pick]], 0.0)
    want = np.array([[pod_c[ptr[j]:ptr[j + 1]].sum(), pod_m[ptr[j]:ptr[j + 1]].sum()] for j in range(len(ptr) - 1)])
    np.testing.assert_allclose(node[:, :2], want, rtol=REL_TOL, atol=0)
    np.testing.assert_allclose(node[:, 2:], 2.0 * want, rtol=REL_TOL, atol=0)
    np.testing.assert_allclose(total, want.sum(axis=0), rtol=REL_TOL)


@pytest.mark.gpu
@pytest.mark.parametrize("pods_per_node", [100, 37])
def test_gpu_usage_one_key_runs_match_per_pod_sums(pods_per_node):
    """usage_fast_kernel<1, true> (1-byte ids, 1-byte keys): where every lane's 16 pods carry one
    key (< 16 keys, the C5 case) a lane's sums are read from the in-order sums of 0..16 pods of
    that key, and a lane's first node is found from the chunk's mean node size.  Both must give
    node sums and integrators bit-identical to the per-pod loop of the 4-byte-key kernel
    (KWK_TUNE_USAGE without KWK_USAGE_KEY8): one column with waves of one-key runs, a mixed stretch, keys >= 16,
    dead pods and churned ids, 100 pods per node (the C5 shape) and 37 (irregular last node)."""
    import bench
    from kwok_amd.host import abi
    n_nodes = 200_000 // pods_per_node
    n = n_nodes * pods_per_node
    ptr = (np.arange(n_nodes + 1, dtype=np.int64) * pods_per_node).astype(np.uint32)
    ptr[-2] = ptr[-1] - 3  # a short last-but-one node
    rng = np.random.default_rng(5)
    cv, mv = rng.random(30) * 3, rng.random(30) * 2**30
    ci, mi, nc = rng.integers(0, 30, 24), rng.integers(0, 30, 24), rng.integers(1, 5, 24)
    dict_keys = (ci | (mi << 14) | (nc << 28)).astype(np.uint32)  # 24 distinct keys
    # blocks of 1024 pods of one key (keys 0..3), a mixed stretch, a stretch of key 20 (>= 16)
    pick = np.repeat(np.arange(n // 1024 + 1) % 4, 1024)[:n]
    pick[40_000:42_000] = rng.integers(0, 24, 2000)
    pick[60_000:70_000] = 20
    keys = dict_keys[pick]
    gone = np.arange(3, n, 17)
    t0 = bench.NOW0 + 10 * 10**9
    got = {}
    for key8 in (1, 0):
        pods, nodes, _ = bench.build_engines(0, n_nodes, pods_per_node, 0, 0x6B776F6B, 0.1)
        try:
            assert pods.stats()["state_bytes"] == 1
            pods.set_tuning(abi.TUNE_USAGE, key8 * abi.USAGE_KEY8 | abi.USAGE_AGG_FUSED)
            pods.usage_config(ptr, keys, cv, mv)
            for k in range(3):  # churned ids (pods deleted by the harness read as dead)
                pods.step(bench.NOW0 + k * 10**9, 1, k)
            pods.delete(gone)
            pods.usage(t0)
            pods.usage(t0 + 2 * 10**9)
            got[key8] = pods.usage_read()
        finally:
            pods.close()
            nodes.close()
    assert np.array_equal(got[1][0], got[0][0]) and np.array_equal(got[1][1], got[0][1])
    node, total = got[1]
    assert node[:, 0].max() > 0
    np.testing.assert_allclose(total, node[:, :2].sum(axis=0), rtol=REL_TOL)


@pytest.mark.gpu
@pytest.mark.parametrize("pods_per_node", [100, 7])
def test_gpu_aggregate_counts_in_usage_pass(pods_per_node):
    """kwk_aggregate on 1-byte ids with usage: the mask counts taken inside the usage kernel's pass
    (KWK_USAGE_AGG_FUSED, the default) equal a count pass of their own (0) and kwk_count, and the
    usage sums are unchanged — 2M pods of the C5 shape after churn steps; 100 pods per node (the
    branch-free rows) and 7 (runs crossing several node boundaries: the per-pod loop)."""
    import bench
    from kwok_amd.host import abi
    from kwok_amd.host.cluster import phase_masks
    n_nodes = 2_000_000 // pods_per_node
    pods, nodes, (pvars, pidx) = bench.build_engines(0, n_nodes, pods_per_node, 0, 0x6B776F6B, 0.1)
    try:
        bench.configure_usage(pods, pvars, pidx, n_nodes, pods_per_node)
        assert pods.stats()["state_bytes"] == 1
        for k in range(5):
            pods.step(bench.NOW0 + k * 10**9, 1, k)
        pm = [0] + list(phase_masks(pods.p, values=("Running", "Succeeded", "Failed")).values())
        pm = pm[:4]
        now = bench.NOW0 + 10 * 10**9
        outs = []
        for fused in (1, 0):
            pods.set_tuning(abi.TUNE_USAGE, abi.USAGE_KEY8 | fused * abi.USAGE_AGG_FUSED)
            n = pods.aggregate(pm, now, usage=True)
            outs.append(pods.aggregate_read(n))
        pods.set_tuning(abi.TUNE_USAGE, abi.USAGE_KEY8 | abi.USAGE_AGG_FUSED)
        assert np.array_equal(outs[0], outs[1])
        counts = pods.count(pm)
        n_st = len(outs[0]) - len(pm) - 2
        assert outs[0][n_st:n_st + len(pm)].astype(np.int64).tolist() == [int(c) for c in counts]
        assert counts[0] > 0 and outs[0][-2] > 0
    finally:
        pods.close()
        nodes.close()


def _mixed_usage_doc(name):
    """A namespaced ResourceUsage named like the pod: container-1 evaluates apart from the others
    (findUsageInUsages, metrics_resource_usage.go:226-264), so the pod takes kwk_usage_mixed."""
    return {"apiVersion": "kwok.x-k8s.io/v1alpha1", "kind": "ResourceUsage",
            "metadata": {"name": name, "namespace": "default"},
            "spec": {"usages": [{"containers": ["container-1"],
                                 "usage": {"cpu": {"value": "300m"}, "memory": {"value": "32Mi"}}},
                                {"usage": {"cpu": {"value": "2"}, "memory": {"expression": 'Quantity("1Gi")'}}}]}}


@pytest.mark.gpu
def test_c4_config_size_sampled_oracle():
    """C4 at its configuration size: 10k nodes / 1M pods, 1-4 containers per
    pod, half of the pods annotated from the workload's usage values (usage-from-annotation), and
    ~250 pods whose containers differ (a pod-named ResourceUsage: kwk_usage_mixed).  Over three
    evaluations (pods deleted before the second), every 97th node's usage and cumulative usage
    against the oracle's nodeResourceUsage / nodeResourceCumulativeUsage restatement (usage_ref)
    within 1e-6 relative, and the cluster totals against the per-variant values summed exactly.
    Reference: pkg/kwok/server/metrics_resource_usage.go:36-224."""
    from kwok_amd.host.compiler import KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files
    n_nodes, n_pods = 10_000, 1_000_000
    cl = W.make_cluster("C4", n_nodes, n_pods, seed=44)
    ptr = cl.node_ptr
    pvars, pidx = cl.pods.variants, cl.pods.index
    sample = list(range(3, n_nodes, 97))
    mixed = sorted(set(range(17, n_pods, 4999)) | {int(ptr[j]) + 1 for j in sample[::2] if ptr[j + 1] - ptr[j] > 1})
    mixed_objs = [cl.pods.materialize(i, i + 1)[0] for i in mixed]
    text = open(GOLDEN).read()
    extra = [_mixed_usage_doc(o["metadata"]["name"]) for o in mixed_objs]
    docs = [d for d in yaml.safe_load_all(text) if d] + extra
    prog = UsageProgram(*load_usage_yaml(text, yaml.safe_dump_all(extra)))
    keys_all, cv, mv, mx, ck = usage_columns(prog, list(pvars) + mixed_objs)
    keys = keys_all[:len(pvars)][pidx]
    keys[mixed] = keys_all[len(pvars):]
    assert mx is not None and len(mx) >= 2 and np.count_nonzero((keys >> 28) == 0) >= len(mixed) // 2
    kp = KindProgram(load_stage_files(*cl.pod_stage_files))
    kp.explore(pvars)
    ing = Ingest(kp)
    hot, dels, rec, cls = ing.variant_columns(pvars, pidx)
    eng = Engine(kp, capacity=n_pods)
    try:
        eng.load_stages()
        eng.load(hot, dels, rec, cls, ing.record_array())
        eng.usage_config(ptr, keys, cv, mv, mx, ck)
        # the sampled nodes' pods, materialised once (the mixed ones carry their real names)
        pods_of = {}
        for j in sample:
            objs = cl.pods.materialize(int(ptr[j]), int(ptr[j + 1]))
            pods_of[j] = objs
        val = {}  # (pod index, resource) -> the pod's usage (the oracle, once)
        for j in sample:
            for k, p in enumerate(pods_of[j]):
                for r in ("cpu", "memory"):
                    val[(int(ptr[j]) + k, r)] = usage_ref.node_usage(docs, [p], r)
        # exact cluster totals from the per-variant values (+ the mixed pods)
        var_val = {r: np.array([usage_ref.node_usage(docs[:1], [v], r) for v in pvars]) for r in ("cpu", "memory")}
        mix_val = {r: np.array([usage_ref.node_usage(docs, [o], r) for o in mixed_objs]) for r in ("cpu", "memory")}
        alive = np.ones(n_pods, dtype=bool)
        cum = usage_ref.Cumulative()
        t = 1_700_000_000 * 10**9
        for k in range(3):
            if k == 1:
                gone = np.arange(11, n_pods, 13)
                eng.delete(gone)
                alive[gone] = False
            eng.usage(t)
            node, total = eng.usage_read()
            for j in sample:
                lo, hi = int(ptr[j]), int(ptr[j + 1])
                want = [sum(val[(i, r)] for i in range(lo, hi) if alive[i]) for r in ("cpu", "memory")]
                wc = [cum.advance((j, r), want[q], t) for q, r in enumerate(("cpu", "memory"))]
                np.testing.assert_allclose(node[j], want + wc, rtol=REL_TOL, atol=0, err_msg=f"evaluation {k}, node {j}")
            plain = alive.copy()
            plain[mixed] = False
            for q, r in enumerate(("cpu", "memory")):
                exact = float(np.bincount(pidx[plain], minlength=len(pvars)) @ var_val[r]) + \
                    float(mix_val[r][alive[mixed]].sum())
                assert total[q] == pytest.approx(exact, rel=REL_TOL), (k, r)
            t += 2_500_000_000 + 123_457 * k
    finally:
        eng.close()
