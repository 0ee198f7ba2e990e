"""C5's cross-GPU aggregates (metrics_resource_usage.go:195-224): the pod
phase histogram (kwk_count), per-stage transition counts (kwk_stats) and the cluster usage
(kwk_usage) of node-block shard engines, summed as the RCCL all-reduce sums them, equal one
whole-cluster engine and the oracle — counts bit-exact, usage within 1e-6 relative."""
import os

import numpy as np
import pytest
import yaml

from kwok_amd import workload as W
from kwok_amd.host.cluster import Aggregates, DeviceReport, engine_aggregates, local_node_ptr, node_block, phase_masks, pod_range
from kwok_amd.host.usage import UsageProgram, load_usage_yaml, usage_columns

GOLDEN = os.path.join(os.path.dirname(os.path.dirname(__file__)), "kwok_amd", "metrics", "usage-from-annotation.yaml")
REL_TOL = 1e-6


def oracle_aggregates(sim, docs, fired_per_stage):
    """The same aggregates from the oracle simulation's JSON objects."""
    from oracle import refcpu, usage_ref
    alive = [o for o in sim.objs if o is not None]
    ph = [(refcpu.query(".status.phase", o) or [None])[0] for o in alive]
    counts = [len(alive), ph.count("Running"), ph.count("Succeeded")]
    usage = [sum(usage_ref.pod_usage(docs, o, r) for o in alive) for r in ("cpu", "memory")]
    return np.array(fired_per_stage), np.array(counts), np.array(usage)


@pytest.mark.gpu
def test_shard_engine_aggregates_equal_whole_engine_and_oracle():
    from tests.parity_util import NOW0, build
    n_nodes, world = 12, 2
    cl = W.make_cluster("C4", n_nodes, 480, seed=31)
    objs = cl.pods.materialize()
    for i, o in enumerate(objs):  # Job-owned pods complete, get deleted and re-created (harness churn)
        if i % 3 == 0:
            o["metadata"]["ownerReferences"] = [{"apiVersion": "batch/v1", "kind": "Job", "name": f"j{i}", "uid": f"u{i}"}]
    text = open(GOLDEN).read()
    up = UsageProgram(*load_usage_yaml(text))
    docs = [d for d in yaml.safe_load_all(text) if d]
    prog, whole, sim = build(cl.pod_stage_files, objs, harness=True)
    keys, cv, mv, mx, ck = usage_columns(up, objs)
    whole.usage_config(cl.node_ptr, keys, cv, mv, mx, ck)
    shards = []
    for r in range(world):
        lo, hi = node_block(n_nodes, world, r)
        plo, phi = pod_range(cl.node_ptr, lo, hi)
        _, eng, _ = build(cl.pod_stage_files, objs[plo:phi], harness=True, slot_base=plo)
        k2, c2, m2, x2, q2 = usage_columns(up, objs[plo:phi])
        eng.usage_config(local_node_ptr(cl.node_ptr, lo, hi), k2, c2, m2, x2, q2)
        shards.append(eng)
    pm = phase_masks(prog, values=("Running", "Succeeded"))
    masks, names = [[0, pm["Running"], pm["Succeeded"]]], [["pods", "Running", "Succeeded"]]
    fired = np.zeros(len(prog.names), dtype=np.int64)
    checked, churn = 0, []
    try:
        for k in range(14):
            now = NOW0 + k * 10**9
            for e in [whole] + shards:
                e.step(now, 11, k)
            for _, s, _ in sim.step(now, 11, k):
                fired[s] += 1
            if k % 3 != 2:
                continue
            a_whole = engine_aggregates([whole], masks, names, now, usage_engine=whole)
            parts = [engine_aggregates([e], masks, names, now, usage_engine=e) for e in shards]
            # the device path the bench's reporter takes (kwk_aggregate, no host round trip)
            dev = [DeviceReport([e], masks, names, usage_engine=e) for e in shards]
            for d in dev:
                d.collect(now)
            d_parts = [d.result() for d in dev]
            for p_host, p_dev in zip(parts, d_parts):
                assert p_dev.fired_per_stage.tolist() == p_host.fired_per_stage.tolist(), f"step {k}"
                assert p_dev.counts.tolist() == p_host.counts.tolist(), f"step {k}"
                np.testing.assert_allclose(p_dev.usage, p_host.usage, rtol=1e-12, err_msg=f"step {k}")
            a_sum = a_whole.unpack(np.sum([p.pack() for p in parts], axis=0))  # what the all-reduce computes
            o_fired, o_counts, o_usage = oracle_aggregates(sim, docs, fired)
            for a in (a_whole, a_sum):
                assert a.fired_per_stage.tolist() == o_fired.tolist(), f"step {k}"
                assert a.counts.tolist() == o_counts.tolist(), f"step {k}"
                np.testing.assert_allclose(a.usage, o_usage, rtol=REL_TOL, err_msg=f"step {k}")
            churn.append(o_counts[0] < len(objs) or o_counts[2] > 0)
            checked += 1
        assert checked == 4 and any(churn)  # deletions / completions reached the aggregates
    finally:
        whole.close()
        for e in shards:
            e.close()


@pytest.mark.gpu
def test_native_rccl_report_world1_equals_engine_aggregates():
    """libkwok_comm (the torch-free collective a Go host links, include/kwok_comm.h) at world
    size 1: kwk_aggregate into the communicator's buffer, ncclAllReduce in place ordered after
    the engines' streams by events, read back — equal to the host-side aggregates of the same
    engines (a one-rank sum is the identity; the N > 1 path is the driver's scaling run)."""
    from kwok_amd.host.comm import NativeComm, NativeReport, unique_id
    from tests.parity_util import NOW0, build
    cl = W.make_cluster("C4", 6, 240, seed=37)
    objs = cl.pods.materialize()
    for i, o in enumerate(objs):
        if i % 4 == 0:
            o["metadata"]["ownerReferences"] = [{"apiVersion": "batch/v1", "kind": "Job", "name": f"j{i}", "uid": f"u{i}"}]
    text = open(GOLDEN).read()
    up = UsageProgram(*load_usage_yaml(text))
    prog, pods, _ = build(cl.pod_stage_files, objs, harness=True)
    nprog, nodes, _ = build(cl.node_stage_files, cl.nodes.materialize(), kind_salt=1)
    pods.usage_config(cl.node_ptr, *usage_columns(up, objs))
    pm = phase_masks(prog, values=("Running", "Succeeded"))
    masks = [[0, pm["Running"], pm["Succeeded"]], [0]]
    names = [["pods", "Running", "Succeeded"], ["nodes"]]
    comm = NativeComm(unique_id(), 0, 1, 0)
    try:
        rep = NativeReport(comm, [pods, nodes], masks, names, usage_engine=pods)
        for k in range(9):
            now = NOW0 + k * 10**9
            pods.step(now, 5, k)
            nodes.step(now, 5, k)
            if k % 3 != 2:
                continue
            rep.collect(now)
            got = rep.result()
            want = engine_aggregates([pods, nodes], masks, names, now, usage_engine=pods)
            assert got.fired_per_stage.tolist() == want.fired_per_stage.tolist(), k
            assert got.counts.tolist() == want.counts.tolist(), k
            np.testing.assert_allclose(got.usage, want.usage, rtol=1e-12)
            assert got.fired_per_stage.sum() > 0
    finally:
        comm.close()
        pods.close()
        nodes.close()
