"""Multi-GPU path on CPU: node-block sharding, shard-invariant workload generation and the
aggregate all-reduce, with the gloo backend at world_size 2 (the GPU run uses the same code
with RCCL).  The oracle simulation of each shard (RNG keyed by global slot) must sum to the
single-process simulation of the whole cluster."""
import os
import socket
import sys

import numpy as np
import pytest

from kwok_amd import workload as W
from kwok_amd.host.cluster import Aggregates, local_node_ptr, node_block, pod_range

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_node_blocks_partition_the_cluster():
    for n, world in ((10, 3), (1_000_000, 8), (7, 8)):
        blocks = [node_block(n, world, r) for r in range(world)]
        assert blocks[0][0] == 0 and blocks[-1][1] == n
        assert all(blocks[r][1] == blocks[r + 1][0] for r in range(world - 1))


def test_bench_pod_variants_are_shard_invariant():
    sys.path.insert(0, ROOT)
    import bench
    full = bench.shard_pod_variants(0, 50_000, 7, 0.1)
    parts = [bench.shard_pod_variants(lo, hi, 7, 0.1) for lo, hi in ((0, 12_345), (12_345, 40_000), (40_000, 50_000))]
    assert np.array_equal(full, np.concatenate(parts))
    assert 0.08 < full.mean() < 0.12


GOLDEN_USAGE = os.path.join(ROOT, "kwok_amd", "metrics", "usage-from-annotation.yaml")


def _shard_aggregates(pods, slot_base, steps, files):
    """A shard's aggregates in the engine's shape (bench.py Reporter / cluster.engine_aggregates):
    per-stage transitions, [alive, Running, Succeeded] counts and the cluster usage, computed
    by the oracle simulation of the shard (RNG keyed by global slot)."""
    import yaml
    from oracle.next_ref import load_stage_docs
    from oracle.sim import OracleSim
    from oracle import refcpu, usage_ref
    sim = OracleSim(load_stage_docs(*files), pods, harness=True, slot_base=slot_base)
    fired = np.zeros(len(sim.stages), dtype=np.int64)
    for k in range(steps):
        for _, s, _ in sim.step(1_700_000_000 * 10**9 + k * 10**9, 99, k):
            fired[s] += 1
    alive = [o for o in sim.objs if o is not None]
    ph = [(refcpu.query(".status.phase", o) or [None])[0] for o in alive]
    docs = [d for d in yaml.safe_load_all(open(GOLDEN_USAGE).read()) if d]
    usage = np.array([sum(usage_ref.pod_usage(docs, o, r) for o in alive) for r in ("cpu", "memory")])
    return Aggregates([s.name for s in sim.stages], fired, np.array([len(alive), ph.count("Running"),
                                                                      ph.count("Succeeded")]),
                      ["pods", "pods_Running", "pods_Succeeded"], usage)


def _worker(rank, world, port, result_path):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cl = W.make_cluster("C4", 6, 60, seed=4)
    lo, hi = node_block(6, world, rank)
    plo, phi = pod_range(cl.node_ptr, lo, hi)
    pods = cl.pods.materialize(plo, phi)
    agg = _shard_aggregates(pods, plo, 7, cl.pod_stage_files).allreduce(dist)
    if rank == 0:
        np.save(result_path, agg.pack())
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_allreduce_of_sharded_aggregates_equals_whole_cluster(tmp_path):
    torch = pytest.importorskip("torch")
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path / "agg.npy")
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    got = np.load(out)
    cl = W.make_cluster("C4", 6, 60, seed=4)
    whole = _shard_aggregates(cl.pods.materialize(), 0, 7, cl.pod_stage_files)
    want = whole.pack()
    n_exact = len(whole.fired_per_stage) + len(whole.counts)
    assert np.array_equal(got[:n_exact], want[:n_exact])  # transitions and phase counts: exact
    np.testing.assert_allclose(got[n_exact:], want[n_exact:], rtol=1e-12)  # usage: reassociated sums
    assert whole.counts[0] > 0 and whole.usage[0] > 0


def test_local_node_ptr():
    ptr = np.array([0, 3, 5, 9, 12])
    assert local_node_ptr(ptr, 1, 3).tolist() == [0, 2, 6]
    assert pod_range(ptr, 1, 3) == (3, 9)


class _FakeEngine:
    """kwk_aggregate's layout without a device: [transitions per stage | counts | usage]."""

    class _P:
        def __init__(self, names):
            self.names = names

    def __init__(self, names, fired, counts, usage):
        self.p = self._P(names)
        self.fired, self.counts, self.usage = fired, counts, usage
        self.buf = None

    def aggregate(self, masks, now_ns=0, usage=False, out_ptr=None):
        assert out_ptr is None and len(masks) == len(self.counts)
        self.buf = np.array(list(self.fired) + list(self.counts) + (list(self.usage) if usage else []), dtype=np.float64)
        return len(self.buf)

    def aggregate_read(self, n):
        return self.buf[:n].copy()


def test_device_report_unpacks_engine_aggregates():
    from kwok_amd.host.cluster import DeviceReport
    pods = _FakeEngine(["pod-ready", "pod-complete"], [7, 3], [10, 6, 1], [1.5, 2048.0])
    nodes = _FakeEngine(["node-initialize"], [2], [2, 2], [0.0, 0.0])
    r = DeviceReport([pods, nodes], [[0, 4, 8], [0, 1]], [["pods", "R", "S"], ["nodes", "N"]], usage_engine=pods)
    with pytest.raises(RuntimeError):
        r.result()
    r.collect(123)
    a = r.result()
    assert a.stage_names == ["pod-ready", "pod-complete", "node-initialize"]
    assert a.fired_per_stage.tolist() == [7, 3, 2]
    assert a.counts.tolist() == [10, 6, 1, 2, 2] and a.count_names == ["pods", "R", "S", "nodes", "N"]
    assert a.usage.tolist() == [1.5, 2048.0]
