"""The N>1 bench path on one GPU: two ranks (torch.distributed, gloo, sharing cuda:0) each own a
node block of the C5-shaped cluster, step their shard engines and all-reduce the reporting
interval's device aggregates (kwk_aggregate -> DeviceReport); the reduced per-stage
transitions and phase histograms must equal the single-rank run of the whole cluster exactly,
and the cluster usage within 1e-9 relative (sums of shard sums)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--steps", "4", "--warmup", "2", "--nodes", "20000", "--no-cpu-baseline", "--no-pmc", "--hbm-nodes", "0",
        "--pcie-steps", "0", "--report-every", "3"]


def _run(cmd):
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.gpu
def test_two_rank_bench_aggregates_equal_one_rank():
    one = _run([sys.executable, "bench.py", "--gpus", "1"] + ARGS)
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", "29571", "bench.py", "--gpus", "2",
                "--dist-backend", "gloo"] + ARGS)
    a1, a2 = one["aggregates"], two["aggregates"]
    assert a1["fired_per_stage"] == a2["fired_per_stage"]
    assert a1["counts"] == a2["counts"]
    for r in ("cpu", "memory"):
        assert a2["usage"][r] == pytest.approx(a1["usage"][r], rel=1e-9)
    assert two["n_gpus"] == 2 and two["config"]["nodes_per_gpu"] == 10000
    assert sum(a1["fired_per_stage"].values()) > 0
