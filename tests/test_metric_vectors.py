"""The metric oracle and the product pinned to the reference's own metric unit tests
(tests/golden/metric_vectors.json, transcribed from pkg/kwok/metrics/{histogram,gauge,counter}_test.go).

* histogram_test.go:29-96 — buckets {0.5, 1, 2.5, 5, 10}, six Set(le, count) calls, cumulative
  counts 0 / 3 / 15 / 15 / 31 / 63, SampleCount 63, SampleSum: checked against the oracle's
  restatement (oracle/metrics_ref.histogram_series), the host form (metrics.histogram_write) and,
  on the GPU, a Metric CR whose bucket values are those counts, evaluated by kwk_histograms_eval.
  A Metric CR calls Set for every bucket (metrics.go:380-390) and exposes the non-hidden les as
  bounds (metrics.go:143-149), so the six pairs are hidden buckets listed after the five visible
  bounds (value 0): an equal le set later wins (SyncMap.Store, histogram.go:161-164), and the
  zero-count keys add nothing to any count or to the sum.
* gauge_test.go:25-74 / counter_test.go:25-65 — the exposition lines after Set(42) / Set(84):
  a node-dimension gauge / counter CR with those constant values through kwk_metrics_eval and the
  host's text exposition.
"""
from __future__ import annotations

import json
import os

import numpy as np
import pytest
import yaml

from kwok_amd.host.metrics import MetricsProgram, go_uint64, histogram_write, load_metric_yaml

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "metric_vectors.json")))


def _cr_buckets():
    """(le, CEL value, hidden) in CR order reproducing histogram_test.go's Set calls."""
    h = GOLD["histogram"]
    vis = [(float(le), "0", False) for le in h["buckets"]]
    return vis + [(float(le), str(c), True) for le, c in h["set"]]


def _want():
    h = GOLD["histogram"]
    total = 0.0
    for le, c in sorted(h["want_sample_sum_ascending"]):  # Write's ascending-le accumulation
        total += float(le) * float(c)
    return h["want_bounds"], h["want_cumulative"], h["want_sample_count"], total


def test_histogram_reference_vector_oracle_and_host():
    from oracle.metrics_ref import histogram_series
    bounds, cum, count, total = _want()
    bks = _cr_buckets()
    b, c, n, s = histogram_series([(le, hid) for le, _, hid in bks], [float(v) for _, v, _ in bks])
    assert b == bounds and c == cum and n == count and s == total
    host = histogram_write([(le, hid) for le, _, hid in bks], [go_uint64(float(v)) for _, v, _ in bks])
    assert host["bounds"] == bounds and host["counts"] == cum and host["count"] == count and host["sum"] == total
    # the direct form of the reference test: Set only the six pairs (no zero-count bounds stored)
    pairs = [(float(le), False if float(le) in GOLD["histogram"]["buckets"] else True) for le, _ in
             GOLD["histogram"]["set"]]
    # bounds 0.5 / 2.5 / 5 are not Set there: they still bound (hidden=False, value 0 adds nothing)
    direct = [(0.5, False), (2.5, False), (5.0, False)] + pairs
    host2 = histogram_write(direct, [0, 0, 0] + [c for _, c in GOLD["histogram"]["set"]])
    assert host2["counts"] == cum and host2["count"] == count


def _metric_yaml() -> str:
    g, c = GOLD["gauge"], GOLD["counter"]
    hist = [{"le": le, "value": v, "hidden": hid} for le, v, hid in _cr_buckets()]
    doc = {"kind": "Metric", "apiVersion": "kwok.x-k8s.io/v1alpha1", "metadata": {"name": "vectors"},
           "spec": {"path": "/metrics/nodes/{nodeName}/metrics/vectors", "metrics": [
               {"name": g["name"], "help": g["help"], "kind": "gauge", "dimension": "node",
                "value": str(g["steps"][-1][1])},
               {"name": c["name"], "help": c["help"], "kind": "counter", "dimension": "node",
                "value": str(c["steps"][-1][1])},
               {"name": "name", "help": "help", "kind": "histogram", "dimension": "node", "buckets": hist}]}}
    return yaml.safe_dump(doc)


def test_vector_metric_cr_lowers_to_device_programs():
    _, configs = load_metric_yaml(_metric_yaml())
    mp = MetricsProgram(configs)
    assert mp.host_metrics == [] and len(mp.programs) == 2 and len(mp.hist_programs) == 1


def test_gauge_counter_exposition_matches_reference_text():
    """The host exposition of the gauge / counter series (values as the device returns them)
    equals the reference test's expected text after each Set."""
    _, configs = load_metric_yaml(_metric_yaml())
    mp = MetricsProgram([m for m in configs if m.kind != "histogram"])
    for step in GOLD["gauge"]["steps"] + GOLD["counter"]["steps"]:
        v = float(step[1])
        out = mp.exposition({GOLD["gauge"]["name"]: [((), v)], GOLD["counter"]["name"]: [((), v)]})
        for key in ("counter", "gauge"):
            want = "\n".join(GOLD[key]["want_exposition"]).replace("{value}", str(step[1]))
            assert want in out, (key, step, out)


@pytest.mark.gpu
@pytest.mark.parametrize("compiler", ["native", "python"])
def test_gpu_metric_cr_reference_vectors(compiler):
    """The gauge / counter / histogram CR above through kwk_metrics_eval / kwk_histograms_eval on
    every node of a small cluster: histogram bounds, cumulative counts and sample count exactly as
    histogram_test.go, the sum equal to Write's ascending accumulation; gauge and counter series
    exposed exactly as gauge_test.go / counter_test.go expect after their last Set.  The device
    programs come from the native Metric CR compiler (kwk_compile_metrics, the Go host's path) or
    from the Python lowering."""
    from kwok_amd import workload as W
    from kwok_amd.host.compiler import KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files
    from kwok_amd.host.usage import UsageProgram, load_usage_yaml, usage_columns
    cl = W.make_cluster("C4", 4, 40, seed=3)
    pods = cl.pods.materialize()
    nodes = cl.nodes.materialize()
    text = open(os.path.join(W.METRICS_DIR, "usage-from-annotation.yaml")).read()
    cols = usage_columns(UsageProgram(*load_usage_yaml(text)), pods)
    kp = KindProgram(load_stage_files(*cl.pod_stage_files))
    kp.explore(pods)
    ing = Ingest(kp)
    eng = Engine(kp, capacity=len(pods))
    bounds, cum, count, total = _want()
    try:
        eng.load_stages()
        eng.load(*ing.columns(pods), ing.record_array())
        eng.usage_config(cl.node_ptr, *cols)
        eng.usage_pods(True)
        if compiler == "native":
            mp = MetricsProgram.from_native(_metric_yaml())
            assert mp.native is not None
        else:
            mp = MetricsProgram(load_metric_yaml(_metric_yaml())[1])
        assert mp.host_metrics == []
        mp.load(eng)
        eng.metrics_inputs(np.full(len(pods), np.iinfo(np.int64).min, dtype=np.int64),
                           np.full(len(nodes), np.iinfo(np.int64).min, dtype=np.int64), np.zeros(len(nodes)), 0.0)
        t = 1_700_000_000 * 10**9
        eng.usage(t)
        for j in range(len(nodes)):
            lo, hi = int(cl.node_ptr[j]), int(cl.node_ptr[j + 1])
            dev = mp.scrape(eng, t, j, [nodes[j]], pods[lo:hi], cl.node_ptr)
            (lab, h), = dev["name"]
            assert lab == () and h["bounds"] == bounds and h["counts"] == cum and h["count"] == count, (j, h)
            assert h["sum"] == total, (j, h["sum"], total)
            out = mp.exposition(dev)
            for key in ("gauge", "counter"):
                want = "\n".join(GOLD[key]["want_exposition"]).replace("{value}", str(GOLD[key]["steps"][-1][1]))
                assert want in out, (key, out)
            assert 'name_bucket{le="+Inf"} 63' in out and "name_count 63" in out
    finally:
        eng.close()
