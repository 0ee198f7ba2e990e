"""Metric CRD values and per-container usage.

CPU: the product's CEL evaluator on the reference's known answers (evaluator_test.go: 17280,
and 18 for the x10 Quantity quirk) and on the e2e usage expectations (1m / 1Mi, 100m / 100Mi),
which also pin the oracle's usage restatement; every value of the shipped Metric CR lowers
to a device program; Go float formatting of the exposition.
GPU: kwk_usage_read_containers and the device-evaluated Metric CR (kwk_metrics_eval) on a
cluster whose pods' containers evaluate differently, scraped node by node over three
evaluations, against the oracle's restatement (oracle/metrics_ref.py) within 1e-6."""
import json
import os

import numpy as np
import pytest
import yaml

from kwok_amd import workload as W
from kwok_amd.host import cel
from kwok_amd.host.metrics import MetricsProgram, go_float, load_metric_yaml
from kwok_amd.host.usage import UsageProgram, load_usage_yaml, usage_columns

HERE = os.path.dirname(os.path.abspath(__file__))
VEC = json.load(open(os.path.join(HERE, "golden", "cel_vectors.json")))
USAGE = os.path.join(os.path.dirname(HERE), "kwok_amd", "metrics", "usage-from-annotation.yaml")
METRICS = os.path.join(os.path.dirname(HERE), "kwok_amd", "metrics", "metrics-resource.yaml")
REL = 1e-6


def _ns(ts):
    return cel._parse_time(ts)


@pytest.mark.parametrize("case", VEC["cases"], ids=lambda c: c["ref"].split(" ")[0])
def test_cel_known_answers(case):
    env = cel.Env(now_ns=_ns(case["now"]) if "now" in case else None,
                  started_containers_total=(lambda n: case["started_containers_total"])
                  if "started_containers_total" in case else None)
    got = cel.evaluate_float64(case["expr"], node=case.get("node"), pod=case.get("pod"), env=env)
    assert got == case["want"]


@pytest.mark.parametrize("case", VEC["e2e_usage"], ids=lambda c: c["ref"])
def test_e2e_usage_values_product_and_oracle(case):
    from oracle import usage_ref
    text = open(USAGE).read()
    docs = [d for d in yaml.safe_load_all(text) if d]
    prog = UsageProgram(*load_usage_yaml(text))
    pod = W.pod_object("pod-0", "node-0", annotations=case["annotations"])
    for r in ("cpu", "memory"):
        assert prog.container_value(pod, "container-0", r) == case[r]
        assert usage_ref.container_usage(docs, pod, "container-0", r) == case[r]


def test_cel_semantics():
    ev = cel.evaluate
    assert ev("1 + 2 * 3") == 7 and ev("7 / 2") == 3 and ev("-7 / 2") == -3 and ev("-7 % 2") == -1
    assert ev("1.0 / 4.0") == 0.25 and ev("2 == 2.0") is True and ev("'a' + 'b'") == "ab"
    for bad in ("1 + 1.0", "9223372036854775807 + 1", "1 / 0", "{'a': 1}['b']", "Quantity('1') + 1"):
        with pytest.raises(cel.CELError):
            ev(bad)
    assert ev("false && (1 / 0 == 1)") is False and ev("true || (1 / 0 == 1)") is True
    assert ev("'k' in pod.metadata.annotations ? 1 : 2", pod={"metadata": {"annotations": {"k": "v"}}}) == 1
    assert ev("size(pod.spec.containers)", pod={"spec": {"containers": [{}, {}]}}) == 2
    assert cel.as_float64(ev("Quantity('1Mi')")) == 1048576.0
    assert cel.as_float64(ev("Quantity('100m') * 3")) == pytest.approx(0.3)
    assert ev("node.status.allocatable['memory']", node={}) == cel.Quantity.nano(0)  # ResourceList.Get: zero


def test_shipped_metric_values_lower_to_device_programs():
    _, configs = load_metric_yaml(open(METRICS).read())
    mp = MetricsProgram(configs)
    assert len(configs) == 8 and mp.host_metrics == []


def test_go_float_format():
    cases = {0.0: "0", 1.0: "1", 1e6: "1e+06", 123456.0: "123456", 1234567.0: "1.234567e+06", 1e-5: "1e-05",
             0.0001: "0.0001", 1048576.0: "1.048576e+06", -2.5: "-2.5", float("nan"): "NaN", float("inf"): "+Inf"}
    for v, want in cases.items():
        assert go_float(v) == want, v


def _mixed_cluster():
    cl = W.make_cluster("C4", 8, 200, seed=51)
    pods = cl.pods.materialize()
    extra = []
    for i, p in enumerate(pods):
        if i % 2 == 0:
            p["metadata"]["creationTimestamp"] = "2023-11-14T00:00:%02dZ" % (i % 60)
        if i % 4 == 1:  # a namespaced ResourceUsage named like the pod: containers evaluate differently
            extra.append({"apiVersion": "kwok.x-k8s.io/v1alpha1", "kind": "ResourceUsage",
                          "metadata": {"name": p["metadata"]["name"], "namespace": "default"},
                          "spec": {"usages": [{"containers": ["container-1"],
                                               "usage": {"cpu": {"value": "300m"}, "memory": {"value": "32Mi"}}},
                                              {"usage": {"cpu": {"value": "2"},
                                                         "memory": {"expression": 'Quantity("1Gi")'}}}]}})
    text = open(USAGE).read() + "\n---\n" + yaml.safe_dump_all(extra)
    return cl, pods, text


def test_mixed_containers_get_mixed_entries():
    cl, pods, text = _mixed_cluster()
    keys, cv, mv, mixed, ckeys = usage_columns(UsageProgram(*load_usage_yaml(text)), pods)
    n_mixed = int(np.count_nonzero((keys >> 28) == 0))
    assert n_mixed > 0 and len(mixed) // 2 >= 1 and len(ckeys) >= 2


@pytest.mark.gpu
@pytest.mark.parametrize("compiler", ["native", "python"])
def test_gpu_container_usage_and_metric_scrape(compiler):
    from kwok_amd.host.compiler import KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files
    from oracle import usage_ref
    from oracle.metrics_ref import MetricsOracle
    cl, pods, text = _mixed_cluster()
    docs = [d for d in yaml.safe_load_all(text) if d]
    cols = usage_columns(UsageProgram(*load_usage_yaml(text)), pods)
    kp = KindProgram(load_stage_files(*cl.pod_stage_files))
    kp.explore(pods)
    ing = Ingest(kp)
    eng = Engine(kp, capacity=len(pods))
    nodes = cl.nodes.materialize()
    try:
        eng.load_stages()
        eng.load(*ing.columns(pods), ing.record_array())
        eng.usage_config(cl.node_ptr, *cols)
        eng.usage_pods(True)
        text_cr = open(METRICS).read()
        mp = MetricsProgram.from_native(text_cr) if compiler == "native" else MetricsProgram(load_metric_yaml(text_cr)[1])
        mp.load(eng)
        created = np.array([_ns(p["metadata"]["creationTimestamp"]) if "creationTimestamp" in p["metadata"]
                            else np.iinfo(np.int64).min for p in pods], dtype=np.int64)
        zero_unix = float(cel.wrap_int64(cel.GO_ZERO_TIME.ns)) / 1e9
        eng.metrics_inputs(created, np.full(len(nodes), np.iinfo(np.int64).min, dtype=np.int64),
                           np.zeros(len(nodes)), zero_unix)
        oracle = MetricsOracle(docs)
        cum = usage_ref.Cumulative()
        alive = np.ones(len(pods), dtype=bool)
        t = 1_700_000_000 * 10**9
        for k in range(3):
            if k == 1:
                gone = np.arange(3, len(pods), 11)
                eng.delete(gone)
                alive[gone] = False
            eng.usage(t)
            # per-container usage (containerResourceUsage / containerResourceCumulativeUsage)
            got = eng.usage_read_containers(0, len(pods))
            want = []
            for i, p in enumerate(pods):
                for c in p["spec"]["containers"]:
                    n = c["name"]
                    if alive[i]:
                        cpu = usage_ref.container_usage(docs, p, n, "cpu")
                        mem = usage_ref.container_usage(docs, p, n, "memory")
                        want.append((cpu, mem, cum.advance((i, n, "cpu"), cpu, t), cum.advance((i, n, "mem"), mem, t)))
                    else:
                        want.append((0.0, 0.0, 0.0, 0.0))
            np.testing.assert_allclose(got, np.array(want), rtol=REL, atol=1e-9, err_msg=f"evaluation {k}")
            # the Metric CR, node by node
            for j in range(len(nodes)):
                lo, hi = int(cl.node_ptr[j]), int(cl.node_ptr[j + 1])
                slots = [pods[i] if alive[i] else None for i in range(lo, hi)]
                dev = mp.scrape(eng, t, j, [nodes[j]], slots, cl.node_ptr)
                exp = oracle.scrape(t, nodes[j], [p for p in slots if p is not None],
                                    lambda p: _ns(p["metadata"]["creationTimestamp"])
                                    if "creationTimestamp" in p["metadata"] else None)
                for name, series in exp.items():
                    d = dict(dev[name])
                    assert set(d) == {lab for lab, _ in series}, (name, j)
                    for lab, v in series:
                        assert d[lab] == pytest.approx(v, rel=REL, abs=1e-9), (name, lab, k)
            text_out = mp.exposition(dev)
            assert "# TYPE container_cpu_usage_seconds_total counter" in text_out
            t += 2_500_000_000 + 123_457 * k
    finally:
        eng.close()


HIST_YAML = """
kind: Metric
apiVersion: kwok.x-k8s.io/v1alpha1
metadata:
  name: histograms
spec:
  path: /metrics/nodes/{nodeName}/metrics/histograms
  metrics:
  - name: pod_memory_mib
    help: pod memory in MiB as bucket counts
    kind: histogram
    dimension: pod
    labels:
    - name: pod
      value: pod.metadata.name
    buckets:
    - le: 1
      value: pod.Usage("memory") / 1048576.0
    - le: 0.5
      hidden: true
      value: "2.5"
    - le: 10
      value: pod.Usage("cpu") * 1000.0
    - le: 1
      value: "3.0"
    - le: 100
      value: pod.Usage("cpu") * -5.0
  - name: node_cpu_hist
    help: node histogram, the last bucket below a hidden one
    kind: histogram
    dimension: node
    buckets:
    - le: 2
      hidden: true
      value: "1.0"
    - le: 1
      value: node.Usage("memory") / 1048576.0
    - le: 3
      hidden: true
      value: "7.9"
  - name: container_cpu_milli
    kind: histogram
    dimension: container
    labels:
    - name: container
      value: container.name
    - name: pod
      value: pod.metadata.name
    buckets:
    - le: 0.25
      value: pod.Usage("cpu", container.name) * 1000.0
    - le: 0.5
      value: pod.Usage("memory", container.name) / 1048576.0
"""


def _hist_expected(name, pod, node_mem, docs, container=None):
    """The bucket values of HIST_YAML restated by hand (oracle usage callbacks), per metric."""
    from oracle import usage_ref
    if name == "pod_memory_mib":
        mem = sum(usage_ref.container_usage(docs, pod, c["name"], "memory") for c in pod["spec"]["containers"])
        cpu = sum(usage_ref.container_usage(docs, pod, c["name"], "cpu") for c in pod["spec"]["containers"])
        return [(1.0, False), (0.5, True), (10.0, False), (1.0, False), (100.0, False)], \
            [mem / 1048576.0, 2.5, cpu * 1000.0, 3.0, cpu * -5.0]
    if name == "node_cpu_hist":
        return [(2.0, True), (1.0, False), (3.0, True)], [1.0, node_mem / 1048576.0, 7.9]  # node memory (exact sum)
    cpu = usage_ref.container_usage(docs, pod, container, "cpu")
    mem = usage_ref.container_usage(docs, pod, container, "memory")
    return [(0.25, False), (0.5, False)], [cpu * 1000.0, mem / 1048576.0]


def test_histogram_write_host_form_equals_oracle():
    """The host fallback of histogram Set + Write and the float64 -> uint64 conversion against
    the oracle's restatement (histogram.go:107-164, Go's amd64 conversion), on edge values:
    duplicate le (last Set wins), hidden buckets, keys above every visible bound, negative / NaN
    / huge values (wrapping uint64 counts)."""
    from kwok_amd.host.metrics import go_uint64, histogram_write
    from oracle.metrics_ref import go_float64_to_uint64, histogram_series
    for x in (0.0, -0.0, 0.99, 1.5, -0.5, -1.5, -1e300, 2.0**63 - 1024, 2.0**63, 2.0**64, 1e300, float("nan"),
              float("inf"), float("-inf"), 12345.678):
        assert go_uint64(x) == go_float64_to_uint64(x), x
    rng = np.random.default_rng(7)
    for trial in range(300):
        n = int(rng.integers(1, 7))
        les = [float(rng.choice([0.1, 0.5, 1.0, 2.0, 5.0, 10.0])) for _ in range(n)]
        hidden = [bool(rng.random() < 0.3) for _ in range(n)]
        vals = [float(rng.choice([0.0, 1.0, 2.7, 100.0, -3.0, 7e18, 1.9e19])) for _ in range(n)]
        host = histogram_write(list(zip(les, hidden)), [go_uint64(v) for v in vals])
        bounds, counts, count, total = histogram_series(list(zip(les, hidden)), vals)
        assert host["bounds"] == bounds and host["counts"] == counts and host["count"] == count, trial
        assert host["sum"] == total, trial


def test_histogram_metric_yaml_lowers():
    _, configs = load_metric_yaml(HIST_YAML)
    mp = MetricsProgram(configs)
    assert [c.kind for c in configs] == ["histogram"] * 3 and mp.host_metrics == []
    assert len(mp.hist_programs) == 3 and len(mp.hist_programs[0][1]) == 5


@pytest.mark.gpu
@pytest.mark.parametrize("compiler", ["native", "python"])
def test_gpu_histogram_metrics_scrape(compiler):
    """Histogram Metric CRs evaluated on the device (kwk_histograms_eval) against the oracle's
    restatement of updateHistogram + histogram.Write (oracle/metrics_ref.py), node by node over
    two evaluations with dead pods: bucket counts, sample counts exactly; sample sums within
    1e-6 relative (north_star's tolerance for usage-derived floats)."""
    from kwok_amd.host.compiler import KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files
    from oracle import usage_ref
    from oracle.metrics_ref import histogram_series
    cl, pods, text = _mixed_cluster()
    docs = [d for d in yaml.safe_load_all(text) if d]
    cols = usage_columns(UsageProgram(*load_usage_yaml(text)), pods)
    kp = KindProgram(load_stage_files(*cl.pod_stage_files))
    kp.explore(pods)
    ing = Ingest(kp)
    eng = Engine(kp, capacity=len(pods))
    nodes = cl.nodes.materialize()
    try:
        eng.load_stages()
        eng.load(*ing.columns(pods), ing.record_array())
        eng.usage_config(cl.node_ptr, *cols)
        eng.usage_pods(True)
        mp = MetricsProgram.from_native(HIST_YAML) if compiler == "native" else MetricsProgram(load_metric_yaml(HIST_YAML)[1])
        mp.load(eng)
        alive = np.ones(len(pods), dtype=bool)
        t = 1_700_000_000 * 10**9
        checked = 0
        for k in range(2):
            if k == 1:
                gone = np.arange(2, len(pods), 7)
                eng.delete(gone)
                alive[gone] = False
            eng.usage(t)
            for j in range(len(nodes)):
                lo, hi = int(cl.node_ptr[j]), int(cl.node_ptr[j + 1])
                slots = [pods[i] if alive[i] else None for i in range(lo, hi)]
                dev = mp.scrape(eng, t, j, [nodes[j]], slots, cl.node_ptr)
                live = [p for p in slots if p is not None]
                node_mem = sum(usage_ref.container_usage(docs, p, c["name"], "memory")
                               for p in live for c in p["spec"]["containers"])
                want = {"node_cpu_hist": [((), _hist_expected("node_cpu_hist", None, node_mem, docs))],
                        "pod_memory_mib": [((("pod", p["metadata"]["name"]),), _hist_expected("pod_memory_mib", p, 0, docs))
                                           for p in live],
                        "container_cpu_milli": [((("container", c["name"]), ("pod", p["metadata"]["name"])),
                                                 _hist_expected("container_cpu_milli", p, 0, docs, c["name"]))
                                                for p in live for c in p["spec"]["containers"]]}
                for name, series in want.items():
                    d = dict(dev[name])
                    assert set(d) == {lab for lab, _ in series}, (name, j)
                    for lab, (bks, vals) in series:
                        bounds, counts, count, total = histogram_series(bks, vals)
                        got = d[lab]
                        assert got["bounds"] == bounds and got["counts"] == counts and got["count"] == count, \
                            (name, lab, k, got, counts)
                        assert got["sum"] == pytest.approx(total, rel=REL, abs=1e-9), (name, lab, k)
                        checked += 1
            out = mp.exposition(dev)
            assert "# TYPE pod_memory_mib histogram" in out and 'le="+Inf"' in out
            t += 3_000_000_000
        assert checked > 500
    finally:
        eng.close()
