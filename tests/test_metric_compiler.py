"""The native Metric CR compiler (include/kwok_metrics.h, libkwok_compiler: kwk_compile_metrics,
kwk_cel_lower) against the host's Python lowering (kwok_amd/host/cel.py lower through
metrics.MetricsProgram), on the CPU.

* The packed device programs — kwk_metric_desc / kwk_metric_op for gauges and counters,
  kwk_histogram_desc / kwk_metric_bucket / kwk_metric_op for histograms — are byte-equal to the
  arrays the Python host packs for kwk_metrics_load / kwk_histograms_load, on the shipped Metric CR
  (kustomize/metrics/resource/metrics-resource.yaml), the histogram CRs of tests/test_metrics.py,
  the reference-vector CR of tests/test_metric_vectors.py (histogram_test.go / gauge_test.go /
  counter_test.go) and a CR whose values have no device form (host metrics, same list and same
  placeholders).
* Expression by expression (kwk_cel_lower vs cel.lower), over every dimension: the same program
  bit for bit, or both "no device form", or both a compile error — on hand-picked cases (CEL's
  typing: no int <-> double arithmetic, overflow, the Quantity x double x10 rule of
  evaluator_test.go:95-117, error-absorbing && / ||) and 4000 generated expressions.
Reference: pkg/kwok/metrics/metrics.go:168-462, evaluator.go:51-144,201-233,
pkg/utils/cel/environment.go:98-138.  cel-go itself is not under /root/reference: the Python
restatement pinned by evaluator_test.go (tests/golden/cel_vectors.json) is the check."""
from __future__ import annotations

import json
import os
import random
import struct

import pytest
import yaml

from kwok_amd.host import cel
from kwok_amd.host.engine import pack_histogram_programs, pack_metric_programs
from kwok_amd.host.metrics import MetricsProgram, load_metric_doc, load_metric_yaml
from kwok_amd.host.native_metrics import MetricCompileError, NativeMetricSet, cel_lower

HERE = os.path.dirname(os.path.abspath(__file__))
METRICS = os.path.join(os.path.dirname(HERE), "kwok_amd", "metrics", "metrics-resource.yaml")

HOST_CR = """
kind: Metric
apiVersion: kwok.x-k8s.io/v1alpha1
metadata: {name: host}
spec:
  path: /metrics/nodes/{nodeName}/metrics/host
  metrics:
  - name: by_field
    kind: gauge
    dimension: pod
    value: 'pod.spec.priority * 1.0'
  - name: mixed_types
    kind: counter
    dimension: node
    value: 'node.Usage("cpu") + 1'
  - name: quantity_const
    kind: gauge
    value: 'Quantity("100m") * 3'
  - name: device_ok
    kind: gauge
    dimension: container
    value: 'pod.Usage("cpu", container.name) * 1000.0 - (2.0 - pod.SinceSecond()) / -4.0'
  - name: hist_host
    kind: histogram
    dimension: pod
    buckets:
    - le: 1
      value: pod.Usage("cpu") * 2.0
    - le: 2
      value: 'pod.Usage("cpu") > 1.0 ? 1.0 : 0.0'
  - name: hist_default_dim
    kind: histogram
    buckets:
    - {le: 0.5, value: 'node.Usage("memory") / 1048576.0', hidden: true}
    - {le: 0.25, value: '7'}
    - {le: 3, value: 'UnixSecond(Now()) - node.metadata.creationTimestamp.UnixSecond()'}
"""


def _crs():
    from tests.test_metric_vectors import _metric_yaml
    from tests.test_metrics import HIST_YAML
    return {"metrics-resource": open(METRICS).read(), "histograms": HIST_YAML, "vectors": _metric_yaml(),
            "host": HOST_CR}


@pytest.mark.parametrize("name", ["metrics-resource", "histograms", "vectors", "host"])
def test_native_programs_byte_equal_to_python(name):
    text = _crs()[name]
    _, configs = load_metric_yaml(text)
    py = MetricsProgram(configs)
    nat = NativeMetricSet(load_metric_doc(text))
    try:
        assert nat.host_metrics == py.host_metrics
        n, descs, n_ops, ops = pack_metric_programs(py.programs)
        want = (bytes(descs)[:n * 16], bytes(ops)[:n_ops * 16])
        assert nat.programs_bytes() == want
        h = pack_histogram_programs(py.hist_programs)
        want_h = (bytes(h[1])[:h[0] * 16], bytes(h[3])[:h[2] * 24], bytes(h[5])[:h[4] * 16])
        assert nat.histograms_bytes() == want_h
        d = nat.describe
        assert [m["name"] for m in d["metrics"]] == [c.name for c in configs]
        assert [m["kind"] for m in d["metrics"]] == [c.kind for c in configs]
        assert [m["device"] for m in d["metrics"]] == [c.name not in py.host_metrics for c in configs]
        assert [[(l["name"], l["value"]) for l in m["labels"]] for m in d["metrics"]] == [c.labels for c in configs]
    finally:
        nat.close()


def test_shipped_and_vector_crs_have_no_host_metrics():
    for name in ("metrics-resource", "histograms", "vectors"):
        nat = NativeMetricSet(load_metric_doc(_crs()[name]))
        assert nat.host_metrics == [], name
        nat.close()
    nat = NativeMetricSet(load_metric_doc(HOST_CR))
    assert nat.host_metrics == ["by_field", "mixed_types", "hist_host"]
    reasons = {m["name"]: m["reason"] for m in nat.describe["metrics"]}
    assert reasons["device_ok"] == "" and reasons["by_field"] and reasons["hist_host"]
    nat.close()


@pytest.mark.parametrize("bad,why", [
    ({"kind": "Metric", "spec": {"metrics": [{"name": "x", "kind": "summary", "value": "1.0"}]}}, "kind"),
    ({"kind": "Metric", "spec": {"metrics": [{"name": "x", "kind": "gauge", "dimension": "cluster"}]}}, "dimension"),
    ({"kind": "Metric", "spec": {"metrics": [{"name": "x", "kind": "histogram"}]}}, "buckets"),
    ({"kind": "Metric", "spec": {"metrics": [{"name": "x", "kind": "gauge", "value": "1 +"}]}}, "syntax"),
    ({"kind": "Metric", "spec": {"metrics": [{"name": "x", "kind": "gauge", "value": "1 / 0"}]}}, "evaluation"),
    ({"kind": "Metric", "spec": {"metrics": [{"name": "x", "kind": "gauge", "value": "'text'"}]}}, "evaluation"),
    ({"kind": "Metric", "spec": {"metrics": [{"kind": "gauge", "value": "1.0"}]}}, "name"),
    ({"kind": "Stage", "spec": {}}, "kind"),
])
def test_compile_errors(bad, why):
    with pytest.raises(MetricCompileError, match=why):
        NativeMetricSet(bad)


def _py_outcome(expr, dim):
    try:
        return ("ok", cel.lower(expr, dim))
    except cel.LowerError:
        return ("lower", None)
    except Exception:  # noqa: BLE001 - CEL / syntax / Python evaluation errors alike: the CR does not compile
        return ("error", None)


def _native_outcome(expr, dim):
    try:
        return ("ok", cel_lower(expr, dim))
    except cel.LowerError:
        return ("lower", None)
    except MetricCompileError:
        return ("error", None)


def _bits(prog):
    return [(op, struct.pack("<d", float(x)) if op == cel.OP_CONST else x) for op, x in prog]


def _same(expr, dim):
    a, b = _py_outcome(expr, dim), _native_outcome(expr, dim)
    assert a[0] == b[0], (expr, dim, a, b)
    if a[0] == "ok":
        assert _bits(a[1]) == _bits(b[1]), (expr, dim, a[1], b[1])
    return a[0]


CASES = [
    # device forms
    'pod.Usage("cpu")', 'pod.Usage("memory", container.name)', 'node.CumulativeUsage("cpu")',
    'pod.CumulativeUsage("memory", container.name) / 1048576.0', 'node.Usage("memory") * 2.5 + 1.0',
    '-pod.Usage("cpu")', '-(pod.Usage("cpu") - -3.0)', 'pod.SinceSecond()', 'SinceSecond(node)', 'SinceSecond(pod)',
    'node.StartedContainersTotal()', 'node.startedContainersTotal()', 'Now().UnixSecond()', 'UnixSecond(now())',
    'UnixSecond(pod.metadata.creationTimestamp)', 'node.metadata.creationTimestamp.UnixSecond()',
    'UnixSecond(Now()) - UnixSecond(node.metadata.creationTimestamp)',
    # constants folded with CEL's semantics
    '1.0', '1', '7u', '-9223372036854775808', '9223372036854775807', '0x10', '-0x10', '1e3', '.5', '2.', '1e400',
    'true', 'false', '3 + 4 * 2', '7 / 2', '-7 / 2', '-7 % 2', '7u - 8u', '9223372036854775807 + 1', '1 / 0',
    '2.0 / 0.0', '-2.0 / 0.0', '0.0 / 0.0', '1 + 1.0', 'double(3) / 2.0', 'int(2.9)', 'int(-2.9)', 'int(1e19)',
    'double("1.5")', 'double(" 2 ")', 'double("x")', 'string(12)', 'size("héllo")', 'size([1, 2, 3])',
    'size({"a": 1})', '[1, 2, 3][1]', '[1, 2][2]', '{"a": 1.5}["a"]', '{"a": 1}.a', '{"a": 1}["b"]',
    '1 == 1.0', '1 == 1u', 'true == 1', '1 < 2.0', '"a" < "b"', '1 in [1.0, 2]', '"x" in {"x": 1}',
    'true ? 1.5 : 2.5', '1 ? 2.0 : 3.0', 'false && (1 / 0 == 1)', 'true || (1 / 0 == 1)', '(1 / 0 == 1) || true',
    '(1 / 0 == 1) && true', '!false', '!1',
    'Quantity("1Mi")', 'Quantity("100m") * 3', 'Quantity("100m") * 3.0', 'Quantity("1.5Gi") / 2',
    'Quantity("1") + Quantity("500m")', 'Quantity("1") - Quantity("2k")', 'Quantity("1") + 1',
    'Quantity("1") > Quantity("999m") ? 1.0 : 0.0', 'Quantity("bad")', 'Quantity("")', 'Quantity("-.e-10")',
    'Quantity("e5")', 'Quantity("1e3") * 1.5', 'Quantity("1.5n")', 'Quantity("0.1Ki")', 'double(Quantity("2Gi"))',
    '-Quantity("3")', 'Quantity("5") == Quantity("5000m")', '"1Mi".Quantity()',
    # mixed: no device form / errors
    'pod.Usage("cpu") + 1', 'pod.Usage("cpu") * 2', 'pod.Usage("cpu") + Quantity("1")', 'pod.Usage(1)',
    'pod.Usage("gpu")', 'container.Usage("cpu")', 'pod.Usage("cpu", "c0")', 'node.Usage("cpu", container.name)',
    'pod.spec.priority', 'pod.metadata.name', 'Rand()', 'Rand() * 2.0', 'pod.Usage("cpu") > 1.0 ? 1.0 : 0.0',
    'pod.Usage("cpu") + (1 / 0)', '(1 / 0) + pod.Usage("cpu")', 'pod.Usage("cpu") + 1 / 0',
    'UnixSecond(pod.status.startTime)', 'container.SinceSecond()', 'double(pod.Usage("cpu"))',
    # syntax
    '', '1 +', '(1', 'a.', '"unterminated', '1 ? 2', '[1, 2', '{"a": 1', '@', '1 = 2', 'a & b', '99999999999999999999',
    '18446744073709551616u', '-1u', '{1: 1.0, 1.0: 2.0}[1]', '{true: 1.0, 1: 2.0}[1]', '{[1]: 2.0}', '"\\q"', 'r"raw\\n"', "'single'", '"a" + "b"', '[1] + [2.0]',
]


@pytest.mark.parametrize("dim", ["node", "pod", "container", "cluster"])
def test_lower_cases_native_equals_python(dim):
    kinds = {_same(e, dim) for e in CASES}
    assert kinds == {"ok", "lower", "error"}


_DYN = ['pod.Usage("cpu")', 'pod.Usage("memory")', 'node.Usage("cpu")', 'node.CumulativeUsage("memory")',
        'pod.CumulativeUsage("cpu")', 'pod.Usage("cpu", container.name)', 'pod.CumulativeUsage("memory", container.name)',
        'pod.SinceSecond()', 'SinceSecond(node)', 'node.StartedContainersTotal()', 'Now().UnixSecond()',
        'UnixSecond(pod.metadata.creationTimestamp)', 'node.metadata.creationTimestamp.UnixSecond()',
        'container.Usage("cpu")', 'pod.spec.priority', 'Rand()']
_CONST = ['1.0', '2.5', '0.0', '-3.75', '1e300', '1e-300', '.5', '3', '-4', '0', '9223372036854775807', '2u', '0u',
          'true', 'false', '"s"', 'null', 'Quantity("1Mi")', 'Quantity("100m")', 'Quantity("1.5Gi")', 'Quantity("2")',
          'Quantity("3e2")', '[1, 2.0]', '{"k": 2.0}', '1048576.0', '1000.0']


def _gen(rng, depth):
    r = rng.random()
    if depth <= 0 or r < 0.3:
        return rng.choice(_DYN) if rng.random() < 0.5 else rng.choice(_CONST)
    a, b = _gen(rng, depth - 1), _gen(rng, depth - 1)
    form = rng.randrange(22)
    if form < 8:
        return f"({a} {rng.choice('+-*/')} {b})"
    if form < 10:
        return f"-({a})"
    if form == 10:
        return f"({a} % {b})"
    if form == 11:
        return f"({a} {rng.choice(['==', '!=', '<', '<=', '>', '>='])} {b}) ? {a} : {b}"
    if form == 12:
        return f"double({a})"
    if form == 13:
        return f"int({a})"
    if form == 14:
        return f"({a} in [{b}, {a}])"
    if form == 15:
        return f"({a} {rng.choice(['&&', '||'])} {b}) ? 1.0 : 2.0"
    if form == 16:
        return f"[{a}, {b}][{rng.choice(['0', '1', '2', '1u', '1.0'])}]"
    if form == 17:
        return f"size([{a}, {b}])"
    if form == 18:
        return f"string({a})"
    if form == 19:
        return f"{{\"x\": {a}}}.x"
    if form == 20:
        return f"({a}) * double({rng.choice(['1', '2u', '0.5', chr(34) + '3' + chr(34)])})"
    return f"{a} - {b}"


def test_lower_generated_native_equals_python():
    rng = random.Random(20261018)
    counts = {"ok": 0, "lower": 0, "error": 0}
    for i in range(4000):
        expr = _gen(rng, rng.randrange(1, 5))
        counts[_same(expr, ("node", "pod", "container")[i % 3])] += 1
    assert min(counts.values()) > 200, counts


def test_metric_json_round_trip_of_shipped_cr():
    """The Go host hands the decoded CR as JSON: YAML -> JSON -> native == YAML -> Python."""
    doc = load_metric_doc(open(METRICS).read())
    nat = NativeMetricSet(json.loads(json.dumps(doc)))
    py = MetricsProgram(load_metric_yaml(yaml.safe_dump(doc))[1])
    n, descs, n_ops, ops = pack_metric_programs(py.programs)
    assert nat.programs_bytes() == (bytes(descs)[:n * 16], bytes(ops)[:n_ops * 16])
    nat.close()
