"""Metric CRs (kustomize/metrics/resource/metrics-resource.yaml) on the engine: per-series
values evaluated on the device, Prometheus text exposition on the host.

Reference: pkg/kwok/metrics/metrics.go — UpdateHandler.Update (:525-571) evaluates, per node
scrape, every MetricConfig of the Metric CR: gauges / counters per node (one series), per pod
of the node (ListPods) or per container of those pods (:168-354), each value a CEL
expression (evaluator.go) turned into float64; labels are CEL string expressions; the
registry is served by promhttp (pkg/kwok/server/metrics.go:129-150).

Here every value is lowered once (cel.lower) into a device program; ``scrape`` runs
kwk_usage + kwk_metrics_eval for a node range and formats the series.  A value with no device
form (it reads object fields the engine does not keep) is evaluated by the host CEL evaluator
per series, with the same usage callbacks answered from the engine's outputs — explicit and
reported in ``MetricsProgram.host_metrics``, never a silent substitute for the device path.
Histograms (metrics.go:133-160,356-462; histogram.go:81-164): every bucket's value is lowered
the same way and kwk_histograms_eval returns, per series, the bucket counts histogram.Write
would expose (cumulative counts of the visible bounds, +Inf, sample count and sum).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import yaml

from . import cel


@dataclass
class MetricConfig:
    name: str
    dimension: str           # node | pod | container
    kind: str                # gauge | counter | histogram
    help: str = ""
    labels: List[Tuple[str, str]] = field(default_factory=list)   # (name, CEL string expression)
    value: str = "0"
    buckets: List[Tuple[float, str, bool]] = field(default_factory=list)  # histogram: (le, CEL value, hidden)


def load_metric_yaml(text: str) -> Tuple[str, List[MetricConfig]]:
    """A Metric document -> (path, configs)."""
    for doc in yaml.safe_load_all(text):
        if doc and doc.get("kind") == "Metric":
            spec = doc.get("spec") or {}
            out = []
            for m in spec.get("metrics") or []:
                if m.get("kind") not in ("gauge", "counter", "histogram"):
                    raise ValueError(f"unknown metric kind {m.get('kind')!r}")
                buckets = [(float(b.get("le", 0)), b.get("value", "0"), bool(b.get("hidden", False)))
                           for b in m.get("buckets") or []]
                if m["kind"] == "histogram" and not buckets:
                    raise ValueError(f"histogram {m['name']!r} has no buckets")
                out.append(MetricConfig(name=m["name"], dimension=m.get("dimension", "node"), kind=m["kind"],
                                        help=m.get("help", ""), value=m.get("value", "0"),
                                        labels=[(l["name"], l["value"]) for l in m.get("labels") or []],
                                        buckets=buckets))
            return spec.get("path", ""), out
    raise ValueError("no Metric document")


def go_float(v: float) -> str:
    """strconv.FormatFloat(v, 'g', -1, 64), as the Prometheus text encoder writes values:
    shortest round-trip digits, %e when the decimal exponent is < -4 or >= 6 (strconv/ftoa.go:
    'shortest' sets eprec = 6), exponent with at least two digits."""
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "+Inf" if v > 0 else "-Inf"
    if v == 0:
        return "-0" if math.copysign(1.0, v) < 0 else "0"
    neg = v < 0
    e = f"{abs(v):.17e}".partition("e")[2]  # the decimal exponent; the shortest digits from repr
    digits = repr(abs(v)).split("e")[0].replace(".", "").lstrip("0").rstrip("0") or "0"
    exp = int(e)
    if exp < -4 or exp >= 6:
        out = digits[0] + ("." + digits[1:] if len(digits) > 1 else "") + f"e{'-' if exp < 0 else '+'}{abs(exp):02d}"
    elif exp >= 0:
        ip = digits[:exp + 1].ljust(exp + 1, "0")
        fp = digits[exp + 1:]
        out = ip + ("." + fp if fp else "")
    else:
        out = "0." + "0" * (-exp - 1) + digits
    return ("-" if neg else "") + out


def _escape_label(v: str) -> str:
    return v.replace("\\", "\\\\").replace("\n", "\\n").replace('"', '\\"')


def _escape_help(v: str) -> str:
    return v.replace("\\", "\\\\").replace("\n", "\\n")


def go_uint64(x: float) -> int:
    """Go's uint64(float64) on amd64 (the compiler's float64ToUint64 lowering: CVTTSD2SQ below
    2^63, else CVTTSD2SQ(x - 2^63) | 1 << 63; out-of-range / NaN truncations give 1 << 63)."""
    def cvtt(v):
        if not (-9223372036854775808.0 < v < 9223372036854775808.0):
            return 1 << 63
        return int(v) & 0xFFFFFFFFFFFFFFFF
    if x < 9223372036854775808.0:
        return cvtt(x)
    return cvtt(x - 9223372036854775808.0) | (1 << 63)


def _go_sort_key(v: float):
    return (0, 0.0) if math.isnan(v) else (1, v)  # sort.Float64s: NaN first


def histogram_write(buckets: Sequence[Tuple[float, bool]], values: Sequence[int]) -> dict:
    """Host form of histogram Set + Write (histogram.go:118-164) for one series: buckets
    [(le, hidden)] in CR order with their uint64 values -> {"bounds", "counts" (visible bounds
    then +Inf), "count", "sum"} (the host-evaluated fallback; the device computes the same)."""
    stored: Dict[float, int] = {}
    for (le, _), v in zip(buckets, values):
        stored[le] = v
    bounds = sorted((le for le, hidden in buckets if not hidden), key=_go_sort_key)
    counts = [0] * (len(bounds) + 1)
    bi, count, total = 0, 0, 0.0
    for le in sorted(stored, key=_go_sort_key):
        while bi < len(bounds) and le > bounds[bi]:
            bi += 1
            counts[bi] += count
        counts[bi] += stored[le]
        count += stored[le]
        total += le * float(stored[le])
    return {"bounds": bounds, "counts": [c & 0xFFFFFFFFFFFFFFFF for c in counts], "count": count & 0xFFFFFFFFFFFFFFFF,
            "sum": total}


def load_metric_doc(text: str) -> dict:
    """The Metric document of a YAML text (what the Go host has decoded and hands the native
    compiler as JSON)."""
    for doc in yaml.safe_load_all(text):
        if doc and doc.get("kind") == "Metric":
            return doc
    raise ValueError("no Metric document")


class MetricsProgram:
    def __init__(self, configs: Sequence[MetricConfig], native=None):
        """native: a native_metrics.NativeMetricSet compiled from the same CR: the device programs
        come from libkwok_compiler (kwk_compile_metrics) instead of cel.lower, and so does the list
        of host-evaluated metrics."""
        self.configs = list(configs)
        self.programs = []          # gauges / counters, in config order
        self.hist_programs = []     # histograms, in config order: (dimension, [(le, hidden, program)])
        self.host_metrics: List[str] = []
        self.native = native
        if native is not None:
            self.host_metrics = list(native.host_metrics)
            self.hist_programs = [(m.dimension, None) for m in self.configs if m.kind == "histogram"]
            return
        for m in self.configs:
            if m.kind == "histogram":
                try:
                    self.hist_programs.append((m.dimension, [(le, hidden, cel.lower(v, m.dimension))
                                                             for le, v, hidden in m.buckets]))
                except cel.LowerError:
                    self.host_metrics.append(m.name)
                    self.hist_programs.append((m.dimension, [(le, hidden, [(cel.OP_CONST, 0.0)])
                                                             for le, _, hidden in m.buckets]))
                continue
            try:
                self.programs.append((m.dimension, cel.lower(m.value, m.dimension)))
            except cel.LowerError:
                self.host_metrics.append(m.name)
                self.programs.append((m.dimension, [(cel.OP_CONST, math.nan)]))

    @classmethod
    def from_native(cls, text: str) -> "MetricsProgram":
        """The Metric CR of a YAML text compiled by the native compiler (kwk_compile_metrics)."""
        from .native_metrics import NativeMetricSet
        _, configs = load_metric_yaml(text)
        return cls(configs, native=NativeMetricSet(load_metric_doc(text)))

    def load(self, pods_engine):
        if self.native is not None:
            self.native.load(pods_engine)
            return
        pods_engine.metrics_load(self.programs)
        if self.hist_programs:
            pods_engine.histograms_load(self.hist_programs)

    @staticmethod
    def _series_keys(m: MetricConfig, nodes, pods, node_ptr, node_first, counts):
        n = len(nodes)
        if m.dimension == "node":
            return [(nodes[j], None, None) for j in range(n)]
        p0, p1 = int(node_ptr[node_first]), int(node_ptr[node_first + n])
        keys = []
        for p in range(p0, p1):
            node = nodes[int(np.searchsorted(node_ptr, p, side="right")) - 1 - node_first]
            pod = pods[p - p0]
            if m.dimension == "pod":
                keys.append((node, pod, None))
                continue
            cs = ((pod or {}).get("spec") or {}).get("containers") or []
            for j in range(int(counts[p])):
                keys.append((node, pod, cs[j] if j < len(cs) else {}))
        return keys

    def scrape(self, pods_engine, now_ns: int, node_first: int, nodes: Sequence[dict], pods: Sequence[Optional[dict]],
               node_ptr: np.ndarray, started: Optional[Dict[str, float]] = None
               ) -> Dict[str, List[Tuple[Tuple[Tuple[str, str], ...], float]]]:
        """Series of every metric for nodes [node_first, node_first + len(nodes)) (their JSON
        objects) whose pods are `pods` (the JSON objects of pod slots node_ptr[node_first] ..,
        None for dead slots), after kwk_usage(now_ns).  -> {metric name: [(labels, value)]}"""
        n = len(nodes)
        vals = pods_engine.metrics_eval(now_ns, node_first, n)
        hvals = pods_engine.histograms_eval(now_ns, node_first, n) if self.hist_programs else None
        counts = pods_engine.usage_containers
        out: Dict[str, List] = {}
        off = hoff = 0
        env = cel.Env(now_ns=now_ns, started_containers_total=lambda name: (started or {}).get(name, 0))
        for m in self.configs:
            keys = self._series_keys(m, nodes, pods, node_ptr, node_first, counts)
            series = []
            words = sum(1 for _, _, hidden in m.buckets if not hidden) + 3
            for i, (node, pod, container) in enumerate(keys):
                if m.dimension != "node" and pod is None:
                    continue  # a dead pod slot: not in ListPods
                if m.kind == "histogram":
                    if m.name in self.host_metrics:
                        vs = [go_uint64(cel.evaluate_float64(v, node=node, pod=pod, container=container, env=env))
                              for _, v, _ in m.buckets]
                        v = histogram_write([(le, h) for le, _, h in m.buckets], vs)
                    else:
                        rec = hvals[hoff + i * words:hoff + (i + 1) * words]
                        bounds = sorted((le for le, _, h in m.buckets if not h), key=_go_sort_key)
                        v = {"bounds": bounds, "counts": [int(x) for x in rec[:words - 2]], "count": int(rec[words - 2]),
                             "sum": float(rec[words - 1:words].view(np.float64)[0])}
                else:
                    v = float(vals[off + i])
                    if m.name in self.host_metrics:
                        v = cel.evaluate_float64(m.value, node=node, pod=pod, container=container, env=env)
                labels = tuple((ln, str(cel.evaluate(lv, node=node, pod=pod, container=container)))
                               for ln, lv in m.labels)
                series.append((labels, v))
            if m.kind == "histogram":
                hoff += len(keys) * words
            else:
                off += len(keys)
            out[m.name] = series
        return out

    def exposition(self, series: Dict[str, List]) -> str:
        """Prometheus text format 0.0.4 (families sorted by name, series by label values, as
        client_golang's Gather)."""
        lines = []
        for m in sorted(self.configs, key=lambda c: c.name):
            lines.append(f"# HELP {m.name} {_escape_help(m.help.rstrip(chr(10)))}")
            lines.append(f"# TYPE {m.name} {m.kind}")
            for labels, v in sorted(series.get(m.name, []), key=lambda s: [x[1] for x in s[0]]):
                lab = ",".join(f'{k}="{_escape_label(x)}"' for k, x in labels)
                if m.kind == "histogram":  # expfmt text_create.go: _bucket{le}, _sum, _count
                    pre = lab + "," if lab else ""
                    for le, c in zip(list(v["bounds"]) + [math.inf], v["counts"]):
                        lines.append(f'{m.name}_bucket{{{pre}le="{go_float(le)}"}} {go_float(float(c))}')
                    lines.append(f"{m.name}_sum{{{lab}}} {go_float(v['sum'])}" if lab else f"{m.name}_sum {go_float(v['sum'])}")
                    lines.append(f"{m.name}_count{{{lab}}} {go_float(float(v['count']))}" if lab
                                 else f"{m.name}_count {go_float(float(v['count']))}")
                    continue
                lines.append(f"{m.name}{{{lab}}} {go_float(v)}" if lab else f"{m.name} {go_float(v)}")
        return "\n".join(lines) + "\n"
