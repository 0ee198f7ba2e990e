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
Histograms (metrics.go:356-523) are not supported (the shipped Metric CRs have none).
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
    kind: str                # gauge | counter
    help: str = ""
    labels: List[Tuple[str, str]] = field(default_factory=list)   # (name, CEL string expression)
    value: str = "0"


def load_metric_yaml(text: str) -> Tuple[str, List[MetricConfig]]:
    """A Metric document -> (path, configs)."""
    for doc in yaml.safe_load_all(text):
        if doc and doc.get("kind") == "Metric":
            spec = doc.get("spec") or {}
            out = []
            for m in spec.get("metrics") or []:
                if m.get("kind") not in ("gauge", "counter"):
                    raise NotImplementedError(f"metric kind {m.get('kind')!r} (histograms are not supported)")
                out.append(MetricConfig(name=m["name"], dimension=m.get("dimension", "node"), kind=m["kind"],
                                        help=m.get("help", ""), value=m.get("value", "0"),
                                        labels=[(l["name"], l["value"]) for l in m.get("labels") or []]))
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


class MetricsProgram:
    def __init__(self, configs: Sequence[MetricConfig]):
        self.configs = list(configs)
        self.programs = []
        self.host_metrics: List[str] = []
        for m in self.configs:
            try:
                self.programs.append((m.dimension, cel.lower(m.value, m.dimension)))
            except cel.LowerError:
                self.host_metrics.append(m.name)
                self.programs.append((m.dimension, [(cel.OP_CONST, math.nan)]))

    def load(self, pods_engine):
        pods_engine.metrics_load(self.programs)

    def scrape(self, pods_engine, now_ns: int, node_first: int, nodes: Sequence[dict], pods: Sequence[Optional[dict]],
               node_ptr: np.ndarray, started: Optional[Dict[str, float]] = None
               ) -> Dict[str, List[Tuple[Tuple[Tuple[str, str], ...], float]]]:
        """Series of every metric for nodes [node_first, node_first + len(nodes)) (their JSON
        objects) whose pods are `pods` (the JSON objects of pod slots node_ptr[node_first] ..,
        None for dead slots), after kwk_usage(now_ns).  -> {metric name: [(labels, value)]}"""
        n = len(nodes)
        vals = pods_engine.metrics_eval(now_ns, node_first, n)
        p0, p1 = int(node_ptr[node_first]), int(node_ptr[node_first + n])
        counts = pods_engine.usage_containers
        out: Dict[str, List] = {}
        off = 0
        for m in self.configs:
            if m.dimension == "node":
                keys = [(nodes[j], None, None) for j in range(n)]
            else:
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
            series = []
            env = cel.Env(now_ns=now_ns, started_containers_total=lambda name: (started or {}).get(name, 0))
            for i, (node, pod, container) in enumerate(keys):
                if m.dimension != "node" and pod is None:
                    continue  # a dead pod slot: not in ListPods
                v = float(vals[off + i])
                if m.name in self.host_metrics:
                    v = cel.evaluate_float64(m.value, node=node, pod=pod, container=container, env=env)
                labels = tuple((ln, str(cel.evaluate(lv, node=node, pod=pod, container=container)))
                               for ln, lv in m.labels)
                series.append((labels, v))
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
                lines.append(f"{m.name}{{{lab}}} {go_float(v)}" if lab else f"{m.name} {go_float(v)}")
        return "\n".join(lines) + "\n"
