"""ResourceUsage / ClusterResourceUsage compilation (host side of kwk_usage).

Restates the per-container resolution of pkg/kwok/server/metrics_resource_usage.go:
``getResourceUsage`` (:226-250: a namespaced ResourceUsage named like the pod wins, else the
first ClusterResourceUsage whose ObjectSelector matches *and* has an entry for the
container), ``findUsageInUsages`` (:252-264: the entry listing the container, else the first
entry with no containers) and ``evaluateContainerResourceUsage`` (:136-168: a static
``value`` via AsApproximateFloat64, or a CEL ``expression`` evaluated with the pod, its node
and the container bound — kwok_amd/host/cel.py; any error -> 0).

Usage expressions are evaluated once per pod variant at ingest, so they must not depend on
the clock or on other usages (``Now``, ``Rand``, ``SinceSecond``, ``Usage``, ...): such an
expression is rejected at compile time rather than frozen.  The device gets, per pod, either
one interned cpu / memory value and the number of containers that carry it, or — when the
pod's containers differ — a {first, count} entry into a per-container key table
(``kwk_usage_mixed``); per-node sums and all cumulative integrators run in ``usage_kernel``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import yaml

from . import cel
from .quantity import parse_quantity_or_none


class UsageCompileError(ValueError):
    pass


_CLOCKED = ("Now", "now", "Rand", "SinceSecond", "Usage", "CumulativeUsage", "StartedContainersTotal",
            "startedContainersTotal")


def _reads_clock(ast) -> bool:
    if not isinstance(ast, tuple):
        return False
    if ast[0] in ("call", "method") and ast[1 if ast[0] == "call" else 2] in _CLOCKED:
        return True
    for x in ast[1:]:
        if isinstance(x, tuple) and _reads_clock(x):
            return True
        if isinstance(x, list) and any(_reads_clock(y) if isinstance(y, tuple) and isinstance(y[0], str)
                                       else any(_reads_clock(z) for z in y) for y in x):
            return True
    return False


@dataclass
class UsageValue:
    value: Optional[str] = None        # resource.Quantity text
    expression: Optional[str] = None

    def compile(self):
        if self.value is not None:
            q = parse_quantity_or_none(str(self.value))
            if q is None:
                raise UsageCompileError(f"invalid quantity {self.value!r}")
            return ("const", q)
        if self.expression is not None:
            try:
                ast = cel.compile(self.expression)
            except cel.CELSyntaxError:
                return ("const", 0.0)  # Compile fails -> 0 (metrics_resource_usage.go:150-155)
            if _reads_clock(ast):
                raise UsageCompileError(f"usage expression depends on the clock / other usages: {self.expression!r}")
            return ("cel", self.expression)
        return ("const", 0.0)


@dataclass
class UsageEntry:
    containers: List[str]
    usage: Optional[Dict[str, UsageValue]]


@dataclass
class ResourceUsage:
    name: str
    namespace: str
    usages: List[UsageEntry]


@dataclass
class ClusterResourceUsage:
    name: str
    match_namespaces: List[str] = field(default_factory=list)
    match_names: List[str] = field(default_factory=list)
    usages: List[UsageEntry] = field(default_factory=list)
    has_selector: bool = False

    def match(self, name: str, namespace: str) -> bool:
        """ObjectSelector.Match (internalversion/object_selector.go:35-47)."""
        if not self.has_selector:
            return True
        if self.match_namespaces and namespace not in self.match_namespaces:
            return False
        if self.match_names and name not in self.match_names:
            return False
        return True


def _entries(spec) -> List[UsageEntry]:
    out = []
    for u in spec.get("usages") or []:
        usage = None
        if u.get("usage") is not None:
            usage = {k: UsageValue(value=None if v.get("value") is None else str(v.get("value")),
                                   expression=v.get("expression")) for k, v in u["usage"].items()}
        out.append(UsageEntry(containers=list(u.get("containers") or []), usage=usage))
    return out


def load_usage_yaml(*texts: str):
    rus, crus = [], []
    for t in texts:
        for doc in yaml.safe_load_all(t):
            if not doc:
                continue
            md = doc.get("metadata") or {}
            spec = doc.get("spec") or {}
            if doc.get("kind") == "ResourceUsage":
                rus.append(ResourceUsage(md.get("name", ""), md.get("namespace", ""), _entries(spec)))
            elif doc.get("kind") == "ClusterResourceUsage":
                sel = spec.get("selector")
                crus.append(ClusterResourceUsage(md.get("name", ""),
                                                 list((sel or {}).get("matchNamespaces") or []),
                                                 list((sel or {}).get("matchNames") or []), _entries(spec),
                                                 has_selector=sel is not None))
    return rus, crus


def find_usage(container: str, usages: List[UsageEntry]) -> Optional[UsageEntry]:
    """findUsageInUsages (metrics_resource_usage.go:252-264)."""
    default = None
    for u in usages:
        if len(u.containers) == 0 and default is None:
            default = u
            continue
        if container in u.containers:
            return u
    return default


class UsageProgram:
    RESOURCES = ("cpu", "memory")

    def __init__(self, resource_usages: Sequence[ResourceUsage], cluster_resource_usages: Sequence[ClusterResourceUsage]):
        self.rus = list(resource_usages)
        self.crus = list(cluster_resource_usages)
        self._compiled = {}
        for group in [r.usages for r in self.rus] + [c.usages for c in self.crus]:
            for e in group:
                for k, v in (e.usage or {}).items():
                    self._compiled[id(v)] = v.compile()

    def _entry(self, pod_name: str, ns: str, container: str) -> Optional[UsageEntry]:
        for r in self.rus:  # getResourceUsage (:226-250)
            if r.name == pod_name and r.namespace == ns:
                return find_usage(container, r.usages)
        for c in self.crus:
            if not c.match(pod_name, ns):
                continue
            u = find_usage(container, c.usages)
            if u is not None:
                return u
        return None

    def container_value(self, pod: dict, container: str, resource: str, node: Optional[dict] = None) -> float:
        """evaluateContainerResourceUsage (:136-168) for the container named `container` (the
        first with that name, as containerResourceUsage's slices.Find, :111-134)."""
        md = pod.get("metadata") or {}
        u = self._entry(md.get("name", ""), md.get("namespace", ""), container)
        if u is None or u.usage is None:
            return 0.0
        v = u.usage.get(resource)
        if v is None:
            return 0.0
        c = self._compiled[id(v)]
        if c[0] == "const":
            return c[1]
        cobj = next((x for x in (pod.get("spec") or {}).get("containers") or [] if x.get("name", "") == container), {})
        try:
            return cel.evaluate_float64(c[1], node=node or {}, pod=pod, container=cobj)
        except cel.CELError:
            return 0.0

    def pod_container_values(self, pod: dict, node: Optional[dict] = None) -> List[Tuple[float, float]]:
        """(cpu, memory) of each of the pod's containers, in spec order."""
        names = [c.get("name", "") for c in (pod.get("spec") or {}).get("containers") or []]
        return [(self.container_value(pod, n, "cpu", node), self.container_value(pod, n, "memory", node)) for n in names]


def usage_columns(program: UsageProgram, pods: Sequence[dict], nodes: Optional[Dict[str, dict]] = None):
    """-> usage_key u32[n], cpu_values f64[], mem_values f64[] (interned), and the mixed tables
    (kwk_usage_mixed): mixed u32[2 * n_mixed] = {first, count}, ckeys u32[n_containers].
    A pod whose containers all evaluate alike (1..15 of them) is one key x its container count;
    any other pod (containers differ, none, or more than 15) gets a mixed entry."""
    cpu_ids: Dict[float, int] = {}
    mem_ids: Dict[float, int] = {}
    keys = np.zeros(len(pods), dtype=np.uint32)
    mixed: List[int] = []
    ckeys: List[int] = []
    memo: Dict[tuple, int] = {}

    def vid(c, m):
        ci = cpu_ids.setdefault(c, len(cpu_ids))
        mi = mem_ids.setdefault(m, len(mem_ids))
        if ci >= 1 << 14 or mi >= 1 << 14:
            raise UsageCompileError("more than 16384 distinct usage values")
        return ci | (mi << 14)

    for i, p in enumerate(pods):
        node = (nodes or {}).get((p.get("spec") or {}).get("nodeName", ""))
        vals = program.pod_container_values(p, node)
        if 1 <= len(vals) <= 15 and all(v == vals[0] for v in vals):
            keys[i] = vid(*vals[0]) | (len(vals) << 28)
            continue
        t = tuple(vals)
        m = memo.get(t)
        if m is None:
            m = memo[t] = len(mixed) // 2
            mixed += [len(ckeys), len(vals)]
            ckeys += [vid(c, mm) for c, mm in vals]
        keys[i] = m
    cv = np.array(sorted(cpu_ids, key=cpu_ids.get), dtype=np.float64) if cpu_ids else np.zeros(1)
    mv = np.array(sorted(mem_ids, key=mem_ids.get), dtype=np.float64) if mem_ids else np.zeros(1)
    return keys, cv, mv, np.array(mixed, dtype=np.uint32), np.array(ckeys, dtype=np.uint32)
