"""ResourceUsage / ClusterResourceUsage compilation (host side of kwk_usage).

Restates the per-container resolution of pkg/kwok/server/metrics_resource_usage.go:
``getResourceUsage`` (:226-250: a namespaced ResourceUsage named like the pod wins, else the
first ClusterResourceUsage whose ObjectSelector matches *and* has an entry for the
container), ``findUsageInUsages`` (:252-264: the entry listing the container, else the first
entry with no containers) and ``evaluateContainerResourceUsage`` (:136-168: a static
``value`` via AsApproximateFloat64, or a CEL ``expression``; any error -> 0).

CEL expressions are compiled for the forms KWOK ships (kustomize/metrics/usage/
usage-from-annotation.yaml): ``"<key>" in pod.metadata.annotations ?
Quantity(pod.metadata.annotations["<key>"]) : Quantity("<default>")`` and
``Quantity("<q>")``; anything else is rejected at compile time.

The device gets, per pod, an interned cpu / memory value and the number of containers that
carry it (``usage_key``); per-node sums and cumulative integrators run in ``usage_kernel``.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import yaml

from .quantity import parse_quantity_or_none


class UsageCompileError(ValueError):
    pass


_ANNOT_FORM = re.compile(
    r'^"(?P<k1>[^"]*)"\s+in\s+pod\.metadata\.annotations\s*\?\s*'
    r'Quantity\(\s*pod\.metadata\.annotations\[\s*"(?P<k2>[^"]*)"\s*\]\s*\)\s*:\s*'
    r'Quantity\(\s*"(?P<d>[^"]*)"\s*\)$')
_CONST_FORM = re.compile(r'^Quantity\(\s*"(?P<q>[^"]*)"\s*\)$')


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
            e = " ".join(self.expression.split())
            m = _ANNOT_FORM.match(e)
            if m and m.group("k1") == m.group("k2"):
                d = parse_quantity_or_none(m.group("d"))
                return ("annot", m.group("k1"), 0.0 if d is None else d)  # CEL error -> 0
            m = _CONST_FORM.match(e)
            if m:
                q = parse_quantity_or_none(m.group("q"))
                return ("const", 0.0 if q is None else q)
            raise UsageCompileError(f"unsupported usage expression: {self.expression!r}")
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

    def container_value(self, pod: dict, container: str, resource: str) -> float:
        """evaluateContainerResourceUsage (:136-168)."""
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
        key, default = c[1], c[2]
        ann = md.get("annotations") or {}
        if key in ann:
            q = parse_quantity_or_none(str(ann[key]))
            return 0.0 if q is None else q
        return default

    def pod_values(self, pod: dict) -> Tuple[float, float, int]:
        """(cpu, memory, containers): per-container value and the container count when every
        container evaluates the same (the common case); else the exact Go-order sum with count 1."""
        names = [c.get("name", "") for c in (pod.get("spec") or {}).get("containers") or []]
        out = []
        for r in self.RESOURCES:
            vals = [self.container_value(pod, n, r) for n in names]
            out.append(vals)
        if not names:
            return 0.0, 0.0, 0
        if all(v == out[0][0] for v in out[0]) and all(v == out[1][0] for v in out[1]) and len(names) < 16:
            return out[0][0], out[1][0], len(names)
        s0 = 0.0
        for v in out[0]:
            s0 += v
        s1 = 0.0
        for v in out[1]:
            s1 += v
        return s0, s1, 1


def usage_columns(program: UsageProgram, pods: Sequence[dict]):
    """-> usage_key u32[n], cpu_values f64[], mem_values f64[] (interned)."""
    cpu_ids: Dict[float, int] = {}
    mem_ids: Dict[float, int] = {}
    keys = np.zeros(len(pods), dtype=np.uint32)
    memo: Dict[int, int] = {}
    for i, p in enumerate(pods):
        c, m, n = program.pod_values(p)
        ci = cpu_ids.setdefault(c, len(cpu_ids))
        mi = mem_ids.setdefault(m, len(mem_ids))
        if ci >= 1 << 14 or mi >= 1 << 14:
            raise UsageCompileError("more than 16384 distinct usage values")
        keys[i] = ci | (mi << 14) | (n << 28)
    cv = np.array(sorted(cpu_ids, key=cpu_ids.get), dtype=np.float64) if cpu_ids else np.zeros(1)
    mv = np.array(sorted(mem_ids, key=mem_ids.get), dtype=np.float64) if mem_ids else np.zeros(1)
    return keys, cv, mv
