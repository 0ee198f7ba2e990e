"""ORACLE / TEST INFRASTRUCTURE — not product code.

Restatement of pkg/kwok/server/metrics_resource_usage.go for the checker: per-node usage
nodeResourceUsage (:195-224) = sum over the node's pods of sum over containers of
evaluateContainerResourceUsage (:136-168), resolution by getResourceUsage /
findUsageInUsages (:226-264), ObjectSelector.Match (internalversion/object_selector.go:35),
cumulative nodeResourceCumulativeUsage (:67-109).  Quantities go through the oracle's own
C++ ParseQuantity restatement (refcpu rc_quantity); the CEL expression forms evaluated are
the ones kustomize/metrics/usage/usage-from-annotation.yaml uses.
"""
from __future__ import annotations

import ctypes as C
import re

from . import refcpu

_ANN = re.compile(r'"([^"]*)"\s+in\s+pod\.metadata\.annotations\s*\?\s*Quantity\(\s*pod\.metadata\.annotations'
                  r'\[\s*"([^"]*)"\s*\]\s*\)\s*:\s*Quantity\(\s*"([^"]*)"\s*\)')


def quantity(s: str):
    L = refcpu.lib()
    L.rc_quantity.argtypes = [C.c_char_p, C.POINTER(C.c_double)]
    d = C.c_double()
    r = L.rc_quantity(s.encode(), C.byref(d))
    if r == -1:
        raise ValueError(f"quantity {s!r} outside the oracle's range")
    return d.value if r == 1 else None


def _find(container, usages):
    default = None
    for u in usages:
        cs = u.get("containers") or []
        if not cs and default is None:
            default = u
            continue
        if container in cs:
            return u
    return default


def container_usage(docs, pod, container, resource):
    md = pod.get("metadata") or {}
    name, ns = md.get("name", ""), md.get("namespace", "")
    entry = None
    found = False
    for d in docs:
        if d["kind"] == "ResourceUsage" and d["metadata"].get("name") == name and d["metadata"].get("namespace", "") == ns:
            entry, found = _find(container, d["spec"].get("usages") or []), True
            break
    if not found:
        for d in docs:
            if d["kind"] != "ClusterResourceUsage":
                continue
            sel = d["spec"].get("selector")
            if sel is not None:
                if sel.get("matchNamespaces") and ns not in sel["matchNamespaces"]:
                    continue
                if sel.get("matchNames") and name not in sel["matchNames"]:
                    continue
            entry = _find(container, d["spec"].get("usages") or [])
            if entry is not None:
                break
    if entry is None or entry.get("usage") is None:
        return 0.0
    r = entry["usage"].get(resource)
    if r is None:
        return 0.0
    if r.get("value") is not None:
        q = quantity(str(r["value"]))
        return 0.0 if q is None else q
    expr = " ".join((r.get("expression") or "").split())
    m = _ANN.fullmatch(expr)
    if m:
        ann = md.get("annotations") or {}
        q = quantity(str(ann[m.group(1)])) if m.group(1) in ann else quantity(m.group(3))
        return 0.0 if q is None else q
    m = re.fullmatch(r'Quantity\(\s*"([^"]*)"\s*\)', expr)
    if m:
        q = quantity(m.group(1))
        return 0.0 if q is None else q
    raise ValueError(f"oracle: unsupported expression {expr!r}")


def node_usage(docs, pods_of_node, resource):
    s = 0.0
    for pod in pods_of_node:
        for c in (pod.get("spec") or {}).get("containers") or []:
            s += container_usage(docs, pod, c.get("name", ""), resource)
    return s


def seconds(d_ns: int) -> float:
    """time.Duration.Seconds()"""
    sec, nsec = int(d_ns / 10**9), d_ns - int(d_ns / 10**9) * 10**9
    return float(sec) + float(nsec) / 1e9


def pod_usage(docs, pod, resource):
    """podResourceUsage (metrics_resource_usage.go:170-193): the sum over the pod's containers."""
    return node_usage(docs, [pod], resource)


class Cumulative:
    """The cumulative-usage integrators of metrics_resource_usage.go:36-109, keyed like the
    reference's (one per container x resource, one per node): each evaluation adds
    seconds(now - last) * value to the key's total and moves last to now; the first
    evaluation of a key only records the time."""

    def __init__(self):
        self.total = {}
        self.last = {}

    def advance(self, key, value, now_ns):
        t = self.total.get(key, 0.0)
        if key in self.last:
            t += seconds(now_ns - self.last[key]) * value
        self.total[key], self.last[key] = t, now_ns
        return t

    def pod(self, docs, pod, resource, now_ns):
        """podResourceCumulativeUsage (:54-65): the pod's containers' integrators, summed."""
        s = 0.0
        name = (pod.get("metadata") or {}).get("name", "")
        for c in (pod.get("spec") or {}).get("containers") or []:
            cn = c.get("name", "")
            s += self.advance((name, cn, resource), container_usage(docs, pod, cn, resource), now_ns)
        return s
