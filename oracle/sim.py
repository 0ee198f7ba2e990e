"""ORACLE / TEST INFRASTRUCTURE — not product code.

Reference-semantics cluster simulation on JSON objects, used to check the HIP engine
step by step.  Per object and step it does exactly what the reference controllers do
between watch events, in the engine's documented order:

  harness churn  (bench/parity workload: re-create deleted objects, delete terminal ones)
  match + delay  refcpu (C++ restatement of lifecycle.Match / Stage.Delay, with the Philox hook)
                 on objects that changed since their last match (informer Modified event)
  schedule       one pending job per object; a match replaces it, no match keeps it
                 (pod_controller.go:222-229, addStageJob :660-671)
  fire           due <= now: playStage's effect — finalizers JSON patch, delete, the status
                 merge patch (oracle/next_ref.py: the oracle's own restatement of the shipped
                 templates, pinned on the reference's golden outputs); an object whose
                 patches changed it is re-matched next step (its Modified event)

Stages are v1alpha1 Stage documents (the YAML kwok loads); nothing here imports the product.
"""
from __future__ import annotations

import copy
from typing import List, Optional, Sequence

from . import labels_ref, refcpu
from .next_ref import Funcs, StageNext, format_rfc3339nano, omitempty, strip_for_recreate

INT64_MAX = (1 << 63) - 1
INT64_MIN = -(1 << 63)


def sat_add(a: int, b: int) -> int:
    return max(INT64_MIN, min(INT64_MAX, a + b))


class OracleSim:
    def __init__(self, stage_docs: Sequence[dict], objs: Sequence[dict], harness: bool = False,
                 terminal=("Succeeded", "Failed"), slot_base: int = 0, kind_salt: int = 0,
                 slots: Optional[Sequence[int]] = None, disregard=None):
        """slots: the engine slot of each object (default: objs[i] is slot i).  Objects are
        independent within a step (a pod reads only its own fields; its node's lease state comes
        in through set_managed) and the Philox counter is the global slot, so a deterministic
        sample of a large engine's slots is simulated exactly by passing their slot numbers.
        disregard: (annotation selector, label selector) of need() (pod_controller.go:397-407): a
        changed object they disregard is not re-matched (its event is skipped; a queued job stays)."""
        self.disregard = disregard
        # NewLifecycle drops stages with a nil selector (lifecycle.go:199-201)
        docs = [d for d in stage_docs if (d.get("spec") or {}).get("selector") is not None]
        self.lc = refcpu.Lifecycle(list(stage_docs))
        assert self.lc.names == [d["metadata"]["name"] for d in docs]
        self.stages = [StageNext(d, self.lc, i) for i, d in enumerate(docs)]
        self.names = self.lc.names
        self.objs: List[Optional[dict]] = [omitempty(copy.deepcopy(o)) for o in objs]
        self.orig = [copy.deepcopy(o) for o in self.objs]
        n = len(objs)
        self.dirty = [True] * n
        self.pending: List[Optional[int]] = [None] * n
        self.due = [0] * n
        self.gen = [0] * n
        self.matcherr = [False] * n
        self.managed = [True] * n   # readOnlyFunc: objects on nodes whose lease is not held are skipped
        self.harness = harness
        self.terminal = set(terminal)
        self.slot_base = slot_base
        self.kind_salt = kind_salt
        self.slots = list(range(n)) if slots is None else [int(x) for x in slots]
        assert len(self.slots) == n

    def _is_terminal(self, o) -> bool:
        ph = refcpu.query(".status.phase", o) or []
        return any(p in self.terminal for p in ph if isinstance(p, str))

    def step(self, now_ns: int, seed: int, step: int):
        key = seed ^ (self.kind_salt << 32)
        F = Funcs(now_ns)
        fired = []
        for i in range(len(self.objs)):
            if not self.managed[i]:  # read-only (watchResources skips it, controller.go:285-288)
                continue
            o = self.objs[i]
            if self.harness:
                if o is None:
                    o = self.objs[i] = strip_for_recreate(self.orig[i])
                    self.gen[i] += 1
                    self.dirty[i] = True
                    self.pending[i] = None
                elif self._is_terminal(o) and "deletionTimestamp" not in o.get("metadata", {}):
                    sec = now_ns // 10**9
                    o.setdefault("metadata", {})["deletionTimestamp"] = format_rfc3339nano(sec * 10**9)
                    self.dirty[i] = True
            if o is None:
                continue
            if self.dirty[i] and self.disregard is not None and labels_ref.disregarded(*self.disregard, o):
                self.dirty[i] = False  # watchResources: need() is false, the event is skipped
            if self.dirty[i]:
                self.dirty[i] = False
                self.matcherr[i] = False
                s, d = self.lc.match(o, now_ns, key, step, self.slot_base + self.slots[i])
                if s == -2:
                    self.matcherr[i] = True
                elif s is not None:
                    self.pending[i] = s
                    self.due[i] = sat_add(now_ns, d)
            s = self.pending[i]
            if s is not None and self.due[i] <= now_ns:
                self.pending[i] = None
                o2, changed = self.stages[s].apply(o, F)
                flags = 0
                if o2 is None:
                    flags |= 1
                    self.objs[i] = None
                else:
                    self.objs[i] = o2
                    if changed:
                        self.dirty[i] = True
                        flags |= 2
                fired.append((self.slots[i], s, flags))
        return fired

    def set_managed(self, i: int, held: bool, resync: bool):
        """Lease sync outcome for object i: MANAGED = Held(); a successful sync re-sends the
        object to preprocess (ManageNode / podsOnNodeSyncWorker), which re-matches it unless a
        job for its current version is queued (pod_controller.go:205-214)."""
        self.managed[i] = held
        if held and resync and self.pending[i] is None and self.objs[i] is not None:
            self.dirty[i] = True

    def deletion_s(self, i: int) -> int:
        o = self.objs[i]
        if o is None:
            return INT64_MIN
        ts = (o.get("metadata") or {}).get("deletionTimestamp")
        if not ts:
            return INT64_MIN
        return refcpu.parse_rfc3339(ts)[0]


def oracle_pred(desc: dict, obj: dict) -> int:
    """Feature bits of a JSON object computed with the oracle's own jq (refcpu), from the
    compiled feature table (KindProgram.describe(): data, the query text and bit of each
    feature)."""
    pred = 0
    for f in desc["features"]:
        lits = list(f["literals"].items())
        m = refcpu.feature(f["query"], obj, [v for v, _ in lits])  # hasValue: strings, bools, gojq ints
        if not m & 1:
            continue
        if f["present_bit"] is not None:
            pred |= 1 << f["present_bit"]
        for i, (_, b) in enumerate(lits):
            if m >> (i + 1) & 1:
                pred |= 1 << b
    if desc["finalizer_other_bit"] is not None:
        for x in (obj.get("metadata") or {}).get("finalizers") or []:
            b = desc["finalizers"].get(x)
            pred |= 1 << (desc["finalizer_other_bit"] if b is None else b)
    dg = desc.get("disregard")
    if dg and labels_ref.disregarded(dg["annotation_selector"], dg["label_selector"], obj):
        pred |= 1 << dg["bit"]
    return pred
