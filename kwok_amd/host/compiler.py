"""Stage compiler: one resource kind's Stage list -> the device stage table.

What ``lifecycle.NewLifecycle``/``NewStage`` build in Go (lifecycle.go:33-46,194-267) —
label/annotation selectors, gojq requirements, weight and delay getters, ``next`` — is
compiled here into integer form the sweep kernel evaluates without strings:

* **Feature bits** (the ``pred`` word).  Every distinct selector query gets a *present*
  bit if some requirement uses Exists/DoesNotExist on it, and one bit per literal that any
  In/NotIn names.  A requirement then becomes a bit test (A4 in SURVEY.md §8):
  Exists = present, DoesNotExist = !present, In = (pred & lits) != 0, NotIn = its negation.
  ``matchLabels``/``matchAnnotations`` entries are In-tests on ``.metadata.labels["k"]``.
  A jq runtime error yields no output, i.e. all bits 0, which gives the reference's
  nil-result outcomes (selector.go:72-78).  ``.metadata.finalizers`` is modelled as a *set*
  of interned values (+1 "other" bit) so ``finalizersModify`` becomes bit algebra.
* **Value slots** for ``weightFrom``/``durationFrom``/``jitterDurationFrom``: the host
  pre-parses each object's query result once (Go ParseInt / ParseDuration / RFC3339 rules,
  goparse.py) into a 16-byte record entry; ``.metadata.deletionTimestamp`` durations read
  a device column instead (the harness can set it on device).
* **Next-state deltas**: for every object *class* (spec shape) and stage, the effect of
  the stage's rendered patch on the feature bits, as ``pred' = (pred & and) | or``.  They
  are derived by exploring the reachable states of one representative per (class, start
  state) with the gotpl mirror (render -> merge patch -> re-extract features) and are
  checked for consistency; anything not derivable is marked UNKNOWN and round-trips to the
  host (fired flag KWK_FIRED_DELTA_UNKNOWN).
"""
from __future__ import annotations

import copy
import json
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from . import abi
from .goparse import f64_to_i64, parse_duration, parse_int, parse_rfc3339nano
from .gotpl import Renderer, rfc3339nano
from .jq import Query, has_value
from .nextstate import apply_next, merge_patch, json_patch, prune_empty, render_patches
from .typed import typed_presence
from .stages import Stage

FIN_QUERIES = {".metadata.finalizers", ".metadata.finalizers.[]", ".metadata.finalizers[]"}
DELETION_QUERY = ".metadata.deletionTimestamp"


class CompileError(ValueError):
    pass


_NORM = re.compile(r'"(?:[^"\\]|\\.)*"|\s+')


def _norm(src: str) -> str:
    """The query without whitespace outside its string literals (the feature / slot key)."""
    return _NORM.sub(lambda m: m.group(0) if m.group(0).startswith('"') else "", src)


_SEG = re.compile(r'\.(?:([A-Za-z_][A-Za-z0-9_]*)|\[\s*"((?:[^"\\]|\\.)*)"\s*\]|"((?:[^"\\]|\\.)*)")')


def path_prefix(src: str) -> List[str]:
    """Leading static path of a query (`.a.b["c"]` ...) before any iteration / pipe."""
    out, i, s = [], 0, src.strip()
    while i < len(s):
        m = _SEG.match(s, i)
        if not m:
            break
        out.append(m.group(1) or json.loads('"%s"' % (m.group(2) if m.group(2) is not None else m.group(3))))
        i = m.end()
    return out


@dataclass
class Feature:
    src: str
    query: Query
    present_bit: Optional[int] = None
    lit_bits: Dict[str, int] = field(default_factory=dict)

    def mask(self) -> int:
        m = 0 if self.present_bit is None else 1 << self.present_bit
        for b in self.lit_bits.values():
            m |= 1 << b
        return m


@dataclass
class HarnessSpec:
    """Device-side churn used by bench / parity runs (include/kwok_engine.h kwk_harness)."""
    terminal_query: str = ".status.phase"
    terminal_values: Tuple[str, ...] = ("Succeeded", "Failed")
    deletion_query: str = DELETION_QUERY


def strip_for_recreate(obj: dict) -> dict:
    """The harness re-creates a deleted object from its original spec: no status, no
    deletionTimestamp, no finalizers."""
    o = copy.deepcopy(obj)
    o.pop("status", None)
    md = o.setdefault("metadata", {})
    for k in ("deletionTimestamp", "deletionGracePeriodSeconds", "finalizers"):
        md.pop(k, None)
    return o


_IDENTITY_META = ("name", "generateName", "namespace", "uid", "resourceVersion", "creationTimestamp", "generation",
                  "managedFields", "deletionTimestamp", "deletionGracePeriodSeconds", "finalizers", "labels",
                  "annotations", "selfLink")


def class_key(obj: dict) -> str:
    """Object class for next-state deltas: the spec shape, with per-object identity
    (names, node name, owner names/uids, labels/annotations) and all dynamic state removed;
    of the typed presence, so that spellings of the same typed object share a class."""
    o = copy.deepcopy(typed_presence(obj))
    o.pop("status", None)
    md = o.get("metadata") or {}
    for k in _IDENTITY_META:
        md.pop(k, None)
    if "ownerReferences" in md:
        md["ownerReferences"] = sorted(r.get("kind", "") for r in md["ownerReferences"] or [])
    spec = o.get("spec")
    if isinstance(spec, dict):
        spec.pop("nodeName", None)
        spec.pop("hostname", None)
    return json.dumps(o, sort_keys=True, separators=(",", ":"))


def exploration_funcs():
    """Deterministic stand-ins for the controller-provided template funcs
    (pod_controller.go / node_controller.go funcMaps)."""
    return {
        "NodeIP": lambda: "10.0.0.1",
        "NodeName": lambda: "node",
        "NodePort": lambda: 10250,
        "PodIP": lambda: "10.0.0.2",
        "NodeIPWith": lambda *a: "10.0.0.1",
        "PodIPWith": lambda *a: "10.0.0.2",
    }


class KindProgram:
    """Compiled Stage set for one resourceRef (one engine)."""

    def __init__(self, stages: Sequence[Stage], harness: Optional[HarnessSpec] = None, disregard=None):
        """disregard: a labelsel.DisregardSpec (the kwok configuration's
        disregardStatusWith{Annotation,Label}Selector): need()'s result becomes one feature bit, and
        a changed object with it set is not re-matched (kwk_stage_table.disregard_mask)."""
        # NewLifecycle drops stages with a nil selector (lifecycle.go:199-201)
        self.stages: List[Stage] = [s for s in stages if s.selector is not None]
        if len(self.stages) > abi.MAX_STAGES:
            raise CompileError(f"{len(self.stages)} stages > {abi.MAX_STAGES}")
        self.names = [s.name for s in self.stages]
        self.harness = harness
        self.disregard = disregard if (disregard is not None and disregard.active) else None
        self.disregard_bit: Optional[int] = None
        self.features: Dict[str, Feature] = {}
        self.nbits = 0
        self.fin_bits: Dict[str, int] = {}
        self.fin_other_bit: Optional[int] = None
        self.slots: List[Tuple[str, str]] = []
        self._slot_q: List[Query] = []
        self._slot_index: Dict[Tuple[str, str], int] = {}
        self.stage_desc: List[abi.StageDesc] = []
        self._compile()
        # classes and deltas (filled by explore())
        self.class_ids: Dict[str, int] = {}
        self.class_reps: Dict[int, List[dict]] = {}
        self.deltas: Dict[Tuple[int, int], Tuple[int, int]] = {}
        self.delta_conflicts: List[str] = []
        self.rematch_mismatch: List[str] = []
        # stages whose patches can leave an object unchanged (Now-independent templates):
        # stage index -> synthetic feature bit "this stage's patch is already applied"
        self.applied_bits: Dict[int, int] = {}
        self._static_renderer = Renderer(exploration_funcs(), now_ns=1_700_000_000 * 10**9)

    # ------------------------------------------------------------------ bits
    def _bit(self) -> int:
        if self.nbits >= 32:
            raise CompileError("stage set needs more than 32 feature bits")
        b = self.nbits
        self.nbits += 1
        return b

    def _feature(self, src: str) -> Feature:
        key = _norm(src)
        f = self.features.get(key)
        if f is None:
            f = self.features[key] = Feature(src=src, query=Query(src))
        return f

    def _present(self, src: str) -> int:
        f = self._feature(src)
        if f.present_bit is None:
            f.present_bit = self._bit()
        return 1 << f.present_bit

    def _lits(self, src: str, values) -> int:
        f = self._feature(src)
        m = 0
        for v in values:
            if v not in f.lit_bits:
                f.lit_bits[v] = self._bit()
            m |= 1 << f.lit_bits[v]
        return m

    def _fin_value(self, v: str) -> int:
        if v not in self.fin_bits:
            self.fin_bits[v] = self._bit()
        return 1 << self.fin_bits[v]

    @property
    def fin_group_mask(self) -> int:
        m = 0
        for b in self.fin_bits.values():
            m |= 1 << b
        if self.fin_other_bit is not None:
            m |= 1 << self.fin_other_bit
        return m

    def _slot(self, typ: str, src: Optional[str]) -> int:
        if src is None:
            return abi.SLOT_NONE
        if typ == "duration" and _norm(src) == DELETION_QUERY:
            return abi.SLOT_DELETION
        key = (typ, _norm(src))
        if key not in self._slot_index:
            self._slot_index[key] = len(self.slots)
            self.slots.append((typ, src))
            self._slot_q.append(Query(src))
        return self._slot_index[key]

    # ------------------------------------------------------------------ compile
    def _compile(self):
        uses_fin = any(s.next.finalizers is not None for s in self.stages) or any(
            _norm(e.key) in FIN_QUERIES for s in self.stages for e in (s.selector.match_expressions or []))
        # finalizer values first so the group is contiguous-ish and stable
        if uses_fin:
            for s in self.stages:
                for e in s.selector.match_expressions or []:
                    if _norm(e.key) in (".metadata.finalizers.[]", ".metadata.finalizers[]") and e.operator in (
                            "In", "NotIn"):
                        for v in e.values:
                            self._fin_value(v)
                if s.next.finalizers is not None:
                    for v in s.next.finalizers.add + s.next.finalizers.remove:
                        self._fin_value(v)
            self.fin_other_bit = self._bit()
        for st in self.stages:
            eq_mask = eq_val = 0
            anys: List[Tuple[int, int]] = []

            def eq(mask, want):
                nonlocal eq_mask, eq_val
                eq_mask |= mask
                if want:
                    eq_val |= mask

            sel = st.selector
            for kind, m in (("labels", sel.match_labels), ("annotations", sel.match_annotations)):
                if m is None:
                    continue
                for k, v in m.items():  # labels.SelectorFromSet: key present with equal value
                    eq(self._lits(f".metadata.{kind}[{json.dumps(k)}]", [v]), True)
            for e in sel.match_expressions or []:
                nk = _norm(e.key)
                if nk in FIN_QUERIES:
                    g = self.fin_group_mask
                    if e.operator in ("Exists", "DoesNotExist"):
                        if e.operator == "Exists":
                            anys.append((g, 1))
                        else:
                            eq(g, False)
                    elif nk == ".metadata.finalizers":
                        # the array itself is never a string: In never holds, NotIn always holds
                        if e.operator == "In":
                            anys.append((0, 1))
                    else:
                        m = 0
                        for v in e.values:
                            m |= 1 << self.fin_bits[v]
                        if e.operator == "In":
                            if bin(m).count("1") == 1:
                                eq(m, True)
                            else:
                                anys.append((m, 1))
                        else:
                            eq(m, False)
                    continue
                if e.operator == "Exists":
                    eq(self._present(e.key), True)
                elif e.operator == "DoesNotExist":
                    eq(self._present(e.key), False)
                else:
                    m = self._lits(e.key, e.values)
                    if e.operator == "In":
                        if bin(m).count("1") == 1:
                            eq(m, True)
                        else:
                            anys.append((m, 1))
                    else:
                        eq(m, False)
            # a stage whose eq-tests contradict (same bit wanted 1 and 0) can never match
            if len(anys) > abi.MAX_ANY:
                raise CompileError(f"stage {st.name}: more than {abi.MAX_ANY} multi-value In requirements")
            d = abi.StageDesc()
            d.eq_mask, d.eq_val = eq_mask, eq_val
            d.n_any = len(anys)
            for i, (m, w) in enumerate(anys):
                d.any_mask[i] = m
                d.any_want |= w << i
            d.weight_default = int(st.weight)
            d.weight_slot = self._slot("int", st.weight_from)
            if st.delay is not None:
                d.has_delay = 1
                d.delay_default = int(st.delay.duration_ms or 0) * 1_000_000
                d.delay_slot = self._slot("duration", st.delay.duration_from)
                if st.delay.jitter_duration_ms is not None or st.delay.jitter_duration_from is not None:
                    d.has_jitter = 1
                    d.jitter_default = int(st.delay.jitter_duration_ms or 0) * 1_000_000
                    d.jitter_default_ok = 1 if st.delay.jitter_duration_ms is not None else 0
                    d.jitter_slot = self._slot("duration", st.delay.jitter_duration_from)
                else:
                    d.jitter_slot = abi.SLOT_NONE
            else:
                d.delay_slot = abi.SLOT_NONE
                d.jitter_slot = abi.SLOT_NONE
            fl = 0
            if st.next.delete:
                fl |= abi.NEXT_DELETE
            if st.immediate_next_stage:
                fl |= abi.NEXT_IMMEDIATE
            if st.next.patches:
                fl |= abi.NEXT_PATCHES
            if st.next.finalizers is not None:
                f = st.next.finalizers
                fl |= abi.NEXT_FIN
                if f.empty:
                    fl |= abi.NEXT_FIN_EMPTY
                if f.remove:
                    fl |= abi.NEXT_FIN_REMOVE
                for v in f.add:
                    d.fin_add |= 1 << self.fin_bits[v]
                for v in f.remove:
                    d.fin_remove |= 1 << self.fin_bits[v]
            d.flags = fl
            self.stage_desc.append(d)
        if self.harness is not None:
            self.deletion_bit = self._present(self.harness.deletion_query)
            self.terminal_mask = self._lits(self.harness.terminal_query, list(self.harness.terminal_values))
        if self.disregard is not None:  # need()'s selector part: labels / annotations (spec, kept on re-creation)
            self.disregard_bit = self._bit()
        # keep mask for harness re-creation: features that do not read status / deletion / finalizers
        keep = 0 if self.disregard_bit is None else 1 << self.disregard_bit
        for f in self.features.values():
            p = path_prefix(f.src)
            dyn = (not p) or p[0] == "status" or p[:2] in (["metadata", "deletionTimestamp"],
                                                           ["metadata", "deletionGracePeriodSeconds"],
                                                           ["metadata", "finalizers"])
            if not dyn:
                keep |= f.mask()
        self.keep_mask = keep

    # ------------------------------------------------------------------ per object
    def pred_of(self, obj: dict) -> int:
        pred = 0
        for f in self.features.values():
            out = f.query.execute(obj)
            if not out:
                continue
            if f.present_bit is not None:
                pred |= 1 << f.present_bit
            for v, b in f.lit_bits.items():
                if any(has_value(d, (v,)) for d in out):
                    pred |= 1 << b
        if self.fin_other_bit is not None:
            for x in (obj.get("metadata") or {}).get("finalizers") or []:
                b = self.fin_bits.get(x)
                pred |= 1 << (self.fin_other_bit if b is None else b)
        for s, b in self.applied_bits.items():
            if self._patch_applied(self.stages[s], obj):
                pred |= 1 << b
        if self.disregard is not None and self.disregard.disregarded(obj):
            pred |= 1 << self.disregard_bit
        return pred

    def _patch_applied(self, st: Stage, obj: dict) -> bool:
        """True iff rendering + applying the stage's patches leaves the object unchanged."""
        try:
            cur = obj
            for ptype, data, _ in render_patches(st, obj, self._static_renderer):
                cur = prune_empty(json_patch(cur, data) if ptype == "json" else merge_patch(cur, data))
        except Exception:
            return False
        return json.dumps(cur, sort_keys=True) == json.dumps(obj, sort_keys=True)

    def stage_matches(self, pred: int) -> int:
        m = 0
        for i, d in enumerate(self.stage_desc):
            ok = ((pred ^ d.eq_val) & d.eq_mask) == 0
            for k in range(d.n_any):
                ok = ok and (((pred & d.any_mask[k]) != 0) == bool((d.any_want >> k) & 1))
            if ok:
                m |= 1 << i
        return m

    def record_of(self, obj: dict) -> Optional[List[Tuple[int, int, int]]]:
        """Pre-parsed *From results: [(kind, value, nsec)] per slot, or None if all default."""
        out = []
        any_set = False
        for (typ, _src), q in zip(self.slots, self._slot_q):
            res = q.execute(obj)
            if not res:
                out.append((abi.V_DEFAULT, 0, 0))
                continue
            t = res[0]
            if typ == "int":  # int64From.Get (value_int_from.go:53-81)
                if isinstance(t, str):
                    if t == "":
                        e = (abi.V_NOTOK, 0, 0)
                    else:
                        n = parse_int(t)
                        e = (abi.V_NOTOK, 0, 0) if n is None else (abi.V_OK, n, 0)
                elif isinstance(t, float):  # float64 (a gojq int falls to the default, as Go's switch)
                    e = (abi.V_OK, f64_to_i64(t), 0)
                else:
                    e = (abi.V_DEFAULT, 0, 0)
            else:  # durationFrom.Get (value_duration_from.go:53-79)
                if isinstance(t, str):
                    if t == "":
                        e = (abi.V_NOTOK, 0, 0)
                    else:
                        ts = parse_rfc3339nano(t)
                        if ts is not None:
                            e = (abi.V_ABSTIME, ts[0], ts[1])
                        else:
                            d = parse_duration(t)
                            e = (abi.V_NOTOK, 0, 0) if d is None else (abi.V_OK, d, 0)
                else:
                    e = (abi.V_NOTOK, 0, 0)
            any_set |= e[0] != abi.V_DEFAULT
            out.append(e)
        return out if any_set else None

    @staticmethod
    def deletion_s(obj: dict) -> int:
        ts = (obj.get("metadata") or {}).get("deletionTimestamp")
        if not isinstance(ts, str) or ts == "":
            return abi.DEL_ABSENT
        t = parse_rfc3339nano(ts)
        if t is None:
            raise CompileError(f"deletionTimestamp {ts!r} is not RFC3339")
        return t[0]

    # ------------------------------------------------------------------ deltas
    def class_of(self, obj: dict, register: bool = True) -> int:
        k = class_key(obj)
        c = self.class_ids.get(k)
        if c is None:
            if not register:
                raise CompileError("unknown object class")
            c = self.class_ids[k] = len(self.class_ids)
            if c >= 1 << 16:
                raise CompileError("more than 65536 object classes")
            self.class_reps[c] = []
        return c

    def explore(self, roots: Sequence[dict], max_states: int = 256):
        """Derive per-(class, stage) deltas from every (class, start-state) representative.

        Each root is expanded by firing every matching stage (any could be picked) and, if a
        harness is configured, its churn edges; transitions (pre -> post feature bits) are
        collected per (class, stage) and turned into and/or masks.  A first pass finds stages
        whose patches can leave the object unchanged; they get an "applied" feature bit and
        the exploration is redone with it."""
        # roots are deduplicated by (class, start features) as they arrive: matching the same
        # objects again (Lifecycle.match_batch explores every batch) re-runs nothing
        if not hasattr(self, "_roots"):
            self._roots, self._root_keys, self._explored = [], set(), False
        added = 0
        for r in roots:
            r = prune_empty(copy.deepcopy(r))
            k = (class_key(r), self.pred_of(r))
            if k in self._root_keys:
                continue
            self._root_keys.add(k)
            self._roots.append(r)
            added += 1
        if self._explored and not added:
            return
        self._explored = True
        for _ in range(2):
            unchanged = self._explore_pass(self._roots, max_states)
            new = [s for s in unchanged if s not in self.applied_bits]
            if not new:
                break
            for s in new:
                self.applied_bits[s] = self._bit()
                d = self.stage_desc[s]
                d.flags |= abi.NEXT_PATCH_STATIC
                d.applied_mask = 1 << self.applied_bits[s]
        self.rematch_mismatch = []

    def _explore_pass(self, roots, max_states):
        self.class_reps = {c: [] for c in self.class_reps}
        self.deltas = {}
        self.delta_conflicts = []
        unchanged = set()
        trans: Dict[Tuple[int, int], List[Tuple[int, int]]] = {}
        renderer = Renderer(exploration_funcs())
        fin = self.fin_group_mask
        seen_roots = set()
        for root in roots:
            root = prune_empty(copy.deepcopy(root))
            c = self.class_of(root)
            start = [root]
            if self.harness is not None:
                start.append(strip_for_recreate(root))
            for r in start:
                rk = (c, self.pred_of(r))
                if rk in seen_roots:
                    continue
                seen_roots.add(rk)
                self.class_reps[c].append(r)
                frontier = [r]
                seen = {self.pred_of(r)}
                t_ns = 1_700_000_000 * 10**9
                while frontier and len(seen) <= max_states:
                    o = frontier.pop()
                    p = self.pred_of(o)
                    m = self.stage_matches(p)
                    succ = []
                    for s in range(len(self.stages)):
                        if not (m >> s) & 1:
                            continue
                        st = self.stages[s]
                        t_ns += 10**9
                        renderer.funcs["Now"] = lambda t=t_ns: rfc3339nano(t)
                        o2, changed = apply_next(st, copy.deepcopy(o), renderer)
                        if st.next.patches and not changed and not st.next.delete:
                            unchanged.add(s)
                        if o2 is None:
                            continue
                        p2 = self.pred_of(o2)
                        trans.setdefault((c, s), []).append((p, p2))
                        # an idempotent (Now-independent) patch: firing again changes nothing
                        if st.next.patches and s not in self.applied_bits and (self.stage_matches(p2) >> s) & 1:
                            _, again = apply_next(st, copy.deepcopy(o2), renderer)
                            if not again:
                                unchanged.add(s)
                        # finalizer set algebra must reproduce the JSON-patch result
                        d = self.stage_desc[s]
                        if d.flags & abi.NEXT_FIN:
                            F = p & fin
                            if (d.flags & abi.NEXT_FIN_EMPTY) or ((d.flags & abi.NEXT_FIN_REMOVE) and (F & ~d.fin_remove) == 0):
                                F2 = d.fin_add
                            else:
                                F2 = (F & ~d.fin_remove) | (d.fin_add & ~F)
                            if F2 != (p2 & fin):
                                raise CompileError(f"stage {st.name}: finalizer algebra mismatch")
                        succ.append(o2)
                    if self.harness is not None and (p & self.terminal_mask) and not (p & self.deletion_bit):
                        o2 = copy.deepcopy(o)
                        o2.setdefault("metadata", {})["deletionTimestamp"] = "2023-11-14T22:13:20Z"
                        succ.append(o2)
                    for o2 in succ:
                        p2 = self.pred_of(o2)
                        if p2 not in seen:
                            seen.add(p2)
                            frontier.append(o2)
        nonfin = 0xFFFFFFFF & ~fin
        for (c, s), ts in trans.items():
            if not self.stages[s].next.patches:
                self.deltas[(c, s)] = (0xFFFFFFFF, 0)
                continue
            and_m, or_m = 0xFFFFFFFF, 0
            ok = True
            for b in range(32):
                bit = 1 << b
                if not (nonfin & bit):
                    continue
                posts = {bool(p2 & bit) for _, p2 in ts}
                if all(bool(p & bit) == bool(p2 & bit) for p, p2 in ts):
                    continue  # keep
                if len(posts) == 1:
                    and_m &= ~bit
                    if posts.pop():
                        or_m |= bit
                else:
                    ok = False
                    self.delta_conflicts.append(f"class {c} stage {self.stages[s].name}: bit {b} depends on pre-state")
            self.deltas[(c, s)] = (and_m & 0xFFFFFFFF, or_m) if ok else abi.DELTA_UNKNOWN
        return unchanged

    # ------------------------------------------------------------------ device tables
    def table(self, version: int = 1) -> abi.StageTable:
        t = abi.StageTable()
        t.n_stages = len(self.stages)
        t.fin_group_mask = self.fin_group_mask
        t.n_classes = max(1, len(self.class_ids))
        t.version = version
        t.pred_bits = self.nbits
        t.disregard_mask = 0 if self.disregard_bit is None else 1 << self.disregard_bit
        for i, d in enumerate(self.stage_desc):
            t.stages[i] = d
        return t

    def delta_array(self):
        import numpy as np
        n_c = max(1, len(self.class_ids))
        n_s = max(1, len(self.stages))
        a = np.zeros((n_c, n_s, 2), dtype=np.uint32)
        a[:, :, 0] = abi.DELTA_UNKNOWN[0]
        a[:, :, 1] = abi.DELTA_UNKNOWN[1]
        for (c, s), (am, om) in self.deltas.items():
            a[c, s] = (am, om)
        for s, st in enumerate(self.stages):
            if not st.next.patches:  # no patches: identity outside the finalizer set
                a[:, s] = (0xFFFFFFFF, 0)
        return a

    def harness_struct(self) -> abi.Harness:
        h = abi.Harness()
        if self.harness is not None:
            h.enable = 1
            h.keep_mask = self.keep_mask
            h.terminal_mask = self.terminal_mask
            h.deletion_bit = self.deletion_bit
            h.track_deletion = 1 if self.uses_deletion_column else 0
        return h

    @property
    def uses_deletion_column(self) -> bool:
        return any(d.delay_slot == abi.SLOT_DELETION or d.jitter_slot == abi.SLOT_DELETION for d in self.stage_desc)

    def describe(self) -> dict:
        feats = []
        for f in self.features.values():
            feats.append({"query": f.src, "present_bit": f.present_bit, "literals": dict(f.lit_bits)})
        return {"stages": self.names, "bits": self.nbits, "features": feats,
                "applied_bits": {self.names[s]: b for s, b in self.applied_bits.items()},
                "finalizers": dict(self.fin_bits), "finalizer_other_bit": self.fin_other_bit,
                "value_slots": [list(s) for s in self.slots], "classes": len(self.class_ids),
                "uses_deletion_column": self.uses_deletion_column,
                "disregard": None if self.disregard is None else {
                    "bit": self.disregard_bit, "annotation_selector": self.disregard.annotation_selector,
                    "label_selector": self.disregard.label_selector}}
