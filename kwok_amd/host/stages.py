"""The Stage CRD surface (v1alpha1 -> internal), host side.

Mirrors ``pkg/apis/v1alpha1/stage_types.go:61-200`` (the CRD a user writes),
``pkg/apis/internalversion/stage_types.go:33-51`` (what the controllers consume), the
conversion ``internalversion/conversion.go:395-425`` (``statusTemplate`` becomes one merge
patch rooted at ``status``) and the defaults ``v1alpha1/zz_generated.defaults.go:55-63``
(``apiGroup: v1``, ``statusSubresource: status``).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import yaml

OPS = ("In", "NotIn", "Exists", "DoesNotExist")


class StageError(ValueError):
    pass


@dataclass
class SelectorRequirement:
    key: str
    operator: str
    values: List[str] = field(default_factory=list)


@dataclass
class StageSelector:
    match_labels: Optional[Dict[str, str]] = None
    match_annotations: Optional[Dict[str, str]] = None
    match_expressions: Optional[List[SelectorRequirement]] = None


@dataclass
class StageDelay:
    duration_ms: Optional[int] = None
    duration_from: Optional[str] = None
    jitter_duration_ms: Optional[int] = None
    jitter_duration_from: Optional[str] = None


@dataclass
class StagePatch:
    root: str = ""
    template: str = ""
    type: str = "merge"  # merge | strategic | json
    subresource: str = ""
    impersonation: Optional[str] = None


@dataclass
class StageFinalizers:
    add: List[str] = field(default_factory=list)
    remove: List[str] = field(default_factory=list)
    empty: bool = False


@dataclass
class StageEvent:
    type: str = ""
    reason: str = ""
    message: str = ""


@dataclass
class StageNext:
    event: Optional[StageEvent] = None
    finalizers: Optional[StageFinalizers] = None
    delete: bool = False
    patches: List[StagePatch] = field(default_factory=list)


@dataclass
class Stage:
    name: str
    api_group: str
    kind: str
    selector: Optional[StageSelector]
    weight: int = 0
    weight_from: Optional[str] = None
    delay: Optional[StageDelay] = None
    next: StageNext = field(default_factory=StageNext)
    immediate_next_stage: bool = False

    @property
    def resource_ref(self):
        return (self.api_group, self.kind)


def _expr_from(x):
    if x is None:
        return None
    if not isinstance(x, dict):
        raise StageError("expressionFrom source must be an object")
    return x.get("expressionFrom", "")


def stage_from_v1alpha1(obj: dict) -> Stage:
    """Convert one v1alpha1 Stage object (as decoded from YAML/JSON) to the internal form."""
    if obj.get("kind", "Stage") != "Stage":
        raise StageError(f"not a Stage: {obj.get('kind')}")
    spec = obj.get("spec") or {}
    ref = spec.get("resourceRef") or {}
    if "kind" not in ref:
        raise StageError("spec.resourceRef.kind is required")
    sel = spec.get("selector")
    selector = None
    if sel is not None:
        exprs = None
        if sel.get("matchExpressions") is not None:
            exprs = []
            for e in sel["matchExpressions"]:
                op = e.get("operator")
                vals = [str(v) for v in (e.get("values") or [])]
                if op in ("In", "NotIn") and not vals:
                    raise StageError("for 'in', 'notin' operators, values set can't be empty")
                if op in ("Exists", "DoesNotExist") and vals:
                    raise StageError("values set must be empty for exists and does not exist")
                if op not in OPS:
                    raise StageError(f"operator {op!r} is not supported")
                exprs.append(SelectorRequirement(e["key"], op, vals))
        ml = sel.get("matchLabels")
        ma = sel.get("matchAnnotations")
        selector = StageSelector(
            match_labels=None if ml is None else {str(k): str(v) for k, v in ml.items()},
            match_annotations=None if ma is None else {str(k): str(v) for k, v in ma.items()},
            match_expressions=exprs,
        )
    d = spec.get("delay")
    delay = None
    if d is not None:
        delay = StageDelay(
            duration_ms=d.get("durationMilliseconds"),
            duration_from=_expr_from(d.get("durationFrom")),
            jitter_duration_ms=d.get("jitterDurationMilliseconds"),
            jitter_duration_from=_expr_from(d.get("jitterDurationFrom")),
        )
    n = spec.get("next") or {}
    fin = None
    if n.get("finalizers") is not None:
        f = n["finalizers"]
        fin = StageFinalizers(
            add=[i.get("value", "") for i in (f.get("add") or [])],
            remove=[i.get("value", "") for i in (f.get("remove") or [])],
            empty=bool(f.get("empty", False)),
        )
    ev = None
    if n.get("event") is not None:
        e = n["event"]
        ev = StageEvent(e.get("type", ""), e.get("reason", ""), e.get("message", ""))
    patches = []
    for p in n.get("patches") or []:
        patches.append(StagePatch(root=p.get("root", ""), template=p.get("template", ""),
                                  type=p.get("type") or "merge", subresource=p.get("subresource", ""),
                                  impersonation=(p.get("impersonation") or {}).get("username")))
    # conversion.go:400-423: statusTemplate -> one merge patch rooted at status
    if n.get("statusTemplate") and not patches:
        sub = n.get("statusSubresource")
        patches.append(StagePatch(root="status", template=n["statusTemplate"], type="merge",
                                  subresource="status" if sub is None else sub,
                                  impersonation=(n.get("statusPatchAs") or {}).get("username")))
    nxt = StageNext(event=ev, finalizers=fin, delete=bool(n.get("delete", False)), patches=patches)
    return Stage(
        name=(obj.get("metadata") or {}).get("name", ""),
        api_group=ref.get("apiGroup") or "v1",
        kind=ref["kind"],
        selector=selector,
        weight=int(spec.get("weight") or 0),
        weight_from=_expr_from(spec.get("weightFrom")),
        delay=delay,
        next=nxt,
        immediate_next_stage=bool(spec.get("immediateNextStage") or False),
    )


def load_stages_yaml(*texts: str) -> List[Stage]:
    out = []
    for t in texts:
        for doc in yaml.safe_load_all(t):
            if doc:
                out.append(stage_from_v1alpha1(doc))
    return out


def load_stage_files(*paths: str) -> List[Stage]:
    return load_stages_yaml(*[open(p).read() for p in paths])


def group_by_ref(stages: List[Stage]):
    """root.go:152 slices.GroupBy: group per resourceRef, preserving input order."""
    out: Dict[tuple, List[Stage]] = {}
    for s in stages:
        out.setdefault(s.resource_ref, []).append(s)
    return out


def to_v1alpha1(stage: Stage) -> dict:
    """Inverse conversion (for handing the same stage set to other consumers)."""
    spec: dict = {"resourceRef": {"apiGroup": stage.api_group, "kind": stage.kind}}
    if stage.selector is not None:
        sel: dict = {}
        if stage.selector.match_labels is not None:
            sel["matchLabels"] = dict(stage.selector.match_labels)
        if stage.selector.match_annotations is not None:
            sel["matchAnnotations"] = dict(stage.selector.match_annotations)
        if stage.selector.match_expressions is not None:
            sel["matchExpressions"] = [dataclasses.asdict(e) for e in stage.selector.match_expressions]
        spec["selector"] = sel
    spec["weight"] = stage.weight
    if stage.weight_from is not None:
        spec["weightFrom"] = {"expressionFrom": stage.weight_from}
    if stage.delay is not None:
        d: dict = {}
        if stage.delay.duration_ms is not None:
            d["durationMilliseconds"] = stage.delay.duration_ms
        if stage.delay.duration_from is not None:
            d["durationFrom"] = {"expressionFrom": stage.delay.duration_from}
        if stage.delay.jitter_duration_ms is not None:
            d["jitterDurationMilliseconds"] = stage.delay.jitter_duration_ms
        if stage.delay.jitter_duration_from is not None:
            d["jitterDurationFrom"] = {"expressionFrom": stage.delay.jitter_duration_from}
        spec["delay"] = d
    nx: dict = {}
    if stage.next.finalizers is not None:
        f = stage.next.finalizers
        nx["finalizers"] = {"add": [{"value": v} for v in f.add], "remove": [{"value": v} for v in f.remove],
                            "empty": f.empty}
    nx["delete"] = stage.next.delete
    if stage.next.patches:
        nx["patches"] = [{"root": p.root, "template": p.template, "type": p.type, "subresource": p.subresource}
                         for p in stage.next.patches]
    spec["next"] = nx
    spec["immediateNextStage"] = stage.immediate_next_stage
    return {"apiVersion": "kwok.x-k8s.io/v1alpha1", "kind": "Stage", "metadata": {"name": stage.name}, "spec": spec}
