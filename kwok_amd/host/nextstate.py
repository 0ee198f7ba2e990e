"""Host-side mirror of a Stage's ``next`` (pkg/utils/lifecycle/next.go, finalizers.go).

Used for the objects the device hands back as *fired*: render their text patches
(next.go:73-173), compute the finalizer JSON patch (finalizers.go:83-111) and — for the
compiler and the test harness — apply those patches to an object as the apiserver would
(RFC 7386 merge patch / RFC 6902 JSON patch for the finalizer ops).
"""
from __future__ import annotations

import copy
import json
from typing import List, Optional

from .gotpl import Renderer
from .stages import Stage, StageFinalizers
from .typed import typed_presence


def finalizers_modify(meta: Optional[List[str]], fin: StageFinalizers):
    """finalizers.go:83-111 (ops as dicts, same order)."""
    meta = list(meta or [])
    ops = []
    is_empty = False
    if fin.empty:
        is_empty = True
    elif fin.remove:
        removed = [{"op": "remove", "path": f"/metadata/finalizers/{i}"}
                   for i in range(len(meta) - 1, -1, -1) if meta[i] in fin.remove]
        if len(removed) == len(meta):
            is_empty = True
        else:
            ops += removed

    def add(m):
        if m:
            return [{"op": "add", "path": "/metadata/finalizers/-", "value": f} for f in fin.add if f not in m]
        return [{"op": "add", "path": "/metadata/finalizers", "value": list(fin.add)}]

    if not is_empty:
        if fin.add:
            ops += add(meta)
    else:
        if meta:
            ops.append({"op": "remove", "path": "/metadata/finalizers"})
        if fin.add:
            ops += add([])
    return ops


def render_patches(stage: Stage, obj: dict, renderer: Renderer):
    """Next.Patches (next.go:73-88) -> [(patch_type, data, subresource)]."""
    out = []
    for p in stage.next.patches:
        data = renderer.to_json(p.template, obj)
        if p.type == "json":
            if p.root:
                data = [dict(op, path="/" + p.root + op.get("path", "")) for op in (data or [])]
            out.append(("json", data, p.subresource))
        else:
            if p.root:
                data = {p.root: data}
            out.append((p.type, data, p.subresource))
    return out


def merge_patch(target, patch):
    """RFC 7386 JSON merge patch (github.com/evanphx/json-patch MergePatch semantics)."""
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    if not isinstance(target, dict):
        target = {}
    out = dict(target)
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


def _ptr(path):
    return [p.replace("~1", "/").replace("~0", "~") for p in path.split("/")[1:]]


def json_patch(obj, ops):
    """RFC 6902 subset (add / remove / replace) used by the finalizer ops."""
    obj = copy.deepcopy(obj)
    for op in ops:
        parts = _ptr(op["path"])
        parent = obj
        for p in parts[:-1]:
            parent = parent[int(p)] if isinstance(parent, list) else parent.setdefault(p, {})
        last = parts[-1]
        if op["op"] in ("add", "replace"):
            if isinstance(parent, list):
                if last == "-":
                    parent.append(copy.deepcopy(op["value"]))
                else:
                    parent.insert(int(last), copy.deepcopy(op["value"]))
            else:
                parent[last] = copy.deepcopy(op["value"])
        elif op["op"] == "remove":
            if isinstance(parent, list):
                del parent[int(last)]
            else:
                del parent[last]
        else:
            raise ValueError(f"unsupported json patch op {op['op']}")
    return obj


def prune_empty(obj):
    """The object after the apiserver's typed round trip (a patch that empties an omitempty field
    removes it): typed.typed_presence, which the informer's objects and ToJSONStandard agree on."""
    return typed_presence(obj)


def apply_next(stage: Stage, obj: dict, renderer: Renderer):
    """playStage's effect on the object (pod_controller.go:290-360): finalizers patch, then
    delete (returns None) or the rendered patches. Returns (new_obj | None, changed)."""
    changed = False
    if stage.next.finalizers is not None:
        ops = finalizers_modify((obj.get("metadata") or {}).get("finalizers"), stage.next.finalizers)
        if ops:
            new = prune_empty(json_patch(obj, ops))
            # a watch event (and so a re-match) follows only if the object really changed
            changed = json.dumps(new, sort_keys=True) != json.dumps(obj, sort_keys=True)
            obj = new
    if stage.next.delete:
        return None, True
    for ptype, data, _sub in render_patches(stage, obj, renderer):
        if ptype == "json":
            new = json_patch(obj, data)
        else:
            new = merge_patch(obj, data)
        new = prune_empty(new)
        if json.dumps(new, sort_keys=True) != json.dumps(obj, sort_keys=True):
            changed = True
            obj = new
    return obj, changed
