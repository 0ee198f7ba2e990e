"""ORACLE / TEST INFRASTRUCTURE — not product code.

`expression.ToJSONStandard` (reference `pkg/utils/expression/query.go:72-88`) feeds the Stage
queries the JSON of the *typed* object: `json.Marshal` of a `*corev1.Pod` / `*corev1.Node`, then
`json.Unmarshal` into `interface{}`.  Go's encoder then decides presence by the struct tags of
k8s.io/api v0.30.2 `core/v1/types.go` and apimachinery `meta/v1/types.go` (go.mod of the
reference; the modules are not vendored, so the tags are restated from their published source):

* a field tagged `omitempty` whose value is the zero value of a string, number, bool, slice or
  map is left out (encoding/json `isEmptyValue`);
* a field whose type is a struct is always written, even when zero (omitempty does not apply to
  structs): `metadata`, `spec`, `status`, a container status's `state` / `lastState`, ...;
* a pointer field is left out only when nil: `"running": {}` stays (a non-nil pointer to a zero
  struct);
* a field without `omitempty` is always written: a condition's `type` / `status`, a container
  status's `ready` / `restartCount` / `image` / `imageID`, an owner reference's identity, ...;
* `metav1.Time` marshals its zero value as `null` (and `""` does not decode at all), which
  `Query.Execute` drops like an absent value (`query.go:63-65`): a null is absent.

`to_json_standard` applies those rules to an object as the apiserver or a hand-written fixture
spells it: empty values of omitempty fields are removed (recursively), nulls are removed, struct
and non-omitempty fields are kept.  Fields the typed decode does not know are kept when non-empty
(the oracle does not restate the whole API schema; the reference's informers never deliver them).
"""
from __future__ import annotations

import copy

from typing import Any, Dict, Optional

# field kinds: K keep (no omitempty: always written), S struct (always written, recurse with the
# named schema), P pointer to struct (written unless null, recurse), L list of the named struct
# (omitempty: dropped when empty), LK list without omitempty (kept when empty), T metav1.Time
# (null when zero).  Unlisted fields are omitempty scalars / slices / maps.
K, S, P, L, LK, T = "K", "S", "P", "L", "LK", "T"

SCHEMA: Dict[str, Dict[str, tuple]] = {
    # meta/v1 types.go ObjectMeta (all omitempty); creationTimestamp is a Time (struct)
    "ObjectMeta": {"creationTimestamp": (T,), "deletionTimestamp": (T,),
                   "ownerReferences": (L, "OwnerReference"), "managedFields": (L, None)},
    # OwnerReference: apiVersion, kind, name, uid have no omitempty
    "OwnerReference": {"apiVersion": (K,), "kind": (K,), "name": (K,), "uid": (K,)},
    "Pod": {"metadata": (S, "ObjectMeta"), "spec": (S, "PodSpec"), "status": (S, "PodStatus")},
    # PodSpec.containers has no omitempty
    "PodSpec": {"containers": (LK, "Container"), "initContainers": (L, "Container"),
                "ephemeralContainers": (L, "Container")},
    "Container": {"name": (K,), "resources": (S, None)},
    "PodStatus": {"conditions": (L, "PodCondition"), "startTime": (T,),
                  "initContainerStatuses": (L, "ContainerStatus"), "containerStatuses": (L, "ContainerStatus"),
                  "ephemeralContainerStatuses": (L, "ContainerStatus")},
    "PodCondition": {"type": (K,), "status": (K,), "lastProbeTime": (T,), "lastTransitionTime": (T,)},
    "ContainerStatus": {"name": (K,), "state": (S, "ContainerState"), "lastState": (S, "ContainerState"),
                        "ready": (K,), "restartCount": (K,), "image": (K,), "imageID": (K,)},
    "ContainerState": {"waiting": (P, None), "running": (P, "ContainerStateRunning"),
                       "terminated": (P, "ContainerStateTerminated")},
    "ContainerStateRunning": {"startedAt": (T,)},
    "ContainerStateTerminated": {"exitCode": (K,), "startedAt": (T,), "finishedAt": (T,)},
    "Node": {"metadata": (S, "ObjectMeta"), "spec": (S, None), "status": (S, "NodeStatus")},
    "NodeStatus": {"conditions": (L, "NodeCondition"), "daemonEndpoints": (S, None), "nodeInfo": (S, "NodeSystemInfo")},
    "NodeCondition": {"type": (K,), "status": (K,), "lastHeartbeatTime": (T,), "lastTransitionTime": (T,)},
    # NodeSystemInfo: no omitempty on any field
    "NodeSystemInfo": {k: (K,) for k in ("machineID", "systemUUID", "bootID", "kernelVersion", "osImage",
                                          "containerRuntimeVersion", "kubeletVersion", "kubeProxyVersion",
                                          "operatingSystem", "architecture")},
}


def _empty(v: Any) -> bool:
    """encoding/json isEmptyValue for what JSON can hold (false, 0, "", empty list / map, null)."""
    return v is None or v is False or (isinstance(v, (int, float)) and not isinstance(v, bool) and v == 0) or \
        (isinstance(v, (str, list, dict)) and len(v) == 0)


def _struct(obj: dict, schema: Optional[str]) -> dict:
    fields = SCHEMA.get(schema or "", {})
    out = {}
    for k, v in obj.items():
        kind = fields.get(k)
        if v is None:
            continue  # a null is absent to every query (Time zero values included)
        if kind is None:  # omitempty scalar / slice / map (entries of a map are kept as they are)
            if not _empty(v):
                out[k] = v
            continue
        tag = kind[0]
        sub = kind[1] if len(kind) > 1 else None
        if tag == K:
            out[k] = v
        elif tag == T:
            if v != "":
                out[k] = v
        elif tag in (S, P):
            out[k] = _struct(v, sub) if isinstance(v, dict) else v
        elif tag in (L, LK):
            if isinstance(v, list):
                v = [_struct(x, sub) if isinstance(x, dict) else x for x in v]
            if tag == LK or not _empty(v):
                out[k] = v
    return out


def to_json_standard(obj: Optional[dict]) -> Optional[dict]:
    """The presence the reference's queries see: a typed Pod / Node round trip
    (PodController / NodeController), or, for every other kind, the object as the StageController
    holds it — *unstructured.Unstructured, whose json.Marshal writes the map as it is, zero values and
    nulls included (pkg/kwok/controllers/stage_controller.go:174-232)."""
    if obj is None:
        return None
    kind = obj.get("kind")
    if kind not in ("Pod", "Node"):
        return copy.deepcopy(obj)
    return _struct(obj, kind)
