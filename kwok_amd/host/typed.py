"""Typed-object presence (`expression.ToJSONStandard`, reference `pkg/utils/expression/query.go:72-88`).

The reference's queries see `json.Marshal` of the typed `*corev1.Pod` / `*corev1.Node`: Go writes
a field tagged `omitempty` only when it is not the zero value of its string / number / bool /
slice / map type, always writes struct-typed fields and fields without `omitempty`, writes a
pointer unless it is nil, and writes a zero `metav1.Time` as `null`, which `Query.Execute`
drops (`query.go:63-65`).  `typed_presence` rewrites an object as an informer or a fixture
spells it into that presence (k8s.io/api v0.30.2 `core/v1/types.go` tags for the fields on the
paths the Stage CRDs query): empty values of omitempty fields and nulls are removed, struct and
non-omitempty fields kept.  Fields outside the table keep their value unless it is empty.

The apiserver serialises the same typed objects, so its JSON is already in this form; the
rewrite matters for hand-written objects (`"podIP": ""`, `"finalizers": []`, `"reason": ""`,
`"labels": {}`), and after a patch (the apiserver round trip drops what a patch emptied)."""
from __future__ import annotations

import copy

from typing import Optional

# kinds: "keep" (no omitempty), "struct" / "ptr" (recurse into the named type), "list" (omitempty
# slice of the named type), "list!" (slice without omitempty), "time" (metav1.Time: null when zero)
_TYPES = {
    "Pod": {"metadata": ("struct", "ObjectMeta"), "spec": ("struct", "PodSpec"), "status": ("struct", "PodStatus")},
    "Node": {"metadata": ("struct", "ObjectMeta"), "spec": ("struct", ""), "status": ("struct", "NodeStatus")},
    "ObjectMeta": {"creationTimestamp": ("time",), "deletionTimestamp": ("time",),
                   "ownerReferences": ("list", "OwnerReference"), "managedFields": ("list", "")},
    "OwnerReference": {"apiVersion": ("keep",), "kind": ("keep",), "name": ("keep",), "uid": ("keep",)},
    "PodSpec": {"containers": ("list!", "Container"), "initContainers": ("list", "Container"),
                "ephemeralContainers": ("list", "Container")},
    "Container": {"name": ("keep",), "resources": ("struct", "")},
    "PodStatus": {"conditions": ("list", "PodCondition"), "startTime": ("time",),
                  "initContainerStatuses": ("list", "ContainerStatus"),
                  "containerStatuses": ("list", "ContainerStatus"),
                  "ephemeralContainerStatuses": ("list", "ContainerStatus")},
    "PodCondition": {"type": ("keep",), "status": ("keep",), "lastProbeTime": ("time",),
                     "lastTransitionTime": ("time",)},
    "ContainerStatus": {"name": ("keep",), "ready": ("keep",), "restartCount": ("keep",), "image": ("keep",),
                        "imageID": ("keep",), "state": ("struct", "ContainerState"),
                        "lastState": ("struct", "ContainerState")},
    "ContainerState": {"waiting": ("ptr", ""), "running": ("ptr", "ContainerStateRunning"),
                       "terminated": ("ptr", "ContainerStateTerminated")},
    "ContainerStateRunning": {"startedAt": ("time",)},
    "ContainerStateTerminated": {"exitCode": ("keep",), "startedAt": ("time",), "finishedAt": ("time",)},
    "NodeStatus": {"conditions": ("list", "NodeCondition"), "daemonEndpoints": ("struct", ""),
                   "nodeInfo": ("struct", "NodeSystemInfo")},
    "NodeCondition": {"type": ("keep",), "status": ("keep",), "lastHeartbeatTime": ("time",),
                      "lastTransitionTime": ("time",)},
    "NodeSystemInfo": {f: ("keep",) for f in ("machineID", "systemUUID", "bootID", "kernelVersion", "osImage",
                                               "containerRuntimeVersion", "kubeletVersion", "kubeProxyVersion",
                                               "operatingSystem", "architecture")},
}


def _is_zero(v) -> bool:
    if v is None or v is False:
        return True
    if isinstance(v, bool):
        return False
    if isinstance(v, (int, float)):
        return v == 0
    return isinstance(v, (str, list, dict)) and not v


def _rewrite(obj: dict, tname: str) -> dict:
    fields = _TYPES.get(tname, {})
    res = {}
    for key, val in obj.items():
        if val is None:
            continue
        spec = fields.get(key)
        if spec is None:
            if not _is_zero(val):
                res[key] = val
            continue
        kind = spec[0]
        if kind == "keep":
            res[key] = val
        elif kind == "time":
            if val != "":
                res[key] = val
        elif kind in ("struct", "ptr"):
            res[key] = _rewrite(val, spec[1]) if isinstance(val, dict) else val
        else:  # list / list!
            if isinstance(val, list):
                val = [_rewrite(x, spec[1]) if isinstance(x, dict) else x for x in val]
            if kind == "list!" or not _is_zero(val):
                res[key] = val
    return res


def typed_presence(obj: Optional[dict]) -> Optional[dict]:
    """A new dict with the presence a typed Pod / Node round trip gives.  Other kinds reach the
    reference's matcher through the StageController as *unstructured.Unstructured
    (stage_controller.go:174-232), whose json.Marshal writes the object map as it is — every field,
    zero values and nulls included — so they are returned unchanged (a copy)."""
    if obj is None:
        return None
    k = obj.get("kind")
    if k not in ("Pod", "Node"):
        return copy.deepcopy(obj)
    return _rewrite(obj, k)
