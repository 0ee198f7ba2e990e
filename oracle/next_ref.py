"""ORACLE / TEST INFRASTRUCTURE — not product code.

The checker's own restatement of a Stage's ``next`` as the reference applies it to an object
(playStage, pkg/kwok/controllers/pod_controller.go:290-360; node_controller.go:355-424):

* finalizers: the JSON-patch ops of finalizersModify come from refcpu (C++,
  pkg/utils/lifecycle/finalizers.go:83-111) and are applied by ``json_patch`` below;
* delete: the object is gone (next.go:68-70);
* patches: ``statusTemplate`` is one merge patch rooted at ``status``
  (pkg/apis/internalversion/conversion.go:395-425), rendered by text/template + sprig and
  YAMLToJSON (pkg/utils/gotpl/renderer.go:59-124), applied as an RFC 7386 merge patch; the
  object changed iff the result differs (checkNeedPatch, controllers/utils.go:162-304).

The oracle does not interpret templates.  Every status template the reference ships
(kustomize/stage/**) is restated below as a plain function of the object, identified by the
sha256 of its text, each citing its YAML; a template with no actions renders to itself.  Any
other template raises — the checker never guesses.  The restatements are pinned on the
reference's golden outputs (kustomize/stage/**/testdata, tests/golden/stages) and, for
pod-general / pod-chaos (no reference fixture), on the hand-derived expected patches of
tests/golden/pod_general_next.json.

Nothing here imports the product package.
"""
from __future__ import annotations

import copy
import datetime as _dt
import hashlib
import json
import re
from typing import Callable, Dict, List, Optional, Tuple

from . import refcpu
from .typed_json import to_json_standard


class RenderError(RuntimeError):
    """The reference's template execution would fail (e.g. `index` out of range)."""


# pkg/utils/gotpl/funcs.go:85-116 (corev1.NodeCondition list behind NodeConditions)
NODE_CONDITIONS = [
    ("Ready", "True", "KubeletReady", "kubelet is posting ready status"),
    ("MemoryPressure", "False", "KubeletHasSufficientMemory", "kubelet has sufficient memory available"),
    ("DiskPressure", "False", "KubeletHasNoDiskPressure", "kubelet has no disk pressure"),
    ("PIDPressure", "False", "KubeletHasSufficientPID", "kubelet has sufficient PID available"),
    ("NetworkUnavailable", "False", "RouteCreated", "RouteController created a route"),
]


def format_rfc3339nano(ns: int) -> str:
    """time.Time.UTC().Format(time.RFC3339Nano): fraction with trailing zeros dropped."""
    sec = ns // 10**9
    frac = ns - sec * 10**9
    t = _dt.datetime(1970, 1, 1) + _dt.timedelta(seconds=sec)
    out = "%04d-%02d-%02dT%02d:%02d:%02d" % (t.year, t.month, t.day, t.hour, t.minute, t.second)
    if frac:
        out += "." + ("%09d" % frac).rstrip("0")
    return out + "Z"


class Funcs:
    """The template functions a controller hands the renderer.  ``concrete``: fixed stand-ins
    for the node / pod IP pools (pod_controller.go, node_controller.go funcMaps); ``placeholder``:
    the stage tester's wrappers, which print the call (pkg/tools/stage/stage.go:128-151)."""

    def __init__(self, now_ns: int = 0, placeholder: bool = False, version: str = "v0.6.0"):
        self.placeholder = placeholder
        self.now_ns = now_ns
        self.ver = version

    @staticmethod
    def _gorepr(v) -> str:  # %#v of the argument values the templates pass
        if isinstance(v, bool):
            return "true" if v else "false"
        if isinstance(v, str):
            return json.dumps(v)
        if v is None:
            return "interface {}(nil)"
        return str(v)

    def _ph(self, name, *args):
        if not args:
            return f"<{name}>"
        return f"<{name}(" + ", ".join(self._gorepr(a) for a in args) + ")>"

    def now(self):
        return self._ph("Now") if self.placeholder else format_rfc3339nano(self.now_ns)

    def version(self):
        return self._ph("Version") if self.placeholder else self.ver

    def node_ip(self):
        return self._ph("NodeIP") if self.placeholder else "10.0.0.1"

    def node_name(self):
        return self._ph("NodeName") if self.placeholder else "node"

    def node_port(self):
        return self._ph("NodePort") if self.placeholder else 10250

    def node_ip_with(self, node):
        return self._ph("NodeIPWith", node) if self.placeholder else "10.0.0.1"

    def pod_ip_with(self, node, host_network, uid, name, namespace):
        if self.placeholder:
            return self._ph("PodIPWith", node, host_network, uid, name, namespace)
        return "10.0.0.2"


# ------------------------------------------------------------------ template value helpers
def _get(o, *path):
    for k in path:
        if not isinstance(o, dict):
            return None
        o = o.get(k)
    return o


def _or(*vals):
    """sprig/text-template `or`: the first truthy argument, else the last."""
    for v in vals:
        if v:
            return v
    return vals[-1]


def _index_check(lst, i: int, what: str):
    """`index $root.status.<list> $index` (the templates bind it to $origin)."""
    if lst is None:
        raise RenderError(f"index of untyped nil ({what})")
    if not isinstance(lst, list) or i >= len(lst):
        raise RenderError(f"index out of range: {i} ({what})")


def _quoted(v):
    """`{{ v | Quote }}` read back by YAML: the value as a string (funcs.go:43-55)."""
    if isinstance(v, str):
        return v
    if v is None:
        return "null"
    return json.dumps(v, separators=(",", ":"))


_INT = re.compile(r"^[-+]?(0|[1-9][0-9]*)$")
_FLOAT = re.compile(r"^[-+]?([0-9]+\.[0-9]*|\.[0-9]+)([eE][-+]?[0-9]+)?$")


def _bare(v):
    """A value printed unquoted into the YAML (`{{ v }}`) and read back: the scalar types the
    shipped templates can produce (ints, bools, null, strings; floats for completeness)."""
    if not isinstance(v, str):
        return v
    if _INT.match(v):
        return int(v)
    if v in ("true", "True", "TRUE"):
        return True
    if v in ("false", "False", "FALSE"):
        return False
    if v in ("", "~", "null", "Null", "NULL"):
        return None
    if _FLOAT.match(v):
        return float(v)
    return v


def _list_or_null(xs):
    """`key:` followed by an empty range renders as null."""
    return xs if xs else None


def _pod_ips(obj, F):
    spec = obj.get("spec") or {}
    md = obj.get("metadata") or {}
    node = spec.get("nodeName")
    return F.node_ip_with(node), F.pod_ip_with(node, _or(spec.get("hostNetwork"), False), _or(md.get("uid"), ""),
                                               _or(md.get("name"), ""), _or(md.get("namespace"), ""))


def _containers(obj, key="containers"):
    return (obj.get("spec") or {}).get(key) or []


def _running(c, now, started=None):
    d = {"image": _quoted(c.get("image")), "name": _quoted(c.get("name")), "ready": True, "restartCount": 0}
    if started is not None:
        d["started"] = started
    d["state"] = {"running": {"startedAt": now}}
    return d


def _terminated(c, now, ready, started=False, exit_code=0, reason="Completed", message=None):
    term = {"exitCode": exit_code, "finishedAt": now, "reason": reason}
    if message is not None:
        term["message"] = message
    term["startedAt"] = now
    d = {"image": _quoted(c.get("image")), "name": _quoted(c.get("name")), "ready": ready, "restartCount": 0}
    if started is not None:
        d["started"] = started
    d["state"] = {"terminated": term}
    return d


def _waiting(c, reason):
    return {"image": _quoted(c.get("image")), "name": _quoted(c.get("name")), "ready": False, "restartCount": 0,
            "started": False, "state": {"waiting": {"reason": reason}}}


def _readiness_gates(obj, now):
    return [{"lastTransitionTime": now, "status": "True", "type": _quoted(g.get("conditionType"))}
            for g in (obj.get("spec") or {}).get("readinessGates") or []]


def _node_conditions(now, ltt, override=None):
    out = []
    for t, st, reason, msg in NODE_CONDITIONS:
        c = {"lastHeartbeatTime": now, "lastTransitionTime": _quoted(ltt), "message": msg, "reason": reason,
             "status": st, "type": t}
        if override is not None:
            c = override(c)
        out.append(c)
    return out


def _node_addresses(obj, F):
    have = _get(obj, "status", "addresses")
    if have:
        return copy.deepcopy(have)
    out = []
    if F.node_ip():
        out.append({"address": _quoted(F.node_ip()), "type": "InternalIP"})
    if F.node_name():
        out.append({"address": _quoted(F.node_name()), "type": "Hostname"})
    return _list_or_null(out)


# ------------------------------------------------------------------ the shipped templates
def _pod_fast_ready(obj, F):
    """kustomize/stage/pod/fast/pod-ready.yaml:21-73"""
    now = F.now()
    conds = [{"lastTransitionTime": now, "status": "True", "type": t} for t in ("Initialized", "Ready", "ContainersReady")]
    conds += _readiness_gates(obj, now)
    ics = []
    for c in _containers(obj, "initContainers"):
        if c.get("restartPolicy") == "Always":  # eq of a missing field and a string is false
            ics.append(_running(c, now, started=True))
        else:
            ics.append(_terminated(c, now, ready=True, started=None))
    hip, pip = _pod_ips(obj, F)
    return {"conditions": conds, "containerStatuses": _list_or_null([_running(c, now) for c in _containers(obj)]),
            "initContainerStatuses": _list_or_null(ics), "hostIP": hip, "podIP": pip, "phase": "Running",
            "startTime": now}


def _pod_fast_complete(obj, F):
    """kustomize/stage/pod/fast/pod-complete.yaml:24-43"""
    now = F.now()
    cs = []
    for i, c in enumerate(_containers(obj)):
        _index_check(_get(obj, "status", "containerStatuses"), i, "status.containerStatuses")
        cs.append(_terminated(c, now, ready=False))
    return {"containerStatuses": _list_or_null(cs), "phase": "Succeeded"}


def _pod_general_create(obj, F):
    """kustomize/stage/pod/general/pod-create.yaml:28-103"""
    now = F.now()
    init = _containers(obj, "initContainers")
    names = lambda cs: "[" + "".join(f" {c.get('name')} " for c in cs) + "]"  # noqa: E731
    if init:
        conds = [{"lastProbeTime": None, "lastTransitionTime": now,
                  "message": "containers with incomplete status: " + names(init), "reason": "ContainersNotInitialized",
                  "status": "False", "type": "Initialized"}]
    else:
        conds = [{"lastProbeTime": None, "lastTransitionTime": now, "status": "True", "type": "Initialized"}]
    for t in ("Ready", "ContainersReady"):
        conds.append({"lastProbeTime": None, "lastTransitionTime": now,
                      "message": "containers with unready status: " + names(_containers(obj)),
                      "reason": "ContainersNotReady", "status": "False", "type": t})
    conds += _readiness_gates(obj, now)
    hip, pip = _pod_ips(obj, F)
    out = {"conditions": conds}
    if init:
        out["initContainerStatuses"] = [_waiting(c, "PodInitializing") for c in init]
        out["containerStatuses"] = _list_or_null([_waiting(c, "PodInitializing") for c in _containers(obj)])
    else:
        out["containerStatuses"] = _list_or_null([_waiting(c, "ContainerCreating") for c in _containers(obj)])
    out.update({"hostIP": hip, "podIP": pip, "phase": "Pending"})
    return out


def _pod_general_init_running(obj, F):
    """kustomize/stage/pod/general/pod-init-container-running.yaml:30-45"""
    now = F.now()
    ics = []
    for i, c in enumerate(_containers(obj, "initContainers")):
        _index_check(_get(obj, "status", "initContainerStatuses"), i, "status.initContainerStatuses")
        ics.append(_running(c, now, started=True))
    return {"initContainerStatuses": _list_or_null(ics)}


def _pod_general_init_completed(obj, F):
    """kustomize/stage/pod/general/pod-init-container-completed.yaml:28-60"""
    now = F.now()
    conds = [{"lastProbeTime": None, "lastTransitionTime": now, "status": "True", "reason": "", "type": "Initialized"}]
    ics = []
    for i, c in enumerate(_containers(obj, "initContainers")):
        _index_check(_get(obj, "status", "initContainerStatuses"), i, "status.initContainerStatuses")
        ics.append(_terminated(c, now, ready=True))
    cs = [_waiting(c, "ContainerCreating") for c in _containers(obj)]
    return {"conditions": conds, "initContainerStatuses": _list_or_null(ics), "containerStatuses": _list_or_null(cs)}


def _pod_general_ready(obj, F):
    """kustomize/stage/pod/general/pod-ready.yaml:30-58"""
    now = F.now()
    conds = [{"lastProbeTime": None, "lastTransitionTime": now, "message": "", "reason": "", "status": "True", "type": t}
             for t in ("Ready", "ContainersReady")]
    cs = []
    for i, c in enumerate(_containers(obj)):
        _index_check(_get(obj, "status", "containerStatuses"), i, "status.containerStatuses")
        cs.append(_running(c, now, started=True))
    return {"conditions": conds, "containerStatuses": _list_or_null(cs), "phase": "Running"}


def _pod_general_complete(obj, F):
    """kustomize/stage/pod/general/pod-complete.yaml:31-51"""
    now = F.now()
    cs = []
    for i, c in enumerate(_containers(obj)):
        _index_check(_get(obj, "status", "containerStatuses"), i, "status.containerStatuses")
        cs.append(_terminated(c, now, ready=True))
    return {"containerStatuses": _list_or_null(cs), "phase": "Succeeded"}


def _chaos_params(obj, stage, default_reason, default_message):
    ann = _or(_get(obj, "metadata", "annotations"), {})
    p = f"{stage}.stage.kwok.x-k8s.io/"
    return (_or(ann.get(p + "container-name"), ""), _or(ann.get(p + "reason"), default_reason),
            _or(ann.get(p + "message"), default_message), _or(ann.get(p + "exit-code"), 1))


def _pod_chaos_container_failed(obj, F):
    """kustomize/stage/pod/chaos/pod-container-running-failed.yaml:23-76"""
    now = F.now()
    name, reason, message, code = _chaos_params(obj, "pod-container-running-failed", "containerFailed",
                                                "container failed")
    conds = [{"lastProbeTime": None, "lastTransitionTime": now, "status": "True", "reason": "", "type": "Initialized"},
             {"lastTransitionTime": now, "status": "False", "reason": "", "type": "Ready"},
             {"lastTransitionTime": now, "status": "False", "reason": "", "type": "ContainersReady"}]
    cs = []
    for c in _containers(obj):
        if not name or c.get("name") == name:
            cs.append(_terminated(c, now, ready=False, exit_code=_bare(str(code)), reason=_bare(str(reason)),
                                  message=_bare(str(message))))
        else:
            cs.append(_running(c, now))
    hip, pip = _pod_ips(obj, F)
    return {"conditions": conds, "containerStatuses": _list_or_null(cs), "hostIP": hip, "podIP": pip,
            "phase": "Failed", "startTime": now}


def _pod_chaos_init_failed(obj, F):
    """kustomize/stage/pod/chaos/pod-init-container-running-failed.yaml:23-88"""
    now = F.now()
    name, reason, message, code = _chaos_params(obj, "pod-init-container-running-failed", "initContainerError",
                                                "initContainer reported errors")
    conds = [{"lastProbeTime": None, "lastTransitionTime": now, "status": "False", "reason": "", "type": "Initialized"},
             {"lastTransitionTime": now, "status": "False", "reason": "", "type": "Ready"},
             {"lastTransitionTime": now, "status": "False", "reason": "", "type": "ContainersReady"}]
    ics = []
    for c in _containers(obj, "initContainers"):
        if not name or c.get("name") == name:
            ics.append(_terminated(c, now, ready=False, exit_code=_bare(str(code)), reason=_bare(str(reason)),
                                   message=_bare(str(message))))
        else:
            ics.append(_terminated(c, now, ready=True, started=None))
    cs = [_waiting(c, "PodInitializing") for c in _containers(obj)]
    hip, pip = _pod_ips(obj, F)
    return {"conditions": conds, "initContainerStatuses": _list_or_null(ics), "containerStatuses": _list_or_null(cs),
            "hostIP": hip, "podIP": pip, "phase": "Failed", "startTime": now}


def _node_initialize(obj, F):
    """kustomize/stage/node/fast/node-initialize.yaml:16-79"""
    now = F.now()
    ltt = _or(_get(obj, "metadata", "creationTimestamp"), now)
    out = {"conditions": _node_conditions(now, ltt), "addresses": _node_addresses(obj, F)}
    if F.node_port():
        out["daemonEndpoints"] = {"kubeletEndpoint": {"Port": _bare(str(F.node_port()))}}
    default = {"cpu": "1k", "memory": "1Ti", "pods": "1M"}
    out["allocatable"] = copy.deepcopy(_or(_get(obj, "status", "allocatable"), default))
    out["capacity"] = copy.deepcopy(_or(_get(obj, "status", "capacity"), default))
    ni = _get(obj, "status", "nodeInfo") or {}
    kv = "kwok-" + str(F.version())
    out["nodeInfo"] = {
        "architecture": _bare(str(_or(ni.get("architecture"), "amd64"))),
        "bootID": _bare(str(ni["bootID"])) if ni.get("bootID") else "",
        "containerRuntimeVersion": _bare(str(_or(ni.get("containerRuntimeVersion"), kv))),
        "kernelVersion": _bare(str(_or(ni.get("kernelVersion"), kv))),
        "kubeProxyVersion": _bare(str(_or(ni.get("kubeProxyVersion"), kv))),
        "kubeletVersion": _bare(str(_or(ni.get("kubeletVersion"), kv))),
        "machineID": _bare(str(ni["machineID"])) if ni.get("machineID") else "",
        "operatingSystem": _bare(str(_or(ni.get("operatingSystem"), "linux"))),
        "osImage": _bare(str(ni["osImage"])) if ni.get("osImage") else "",
        "systemUUID": _bare(str(ni["systemUUID"])) if ni.get("systemUUID") else "",
    }
    out["phase"] = "Running"
    return out


def _node_heartbeat(obj, F):
    """kustomize/stage/node/heartbeat/node-heartbeat.yaml:24-35"""
    now = F.now()
    return {"conditions": _node_conditions(now, _or(_get(obj, "metadata", "creationTimestamp"), now))}


def _node_heartbeat_with_lease(obj, F):
    """kustomize/stage/node/heartbeat-with-lease/node-heartbeat-with-lease.yaml:24-54"""
    now = F.now()
    out = {"conditions": _node_conditions(now, _or(_get(obj, "metadata", "creationTimestamp"), now)),
           "addresses": _node_addresses(obj, F)}
    if F.node_port():
        out["daemonEndpoints"] = {"kubeletEndpoint": {"Port": _bare(str(F.node_port()))}}
    return out


def _node_not_ready(obj, F):
    """kustomize/stage/node/chaos/node-not-ready.yaml:30-66"""
    now = F.now()
    ann = _or(_get(obj, "metadata", "annotations"), {})
    p = "node-not-ready.stage.kwok.x-k8s.io/"
    ftype = _or(ann.get(p + "type"), "")
    reason = _or(ann.get(p + "reason"), "nodeFailed")
    message = _or(ann.get(p + "message"), "node failed")

    def override(c):
        if c["type"] == "Ready":
            return dict(c, message=_quoted(message), reason=_quoted(reason), status="False")
        if c["type"] == ftype:
            return dict(c, message=_quoted(message), reason=_quoted(reason), status="True")
        return c

    return {"conditions": _node_conditions(now, _or(_get(obj, "metadata", "creationTimestamp"), now), override)}


# sha256 of each shipped statusTemplate (the text as the YAML decodes it) -> its restatement
TEMPLATES: Dict[str, Tuple[str, Callable]] = {
    "47b5d6f368c074da": ("pod/fast/pod-ready", _pod_fast_ready),
    "1fe329758ca19907": ("pod/fast/pod-complete", _pod_fast_complete),
    "da0c20a946426d52": ("pod/general/pod-create", _pod_general_create),
    "004a6db424df147d": ("pod/general/pod-init-container-running", _pod_general_init_running),
    "a07eca9635a4dba6": ("pod/general/pod-init-container-completed", _pod_general_init_completed),
    "e9497b20d12a6974": ("pod/general/pod-ready", _pod_general_ready),
    "a7dc03cef8bc7e97": ("pod/general/pod-complete", _pod_general_complete),
    "35aa8453ab842050": ("pod/chaos/pod-container-running-failed", _pod_chaos_container_failed),
    "f5175f64264b0d8b": ("pod/chaos/pod-init-container-running-failed", _pod_chaos_init_failed),
    "0a93b9241f101ae9": ("node/fast/node-initialize", _node_initialize),
    "5cf30ae4f1e49abe": ("node/heartbeat/node-heartbeat", _node_heartbeat),
    "62b0991db315f0cb": ("node/heartbeat-with-lease/node-heartbeat-with-lease", _node_heartbeat_with_lease),
    "760e1202d2c2c056": ("node/chaos/node-not-ready", _node_not_ready),
}


def template_key(text: str) -> str:
    return hashlib.sha256(text.encode()).hexdigest()[:16]


def render_status(text: str, obj: dict, F: Funcs):
    """The status patch a statusTemplate renders for obj (renderer.go:59-124 + YAMLToJSON)."""
    if "{{" not in text:  # no actions: the text is the output
        import yaml
        return yaml.safe_load(text)
    hit = TEMPLATES.get(template_key(text))
    if hit is None:
        raise NotImplementedError("oracle: no restatement of this status template "
                                  f"(sha256 {template_key(text)}); only kwok's shipped templates are covered")
    return hit[1](obj, F)


# ------------------------------------------------------------------ patch application
def merge_patch(target, patch):
    """RFC 7386: objects merge key by key, null deletes, anything else replaces."""
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    out = copy.deepcopy(target) if isinstance(target, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        elif isinstance(v, dict):
            out[k] = merge_patch(out.get(k), v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def json_patch(obj, ops):
    """RFC 6902 add / remove, as finalizersModify emits them (/metadata/finalizers[/i|/-])."""
    obj = copy.deepcopy(obj)
    for op in ops:
        parts = [p.replace("~1", "/").replace("~0", "~") for p in op["path"].split("/")[1:]]
        node = obj
        for p in parts[:-1]:
            node = node[int(p)] if isinstance(node, list) else node.setdefault(p, {})
        last = parts[-1]
        if op["op"] == "add":
            if isinstance(node, list):
                node.insert(len(node) if last == "-" else int(last), copy.deepcopy(op["value"]))
            else:
                node[last] = copy.deepcopy(op["value"])
        elif op["op"] == "remove":
            if isinstance(node, list):
                node.pop(int(last))
            else:
                node.pop(last)
        else:
            raise ValueError(f"oracle: json patch op {op['op']!r}")
    return obj


def omitempty(obj):
    """The apiserver stores typed objects: what a patch empties vanishes (omitempty), and a
    query sees the typed presence (ToJSONStandard): typed_json.to_json_standard."""
    return to_json_standard(obj)


def _canon(o) -> str:
    return json.dumps(o, sort_keys=True, separators=(",", ":"))


def strip_for_recreate(obj: dict) -> dict:
    """The workload harness re-creates a deleted object from its spec: no status,
    deletionTimestamp, deletionGracePeriodSeconds or finalizers."""
    o = copy.deepcopy(obj)
    o.pop("status", None)
    md = o.setdefault("metadata", {})
    for k in ("deletionTimestamp", "deletionGracePeriodSeconds", "finalizers"):
        md.pop(k, None)
    return o


class StageNext:
    """One Stage's next (v1alpha1 document) and its effect on an object."""

    def __init__(self, doc: dict, lifecycle: "refcpu.Lifecycle", index: int):
        self.name = doc["metadata"]["name"]
        n = (doc.get("spec") or {}).get("next") or {}
        self.delete = bool(n.get("delete"))
        self.has_fin = n.get("finalizers") is not None
        self.lc, self.index = lifecycle, index
        patches = list(n.get("patches") or [])
        if n.get("statusTemplate") and not patches:  # conversion.go:401-422
            patches = [{"root": "status", "template": n["statusTemplate"], "type": "merge",
                        "subresource": n.get("statusSubresource") or "status"}]
        for p in patches:
            if (p.get("type") or "merge") != "merge" or p.get("root") != "status":
                raise NotImplementedError("oracle: only statusTemplate merge patches are restated")
        self.templates = [p["template"] for p in patches]

    def patches(self, obj, F: Funcs) -> List[dict]:
        return [{"status": render_status(t, obj, F)} for t in self.templates]

    def apply(self, obj: dict, F: Funcs) -> Tuple[Optional[dict], bool]:
        """-> (object after the fire or None if deleted, whether it changed)."""
        changed = False
        if self.has_fin:
            ops = self.lc.finalizers(self.index, (obj.get("metadata") or {}).get("finalizers"))
            if ops:
                new = omitempty(json_patch(obj, ops))
                changed = _canon(new) != _canon(obj)
                obj = new
        if self.delete:
            return None, True
        for patch in self.patches(obj, F):
            new = omitempty(merge_patch(obj, patch))
            if _canon(new) != _canon(obj):
                changed = True
                obj = new
        return obj, changed


def load_stage_docs(*paths) -> List[dict]:
    import yaml
    out = []
    for p in paths:
        with open(p) as f:
            out += [d for d in yaml.safe_load_all(f) if d and d.get("kind") == "Stage"]
    return out
