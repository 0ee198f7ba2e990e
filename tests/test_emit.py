"""Device patch emission, host half (CPU): the skeletons libkwok_patch builds (kwk_patch_skeleton)
filled with Now and the objects' call values equal kwk_patch_render byte for byte for every object
kwk_patch_object_values accepts; the status guard decides exactly the objects whose render fails;
ineligible templates are refused with their reason; libkwok_emit exports its ABI.

Reference: pkg/utils/lifecycle/next.go:73-160 and pkg/utils/gotpl/renderer.go:59-124 (the render
the skeleton stands for); the guard is the `$origin := index $root.status.containerStatuses $index`
line of kustomize/stage/pod/general/pod-ready.yaml / pod-complete.yaml and the init-container
Stages.  The GPU half (tests/test_gpu_emit.py) checks the device's bytes."""
import collections
import ctypes as C
import json

import pytest

from kwok_amd.host import emit, patchtpl
from kwok_amd.host.compiler import class_key
from kwok_amd.host.stages import load_stage_files, stage_from_v1alpha1
from tests.test_patch import FILES, FUNCS, NOW, _workload_states


def _pod_program():
    stages = [s for s in load_stage_files(*FILES) if s.kind == "Pod"]
    return stages, patchtpl.PatchProgram(stages, FUNCS)


def _classes(objs):
    keys, cls, reps = {}, [], {}
    for o in objs:
        c = keys.setdefault(class_key(o), len(keys))
        reps.setdefault(c, o)
        cls.append(c)
    return cls, reps


@pytest.mark.parametrize("config", ["C1", "C2"])
def test_skeleton_fill_equals_native_render(config):
    _, states = _workload_states(config, 10, 400, seed=73)
    stages, pp = _pod_program()
    pods = [o for o in states if o.get("kind", "Pod") == "Pod"]
    cls, reps = _classes(pods)
    ep = emit.EmitProgram(stages, pp, reps, len(reps))
    counts = collections.Counter()
    by = collections.defaultdict(list)
    for o, c in zip(pods, cls):
        by[c].append(o)
    for (c, tid), sk in sorted(ep.skel.items()):
        group = by[c]
        vals, ok = pp.object_values(tid, group, sk["text"], sk["calls"], ep.stride)
        got = pp.render([tid] * len(group), group, NOW)
        for o, v, k, g in zip(group, vals, ok, got):
            assert k, (c, tid, "an object of the class not accepted")
            values = [bytes(v[j][1:1 + v[j][0]]).decode() for j in range(sk["calls"])]
            guard_ok = all(emit.guard_holds(o, gd) for gd in sk["guard_list"])
            if not guard_ok:  # the render fails (index out of range / of nil): the host's
                assert g is None, (c, tid)
                counts["guard"] += 1
                continue
            assert g is not None, (c, tid, "guard met but the native render failed")
            assert emit.substitute(sk, NOW, values) == g, (c, tid)
            counts["ok"] += 1
    assert counts["ok"] > 1000 and counts["guard"] > 0, counts
    assert ep.guards and ep.guards[0] == (("status", "containerStatuses"), ("spec", "containers"))


def test_unquoted_value_slot_is_ineligible():
    """a skeleton whose Now / call-value slot sits outside a JSON string (a template
    rendering a number or bool there) cannot be analysed with stand-in text; EmitProgram marks
    that (class, template) ineligible with a reason instead of raising."""
    _, states = _workload_states("C2", 10, 100, seed=75)
    stages, pp = _pod_program()
    pods = [o for o in states if o.get("kind", "Pod") == "Pod"]
    cls, reps = _classes(pods)
    first = emit.EmitProgram(stages, pp, reps, len(reps))
    (c0, t0), sk0 = sorted(first.skel.items())[0]

    class Unquoted:  # the native program, with one skeleton's first slot moved out of its string
        def __init__(self, inner):
            self.inner = inner

        def __getattr__(self, name):
            return getattr(self.inner, name)

        def skeleton(self, tid, rep):
            sk = self.inner.skeleton(tid, rep)
            if tid == t0 and sk["eligible"] and sk["slots"]:
                sk = dict(sk, lits=['{"n": '] + ['0, "m": "'] * (len(sk["slots"]) - 1) + ['"}'] if len(sk["slots"]) > 1
                          else ['{"n": ', '}'])
            return sk

    ep = emit.EmitProgram(stages, Unquoted(pp), reps, len(reps))
    bad = [k for k in first.skel if k[1] == t0 and first.skel[k]["slots"]]
    assert bad and all(k not in ep.skel for k in bad)
    assert all(ep.reasons[k] == "a value slot outside a JSON string" for k in bad)
    assert set(ep.skel) == set(first.skel) - set(bad)


def test_emit_program_guard_effects():
    _, states = _workload_states("C2", 10, 400, seed=74)
    stages, pp = _pod_program()
    pods = [o for o in states if o.get("kind", "Pod") == "Pod"]
    cls, reps = _classes(pods)
    ep = emit.EmitProgram(stages, pp, reps, len(reps))
    names = {tid: stages[si].name for (si, pi), tid in pp.template_of.items()}
    tmpl = {tid: stages[si].next.patches[pi].template for (si, pi), tid in pp.template_of.items()}
    gbit = 1 << ep.guards.index((("status", "containerStatuses"), ("spec", "containers")))
    seen = set()
    for (c, tid), sk in ep.skel.items():
        n = names[tid]
        if not reps[c].get("spec", {}).get("containers"):
            continue
        if "index $root.status.containerStatuses" in tmpl[tid]:  # render needs the guard, the patch keeps it met
            assert sk["need"] & gbit and sk["set"] & gbit and not sk["keep"] & gbit, (n, sk["need"], sk["set"])
            seen.add(n)
        if n == "pod-create" and "range .spec.containers" in tmpl[tid]:  # writes one status per container: the guard holds afterwards
            assert not sk["need"] & gbit and sk["set"] & gbit, (n, sk["keep"], sk["set"])
            seen.add(n)
    assert {"pod-ready", "pod-complete", "pod-create"} <= seen
    for c, rep in reps.items():  # re-created from spec: no container statuses
        assert ep.fresh_bits(c) & gbit == (0 if rep.get("spec", {}).get("containers") else gbit)


def _stage(name, template):
    return stage_from_v1alpha1({
        "apiVersion": "kwok.x-k8s.io/v1alpha1", "kind": "Stage", "metadata": {"name": name},
        "spec": {"resourceRef": {"apiGroup": "v1", "kind": "Pod"}, "selector": {},
                 "next": {"statusTemplate": template}}})


POD = {"apiVersion": "v1", "kind": "Pod",
       "metadata": {"name": "p", "namespace": "d", "uid": "u1", "labels": {"a": "b"}},
       "spec": {"nodeName": "n1", "containers": [{"name": "c", "image": "i"}]},
       "status": {"phase": "Pending", "hostIP": "10.0.0.9"}}


@pytest.mark.parametrize("template,reason", [
    ("phase: {{ .status.phase }}\n", "per-object data reaches the output or a test"),
    ("phase: '{{ .metadata.name }}'\n", "per-object data reaches the output or a test"),
    ("startTime: {{ Now }}\n", "a Now / call value is tested or transformed"),
    ("phase: x\n{{ if .metadata.labels }}\nreason: y\n{{ end }}\n", "per-object data reaches the output or a test"),
    ("podIP: {{ PodIPWith .status.hostIP | Quote }}\n", "a call argument reads status"),
    ("a: {{ index .status.conditions 0 | Quote }}\n", "per-object data indexed"),
    ("{{ $now := Now }}\nphase: x\n{{ if eq $now \"x\" }}\nreason: y\n{{ end }}\n",
     "a Now / call value is tested or transformed"),
])
def test_skeleton_ineligible(template, reason):
    pp = patchtpl.PatchProgram([_stage("s", template)], FUNCS)
    assert (0, 0) in pp.template_of, pp.unsupported
    sk = pp.skeleton(0, POD)
    assert not sk["eligible"] and sk["reason"] == reason, sk


def test_skeleton_eligible_slots():
    t = ("hostIP: {{ NodeIPWith .spec.nodeName | Quote }}\nmessage: 'at {{ Now }} on {{ .spec.containers | len }}'\n"
         "phase: Running\n")
    pp = patchtpl.PatchProgram([_stage("s", t)], FUNCS)
    sk = pp.skeleton(0, POD)
    assert sk["eligible"] and sk["calls"] == 1 and sorted(sk["slots"]) == [0, 1] and not sk["guards"], sk
    other = json.loads(json.dumps(POD))
    other["metadata"].update(name="q", uid="u2")
    other["spec"]["nodeName"] = "n2"
    other["status"] = {"phase": "Running"}
    vals, ok = pp.object_values(0, [POD, other], sk["text"], 1, 32)
    got = pp.render([0, 0], [POD, other], NOW)
    for v, k, g in zip(vals, ok, got):
        assert k and g == emit.substitute(sk, NOW, [bytes(v[0][1:1 + v[0][0]]).decode()])
    # a value JSON would escape is refused per object (the host renders it)
    pp2 = patchtpl.PatchProgram([_stage("s", t)], dict(FUNCS, NodeIPWith=lambda n: 'a"b'))
    vals, ok = pp2.object_values(0, [POD], sk["text"], 1, 32)
    assert ok[0] == 0 and vals[0][0][0] == 0xFF


def test_emit_library_exports():
    from kwok_amd.host import abi
    abi.lib()
    L = C.CDLL(emit.LIB_PATH)
    for name in emit.EXPORTS:
        assert hasattr(L, name), name
    hdr = open(emit.LIB_PATH.replace("kwok_amd/lib/libkwok_emit.so", "include/kwok_emit.h")).read()
    import re
    declared = set(re.findall(r"\b(kwk_emit\w*|kwk_emitter_\w+)\s*\(", hdr)) - {"kwk_emit_piece", "kwk_emit_skel"}
    declared = {d for d in declared if not d.isupper()}
    assert declared <= set(emit.EXPORTS), declared - set(emit.EXPORTS)
    plib = patchtpl.lib()
    for name in ("kwk_patch_skeleton", "kwk_patch_object_values"):
        assert hasattr(plib, name)
