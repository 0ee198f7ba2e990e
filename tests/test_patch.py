"""Native patch renderer (kwok_amd/csrc/patch.cpp, include/kwok_patch.h; SURVEY.md §8(f)
rank 2): precompiled merge-patch byte templates against

* the reference's golden patches (kustomize/stage/**/testdata/*.output.yaml, rendered with
  the stage tester's placeholder functions, pkg/tools/stage/stage.go:128-193);
* the oracle's independent restatement of every shipped template (oracle/next_ref.py);
* the host renderer's bytes (gotpl.Renderer.to_json + encoding/json Marshal), byte for byte,
  on the C1 / C2 workloads, the compiler's explored states and their successors, and edge
  values (HTML-escaped characters, unicode, line separators, numbers, raw chaos parameters);
plus its throughput (objects/s, reported, not asserted).  All CPU: the renderer is host code."""
import copy
import glob
import hashlib
import json
import os
import time

import pytest
import yaml

from kwok_amd import workload as W
from kwok_amd.host import gotpl, patchtpl
from kwok_amd.host.compiler import HarnessSpec, KindProgram, exploration_funcs
from kwok_amd.host.nextstate import apply_next
from kwok_amd.host.stages import load_stage_files, stage_from_v1alpha1

HERE = os.path.dirname(os.path.abspath(__file__))
STAGE_DIR = os.path.join(HERE, "golden", "stages")
NOW = 1_700_000_000_123_456_789
SHIPPED = os.path.join(os.path.dirname(HERE), "kwok_amd", "stages")
FILES = sorted(glob.glob(os.path.join(SHIPPED, "**", "*.yaml"), recursive=True))


def _ip(prefix, *args):
    h = hashlib.sha256(json.dumps([str(a) for a in args]).encode()).digest()
    return f"{prefix}.{h[0]}.{h[1]}"


FUNCS = {"NodeIPWith": lambda node: _ip("10.1", node), "PodIPWith": lambda *a: _ip("10.2", *a),
         "NodeIP": lambda: "10.0.0.1", "NodeName": lambda: "node", "NodePort": lambda: 10250,
         "PodIP": lambda: "10.0.0.2"}


def _program(stages, funcs=FUNCS, **kw):
    return patchtpl.PatchProgram(stages, funcs, **kw)


def _compare(pp, stages, objs, renderer, allow_fallback=()):
    """native bytes == host bytes wherever native renders; NEEDS_RENDER only where the host
    renderer fails or the object holds a value listed in allow_fallback."""
    counts = {"ok": 0, "host_error": 0, "fallback": 0}
    for (si, pi), tid in pp.template_of.items():
        st = stages[si]
        p = st.next.patches[pi]
        kind_objs = [o for o in objs if o.get("kind", "Pod") == st.kind]
        if not kind_objs:
            continue
        got = pp.render([tid] * len(kind_objs), kind_objs, NOW)
        for o, g in zip(kind_objs, got):
            try:
                want = patchtpl.render_patch_bytes(p.template, p.root, o, renderer)
            except (gotpl.TemplateError, yaml.YAMLError):  # the reference's render fails too
                want = None
            if g is None:
                if want is None:
                    counts["host_error"] += 1
                    continue
                assert any(v in json.dumps(o, ensure_ascii=False) for v in allow_fallback), (st.name, o)
                counts["fallback"] += 1
                continue
            assert want is not None, (st.name, "native rendered where the template fails", o)
            assert g == want, (st.name, g, want)
            counts["ok"] += 1
    return counts


def test_shipped_templates_compile():
    stages = load_stage_files(*FILES)
    pp = _program(stages)
    names = {stages[si].name for si, _ in pp.unsupported}
    # node-initialize / node-heartbeat-with-lease embed {{ with }} + {{ YAML . 1 }} (one fire per
    # node lifetime / lease-renewed nodes): the host renderer keeps them
    assert names == {"node-initialize", "node-heartbeat-with-lease"}
    compiled = {stages[si].name for si, _ in pp.template_of}
    assert {"pod-ready", "pod-complete", "pod-create", "pod-init-container-running", "pod-init-container-completed",
            "pod-container-running-failed", "pod-init-container-running-failed", "node-heartbeat",
            "node-not-ready"} <= compiled


def _golden_cases():
    return sorted(glob.glob(os.path.join(STAGE_DIR, "**", "testdata", "*.input.yaml"), recursive=True))


@pytest.mark.parametrize("path", _golden_cases(), ids=lambda p: os.path.relpath(p, STAGE_DIR))
def test_reference_golden_patches(path):
    """The reference's rendered patches (placeholder functions, as the stage tester)."""
    from tests.test_oracle_golden import load_stage_case
    obj, docs, want = load_stage_case(path)
    stages = [stage_from_v1alpha1(d) for d in docs]
    pp = _program(stages, gotpl.placeholder_funcs())
    byname = {s.name: i for i, s in enumerate(stages)}
    checked = 0
    for w in want["stages"]:
        si = byname[w["stage"]]
        exp = [n["data"] for n in w["next"] if n["kind"] == "patch" and n["type"] == "application/merge-patch+json"]
        tids = [pp.template_of[(si, pi)] for pi in range(len(stages[si].next.patches)) if (si, pi) in pp.template_of]
        if len(tids) != len(exp):
            assert (si, 0) in pp.unsupported
            continue
        for tid, e in zip(tids, exp):
            got = pp.render([tid], [obj], NOW)[0]
            assert got is not None
            assert json.loads(got) == e
            assert got.decode() == patchtpl.go_json_bytes(e)  # Go's Marshal of the golden value
            checked += 1
    assert checked or all((byname[w["stage"]], 0) in pp.unsupported or stages[byname[w["stage"]]].next.delete
                          for w in want["stages"])


def _workload_states(config, n_nodes, n_pods, seed):
    cl = W.make_cluster(config, n_nodes, n_pods, seed=seed)
    pods = cl.pods.materialize()
    stages = load_stage_files(*cl.pod_stage_files)
    prog = KindProgram(stages, HarnessSpec())
    prog.explore(pods)
    states = list(pods[:150])
    for reps in prog.class_reps.values():
        states += reps
    r = gotpl.Renderer(exploration_funcs(), now_ns=NOW)
    more = []
    for o in states[-200:]:
        for st in prog.stages:
            try:
                o2, _ = apply_next(st, copy.deepcopy(o), r)
            except Exception:
                continue
            if o2 is not None:
                more.append(o2)
    return cl, states + more


@pytest.mark.parametrize("config", ["C1", "C2"])
def test_native_equals_host_renderer_workload(config):
    cl, states = _workload_states(config, 10, 400, seed=71)
    stages = load_stage_files(*FILES)
    pp = _program(stages, n_threads=4)
    r = gotpl.Renderer(FUNCS, now_ns=NOW)
    nodes = cl.nodes.materialize()
    c = _compare(pp, stages, states + nodes, r)
    assert c["ok"] > 1000 and c["fallback"] == 0, c


def test_native_equals_oracle_restatement():
    """The oracle's template restatements (no template interpreter, oracle/next_ref.py)."""
    from oracle import next_ref
    cl, states = _workload_states("C2", 10, 600, seed=72)
    stages = load_stage_files(*FILES)
    F = next_ref.Funcs(now_ns=NOW)
    consts = {"NodeIPWith": F.node_ip_with(""), "PodIPWith": F.pod_ip_with("", False, "", "", ""),
              "NodeIP": F.node_ip(), "NodeName": F.node_name(), "NodePort": str(F.node_port()), "PodIP": "10.0.0.2"}
    pp = _program(stages, consts)
    checked = 0
    for (si, pi), tid in pp.template_of.items():
        st = stages[si]
        objs = [o for o in states + cl.nodes.materialize() if o.get("kind", "Pod") == st.kind]
        got = pp.render([tid] * len(objs), objs, NOW)
        for o, g in zip(objs, got):
            try:
                want = next_ref.render_status(st.next.patches[pi].template, o, F)
            except next_ref.RenderError:
                assert g is None
                continue
            assert g is not None
            assert json.loads(g) == {"status": want}, st.name
            checked += 1
    assert checked > 2000


def _edge_pods():
    vals = ["a<b>&c", "ünï☃", "line sep", 'q"uote', "back\\slash", "tab\tx", "ctl\x01x", "nel\x85x",
            "del\x7fx", "emoji\U0001F600", "", "123", "true", "yes", "~", "a: b", "x'y", "  lead", "trail  ",
            "1.5", "0x10", "-0", "y", "null", "containerFailed", "many words here", "dash-ed.dot/slash"]
    out = []
    for i, v in enumerate(vals):
        p = W.pod_object(f"edge-{i}", "node-0", annotations={
            "pod-container-running-failed.stage.kwok.x-k8s.io/reason": v,
            "pod-container-running-failed.stage.kwok.x-k8s.io/message": v,
            "pod-container-running-failed.stage.kwok.x-k8s.io/exit-code": v,
            "pod-container-running-failed.stage.kwok.x-k8s.io/container-name": "container-0" if i % 2 else ""})
        p["spec"]["containers"][0]["image"] = v
        p["spec"]["containers"].append({"name": v or "c", "image": 7 if i % 3 == 0 else v})
        if i % 4 == 0:
            p["spec"]["initContainers"] = [{"name": "init-" + v, "image": v, "restartPolicy": "Always" if i % 8 else "Never"}]
        if i % 5 == 0:
            p["spec"]["readinessGates"] = [{"conditionType": v}]
        if i % 6 == 0:
            p["spec"]["hostNetwork"] = True
        p["status"] = {"containerStatuses": [{"name": c["name"]} for c in p["spec"]["containers"]],
                       "initContainerStatuses": [{"name": c["name"]} for c in p["spec"].get("initContainers", [])]}
        out.append(p)
    node = W.node_object("edge-node", annotations={"node-not-ready.stage.kwok.x-k8s.io/type": "MemoryPressure",
                                                   "node-not-ready.stage.kwok.x-k8s.io/reason": "a<b>",
                                                   "node-not-ready.stage.kwok.x-k8s.io/message": "ünï "})
    return out + [node]


def test_native_equals_host_renderer_edge_values():
    stages = load_stage_files(*FILES)
    pp = _program(stages)
    r = gotpl.Renderer(FUNCS, now_ns=NOW)
    # printed (unquoted) chaos parameters that YAML re-types or rejects, and characters a YAML
    # scalar does not carry unchanged, go to the host renderer
    fallback = ["123", "true", "yes", "~", "a: b", "x'y", "  lead", "trail  ", "1.5", "0x10", "-0", "null",
                "\\u0001", "\\u0085", "\\u007f", "\u0085", "\x7f", "<b>", "a<b>&c", "ünï", " ", 'q\\"uote',
                "back\\\\slash", "\\t", "\U0001F600", "emoji", '"y"', '"exit-code": ""', '"message": ""']
    c = _compare(pp, stages, _edge_pods(), r, allow_fallback=fallback)
    assert c["ok"] > 100, c


def test_rfc3339nano_and_no_fraction():
    stages = load_stage_files(os.path.join(SHIPPED, "node", "heartbeat", "node-heartbeat.yaml"))
    pp = _program(stages)
    node = W.node_object("n0")
    for ns in (0, 1_700_000_000 * 10**9, 1_700_000_000 * 10**9 + 120_000_000, 951_782_400 * 10**9 + 1):
        got = pp.render([0], [node], ns)[0]
        want = gotpl.rfc3339nano(ns)
        assert json.loads(got)["status"]["conditions"][0]["lastHeartbeatTime"] == want


def test_bad_spec_rejected():
    with pytest.raises(Exception):
        patchtpl.lib()
        import ctypes as C
        h = C.c_void_p()
        patchtpl._check(patchtpl.lib().kwk_patcher_create(b'{"templates": [{"n_vars": 0, "n_regs": 0, "exprs": [], '
                                                          b'"prologue": [], "head": "", "tail": "", "body": ["q", 3]}],'
                                                          b' "funcs": [], "consts": []}', C.byref(h)), "create")


def test_native_patch_throughput_report(capsys):
    """patches/s of kwk_patch_render on fired-state C2 pods (pod-general's create / ready /
    complete templates), JSON bytes prepared beforehand, vs the host renderer."""
    from kwok_amd.host.encoder import pack_json
    import numpy as np
    cl, states = _workload_states("C2", 10, 600, seed=73)
    stages = load_stage_files(*cl.pod_stage_files)
    consts = {k: "10.0.0.1" for k in ("NodeIPWith", "PodIPWith", "NodeIP", "PodIP")}
    consts.update({"NodeName": "node", "NodePort": "10250"})
    pp = _program(stages, consts)
    r = gotpl.Renderer({k: (lambda v: (lambda *a: v))(v) for k, v in consts.items()}, now_ns=NOW)
    pick = [(si, tid) for (si, pi), tid in pp.template_of.items()
            if stages[si].name in ("pod-create", "pod-ready", "pod-complete")]
    objs, tids, tpl = [], [], []
    for o in states:
        for si, tid in pick:
            try:
                patchtpl.render_patch_bytes(stages[si].next.patches[0].template, "status", o, r)
            except gotpl.TemplateError:
                continue
            objs.append(o)
            tids.append(tid)
            tpl.append(stages[si].next.patches[0].template)
    reps = max(1, 40000 // len(objs))
    objs, tids = objs * reps, tids * reps
    buf, offs = pack_json(objs)
    rates = {}
    for t in (1, 8):
        pp.n_threads = t
        t0 = time.perf_counter()
        out, o, st = pp.render_buffer(np.asarray(tids), buf, offs, NOW)
        rates[t] = len(objs) / (time.perf_counter() - t0)
        assert (st == 0).all()
    t0 = time.perf_counter()
    for ob, text in zip(objs[:2000], tpl[:2000]):
        patchtpl.render_patch_bytes(text, "status", ob, r)
    host = min(2000, len(tpl)) / (time.perf_counter() - t0)
    with capsys.disabled():
        print(f"\nnative patch renderer: {rates[1]:.0f} patches/s (1 thread), {rates[8]:.0f} patches/s (8 threads); "
              f"host renderer {host:.0f} patches/s")
    assert rates[1] > host
