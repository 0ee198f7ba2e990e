"""The oracle's next-state leg (oracle/next_ref.py) is the checker's own restatement: pin it on
the reference's golden stage outputs and on the hand-derived pod-general / pod-chaos cases,
and check the product's next-state code (kwok_amd/host/nextstate.py + gotpl.py, which the
compiler derives the device deltas from) against the same fixtures and against the oracle on
every state the compiler explores."""
import copy
import json
import os

import pytest

from kwok_amd import workload as W
from kwok_amd.host.compiler import HarnessSpec, KindProgram, exploration_funcs
from kwok_amd.host.gotpl import Renderer, placeholder_funcs, rfc3339nano
from kwok_amd.host.nextstate import apply_next, finalizers_modify, render_patches
from kwok_amd.host.stages import load_stage_files, stage_from_v1alpha1
from oracle import refcpu
from oracle.next_ref import Funcs, StageNext, format_rfc3339nano, load_stage_docs, template_key, TEMPLATES
from tests.test_oracle_golden import _stage_cases, load_stage_case

HERE = os.path.dirname(os.path.abspath(__file__))
HAND = json.load(open(os.path.join(HERE, "golden", "pod_general_next.json")))


def _oracle_stage(doc):
    lc = refcpu.Lifecycle([doc])
    return StageNext(doc, lc, 0)


def test_every_shipped_template_is_restated():
    for path in W.stage_paths(W.POD_FAST + W.POD_GENERAL + W.POD_CHAOS + W.NODE_FAST + W.NODE_HEARTBEAT +
                              W.NODE_HEARTBEAT_LEASE + W.NODE_CHAOS):
        for d in load_stage_docs(path):
            t = (d["spec"].get("next") or {}).get("statusTemplate")
            if t:
                assert template_key(t) in TEMPLATES, path


@pytest.mark.parametrize("path", _stage_cases(), ids=os.path.basename)
def test_oracle_next_pinned_on_reference_goldens(path):
    """kustomize/stage/**/testdata/*.output.yaml: the rendered patch / delete of every listed
    stage (placeholder funcs, pkg/tools/stage/stage.go:128-151)."""
    obj, stages, want = load_stage_case(path)
    byname = {s["metadata"]["name"]: s for s in stages}
    for w in want["stages"]:
        st = _oracle_stage(byname[w["stage"]])
        kinds = [n["kind"] for n in w["next"]]
        assert st.delete == ("delete" in kinds)
        if st.delete:
            continue
        exp = [n["data"] for n in w["next"] if n["kind"] == "patch" and n["type"] == "application/merge-patch+json"]
        assert st.patches(obj, Funcs(placeholder=True)) == exp


@pytest.mark.parametrize("case", HAND["cases"], ids=lambda c: c["stage"].split("/")[-1] + ":" + c["input"]["metadata"]["name"])
def test_hand_derived_pod_general_next(case):
    """tests/golden/pod_general_next.json against the oracle AND the product."""
    doc = load_stage_docs(os.path.join(W.STAGE_DIR, case["stage"]))[0]
    obj = case["input"]
    # oracle
    st = _oracle_stage(doc)
    assert st.delete == case["delete"]
    assert (refcpu.Lifecycle([doc]).finalizers(0, obj["metadata"].get("finalizers")) or []) == case["finalizer_ops"]
    got = st.patches(obj, Funcs(placeholder=True))
    assert got == ([] if case["status_patch"] is None else [{"status": case["status_patch"]}])
    # product
    pst = stage_from_v1alpha1(doc)
    if pst.next.finalizers is not None:
        assert finalizers_modify(obj["metadata"].get("finalizers"), pst.next.finalizers) == case["finalizer_ops"]
    else:
        assert case["finalizer_ops"] == []
    assert pst.next.delete == case["delete"]
    pgot = [d for _, d, _ in render_patches(pst, obj, Renderer(placeholder_funcs()))]
    assert pgot == ([] if case["status_patch"] is None else [{"status": case["status_patch"]}])


def test_now_format_matches_go():
    for ns in (0, 1_700_000_000 * 10**9, 1_700_000_000 * 10**9 + 5 * 10**8, 1_700_000_000 * 10**9 + 123_456_789, 1):
        assert format_rfc3339nano(ns) == rfc3339nano(ns)
    assert format_rfc3339nano(1_700_000_000 * 10**9 + 5 * 10**8) == "2023-11-14T22:13:20.5Z"


@pytest.mark.parametrize("config,kind", [("C1", "pods"), ("C2", "pods"), ("C1", "nodes"), ("chaos", "nodes")])
def test_oracle_next_equals_product_on_explored_states(config, kind):
    """Every (state, matching stage) pair the compiler's exploration reaches: the oracle's
    restated next state == the product's (rendered with the same funcs and clock)."""
    if config == "chaos":
        objs = [W.node_object(f"n{i}", labels={"node-not-ready.stage.kwok.x-k8s.io": "true"}) for i in range(3)]
        files = W.stage_paths(W.NODE_FAST + W.NODE_HEARTBEAT + W.NODE_CHAOS)
    else:
        cl = W.make_cluster(config, 10, 200, seed=3)
        objs = cl.pods.materialize() if kind == "pods" else cl.nodes.materialize()
        files = cl.pod_stage_files if kind == "pods" else cl.node_stage_files
    prog = KindProgram(load_stage_files(*files), HarnessSpec() if kind == "pods" else None)
    prog.explore(objs)
    docs = load_stage_docs(*files)
    lc = refcpu.Lifecycle(docs)
    onext = [StageNext(d, lc, i) for i, d in enumerate(docs)]
    now = 1_700_000_123 * 10**9 + 456
    F = Funcs(now)
    r = Renderer(exploration_funcs(), now_ns=now)
    r.funcs["Now"] = lambda: rfc3339nano(now)
    states = [o for reps in prog.class_reps.values() for o in reps]
    seen, checked = set(), 0
    while states:
        o = states.pop()
        key = json.dumps(o, sort_keys=True)
        if key in seen or len(seen) > 400:
            continue
        seen.add(key)
        m = lc.match_mask(o)
        for s in range(len(docs)):
            if not (m >> s) & 1:
                continue
            o_or, ch_or = onext[s].apply(copy.deepcopy(o), F)
            o_pr, ch_pr = apply_next(prog.stages[s], copy.deepcopy(o), r)
            assert (o_or, ch_or) == (o_pr, ch_pr), (prog.names[s], o)
            checked += 1
            if o_or is not None:
                states.append(o_or)
        ph = (o.get("status") or {}).get("phase")
        if ph in ("Succeeded", "Failed") and "deletionTimestamp" not in o.get("metadata", {}):
            o2 = copy.deepcopy(o)  # the workload harness deletes finished pods
            o2["metadata"]["deletionTimestamp"] = "2023-11-14T22:13:20Z"
            states.append(o2)
    assert checked >= 2
