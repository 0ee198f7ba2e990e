"""The native Stage compiler (libkwok_compiler, include/kwok_compiler.h) against the host's Python
compiler (kwok_amd/host/compiler.py KindProgram, its CPU cross-check), VERDICT r3 item 1: for
every shipped stage set — pod-fast, pod-general + pod-chaos, node-fast + node-heartbeat,
node-fast + node-heartbeat-with-lease, node-chaos — with and without the churn harness, explored
from the workloads' representative objects, the device stage table, the (class, stage) delta
table, the harness masks, the class keys, describe(), the encoder spec and the patch spec (with
the controllers' template functions) are byte-equal.

Reference: lifecycle.NewLifecycle / NewStage (pkg/utils/lifecycle/lifecycle.go:33-46,194-267),
conversion.go:395-425, next.go:73-173."""
import ctypes as C
import json

import numpy as np
import pytest

from kwok_amd import workload as W
from kwok_amd.host.compiler import HarnessSpec, KindProgram, exploration_funcs
from kwok_amd.host.native_compiler import CompileError, NativeProgram, stage_docs_from_files
from kwok_amd.host.stages import load_stage_files

POD_ROOTS = [W.pod_object("p", "n"), W.pod_object("p", "n", job=True), W.pod_object("p", "n", init=1),
             W.pod_object("p", "n", init=2, labels={"pod-init-container-running-failed.stage.kwok.x-k8s.io": "true"}),
             W.pod_object("p", "n", labels={"pod-container-running-failed.stage.kwok.x-k8s.io": "true"}),
             W.pod_object("p", "n", deletion="2023-11-14T22:13:50Z"),
             W.pod_object("p", "n", job=True, annotations={"pod-ready.stage.kwok.x-k8s.io/weight": "0x10",
                                                           "pod-delete.stage.kwok.x-k8s.io/delay": "1s"})]
NODE_ROOTS = [W.node_object("node"), W.node_object("n2", labels={"node-not-ready.stage.kwok.x-k8s.io": "true"}),
              W.node_object("n3", annotations={"example.com/zone": "b"})]

SETS = {
    "pod-fast": (W.POD_FAST, POD_ROOTS),
    "pod-general+chaos": (W.POD_GENERAL + W.POD_CHAOS, POD_ROOTS),
    "node-fast+heartbeat": (W.NODE_FAST + W.NODE_HEARTBEAT, NODE_ROOTS),
    "node-fast+heartbeat-with-lease": (W.NODE_FAST + W.NODE_HEARTBEAT_LEASE, NODE_ROOTS),
    "node-chaos": (W.NODE_CHAOS + W.NODE_FAST + W.NODE_HEARTBEAT, NODE_ROOTS),
}


def _pair(name, harness, roots=None):
    files, r = SETS[name]
    paths = W.stage_paths(files)
    kp = KindProgram(load_stage_files(*paths), HarnessSpec() if harness else None)
    np_ = NativeProgram(stage_docs_from_files(*paths), HarnessSpec() if harness else None)
    roots = r if roots is None else roots
    kp.explore(roots)
    np_.explore(roots)
    return kp, np_


def _assert_equal(kp, nat):
    assert bytes(nat.table(7)) == bytes(kp.table(7))
    assert np.array_equal(nat.delta_array(), kp.delta_array())
    assert bytes(nat.harness_struct()) == bytes(kp.harness_struct())
    assert nat.describe() == kp.describe()
    assert nat.class_ids == kp.class_ids
    assert nat.names == kp.names
    from kwok_amd.host.encoder import EncoderUnsupported, encoder_spec
    try:
        want = encoder_spec(kp)
    except EncoderUnsupported:
        want = None
    if want is None:  # "patch already applied" bits: the native spec carries the patches (below)
        assert kp.applied_bits and json.loads(nat.encoder_spec())["applied"]
    else:
        assert nat.encoder_spec() == want
    from kwok_amd.host.patchtpl import PatchProgram
    pp = PatchProgram(kp.stages, exploration_funcs())
    spec, tof = nat.patch_spec(exploration_funcs())
    assert spec == pp.spec
    assert tof == pp.template_of
    pp.close()
    pp0 = PatchProgram(kp.stages, {"NodeName": "node-0"})  # a constant function, and the rest unsupported
    spec0, tof0 = nat.patch_spec({"NodeName": "node-0"})
    assert spec0 == pp0.spec and tof0 == pp0.template_of
    pp0.close()


@pytest.mark.parametrize("harness", [False, True])
@pytest.mark.parametrize("name", sorted(SETS))
def test_native_compiler_byte_equal(name, harness):
    kp, nat = _pair(name, harness)
    try:
        _assert_equal(kp, nat)
        assert not kp.delta_conflicts
    finally:
        nat.close()


def test_native_compiler_workload_roots_and_reexplore():
    """C2's representative objects (every variant of the 1M-pod mix) and a second explore with a
    new root: both compilers register classes in the same order and re-derive the same deltas."""
    variants, _ = W.c2_pod_variants(0, 200_000, seed=W.CLUSTER_SEED)
    kp, nat = _pair("pod-general+chaos", True, roots=variants[: len(variants) // 2])
    try:
        _assert_equal(kp, nat)
        rest = variants[len(variants) // 2:]
        kp.explore(rest)
        nat.explore(rest)
        _assert_equal(kp, nat)
        # class_of: a known class, an unknown one registered (its deltas UNKNOWN until explored)
        o = W.pod_object("x", "y", containers=3)
        assert nat.class_of(variants[0], register=False) == kp.class_of(variants[0], register=False)
        assert nat.class_of(o) == kp.class_of(o)
        _assert_equal(kp, nat)
    finally:
        nat.close()


def test_native_compiler_errors_and_drops():
    """NewLifecycle drops a stage without a selector (lifecycle.go:199-201); a requirement that
    violates the operator's value rule, two resourceRefs in one program and a jq construct outside
    the native step form are compile errors."""
    docs = stage_docs_from_files(*W.stage_paths(W.POD_FAST))
    nosel = json.loads(json.dumps(docs[0]))
    nosel["metadata"]["name"] = "no-selector"
    del nosel["spec"]["selector"]
    nat = NativeProgram([nosel] + docs)
    assert nat.names == [d["metadata"]["name"] for d in docs]
    nat.close()
    bad = json.loads(json.dumps(docs[0]))
    bad["spec"]["selector"]["matchExpressions"][0]["operator"] = "In"
    bad["spec"]["selector"]["matchExpressions"][0].pop("values", None)
    with pytest.raises(CompileError, match="values set can't be empty"):
        NativeProgram([bad])
    node = stage_docs_from_files(*W.stage_paths(W.NODE_FAST))
    with pytest.raises(CompileError, match="resourceRef"):
        NativeProgram(docs + node)
    jq = json.loads(json.dumps(docs[0]))
    jq["spec"]["selector"]["matchExpressions"][0]["key"] = ".status.conditions | .[] as $c | $c.type"
    with pytest.raises(CompileError, match="jq construct not supported natively: 'as'"):
        NativeProgram([jq])
    jq["spec"]["selector"]["matchExpressions"][0]["key"] = '.metadata.name | test("^a")'
    with pytest.raises(CompileError, match="function test/1"):
        NativeProgram([jq])


def test_native_compiler_exports():
    """Every kwk_program* symbol include/kwok_compiler.h declares is exported."""
    import re
    from kwok_amd.host.native_compiler import LIB_PATH
    hdr = open(__file__.replace("tests/test_native_compiler.py", "include/kwok_compiler.h")).read()
    names = set(re.findall(r"\b(kwk_(?:program|compile)_[a-z_]+)\s*\(", hdr))
    L = C.CDLL(LIB_PATH)
    for n in names:
        assert hasattr(L, n), n
    assert len(names) >= 12


def _states(kp, roots, times):
    """The roots and what firing each matching stage makes of them, with Now at the given times."""
    from kwok_amd.host.gotpl import Renderer, rfc3339nano
    from kwok_amd.host.nextstate import apply_next, prune_empty
    import copy
    out = [prune_empty(copy.deepcopy(r)) for r in roots]
    frontier = list(out)
    for _ in range(3):
        nxt = []
        for o in frontier:
            m = kp.stage_matches(kp.pred_of(o))
            for s, st in enumerate(kp.stages):
                if not (m >> s) & 1:
                    continue
                for t in times:
                    r = Renderer(exploration_funcs(), now_ns=t)
                    r.funcs["Now"] = lambda t=t: rfc3339nano(t)
                    o2, _ = apply_next(st, copy.deepcopy(o), r)
                    if o2 is not None:
                        nxt.append(o2)
        out += nxt
        frontier = nxt
    return out


@pytest.mark.parametrize("name", sorted(SETS))
def test_native_encoder_rows_from_native_spec(name):
    """libkwok_encoder built from the native compiler's spec encodes every state the stages reach
    exactly as the Python Ingest of KindProgram: feature bits — including the "patch already
    applied" bits of node-heartbeat, which the native encoder evaluates with its template renderer
    (a node whose heartbeat patch rendered at the static renderer's Now is a no-op gets the bit) —
    value records, deletion column and classes."""
    from kwok_amd.host.encoder import NativeIngest
    from kwok_amd.host.engine import Ingest
    kp, nat = _pair(name, True)
    try:
        t0 = 1_700_000_000 * 10**9
        objs = _states(kp, SETS[name][1], [t0, t0 + 7 * 10**9])
        py = Ingest(kp)
        want = py.columns(objs)
        ing = NativeIngest(nat, n_threads=3)
        got = ing.columns(objs)
        for w, g, col in zip(want, got, ("hot", "deletion", "rec", "cls")):
            assert np.array_equal(w, g), col
        if kp.applied_bits:
            ab = sum(1 << b for b in kp.applied_bits.values())
            hits = int(np.count_nonzero(want[0]["pred"] & ab))
            assert 0 < hits < len(objs), hits  # both outcomes occur
        assert np.array_equal(py.record_array(), ing.record_array())
        ing.close()
    finally:
        nat.close()
