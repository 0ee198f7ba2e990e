"""CPU-only checks of the host side (no GPU): the product's jq / Go parsers / renderer /
stage compiler against the oracle and the reference's golden fixtures, and the C ABI
library's exported symbols."""
import copy
import ctypes
import json
import os
import random
import re
import subprocess

import pytest

from kwok_amd import workload as W
from kwok_amd.host import abi, goparse
from kwok_amd.host.compiler import HarnessSpec, KindProgram, strip_for_recreate
from kwok_amd.host.gotpl import Renderer, placeholder_funcs
from kwok_amd.host.jq import Query
from kwok_amd.host.nextstate import render_patches
from kwok_amd.host.stages import load_stage_files, stage_from_v1alpha1, to_v1alpha1
from oracle import refcpu
from tests.test_oracle_golden import VEC, _obj, _stage_cases, load_stage_case

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ------------------------------------------------------------------ C ABI library
def _header_functions():
    text = open(os.path.join(ROOT, "include", "kwok_engine.h")).read()
    return sorted(set(re.findall(r"^\s*(?:kwk_status|const char\*|uint32_t)\s+(kwk_\w+)\s*\(", text, re.M)))


@pytest.mark.parametrize("header,lib", [("kwok_engine.h", "libkwok_engine.so"), ("kwok_encoder.h", "libkwok_encoder.so"),
                                        ("kwok_patch.h", "libkwok_patch.so"), ("kwok_comm.h", "libkwok_comm.so"),
                                        ("kwok_compiler.h", "libkwok_compiler.so"), ("kwok_metrics.h", "libkwok_compiler.so"),
                                        ("kwok_emit.h", "libkwok_emit.so")])
def test_every_header_declaration_is_exported(header, lib):
    """Each C-ABI library loads (no GPU needed) and defines every function its include/*.h
    declares (a header's own declarations, not the engine types it includes)."""
    from kwok_amd import build
    build.build()
    path = os.path.join(ROOT, "kwok_amd", "lib", lib)
    ctypes.CDLL(path)
    text = open(os.path.join(ROOT, "include", header)).read()
    declared = set(re.findall(r"^\s*(?:kwk_status|const char\*|uint32_t)\s+(kwk_\w+)\s*\(", text, re.M))
    assert declared
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (kwk_\w+)", out))
    assert declared <= exported, sorted(declared - exported)


def test_abi_exports_every_header_symbol():
    from kwok_amd import build
    build.build()
    lib = ctypes.CDLL(abi.LIB_PATH)
    declared = _header_functions()
    assert declared == sorted(abi.EXPORTS)
    for name in declared:
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", abi.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (kwk_\w+)", out))
    assert set(declared) <= exported


def test_abi_struct_layout_matches_header():
    # sizes the device code relies on (16-byte hot record / value entry, 96-byte stage desc)
    assert ctypes.sizeof(abi.Hot) == 16 and ctypes.sizeof(abi.Value) == 16
    assert ctypes.sizeof(abi.StageDesc) == 96 and ctypes.sizeof(abi.FiredRec) == 8
    assert ctypes.sizeof(abi.StageTable) == 32 + 32 * 96
    assert ctypes.sizeof(abi.StepStats) == 8 * (4 + 32 + 2) and ctypes.sizeof(abi.EngineDesc) == 32


def test_engine_fails_loudly_without_gpu():
    pytest.importorskip("torch")
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    prog = KindProgram(load_stage_files(*W.stage_paths(W.POD_FAST)))
    from kwok_amd.host.engine import Engine
    with pytest.raises(abi.EngineError):
        Engine(prog, capacity=16)


# ------------------------------------------------------------------ jq / parsers vs oracle
@pytest.mark.parametrize("case", [c for c in VEC["query"] if "=" not in c["src"]], ids=lambda c: c["ref"])
def test_product_jq_vectors(case):
    assert Query(case["src"]).execute(_obj(case["obj"])) == case["want"]


def test_product_jq_matches_oracle_on_stage_queries():
    cl = W.make_cluster("C2", 20, 200, seed=3)
    objs = cl.pods.materialize()
    prog = KindProgram(load_stage_files(*cl.pod_stage_files), HarnessSpec())
    prog.explore(objs[:50])
    states = [o for reps in prog.class_reps.values() for o in reps] + objs
    queries = [f.src for f in prog.features.values()] + [s for _, s in prog.slots]
    for o in states:
        for q in queries:
            assert Query(q).execute(o) == refcpu.query(q, o), (q, o)


def test_go_parsers_match_oracle_fuzz():
    rnd = random.Random(7)
    alphabet = "0123456789xob_-+.smhuµnT:Z"
    cases = W.OVERRIDE_VALUES + ["0", "08", "1e3", "-0x_f", "9999-12-31T23:59:59.999999999+23:59"]
    cases += ["".join(rnd.choice(alphabet) for _ in range(rnd.randint(1, 9))) for _ in range(5000)]
    for s in cases:
        a, (b, ok) = goparse.parse_int(s), refcpu.parse_int(s)
        assert (a is not None, a or 0) == (ok, b), s
        a, (b, ok) = goparse.parse_duration(s), refcpu.parse_duration(s)
        assert (a is not None, a or 0) == (ok, b), s
        assert goparse.parse_rfc3339nano(s) == refcpu.parse_rfc3339(s), s


# ------------------------------------------------------------------ renderer vs golden outputs
@pytest.mark.parametrize("path", _stage_cases(), ids=os.path.basename)
def test_renderer_golden(path):
    obj, stages, want = load_stage_case(path)
    byname = {s["metadata"]["name"]: stage_from_v1alpha1(s) for s in stages}
    r = Renderer(placeholder_funcs())
    for w in want["stages"]:
        st = byname[w["stage"]]
        if st.next.delete:
            continue
        exp = [n["data"] for n in w["next"] if n["kind"] == "patch" and n["type"] == "application/merge-patch+json"]
        assert [d for _, d, _ in render_patches(st, obj, r)] == exp


# ------------------------------------------------------------------ compiler vs oracle
@pytest.mark.parametrize("config", ["C1", "C2"])
def test_compiled_match_equals_oracle(config):
    """pred bits + compiled clauses == refcpu's Lifecycle.match on every reachable state."""
    cl = W.make_cluster(config, 20, 300, seed=5)
    objs = cl.pods.materialize()
    stages = load_stage_files(*cl.pod_stage_files)
    prog = KindProgram(stages, HarnessSpec())
    prog.explore(objs)
    assert not prog.delta_conflicts
    lc = refcpu.Lifecycle([to_v1alpha1(s) for s in stages])
    states = [o for reps in prog.class_reps.values() for o in reps] + objs
    for o in states:
        assert prog.stage_matches(prog.pred_of(o)) == lc.match_mask(o)


def test_records_reproduce_oracle_getters():
    """Host pre-parsed *From records give the same (value, ok) as the oracle's getters."""
    cl = W.make_cluster("C2", 20, 2000, seed=9)
    objs = [o for o in cl.pods.materialize() if o["metadata"].get("annotations")]
    stages = load_stage_files(*cl.pod_stage_files)
    prog = KindProgram(stages)
    lc = refcpu.Lifecycle([to_v1alpha1(s) for s in stages])
    now = 1_700_000_000 * 10**9
    for o in objs[:200]:
        rec = prog.record_of(o)
        for si, d in enumerate(prog.stage_desc):
            w_exp = lc.weight(si, o)
            if d.weight_slot >= 0 and rec is not None and rec[d.weight_slot][0] != abi.V_DEFAULT:
                kind, v, _ = rec[d.weight_slot]
                got = (v, True) if kind == abi.V_OK else (0, False)
            else:
                got = (d.weight_default, True)
            assert got == w_exp, (prog.names[si], o["metadata"]["annotations"])


def test_finalizer_algebra_and_deltas_consistent():
    cl = W.make_cluster("C2", 10, 200, seed=2)
    prog = KindProgram(load_stage_files(*cl.pod_stage_files), HarnessSpec())
    prog.explore(cl.pods.materialize())
    assert not prog.delta_conflicts and not prog.rematch_mismatch
    # re-creation keeps exactly the static feature bits
    for reps in prog.class_reps.values():
        for o in reps:
            assert prog.pred_of(strip_for_recreate(o)) == prog.pred_of(o) & prog.keep_mask


def test_stage_selector_nil_dropped_and_errors():
    st = stage_from_v1alpha1({"kind": "Stage", "metadata": {"name": "x"},
                              "spec": {"resourceRef": {"kind": "Pod"}, "next": {}}})
    assert KindProgram([st]).stages == []
    with pytest.raises(ValueError):
        stage_from_v1alpha1({"kind": "Stage", "metadata": {"name": "x"},
                             "spec": {"resourceRef": {"kind": "Pod"}, "selector": {"matchExpressions": [
                                 {"key": ".a", "operator": "In", "values": []}]}, "next": {}}})
