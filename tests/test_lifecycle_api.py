"""The reference's lifecycle interface (kwok_amd.host.lifecycle) driven like the reference's
own tests: the stage-tester flow over the golden fixtures (ListAllPossible, Weight, Delay,
Next) on the host, and Match + Delay through the HIP engine against the oracle."""
import os

import pytest

from kwok_amd import workload as W
from kwok_amd.host.gotpl import Renderer, placeholder_funcs
from kwok_amd.host.lifecycle import Lifecycle, philox_u64
from kwok_amd.host.stages import load_stage_files, stage_from_v1alpha1, to_v1alpha1
from oracle import refcpu
from tests.test_oracle_golden import _stage_cases, load_stage_case


def test_philox_hook_matches_oracle():
    for seed, slot, step, site in [(0, 0, 0, 1), (0x6B776F6B, 12345, 7, 2), ((1 << 64) - 1, (1 << 32) - 1, 1 << 40, 1)]:
        assert philox_u64(seed, slot, step, site) == refcpu.philox_u64(seed, slot, step, site)


@pytest.mark.parametrize("path", _stage_cases(), ids=os.path.basename)
def test_stage_tester_flow_golden(path):
    """pkg/tools/stage/stage.go:37-151 through the mirror API."""
    obj, stages, want = load_stage_case(path)
    lc = Lifecycle.new([stage_from_v1alpha1(s) for s in stages])
    got = lc.list_all_possible(obj)
    assert [s.name() for s in got] == [w["stage"] for w in want["stages"]]
    r = Renderer(placeholder_funcs())
    for s, w in zip(got, want["stages"]):
        weight, ok = s.weight(obj)
        assert ("weight" in w) == ok and (not ok or weight == w["weight"])
        delay, ok = s.delay({}, 0)  # the tester passes the Stage value itself: every *From query is empty
        assert ("delay" in w) == ok and (not ok or delay == w["delay"])
        nxt = s.next()
        exp_fin = [n["data"] for n in w["next"] if n["kind"] == "patch" and n["type"] == "application/json-patch+json"]
        assert (nxt.finalizers(obj.get("metadata", {}).get("finalizers")) or None) == (exp_fin[0] if exp_fin else None)
        assert nxt.delete() == any(n["kind"] == "delete" for n in w["next"])
        if not nxt.delete():
            exp = [n["data"] for n in w["next"] if n["kind"] == "patch" and n["type"] == "application/merge-patch+json"]
            assert [d for _, d, _ in nxt.patches(obj, r)] == exp
        assert s.immediate_next_stage() == any(n["kind"] == "immediate" for n in w["next"])


def test_host_delay_matches_oracle():
    """Stage.Delay on pod-general stages with override annotations (incl. RFC3339 and invalid
    values) and the jitter hook: host mirror == oracle restatement."""
    cl = W.make_cluster("C2", 10, 400, seed=31)
    stages = load_stage_files(*cl.pod_stage_files)
    lc = Lifecycle.new(stages)
    orc = refcpu.Lifecycle([to_v1alpha1(s) for s in stages])
    now = 1_700_000_000 * 10**9
    for slot, o in enumerate(cl.pods.materialize()):
        for i, s in enumerate(lc.stages):
            assert s.delay(o, now, key=99, slot=slot, step=3) == orc.delay(i, o, now, 99, 3, slot)
            assert s.weight(o) == orc.weight(i, o)


@pytest.mark.gpu
def test_match_on_gpu_equals_oracle():
    cl = W.make_cluster("C2", 20, 800, seed=32)
    stages = load_stage_files(*cl.pod_stage_files)
    objs = cl.pods.materialize()
    lc = Lifecycle.new(stages)
    orc = refcpu.Lifecycle([to_v1alpha1(s) for s in stages])
    now = 1_700_000_000 * 10**9
    try:
        got = lc.match_batch(objs, now, seed=5, step=2)
        for slot, (o, (st, d)) in enumerate(zip(objs, got)):
            s, de = orc.match(o, now, 5, 2, slot)
            assert (None if st is None else st.index) == s
            if s is not None:
                assert d == de
        st, d = lc.match(objs[0], now, seed=5, step=2, slot=0)
        assert (None if st is None else st.index) == orc.match(objs[0], now, 5, 2, 0)[0]
    finally:
        lc.close()
