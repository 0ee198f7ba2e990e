"""The host libraries in the GPU-checked loop: KindController on its native
path — the fired hand-back of the engine (kwk_step / kwk_fired) rendered by libkwok_patch
(kwk_patch_render, the precompiled merge-patch byte templates) and every fired object's new
state re-encoded by libkwok_encoder (kwk_encode) — stepped beside the oracle.  At every step:
the fired set equals the oracle's, the host's object cache equals the oracle's objects (so every
rendered patch applied equals oracle/next_ref.py's restatement of the template), and every
re-encoded row's feature bits equal both the oracle's jq (oracle_pred) and the device row.
Reference: pkg/kwok/controllers/pod_controller.go:290-360 (playStage), 412-478 (the watch
event's re-encode), pkg/utils/lifecycle/next.go:73-88."""
import numpy as np
import pytest

from kwok_amd import workload as W
from kwok_amd.host import abi

pytestmark = pytest.mark.gpu


def _run(cl, steps, dt_ns, seed, compiler="python"):
    from kwok_amd.host.compiler import KindProgram
    from kwok_amd.host.controller import KindController
    from kwok_amd.host.encoder import NativeIngest
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files
    from oracle.next_ref import load_stage_docs
    from oracle.sim import OracleSim, oracle_pred
    from tests.parity_util import NOW0, compare_state
    objs = cl.pods.materialize()
    if compiler == "native":  # the Go host's path: libkwok_compiler, no Python compiler
        from kwok_amd.host.native_compiler import NativeProgram, stage_docs_from_files
        prog = NativeProgram(stage_docs_from_files(*cl.pod_stage_files))
        ing = None
    else:
        prog = KindProgram(load_stage_files(*cl.pod_stage_files))
        ing = Ingest(prog)
    prog.explore(objs)
    # the initial list too goes through the native encoder
    nat = NativeIngest(prog)
    hot, dels, rec, cls = nat.columns(objs)
    eng = Engine(prog, capacity=len(objs), max_records=len(nat.record_array()) + 64)
    ctl = KindController(prog, eng, ing, objs, native=True)
    sim = OracleSim(load_stage_docs(*cl.pod_stage_files), objs)
    desc = prog.describe()
    applied = sum(1 << b for b in desc["applied_bits"].values())
    checked = 0
    try:
        eng.load_stages()
        eng.load(hot, dels, rec, cls, nat.record_array())
        for k in range(steps):
            now = NOW0 + k * dt_ns
            got = ctl.step(now, seed, k)
            exp = sim.step(now, seed, k)
            g = sorted((int(r["slot"]), int(r["stage"]), int(r["flags"]) & ~abi.FIRED_DELTA_UNKNOWN) for r in got)
            assert g == sorted(exp), f"step {k}"
            compare_state(prog, eng, sim, k)
            assert ctl.objs == sim.objs, f"step {k}: rendered patches != oracle next state"
            dev, _ = eng.read()
            for i, row in ctl.last_rows.items():
                assert row[0] == oracle_pred(desc, sim.objs[i]), (k, i)
                assert row[0] == int(dev["pred"][i]) & ~applied, (k, i)
                checked += 1
        assert ctl.native_renders > 0
        return checked, ctl
    finally:
        ctl.close()
        nat.close()
        eng.close()


def test_native_controller_c1_pod_fast():
    cl = W.make_cluster("C1", 20, 300, seed=61)
    checked, ctl = _run(cl, steps=6, dt_ns=10**9, seed=0x61)
    assert checked >= 300 and ctl.host_renders == 0  # every pod-fast template renders natively


def test_native_controller_c2_pod_general():
    cl = W.make_cluster("C2", 30, 400, seed=62)
    checked, ctl = _run(cl, steps=30, dt_ns=500 * 10**6, seed=0x62)
    assert checked >= 400


@pytest.mark.parametrize("config", ["C1", "C2"])
def test_native_controller_with_native_compiler(config):
    """The whole Go-host path with no Python compiler: libkwok_compiler's table / deltas / encoder
    spec / patch spec, libkwok_encoder rows, libkwok_patch renders, the engine — stepped beside the
    oracle (fired sets, host object cache = oracle objects, re-encoded feature bits)."""
    if config == "C1":
        checked, ctl = _run(W.make_cluster("C1", 20, 300, seed=63), steps=6, dt_ns=10**9, seed=0x63, compiler="native")
        assert checked >= 300 and ctl.host_renders == 0
    else:
        checked, ctl = _run(W.make_cluster("C2", 30, 400, seed=64), steps=30, dt_ns=500 * 10**6, seed=0x64,
                            compiler="native")
        assert checked >= 400
