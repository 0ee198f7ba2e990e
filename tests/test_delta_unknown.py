"""The KWK_FIRED_DELTA_UNKNOWN round trip (kwok_amd/host/controller.py): objects of a class the
stage compiler never explored fire with UNKNOWN deltas; the host renders their patch, re-encodes
them and writes the rows back (kwk_replace), as the reference re-matches from the watch event
(pod_controller.go:336-351).  The run stays bit-exact with the oracle, and the host's object
cache equals the oracle's objects."""
import numpy as np
import pytest

from kwok_amd import workload as W
from kwok_amd.host import abi
from kwok_amd.host.compiler import KindProgram
from kwok_amd.host.stages import load_stage_files


def _unexplored_job_program():
    cl = W.make_cluster("C1", 10, 240, seed=41)
    objs = cl.pods.materialize()
    prog = KindProgram(load_stage_files(*cl.pod_stage_files))
    prog.explore([o for o in objs if not o["metadata"].get("ownerReferences")])  # the Job class is never explored
    return cl, objs, prog


def test_unexplored_class_gets_unknown_deltas():
    from kwok_amd.host.engine import Ingest
    cl, objs, prog = _unexplored_job_program()
    ing = Ingest(prog)
    ing.columns(objs)  # registers the Job class without exploring it
    assert len(prog.class_ids) == 2
    job = next(o for o in objs if o["metadata"].get("ownerReferences"))
    c = prog.class_of(job, register=False)
    d = prog.delta_array()
    for s, st in enumerate(prog.stages):
        if st.next.patches:
            assert tuple(d[c, s]) == abi.DELTA_UNKNOWN, prog.names[s]


@pytest.mark.gpu
def test_delta_unknown_round_trip_parity():
    from kwok_amd.host.controller import KindController
    from kwok_amd.host.engine import Engine, Ingest
    from oracle.next_ref import load_stage_docs
    from oracle.sim import OracleSim
    from tests.parity_util import NOW0, compare_state
    cl, objs, prog = _unexplored_job_program()
    ing = Ingest(prog)
    hot, dels, rec, cls = ing.columns(objs)
    eng = Engine(prog, capacity=len(objs))
    eng.load_stages()
    eng.load(hot, dels, rec, cls, ing.record_array())
    ctl = KindController(prog, eng, ing, objs)
    sim = OracleSim(load_stage_docs(*cl.pod_stage_files), objs)
    n_unknown = 0
    try:
        for k in range(8):
            now = NOW0 + k * 10**9
            got = ctl.step(now, 21, k)
            exp = sim.step(now, 21, k)
            n_unknown += int(np.count_nonzero(got["flags"] & abi.FIRED_DELTA_UNKNOWN))
            g = sorted((int(r["slot"]), int(r["stage"]), int(r["flags"]) & ~abi.FIRED_DELTA_UNKNOWN) for r in got)
            assert g == sorted(exp), f"step {k}"
            compare_state(prog, eng, sim, k)
            assert ctl.objs == sim.objs, f"step {k}: host cache != oracle objects"
        assert n_unknown > 0 and ctl.round_trips == n_unknown
    finally:
        eng.close()


@pytest.mark.gpu
def test_native_new_class_with_value_slots_round_trip_parity():
    """The native controller (libkwok_encoder rows) on the C2 mix — weight / delay / jitter value
    slots from override annotations — with the Job class never explored: the initial list's Job
    pods get their class registered and are re-encoded natively (NativeIngest.columns(register=
    True), kwk_encoder_add_classes), so every row's record id points into the native record table;
    their fires round-trip (DELTA_UNKNOWN: set_records, then kwk_replace, then the next step reads
    the records).  Fired sets, due times (record-driven delays and weights) and the host's object
    cache stay equal to the oracle's at every step."""
    from kwok_amd.host.controller import KindController
    from kwok_amd.host.encoder import NativeIngest
    from kwok_amd.host.engine import Engine, Ingest
    from oracle.next_ref import load_stage_docs
    from oracle.sim import OracleSim
    from tests.parity_util import NOW0, compare_state
    cl = W.make_cluster("C2", 20, 320, seed=43)
    objs = cl.pods.materialize()
    prog = KindProgram(load_stage_files(*cl.pod_stage_files))
    prog.explore([o for o in objs if not o["metadata"].get("ownerReferences")])
    n_explored = len(prog.class_ids)
    nat = NativeIngest(prog)
    hot, dels, rec, cls = nat.columns(objs, register=True)
    assert len(prog.class_ids) > n_explored and len(nat.record_array()) > 1
    ing = Ingest(prog)
    eng = Engine(prog, capacity=len(objs), max_records=len(nat.record_array()) + 64)
    eng.load_stages()
    eng.load(hot, dels, rec, cls, nat.record_array())
    ctl = KindController(prog, eng, ing, objs, native=True)
    ctl.nenc.close()
    ctl.nenc = nat  # the encoder whose record table the loaded rows index
    sim = OracleSim(load_stage_docs(*cl.pod_stage_files), objs)
    n_unknown = 0
    try:
        for k in range(24):
            now = NOW0 + k * 500 * 10**6
            got = ctl.step(now, 23, k)
            exp = sim.step(now, 23, k)
            n_unknown += int(np.count_nonzero(got["flags"] & abi.FIRED_DELTA_UNKNOWN))
            g = sorted((int(r["slot"]), int(r["stage"]), int(r["flags"]) & ~abi.FIRED_DELTA_UNKNOWN) for r in got)
            assert g == sorted(exp), f"step {k}"
            compare_state(prog, eng, sim, k)
            assert ctl.objs == sim.objs, f"step {k}: host cache != oracle objects"
        assert n_unknown > 0 and ctl.round_trips == n_unknown
    finally:
        ctl.close()
        eng.close()
