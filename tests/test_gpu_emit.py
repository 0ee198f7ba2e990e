"""Device patch emission on the GPU (include/kwok_emit.h): the native controller loop of
tests/test_controller_native.py with libkwok_emit beside it.  Every step, kwk_emit expands the
engine's fired list (kwk_fired records on even steps, 4-byte packed records on odd ones) on the
device (each record written by one lane through a 16-byte register window: records sharing a
16-byte window at both ends of every record, patches of every length); each item it emits equals, byte for byte, the patch the controller rendered for that
object with kwk_patch_render (itself checked against the oracle's next state there), and each
item it leaves to the host is one the skeleton cannot stand for (status guard not met, template
ineligible for the class).  After the host's hand-back, the guard bits the device carried equal
the guards evaluated on the host's objects.

Reference: pkg/kwok/controllers/pod_controller.go:290-360 (playStage), pkg/utils/lifecycle/
next.go:73-160, pkg/utils/gotpl/renderer.go:59-124."""
import collections

import numpy as np
import pytest

from kwok_amd import workload as W

pytestmark = pytest.mark.gpu


def _run(cl, steps, dt_ns, seed, room=0):
    from kwok_amd.host import emit
    from kwok_amd.host.compiler import KindProgram
    from kwok_amd.host.controller import KindController
    from kwok_amd.host.encoder import NativeIngest
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files
    from tests.parity_util import NOW0
    from tests.test_patch import FUNCS
    objs = cl.pods.materialize()
    prog = KindProgram(load_stage_files(*cl.pod_stage_files))
    prog.explore(objs)
    nat = NativeIngest(prog)
    hot, dels, rec, cls = nat.columns(objs)
    eng = Engine(prog, capacity=len(objs), max_records=len(nat.record_array()) + 64)
    ctl = KindController(prog, eng, Ingest(prog), objs, funcs=FUNCS, native=True)
    classes = [prog.class_of(o, register=False) for o in ctl.objs]
    reps = {}
    for o, c in zip(ctl.objs, classes):
        reps.setdefault(c, o)
    ep = emit.EmitProgram(prog.stages, ctl.patcher, reps, len(prog.class_ids))
    em = emit.Emitter(eng, len(objs), ep)
    counts = collections.Counter()
    if room:  # reserved up front for every record's worst case (no re-emit after KWK_ECAP)
        em.reserve(len(objs) * 16, len(objs) * room)
    try:
        words, cols = ep.rows(ctl.objs, classes)
        em.set_rows(0, words, cols)
        eng.load_stages()
        eng.load(hot, dels, rec, cls, nat.record_array())
        for k in range(steps):
            now = NOW0 + k * dt_ns
            packed = k % 2 == 1
            eng.step(now, seed, k)
            eng.fired_compact(packed=packed)
            items, offs, out = em.run(now, packed=packed)
            fired = eng.fired()
            pre = {int(r["slot"]): ctl.objs[int(r["slot"])] for r in fired}
            ctl.handle(fired, now)
            # the items: every patch of every fired stage, in list order
            want_items = [(j, t) for j, r in enumerate(fired) for t in ep.stage_tpl[int(r["stage"])]]
            assert [(int(i["rec"]), int(i["tid"])) for i in items] == want_items, f"step {k}"
            host_slots = set()
            pos = collections.Counter()
            for n, it in enumerate(items):
                r = fired[int(it["rec"])]
                slot, stage = int(r["slot"]), int(r["stage"])
                pi = pos[int(it["rec"])]
                pos[int(it["rec"])] += 1
                c = classes[slot]
                if int(it["status"]) == emit.STATUS_OK:
                    got = out[int(offs[n]):int(offs[n + 1])]
                    assert got == ctl.last_patches[(slot, pi)], (k, slot, prog.stages[stage].name)
                    counts["device"] += 1
                    continue
                host_slots.add(slot)
                sk = ep.skel.get((c, int(it["tid"])))
                if sk is not None:  # eligible: the object's guard was not met before this fire
                    assert not all(emit.guard_holds(pre[slot], g) for g in sk["guard_list"]), (k, slot)
                    counts["guard"] += 1
                else:
                    counts["host"] += 1
            # the host sets the words of the objects it rendered (or deleted) itself
            live = [s for s in host_slots if ctl.objs[s] is not None]
            if live:
                w, cc = ep.rows([ctl.objs[s] for s in live], [classes[s] for s in live])
                em.set_slots(np.asarray(live), w, cc)
            dev = em.words(0, len(objs))
            # the device's value-length cache in bits 24-31 stays internal (kwk_emit_get_words: 0)
            assert not np.any((dev >> np.uint64(24)) & np.uint64(0xFF)), k
            for s, o in enumerate(ctl.objs):
                if o is not None:
                    assert (int(dev[s]) >> 16) & 0xFF == ep.guard_bits(o), (k, s)
        return counts
    finally:
        em.close()
        ctl.close()
        nat.close()
        eng.close()


def _big_stage_run(steps, room=0):
    """Patches longer than the emitter's per-wave LDS window (6 KiB): the staged writer sends such a
    record straight to global memory; a short second stage keeps the windows in use around it."""
    from kwok_amd.host import emit
    from kwok_amd.host.compiler import KindProgram
    from kwok_amd.host.controller import KindController
    from kwok_amd.host.encoder import NativeIngest
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import stage_from_v1alpha1
    from tests.parity_util import NOW0
    from tests.test_patch import FUNCS

    def doc(name, key, op, vals, template):
        sel = {"key": key, "operator": op}
        if vals:
            sel["values"] = vals
        return stage_from_v1alpha1({
            "apiVersion": "kwok.x-k8s.io/v1alpha1", "kind": "Stage", "metadata": {"name": name},
            "spec": {"resourceRef": {"apiGroup": "v1", "kind": "Pod"}, "selector": {"matchExpressions": [sel]},
                     "next": {"statusTemplate": template}}})
    big = "x" * 7000
    stages = [doc("big", ".status.phase", "DoesNotExist", None,
                  "phase: Pending\nmessage: '" + big + " at {{ Now }}'\nhostIP: {{ NodeIPWith .spec.nodeName | Quote }}\n"),
              doc("small", ".status.phase", "In", ["Pending"], "phase: Running\nreason: '{{ Now }}'\n")]
    objs = [{"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"p{i}", "namespace": "d", "uid": f"u{i}"},
             "spec": {"nodeName": f"n{i % 7}", "containers": [{"name": "c", "image": "i"}]}} for i in range(3000)]
    prog = KindProgram(stages)
    prog.explore(objs)
    nat = NativeIngest(prog)
    hot, dels, rec, cls = nat.columns(objs)
    eng = Engine(prog, capacity=len(objs), max_records=len(nat.record_array()) + 64)
    ctl = KindController(prog, eng, Ingest(prog), objs, funcs=FUNCS, native=True)
    classes = [prog.class_of(o, register=False) for o in ctl.objs]
    ep = emit.EmitProgram(prog.stages, ctl.patcher, {classes[0]: ctl.objs[0]}, len(prog.class_ids))
    em = emit.Emitter(eng, len(objs), ep)
    n_dev = 0
    if room:
        em.reserve(len(objs) * 16, len(objs) * room)
    try:
        w, cc = ep.rows(ctl.objs, classes)
        em.set_rows(0, w, cc)
        eng.load_stages()
        eng.load(hot, dels, rec, cls, nat.record_array())
        for k in range(steps):
            now = NOW0 + k * 10**9
            eng.step(now, 7, k)
            eng.fired_compact(packed=True)
            items, offs, out = em.run(now, packed=True)
            fired = eng.fired()
            ctl.handle(fired, now)
            for n, it in enumerate(items):
                slot = int(fired[int(it["rec"])]["slot"])
                assert int(it["status"]) == emit.STATUS_OK, (k, slot)
                assert out[int(offs[n]):int(offs[n + 1])] == ctl.last_patches[(slot, 0)], (k, slot)
                n_dev += 1
        return n_dev
    finally:
        em.close()
        ctl.close()
        nat.close()
        eng.close()


def test_gpu_emit_records_larger_than_the_window():
    assert _big_stage_run(steps=4) >= 6000


def test_gpu_emit_reserved_records_larger_than_the_window():
    assert _big_stage_run(steps=4, room=16384) >= 6000


def test_gpu_emit_reserved_c2_pod_general_equals_native_render():
    """Room reserved up front for every record's worst case (the first kwk_emit of each step
    succeeds): the same bytes, items, offsets and guard words.  C2 at 40k pods: a list of many
    tiles, records of mixed lengths, items left to the host."""
    cl = W.make_cluster("C2", 300, 40000, seed=94)
    c = _run(cl, steps=6, dt_ns=500 * 10**6, seed=0x94, room=8192)
    assert c["device"] >= 10000, c


def test_gpu_emit_c2_pod_general_equals_native_render():
    cl = W.make_cluster("C2", 30, 400, seed=91)
    c = _run(cl, steps=30, dt_ns=500 * 10**6, seed=0x91)
    assert c["device"] >= 400, c


def test_gpu_emit_c1_pod_fast_equals_native_render():
    cl = W.make_cluster("C1", 20, 300, seed=92)
    c = _run(cl, steps=8, dt_ns=10**9, seed=0x92)
    assert c["device"] >= 300 and c["host"] == 0, c


def test_gpu_emit_after_stream_recreated_and_column_rewritten():
    """Stream ordering: the emitter is created before KWK_TUNE_STREAM_PRIORITY re-creates
    the engine's stream; its value columns are first filled with decoy call values, then rewritten
    whole (a multi-MB upload) and the step is emitted at once.  Every device item must equal the
    native render, so the emission ran on the live stream and after the rewrite landed."""
    from kwok_amd.host import abi, emit
    from kwok_amd.host.compiler import KindProgram
    from kwok_amd.host.controller import KindController
    from kwok_amd.host.encoder import NativeIngest
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files
    from tests.parity_util import NOW0
    from tests.test_patch import FUNCS
    cl = W.make_cluster("C1", 400, 40000, seed=93)
    objs = cl.pods.materialize()
    prog = KindProgram(load_stage_files(*cl.pod_stage_files))
    prog.explore(objs)
    nat = NativeIngest(prog)
    hot, dels, rec, cls = nat.columns(objs)
    eng = Engine(prog, capacity=len(objs), max_records=len(nat.record_array()) + 64)
    ctl = KindController(prog, eng, Ingest(prog), objs, funcs=FUNCS, native=True)
    classes = [prog.class_of(o, register=False) for o in ctl.objs]
    reps = {}
    for o, c in zip(ctl.objs, classes):
        reps.setdefault(c, o)
    ep = emit.EmitProgram(prog.stages, ctl.patcher, reps, len(prog.class_ids))
    em = emit.Emitter(eng, len(objs), ep)
    try:
        words, cols = ep.rows(ctl.objs, classes)
        assert ep.n_columns >= 1
        decoy = {}
        for c, rows in cols.items():
            d = np.zeros_like(rows)
            d[:, 0] = 7
            d[:, 1:8] = np.frombuffer(b"9.9.9.9", dtype=np.uint8)
            decoy[c] = d
        em.set_rows(0, words, decoy)
        eng.set_tuning(abi.TUNE_STREAM_PRIORITY, 1)   # the stream the emitter saw at create is gone
        eng.load_stages()
        eng.load(hot, dels, rec, cls, nat.record_array())
        n_dev = 0
        for k in range(3):
            now = NOW0 + k * 10**9
            if k == 1:
                eng.set_tuning(abi.TUNE_STREAM_PRIORITY, 2)
            for c, rows in cols.items():            # the real values, rewritten whole right before the emit
                em.set_column(c, 0, rows)
            eng.step(now, 0x93, k)
            eng.fired_compact(packed=True)
            items, offs, out = em.run(now, packed=True)
            fired = eng.fired()
            ctl.handle(fired, now)
            pos = collections.Counter()
            for n, it in enumerate(items):
                r = int(it["rec"])
                slot = int(fired[r]["slot"])
                pi = pos[r]
                pos[r] += 1
                assert int(it["status"]) == emit.STATUS_OK, (k, slot)
                assert out[int(offs[n]):int(offs[n + 1])] == ctl.last_patches[(slot, pi)], (k, slot)
                n_dev += 1
            for c in cols:                           # decoys again: a later emit must not see them
                em.set_column(c, 0, decoy[c])
        assert n_dev >= 40000, n_dev
    finally:
        em.close()
        ctl.close()
        nat.close()
        eng.close()
