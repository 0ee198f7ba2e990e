"""Error reporting across the C ABIs: a failing call's message is kept per handle (engine,
encoder, patcher), so a caller that changes OS threads between the failing call and the message
read — a Go goroutine over cgo — still gets its own call's message; calls
without a handle (create) leave it in the calling thread's slot.  SURVEY §8(b): "message via
kwk_last_error (per engine)"."""
import ctypes as C
import threading

import numpy as np
import pytest

from kwok_amd import workload as W
from kwok_amd.host import abi
from kwok_amd.host.compiler import KindProgram
from kwok_amd.host.stages import load_stage_files


def _in_thread(fn):
    out = {}

    def run():
        out["r"] = fn()
    t = threading.Thread(target=run)
    t.start()
    t.join()
    return out["r"]


def test_engine_create_errors_stay_in_their_thread():
    L = abi.lib()

    def bad_capacity():
        d = abi.EngineDesc(device=0, capacity=0)
        h = C.c_void_p()
        st = L.kwk_engine_create(C.byref(d), C.byref(h))
        return st, L.kwk_last_error(None).decode()

    def null_desc():
        h = C.c_void_p()
        st = L.kwk_engine_create(None, C.byref(h))
        return st, L.kwk_last_error(None).decode()

    a = _in_thread(bad_capacity)
    b = _in_thread(null_desc)
    assert a == (abi.KWK_EINVAL, "capacity must be > 0")
    assert b == (abi.KWK_EINVAL, "null argument")
    # this thread made no failing call
    assert L.kwk_last_error(None).decode() == ""


def test_encoder_errors_per_handle_across_threads():
    from kwok_amd.host import encoder as E
    prog = KindProgram(load_stage_files(*W.stage_paths(W.POD_FAST)))
    prog.explore([W.pod_object("p", "n")])
    h1, h2 = E.NativeIngest(prog), E.NativeIngest(prog)
    try:
        L = E.lib()
        n = 2
        hot = np.zeros(n, dtype=abi.HOT_DTYPE)
        dels = np.zeros(n, dtype=np.int64)
        rec = np.zeros(n, dtype=np.uint32)
        cls = np.zeros(n, dtype=np.uint16)
        buf = b"{}{}"
        bad_offs = np.array([0, 2, 1], dtype=np.uint64)  # not ascending

        def fail1():
            return L.kwk_encode(h1.h, n, buf, abi.ptr(bad_offs), 1, abi.ptr(hot), abi.ptr(dels), abi.ptr(rec),
                                abi.ptr(cls), None)

        def fail2():
            return L.kwk_encode(h2.h, n, None, abi.ptr(bad_offs), 1, abi.ptr(hot), abi.ptr(dels), abi.ptr(rec),
                                abi.ptr(cls), None)
        assert _in_thread(fail1) == abi.KWK_EINVAL
        assert _in_thread(fail2) == abi.KWK_EINVAL
        # read from a third thread (this one): each handle holds its own message
        assert L.kwk_encoder_last_error(h1.h).decode() == "offsets must be non-decreasing"
        assert L.kwk_encoder_last_error(h2.h).decode() == "null argument"
    finally:
        h1.close()
        h2.close()


def test_patcher_errors_per_handle_across_threads():
    from kwok_amd.host import patchtpl as P
    stages = load_stage_files(*W.stage_paths(W.POD_FAST))
    p1, p2 = P.PatchProgram(stages), P.PatchProgram(stages)
    L = P.lib()
    objs = b"{}{}"
    out = C.c_char_p()
    oo = np.zeros(3, dtype=np.uint64)
    status = np.zeros(2, dtype=np.uint8)

    def call(p, tids, offs):
        return L.kwk_patch_render(p.h, 2, abi.ptr(tids), objs, abi.ptr(offs), 0, p._fn, None, 1, C.byref(out),
                                  abi.ptr(oo), abi.ptr(status))
    bad_tid = np.array([0, 999], dtype=np.uint16)
    ok_offs = np.array([0, 2, 4], dtype=np.uint64)
    bad_offs = np.array([0, 3, 2], dtype=np.uint64)
    assert _in_thread(lambda: call(p1, bad_tid, ok_offs)) == abi.KWK_EINVAL
    assert _in_thread(lambda: call(p2, np.zeros(2, dtype=np.uint16), bad_offs)) == abi.KWK_EINVAL
    assert L.kwk_patch_last_error(p1.h).decode() == "template id out of range"
    assert L.kwk_patch_last_error(p2.h).decode() == "object offsets not ascending"


@pytest.mark.gpu
def test_engine_errors_per_engine_across_threads():
    """Two engines, each failing a different call on its own thread; the messages are read back
    on a third thread, each from its engine."""
    from kwok_amd.host.engine import Engine
    prog = KindProgram(load_stage_files(*W.stage_paths(W.POD_FAST)))
    prog.explore([W.pod_object("p", "n")])
    e1, e2 = Engine(prog, capacity=64), Engine(prog, capacity=64)
    try:
        L = abi.lib()
        slots = np.array([5], dtype=np.uint32)
        assert _in_thread(lambda: L.kwk_delete(e1.h, 1, abi.ptr(slots))) == abi.KWK_EINVAL
        assert _in_thread(lambda: L.kwk_set_tuning(e2.h, 12345, 0)) == abi.KWK_EINVAL
        assert L.kwk_last_error(e1.h).decode() == "slot not active"
        assert L.kwk_last_error(e2.h).decode() == "unknown tuning key 12345"
        # a later failing call on e1 replaces e1's message only
        assert _in_thread(lambda: L.kwk_step(e1.h, 0, 0, 0)) == abi.KWK_ESTATE
        assert L.kwk_last_error(e1.h).decode().startswith("kwk_load_stages must be called")
        assert L.kwk_last_error(e2.h).decode() == "unknown tuning key 12345"
        with pytest.raises(abi.EngineError, match="slot not active"):
            e1.delete([9])
    finally:
        e1.close()
        e2.close()
