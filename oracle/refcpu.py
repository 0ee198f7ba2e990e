"""ORACLE / TEST INFRASTRUCTURE — not product code.

ctypes binding for ``oracle/build/librefcpu.so``, the C++ CPU restatement of KWOK's
Stage lifecycle hot path (see ``oracle/refcpu/refcpu.cpp`` for the reference file:line
map).  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg import this module, and only as the checker / CPU baseline.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "librefcpu.so")
_lib = None


def build(force: bool = False) -> str:
    """Compile the restatement with the committed Makefile (gcc only)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.rc_last_error.restype = C.c_char_p
        L.rc_query.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int]
        L.rc_requirement.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p]
        L.rc_feature.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p]
        L.rc_feature.restype = C.c_int64
        L.rc_int_from.argtypes = [C.c_int, C.c_int64, C.c_char_p, C.c_char_p, C.POINTER(C.c_int64)]
        L.rc_duration_from.argtypes = [C.c_int, C.c_int64, C.c_char_p, C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]
        L.rc_parse_int.argtypes = [C.c_char_p, C.POINTER(C.c_int64)]
        L.rc_parse_duration.argtypes = [C.c_char_p, C.POINTER(C.c_int64)]
        L.rc_parse_rfc3339.argtypes = [C.c_char_p, C.POINTER(C.c_int64), C.POINTER(C.c_int32)]
        L.rc_philox_u64.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32]
        L.rc_philox_u64.restype = C.c_uint64
        L.rc_finalizers_modify.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int]
        L.rc_lifecycle_new.argtypes = [C.c_char_p]
        L.rc_lifecycle_new.restype = C.c_void_p
        L.rc_lifecycle_free.argtypes = [C.c_void_p]
        L.rc_lifecycle_len.argtypes = [C.c_void_p]
        L.rc_lifecycle_name.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_int]
        L.rc_stage_flags.argtypes = [C.c_void_p, C.c_int]
        L.rc_match.argtypes = [C.c_void_p, C.c_char_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_uint64,
                               C.POINTER(C.c_int64)]
        L.rc_list_all_possible.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_int), C.c_int]
        L.rc_match_mask.argtypes = [C.c_void_p, C.c_char_p]
        L.rc_match_mask.restype = C.c_int64
        L.rc_stage_weight.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.POINTER(C.c_int64)]
        L.rc_stage_delay.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_int64, C.c_uint64, C.c_uint64,
                                     C.c_uint64, C.POINTER(C.c_int64)]
        L.rc_stage_finalizers.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_char_p, C.c_int]
        L.rc_match_batch.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_int64), C.c_int64, C.c_int64,
                                     C.c_uint64, C.c_uint64, C.c_uint64, C.POINTER(C.c_int32),
                                     C.POINTER(C.c_int64), C.c_int]
        L.rc_match_batch.restype = C.c_int64
        _lib = L
    return _lib


def _s(x) -> bytes:
    return x.encode() if isinstance(x, str) else x


def _call_str(fn, *args) -> str:
    cap = 1 << 16
    while True:
        buf = C.create_string_buffer(cap)
        n = fn(*args, buf, cap)
        if n == -1000000:
            raise RuntimeError(lib().rc_last_error().decode())
        if n < 0:
            cap = -n + 16
            continue
        return buf.value.decode()


def dumps(obj) -> bytes:
    return json.dumps(obj, separators=(",", ":")).encode()


def query(src: str, obj):
    """Query.Execute: list of outputs, or None for the nil result."""
    return json.loads(_call_str(lib().rc_query, _s(src), dumps(obj)))


def feature(src: str, obj, literals) -> int:
    """bit 0: the query has an output; bit 1 + i: some output hasValue literal i (selector.go:101-111)."""
    r = lib().rc_feature(_s(src), dumps(obj), dumps(list(literals)))
    if r < 0:
        raise ValueError(lib().rc_last_error().decode())
    return int(r)


def requirement(key: str, op: str, values, obj) -> bool:
    r = lib().rc_requirement(_s(key), _s(op), dumps(list(values)), dumps(obj))
    if r < 0:
        raise ValueError(lib().rc_last_error().decode())
    return bool(r)


def int_from(value, src, obj):
    out = C.c_int64()
    r = lib().rc_int_from(0 if value is None else 1, value or 0, None if src is None else _s(src), dumps(obj),
                          C.byref(out))
    if r < 0:
        raise ValueError(lib().rc_last_error().decode())
    return out.value, bool(r)


def duration_from(value, src, obj, now_ns: int):
    out = C.c_int64()
    r = lib().rc_duration_from(0 if value is None else 1, value or 0, None if src is None else _s(src), dumps(obj),
                               now_ns, C.byref(out))
    if r < 0:
        raise ValueError(lib().rc_last_error().decode())
    return out.value, bool(r)


def parse_int(s: str):
    out = C.c_int64()
    ok = lib().rc_parse_int(_s(s), C.byref(out))
    return out.value, bool(ok)


def parse_duration(s: str):
    out = C.c_int64()
    ok = lib().rc_parse_duration(_s(s), C.byref(out))
    return out.value, bool(ok)


def parse_rfc3339(s: str):
    sec, nsec = C.c_int64(), C.c_int32()
    ok = lib().rc_parse_rfc3339(_s(s), C.byref(sec), C.byref(nsec))
    return (sec.value, nsec.value) if ok else None


def philox_u64(seed: int, slot: int, step: int, site: int) -> int:
    return lib().rc_philox_u64(seed, slot, step, site)


def finalizers_modify(meta, fin):
    return json.loads(_call_str(lib().rc_finalizers_modify, dumps(meta), dumps(fin)))


class Lifecycle:
    """lifecycle.NewLifecycle over v1alpha1 Stage objects (dicts)."""

    def __init__(self, stages):
        self._p = lib().rc_lifecycle_new(dumps(list(stages)))
        if not self._p:
            raise ValueError(lib().rc_last_error().decode())
        n = lib().rc_lifecycle_len(self._p)
        self.names = [_call_str(lib().rc_lifecycle_name, self._p, i) for i in range(n)]
        self.flags = [lib().rc_stage_flags(self._p, i) for i in range(n)]

    def __del__(self):
        if getattr(self, "_p", None):
            lib().rc_lifecycle_free(self._p)
            self._p = None

    def __len__(self):
        return len(self.names)

    def match(self, obj, now_ns: int, seed: int, step: int, slot: int):
        """Match + Delay: (stage index | None, delay_ns).  -2 = Go would panic."""
        d = C.c_int64()
        s = lib().rc_match(self._p, dumps(obj), now_ns, seed, step, slot, C.byref(d))
        if s == -3:
            raise ValueError(lib().rc_last_error().decode())
        if s == -1:
            return None, 0
        return s, d.value

    def match_mask(self, obj) -> int:
        return lib().rc_match_mask(self._p, dumps(obj))

    def list_all_possible(self, obj):
        out = (C.c_int * 64)()
        n = lib().rc_list_all_possible(self._p, dumps(obj), out, 64)
        if n < 0:
            raise ValueError(lib().rc_last_error().decode())
        return [out[i] for i in range(n)]

    def weight(self, i: int, obj):
        out = C.c_int64()
        ok = lib().rc_stage_weight(self._p, i, dumps(obj), C.byref(out))
        return out.value, bool(ok)

    def delay(self, i: int, obj, now_ns: int, seed: int = 0, step: int = 0, slot: int = 0):
        out = C.c_int64()
        ok = lib().rc_stage_delay(self._p, i, dumps(obj), now_ns, seed, step, slot, C.byref(out))
        return out.value, bool(ok)

    def finalizers(self, i: int, meta):
        return json.loads(_call_str(lib().rc_stage_finalizers, self._p, i, dumps(meta)))

    def match_batch(self, objs_json, now_ns, seed, step, slot_base=0, nthreads=1):
        """Reference-faithful batch: re-parse each object's JSON then Match + Delay."""
        import numpy as np
        blob = b"".join(objs_json)
        offs = np.zeros(len(objs_json) + 1, dtype=np.int64)
        np.cumsum([len(o) for o in objs_json], out=offs[1:])
        st = np.zeros(len(objs_json), dtype=np.int32)
        de = np.zeros(len(objs_json), dtype=np.int64)
        n = lib().rc_match_batch(self._p, blob, offs.ctypes.data_as(C.POINTER(C.c_int64)), len(objs_json), now_ns,
                                 seed, step, slot_base, st.ctypes.data_as(C.POINTER(C.c_int32)),
                                 de.ctypes.data_as(C.POINTER(C.c_int64)), nthreads)
        return st, de, n


def soa_steps(table, deltas, harness, pred, sched, due, now0_ns: int, dt_ns: int, steps: int, seed: int,
              nthreads: int) -> int:
    """TIMING BASELINE ONLY: the compiled stage program stepped over SoA columns on nthreads
    host threads (rc_soa_steps); the columns are updated in place.  -> transitions fired."""
    import numpy as np
    L = lib()
    L.rc_soa_steps.restype = C.c_int64
    L.rc_soa_steps.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                               C.c_int64, C.c_int64, C.c_int, C.c_uint64, C.c_int]
    d = np.ascontiguousarray(deltas, dtype=np.uint32)
    return L.rc_soa_steps(C.addressof(table), d.ctypes.data, C.addressof(harness), pred.ctypes.data, sched.ctypes.data,
                          due.ctypes.data, len(pred), now0_ns, dt_ns, steps, seed, nthreads)
