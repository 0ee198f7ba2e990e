"""ctypes binding of libkwok_comm (include/kwok_comm.h): the reporting interval's RCCL all-reduce
of the engines' device aggregates without torch.distributed — the path a Go host takes.

``NativeReport`` is ``cluster.DeviceReport`` on it: per engine kwk_aggregate into the
communicator's device buffer, then one in-place all-reduce ordered after the engines' streams.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import abi

LIB_PATH = os.path.join(os.path.dirname(abi.LIB_PATH), "libkwok_comm.so")
ID_BYTES = 128
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise abi.EngineError(f"native collective library missing: {LIB_PATH} (run python -m kwok_amd.build)")
        abi.lib()  # the engine library first (libkwok_comm links it)
        L = C.CDLL(LIB_PATH)
        L.kwk_comm_last_error.restype = C.c_char_p
        L.kwk_comm_last_error.argtypes = [C.c_void_p]
        L.kwk_comm_unique_id.argtypes = [C.c_void_p]
        L.kwk_comm_init.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]
        L.kwk_comm_destroy.argtypes = [C.c_void_p]
        L.kwk_comm_buffer.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)]
        L.kwk_comm_allreduce.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32]
        L.kwk_comm_read.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        for n in ("kwk_comm_unique_id", "kwk_comm_init", "kwk_comm_destroy", "kwk_comm_buffer", "kwk_comm_allreduce",
                  "kwk_comm_read"):
            getattr(L, n).restype = C.c_int32
        _lib = L
    return _lib


def _check(st, what, h=None):
    if st != abi.KWK_OK:
        raise abi.EngineError(f"{what} failed ({st}): {lib().kwk_comm_last_error(h).decode(errors='replace')}")


def unique_id() -> bytes:
    buf = (C.c_uint8 * ID_BYTES)()
    _check(lib().kwk_comm_unique_id(buf), "kwk_comm_unique_id")
    return bytes(buf)


class NativeComm:
    def __init__(self, uid: bytes, rank: int, world: int, device: int = 0):
        assert len(uid) == ID_BYTES
        self.h = C.c_void_p()
        ub = (C.c_uint8 * ID_BYTES).from_buffer_copy(uid)
        _check(lib().kwk_comm_init(ub, rank, world, device, C.byref(self.h)), "kwk_comm_init")
        self.rank, self.world = rank, world

    def buffer(self, n: int) -> int:
        """The communicator's device buffer for n float64 (growing it frees the previous one:
        a report holding an older pointer fails loudly in collect, see NativeReport)."""
        p = C.c_void_p()
        _check(lib().kwk_comm_buffer(self.h, n, C.byref(p)), "kwk_comm_buffer", self.h)
        self.base = int(p.value)
        return self.base

    def allreduce(self, n: int, engines):
        arr = (C.c_void_p * max(1, len(engines)))(*[e.h.value for e in engines])
        _check(lib().kwk_comm_allreduce(self.h, n, arr, len(engines)), "kwk_comm_allreduce", self.h)

    def read(self, n: int) -> np.ndarray:
        out = np.zeros(n, dtype=np.float64)
        _check(lib().kwk_comm_read(self.h, abi.ptr(out), n), "kwk_comm_read", self.h)
        return out

    def close(self):
        if self.h:
            lib().kwk_comm_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class NativeReport:
    """cluster.DeviceReport over libkwok_comm: the aggregates of `engines` back to back in the
    communicator's buffer, all-reduced in place (enqueue only); `result` reads them back."""

    def __init__(self, comm: NativeComm, engines, count_masks, count_names, usage_engine=None):
        from .cluster import DeviceReport
        self._layout = DeviceReport(engines, count_masks, count_names, usage_engine)  # sizes + result decoding
        self.comm, self.engines = comm, engines
        self.n = sum(self._layout.sizes)
        self.base = comm.buffer(self.n)

    def collect(self, now_ns: int):
        if self.comm.base != self.base:
            raise abi.EngineError("the communicator's buffer was reallocated by a larger report after this one "
                                  "was created: size the buffer for every report first")
        off = 0
        L = self._layout
        for e, m, size in zip(self.engines, L.masks, L.sizes):
            n = e.aggregate(m, now_ns, usage=e is L.usage_engine, out_ptr=self.base + 8 * off)
            assert n == size, (n, size)
            off += size
        self.comm.allreduce(self.n, self.engines)

    def result(self):
        return self._layout.decode(self.comm.read(self.n))
