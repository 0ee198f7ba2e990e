"""ctypes binding of the native Metric CR compiler in libkwok_compiler.so (include/kwok_metrics.h):
a Metric CR's gauge / counter / histogram values lowered to the device programs of
kwk_metrics_load / kwk_histograms_load by C++ (kwok_amd/csrc/metrics_compiler.cpp, celc.hpp) —
what a Go host calls through cgo instead of compiling CEL per scrape
(pkg/kwok/metrics/metrics.go:168-462, evaluator.go:51-144; INTEGRATION.md: LoadMetrics).

The Python lowering (cel.lower through metrics.MetricsProgram) is its CPU cross-check: the packed
arrays are byte-equal (tests/test_metric_compiler.py)."""
from __future__ import annotations

import ctypes as C
import json
from typing import List, Tuple

from . import abi, cel
from .native_compiler import lib as _compiler_lib

KWK_ENOLOWER = -5

_bound = False


def lib():
    global _bound
    L = _compiler_lib()
    if not _bound:
        L.kwk_metric_set_last_error.restype = C.c_char_p
        L.kwk_metric_set_last_error.argtypes = [C.c_void_p]
        L.kwk_compile_metrics.argtypes = [C.c_char_p, C.POINTER(C.c_void_p)]
        L.kwk_metric_set_destroy.argtypes = [C.c_void_p]
        L.kwk_metric_set_programs.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_void_p),
                                              C.POINTER(C.c_uint32), C.POINTER(C.c_void_p)]
        L.kwk_metric_set_histograms.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_void_p),
                                                C.POINTER(C.c_uint32), C.POINTER(C.c_void_p),
                                                C.POINTER(C.c_uint32), C.POINTER(C.c_void_p)]
        L.kwk_metric_set_describe.argtypes = [C.c_void_p, C.POINTER(C.c_char_p)]
        L.kwk_cel_lower.argtypes = [C.c_char_p, C.c_uint32, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]
        for n in ("kwk_compile_metrics", "kwk_metric_set_destroy", "kwk_metric_set_programs",
                  "kwk_metric_set_histograms", "kwk_metric_set_describe", "kwk_cel_lower"):
            getattr(L, n).restype = C.c_int32
        _bound = True
    return L


class MetricCompileError(ValueError):
    pass


DIMS = {"node": 0, "pod": 1, "container": 2}


def cel_lower(expr: str, dimension: str) -> List[Tuple[int, float]]:
    """kwk_cel_lower in cel.lower's output form [(op, operand)] (operand: the input index for a
    load, the constant for a constant, 0.0 otherwise); cel.LowerError when the expression has no
    device form, MetricCompileError when it does not compile."""
    L = lib()
    n = C.c_uint32()
    cap = 256
    ops = (abi.MetricOp * cap)()
    st = L.kwk_cel_lower(expr.encode(), DIMS.get(dimension, 3), ops, cap, C.byref(n))
    if st == abi.KWK_ECAP and n.value > cap:  # a longer program: *n_ops = the length it needs
        cap = n.value
        ops = (abi.MetricOp * cap)()
        st = L.kwk_cel_lower(expr.encode(), DIMS.get(dimension, 3), ops, cap, C.byref(n))
    if st == KWK_ENOLOWER:
        raise cel.LowerError(L.kwk_metric_set_last_error(None).decode(errors="replace"))
    if st != 0:
        raise MetricCompileError(L.kwk_metric_set_last_error(None).decode(errors="replace"))
    out = []
    for o in ops[:n.value]:
        out.append((int(o.op), int(o.arg) if o.op == cel.OP_LOAD else float(o.value) if o.op == cel.OP_CONST else 0.0))
    return out


class NativeMetricSet:
    """One Metric CR compiled by kwk_compile_metrics."""

    def __init__(self, metric_doc: dict):
        self.h = C.c_void_p()
        L = lib()
        st = L.kwk_compile_metrics(json.dumps(metric_doc).encode(), C.byref(self.h))
        if st != 0:
            raise MetricCompileError(L.kwk_metric_set_last_error(None).decode(errors="replace"))
        s = C.c_char_p()
        L.kwk_metric_set_describe(self.h, C.byref(s))
        self.describe = json.loads(s.value.decode())
        self.host_metrics: List[str] = list(self.describe["host_metrics"])

    def close(self):
        if self.h:
            lib().kwk_metric_set_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def programs_raw(self):
        """(n_metrics, desc pointer, n_ops, op pointer) owned by the set: kwk_metrics_load's arguments."""
        n, d, no, o = C.c_uint32(), C.c_void_p(), C.c_uint32(), C.c_void_p()
        st = lib().kwk_metric_set_programs(self.h, C.byref(n), C.byref(d), C.byref(no), C.byref(o))
        if st != 0:
            raise MetricCompileError("kwk_metric_set_programs")
        return n.value, d, no.value, o

    def histograms_raw(self):
        n, d, nb, b, no, o = C.c_uint32(), C.c_void_p(), C.c_uint32(), C.c_void_p(), C.c_uint32(), C.c_void_p()
        st = lib().kwk_metric_set_histograms(self.h, C.byref(n), C.byref(d), C.byref(nb), C.byref(b), C.byref(no),
                                             C.byref(o))
        if st != 0:
            raise MetricCompileError("kwk_metric_set_histograms")
        return n.value, d, nb.value, b, no.value, o

    def programs_bytes(self) -> Tuple[bytes, bytes]:
        n, d, no, o = self.programs_raw()
        return C.string_at(d, n * C.sizeof(abi.MetricDesc)) if n else b"", \
            C.string_at(o, no * C.sizeof(abi.MetricOp)) if no else b""

    def histograms_bytes(self) -> Tuple[bytes, bytes, bytes]:
        n, d, nb, b, no, o = self.histograms_raw()
        return (C.string_at(d, n * C.sizeof(abi.HistogramDesc)) if n else b"",
                C.string_at(b, nb * C.sizeof(abi.MetricBucket)) if nb else b"",
                C.string_at(o, no * C.sizeof(abi.MetricOp)) if no else b"")

    def load(self, pods_engine):
        """kwk_metrics_load (+ kwk_histograms_load when the CR has histograms) from the set's arrays."""
        pods_engine.metrics_load_arrays(*self.programs_raw())
        h = self.histograms_raw()
        if h[0]:
            pods_engine.histograms_load_arrays(*h)
