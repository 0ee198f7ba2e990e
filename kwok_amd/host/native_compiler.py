"""ctypes binding of libkwok_compiler.so (include/kwok_compiler.h): the native Stage compiler, i.e.
lifecycle.NewLifecycle's compilation (pkg/utils/lifecycle/lifecycle.go:33-46,194-267) behind the
C ABI — what a Go host calls through cgo (LoadStages).

``NativeProgram`` offers the part of ``compiler.KindProgram``'s interface the engine, the native
encoder and the native patch renderer consume (table / delta_array / harness_struct / describe /
class_of / explore / the encoder and patch specs), computed by the C++ library; the Python
KindProgram is its CPU cross-check (tests/test_native_compiler.py: byte-equal outputs).
"""
from __future__ import annotations

import ctypes as C
import json
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import yaml

from . import abi

LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libkwok_compiler.so")
MAX_PATCHES = 8  # KWK_MAX_PATCHES

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise abi.EngineError(f"native compiler library missing: {LIB_PATH} (run python -m kwok_amd.build)")
        L = C.CDLL(LIB_PATH)
        L.kwk_program_last_error.restype = C.c_char_p
        L.kwk_program_last_error.argtypes = [C.c_void_p]
        L.kwk_compile_stages.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_void_p)]
        L.kwk_program_destroy.argtypes = [C.c_void_p]
        L.kwk_program_explore.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, C.c_void_p]
        L.kwk_program_class.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64, C.c_int32, C.POINTER(C.c_uint32)]
        L.kwk_program_table.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
        L.kwk_program_deltas.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.kwk_program_harness.argtypes = [C.c_void_p, C.c_void_p]
        L.kwk_program_value_slots.argtypes = [C.c_void_p, C.POINTER(C.c_uint32)]
        for n in ("kwk_program_describe", "kwk_program_class_keys", "kwk_program_encoder_spec"):
            getattr(L, n).argtypes = [C.c_void_p, C.POINTER(C.c_char_p)]
        L.kwk_program_patch_spec.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.POINTER(C.c_char_p), C.c_void_p,
                                             C.c_uint32]
        for n in ("kwk_compile_stages", "kwk_program_destroy", "kwk_program_explore", "kwk_program_class",
                  "kwk_program_table", "kwk_program_deltas", "kwk_program_harness", "kwk_program_value_slots",
                  "kwk_program_describe", "kwk_program_class_keys", "kwk_program_encoder_spec",
                  "kwk_program_patch_spec"):
            getattr(L, n).restype = C.c_int32
        _lib = L
    return _lib


class CompileError(ValueError):
    pass


def stage_docs_from_files(*paths: str) -> List[dict]:
    """The v1alpha1 Stage documents of YAML files, in file order (the Go host has them decoded)."""
    out = []
    for p in paths:
        for d in yaml.safe_load_all(open(p).read()):
            if d:
                out.append(d)
    return out


class NativeProgram:
    """One resourceRef's Stage list compiled by libkwok_compiler (kwk_compile_stages)."""

    def __init__(self, stage_docs: Sequence[dict], harness=None, disregard=None):
        """harness: None, True (the default HarnessSpec) or a compiler.HarnessSpec; disregard: a
        labelsel.DisregardSpec (need()'s selectors)."""
        o = {}
        if harness is not None:
            o["harness"] = {} if harness is True else {"terminal_query": harness.terminal_query,
                                                       "terminal_values": list(harness.terminal_values),
                                                       "deletion_query": harness.deletion_query}
        if disregard is not None and disregard.active:
            o["disregard"] = {"annotation_selector": disregard.annotation_selector,
                              "label_selector": disregard.label_selector}
        opts = json.dumps(o).encode() if o else None
        self.harness = harness
        self.h = C.c_void_p()
        st = lib().kwk_compile_stages(json.dumps(list(stage_docs)).encode(), opts, C.byref(self.h))
        if st != 0:
            raise CompileError(lib().kwk_program_last_error(None).decode(errors="replace"))
        # the typed Stage objects the host keeps beside the program (the Go host has them decoded):
        # the controller applies their finalizer / delete / patch lists to its object cache
        from .stages import stage_from_v1alpha1
        self.stages = [s for s in (stage_from_v1alpha1(d) for d in stage_docs) if s.selector is not None]
        self._refresh()

    def _check(self, st, what):
        if st != 0:
            raise CompileError(f"{what} failed ({st}): {lib().kwk_program_last_error(self.h).decode(errors='replace')}")

    def _json(self, fn) -> str:
        p = C.c_char_p()
        self._check(fn(self.h, C.byref(p)), fn.__name__)
        return p.value.decode()

    def _refresh(self):
        self._desc = json.loads(self._json(lib().kwk_program_describe))
        self.names: List[str] = self._desc["stages"]
        self.slots: List[Tuple[str, str]] = [tuple(s) for s in self._desc["value_slots"]]
        self.class_ids: Dict[str, int] = json.loads(self._json(lib().kwk_program_class_keys))
        self.applied_bits = {self.names.index(n): b for n, b in self._desc["applied_bits"].items()}

    def close(self):
        if self.h:
            lib().kwk_program_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- KindProgram's interface
    def explore(self, roots: Sequence):
        from .encoder import pack_json
        if not len(roots):
            return
        buf, offs = pack_json(roots)
        self._check(lib().kwk_program_explore(self.h, len(roots), buf, abi.ptr(np.ascontiguousarray(offs))),
                    "kwk_program_explore")
        self._refresh()

    def class_of(self, obj, register: bool = True) -> int:
        b = obj if isinstance(obj, (bytes, bytearray)) else json.dumps(obj, separators=(",", ":")).encode()
        c = C.c_uint32()
        self._check(lib().kwk_program_class(self.h, b, len(b), 1 if register else 0, C.byref(c)), "kwk_program_class")
        if c.value == 0xFFFFFFFF:
            raise CompileError("unknown object class")
        self._refresh()
        return int(c.value)

    def table(self, version: int = 1) -> abi.StageTable:
        t = abi.StageTable()
        self._check(lib().kwk_program_table(self.h, version, C.byref(t)), "kwk_program_table")
        return t

    def delta_array(self) -> np.ndarray:
        nc, ns = C.c_uint32(), C.c_uint32()
        self._check(lib().kwk_program_deltas(self.h, None, 0, C.byref(nc), C.byref(ns)), "kwk_program_deltas")
        a = np.zeros((nc.value, ns.value, 2), dtype=np.uint32)
        self._check(lib().kwk_program_deltas(self.h, abi.ptr(a), nc.value * ns.value, C.byref(nc), C.byref(ns)),
                    "kwk_program_deltas")
        return a

    def harness_struct(self) -> abi.Harness:
        h = abi.Harness()
        self._check(lib().kwk_program_harness(self.h, C.byref(h)), "kwk_program_harness")
        return h

    def describe(self) -> dict:
        return dict(self._desc)

    @property
    def uses_deletion_column(self) -> bool:
        return bool(self._desc["uses_deletion_column"])

    def encoder_spec(self) -> str:
        return self._json(lib().kwk_program_encoder_spec)

    def patch_spec(self, funcs: Optional[Dict[str, object]] = None, version: str = "v0.6.0"):
        """-> (spec JSON for kwk_patcher_create, {(stage, patch): template id}) — PatchProgram's
        spec for the same controller functions (a str value is a constant, anything else a
        callback)."""
        fl = [{"name": n, "const": v} if isinstance(v, str) else {"name": n, "callback": True}
              for n, v in sorted((funcs or {}).items())]
        n = max(1, len(self.names)) * MAX_PATCHES
        tof = np.zeros(n, dtype=np.int32)
        p = C.c_char_p()
        self._check(lib().kwk_program_patch_spec(self.h, json.dumps(fl).encode(), version.encode(), C.byref(p),
                                                 abi.ptr(tof), n), "kwk_program_patch_spec")
        tmap = {(s, k): int(tof[s * MAX_PATCHES + k]) for s in range(len(self.names)) for k in range(MAX_PATCHES)
                if tof[s * MAX_PATCHES + k] >= 0}
        return p.value.decode(), tmap
