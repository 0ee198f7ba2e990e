"""Native ingestion encoder: the stage compiler's feature table as a
spec for libkwok_encoder.so (kwok_amd/csrc/encoder.cpp, include/kwok_encoder.h), and
``NativeIngest``, a drop-in for ``engine.Ingest`` that encodes JSON bytes without per-object
Python (a Go host hands the informer's bytes straight to kwk_encode).

Feature and *From queries travel as their jq source; the encoder compiles them with the native
jq subset (kwok_amd/csrc/jqc.hpp; the Python mirror is jq.py): path steps and select(path ==
literal) — the forms of kustomize/stage/** — run as step programs, everything else (length, not,
comparisons, //, has, arithmetic, ...) through the evaluator.  A query outside the subset is
rejected at ``encoder_spec`` time with the construct named.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import re
from typing import List, Optional, Sequence

import numpy as np

from . import abi
from .compiler import _IDENTITY_META, KindProgram
from .jq import JqError, Query

LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libkwok_encoder.so")
CLASS_UNKNOWN = 0xFFFF


class EncoderUnsupported(ValueError):
    pass


def check_query(src: str) -> str:
    """A selector key / getter query the native encoder compiles (kwok_amd/csrc/jqc.hpp, mirrored
    by jq.py), or EncoderUnsupported naming the construct."""
    try:
        Query(src)
    except JqError as e:
        raise EncoderUnsupported(str(e)) from None
    return src


def encoder_spec(program: KindProgram) -> str:
    if hasattr(program, "encoder_spec"):  # native_compiler.NativeProgram: libkwok_compiler writes it
        return program.encoder_spec()
    if program.applied_bits:
        raise EncoderUnsupported("'patch already applied' features need the host renderer")
    feats = [{"query": check_query(f.src), "present_bit": f.present_bit, "literals": dict(f.lit_bits)}
             for f in program.features.values()]
    slots = [{"type": typ, "query": check_query(src)} for typ, src in program.slots]
    spec = {"features": feats, "finalizers": dict(program.fin_bits), "finalizer_other_bit": program.fin_other_bit,
            "slots": slots, "classes": dict(program.class_ids), "identity_meta": list(_IDENTITY_META)}
    if program.disregard is not None:  # need()'s selectors, evaluated by the encoder into one bit
        spec["disregard"] = program.describe()["disregard"]
    return json.dumps(spec)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise abi.EngineError(f"native encoder library missing: {LIB_PATH} (run python -m kwok_amd.build)")
        L = C.CDLL(LIB_PATH)
        L.kwk_encoder_last_error.restype = C.c_char_p
        L.kwk_encoder_last_error.argtypes = [C.c_void_p]
        L.kwk_encoder_create.argtypes = [C.c_char_p, C.POINTER(C.c_void_p)]
        L.kwk_encoder_destroy.argtypes = [C.c_void_p]
        L.kwk_encode.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                 C.c_void_p, C.c_void_p, C.POINTER(C.c_uint32)]
        L.kwk_encoder_records.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]
        L.kwk_jq_eval.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_uint32, C.POINTER(C.c_uint32)]
        L.kwk_encoder_add_classes.argtypes = [C.c_void_p, C.c_char_p]
        for n in ("kwk_encoder_create", "kwk_encoder_destroy", "kwk_encode", "kwk_encoder_records", "kwk_jq_eval",
                  "kwk_encoder_add_classes"):
            getattr(L, n).restype = C.c_int32
        _lib = L
    return _lib


def _check(st, what, h=None):
    """Raise for a failed call; the message is the handle's own (per handle), or the calling
    thread's for create."""
    if st != 0:
        raise abi.EngineError(f"{what} failed ({st}): {lib().kwk_encoder_last_error(h).decode(errors='replace')}")


def pack_json(objs: Sequence) -> tuple:
    """Objects (dicts or JSON bytes) -> (contiguous buffer, n + 1 offsets)."""
    parts = [o if isinstance(o, (bytes, bytearray)) else json.dumps(o, separators=(",", ":")).encode() for o in objs]
    offs = np.zeros(len(parts) + 1, dtype=np.uint64)
    np.cumsum([len(p) for p in parts], out=offs[1:])
    return b"".join(parts), offs


def jq_eval(query: str, doc) -> Optional[list]:
    """kwk_jq_eval: Query.Execute of `query` on `doc` (a dict or JSON text) with the native jq subset
    -> the outputs (nulls dropped) or None for the nil result; EncoderUnsupported outside the subset."""
    text = doc if isinstance(doc, (str, bytes)) else json.dumps(doc)
    text = text.encode() if isinstance(text, str) else text
    n = C.c_uint32()
    cap = 4096
    while True:
        buf = C.create_string_buffer(cap)
        st = lib().kwk_jq_eval(query.encode(), text, buf, cap, C.byref(n))
        if st == abi.KWK_ECAP:
            cap = n.value + 1
            continue
        if st == abi.KWK_EINVAL:
            raise EncoderUnsupported(lib().kwk_encoder_last_error(None).decode(errors="replace"))
        _check(st, "kwk_jq_eval")
        return json.loads(buf.value.decode())


class NativeIngest:
    """engine.Ingest through libkwok_encoder: columns() of JSON objects / bytes."""

    def __init__(self, program: KindProgram, n_threads: int = 1):
        self.p = program
        self.n_threads = n_threads
        self.h = C.c_void_p()
        _check(lib().kwk_encoder_create(encoder_spec(program).encode(), C.byref(self.h)), "kwk_encoder_create")

    def close(self):
        if self.h:
            lib().kwk_encoder_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def encode_buffer(self, buf: bytes, offsets: np.ndarray):
        n = len(offsets) - 1
        hot = np.zeros(n, dtype=abi.HOT_DTYPE)
        dels = np.zeros(n, dtype=np.int64)
        rec = np.zeros(n, dtype=np.uint32)
        cls = np.zeros(n, dtype=np.uint16)
        unknown = C.c_uint32()
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        _check(lib().kwk_encode(self.h, n, buf, abi.ptr(offsets), self.n_threads, abi.ptr(hot), abi.ptr(dels),
                                abi.ptr(rec), abi.ptr(cls), C.byref(unknown)), "kwk_encode", self.h)
        self.unknown_classes = unknown.value
        return hot, dels, rec, cls

    def refresh_classes(self):
        """Hand the classes the stage compiler registered since to the native encoder
        (kwk_encoder_add_classes); its record table stays as it is."""
        _check(lib().kwk_encoder_add_classes(self.h, json.dumps(dict(self.p.class_ids)).encode()),
               "kwk_encoder_add_classes", self.h)

    def columns(self, objs: Sequence, register: bool = False):
        """register: objects of a class the compiler has not seen get it registered (their
        deltas are then UNKNOWN until explored) and are re-encoded natively, so that every row's
        record id points into this encoder's record table."""
        out = self.encode_buffer(*pack_json(objs))
        unknown = np.flatnonzero(out[3] == CLASS_UNKNOWN)
        if register and len(unknown):
            for i in unknown:
                self.p.class_of(json.loads(objs[i]) if isinstance(objs[i], (bytes, bytearray)) else objs[i])
            self.refresh_classes()
            again = self.encode_buffer(*pack_json([objs[i] for i in unknown]))
            for col, new in zip(out, again):
                col[unknown] = new
            assert not np.any(out[3] == CLASS_UNKNOWN)
        return out

    def record_array(self) -> np.ndarray:
        ns = max(1, len(self.p.slots))
        n = C.c_uint32()
        _check(lib().kwk_encoder_records(self.h, None, 0, C.byref(n)), "kwk_encoder_records", self.h)
        a = np.zeros((max(1, n.value), ns), dtype=abi.VALUE_DTYPE)
        if n.value and self.p.slots:
            _check(lib().kwk_encoder_records(self.h, abi.ptr(a), n.value, C.byref(n)), "kwk_encoder_records", self.h)
        return a
