"""Device patch emission (include/kwok_emit.h), host side: skeleton table, per-object words and
value columns, and the emitter handle.

Reference: playStage's per-fire patch rendering (pkg/utils/lifecycle/next.go:73-160,
pkg/utils/gotpl/renderer.go:59-124).  ``EmitProgram`` builds, once per (class, template), the
skeleton kwk_patch_skeleton returns (literal runs + Now / call-value slots + status guards) and
derives each guard's effect of the template's patch by applying it (nextstate.merge_patch) to
the class representative with the guard met and not met.  ``EmitProgram.rows`` checks objects
with kwk_patch_object_values (their render equals the class skeleton; their call values fixed)
and returns the slot words and value-column rows the device needs.  ``Emitter`` runs
kwk_emit over the engine's fired list and hands back the patches; items with status
KWK_EMIT_HOST are rendered by the host (``PatchProgram.render`` / the full renderer).
"""
from __future__ import annotations

import copy
import ctypes as C
import json
import os
from collections import defaultdict
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .gotpl import rfc3339nano
from .nextstate import merge_patch

LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libkwok_emit.so")
NO_SLOT = 0xFFFF
STATUS_OK, STATUS_HOST = 0, 1
FROM_RECORDS, FROM_PACKED = 0, 1
MAX_GUARDS = 8
MARKER = "\U0010FFFD"


class EmitPiece(C.Structure):
    _fields_ = [("lit_off", C.c_uint32), ("lit_len", C.c_uint16), ("slot", C.c_uint16)]


class EmitSkel(C.Structure):
    _fields_ = [("first_piece", C.c_uint32), ("n_pieces", C.c_uint32), ("need", C.c_uint8), ("keep", C.c_uint8),
                ("set", C.c_uint8), ("reserved", C.c_uint8)]


class EmitProgramStruct(C.Structure):
    _fields_ = [("n_classes", C.c_uint32), ("n_templates", C.c_uint32), ("n_stages", C.c_uint32),
                ("n_skels", C.c_uint32), ("n_pieces", C.c_uint32), ("n_columns", C.c_uint32),
                ("n_lit_bytes", C.c_uint64), ("stage_tpl_ptr", C.c_void_p), ("stage_tpl", C.c_void_p),
                ("stage_delete", C.c_void_p), ("skel_of", C.c_void_p), ("skels", C.c_void_p), ("pieces", C.c_void_p),
                ("lits", C.c_void_p), ("fresh_guards", C.c_void_p), ("column_stride", C.c_void_p)]


class EmitItem(C.Structure):
    _fields_ = [("rec", C.c_uint32), ("tid", C.c_uint16), ("status", C.c_uint8), ("reserved", C.c_uint8)]


ITEM_DTYPE = np.dtype([("rec", "<u4"), ("tid", "<u2"), ("status", "u1"), ("reserved", "u1")])


def _get(obj, path):
    v = obj
    for k in path:
        if not isinstance(v, dict) or k not in v:
            return None
        v = v[k]
    return v


def guard_holds(obj: dict, guard) -> bool:
    """The render's `index $root.<P> $i` for every index of `range $i := <B>` succeeds."""
    p, b = guard
    bl = _get(obj, b)
    n = len(bl) if isinstance(bl, list) else 0
    if n == 0:
        return True
    pv = _get(obj, p)
    return isinstance(pv, dict) or (isinstance(pv, list) and len(pv) >= n)


def _set_path(obj, path, value):
    o = obj
    for k in path[:-1]:
        if not isinstance(o.get(k), dict):
            o[k] = {}
        o = o[k]
    if value is None:
        o.pop(path[-1], None)
    else:
        o[path[-1]] = value


class EmitProgram:
    """Skeleton table of a PatchProgram's templates over object classes.

    stages: the Stage list the engine's table was built from (stage index order);
    patch_program: patchtpl.PatchProgram over those stages; reps: {class id: representative
    object}; n_classes: the engine's class count (classes without a representative are rendered
    by the host); stride: bytes per call value row ([length][text], at most stride - 1 chars).
    """

    def __init__(self, stages, patch_program, reps: Dict[int, dict], n_classes: int, stride: int = 32):
        self.stages, self.pp, self.stride = list(stages), patch_program, stride
        self.n_classes = n_classes
        n_pp = 1 + max(patch_program.template_of.values(), default=-1)
        self.host_tid = n_pp  # stands for a patch libkwok_patch does not compile: always the host's
        self.n_templates = n_pp + 1
        if self.n_templates > 32:
            raise ValueError("more than 31 patch templates: the emitter's accepted mask is 32 bits")
        self.stage_tpl: List[List[int]] = []
        for si, st in enumerate(self.stages):
            tids = []
            for pi in range(0 if st.next.delete else len(st.next.patches)):  # a delete applies no patch
                tids.append(patch_program.template_of.get((si, pi), self.host_tid))
            self.stage_tpl.append(tids)
        self.guards: List[Tuple[tuple, tuple]] = []
        self.skel: Dict[Tuple[int, int], dict] = {}  # (class, tid) -> skeleton (eligible ones)
        self.reasons: Dict[Tuple[int, int], str] = {}
        self.calls: Dict[int, int] = {}  # tid -> call sites (the same for every class)
        self.reps = dict(reps)
        for cls, rep in sorted(self.reps.items()):
            for tid in range(n_pp):
                sk = patch_program.skeleton(tid, rep)
                if not sk["eligible"]:
                    self.reasons[(cls, tid)] = sk["reason"]
                    continue
                gs = [(tuple(p), tuple(b)) for p, b in sk["guards"]]
                bits = 0
                for g in gs:
                    if g not in self.guards:
                        if len(self.guards) == MAX_GUARDS:
                            self.reasons[(cls, tid)] = "more than 8 status guards"
                            bits = None
                            break
                        self.guards.append(g)
                    bits |= 1 << self.guards.index(g)
                if bits is None:
                    continue
                if self.calls.setdefault(tid, sk["calls"]) != sk["calls"]:
                    self.reasons[(cls, tid)] = "call sites differ between classes"
                    continue
                sk["need"] = bits
                sk["guard_list"] = gs
                self.skel[(cls, tid)] = sk
        for key in list(self.skel):  # every guard known: each patch's effect on each
            sk = self.skel[key]
            try:
                sk["keep"], sk["set"] = self._effect(self.reps[key[0]], key[1], sk, sk["guard_list"])
            except ValueError:  # a Now / call-value slot outside a JSON string: no stand-in text parses
                del self.skel[key]
                self.reasons[key] = "a value slot outside a JSON string"
        # value columns: one per (template, call site)
        self.col_base: Dict[int, int] = {}
        n_cols = 0
        for tid in sorted(self.calls):
            self.col_base[tid] = n_cols
            n_cols += self.calls[tid]
        self.n_columns = n_cols
        self._build_struct()

    def _effect(self, rep, tid, sk, needed):
        """(keep, set) masks over every guard: the patch applied with each guard met / not met."""
        keep = setv = 0
        text = sk["lits"][0]
        for j, s in enumerate(sk["slots"]):
            text += ("2000-01-01T00:00:00Z" if s == 0 else "x") + sk["lits"][j + 1]
        patch = json.loads(text)
        for k, g in enumerate(self.guards):
            p, b = g
            bl = _get(rep, b)
            n = len(bl) if isinstance(bl, list) else 0
            post = []
            for met in (True, False):
                o = copy.deepcopy(rep)
                _set_path(o, p, [{} for _ in range(n)] if met else None)
                post.append(guard_holds(merge_patch(o, patch), g))
            if g in needed:  # rendered only with the guard met
                setv |= int(post[0]) << k
            elif post[0] and not post[1]:
                keep |= 1 << k
            elif post[0] == post[1]:
                setv |= int(post[0]) << k
        return keep, setv

    def guard_bits(self, obj) -> int:
        return sum(1 << k for k, g in enumerate(self.guards) if guard_holds(obj, g))

    def fresh_bits(self, cls) -> int:
        rep = self.reps.get(cls)
        if rep is None:
            return 0
        o = copy.deepcopy(rep)
        o.pop("status", None)
        return self.guard_bits(o)

    def _build_struct(self):
        lits = bytearray()
        pieces: List[tuple] = []
        skels: List[tuple] = []
        skel_of = np.full((self.n_classes, self.n_templates), -1, dtype=np.int32)
        for (cls, tid), sk in sorted(self.skel.items()):
            if cls >= self.n_classes:
                continue
            first = len(pieces)
            for j, lit in enumerate(sk["lits"]):
                b = lit.encode()
                if len(b) > 0xFFFF:
                    raise ValueError("literal run above 64 KiB")
                slot = NO_SLOT
                if j < len(sk["slots"]):
                    s = sk["slots"][j]
                    slot = 0 if s == 0 else 1 + self.col_base[tid] + (s - 1)
                pieces.append((len(lits), len(b), slot))
                lits += b
            skel_of[cls, tid] = len(skels)
            skels.append((first, len(pieces) - first, sk["need"], sk["keep"], sk["set"], 0))
        ptr = [0]
        flat: List[int] = []
        for tids in self.stage_tpl:
            flat += tids
            ptr.append(len(flat))
        self._a = {
            "stage_tpl_ptr": np.asarray(ptr, dtype=np.uint32),
            "stage_tpl": np.asarray(flat or [0], dtype=np.uint16),
            "stage_delete": np.asarray([1 if st.next.delete else 0 for st in self.stages] or [0], dtype=np.uint8),
            "skel_of": skel_of,
            "skels": (EmitSkel * max(1, len(skels)))(*[EmitSkel(*s) for s in skels]),
            "pieces": (EmitPiece * max(1, len(pieces)))(*[EmitPiece(*p) for p in pieces]),
            "lits": bytes(lits) or b"\0",
            "fresh": np.asarray([self.fresh_bits(c) for c in range(self.n_classes)] or [0], dtype=np.uint8),
            "stride": np.full(max(1, self.n_columns), self.stride, dtype=np.uint32),
        }
        a = self._a
        self.struct = EmitProgramStruct(
            self.n_classes, self.n_templates, len(self.stages), len(skels), len(pieces), self.n_columns, len(lits),
            abi.ptr(a["stage_tpl_ptr"]), abi.ptr(a["stage_tpl"]), abi.ptr(a["stage_delete"]), abi.ptr(a["skel_of"]),
            C.addressof(a["skels"]), C.addressof(a["pieces"]), C.cast(C.c_char_p(a["lits"]), C.c_void_p),
            abi.ptr(a["fresh"]), abi.ptr(a["stride"]))

    def rows(self, objs: Sequence[dict], classes: Sequence[int]):
        """-> (words uint64 [n], {column: uint8 [n, stride]}) for these objects (their current
        status gives the guard bits)."""
        n = len(objs)
        words = np.zeros(n, dtype=np.uint64)
        cols = {c: np.full((n, self.stride), 0xFF, dtype=np.uint8) for c in range(self.n_columns)}
        accepted = np.zeros(n, dtype=np.uint64)
        by = defaultdict(list)
        for i, c in enumerate(classes):
            by[int(c)].append(i)
        for cls, idx in by.items():
            group = [objs[i] for i in idx]
            for tid in range(self.host_tid):
                sk = self.skel.get((cls, tid))
                if sk is None:
                    continue
                vals, ok = self.pp.object_values(tid, group, sk["text"], sk["calls"], self.stride)
                ii = np.asarray(idx)
                accepted[ii] |= ok.astype(np.uint64) << np.uint64(tid)
                for c in range(sk["calls"]):
                    cols[self.col_base[tid] + c][ii] = vals[:, c, :]
        for i, (o, c) in enumerate(zip(objs, classes)):
            words[i] = (int(c) & 0xFFFF) | (self.guard_bits(o) << 16) | (int(accepted[i]) << 32)
        return words, cols


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise abi.EngineError(f"native emitter library missing: {LIB_PATH} (run python -m kwok_amd.build)")
        abi.lib()  # the engine library first (the emitter links to it)
        L = C.CDLL(LIB_PATH)
        L.kwk_emit_last_error.restype = C.c_char_p
        L.kwk_emit_last_error.argtypes = [C.c_void_p]
        L.kwk_emitter_create.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(EmitProgramStruct), C.POINTER(C.c_void_p)]
        L.kwk_emitter_destroy.argtypes = [C.c_void_p]
        L.kwk_emit_set_words.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
        L.kwk_emit_get_words.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
        L.kwk_emit_set_column.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]
        L.kwk_emit_reserve.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64]
        L.kwk_emit.argtypes = [C.c_void_p, C.c_int64, C.c_uint32]
        L.kwk_emit_result.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]
        L.kwk_emit_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]
        L.kwk_emit_device.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.kwk_emit_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.kwk_emit_elapsed.argtypes = [C.c_void_p, C.POINTER(C.c_float)]
        for n in EXPORTS:
            if n != "kwk_emit_last_error":
                getattr(L, n).restype = C.c_int32
        _lib = L
    return _lib


EXPORTS = ("kwk_emit_last_error", "kwk_emitter_create", "kwk_emitter_destroy", "kwk_emit_set_words",
           "kwk_emit_get_words", "kwk_emit_set_column", "kwk_emit_reserve", "kwk_emit", "kwk_emit_result",
           "kwk_emit_stats", "kwk_emit_device", "kwk_emit_copy", "kwk_emit_elapsed")


class Emitter:
    """kwk_emitter over an Engine's fired lists."""

    def __init__(self, engine, capacity: int, program: EmitProgram):
        self.program = program
        self.h = C.c_void_p()
        st = lib().kwk_emitter_create(engine.h, capacity, C.byref(program.struct), C.byref(self.h))
        if st != 0:
            raise abi.EngineError(f"kwk_emitter_create failed ({st}): {lib().kwk_emit_last_error(None).decode()}")
        self.engine = engine

    def _check(self, st, what):
        if st != 0:
            raise abi.EngineError(f"{what} failed ({st}): {lib().kwk_emit_last_error(self.h).decode(errors='replace')}")

    def close(self):
        if self.h:
            lib().kwk_emitter_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_rows(self, first: int, words: np.ndarray, cols: Dict[int, np.ndarray]):
        w = np.ascontiguousarray(words, dtype=np.uint64)
        self._check(lib().kwk_emit_set_words(self.h, first, len(w), abi.ptr(w)), "kwk_emit_set_words")
        for c, rows in cols.items():
            r = np.ascontiguousarray(rows, dtype=np.uint8)
            self._check(lib().kwk_emit_set_column(self.h, c, first, len(r), abi.ptr(r)), "kwk_emit_set_column")

    def set_slots(self, slots: np.ndarray, words: np.ndarray, cols: Dict[int, np.ndarray]):
        """Scattered slots (runs of consecutive slots go up together)."""
        slots = np.asarray(slots, dtype=np.int64)
        if len(slots) == 0:
            return
        order = np.argsort(slots, kind="stable")
        s = slots[order]
        breaks = np.flatnonzero(np.diff(s) != 1) + 1
        for a, b in zip(np.r_[0, breaks], np.r_[breaks, len(s)]):
            sel = order[a:b]
            self.set_rows(int(s[a]), words[sel], {c: v[sel] for c, v in cols.items()})

    def set_column(self, c: int, first: int, rows: np.ndarray):
        r = np.ascontiguousarray(rows, dtype=np.uint8)
        self._check(lib().kwk_emit_set_column(self.h, c, first, len(r), abi.ptr(r)), "kwk_emit_set_column")

    def words(self, first: int, n: int) -> np.ndarray:
        w = np.zeros(n, dtype=np.uint64)
        self._check(lib().kwk_emit_get_words(self.h, first, n, abi.ptr(w)), "kwk_emit_get_words")
        return w

    def reserve(self, items: int, nbytes: int):
        self._check(lib().kwk_emit_reserve(self.h, int(items), int(nbytes)), "kwk_emit_reserve")

    def emit(self, now_ns: int, packed: bool = True):
        """Enqueue the emission of the engine's last compacted list."""
        src = FROM_PACKED if packed else FROM_RECORDS
        self._check(lib().kwk_emit(self.h, int(now_ns), src), "kwk_emit")

    def result(self) -> Tuple[int, int]:
        """(items, bytes) of the last emission; abi.EngineError with KWK_ECAP when over the reservation."""
        ni, nb = C.c_uint32(), C.c_uint64()
        st = lib().kwk_emit_result(self.h, C.byref(ni), C.byref(nb))
        if st == abi.KWK_ECAP:
            return -int(ni.value) - 1, int(nb.value)
        self._check(st, "kwk_emit_result")
        return int(ni.value), int(nb.value)

    def stats(self) -> Tuple[int, int, int]:
        """(items, items emitted on the device, bytes) of the last emission."""
        ni, ne, nb = C.c_uint32(), C.c_uint32(), C.c_uint64()
        self._check(lib().kwk_emit_stats(self.h, C.byref(ni), C.byref(ne), C.byref(nb)), "kwk_emit_stats")
        return int(ni.value), int(ne.value), int(nb.value)

    def run(self, now_ns: int, packed: bool = True):
        """Emit (re-emitting once with enough room) -> (items structured array, offsets, bytes)."""
        self.emit(now_ns, packed)
        ni, nb = self.result()
        if ni < 0:
            self.reserve(-ni - 1, max(nb, 1))
            self.emit(now_ns, packed)
            ni, nb = self.result()
            if ni < 0:
                raise abi.EngineError("kwk_emit: reservation still too small")
        items = np.zeros(ni, dtype=ITEM_DTYPE)
        offs = np.zeros(ni + 1, dtype=np.uint64)
        out = np.zeros(max(nb, 1), dtype=np.uint8)
        self._check(lib().kwk_emit_copy(self.h, abi.ptr(items) if ni else None, abi.ptr(offs), abi.ptr(out)),
                    "kwk_emit_copy")
        return items, offs, out[:nb].tobytes()

    def elapsed_ms(self) -> float:
        ms = C.c_float()
        self._check(lib().kwk_emit_elapsed(self.h, C.byref(ms)), "kwk_emit_elapsed")
        return float(ms.value)


def substitute(sk: dict, now_ns: int, values: Sequence[str]) -> bytes:
    """A skeleton with its slots filled (the bytes the device writes; tests)."""
    now = rfc3339nano(now_ns)
    out = sk["lits"][0]
    for j, s in enumerate(sk["slots"]):
        out += (now if s == 0 else values[s - 1]) + sk["lits"][j + 1]
    return out.encode()
