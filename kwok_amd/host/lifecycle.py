"""Mirror of the reference's ``pkg/utils/lifecycle`` interface over the engine.

The Go controllers consume ``lifecycle.Lifecycle`` (lifecycle.go:49) through
``Match(ctx, labels, annotations, data) (*Stage, error)`` and then call
``Stage.Delay / Next / Name / ImmediateNextStage``.  This module keeps those names and
meanings so code (and tests) written against the reference read the same:

* ``Lifecycle.match(...)`` / ``match_batch(...)`` run the HIP sweep kernel in match-only
  mode (``kwk_match`` on a scratch engine over the given objects): matching, weighted pick
  and delay are computed on the GPU exactly as in ``kwk_step``, nothing fires;
* ``list_all_possible``, ``Stage.weight`` and ``Stage.delay`` are the deterministic helpers
  the stage tester uses (pkg/tools/stage/stage.go:37-85); they evaluate the compiled table on
  the host from the interned feature bits / pre-parsed records;
* ``Stage.next()`` returns the finalizer JSON patch / delete / rendered patches that the Go
  host produces for fired objects (next.go).

Randomness uses the same Philox4x32-10 hook as the device.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .compiler import KindProgram
from .engine import Engine, Ingest
from .goparse import INT64_MAX, INT64_MIN
from .gotpl import Renderer
from .nextstate import finalizers_modify, render_patches
from .stages import Stage as StageSpec

SITE_PICK, SITE_JITTER = 1, 2
_M = (1 << 32) - 1


def philox_u64(key: int, slot: int, step: int, site: int) -> int:
    """Philox4x32-10 (key = seed ^ kind_salt << 32, counter = (slot, step lo, step hi, site)); the
    pick (site 1) and the jitter (site 2) share the block of counter site 1: words 0-1 / 2-3."""
    jit = site == SITE_JITTER
    c0, c1, c2, c3 = slot & _M, step & _M, (step >> 32) & _M, (SITE_PICK if jit else site) & _M
    k0, k1 = key & _M, (key >> 32) & _M
    for _ in range(10):
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & _M, p1 & _M, ((p0 >> 32) ^ c3 ^ k1) & _M, p0 & _M
        k0 = (k0 + 0x9E3779B9) & _M
        k1 = (k1 + 0xBB67AE85) & _M
    return (c2 | (c3 << 32)) if jit else (c0 | (c1 << 32))


def rng_below(key: int, slot: int, step: int, site: int, n: int) -> int:
    return (philox_u64(key, slot, step, site) * n) >> 64


class Next:
    """lifecycle.Next (next.go:30-88)."""

    def __init__(self, spec: StageSpec):
        self._s = spec

    def finalizers(self, meta_finalizers) -> Optional[list]:
        if self._s.next.finalizers is None:
            return None
        ops = finalizers_modify(meta_finalizers, self._s.next.finalizers)
        return ops or None

    def delete(self) -> bool:
        return self._s.next.delete

    def event(self):
        return self._s.next.event

    def patches(self, resource: dict, renderer: Renderer):
        return render_patches(self._s, resource, renderer)


class Stage:
    """lifecycle.Stage (lifecycle.go:270-361)."""

    def __init__(self, lc: "Lifecycle", index: int):
        self._lc, self.index = lc, index
        self._spec = lc.program.stages[index]
        self._d = lc.program.stage_desc[index]

    def name(self) -> str:
        return self._spec.name

    def immediate_next_stage(self) -> bool:
        return self._spec.immediate_next_stage

    def next(self) -> Next:
        return Next(self._spec)

    def _getter(self, slot, default, default_ok, rec, dels, now, duration):
        if slot == abi.SLOT_NONE:
            return default, default_ok
        if slot == abi.SLOT_DELETION:
            if dels == abi.DEL_ABSENT:
                return default, default_ok
            return max(INT64_MIN, min(INT64_MAX, dels * 10**9 - now)), True
        if rec is None:
            return default, default_ok
        kind, value, nsec = rec[slot]
        if kind == abi.V_OK:
            return value, True
        if kind == abi.V_NOTOK:
            return 0, False
        if kind == abi.V_ABSTIME:
            if not duration:
                return 0, False
            return max(INT64_MIN, min(INT64_MAX, value * 10**9 + nsec - now)), True
        return default, default_ok

    def weight(self, data: dict) -> Tuple[int, bool]:
        """Stage.Weight (lifecycle.go:359-361)."""
        rec = self._lc.program.record_of(data)
        return self._getter(self._d.weight_slot, self._d.weight_default, True, rec, abi.DEL_ABSENT, 0, False)

    def delay(self, data: dict, now_ns: int, key: int = 0, slot: int = 0, step: int = 0) -> Tuple[int, bool]:
        """Stage.Delay (lifecycle.go:313-341) with the Philox jitter hook."""
        d = self._d
        if not d.has_delay:
            return 0, False
        rec = self._lc.program.record_of(data)
        dels = KindProgram.deletion_s(data)
        v, ok = self._getter(d.delay_slot, d.delay_default, True, rec, dels, now_ns, True)
        if not ok:
            return 0, False
        if not d.has_jitter:
            return v, True
        j, jok = self._getter(d.jitter_slot, d.jitter_default, bool(d.jitter_default_ok), rec, dels, now_ns, True)
        if not jok:
            return v, True
        if j < v:
            return j, True
        jit = (j - v) & ((1 << 64) - 1)
        jit = jit - (1 << 64) if jit >= 1 << 63 else jit
        if jit > 0:
            v = v + rng_below(key, slot, step, SITE_JITTER, jit)
            v = ((v + (1 << 63)) % (1 << 64)) - (1 << 63)
        return v, True


class Lifecycle:
    """lifecycle.Lifecycle for one resource kind, backed by a scratch engine."""

    def __init__(self, stages: Sequence[StageSpec], device: int = 0, capacity: int = 4096):
        self.program = KindProgram(stages)
        self.stages = [Stage(self, i) for i in range(len(self.program.stages))]
        self._device = device
        self._capacity = capacity
        self._engine: Optional[Engine] = None

    @classmethod
    def new(cls, stages: Sequence[StageSpec], **kw) -> "Lifecycle":
        """NewLifecycle (lifecycle.go:33-46): stages without a selector are dropped."""
        return cls(stages, **kw)

    def __len__(self):
        return len(self.stages)

    def list_all_possible(self, data: dict) -> List[Stage]:
        """ListAllPossible (lifecycle.go:66-122): the stage tester's deterministic view."""
        m = self.program.stage_matches(self.program.pred_of(data))
        st = [self.stages[i] for i in range(len(self.stages)) if (m >> i) & 1]
        if len(st) <= 1:
            return st
        ws = [s.weight(data) for s in st]
        nerr = sum(1 for _, ok in ws if not ok)
        total = sum(w for w, ok in ws if ok)
        if nerr == len(st):
            return st
        if total == 0:
            if nerr == 0:
                return st
            return [s for s, (w, ok) in zip(st, ws) if ok and w >= 0]
        return [s for s, (w, ok) in zip(st, ws) if ok and w > 0]

    def close(self):
        if self._engine is not None:
            self._engine.close()
            self._engine = None

    def match_batch(self, objects: Sequence[dict], now_ns: int, seed: int = 0, step: int = 0, slot_base: int = 0):
        """Match + Delay for many objects in one device step: [(Stage | None, delay_ns)].
        The i-th object takes RNG slot slot_base + i (its informer slot)."""
        n = len(objects)
        if n == 0:
            return []
        self.program.explore(objects)
        ing = Ingest(self.program)
        hot, dels, rec, cls = ing.columns(objects)
        if self._engine is None or n > self._capacity or self._engine.slot_base != slot_base:
            self.close()
            self._capacity = max(self._capacity, n)
            self._engine = Engine(self.program, capacity=self._capacity, device=self._device, slot_base=slot_base,
                                  max_records=max(1, len(ing.records)) + 1024)
        eng = self._engine
        eng.load_stages()
        eng.load(hot, dels, rec, cls, ing.record_array())
        eng.match(now_ns, seed, step)
        out_hot, _ = eng.read(0, n)
        res = []
        for i in range(n):
            st = int(out_hot["sched"][i]) & 0xFF
            s = None if st == abi.STAGE_NONE else st
            if s is None:
                res.append((None, 0))
            else:
                res.append((self.stages[s], int(out_hot["due"][i]) - now_ns))
        return res

    def match(self, data: dict, now_ns: int, seed: int = 0, step: int = 0, slot: int = 0):
        """Match (lifecycle.go:125-191) + Stage.Delay as preprocess calls them
        (pod_controller.go:222-234): (Stage | None, delay_ns)."""
        return self.match_batch([data], now_ns, seed, step, slot_base=slot)[0]
