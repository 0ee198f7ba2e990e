"""The Go host's side of one engine, restated in Python (what INTEGRATION.md's cgo wrapper does):
the informer cache of JSON objects, the patch for every fired object (playStage's render,
pod_controller.go:290-360 -> next.go:73-88), and the round trip for fires whose next state the
device could not derive.

A fired record flagged KWK_FIRED_DELTA_UNKNOWN means the engine applied the stage's finalizer
ops, delete and re-match flag but left the object's feature bits as they were: its (class,
stage) delta was not derivable at compile time (a class the stage compiler never explored, or
a patch whose effect depends on the object's state).  The reference re-matches such an object
from the apiserver's watch event (pod_controller.go:336-351, 412-478): here the host renders and
applies the patch to its cached object, re-encodes it (Ingest) and writes the row back with
kwk_replace — DIRTY iff the patch changed the object, so the next step re-matches it exactly
when the reference's Modified event would.  A class first seen here is registered and the
stage table reloaded with UNKNOWN deltas for it (every later fire of that class round-trips).
"""
from __future__ import annotations

import copy
from typing import List, Optional, Sequence

import numpy as np

from . import abi
from .compiler import KindProgram, exploration_funcs
from .engine import Engine, Ingest
from .gotpl import Renderer, rfc3339nano
from .nextstate import apply_next, prune_empty


class KindController:
    def __init__(self, program: KindProgram, engine: Engine, ingest: Ingest, objects: Sequence[dict], funcs=None):
        self.p, self.eng, self.ing = program, engine, ingest
        self.objs: List[Optional[dict]] = [prune_empty(copy.deepcopy(o)) for o in objects]
        self.funcs = funcs or exploration_funcs()
        self.n_classes = len(program.class_ids)
        self.round_trips = 0

    def step(self, now_ns: int, seed: int, step: int) -> np.ndarray:
        """kwk_step, then the fired hand-back: every fired object's patch applied to the cache,
        the DELTA_UNKNOWN ones re-encoded and written back (kwk_replace)."""
        self.eng.step(now_ns, seed, step)
        fired = self.eng.fired()
        r = Renderer(self.funcs, now_ns=now_ns)
        r.funcs["Now"] = lambda: rfc3339nano(now_ns)
        slots, rows = [], []
        for rec in fired:
            i, s, fl = int(rec["slot"]), int(rec["stage"]), int(rec["flags"])
            new, changed = apply_next(self.p.stages[s], copy.deepcopy(self.objs[i]), r)
            self.objs[i] = new
            if fl & abi.FIRED_DELTA_UNKNOWN and new is not None:
                slots.append(i)
                rows.append((self.ing.encode(new), changed))
        if slots:
            if len(self.p.class_ids) != self.n_classes:  # a class first seen now: reload the table
                self.n_classes = len(self.p.class_ids)
                self.eng.load_stages()
            n = len(slots)
            hot = np.zeros(n, dtype=abi.HOT_DTYPE)
            dels = np.zeros(n, dtype=np.int64)
            recs = np.zeros(n, dtype=np.uint32)
            cls = np.zeros(n, dtype=np.uint16)
            for j, ((pred, flags, d, rid, c), changed) in enumerate(rows):
                flags = flags & ~abi.F_DIRTY | (abi.F_DIRTY if changed else 0)
                hot[j] = (pred, flags | abi.STAGE_NONE, 0)
                dels[j], recs[j], cls[j] = d, rid, c
            if self.ing.records:  # value records interned for the new rows
                self.eng.set_records(self.ing.record_array())
            self.eng.replace(np.asarray(slots, dtype=np.uint32), hot, dels, recs, cls)
            self.round_trips += n
        return fired
