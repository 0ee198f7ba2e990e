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

``native=True`` is the Go host's path: fired objects' patches are rendered by
libkwok_patch (kwk_patch_render: the precompiled byte templates; an object or template it marks
NEEDS_RENDER / unsupported takes the text/template mirror, counted in ``host_renders``) and
re-encoded rows come from libkwok_encoder (kwk_encode), not the Python Ingest.
"""
from __future__ import annotations

import copy
import json
from typing import List, Optional, Sequence

import numpy as np

from . import abi
from .compiler import KindProgram, exploration_funcs
from .engine import Engine, Ingest
from .gotpl import Renderer, rfc3339nano
from .nextstate import apply_next, prune_empty


class KindController:
    def __init__(self, program: KindProgram, engine: Engine, ingest: Ingest, objects: Sequence[dict], funcs=None,
                 native: bool = False, n_threads: int = 1):
        self.p, self.eng, self.ing = program, engine, ingest
        self.objs: List[Optional[dict]] = [prune_empty(copy.deepcopy(o)) for o in objects]
        self.funcs = funcs or exploration_funcs()
        self.n_classes = len(program.class_ids)
        self.round_trips = 0
        self.native = native
        self.native_renders = 0   # patches rendered by kwk_patch_render
        self.host_renders = 0     # patches the native renderer handed back (NEEDS_RENDER / unsupported)
        self.last_rows = {}       # slot -> kwk_encode row of every object the last step fired (native)
        self.last_patches = {}    # (slot, patch index) -> the patch bytes the last step applied (native)
        if native:
            from .encoder import NativeIngest
            from .patchtpl import PatchProgram
            self.nenc = NativeIngest(program, n_threads=n_threads)
            native_prog = program if hasattr(program, "patch_spec") else None  # libkwok_compiler's spec
            self.patcher = PatchProgram(program.stages, self.funcs, n_threads=n_threads, program=native_prog)

    def close(self):
        if self.native:
            self.nenc.close()
            self.patcher.close()

    def _apply_native(self, fired, now_ns: int):
        """playStage's effect for every fired object with the native libraries: finalizer ops and
        delete from the stage (next.go:43-70), the merge patches rendered in one kwk_patch_render
        call against the objects after their finalizer ops (next.go:73-88 renders every patch of a
        stage against the same object), applied in order; -> [(slot, new object | None, changed)]."""
        from .gotpl import Renderer, rfc3339nano
        from .nextstate import finalizers_modify, json_patch, merge_patch
        from .patchtpl import render_patch_bytes
        items, jobs = [], []  # jobs: (item index, patch index, template id | None)
        for rec in fired:
            i, s = int(rec["slot"]), int(rec["stage"])
            st = self.p.stages[s]
            obj = copy.deepcopy(self.objs[i])
            changed = False
            if st.next.finalizers is not None:
                ops = finalizers_modify((obj.get("metadata") or {}).get("finalizers"), st.next.finalizers)
                if ops:
                    new = prune_empty(json_patch(obj, ops))
                    changed = json.dumps(new, sort_keys=True) != json.dumps(obj, sort_keys=True)
                    obj = new
            items.append([i, s, obj, changed])
            if st.next.delete:
                continue
            for pi, pt in enumerate(st.next.patches):
                jobs.append((len(items) - 1, pi, self.patcher.template_of.get((s, pi))))
        nat = [j for j in jobs if j[2] is not None]
        rendered = self.patcher.render([t for _, _, t in nat], [items[k][2] for k, _, _ in nat], now_ns) if nat else []
        out_bytes = {}
        for (k, pi, _), b in zip(nat, rendered):
            out_bytes[(k, pi)] = b
        r = None
        for k, pi, _ in jobs:
            if out_bytes.get((k, pi)) is None:  # NEEDS_RENDER / unsupported template: the host mirror
                if r is None:
                    r = Renderer(self.funcs, now_ns=now_ns)
                    r.funcs["Now"] = lambda: rfc3339nano(now_ns)
                pt = self.p.stages[items[k][1]].next.patches[pi]
                out_bytes[(k, pi)] = render_patch_bytes(pt.template, pt.root, items[k][2], r)
                self.host_renders += 1
            else:
                self.native_renders += 1
        self.last_patches = {(items[k][0], pi): b for (k, pi), b in out_bytes.items()}
        result = []
        for k, (i, s, obj, changed) in enumerate(items):
            st = self.p.stages[s]
            if st.next.delete:
                result.append((i, None, True))
                continue
            for pi, pt in enumerate(st.next.patches):
                data = json.loads(out_bytes[(k, pi)])
                new = prune_empty(json_patch(obj, data) if pt.type == "json" else merge_patch(obj, data))
                if json.dumps(new, sort_keys=True) != json.dumps(obj, sort_keys=True):
                    changed = True
                    obj = new
            result.append((i, obj, changed))
        return result

    def step(self, now_ns: int, seed: int, step: int) -> np.ndarray:
        """kwk_step, then the fired hand-back: every fired object's patch applied to the cache,
        the DELTA_UNKNOWN ones re-encoded and written back (kwk_replace)."""
        self.eng.step(now_ns, seed, step)
        fired = self.eng.fired()
        self.handle(fired, now_ns)
        return fired

    def handle(self, fired, now_ns: int):
        """The hand-back of one step's fired list (kwk_fired records): patches applied to the
        cache, the DELTA_UNKNOWN rows written back."""
        slots, rows = [], []
        if self.native:
            applied = self._apply_native(fired, now_ns)
            for i, new, _ in applied:
                self.objs[i] = new
            # every fired object's new state re-encoded by libkwok_encoder (the informer event's row)
            live = [(i, new, ch) for i, new, ch in applied if new is not None]
            # a class first seen now is registered with the compiler and the row re-encoded
            # natively, so its record id points into the native encoder's record table
            enc = self.nenc.columns([new for _, new, _ in live], register=True) if live else None
            self.last_rows = {}
            unknown = {int(rec["slot"]) for rec in fired if int(rec["flags"]) & abi.FIRED_DELTA_UNKNOWN}
            for j, (i, new, changed) in enumerate(live):
                h, d, rc, c = enc[0][j], enc[1][j], enc[2][j], enc[3][j]
                row = (int(h["pred"]), int(h["sched"]) & ~abi.STAGE_NONE, int(d), int(rc), int(c))
                self.last_rows[i] = row
                if i in unknown:
                    slots.append(i)
                    rows.append((row, changed))
        else:
            r = Renderer(self.funcs, now_ns=now_ns)
            r.funcs["Now"] = lambda: rfc3339nano(now_ns)
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
            if self.native:
                recs_native = self.nenc.record_array()
                if len(self.nenc.p.slots):
                    self.eng.set_records(recs_native)
            elif self.ing.records:  # value records interned for the new rows
                self.eng.set_records(self.ing.record_array())
            self.eng.replace(np.asarray(slots, dtype=np.uint32), hot, dels, recs, cls)
            self.round_trips += n
