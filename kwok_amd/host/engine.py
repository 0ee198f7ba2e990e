"""Host driver for one engine (one resource kind on one GPU).

``Ingest`` turns objects into the device's SoA columns (the Go host's informer-side
encoder); ``Engine`` owns the C-ABI handle.  Objects are interned
by *variant*: objects that differ only in identity (name, uid, node) share one feature /
record / class computation, which is what makes 10^8-object clusters ingestible.
"""
from __future__ import annotations

import copy
import ctypes as C
import json
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import abi
from .compiler import KindProgram, path_prefix
from .nextstate import prune_empty


def _variant_key(obj: dict) -> str:
    o = copy.deepcopy(obj)
    md = o.get("metadata") or {}
    for k in ("name", "generateName", "uid", "resourceVersion", "creationTimestamp", "selfLink", "managedFields"):
        md.pop(k, None)
    if isinstance(o.get("spec"), dict):
        o["spec"].pop("nodeName", None)
    for r in md.get("ownerReferences") or []:
        r.pop("uid", None)
        r.pop("name", None)
    return json.dumps(o, sort_keys=True, separators=(",", ":"))


class Ingest:
    """Objects -> (hot, deletion_s, rec_idx, cls, records) for one KindProgram."""

    def __init__(self, program: KindProgram):
        self.p = program
        # variant memoisation is valid only if no query reads an identity field
        self.memo_ok = not any(path_prefix(f.src)[:2] in (["metadata", "name"], ["metadata", "uid"], ["spec", "nodeName"])
                               for f in program.features.values())
        self._memo: Dict[str, tuple] = {}
        self.records: List[List[tuple]] = []
        self._rec_ids: Dict[str, int] = {}

    def encode(self, obj: dict, register_class: bool = True):
        """-> (pred, sched_flags, del_s, rec_idx, cls) for one object (sched without stage)."""
        key = _variant_key(obj) if self.memo_ok else None
        hit = self._memo.get(key) if key is not None else None
        if hit is None:
            obj = prune_empty(copy.deepcopy(obj))
            pred = self.p.pred_of(obj)
            rec = self.p.record_of(obj)
            rid = 0
            flags = abi.F_ALIVE | abi.F_MANAGED | abi.F_DIRTY
            if rec is not None:
                rk = json.dumps(rec)
                rid = self._rec_ids.get(rk)
                if rid is None:
                    rid = self._rec_ids[rk] = len(self.records)
                    self.records.append(rec)
                flags |= abi.F_HASREC
            cls = self.p.class_of(obj, register=register_class)
            dels = self.p.deletion_s(obj)
            hit = (pred, flags, dels, rid, cls)
            if key is not None:
                self._memo[key] = hit
        return hit

    def columns(self, objs: Sequence[dict]):
        n = len(objs)
        hot = np.zeros(n, dtype=abi.HOT_DTYPE)
        dels = np.zeros(n, dtype=np.int64)
        rec = np.zeros(n, dtype=np.uint32)
        cls = np.zeros(n, dtype=np.uint16)
        for i, o in enumerate(objs):
            pred, flags, d, rid, c = self.encode(o)
            hot[i] = (pred, flags | abi.STAGE_NONE, 0)
            dels[i], rec[i], cls[i] = d, rid, c
        return hot, dels, rec, cls

    def variant_columns(self, variants: Sequence[dict], index: np.ndarray):
        """Columns for objects given as variant ids (index[i] -> variants[index[i]])."""
        enc = [self.encode(v) for v in variants]
        pred = np.array([e[0] for e in enc], dtype=np.uint32)
        flags = np.array([e[1] for e in enc], dtype=np.uint32)
        dls = np.array([e[2] for e in enc], dtype=np.int64)
        rid = np.array([e[3] for e in enc], dtype=np.uint32)
        cl = np.array([e[4] for e in enc], dtype=np.uint16)
        hot = np.empty(len(index), dtype=abi.HOT_DTYPE)
        hot["pred"] = pred[index]
        hot["sched"] = flags[index] | abi.STAGE_NONE
        hot["due"] = 0
        return hot, dls[index], rid[index], cl[index]

    def record_array(self) -> np.ndarray:
        ns = max(1, len(self.p.slots))
        a = np.zeros((max(1, len(self.records)), ns), dtype=abi.VALUE_DTYPE)
        for r, rec in enumerate(self.records):
            for s, (kind, value, nsec) in enumerate(rec):
                a[r, s] = (value, nsec, kind)
        return a


class PinnedBuffer:
    """kwk_alloc_host / kwk_free_host: a page-locked host buffer reused across steps."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        self.p = C.c_void_p()
        abi.check(abi.lib().kwk_alloc_host(self.nbytes, C.byref(self.p)), "kwk_alloc_host")

    def array(self, dtype, n: int) -> np.ndarray:
        dtype = np.dtype(dtype)
        if n * dtype.itemsize > self.nbytes:
            raise abi.EngineError(f"pinned buffer of {self.nbytes} bytes too small for {n} x {dtype}")
        if n == 0:
            return np.zeros(0, dtype=dtype)
        buf = (C.c_char * (n * dtype.itemsize)).from_address(self.p.value)
        return np.frombuffer(buf, dtype=dtype, count=n)

    def close(self):
        if self.p:
            abi.lib().kwk_free_host(self.p)
            self.p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _compact_code(compact) -> int:
    if compact == "packed16":
        return abi.COMPACT_PACKED16
    if compact == "bits":
        return abi.COMPACT_BITS
    if compact == "packed":
        return abi.COMPACT_PACKED
    return 1 if compact else 0


class Engine:
    """One kwk_engine (C ABI) for one KindProgram."""

    def __init__(self, program: KindProgram, capacity: int, device: int = 0, slot_base: int = 0, kind_salt: int = 0,
                 max_records: int = 1 << 16, wide_state: bool = False, state: str = "auto"):
        """state: "auto" (the narrowest format: 1-byte dictionary ids for table-only programs
        whose words close within 255 ids, else the packed 2 bytes the stage table fits, else the
        8-byte record of a packed word fused with its relative due time when the word fits 28
        bits, else 4-byte words, else 8), "u16" (never the 1-byte ids), "dw" (never fewer than 4
        bytes: the fused record when it fits), "u32" (4-byte packed words and the separate due
        column) or "wide" (always 8 bytes; = wide_state)."""
        self.p = program
        L = abi.lib()
        if wide_state:
            state = "wide"
        flags = {"auto": 0, "u16": abi.ENGINE_STATE16, "dw": abi.ENGINE_STATE32,
                 "u32": abi.ENGINE_STATE32 | abi.ENGINE_SPLIT_DUE, "wide": abi.ENGINE_WIDE_STATE}[state]
        d = abi.EngineDesc(device=device, capacity=capacity, value_slots=max(1, len(program.slots)),
                           max_records=max_records, slot_base=slot_base, kind_salt=kind_salt, flags=flags)
        h = C.c_void_p()
        abi.check(L.kwk_engine_create(C.byref(d), C.byref(h)), "kwk_engine_create")  # thread slot
        self.h = h
        self.capacity = capacity
        self.n = 0
        self.kind_salt = kind_salt
        self.slot_base = slot_base

    def _check(self, status: int, what: str):
        abi.check(status, what, self.h)

    def close(self):
        if getattr(self, "h", None):
            abi.lib().kwk_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_stages(self, version: int = 1):
        t = self.p.table(version)
        deltas = np.ascontiguousarray(self.p.delta_array())
        self._check(abi.lib().kwk_load_stages(self.h, C.byref(t), abi.ptr(deltas)), "kwk_load_stages")
        h = self.p.harness_struct()
        self._check(abi.lib().kwk_set_harness(self.h, C.byref(h)), "kwk_set_harness")

    def set_harness(self, enable: bool):
        h = self.p.harness_struct()
        h.enable = 1 if (enable and self.p.harness is not None) else 0
        self._check(abi.lib().kwk_set_harness(self.h, C.byref(h)), "kwk_set_harness")

    def load(self, hot, dels, rec, cls, records: Optional[np.ndarray] = None):
        hot = np.ascontiguousarray(hot)
        dels = np.ascontiguousarray(dels, dtype=np.int64)
        rec = np.ascontiguousarray(rec, dtype=np.uint32)
        cls = np.ascontiguousarray(cls, dtype=np.uint16)
        n_rec = 0 if records is None else records.shape[0]
        recs = None if records is None else np.ascontiguousarray(records)
        self._check(abi.lib().kwk_load(self.h, len(hot), abi.ptr(hot), abi.ptr(dels), abi.ptr(rec), abi.ptr(cls), n_rec,
                                     abi.ptr(recs)), "kwk_load")
        self.n = len(hot)

    def upsert(self, slots, hot, dels, rec, cls):
        slots = np.ascontiguousarray(slots, dtype=np.uint32)
        hot = np.ascontiguousarray(hot)
        self._check(abi.lib().kwk_upsert(self.h, len(slots), abi.ptr(slots), abi.ptr(hot),
                                       abi.ptr(np.ascontiguousarray(dels, dtype=np.int64)),
                                       abi.ptr(np.ascontiguousarray(rec, dtype=np.uint32)),
                                       abi.ptr(np.ascontiguousarray(cls, dtype=np.uint16))), "kwk_upsert")
        self.n = max(self.n, int(slots.max()) + 1)

    def replace(self, slots, hot, dels, rec, cls):
        """kwk_replace: rows written as given (no implicit DIRTY)."""
        slots = np.ascontiguousarray(slots, dtype=np.uint32)
        hot = np.ascontiguousarray(hot)
        self._check(abi.lib().kwk_replace(self.h, len(slots), abi.ptr(slots), abi.ptr(hot),
                                        abi.ptr(np.ascontiguousarray(dels, dtype=np.int64)),
                                        abi.ptr(np.ascontiguousarray(rec, dtype=np.uint32)),
                                        abi.ptr(np.ascontiguousarray(cls, dtype=np.uint16))), "kwk_replace")

    def set_records(self, records: np.ndarray, first: int = 0):
        recs = np.ascontiguousarray(records)
        self._check(abi.lib().kwk_set_records(self.h, first, recs.shape[0], abi.ptr(recs)), "kwk_set_records")

    def delete(self, slots):
        slots = np.ascontiguousarray(slots, dtype=np.uint32)
        self._check(abi.lib().kwk_delete(self.h, len(slots), abi.ptr(slots)), "kwk_delete")

    def retry(self, now_ns: int, seed: int, step: int, slots, hot, cls, stages, retry_count, backoff=None):
        """kwk_retry: re-queue failed playStage jobs (pod_controller.go:273-284) with the
        host's unchanged rows (`hot` / `cls` as Ingest.columns gives them)."""
        slots = np.ascontiguousarray(slots, dtype=np.uint32)
        hot = np.ascontiguousarray(hot, dtype=abi.HOT_DTYPE)
        cls = np.ascontiguousarray(cls, dtype=np.uint16)
        stages = np.ascontiguousarray(stages, dtype=np.uint16)
        rc = np.ascontiguousarray(retry_count, dtype=np.uint32)
        b = abi.Backoff(**(backoff or abi.DEFAULT_BACKOFF))
        self._check(abi.lib().kwk_retry(self.h, now_ns, seed, step, len(slots), abi.ptr(slots), abi.ptr(hot), abi.ptr(cls),
                                      abi.ptr(stages), abi.ptr(rc), C.byref(b)), "kwk_retry")

    def step(self, now_ns: int, seed: int, step: int):
        self._check(abi.lib().kwk_step(self.h, now_ns, seed, step), "kwk_step")

    def step_n(self, n: int, now0_ns: int, dt_ns: int, seed: int, step0: int, compact=True, ev_every: int = 0,
               ev_j0: int = 0):
        """kwk_step_n: n steps (+ device compaction after each) enqueued by one call; compact =
        True (kwk_fired_rec), "packed" (4-byte records), "packed16" (2-byte records where the sweep
        has them, else 4-byte) or False."""
        c = _compact_code(compact)
        self._check(abi.lib().kwk_step_n(self.h, n, now0_ns, dt_ns, seed, step0, c, ev_every, ev_j0), "kwk_step_n")

    def step_n_pair(self, other: "Engine", n: int, now0_ns: int, dt_ns: int, seed: int, step0: int, compact=True,
                    ev_every: int = 0, ev_j0: int = 0):
        """kwk_step_n_pair: this engine's and `other`'s steps enqueued in turn, step by step."""
        c = _compact_code(compact)
        self._check(abi.lib().kwk_step_n_pair(self.h, other.h, n, now0_ns, dt_ns, seed, step0, c, ev_every, ev_j0),
                    "kwk_step_n_pair")

    def fired_compact(self, packed=False):
        """kwk_fired_compact (/ _packed, packed = True; / _packed16, packed = "16"): the last step's fired
        list compacted on the device (enqueue only)."""
        if packed == "16":
            self._check(abi.lib().kwk_fired_compact_packed16(self.h), "kwk_fired_compact_packed16")
        elif packed == "bits":
            self._check(abi.lib().kwk_fired_compact_bits(self.h), "kwk_fired_compact_bits")
        elif packed:
            self._check(abi.lib().kwk_fired_compact_packed(self.h), "kwk_fired_compact_packed")
        else:
            self._check(abi.lib().kwk_fired_compact(self.h), "kwk_fired_compact")

    def fired_packed(self, pinned: Optional["PinnedBuffer"] = None) -> np.ndarray:
        """The last step's fired list as packed u32 records (kwk_fired_packed): stage = r >> 27,
        slot = r & (2**27 - 1)."""
        n = C.c_uint32()
        L = abi.lib()
        self._check(L.kwk_fired_packed(self.h, None, 0, C.byref(n)), "kwk_fired_packed")
        out = pinned.array(np.uint32, n.value) if pinned is not None else np.zeros(n.value, dtype=np.uint32)
        if n.value:
            self._check(L.kwk_fired_packed(self.h, abi.ptr(out), n.value, C.byref(n)), "kwk_fired_packed")
        return out

    def fetch_async(self, out: "PinnedBuffer", counts: Optional["PinnedBuffer"] = None) -> dict:
        """kwk_fired_fetch_async: the last step's compacted list (and, for 2-byte records, the records per
        segment) copied into `out` / `counts` on the engine's copy stream; returns the list's shape
        at once ({n_records, record_bytes, n_segs, region_slots}).  The buffers hold the copy after
        fetch_wait() (or the next fetch)."""
        info = abi.FetchInfo()
        self._check(abi.lib().kwk_fired_fetch_async(self.h, out.p, out.nbytes, counts.p if counts is not None else None,
                                                   counts.nbytes // 4 if counts is not None else 0, C.byref(info)),
                    "kwk_fired_fetch_async")
        return {k: getattr(info, k) for k, _ in abi.FetchInfo._fields_}

    def fetch_wait(self):
        """kwk_fired_fetch_wait: the last fetch's copies are in the host buffers."""
        self._check(abi.lib().kwk_fired_fetch_wait(self.h), "kwk_fired_fetch_wait")

    def fired_keep(self, depth: int):
        """kwk_fired_keep: keep the lists of the last `depth` compactions readable by step
        (fetch_step), each compaction signalling its own completion."""
        self._check(abi.lib().kwk_fired_keep(self.h, depth), "kwk_fired_keep")

    def fetch_step(self, step: int, out: "PinnedBuffer", counts: Optional["PinnedBuffer"] = None) -> dict:
        """kwk_fired_fetch_step: step `step`'s list (any step of a kwk_step_n call still in the ring)
        copied into `out` / `counts` on the copy stream, as fetch_async; the buffers hold it after
        fetch_wait()."""
        info = abi.FetchInfo()
        self._check(abi.lib().kwk_fired_fetch_step(self.h, step, out.p, out.nbytes,
                                                  counts.p if counts is not None else None,
                                                  counts.nbytes // 4 if counts is not None else 0, C.byref(info)),
                    "kwk_fired_fetch_step")
        return {k: getattr(info, k) for k, _ in abi.FetchInfo._fields_}

    def fired_bits(self):
        """The last step's list as per-segment fired maps + 2-bit stage codes (kwk_fired_bits) ->
        (words u32, transitions, segments, region_slots); abi.bits_decode gives (slot, stage)."""
        nw, nr, ns, rs = C.c_uint64(), C.c_uint32(), C.c_uint32(), C.c_uint32()
        L = abi.lib()
        self._check(L.kwk_fired_bits(self.h, None, 0, C.byref(nw), C.byref(nr), C.byref(ns), C.byref(rs)), "kwk_fired_bits")
        out = np.zeros(nw.value, dtype=np.uint32)
        if nw.value:
            self._check(L.kwk_fired_bits(self.h, abi.ptr(out), nw.value, C.byref(nw), C.byref(nr), C.byref(ns), C.byref(rs)),
                        "kwk_fired_bits")
        return out, nr.value, ns.value, rs.value

    def fired_packed16(self, pinned=None):
        """The last step's list as 2-byte records (kwk_fired_packed16) -> (records u16, records per
        segment u32, region_slots); abi.EngineError (KWK_ESTATE) when the sweep has no 2-byte records.
        pinned: (PinnedBuffer for the records, PinnedBuffer for the counts)."""
        n, ns, rs = C.c_uint32(), C.c_uint32(), C.c_uint32()
        L = abi.lib()
        self._check(L.kwk_fired_packed16(self.h, None, 0, C.byref(n), None, 0, C.byref(ns), C.byref(rs)),
                    "kwk_fired_packed16")
        if pinned is not None:
            out, cnt = pinned[0].array(np.uint16, n.value), pinned[1].array(np.uint32, ns.value)
        else:
            out, cnt = np.zeros(n.value, dtype=np.uint16), np.zeros(ns.value, dtype=np.uint32)
        self._check(L.kwk_fired_packed16(self.h, abi.ptr(out) if n.value else None, n.value, C.byref(n),
                                         abi.ptr(cnt) if ns.value else None, ns.value, C.byref(ns), C.byref(rs)),
                    "kwk_fired_packed16")
        return out, cnt, int(rs.value)

    def set_tuning(self, key: int, value: int):
        """kwk_set_tuning: an explicit kernel choice (abi.TUNE_*)."""
        self._check(abi.lib().kwk_set_tuning(self.h, key, value), "kwk_set_tuning")

    def match(self, now_ns: int, seed: int, step: int):
        """kwk_match: pick + delay for dirty objects, nothing fires."""
        self._check(abi.lib().kwk_match(self.h, now_ns, seed, step), "kwk_match")

    def last_sweep(self) -> dict:
        """kwk_last_sweep: the kernel shape the last kwk_step / kwk_match launched."""
        i = abi.SweepInfo()
        self._check(abi.lib().kwk_last_sweep(self.h, C.byref(i)), "kwk_last_sweep")
        return {k: getattr(i, k) for k, _ in abi.SweepInfo._fields_}

    def sync(self):
        self._check(abi.lib().kwk_sync(self.h), "kwk_sync")

    def fired(self, pinned: Optional["PinnedBuffer"] = None) -> np.ndarray:
        """The last step's fired records (kwk_fired).  With `pinned` (a PinnedBuffer) the copy
        lands in page-locked memory and the returned array is a view of it."""
        n = C.c_uint32()
        L = abi.lib()
        self._check(L.kwk_fired(self.h, None, 0, C.byref(n)), "kwk_fired")
        if pinned is not None:
            out = pinned.array(abi.FIRED_DTYPE, n.value)
        else:
            out = np.zeros(n.value, dtype=abi.FIRED_DTYPE)
        if n.value:
            self._check(L.kwk_fired(self.h, abi.ptr(out), n.value, C.byref(n)), "kwk_fired")
        return out

    def stats(self) -> dict:
        s = abi.StepStats()
        self._check(abi.lib().kwk_stats(self.h, C.byref(s)), "kwk_stats")
        return {"steps": s.steps, "matched": s.matched, "fired": s.fired, "bytes": s.bytes,
                "state_bytes": s.state_bytes, "line_bytes": s.line_bytes,
                "fired_per_stage": {self.p.names[i]: s.fired_per_stage[i] for i in range(len(self.p.names))}}

    def read(self, first: int = 0, n: Optional[int] = None):
        n = self.n - first if n is None else n
        hot = np.zeros(n, dtype=abi.HOT_DTYPE)
        dels = np.zeros(n, dtype=np.int64)
        self._check(abi.lib().kwk_read(self.h, first, n, abi.ptr(hot), abi.ptr(dels)), "kwk_read")
        return hot, dels

    def count(self, masks) -> np.ndarray:
        """kwk_count: alive objects with (pred & mask) != 0 per mask (0 = all alive)."""
        m = np.ascontiguousarray(masks, dtype=np.uint32)
        out = np.zeros(len(m), dtype=np.uint64)
        self._check(abi.lib().kwk_count(self.h, len(m), abi.ptr(m), abi.ptr(out)), "kwk_count")
        return out

    def aggregate(self, masks, now_ns: int = 0, usage: bool = False, out_ptr: Optional[int] = None) -> int:
        """kwk_aggregate: per-stage transitions, kwk_count of `masks` and (usage) the cluster usage
        at now_ns, written as float64 on the device — into `out_ptr` (device memory, e.g. an RCCL
        buffer) or the engine's own buffer (aggregate_read).  Enqueue only; returns the count."""
        m = np.ascontiguousarray(masks, dtype=np.uint32)
        self._agg_masks = m  # kept alive until the stream has copied it
        n = C.c_uint32()
        self._check(abi.lib().kwk_aggregate(self.h, len(m), abi.ptr(m) if len(m) else None, now_ns,
                                          abi.AGG_USAGE if usage else 0, out_ptr, C.byref(n)), "kwk_aggregate")
        return n.value

    def aggregate_read(self, n: int) -> np.ndarray:
        """The engine-owned aggregate buffer (synchronises)."""
        out = np.zeros(n, dtype=np.float64)
        self._check(abi.lib().kwk_aggregate_read(self.h, abi.ptr(out), n), "kwk_aggregate_read")
        return out

    # usage
    def usage_config(self, node_ptr, usage_key, cpu_values, mem_values, mixed=None, ckeys=None):
        """kwk_usage_config (+ kwk_usage_mixed when some pod's containers differ): the columns
        usage.usage_columns computes."""
        self._uargs = [np.ascontiguousarray(node_ptr, dtype=np.uint32), np.ascontiguousarray(usage_key, dtype=np.uint32),
                       np.ascontiguousarray(cpu_values, dtype=np.float64),
                       np.ascontiguousarray(mem_values, dtype=np.float64)]
        np_, uk, cv, mv = self._uargs
        self.n_nodes = len(np_) - 1
        self._check(abi.lib().kwk_usage_config(self.h, self.n_nodes, abi.ptr(np_), abi.ptr(uk), len(cv), abi.ptr(cv),
                                             len(mv), abi.ptr(mv)), "kwk_usage_config")
        mixed = np.zeros(0, dtype=np.uint32) if mixed is None else np.ascontiguousarray(mixed, dtype=np.uint32)
        ckeys = np.zeros(0, dtype=np.uint32) if ckeys is None else np.ascontiguousarray(ckeys, dtype=np.uint32)
        if len(mixed) or np.any((uk >> 28) == 0):
            self._check(abi.lib().kwk_usage_mixed(self.h, len(mixed) // 2, abi.ptr(mixed), len(ckeys), abi.ptr(ckeys)),
                      "kwk_usage_mixed")
        # containers per pod (series of a container metric)
        nc = (uk >> 28).astype(np.int64)
        mx = nc == 0
        if np.any(mx):
            nc[mx] = mixed[1::2].astype(np.int64)[(uk[mx] & 0x0FFFFFFF).astype(np.int64)]
        self.usage_containers = nc

    def usage_read_containers(self, first: int = 0, n: Optional[int] = None) -> np.ndarray:
        """containers x {cpu, mem, cpu_cumulative, mem_cumulative} of pods [first, first+n)."""
        n = self.n - first if n is None else n
        cnt = C.c_uint32()
        L = abi.lib()
        self._check(L.kwk_usage_read_containers(self.h, first, n, None, 0, C.byref(cnt)), "kwk_usage_read_containers")
        out = np.zeros((cnt.value, 4), dtype=np.float64)
        if cnt.value:
            self._check(L.kwk_usage_read_containers(self.h, first, n, abi.ptr(out), cnt.value, C.byref(cnt)),
                      "kwk_usage_read_containers")
        return out

    # Metric CRD values (kwok_amd/host/metrics.py)
    def metrics_load(self, programs):
        """programs: [(dimension name, [(op, arg), ...])] from cel.lower()."""
        n, descs, n_ops, ops = pack_metric_programs(programs)
        self.metrics_load_arrays(n, descs, n_ops, ops)

    def metrics_load_arrays(self, n, descs, n_ops, ops):
        """kwk_metrics_load over packed kwk_metric_desc / kwk_metric_op arrays (pointers or ctypes
        arrays: pack_metric_programs, or the native compiler's kwk_metric_set_programs)."""
        self._check(abi.lib().kwk_metrics_load(self.h, n, descs, n_ops, ops), "kwk_metrics_load")

    def histograms_load(self, histograms):
        """histograms: [(dimension name, [(le, hidden, [(op, arg), ...]), ...])] (cel.lower per bucket)."""
        self.histograms_load_arrays(*pack_histogram_programs(histograms))

    def histograms_load_arrays(self, n, descs, n_buckets, buckets, n_ops, ops):
        self._check(abi.lib().kwk_histograms_load(self.h, n, descs, n_buckets, buckets, n_ops, ops),
                    "kwk_histograms_load")

    def histograms_eval(self, now_ns: int, node_first: int, n_nodes: int) -> np.ndarray:
        """Every histogram's series records (uint64 words, see kwk_histograms_eval)."""
        cnt = C.c_uint64()
        L = abi.lib()
        self._check(L.kwk_histograms_eval(self.h, now_ns, node_first, n_nodes, None, 0, C.byref(cnt)),
                    "kwk_histograms_eval")
        out = np.zeros(cnt.value, dtype=np.uint64)
        if cnt.value:
            self._check(L.kwk_histograms_eval(self.h, now_ns, node_first, n_nodes, abi.ptr(out), cnt.value,
                                              C.byref(cnt)), "kwk_histograms_eval")
        return out

    def metrics_inputs(self, pod_created_ns, node_created_ns, node_started, zero_time_unix_s: float):
        self._minputs = [np.ascontiguousarray(pod_created_ns, dtype=np.int64),
                         np.ascontiguousarray(node_created_ns, dtype=np.int64),
                         np.ascontiguousarray(node_started, dtype=np.float64)]
        a, b, c = self._minputs
        self._check(abi.lib().kwk_metrics_inputs(self.h, abi.ptr(a), abi.ptr(b), abi.ptr(c), zero_time_unix_s),
                  "kwk_metrics_inputs")

    def metrics_eval(self, now_ns: int, node_first: int, n_nodes: int) -> np.ndarray:
        cnt = C.c_uint64()
        L = abi.lib()
        self._check(L.kwk_metrics_eval(self.h, now_ns, node_first, n_nodes, None, 0, C.byref(cnt)), "kwk_metrics_eval")
        out = np.zeros(cnt.value, dtype=np.float64)
        if cnt.value:
            self._check(L.kwk_metrics_eval(self.h, now_ns, node_first, n_nodes, abi.ptr(out), cnt.value, C.byref(cnt)),
                      "kwk_metrics_eval")
        return out

    def metrics_eval_device(self, now_ns: int, node_first: int, n_nodes: int) -> int:
        """kwk_metrics_eval_device: the scrape's values left on the device (enqueue only) -> their count."""
        p, cnt = C.c_void_p(), C.c_uint64()
        self._check(abi.lib().kwk_metrics_eval_device(self.h, now_ns, node_first, n_nodes, C.byref(p), C.byref(cnt)),
                    "kwk_metrics_eval_device")
        return int(cnt.value)

    def histograms_eval_device(self, now_ns: int, node_first: int, n_nodes: int) -> int:
        p, cnt = C.c_void_p(), C.c_uint64()
        self._check(abi.lib().kwk_histograms_eval_device(self.h, now_ns, node_first, n_nodes, C.byref(p),
                                                          C.byref(cnt)), "kwk_histograms_eval_device")
        return int(cnt.value)

    def usage(self, now_ns: int):
        self._check(abi.lib().kwk_usage(self.h, now_ns), "kwk_usage")

    def usage_pods(self, enable: bool = True):
        self._check(abi.lib().kwk_usage_pods(self.h, 1 if enable else 0), "kwk_usage_pods")

    def usage_read_pods(self, first: int = 0, n: Optional[int] = None) -> np.ndarray:
        """n x {cpu, mem, cpu_cumulative, mem_cumulative} per pod slot."""
        n = self.n - first if n is None else n
        out = np.zeros((n, 4), dtype=np.float64)
        self._check(abi.lib().kwk_usage_read_pods(self.h, first, n, abi.ptr(out)), "kwk_usage_read_pods")
        return out

    def usage_read(self, node_out: bool = True):
        """(per-node {cpu, mem, cpu_cumulative, mem_cumulative} or None, cluster {cpu, mem})."""
        node = np.zeros((self.n_nodes, 4), dtype=np.float64) if node_out else None
        cl = np.zeros(2, dtype=np.float64)
        self._check(abi.lib().kwk_usage_read(self.h, abi.ptr(node), abi.ptr(cl)), "kwk_usage_read")
        return node, cl

    # node leases (NodeLeaseController, node_lease_controller.go)
    def lease_config(self, holder_id: int, lease_duration_s: int, renew_interval_ns: int = None,
                     renew_jitter: float = 0.04, manage_nodes: bool = True):
        """renew interval defaults to leaseDuration / 4 and jitter to 0.04 (controller.go:245-249)."""
        if renew_interval_ns is None:
            renew_interval_ns = lease_duration_s * 10**9 // 4
        p = abi.LeaseParams(holder_id=holder_id, lease_duration_s=lease_duration_s,
                            renew_interval_ns=renew_interval_ns, renew_jitter=renew_jitter,
                            manage_nodes=1 if manage_nodes else 0)
        self._check(abi.lib().kwk_lease_config(self.h, C.byref(p)), "kwk_lease_config")

    def lease_set(self, leases: np.ndarray, first: int = 0):
        a = np.ascontiguousarray(leases, dtype=abi.LEASE_DTYPE)
        self._check(abi.lib().kwk_lease_set(self.h, first, len(a), abi.ptr(a)), "kwk_lease_set")

    def lease_step(self, now_ns: int, seed: int, step: int):
        self._check(abi.lib().kwk_lease_step(self.h, now_ns, seed, step), "kwk_lease_step")

    def lease_ops(self) -> np.ndarray:
        n = C.c_uint32()
        L = abi.lib()
        self._check(L.kwk_lease_ops(self.h, None, 0, C.byref(n)), "kwk_lease_ops")
        out = np.zeros(n.value, dtype=abi.FIRED_DTYPE)
        if n.value:
            self._check(L.kwk_lease_ops(self.h, abi.ptr(out), n.value, C.byref(n)), "kwk_lease_ops")
        return out

    def lease_read(self, first: int = 0, n: Optional[int] = None) -> np.ndarray:
        n = self.n - first if n is None else n
        out = np.zeros(n, dtype=abi.LEASE_DTYPE)
        self._check(abi.lib().kwk_lease_read(self.h, first, n, abi.ptr(out)), "kwk_lease_read")
        return out

    def lease_fail(self, now_ns: int, seed: int, step: int, slots, old: np.ndarray):
        """kwk_lease_fail: the apiserver rejected these nodes' lease writes of the last lease
        step; `old` = the leases the informer still holds."""
        slots = np.ascontiguousarray(slots, dtype=np.uint32)
        old = np.ascontiguousarray(old, dtype=abi.LEASE_DTYPE)
        self._check(abi.lib().kwk_lease_fail(self.h, now_ns, seed, step, len(slots), abi.ptr(slots), abi.ptr(old)),
                  "kwk_lease_fail")

    def lease_stats(self) -> dict:
        c = abi.LeaseCounters()
        self._check(abi.lib().kwk_lease_stats(self.h, C.byref(c)), "kwk_lease_stats")
        return {k: getattr(c, k) for k, _ in abi.LeaseCounters._fields_}

    def lease_sync_pods(self, pods: "Engine", node_ptr):
        """Pods on the nodes synced by this engine's last lease step (podsOnNodeSyncWorker)."""
        ptr = np.ascontiguousarray(node_ptr, dtype=np.uint32)
        self._check(abi.lib().kwk_lease_sync_pods(pods.h, self.h, len(ptr) - 1, abi.ptr(ptr)), "kwk_lease_sync_pods")

    # the fused reconciliation tick (this engine = the node engine)
    def tick_bind(self, nodes: "Engine", node_ptr):
        """kwk_tick_bind on this POD engine: the node engine and node_ptr its fused ticks use."""
        ptr = np.ascontiguousarray(node_ptr, dtype=np.uint32)
        self._check(abi.lib().kwk_tick_bind(self.h, nodes.h, len(ptr) - 1, abi.ptr(ptr)), "kwk_tick_bind")

    @staticmethod
    def _tick_flags(compact) -> int:
        return abi.TICK_COMPACT_PACKED if compact == "packed" else (abi.TICK_COMPACT if compact else 0)

    def tick(self, pods: Optional["Engine"], now_ns: int, seed: int, step: int, compact=False):
        """kwk_tick: lease step -> pod sync -> node step -> pod step, one call (enqueue only)."""
        self._check(abi.lib().kwk_tick(self.h, pods.h if pods is not None else None, now_ns, seed, step,
                                       self._tick_flags(compact)), "kwk_tick")

    def tick_n(self, pods: Optional["Engine"], n: int, now0_ns: int, dt_ns: int, seed: int, step0: int,
               compact=False):
        self._check(abi.lib().kwk_tick_n(self.h, pods.h if pods is not None else None, n, now0_ns, dt_ns, seed, step0,
                                         self._tick_flags(compact)), "kwk_tick_n")

    # timing
    def stream_handle(self) -> int:
        """kwk_stream: the engine's hipStream_t (for torch.cuda.ExternalStream)."""
        h = C.c_void_p()
        self._check(abi.lib().kwk_stream(self.h, C.byref(h)), "kwk_stream")
        return int(h.value or 0)

    def event_record(self, idx: int):
        self._check(abi.lib().kwk_event_record(self.h, idx), "kwk_event_record")

    def event_elapsed_ms(self, a: int, b: int) -> float:
        ms = C.c_float()
        self._check(abi.lib().kwk_event_elapsed(self.h, a, b, C.byref(ms)), "kwk_event_elapsed")
        return float(ms.value)


def _pack_ops(flat):
    from . import cel
    ops = (abi.MetricOp * max(1, len(flat)))()
    for i, (op, x) in enumerate(flat):
        ops[i] = abi.MetricOp(op, int(x) if op == cel.OP_LOAD else 0, float(x) if op == cel.OP_CONST else 0.0)
    return ops


def pack_metric_programs(programs):
    """[(dimension name, [(op, arg), ...])] -> (n, kwk_metric_desc array, n_ops, kwk_metric_op array),
    the arrays kwk_metrics_load takes."""
    descs = (abi.MetricDesc * max(1, len(programs)))()
    flat = []
    for i, (dim, prog) in enumerate(programs):
        descs[i] = abi.MetricDesc(abi.METRIC_DIM[dim], len(flat), len(prog), 0)
        flat += prog
    return len(programs), descs, len(flat), _pack_ops(flat)


def pack_histogram_programs(histograms):
    """[(dimension name, [(le, hidden, [(op, arg), ...]), ...])] -> the six kwk_histograms_load
    arguments after the engine."""
    descs = (abi.HistogramDesc * max(1, len(histograms)))()
    buckets, flat = [], []
    for i, (dim, bks) in enumerate(histograms):
        descs[i] = abi.HistogramDesc(abi.METRIC_DIM[dim], len(buckets), len(bks), 0)
        for le, hidden, prog in bks:
            buckets.append(abi.MetricBucket(float(le), 1 if hidden else 0, len(flat), len(prog), 0))
            flat += prog
    barr = (abi.MetricBucket * max(1, len(buckets)))(*buckets)
    return len(histograms), descs, len(buckets), barr, len(flat), _pack_ops(flat)
