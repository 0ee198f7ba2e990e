"""ctypes mirror of include/kwok_engine.h and the loader for the HIP engine library.

This is the Python stand-in for the cgo binding a Go host would use (INTEGRATION.md shows
the Go side).  The library is the product: there is no CPU fallback — if it is missing or
cannot open a GPU, every call raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(_HERE)
LIB_PATH = os.path.join(PKG, "lib", "libkwok_engine.so")

KWK_OK, KWK_EINVAL, KWK_ECAP, KWK_EHIP, KWK_ESTATE = 0, -1, -2, -3, -4
STAGE_NONE = 0xFF
F_ALIVE, F_DIRTY, F_MANAGED, F_HASREC, F_MATCHERR = 1 << 8, 1 << 9, 1 << 10, 1 << 11, 1 << 12
CLASS_SHIFT = 16
CLASS_MASK = 0xFFFF0000
V_DEFAULT, V_OK, V_NOTOK, V_ABSTIME = 0, 1, 2, 3
DEL_ABSENT = -(1 << 63)
MAX_STAGES, MAX_ANY = 32, 4
SLOT_NONE, SLOT_DELETION = -1, -2
NEXT_DELETE, NEXT_IMMEDIATE, NEXT_PATCHES, NEXT_FIN, NEXT_FIN_EMPTY, NEXT_FIN_REMOVE = 1, 2, 4, 8, 16, 32
NEXT_PATCH_STATIC = 64
DELTA_UNKNOWN = (0, 0xFFFFFFFF)
FIRED_DELETED, FIRED_REMATCH, FIRED_DELTA_UNKNOWN = 1, 2, 4


class Hot(C.Structure):
    _fields_ = [("pred", C.c_uint32), ("sched", C.c_uint32), ("due", C.c_int64)]


class Value(C.Structure):
    _fields_ = [("value", C.c_int64), ("nsec", C.c_int32), ("kind", C.c_int32)]


class StageDesc(C.Structure):
    _fields_ = [
        ("eq_mask", C.c_uint32), ("eq_val", C.c_uint32), ("n_any", C.c_uint32), ("any_want", C.c_uint32),
        ("any_mask", C.c_uint32 * MAX_ANY),
        ("weight_default", C.c_int64), ("weight_slot", C.c_int32),
        ("has_delay", C.c_int32), ("delay_default", C.c_int64), ("delay_slot", C.c_int32),
        ("has_jitter", C.c_int32), ("jitter_default", C.c_int64), ("jitter_default_ok", C.c_int32),
        ("jitter_slot", C.c_int32),
        ("flags", C.c_uint32), ("fin_add", C.c_uint32), ("fin_remove", C.c_uint32), ("applied_mask", C.c_uint32),
    ]


class StageTable(C.Structure):
    _fields_ = [("n_stages", C.c_uint32), ("fin_group_mask", C.c_uint32), ("n_classes", C.c_uint32),
                ("version", C.c_uint32), ("pred_bits", C.c_uint32), ("disregard_mask", C.c_uint32),
                ("reserved", C.c_uint32 * 2),
                ("stages", StageDesc * MAX_STAGES)]


class Delta(C.Structure):
    _fields_ = [("and_mask", C.c_uint32), ("or_mask", C.c_uint32)]


class Harness(C.Structure):
    _fields_ = [("enable", C.c_uint32), ("keep_mask", C.c_uint32), ("terminal_mask", C.c_uint32),
                ("deletion_bit", C.c_uint32), ("track_deletion", C.c_uint32), ("reserved", C.c_uint32 * 3)]


class FiredRec(C.Structure):
    _fields_ = [("slot", C.c_uint32), ("stage", C.c_uint16), ("flags", C.c_uint16)]


class StepStats(C.Structure):
    _fields_ = [("steps", C.c_uint64), ("matched", C.c_uint64), ("fired", C.c_uint64), ("bytes", C.c_uint64),
                ("fired_per_stage", C.c_uint64 * MAX_STAGES), ("state_bytes", C.c_uint64),
                ("line_bytes", C.c_uint64)]


class FetchInfo(C.Structure):
    """kwk_fetch_info (kwk_fired_fetch_async / kwk_fired_fetch_step)."""
    _fields_ = [("n_records", C.c_uint32), ("record_bytes", C.c_uint32), ("n_segs", C.c_uint32),
                ("region_slots", C.c_uint32), ("format", C.c_uint32), ("reserved", C.c_uint32), ("bytes", C.c_uint64),
                ("step", C.c_uint64)]


class SweepInfo(C.Structure):
    _fields_ = [(k, C.c_uint32) for k in ("kernel", "q", "persistent", "depth", "grid", "tiles", "harness", "steps")]


SWEEP_16, SWEEP_16_FSM, SWEEP_W4, SWEEP_W8, SWEEP_8, SWEEP_WD = 1, 2, 3, 4, 5, 6  # KWK_SWEEP_*


class EngineDesc(C.Structure):
    _fields_ = [("device", C.c_int32), ("capacity", C.c_uint32), ("value_slots", C.c_uint32),
                ("max_records", C.c_uint32), ("slot_base", C.c_uint64), ("kind_salt", C.c_uint32),
                ("flags", C.c_uint32)]


ENGINE_WIDE_STATE = 1
ENGINE_STATE32 = 2
ENGINE_STATE16 = 4   # never the 1-byte dictionary format
ENGINE_SPLIT_DUE = 8  # never the fused 8-byte record {packed word, relative due}
TUNE_SWEEP16 = 18  # KWK_SWEEP16_SHAPE(q, persistent, kernel, table): sweep16_shape()
TUNE_USAGE = 19    # USAGE_KEY8 | USAGE_AGG_FUSED
USAGE_KEY8, USAGE_AGG_FUSED = 1, 2
TUNE_COMPACT_SMALL = 8
TUNE_BYTE_STATE = 9
TUNE_WORD_TILES = 10
TUNE_STREAM_PRIORITY = 15
TUNE_FUSE_STEPS = 17
TUNE_TAIL_HANDBACK = 20  # the 2-byte one-tile-per-workgroup sweep writes its step's list itself (1) or not (0)


def sweep16_shape(q: int = 4, persistent: int = 1, kernel: int = 2, table: int = 1) -> int:
    """KWK_SWEEP16_SHAPE: the value of KWK_TUNE_SWEEP16 (defaults = KWK_SWEEP16_DEFAULT)."""
    return q | persistent << 4 | kernel << 8 | table << 12


class Lease(C.Structure):
    _fields_ = [("renew_ns", C.c_int64), ("next_try_ns", C.c_int64), ("holder", C.c_uint32), ("duration_s", C.c_int32),
                ("transitions", C.c_int32), ("flags", C.c_uint32)]


class LeaseParams(C.Structure):
    _fields_ = [("holder_id", C.c_uint32), ("lease_duration_s", C.c_int32), ("renew_interval_ns", C.c_int64),
                ("renew_jitter", C.c_double), ("manage_nodes", C.c_uint32), ("reserved", C.c_uint32)]


class LeaseCounters(C.Structure):
    _fields_ = [("steps", C.c_uint64), ("creates", C.c_uint64), ("renews", C.c_uint64), ("acquires", C.c_uint64),
                ("busy", C.c_uint64)]


LEASE_EXISTS, LEASE_HOLDER, LEASE_DURATION, LEASE_RENEW, LEASE_HOLD, LEASE_QUEUED = 1, 2, 4, 8, 16, 32
LEASE_OP_CREATE, LEASE_OP_RENEW, LEASE_OP_ACQUIRE, LEASE_OP_BUSY = 1, 2, 3, 4
LEASE_DTYPE = np.dtype([("renew_ns", "<i8"), ("next_try_ns", "<i8"), ("holder", "<u4"), ("duration_s", "<i4"),
                        ("transitions", "<i4"), ("flags", "<u4")])

HOT_DTYPE = np.dtype([("pred", "<u4"), ("sched", "<u4"), ("due", "<i8")])
VALUE_DTYPE = np.dtype([("value", "<i8"), ("nsec", "<i4"), ("kind", "<i4")])
FIRED_DTYPE = np.dtype([("slot", "<u4"), ("stage", "<u2"), ("flags", "<u2")])


class MetricOp(C.Structure):
    _fields_ = [("op", C.c_uint32), ("arg", C.c_uint32), ("value", C.c_double)]


class MetricDesc(C.Structure):
    _fields_ = [("dimension", C.c_uint32), ("first_op", C.c_uint32), ("n_ops", C.c_uint32), ("reserved", C.c_uint32)]


METRIC_DIM = {"node": 0, "pod": 1, "container": 2}


class MetricBucket(C.Structure):
    _fields_ = [("le", C.c_double), ("hidden", C.c_uint32), ("first_op", C.c_uint32), ("n_ops", C.c_uint32),
                ("reserved", C.c_uint32)]


class HistogramDesc(C.Structure):
    _fields_ = [("dimension", C.c_uint32), ("first_bucket", C.c_uint32), ("n_buckets", C.c_uint32),
                ("reserved", C.c_uint32)]


class Backoff(C.Structure):
    """kwk_backoff = wait.Backoff; default = defaultBackoff (controllers/utils.go:133-135)."""
    _fields_ = [("duration_ns", C.c_int64), ("factor", C.c_double), ("jitter", C.c_double), ("cap_ns", C.c_int64)]


DEFAULT_BACKOFF = dict(duration_ns=10**9, factor=2.0, jitter=0.2, cap_ns=32 * 60 * 10**9)

assert C.sizeof(MetricOp) == 16 and C.sizeof(MetricDesc) == 16
assert C.sizeof(MetricBucket) == 24 and C.sizeof(HistogramDesc) == 16
assert C.sizeof(Hot) == 16 and C.sizeof(Value) == 16 and C.sizeof(StageDesc) == 96
assert C.sizeof(Lease) == 32 == LEASE_DTYPE.itemsize and C.sizeof(LeaseParams) == 32
assert HOT_DTYPE.itemsize == 16 and VALUE_DTYPE.itemsize == 16 and FIRED_DTYPE.itemsize == 8

# every symbol include/kwok_engine.h declares (checked by the CPU test suite)
EXPORTS = [
    "kwk_last_error", "kwk_engine_create", "kwk_engine_destroy", "kwk_load_stages", "kwk_set_harness", "kwk_load",
    "kwk_upsert", "kwk_set_records", "kwk_delete", "kwk_step", "kwk_match", "kwk_fired", "kwk_stats", "kwk_read", "kwk_sync",
    "kwk_usage_config", "kwk_usage", "kwk_usage_read", "kwk_device_ptrs", "kwk_event_record", "kwk_event_elapsed", "kwk_stream", "kwk_step_n", "kwk_step_n_pair",
    "kwk_abi_version", "kwk_tile_objects", "kwk_count", "kwk_lease_config", "kwk_lease_set", "kwk_lease_step",
    "kwk_lease_ops", "kwk_lease_read", "kwk_lease_stats", "kwk_lease_sync_pods", "kwk_usage_pods",
    "kwk_usage_read_pods", "kwk_retry", "kwk_lease_fail", "kwk_set_tuning", "kwk_fired_compact", "kwk_fired_device",
    "kwk_alloc_host", "kwk_free_host", "kwk_replace", "kwk_usage_mixed", "kwk_usage_read_containers",
    "kwk_metrics_load", "kwk_metrics_inputs", "kwk_metrics_eval", "kwk_aggregate", "kwk_aggregate_read",
    "kwk_last_sweep", "kwk_tick_bind", "kwk_tick", "kwk_tick_n", "kwk_histograms_load", "kwk_histograms_eval",
    "kwk_fired_compact_packed", "kwk_fired_packed", "kwk_fired_packed_device", "kwk_fired_compact_packed16",
    "kwk_fired_packed16", "kwk_fired_fetch_async", "kwk_fired_fetch_wait",
    "kwk_fired_compact_bits", "kwk_fired_bits", "kwk_fired_keep", "kwk_fired_fetch_step",
    "kwk_metrics_eval_device", "kwk_histograms_eval_device",
]
ABI_VERSION = 2  # KWK_ABI_VERSION of include/kwok_engine.h: the library must match the structs above
TICK_COMPACT = 1 << 0  # KWK_TICK_COMPACT
TICK_COMPACT_PACKED = 1 << 1  # KWK_TICK_COMPACT_PACKED
COMPACT_PACKED = 2  # kwk_step_n compact = KWK_COMPACT_PACKED
COMPACT_PACKED16 = 3  # kwk_step_n compact = KWK_COMPACT_PACKED16 (2-byte records where the sweep has them)
COMPACT_BITS = 4  # kwk_step_n compact = KWK_COMPACT_BITS (per-segment fired maps + 2-bit stage codes, same engines)
AGG_USAGE = 1 << 0  # KWK_AGG_USAGE

_lib = None


class EngineError(RuntimeError):
    pass


def _p(t):
    return C.POINTER(t)


def lib():
    """Load libkwok_engine.so (built in-tree by __graft_entry__.build / kwok_amd.build)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EngineError(f"HIP engine library missing: {LIB_PATH} (run python -m kwok_amd.build)")
    L = C.CDLL(LIB_PATH)
    s = C.c_int32
    L.kwk_last_error.restype = C.c_char_p
    L.kwk_last_error.argtypes = [C.c_void_p]
    L.kwk_engine_create.argtypes = [_p(EngineDesc), _p(C.c_void_p)]
    L.kwk_engine_destroy.argtypes = [C.c_void_p]
    L.kwk_load_stages.argtypes = [C.c_void_p, _p(StageTable), C.c_void_p]
    L.kwk_set_harness.argtypes = [C.c_void_p, _p(Harness)]
    L.kwk_load.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                           C.c_void_p]
    L.kwk_upsert.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.kwk_replace.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.kwk_usage_mixed.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p]
    L.kwk_usage_read_containers.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32, _p(C.c_uint32)]
    L.kwk_metrics_load.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p]
    L.kwk_metrics_inputs.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_double]
    L.kwk_metrics_eval.argtypes = [C.c_void_p, C.c_int64, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64, _p(C.c_uint64)]
    L.kwk_metrics_eval_device.argtypes = [C.c_void_p, C.c_int64, C.c_uint32, C.c_uint32, _p(C.c_void_p),
                                          _p(C.c_uint64)]
    L.kwk_histograms_eval_device.argtypes = [C.c_void_p, C.c_int64, C.c_uint32, C.c_uint32, _p(C.c_void_p),
                                             _p(C.c_uint64)]
    L.kwk_histograms_load.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p]
    L.kwk_histograms_eval.argtypes = [C.c_void_p, C.c_int64, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64,
                                      _p(C.c_uint64)]
    L.kwk_set_records.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
    L.kwk_delete.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
    L.kwk_retry.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p,
                            C.c_void_p, C.c_void_p, C.c_void_p, _p(Backoff)]
    L.kwk_step.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64]
    L.kwk_match.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64]
    L.kwk_fired.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, _p(C.c_uint32)]
    L.kwk_fired_compact.argtypes = [C.c_void_p]
    L.kwk_step_n.argtypes = [C.c_void_p, C.c_uint32, C.c_int64, C.c_int64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32,
                             C.c_uint32]
    L.kwk_step_n_pair.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_int64, C.c_int64, C.c_uint64, C.c_uint64,
                                  C.c_uint32, C.c_uint32, C.c_uint32]
    L.kwk_fired_device.argtypes = [C.c_void_p, _p(C.c_void_p), _p(C.c_void_p)]
    L.kwk_fired_compact_packed.argtypes = [C.c_void_p]
    L.kwk_fired_packed.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, _p(C.c_uint32)]
    L.kwk_fired_compact_packed16.argtypes = [C.c_void_p]
    L.kwk_fired_packed16.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, _p(C.c_uint32), C.c_void_p, C.c_uint32,
                                     _p(C.c_uint32), _p(C.c_uint32)]
    L.kwk_fired_packed_device.argtypes = [C.c_void_p, _p(C.c_void_p), _p(C.c_void_p)]
    L.kwk_fired_fetch_async.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, _p(FetchInfo)]
    L.kwk_fired_fetch_wait.argtypes = [C.c_void_p]
    L.kwk_fired_compact_bits.argtypes = [C.c_void_p]
    L.kwk_fired_bits.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, _p(C.c_uint64), _p(C.c_uint32), _p(C.c_uint32),
                                 _p(C.c_uint32)]
    L.kwk_fired_keep.argtypes = [C.c_void_p, C.c_uint32]
    L.kwk_fired_fetch_step.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32,
                                       _p(FetchInfo)]
    L.kwk_alloc_host.argtypes = [C.c_uint64, _p(C.c_void_p)]
    L.kwk_free_host.argtypes = [C.c_void_p]
    L.kwk_set_tuning.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
    L.kwk_stats.argtypes = [C.c_void_p, _p(StepStats)]
    L.kwk_read.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p]
    L.kwk_sync.argtypes = [C.c_void_p]
    L.kwk_usage_config.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                   C.c_uint32, C.c_void_p]
    L.kwk_usage.argtypes = [C.c_void_p, C.c_int64]
    L.kwk_usage_read.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.kwk_usage_pods.argtypes = [C.c_void_p, C.c_uint32]
    L.kwk_usage_read_pods.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
    L.kwk_device_ptrs.argtypes = [C.c_void_p, _p(C.c_void_p), _p(C.c_void_p), _p(C.c_void_p)]
    L.kwk_event_record.argtypes = [C.c_void_p, C.c_uint32]
    L.kwk_stream.argtypes = [C.c_void_p, _p(C.c_void_p)]
    L.kwk_event_elapsed.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, _p(C.c_float)]
    L.kwk_count.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
    L.kwk_aggregate.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_int64, C.c_uint32, C.c_void_p, _p(C.c_uint32)]
    L.kwk_aggregate_read.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32]
    L.kwk_lease_config.argtypes = [C.c_void_p, _p(LeaseParams)]
    L.kwk_lease_set.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
    L.kwk_lease_step.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64]
    L.kwk_lease_ops.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, _p(C.c_uint32)]
    L.kwk_lease_read.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
    L.kwk_lease_fail.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p]
    L.kwk_lease_stats.argtypes = [C.c_void_p, _p(LeaseCounters)]
    L.kwk_lease_sync_pods.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]
    L.kwk_last_sweep.argtypes = [C.c_void_p, _p(SweepInfo)]
    L.kwk_tick_bind.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]
    L.kwk_tick.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_uint32]
    L.kwk_tick_n.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_int64, C.c_int64, C.c_uint64, C.c_uint64,
                             C.c_uint32]
    L.kwk_abi_version.restype = C.c_uint32
    L.kwk_tile_objects.restype = C.c_uint32
    for name in EXPORTS:
        fn = getattr(L, name)
        if name not in ("kwk_last_error", "kwk_abi_version", "kwk_tile_objects"):
            fn.restype = s
    if L.kwk_abi_version() != ABI_VERSION:
        raise EngineError(f"{LIB_PATH}: ABI version {L.kwk_abi_version()}, this binding needs {ABI_VERSION} "
                          "(rebuild: python -m kwok_amd.build)")
    _lib = L
    return L


def check(status: int, what: str = "", eng=None):
    """Raise EngineError for a failed call; the message is the engine's own (kwk_last_error(eng)),
    or the calling thread's for calls without an engine."""
    if status != KWK_OK:
        msg = lib().kwk_last_error(eng).decode(errors="replace")
        raise EngineError(f"{what} failed ({status}): {msg}")


def ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def bits_slot(i: np.ndarray) -> np.ndarray:
    """KWK_BITS_SLOT: the slot within its segment of map bit i (lane i >> 5, phase-1 bit k = i & 31 of
    that lane, i.e. byte k >> 3 of its dword k & 7)."""
    i = i.astype(np.uint32)
    jj, lane, b = i & np.uint32(7), (i >> np.uint32(5)) & np.uint32(63), (i >> np.uint32(3)) & np.uint32(3)
    return (jj >> np.uint32(2)) * np.uint32(1024) + lane * np.uint32(16) + (jj & np.uint32(3)) * np.uint32(4) + b


def bits_decode(words: np.ndarray, n_segs: int, region_slots: int):
    """(slot, stage) arrays of a kwk_fired_bits list (KWK_COMPACT_BITS in kwok_engine.h): per segment
    {records c, nonzero map bytes z} up front, then its 8 summary words, its z nonzero map bytes
    and its c stage codes at the running offset."""
    words = np.asarray(words, dtype=np.uint32)
    n = int(n_segs)
    head = words[:n]
    c = (head & np.uint32(0xFFFF)).astype(np.int64)
    z = (head >> np.uint32(16)).astype(np.int64)
    zw = (z + 3) // 4
    size = 8 + zw + (c + 15) // 16
    base = n + np.concatenate(([0], np.cumsum(size)))[:-1]
    summ = words[base[:, None] + np.arange(8)]  # n x 8
    nzb = np.unpackbits(np.ascontiguousarray(summ).view(np.uint8), bitorder="little").reshape(n, 256)
    seg, m = np.nonzero(nzb)  # the nonzero map bytes, in order
    assert np.array_equal(np.bincount(seg, minlength=n), z), "summary / byte count mismatch"
    rank = np.arange(len(seg), dtype=np.int64) - np.repeat(np.concatenate(([0], np.cumsum(z)))[:-1], z)
    byte_view = words.view(np.uint8)
    mb = byte_view[4 * (base[seg] + 8) + rank]
    bits = np.unpackbits(mb[:, None], axis=1, bitorder="little")  # one row per nonzero byte
    row, b = np.nonzero(bits)
    seg_b = seg[row]
    i = m[row] * 8 + b
    assert np.array_equal(np.bincount(seg_b, minlength=n), c), "map / record count mismatch"
    rank2 = np.arange(len(seg_b), dtype=np.int64) - np.repeat(np.concatenate(([0], np.cumsum(c)))[:-1], c)
    w = words[base[seg_b] + 8 + zw[seg_b] + rank2 // 16]
    stage = (w >> (2 * (rank2 % 16)).astype(np.uint32)) & np.uint32(3)
    slot = seg_b.astype(np.int64) * int(region_slots) + bits_slot(i).astype(np.int64)
    return slot, stage


def fired16_decode(recs: np.ndarray, seg_counts: np.ndarray, region_slots: int):
    """(slot, stage, flags) arrays of a kwk_fired_packed16 list (KWK_FIRED16_* in kwok_engine.h)."""
    r = recs.astype(np.uint32)
    x = r & np.uint32(0x7FF)
    jj = x >> np.uint32(8)
    lane = ((x >> np.uint32(2)) & np.uint32(63)) ^ jj
    within = (jj >> np.uint32(2)) * np.uint32(1024) + lane * np.uint32(16) + (jj & np.uint32(3)) * np.uint32(4) + \
        (x & np.uint32(3))
    seg = np.repeat(np.arange(len(seg_counts), dtype=np.int64), seg_counts.astype(np.int64))
    slot = seg * int(region_slots) + within.astype(np.int64)
    return slot, (r >> np.uint32(11)) & np.uint32(3), (r >> np.uint32(13)) & np.uint32(7)
