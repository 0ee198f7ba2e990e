"""Multi-GPU layout: nodes sharded in contiguous blocks, pods colocated with their node.

Every Stage decision reads one object's own columns, so a step needs no communication
between GPUs.  Random draws are keyed by the GLOBAL object slot
(``slot_base`` of each engine), so any sharding of a cluster reproduces the single-GPU run bit
for bit.  The only collective is the all-reduce of the small cluster aggregates below (RCCL
over xGMI with the "nccl" backend on ROCm; gloo in the CPU tests), once per reporting
interval.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Sequence, Tuple

import numpy as np


def node_block(n_nodes: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous node block of `rank`: [n*r/W, n*(r+1)/W)."""
    return n_nodes * rank // world, n_nodes * (rank + 1) // world


def pod_range(node_ptr: np.ndarray, node_lo: int, node_hi: int) -> Tuple[int, int]:
    """Node-sorted pods: node j owns [node_ptr[j], node_ptr[j+1])."""
    return int(node_ptr[node_lo]), int(node_ptr[node_hi])


def local_node_ptr(node_ptr: np.ndarray, node_lo: int, node_hi: int) -> np.ndarray:
    return (node_ptr[node_lo:node_hi + 1] - node_ptr[node_lo]).astype(np.uint32)


@dataclass
class Aggregates:
    """Cluster-wide counters summed over GPUs (one all-reduce of < 1 KB)."""
    stage_names: List[str]
    fired_per_stage: np.ndarray                 # int64 [n_stages]
    counts: np.ndarray                          # int64 [n_counts] (phase histogram, ready nodes, ...)
    count_names: List[str] = field(default_factory=list)
    usage: np.ndarray = field(default_factory=lambda: np.zeros(2))  # cpu, memory (float64)

    def pack(self) -> np.ndarray:
        return np.concatenate([self.fired_per_stage.astype(np.float64), self.counts.astype(np.float64),
                               self.usage.astype(np.float64)])

    def unpack(self, v: np.ndarray) -> "Aggregates":
        ns, nc = len(self.fired_per_stage), len(self.counts)
        return Aggregates(self.stage_names, np.rint(v[:ns]).astype(np.int64), np.rint(v[ns:ns + nc]).astype(np.int64),
                          self.count_names, v[ns + nc:ns + nc + 2].copy())

    def allreduce(self, dist, device=None) -> "Aggregates":
        """Sum over all ranks.  float64 carries counts exactly up to 2^53."""
        if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
            return self
        import torch
        t = torch.from_numpy(self.pack())
        if device is not None:
            t = t.to(device)
        dist.all_reduce(t)
        return self.unpack(t.cpu().numpy())

    def as_dict(self) -> dict:
        return {"fired_per_stage": dict(zip(self.stage_names, self.fired_per_stage.tolist())),
                "counts": dict(zip(self.count_names, self.counts.tolist())),
                "usage": {"cpu": float(self.usage[0]), "memory": float(self.usage[1])}}


def phase_masks(program, query: str = ".status.phase", values: Sequence[str] = ()) -> Dict[str, int]:
    """pred masks for a phase histogram from the compiled feature bits (only phases some stage
    or the harness names are interned; everything else falls into 'other')."""
    out: Dict[str, int] = {}
    f = program.features.get(query.replace(" ", ""))
    lits = dict(f.lit_bits) if f is not None else {}
    for v in values or sorted(lits):
        if v in lits:
            out[v] = 1 << lits[v]
    return out


def engine_aggregates(engines, count_masks, count_names, now_ns: int = None, usage_engine=None) -> Aggregates:
    """This shard's aggregates straight from its engines (device work, C ABI): per-stage
    transition counts (kwk_stats) of every engine in order, kwk_count of each engine's masks,
    and — when `usage_engine` is given — the cluster usage of its pods at now_ns (kwk_usage,
    metrics_resource_usage.go:195-224).  `count_masks` / `count_names` are one list per engine."""
    names, fired, counts, cnames = [], [], [], []
    for e, masks, mnames in zip(engines, count_masks, count_names):
        st = e.stats()
        names += list(st["fired_per_stage"])
        fired += list(st["fired_per_stage"].values())
        counts += [int(c) for c in e.count(masks)] if len(masks) else []
        cnames += list(mnames)
    usage = np.zeros(2)
    if usage_engine is not None:
        usage_engine.usage(now_ns)
        _, usage = usage_engine.usage_read(node_out=False)
    return Aggregates(names, np.asarray(fired, dtype=np.int64), np.asarray(counts, dtype=np.int64), cnames,
                      np.asarray(usage, dtype=np.float64))


class DeviceReport:
    """A reporting interval's aggregates computed on the device (kwk_aggregate) with no host
    round trip: per engine [transitions per stage | counts per mask | cluster usage] as float64,
    laid out back to back — in one torch device buffer all-reduced in place over RCCL when the
    job has several ranks, else in each engine's own buffer.  `collect` only enqueues: with
    several ranks the collective is ordered after the engines' streams by stream waits (no host
    synchronisation); `result` reads the last interval back."""

    def __init__(self, engines, count_masks, count_names, usage_engine=None, dist=None, device=None):
        self.engines, self.masks, self.count_names, self.usage_engine = engines, count_masks, count_names, usage_engine
        self.dist = dist if dist is not None and dist.is_initialized() and dist.get_world_size() > 1 else None
        self.sizes = [len(e.p.names) + len(m) + (2 if e is usage_engine else 0) for e, m in zip(engines, count_masks)]
        self.buf = None
        if self.dist is not None:
            import torch
            self.buf = torch.zeros(sum(self.sizes), dtype=torch.float64, device=device)
        self.collected = False

    def collect(self, now_ns: int):
        off = 0
        for e, m, size in zip(self.engines, self.masks, self.sizes):
            ptr = None if self.buf is None else self.buf.data_ptr() + 8 * off
            n = e.aggregate(m, now_ns, usage=e is self.usage_engine, out_ptr=ptr)
            assert n == size, (n, size)
            off += size
        if self.buf is not None:
            if self.buf.is_cuda:
                # stream order, no host sync: the collective's stream waits for the engines'
                # streams, and the engines' later work (the next interval writes this buffer)
                # waits for the collective
                import torch
                cur = torch.cuda.current_stream(self.buf.device)
                ext = [torch.cuda.ExternalStream(e.stream_handle(), device=self.buf.device) for e in self.engines]
                for x in ext:
                    cur.wait_stream(x)
                self.dist.all_reduce(self.buf)  # RCCL over xGMI
                for x in ext:
                    x.wait_stream(cur)
            else:
                for e in self.engines:
                    e.sync()
                self.dist.all_reduce(self.buf)
        self.collected = True

    def result(self) -> Aggregates:
        if not self.collected:
            raise RuntimeError("DeviceReport.result before collect")
        if self.buf is not None:
            flat = self.buf.cpu().numpy()
        else:
            flat = np.concatenate([e.aggregate_read(size) for e, size in zip(self.engines, self.sizes)])
        return self.decode(flat)

    def decode(self, flat: np.ndarray) -> Aggregates:
        """The packed float64 aggregates (this report's layout) -> Aggregates."""
        names, fired, counts, cnames, usage, off = [], [], [], [], np.zeros(2), 0
        for e, m, mn, size in zip(self.engines, self.masks, self.count_names, self.sizes):
            ns = len(e.p.names)
            names += list(e.p.names)
            fired += flat[off:off + ns].tolist()
            counts += flat[off + ns:off + ns + len(m)].tolist()
            cnames += list(mn)
            if e is self.usage_engine:
                usage = flat[off + ns + len(m):off + size].copy()
            off += size
        return Aggregates(names, np.rint(fired).astype(np.int64), np.rint(counts).astype(np.int64), cnames, usage)
