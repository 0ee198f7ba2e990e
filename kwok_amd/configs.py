"""Single-GPU runs of the other BASELINE.json configurations (C1-C4) for ``bench.py --config``.

The headline line is C5 (bench.py's default); these measure the remaining rows of
SURVEY.md §8(d) on one GPU with the same contract (synthetic seeded objects, HIP-event timing
of the engine's own stream, algorithmic bytes from the kernels' own counters).  C1-C4 working
sets fit the 256 MB Infinity Cache: they are reported as absolute throughput, "cache-resident".

  C1  pod-fast + node-fast/heartbeat, 1k nodes / 100k pods, harness churn
  C2  pod-general + pod-chaos, 10k nodes / 1M pods (init containers, override annotations,
      chaos labels, deletionTimestamps), harness churn
  C3  node-initialize + node-heartbeat + node leases, 100k nodes, 10 ms tick
  C4  ResourceUsage / ClusterResourceUsage (usage-from-annotation), 10k nodes / 1M pods
"""
from __future__ import annotations

import os
import time

import numpy as np

from . import workload as W
from .host import abi
from .host.compiler import HarnessSpec, KindProgram
from .host.engine import Engine, Ingest
from .host.stages import load_stage_files

NOW0 = 1_700_000_000 * 10**9
USAGE_YAML = os.path.join(W.METRICS_DIR, "usage-from-annotation.yaml")


def _engine(stage_files, variants, index, harness, kind_salt, device=0):
    prog = KindProgram(load_stage_files(*stage_files), HarnessSpec() if harness else None)
    prog.explore(variants)
    ing = Ingest(prog)
    cols = ing.variant_columns(variants, index)
    eng = Engine(prog, capacity=len(index), device=device, kind_salt=kind_salt,
                 max_records=max(1, len(ing.records)) + 16)
    eng.load_stages()
    eng.set_harness(harness)
    eng.load(*cols, ing.record_array())
    return prog, eng


def _timed(engines_step, sync_engines, timing_engine, steps, warmup):
    for k in range(warmup):
        engines_step(k)
    for e in sync_engines:
        e.sync()
    timing_engine.event_record(0)
    t0 = time.perf_counter()
    for k in range(warmup, warmup + steps):
        engines_step(k)
    timing_engine.event_record(1)
    for e in sync_engines:
        e.sync()
    wall = time.perf_counter() - t0
    return wall, timing_engine.event_elapsed_ms(0, 1) / 1e3


def _timed_n(run_n, sync_engines, timing_engine, steps, warmup):
    run_n(0, warmup)
    for e in sync_engines:
        e.sync()
    timing_engine.event_record(0)
    t0 = time.perf_counter()
    run_n(warmup, steps)
    timing_engine.event_record(1)
    for e in sync_engines:
        e.sync()
    wall = time.perf_counter() - t0
    return wall, timing_engine.event_elapsed_ms(0, 1) / 1e3


HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md


def _roofline(bytes_per_step: float, seconds_per_step: float, what: str, working_set_mb: float) -> dict:
    """The dominant device work of a C1-C4 step against the HBM roofline.  These working sets fit
    the 256 MB Infinity Cache: the fraction is of the HBM peak, but the bytes are
    cache-served, so it is a throughput figure, not an HBM claim (the HBM claim is C5 / C2 at
    100M pods, bench.py's default line)."""
    achieved = bytes_per_step / seconds_per_step / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "kernel": what,
            "bytes_per_step": int(bytes_per_step), "working_set_MB": round(working_set_mb, 1),
            "note": "cache-resident working set: Infinity-Cache served, HBM roofline not applicable"}


def run(config: str, steps: int, warmup: int, seed: int) -> dict:
    if config in ("C1", "C2"):
        n_nodes, n_pods = (1000, 100_000) if config == "C1" else (10_000, 1_000_000)
        cl = W.make_cluster(config, n_nodes, n_pods, seed=seed)
        pprog, pods = _engine(cl.pod_stage_files, cl.pods.variants, cl.pods.index, True, 0)
        nprog, nodes = _engine(cl.node_stage_files, cl.nodes.variants, cl.nodes.index, False, 1)
        dt = 10**9 if config == "C1" else 500 * 10**6

        def run_n(k0, n):  # kwk_step_n: the steps enqueued by one native call per engine
            pods.step_n(n, NOW0 + k0 * dt, dt, seed, k0, False)
            nodes.step_n(n, NOW0 + k0 * dt, dt, seed, k0, False)

        s0p, s0n = pods.stats(), nodes.stats()
        wall, pod_s = _timed_n(run_n, (pods, nodes), pods, steps, warmup)
        s1p, s1n = pods.stats(), nodes.stats()
        fired = (s1p["fired"] - s0p["fired"]) + (s1n["fired"] - s0n["fired"])
        pbytes = s1p["bytes"] - s0p["bytes"]
        ws_mb = n_pods * (s1p["state_bytes"] + 8) / 1e6  # state + due columns
        out = {"metric": "stage transitions/sec", "value": fired / wall, "ms_per_step": wall / steps * 1e3,
               "roofline": _roofline(pbytes / steps, pod_s / steps, "pod sweep (kwk_step_stats bytes)", ws_mb),
               "pod_sweep_us": pod_s / steps * 1e6, "algorithmic_GBps": pbytes / pod_s / 1e9,
               "state_bytes_per_object": s1p["state_bytes"], "transitions_per_step": fired / steps,
               "workload": f"{config}: {n_nodes} nodes / {n_pods} pods, sim dt {dt / 1e6:.0f} ms, harness churn",
               "per_stage": {k: s1p["fired_per_stage"][k] - s0p["fired_per_stage"][k] for k in s1p["fired_per_stage"]}}
        pods.close()
        nodes.close()
        return out
    if config == "C3":
        n_nodes = 100_000
        variants = [W.node_object("node")]
        prog, nodes = _engine(W.stage_paths(W.NODE_FAST + W.NODE_HEARTBEAT), variants, np.zeros(n_nodes, np.int32),
                              False, 1)
        # leases: 60 % to create, 30 % our own stale lease, 10 % foreign expiring within 30 s;
        # every node in the hold set, its first sync queued now (TryHold)
        rng = np.random.default_rng(seed)
        r = rng.random(n_nodes)
        le = np.zeros(n_nodes, dtype=abi.LEASE_DTYPE)
        full = abi.LEASE_EXISTS | abi.LEASE_HOLDER | abi.LEASE_DURATION | abi.LEASE_RENEW
        own = (r >= 0.6) & (r < 0.9)
        foreign = r >= 0.9
        le["flags"] = abi.LEASE_HOLD | abi.LEASE_QUEUED
        le["flags"][own | foreign] |= full
        le["holder"][own] = 1
        le["holder"][foreign] = 7
        le["duration_s"][own | foreign] = 40
        le["renew_ns"][own] = NOW0 - 50 * 10**9
        le["renew_ns"][foreign] = NOW0 - (40 - rng.integers(0, 30, foreign.sum())) * 10**9
        le["next_try_ns"] = NOW0
        nodes.lease_config(1, 40, 10 * 10**9, 0.04, manage_nodes=True)
        nodes.lease_set(le)
        dt = 10 * 10**6

        def run_n(k0, n):  # kwk_tick_n: lease step + node step per tick, all ticks enqueued by one call
            nodes.tick_n(None, n, NOW0 + k0 * dt, dt, seed, k0)

        s0, l0 = nodes.stats(), nodes.lease_stats()
        wall, dev_s = _timed_n(run_n, (nodes,), nodes, steps, warmup)
        s1, l1 = nodes.stats(), nodes.lease_stats()
        fired = s1["fired"] - s0["fired"]
        writes = sum(l1[k] - l0[k] for k in ("creates", "renews", "acquires"))
        syncs = writes + (l1["busy"] - l0["busy"])
        # the tick's algorithmic bytes: the node sweep's count, every lease record read (32 B) and
        # each synced record written back (32 B)
        tbytes = (s1["bytes"] - s0["bytes"]) + steps * n_nodes * 32 + syncs * 32
        out = {"metric": "node transitions + lease writes /sec", "value": (fired + writes) / wall,
               "ms_per_step": wall / steps * 1e3, "device_us_per_step": dev_s / steps * 1e6,
               "roofline": _roofline(tbytes / steps, dev_s / steps, "lease step + node sweep per tick",
                                     n_nodes * (32 + s1["state_bytes"] + 8) / 1e6),
               "state_bytes_per_object": s1["state_bytes"],
               "node_transitions_per_step": fired / steps, "lease_writes_per_step": writes / steps,
               "lease_counts": {k: l1[k] - l0[k] for k in ("creates", "renews", "acquires", "busy")},
               "workload": f"C3: {n_nodes} nodes, node-initialize + node-heartbeat (20 s / 25 s) + leases "
                           "(40 s, renew 10 s +- 4 %), 10 ms tick"}
        nodes.close()
        return out
    if config == "C4":
        from .host.usage import UsageProgram, load_usage_yaml, usage_columns
        n_nodes, n_pods = 10_000, 1_000_000
        cl = W.make_cluster("C4", n_nodes, n_pods, seed=seed)
        uprog = UsageProgram(*load_usage_yaml(open(USAGE_YAML).read()))
        vkeys, cv, mv, mx, ck = usage_columns(uprog, cl.pods.variants)  # no per-name ResourceUsage: per variant
        keys = vkeys[cl.pods.index]
        prog, pods = _engine(cl.pod_stage_files, cl.pods.variants, cl.pods.index, False, 0)
        pods.usage_config(cl.node_ptr, keys, cv, mv, mx, ck)
        containers = int((keys >> 28).astype(np.int64).sum())

        def step(k):
            pods.usage(NOW0 + k * 10**9)

        wall, dev_s = _timed(step, (pods,), pods, steps, warmup)
        node, cluster = pods.usage_read()
        ubytes = n_pods * (4 + 4) + n_nodes * (4 + 32 + 24)
        out = {"metric": "container usage evaluations/sec", "value": containers * steps / wall,
               "ms_per_step": wall / steps * 1e3, "device_us_per_step": dev_s / steps * 1e6,
               "roofline": _roofline(ubytes, dev_s / steps, "usage evaluation (state + usage key per pod, "
                                     "node_ptr + outputs + integrators per node)", ubytes / 1e6),
               "algorithmic_GBps": ubytes / (dev_s / steps) / 1e9, "containers": containers,
               "cluster_cpu": float(cluster[0]), "cluster_memory": float(cluster[1]),
               "workload": f"C4: {n_nodes} nodes / {n_pods} pods, 1-4 containers, 50 % annotated, "
                           "usage-from-annotation ClusterResourceUsage"}
        pods.close()
        return out
    raise ValueError(config)
