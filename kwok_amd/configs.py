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


# ------------------------------------------------------------------ Metric CR evaluation at scale
METRIC_CR = os.path.join(W.METRICS_DIR, "metrics-resource.yaml")


def c4_pod_workload(n_nodes: int, n_pods: int, seed: int):
    """The C4 pod shape (workload._usage_workload: 1-4 containers, half annotated with the usage
    values) for any size, vectorised: (variants, per-pod variant index, node_ptr)."""
    rng = np.random.default_rng(seed)
    ncont = rng.integers(1, 5, n_pods)
    ann = rng.random(n_pods) < 0.5
    cpu = np.where(ann, rng.integers(0, len(W.CPU_VALUES), n_pods), -1)
    mem = np.where(ann, rng.integers(0, len(W.MEM_VALUES), n_pods), -1)
    code = ((ncont - 1) * 17 + (cpu + 1)) * 17 + (mem + 1)
    del ncont, ann, cpu, mem
    present = np.bincount(code, minlength=4 * 17 * 17) > 0  # the codes that occur, in order: the variants
    uniq = np.nonzero(present)[0]
    remap = (np.cumsum(present) - 1).astype(np.int32)
    idx = remap[code]
    variants = []
    for c in uniq.tolist():
        m, c = c % 17 - 1, c // 17
        cp, k = c % 17 - 1, c // 17 + 1
        a = None if cp < 0 else {"kwok.x-k8s.io/usage-cpu": W.CPU_VALUES[cp], "kwok.x-k8s.io/usage-memory": W.MEM_VALUES[m]}
        variants.append(W.pod_object("p", "n", containers=k, annotations=a))
    node_ptr = np.zeros(n_nodes + 1, dtype=np.int64)
    ppn = np.full(n_nodes, n_pods // n_nodes, dtype=np.int64)
    ppn[: n_pods % n_nodes] += 1
    np.cumsum(ppn, out=node_ptr[1:])
    return variants, idx.astype(np.int32), node_ptr


def _metric_series_bytes(programs, n_nodes, n_pods, n_containers):
    """Algorithmic bytes of one scrape's metric kernels: per series its output (8 B) and its own
    inputs — for pod / container series the pod's state id (1 B; 4 B of cptr for a container),
    per load of a per-pod / per-container input 8 B (usage values from the key: the 4-byte key;
    node inputs are shared by ~100 pods: not counted per series)."""
    from .host import cel
    total = 0
    for dim, ops in programs:
        n = {"node": n_nodes, "pod": n_pods, "container": n_containers}[dim]
        per = 8 + (0 if dim == "node" else 1) + (4 if dim == "container" else 0)
        for op, x in ops:
            if op != cel.OP_LOAD:
                continue
            x = int(x)
            if x in (cel.IN_CONTAINER_CPU, cel.IN_CONTAINER_MEM):
                per += 4
            elif cel.IN_CONTAINER_CUM_CPU <= x <= cel.IN_POD_CUM_MEM or x in (cel.IN_POD_SINCE, cel.IN_POD_CREATED):
                per += 8
            elif dim == "node" and x != cel.IN_NOW_S:
                per += 8
        total += n * per
    return total


def run_metrics(n_nodes: int, n_pods: int, scrapes: int, warmup: int, seed: int, sample_every: int = 97,
                copy: bool = True, device: int = 0) -> dict:
    """kwok_amd/metrics/metrics-resource.yaml (kwok's shipped Metric CR: node / pod / container
    gauges and counters of Usage, CumulativeUsage and SinceSecond) evaluated for every series of
    the cluster per scrape (pkg/kwok/metrics/metrics.go:168-462: the per-node endpoint, all nodes'
    scrapes in one batch): kwk_usage (the usage-from-annotation ClusterResourceUsage, per-pod
    outputs) + kwk_metrics_eval_device, timed by HIP events on the engine's stream; with `copy`
    also the rate with every value copied to the host (kwk_metrics_eval).  Every `sample_every`-th
    node's series are checked against oracle/metrics_ref.py (the shipped CR's values restated)
    within 1e-6 relative over two scrapes."""
    import copy as _copy
    import math
    from .host import cel
    from .host.metrics import MetricsProgram, load_metric_yaml
    from .host.usage import UsageProgram, load_usage_yaml, usage_columns
    t_setup = time.perf_counter()
    pvars, pidx, node_ptr = c4_pod_workload(n_nodes, n_pods, seed)
    prog = KindProgram(load_stage_files(*W.stage_paths(W.POD_FAST)))
    prog.explore(pvars)
    ing = Ingest(prog)
    hot, dels, rec, cls = ing.variant_columns(pvars, pidx)
    pods = Engine(prog, capacity=n_pods, device=device, max_records=max(1, len(ing.records)) + 16)
    pods.load_stages()
    pods.load(hot, dels, rec, cls, ing.record_array())
    del hot, dels, rec, cls
    up = UsageProgram(*load_usage_yaml(open(USAGE_YAML).read()))
    vkeys, cv, mv, mx, ck = usage_columns(up, pvars)
    keys = vkeys[pidx]
    pods.usage_config(node_ptr, keys, cv, mv, mx, ck)
    n_containers = int((keys >> 28).astype(np.int64).sum())
    del keys
    pods.usage_pods(True)
    text = open(METRIC_CR).read()
    mp = MetricsProgram.from_native(text)
    mp.load(pods)
    # creation times: a day's spread of whole seconds, some pods without one (the Go zero time)
    slots = np.arange(n_pods, dtype=np.int64)
    created = NOW0 - ((slots * 7919) % 86400) * 10**9 - 3600 * 10**9
    created[slots % 101 == 0] = np.iinfo(np.int64).min
    zero_unix = float(cel.wrap_int64(cel.GO_ZERO_TIME.ns)) / 1e9
    pods.metrics_inputs(created, np.full(n_nodes, np.iinfo(np.int64).min, dtype=np.int64), np.zeros(n_nodes), zero_unix)
    setup_s = time.perf_counter() - t_setup
    programs = MetricsProgram(load_metric_yaml(text)[1]).programs
    mbytes = _metric_series_bytes(programs, n_nodes, n_pods, n_containers)
    ubytes = n_pods * (1 + 1 + 56) + n_nodes * (4 + 32 + 24)  # id, usage key, per-pod outputs; per node
    t = NOW0
    dt = 10 * 10**9  # kwok's resource-metrics scrape interval is tens of seconds
    n_series = 0
    for k in range(warmup):
        pods.usage(t)
        n_series = pods.metrics_eval_device(t, 0, n_nodes)
        t += dt
    pods.sync()
    ev_u, ev_m = [], []
    t0 = time.perf_counter()
    for k in range(scrapes):
        pods.event_record(3 * k)
        pods.usage(t)
        pods.event_record(3 * k + 1)
        pods.metrics_eval_device(t, 0, n_nodes)
        pods.event_record(3 * k + 2)
        t += dt
    pods.sync()
    wall = (time.perf_counter() - t0) / scrapes
    for k in range(scrapes):
        ev_u.append(pods.event_elapsed_ms(3 * k, 3 * k + 1) / 1e3)
        ev_m.append(pods.event_elapsed_ms(3 * k + 1, 3 * k + 2) / 1e3)
    us_s, m_s = float(np.median(ev_u)), float(np.median(ev_m))
    out = {"metric": "metric series evaluations/sec (all nodes' scrapes per interval)",
           "value": n_series / (us_s + m_s), "series_per_scrape": n_series, "containers": n_containers,
           "device_us_per_scrape": round((us_s + m_s) * 1e6, 1), "usage_us": round(us_s * 1e6, 1),
           "metrics_us": round(m_s * 1e6, 1), "wall_ms_per_scrape": round(wall * 1e3, 3),
           "roofline": {"bound": "hbm", "achieved": round(mbytes / m_s / 1e9, 1), "peak": 8000.0, "unit": "GB/s",
                        "frac": round(mbytes / m_s / 1e9 / 8000.0, 4), "traffic": None,
                        "kernel": "metrics_kernel (node series) + metrics_pod_kernel (every pod / container metric in one launch)",
                        "bytes_per_scrape": int(mbytes)},
           "usage_roofline_frac": round(ubytes / us_s / 1e9 / 8000.0, 4), "usage_bytes_per_scrape": int(ubytes),
           "setup_s": round(setup_s, 1),
           "workload": f"{n_nodes} nodes / {n_pods} pods (C4 shape: 1-4 containers, 50 % annotated), "
                       f"{n_containers} containers; metrics-resource.yaml, {n_series} series per scrape"}
    if copy:
        from .host.engine import PinnedBuffer
        buf = PinnedBuffer(8 * n_series)
        L = abi.lib()
        import ctypes as C
        cnt = C.c_uint64()
        t1 = time.perf_counter()
        for k in range(scrapes):
            pods.usage(t)
            pods._check(L.kwk_metrics_eval(pods.h, t, 0, n_nodes, buf.p, n_series, C.byref(cnt)),
                        "kwk_metrics_eval")
            t += dt
        out["with_host_copy_ms_per_scrape"] = round((time.perf_counter() - t1) / scrapes * 1e3, 3)
        out["with_host_copy_series_per_s"] = n_series / ((time.perf_counter() - t1) / scrapes)
        buf.close()
    # sampled oracle check: every sample_every-th node over two more scrapes
    from oracle.metrics_ref import MetricsOracle
    docs = [d for d in __import__("yaml").safe_load_all(open(USAGE_YAML).read()) if d]
    oracle = MetricsOracle(docs)
    sample = list(range(3, n_nodes, sample_every))
    objs = {}
    for j in sample:
        lo, hi = int(node_ptr[j]), int(node_ptr[j + 1])
        lst = []
        for i in range(lo, hi):
            o = _copy.deepcopy(pvars[int(pidx[i])])
            o["metadata"]["name"] = f"pod-{i}"
            lst.append(o)
        objs[j] = lst
    bad, checked = 0, 0
    first_bad = []
    nodes = {j: {"metadata": {"name": f"node-{j}"}} for j in sample}
    rel = 1e-6
    prev = {}  # the cumulative counters' device values at the first checked scrape
    for k in range(2):
        t_k = t + k * dt
        pods.usage(t_k)
        for j in sample:
            lo = int(node_ptr[j])
            name_to_slot = {o["metadata"]["name"]: lo + q for q, o in enumerate(objs[j])}
            dev = mp.scrape(pods, t_k, j, [nodes[j]], objs[j], node_ptr)
            exp = oracle.scrape(t_k, nodes[j], objs[j],
                                lambda p: None if created[name_to_slot[p["metadata"]["name"]]] == np.iinfo(np.int64).min
                                else int(created[name_to_slot[p["metadata"]["name"]]]))
            for name, series in exp.items():
                d = dict(dev[name])
                cum = "cpu_usage_seconds_total" in name
                if cum and k == 0:
                    # the device's integrators ran over every scrape before, the oracle's start here:
                    # compare the increments (the oracle's value at the second scrape is its first one)
                    for lab, _ in series:
                        prev[(name, j, lab)] = d.get(lab)
                    continue
                for lab, v in series:
                    checked += 1
                    got = d.get(lab)
                    if cum and got is not None:
                        got = None if prev.get((name, j, lab)) is None else got - prev[(name, j, lab)]
                    if got is None or not (got == v or abs(got - v) <= rel * max(abs(v), 1e-300) or
                                           (math.isnan(got) and math.isnan(v))):
                        bad += 1
                        if len(first_bad) < 5:
                            first_bad.append([name, j, [list(x) for x in lab], got, v])
    out["sampled_oracle"] = {"nodes": len(sample), "series_checked": checked, "mismatches": bad,
                             "first_mismatches": first_bad,
                             "note": "every %d-th node's series against oracle/metrics_ref.py (1e-6 rel) over two "
                                     "scrapes; the cumulative counters as the increment between them (the device's "
                                     "integrators started at the engine's first scrape)" % sample_every}
    pods.close()
    return out
