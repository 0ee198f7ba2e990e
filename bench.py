"""Headline benchmark: stage transitions/sec at 1M nodes / 100M pods (BASELINE.json).

One *step* = one reconciliation pass of the HIP engines over the whole resident cluster
(pods + nodes): harness churn, match of changed objects, weighted pick + delay/jitter,
firing of due objects and their next-state deltas.  Inputs are resident in HBM before the
timed region; the fired lists stay on the device (the Go host would pull them with
kwk_fired — the PCIe-inclusive rate is reported in DESIGN.md, never here).

    python bench.py [--gpus N --steps K --warmup W]          # N>1 under torch.distributed.run

Multi-GPU (one process per GPU): every rank owns a contiguous block of nodes and the pods
on them (no data-path collective); the cluster-wide aggregates (transitions per stage, bytes)
are summed with one RCCL all-reduce after the timed region.  Default "scaling": "weak" — each
rank keeps the full C5 shard (--nodes x --pods-per-node), so N GPUs simulate an N-times
larger cluster; --scaling strong splits --nodes over the ranks instead.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "stage transitions/sec (whole node), 1M nodes/100M pods; achieved HBM GB/s"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)).astype(np.uint64)
    x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)).astype(np.uint64)
    x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)).astype(np.uint64)
    return x ^ (x >> np.uint64(31))


def shard_pod_variants(pod_lo: int, pod_hi: int, seed: int, job_frac: float) -> np.ndarray:
    """Variant id per pod (0 plain, 1 Job-owned): a hash of the GLOBAL pod id, so every
    sharding of the cluster sees the same objects."""
    out = np.empty(pod_hi - pod_lo, dtype=np.int32)
    chunk = 1 << 24
    thr = np.uint64(int(job_frac * (1 << 32)))
    for a in range(pod_lo, pod_hi, chunk):
        b = min(pod_hi, a + chunk)
        h = splitmix64(np.arange(a, b, dtype=np.uint64) ^ np.uint64(seed))
        out[a - pod_lo:b - pod_lo] = ((h >> np.uint64(32)) < thr).astype(np.int32)
    return out


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def build_engines(n_nodes, pods_per_node, rank, world, device, seed, job_frac, weak=True, wide_state=False):
    from kwok_amd import workload as W
    from kwok_amd.host.compiler import HarnessSpec, KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files

    if weak:  # rank r owns global nodes [r*n, (r+1)*n)
        node_lo, node_hi = n_nodes * rank, n_nodes * (rank + 1)
    else:
        node_lo, node_hi = n_nodes * rank // world, n_nodes * (rank + 1) // world
    pod_lo, pod_hi = node_lo * pods_per_node, node_hi * pods_per_node
    # pods: pod-fast (C1 stage mix) with harness churn
    pvars = [W.pod_object("p", "n"), W.pod_object("p", "n", job=True)]
    pprog = KindProgram(load_stage_files(*W.stage_paths(W.POD_FAST)), HarnessSpec())
    pprog.explore(pvars)
    ping = Ingest(pprog)
    log(f"rank {rank}: generating pods [{pod_lo}, {pod_hi})")
    pidx = shard_pod_variants(pod_lo, pod_hi, seed, job_frac)
    phot, pdel, prec, pcls = ping.variant_columns(pvars, pidx)
    log(f"rank {rank}: loading {pod_hi - pod_lo} pods onto device {device}")
    del pidx
    pods = Engine(pprog, capacity=pod_hi - pod_lo, device=device, slot_base=pod_lo, kind_salt=0, wide_state=wide_state)
    pods.load_stages()
    pods.load(phot, pdel, prec, pcls, ping.record_array())
    del phot, pdel, prec, pcls
    # nodes: node-initialize + node-heartbeat
    nvars = [W.node_object("node")]
    nprog = KindProgram(load_stage_files(*W.stage_paths(W.NODE_FAST + W.NODE_HEARTBEAT)))
    nprog.explore(nvars)
    ning = Ingest(nprog)
    nidx = np.zeros(node_hi - node_lo, dtype=np.int32)
    nhot, ndel, nrec, ncls = ning.variant_columns(nvars, nidx)
    nodes = Engine(nprog, capacity=node_hi - node_lo, device=device, slot_base=node_lo, kind_salt=1,
                   wide_state=wide_state)
    nodes.load_stages()
    nodes.load(nhot, ndel, nrec, ncls, ning.record_array())
    return pods, nodes, (node_lo, node_hi, pod_lo, pod_hi)


def cpu_baseline(sample_s: float, seed: int):
    """The oracle (refcpu, C++ restatement of the Go path) timed on this host: per object a
    JSON re-parse (ToJSONStandard), Lifecycle.Match and Stage.Delay, on one thread (the
    reference's single preprocess goroutine, pod_controller.go:150).  Each stage transition
    costs the reference at least one such match, so objects/sec bounds its transitions/sec."""
    from kwok_amd import workload as W
    from kwok_amd.host.stages import load_stage_files, to_v1alpha1
    from oracle import refcpu
    stages = load_stage_files(*W.stage_paths(W.POD_FAST))
    lc = refcpu.Lifecycle([to_v1alpha1(s) for s in stages])
    # a sample in the steady-state mix: Pending (fresh / re-created), Running, Succeeded+deleting
    base = W.make_cluster("C1", 100, 20000, seed=seed).pods.materialize()
    objs = []
    for i, o in enumerate(base):
        r = i % 10
        if r < 4:
            o["status"] = {"phase": "Running", "podIP": "10.0.0.2", "hostIP": "10.0.0.1"}
        elif r < 6 and o["metadata"].get("ownerReferences"):
            o["status"] = {"phase": "Succeeded", "podIP": "10.0.0.2"}
            o["metadata"]["deletionTimestamp"] = "2023-11-14T22:13:20Z"
        objs.append(json.dumps(o, separators=(",", ":")).encode())
    now = 1_700_000_000 * 10**9
    lc.match_batch(objs[:2000], now, seed, 0)  # warm-up
    t0 = time.perf_counter()
    n = 0
    reps = 0
    while time.perf_counter() - t0 < sample_s:
        lc.match_batch(objs, now, seed, reps + 1)
        n += len(objs)
        reps += 1
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "stage transitions/sec (upper bound: matches/sec)", "cores": 1,
            "kind": "port",
            "sample": f"{len(objs)} pod JSON objects x {reps} passes ({dt:.1f} s): JSON re-parse + Match + Delay "
                      f"(pod-fast stages), 1 thread = the reference's preprocess goroutine; CPU "
                      f"{_cpu_model()} ({os.cpu_count()} logical CPUs visible)"}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--nodes", type=int, default=1_000_000, help="nodes per GPU (weak) or in total (strong)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak")
    ap.add_argument("--config", choices=("C1", "C2", "C3", "C4", "C5"), default="C5",
                    help="BASELINE.json configuration; C5 is the headline line, C1-C4 run on one GPU")
    ap.add_argument("--pods-per-node", type=int, default=100)
    ap.add_argument("--job-frac", type=float, default=0.1)
    ap.add_argument("--seed", type=int, default=0x6B776F6B)
    ap.add_argument("--dt-ms", type=int, default=1000, help="simulated time per step")
    ap.add_argument("--cpu-sample-s", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-harness", action="store_true", help="diagnostic: no churn (steady state is an idle sweep)")
    ap.add_argument("--wide-state", action="store_true", default=os.environ.get("KWOK_BENCH_WIDE") == "1",
                    help="diagnostic: force the 8-byte device state format")
    args = ap.parse_args()

    if args.config != "C5":
        from kwok_amd import build as kbuild
        from kwok_amd import configs
        if not os.path.exists(kbuild.OUT):
            kbuild.build()
        r = configs.run(args.config, args.steps, args.warmup, args.seed)
        line = {"metric": r.pop("metric"), "value": round(r.pop("value"), 1), "n_gpus": 1, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(r.pop("ms_per_step"), 4), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "u32/i64" if args.config != "C4" else "f64",
                "data": "synthetic (seeded kwokctl-shaped objects), cache-resident working set",
                "config": {"workload": r.pop("workload")}, "detail": r}
        print(json.dumps(line), flush=True)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")

    from kwok_amd import build as kbuild
    if rank == 0 and not os.path.exists(kbuild.OUT):
        kbuild.build()

    t_setup = time.perf_counter()
    pods, nodes, (nlo, nhi, plo, phi) = build_engines(args.nodes, args.pods_per_node, rank, world, local_rank,
                                                      args.seed, args.job_frac, weak=args.scaling == "weak",
                                                      wide_state=args.wide_state)
    setup_s = time.perf_counter() - t_setup
    if args.no_harness:
        pods.set_harness(False)
    now0 = 1_700_000_000 * 10**9
    dt = args.dt_ms * 10**6

    def step(k):
        now = now0 + k * dt
        pods.step(now, args.seed, k)
        nodes.step(now, args.seed, k)

    log(f"setup {setup_s:.1f} s; warmup {args.warmup} steps")
    for k in range(args.warmup):
        step(k)
    pods.sync()
    nodes.sync()
    s0p, s0n = pods.stats(), nodes.stats()

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    pods.sync()
    nodes.sync()
    t0 = time.perf_counter()
    pods.event_record(0)
    nodes.event_record(0)
    for k in range(args.warmup, args.warmup + args.steps):
        step(k)
    pods.event_record(1)
    nodes.event_record(1)
    pods.sync()
    nodes.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    pod_ms = pods.event_elapsed_ms(0, 1)
    node_ms = nodes.event_elapsed_ms(0, 1)
    s1p, s1n = pods.stats(), nodes.stats()

    fired = (s1p["fired"] - s0p["fired"]) + (s1n["fired"] - s0n["fired"])
    pbytes = s1p["bytes"] - s0p["bytes"]
    plines = s1p["line_bytes"] - s0p["line_bytes"]
    per_stage = {k: s1p["fired_per_stage"][k] - s0p["fired_per_stage"][k] for k in s1p["fired_per_stage"]}
    per_stage.update({k: s1n["fired_per_stage"][k] - s0n["fired_per_stage"][k] for k in s1n["fired_per_stage"]})

    agg = np.array([fired, pbytes, elapsed * 1e9], dtype=np.float64)
    if dist is not None:
        import torch
        t = torch.tensor([float(fired), float(pbytes)], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(t)  # cluster-wide aggregates over RCCL (xGMI)
        tm = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        agg = np.array([t[0].item(), t[1].item(), tm.item() * 1e9])
    total_fired, total_bytes, max_ns = agg
    max_s = max_ns / 1e9

    total_nodes = args.nodes * world if args.scaling == "weak" else args.nodes
    if rank == 0:
        value = total_fired / max_s
        pod_kernel_s = pod_ms / 1e3 / args.steps
        achieved = (pbytes / args.steps) / pod_kernel_s / 1e9
        sb = int(s1p["state_bytes"])
        traffic = _pmc_traffic(sb)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_GBps": (round(traffic / pod_kernel_s / 1e9, 1) if traffic else None),
                "kernel": ("sweep16_kernel" if sb == 2 else "sweep_kernel") + " (pods)",
                "bytes_per_launch": int(pbytes / args.steps), "state_bytes_per_object": sb,
                # the same count with state writes as the whole 128-byte lines the sweep stores
                # (at ~10 % churn nearly every line of the 2-byte column holds a changed word)
                "line_bytes_per_launch": int(plines / args.steps),
                "line_achieved": round(plines / args.steps / pod_kernel_s / 1e9, 1),
                "line_frac": round(plines / args.steps / pod_kernel_s / 1e9 / HBM_PEAK_GBS, 4),
                "avg_launch_us": round(pod_kernel_s * 1e6, 2)}
        cpu = None
        log(f"timed {args.steps} steps in {max_s:.3f} s; cpu baseline next")
        if not args.no_cpu_baseline and world == 1:  # the CPU leg runs on rank 0 at N=1 only
            cpu = cpu_baseline(args.cpu_sample_s, args.seed)
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "stage transitions/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(max_s / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
            "dtype": {2: "u16", 4: "u32", 8: "u32x2"}[sb] + "/i64",
            "data": "synthetic (seeded kwokctl-shaped pods/nodes; pod-fast + node-fast/heartbeat stages)",
            "config": {"workload": f"C5: {args.nodes:,} nodes / {args.nodes * args.pods_per_node:,} pods "
                                   f"{'per GPU' if args.scaling == 'weak' else 'in total'}, pod-fast + "
                                   "node-initialize/heartbeat, harness churn (Succeeded -> delete -> re-create), "
                                   "10% Job-owned",
                       "nodes": total_nodes, "pods": total_nodes * args.pods_per_node,
                       "nodes_per_gpu": nhi - nlo, "parallelism": f"node-shard{world}",
                       "sim_dt_ms": args.dt_ms},
            "roofline": roof,
            "cpu_baseline": cpu,
            "detail": {"transitions_per_step": total_fired / args.steps, "per_stage_rank0": per_stage,
                       "pod_kernel_ms_per_step": round(pod_ms / args.steps, 4),
                       "node_kernel_ms_per_step": round(node_ms / args.steps, 4), "setup_s": round(setup_s, 1)},
        }
        print(json.dumps(line), flush=True)
    pods.close()
    nodes.close()
    if dist is not None:
        dist.destroy_process_group()


def _pmc_traffic(state_bytes):
    """HBM bytes per pod-sweep launch from the committed rocprofv3 PMC passes
    (profiles/pmc_traffic.json, tools/pmc_traffic.py), or None when they were taken on
    another state format (a different kernel)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))
    except (OSError, ValueError):
        return None
    if d.get("state_bytes_per_object") != state_bytes:
        return None
    return d.get("hbm_bytes_per_launch")


if __name__ == "__main__":
    main()
