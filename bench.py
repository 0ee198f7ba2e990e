"""Headline benchmark: stage transitions/sec at 1M nodes / 100M pods (BASELINE.json, config C5).

One *step* = one reconciliation pass of the HIP engines over the whole resident cluster
(pods + nodes): harness churn, match of changed objects, weighted pick + delay/jitter,
firing of due objects, their next-state deltas, and the fired hand-back — each engine's
fired list compacted into one dense device list every step (pods: kwk_fired_compact_packed16, the
1-byte sweep's 2-byte records {offset, stage, flags} grouped by 2048-slot segment; nodes:
kwk_fired_compact_packed, 4-byte records, 27-bit slot | 5-bit stage; --handback packed / rec: 4-byte
records / 8-byte kwk_fired_rec for both; the Go host would DMA it from there).  Every `--report-every` steps (the reporting interval) the cluster
aggregates are computed on the device and summed over all GPUs with one RCCL all-reduce:
per-stage transition counts, the pod / node phase histograms (kwk_count) and the cluster
CPU / memory usage (kwk_usage over the default usage-from-annotation ClusterResourceUsage).
All of it is inside the timed region.  Inputs are resident in HBM before it starts.

    python bench.py [--gpus N --steps K --warmup W]          # N>1 under torch.distributed.run

Multi-GPU (one process per GPU): rank r owns the contiguous node block [r*n/N, (r+1)*n/N) and
every pod on those nodes (no data-path collective).  Default "scaling": "strong" — the C5
cluster (--nodes total) is split over the ranks; --scaling weak keeps --nodes per rank.

The JSON line carries `roofline` for the pod sweep kernel (algorithmic bytes per launch /
its HIP-event duration on the engine's stream; `traffic` = HBM bytes per launch from two
rocprofv3 PMC passes of this same workload run as child processes at N=1, FETCH_SIZE x 2 —
the gfx950 correction of MI355X_MICROARCH.md — + WRITE_SIZE, or null when they cannot run),
`cpu_baseline` (the oracle timed on this host), `pcie_inclusive` (the rate when every step's
fired list is also copied to pinned host memory) and `hbm_working_set` (the C2 stage mix at
100M pods: 4-byte words, 0.4 GB of state, beyond the 256 MiB Infinity Cache).
"""
from __future__ import annotations

import argparse
import json
import os
import sqlite3
import statistics
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "stage transitions/sec (whole node), 1M nodes/100M pods; achieved HBM GB/s"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
NOW0 = 1_700_000_000 * 10**9


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


def node_range(n_nodes, rank, world, weak):
    if weak:  # rank r owns global nodes [r*n, (r+1)*n)
        return n_nodes * rank, n_nodes * (rank + 1)
    from kwok_amd.host.cluster import node_block
    return node_block(n_nodes, world, rank)


def build_engines(node_lo, node_hi, pods_per_node, device, seed, job_frac, wide_state=False, mix="fast", state="auto"):
    """Pod and node engines of one shard.  mix "fast": pod-fast (C1/C5 stage mix, 2-byte words);
    "general": pod-general + pod-chaos (C2 stage mix, 4-byte words)."""
    from kwok_amd import workload as W
    from kwok_amd.host.compiler import HarnessSpec, KindProgram
    from kwok_amd.host.engine import Engine, Ingest
    from kwok_amd.host.stages import load_stage_files

    pod_lo, pod_hi = node_lo * pods_per_node, node_hi * pods_per_node
    if mix == "fast":
        pvars = [W.pod_object("p", "n"), W.pod_object("p", "n", job=True)]
        pidx = shard_pod_variants(pod_lo, pod_hi, seed, job_frac)
        files = W.POD_FAST
    else:
        pvars, pidx = W.c2_pod_variants(pod_lo, pod_hi, seed=seed, job_frac=job_frac)
        files = W.POD_GENERAL + W.POD_CHAOS
    pprog = KindProgram(load_stage_files(*W.stage_paths(files)), HarnessSpec())
    pprog.explore(pvars)
    ping = Ingest(pprog)
    phot, pdel, prec, pcls = ping.variant_columns(pvars, pidx)
    pods = Engine(pprog, capacity=pod_hi - pod_lo, device=device, slot_base=pod_lo, kind_salt=0, wide_state=wide_state,
                  state=state,
                  max_records=max(1, len(ping.records)) + 16)
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
    return pods, nodes, (pvars, pidx)


def configure_usage(pods, pvars, pidx, n_nodes_local, pods_per_node):
    """kwk_usage_config for the shard: the default usage-from-annotation ClusterResourceUsage
    (kustomize/metrics/usage/usage-from-annotation.yaml) evaluated once per variant."""
    from kwok_amd.host.usage import UsageProgram, load_usage_yaml, usage_columns
    path = os.path.join(ROOT, "kwok_amd", "metrics", "usage-from-annotation.yaml")
    up = UsageProgram(*load_usage_yaml(open(path).read()))
    vkeys, cv, mv, mx, ck = usage_columns(up, pvars)
    node_ptr = np.arange(n_nodes_local + 1, dtype=np.uint32) * np.uint32(pods_per_node)
    pods.usage_config(node_ptr, vkeys[pidx], cv, mv, mx, ck)


class Reporter:
    """One reporting interval: this shard's aggregates computed on the device (kwk_aggregate:
    per-stage transitions, phase histograms, cluster usage) and, with several GPUs, summed in
    place by one RCCL all-reduce — no host round trip except the wait before the collective."""

    def __init__(self, pods, nodes, dist, device, collective="torch", local_rank=0):
        from kwok_amd.host.cluster import DeviceReport, phase_masks
        pm = phase_masks(pods.p, values=("Running", "Succeeded", "Failed"))
        nm = phase_masks(nodes.p, values=("Running",))
        masks = [[0] + list(pm.values()), [0] + list(nm.values())]
        names = [["pods"] + [f"pods_{k}" for k in pm], ["nodes"] + [f"nodes_{k}" for k in nm]]
        self.comm = None
        if collective == "native" and dist is not None:
            # libkwok_comm: the torch-free RCCL path a Go host links (include/kwok_comm.h); the
            # 128-byte unique id travels over the existing process group
            from kwok_amd.host.comm import NativeComm, NativeReport, unique_id
            box = [unique_id() if dist.get_rank() == 0 else None]
            dist.broadcast_object_list(box, src=0)
            self.comm = NativeComm(box[0], dist.get_rank(), dist.get_world_size(), local_rank)
            self.report = NativeReport(self.comm, [pods, nodes], masks, names, usage_engine=pods)
        else:
            self.report = DeviceReport([pods, nodes], masks, names, usage_engine=pods, dist=dist, device=device)

    def collect(self, now_ns):
        self.report.collect(now_ns)
        return self.report


SWEEP_NAMES = {1: "sweep16_kernel", 2: "sweep16_fsm_kernel", 3: "sweepw_kernel<4>", 4: "sweepw_kernel<8>",
               5: "sweep8_kernel"}  # kwk_last_sweep kernel codes (KWK_SWEEP_*)
EV_EVERY = 10  # HIP events bracket the pod sweep of every 10th step (2 launches of 20, 5 of the default 50):
               # each marker idles the stream ~4.6-7 us (r4e / r4w traces), ~0.9 us per step at this spacing
               # (2.3 us every 4th step); the kernel trace of the same command cross-checks the mean


# --handback: kwk_step_n's compaction (2-byte records where the sweep has them / 4-byte packed / kwk_fired_rec)
HANDBACK = {"packed16": "packed16", "bits": "bits", "packed": "packed", "rec": True}
HANDBACK_NAMES = {"packed16": "2-byte pod records + 4-byte packed node records",
                  "bits": "per-segment pod fired maps + 2-bit stage codes + 4-byte packed node records",
                  "packed": "packed 4-byte", "rec": "8-byte kwk_fired_rec"}


def run_steps(pods, nodes, seed, dt, k0, k1, ev_base=None, reporter=None, report_every=0, pinned=None,
              handback="packed"):
    """Steps k0..k1-1; ev_base (0): record HIP events (pod stream) around the pod sweep of every
    EV_EVERY-th step (events 2i, 2i+1 of sample i).  Each engine's steps up to the next
    reporting point are enqueued by one native call (kwk_step_n_pair: per step the pod sweep + device
    compaction, then the node engine's, the same work as the per-step calls); the pinned-copy run
    keeps one call per step."""
    assert ev_base in (None, 0)
    if pinned is None:
        last, k = None, k0
        while k < k1:
            j = k - k0
            end = k1
            if reporter is not None and report_every:
                end = min(k1, k0 + (j // report_every + 1) * report_every)
            now = NOW0 + k * dt
            # pods and nodes enqueued step by step in turn (kwk_step_n_pair): the node stream starts
            # with the pod stream instead of after the host has enqueued every pod step
            pods.step_n_pair(nodes, end - k, now, dt, seed, k, HANDBACK[handback], EV_EVERY if ev_base is not None else 0, j)
            k = end
            if reporter is not None and report_every and (k - k0) % report_every == 0:
                last = reporter.collect(NOW0 + (k - 1) * dt)
        return last, 0
    # every step's fired lists to pinned host memory on the fused path: one kwk_step_n_pair call for
    # the steps (pod launches of 4 + 4 + 2 steps, each launch's hand-backs in one launch), every
    # step's list kept in the engines' hand-back rings (kwk_fired_keep) and fetched by step
    # (kwk_fired_fetch_step: waits for that step's compaction only, the copy runs on the copy stream
    # while the later steps sweep); pinned[j] = step j's (pod list, node list, pod segment counts)
    n = k1 - k0
    assert len(pinned) >= n
    pods.step_n_pair(nodes, n, NOW0 + k0 * dt, dt, seed, k0, HANDBACK[handback])
    n_fired_host = 0
    for j in range(n):
        n_fired_host += pods.fetch_step(k0 + j, pinned[j][0], pinned[j][2])["n_records"]
        n_fired_host += nodes.fetch_step(k0 + j, pinned[j][1])["n_records"]
    pods.fetch_wait()
    nodes.fetch_wait()
    return None, n_fired_host


def synth_ipv4(first: int, n: int, lead: int, stride: int) -> np.ndarray:
    """[length][text] rows of distinct-looking IPv4 strings "<lead>.ddd.ddd.ddd" (octets 100-255,
    14 characters) for slots first..first+n: the bench's stand-in for the controller's per-pod
    funcPodIPWith / funcNodeIPWith values (pod_controller.go:563-600)."""
    s = np.arange(first, first + n, dtype=np.int64)
    rows = np.zeros((n, stride), dtype=np.uint8)
    rows[:, 0] = 14
    rows[:, 1:3] = np.frombuffer(str(lead).encode(), dtype=np.uint8)
    for k, div in enumerate((156 * 156, 156, 1)):
        o = 100 + (s // div) % 156
        base = 3 + 4 * k
        rows[:, base] = ord(".")
        rows[:, base + 1] = ord("0") + o // 100
        rows[:, base + 2] = ord("0") + (o // 10) % 10
        rows[:, base + 3] = ord("0") + o % 10
    return rows


def measure_patch_emit(pods, pvars, pidx, args, dt, k0):
    """Device patch emission (include/kwok_emit.h) over the C5 pod lists: per step, the pod sweep
    with packed hand-back, then kwk_emit expands the fired list into the merge-patch bytes of every
    fired pod (pod-ready / pod-complete statusTemplate; pod-delete has none) on the device.  The
    skeletons come from the variant objects (kwk_patch_skeleton / kwk_patch_object_values); the
    per-pod call values (NodeIPWith / PodIPWith) are synthetic IPv4 text (synth_ipv4); guard bits
    start from the variants' status and are carried by the emitter.  Timed with HIP events around
    the three emission kernels; bytes = the patch bytes written."""
    from kwok_amd.host import emit
    from kwok_amd.host.patchtpl import PatchProgram
    pprog = pods.p
    pp = PatchProgram(pprog.stages, {"NodeIPWith": lambda *a: "10.100.100.100", "PodIPWith": lambda *a: "11.100.100.100"})
    vcls = [pprog.class_of(v, register=False) for v in pvars]
    ep = emit.EmitProgram(pprog.stages, pp, dict(zip(vcls, pvars)), len(pprog.class_ids), stride=16)
    wv = []
    for c, v in zip(vcls, pvars):
        acc = 0
        for tid in range(ep.host_tid):
            sk = ep.skel.get((c, tid))
            if sk is not None:
                acc |= int(pp.object_values(tid, [v], sk["text"], sk["calls"], ep.stride)[1][0]) << tid
        wv.append(c | ep.guard_bits(v) << 16 | acc << 32)
    n = pods.capacity
    em = emit.Emitter(pods, n, ep)
    chunk = 1 << 24
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        em.set_rows(a, np.asarray(wv, dtype=np.uint64)[pidx[a:b]], {})
        for c in range(ep.n_columns):
            em.set_column(c, a, synth_ipv4(a, b - a, 10 + c, ep.stride))
    max_skel = max((sum(len(x.encode()) for x in sk["lits"]) + 40 * len(sk["slots"]) for sk in ep.skel.values()),
                   default=1)
    times, nbytes, recs, emitted = [], 0, 0, 0
    for k in range(k0, k0 + args.emit_steps + 1):  # the first step sizes the output buffers (untimed)
        now = NOW0 + k * dt
        pods.step_n(1, now, dt, args.seed, k, "packed")
        em.emit(now, packed=True)
        ni, nb = em.result()
        if ni < 0:
            ni = -ni - 1
            em.reserve(int(ni * 1.5) + 1024, int(max(nb, ni * max_skel) * 1.5) + 4096)
            em.emit(now, packed=True)
            ni, nb = em.result()
            assert ni >= 0, "emission reservation"
        if k == k0:
            continue
        times.append(em.elapsed_ms())
        ni, ne, nb = em.stats()
        nbytes += nb
        recs += ni
        emitted += ne
    em.close()
    t = sum(times) / 1e3
    return {"patches_per_s": round(emitted / t, 1) if t else None, "unit": "merge patches/sec (device bytes)",
            "steps": args.emit_steps, "items_per_step": recs / max(1, len(times)),
            "host_items_per_step": (recs - emitted) / max(1, len(times)),
            "patch_bytes_per_step": nbytes / max(1, len(times)),
            "avg_emit_us": round(statistics.mean(times) * 1e3, 2) if times else None,
            "written_GBps": round(nbytes / t / 1e9, 1) if t else None,
            "write_frac_of_hbm_peak": round(nbytes / t / 1e9 / HBM_PEAK_GBS, 4) if t else None,
            "skeletons": len(ep.skel), "guards": [["/".join(p), "/".join(b)] for p, b in ep.guards],
            "note": "kwk_emit after each pod step (packed list): emit_size + emit_scan + emit_write kernels, "
                    "HIP events; call values synthetic IPv4 text; parity: tests/test_gpu_emit.py"}


def sweep_launches(n_steps, report_every, fuse_max):
    """Pod sweep launches of run_steps' kwk_step_n_pair calls (one per reporting interval): with
    fused steps (KWK_TUNE_FUSE_STEPS) the host takes 4, 2 or 1 steps per launch, the most the
    call's steps left allow (the HIP event samples, every EV_EVERY >= 4 steps, are never two in
    one launch)."""
    sizes = [report_every] * (n_steps // report_every) + ([n_steps % report_every] if n_steps % report_every else []) \
        if report_every else [n_steps]
    launches = 0
    for n in sizes:
        while n:
            m = fuse_max if fuse_max >= 2 else 1
            while m > n:
                m >>= 1
            launches += 1
            n -= m
    return launches


def sweep_bytes(s0, s1):
    return s1["bytes"] - s0["bytes"], s1["line_bytes"] - s0["line_bytes"]


def measure_hbm_working_set(args, device):
    """The C2 stage mix (pod-general + chaos: weighted picks, jitter, value records) at 100M
    pods on one GPU: 8-byte records of a packed word fused with its relative due time = 0.8 GB
    (4-byte words + the 8-byte due column = 1.2 GB before round 3), beyond the 256 MiB
    Infinity Cache, so the roofline fraction is an HBM claim."""
    n_nodes = args.hbm_nodes
    pods, nodes, _ = build_engines(0, n_nodes, args.pods_per_node, device, args.seed, args.job_frac, mix="general",
                                   state=getattr(args, "hbm_state", "auto"))
    try:
        dt = 500 * 10**6
        steps, warm = args.hbm_steps, args.hbm_warmup
        hb = getattr(args, "handback", "packed")
        run_steps(pods, nodes, args.seed, dt, 0, warm, handback=hb)
        pods.sync()
        nodes.sync()
        s0 = pods.stats()
        t0 = time.perf_counter()
        run_steps(pods, nodes, args.seed, dt, warm, warm + steps, ev_base=0, handback=hb)
        pods.sync()
        nodes.sync()
        wall = time.perf_counter() - t0
        s1 = pods.stats()
        from kwok_amd.host import abi
        fused = pods.last_sweep()["kernel"] == abi.SWEEP_WD
        n_ev = (steps + EV_EVERY - 1) // EV_EVERY
        sweep_ms = statistics.mean(pods.event_elapsed_ms(2 * i, 2 * i + 1) for i in range(n_ev))
        b, lb = sweep_bytes(s0, s1)
        us = sweep_ms * 1e3
        ach = b / steps / (us * 1e-6) / 1e9
        return {"workload": f"C2 stage mix at {n_nodes * args.pods_per_node:,} pods ({n_nodes:,} nodes): pod-general + "
                            "pod-chaos, harness churn, 0.5 s per step",
                "kernel": {4: "sweepw_kernel<4-byte words, due column>", 8: "sweepw_kernel<8-byte fused records>"
                           if fused else "sweepw_kernel<8-byte wide words, due column>"}[int(s1["state_bytes"])] + " (pods)",
                "state_bytes_per_object": int(s1["state_bytes"]),
                "state_column_GB": round(n_nodes * args.pods_per_node * int(s1["state_bytes"]) / 1e9, 3),
                "transitions_per_s": round((s1["fired"] - s0["fired"]) / wall, 1),
                "transitions_per_step": (s1["fired"] - s0["fired"]) / steps,
                "avg_launch_us": round(us, 2), "bytes_per_launch": int(b / steps),
                "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                "line_bytes_per_launch": int(lb / steps),
                "line_frac": round(lb / steps / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4), "steps": steps}
    finally:
        pods.close()
        nodes.close()


# ------------------------------------------------------------------ PMC traffic (child passes)
def _pmc_pass(counter, args, outdir):
    """One rocprofv3 --pmc pass over a short run of this workload (a child process: this
    process has not touched the GPU).  -> mean counter value per pod-sweep launch (KiB)."""
    d = os.path.join(outdir, counter.lower())
    cmd = ["rocprofv3", "--pmc", counter, "-d", d, "-o", "run", "--", sys.executable, os.path.abspath(__file__),
           "--pmc-child", "--steps", "8", "--warmup", "4", "--nodes", str(args.nodes),
           "--pods-per-node", str(args.pods_per_node), "--seed", str(args.seed), "--fuse-steps", str(args.fuse_steps)]
    env = dict(os.environ, TMPDIR=outdir)
    r = subprocess.run(cmd, cwd=outdir, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=150)
    if r.returncode != 0:
        raise RuntimeError(f"rocprofv3 {counter}: rc {r.returncode}: {r.stderr.decode(errors='replace')[-400:]}")
    dbs = [os.path.join(dp, f) for dp, _, fs in os.walk(d) for f in fs if f.endswith(".db")]
    if not dbs:
        raise RuntimeError(f"rocprofv3 {counter}: no results database")
    per = {}
    c = sqlite3.connect(dbs[0])
    for disp, name, cn, v in c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection"):
        if "sweep" in name and "<true" in name and cn == counter:  # the pod engine (harness) only
            per[disp] = per.get(disp, 0.0) + float(v)
    # past the warm-up launches: 4 steps, then 8 timed — one launch per step, or with fused steps
    # (KWK_TUNE_FUSE_STEPS 4) one 4-step launch, then two
    f = args.fuse_steps
    fused = f >= 2 and len(per) == sweep_launches(4, 0, f) + sweep_launches(8, 0, f)
    timed = sweep_launches(8, 0, f) if fused else 8
    vals = [per[k] for k in sorted(per)][len(per) - timed:]
    if not vals:
        raise RuntimeError(f"rocprofv3 {counter}: no pod sweep dispatches")
    return statistics.mean(vals), len(vals)


def pmc_traffic(args):
    """HBM bytes per pod-sweep launch: FETCH_SIZE x 2 (gfx950: 128-B requests tallied at 64 B,
    MI355X_MICROARCH.md HBM) + WRITE_SIZE, from two separate PMC passes (FETCH_SIZE and
    WRITE_SIZE do not fit one pass).  Infinity-Cache hits are counted, not excluded."""
    outdir = tempfile.mkdtemp(prefix="kwok_pmc_", dir="/tmp")
    try:
        fetch_kib, nf = _pmc_pass("FETCH_SIZE", args, outdir)
        write_kib, nw = _pmc_pass("WRITE_SIZE", args, outdir)
    except Exception as e:  # noqa: BLE001 - the bench line still prints, with traffic null
        log(f"PMC passes failed: {e}")
        return None, str(e)[:200]
    return {"read": int(fetch_kib * 1024 * 2), "write": int(write_kib * 1024), "launches": [nf, nw]}, None


# ------------------------------------------------------------------ CPU baseline
def cpu_baseline(sample_s: float, seed: int):
    """The oracle (refcpu, C++ restatement of the Go path) timed on this host: per object a
    JSON re-parse (ToJSONStandard), Lifecycle.Match and Stage.Delay, on one thread (the
    reference's single preprocess goroutine, pod_controller.go:150).  Each stage transition
    costs the reference at least one such match, so objects/sec bounds its transitions/sec."""
    import yaml
    from kwok_amd import workload as W
    from oracle import refcpu
    lc = refcpu.Lifecycle([yaml.safe_load(open(p)) for p in W.stage_paths(W.POD_FAST)])
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
    now = NOW0
    lc.match_batch(objs[:2000], now, seed, 0)  # warm-up
    t0 = time.perf_counter()
    n = 0
    reps = 0
    while time.perf_counter() - t0 < sample_s:
        lc.match_batch(objs, now, seed, reps + 1)
        n += len(objs)
        reps += 1
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 1), "unit": "stage transitions/sec (upper bound: matches/sec)", "cores": 1,
            "kind": "port",
            "sample": f"{len(objs)} pod JSON objects x {reps} passes ({dt:.1f} s): JSON re-parse + Match + Delay "
                      f"(pod-fast stages), 1 thread = the reference's preprocess goroutine; CPU "
                      f"{_cpu_model()} ({os.cpu_count()} logical CPUs visible)"}


def cpu_baseline_c2(sample_s: float, seed: int):
    """The reference-faithful matcher (refcpu: JSON re-parse + Match + Delay, 1 thread) on a
    C2-shaped sample with the pod-general + chaos stages (weighted picks, jitter draws, value
    getters): the CPU leg beside the hbm_working_set line."""
    import yaml
    from kwok_amd import workload as W
    from oracle import refcpu
    cl = W.make_cluster("C2", 200, 20000, seed=seed)
    lc = refcpu.Lifecycle([yaml.safe_load(open(p)) for p in cl.pod_stage_files])
    objs = [json.dumps(o, separators=(",", ":")).encode() for o in cl.pods.materialize()]
    lc.match_batch(objs[:2000], NOW0, seed, 0)  # warm-up
    t0, n, reps = time.perf_counter(), 0, 0
    while time.perf_counter() - t0 < sample_s:
        lc.match_batch(objs, NOW0, seed, reps + 1)
        n += len(objs)
        reps += 1
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 1), "unit": "stage transitions/sec (upper bound: matches/sec)", "cores": 1,
            "kind": "port",
            "sample": f"{len(objs)} C2 pod JSON objects x {reps} passes ({dt:.1f} s): JSON re-parse + Match + Delay "
                      f"(pod-general + pod-chaos stages), 1 thread; CPU {_cpu_model()}"}


def cpu_baseline_soa(sample_s: float, seed: int, n_pods: int = 20_000_000):
    """All-cores SoA mode: the compiled pod-fast program stepped over
    integer columns by every host thread this job may use (oracle/refcpu rc_soa_steps), on a
    C5-shaped sample with the bench's churn; transitions per second."""
    from kwok_amd import workload as W
    from kwok_amd.host.compiler import HarnessSpec, KindProgram
    from kwok_amd.host.engine import Ingest
    from kwok_amd.host.stages import load_stage_files
    from oracle import refcpu
    cores = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    pvars = [W.pod_object("p", "n"), W.pod_object("p", "n", job=True)]
    prog = KindProgram(load_stage_files(*W.stage_paths(W.POD_FAST)), HarnessSpec())
    prog.explore(pvars)
    hot, _, _, cls = Ingest(prog).variant_columns(pvars, shard_pod_variants(0, n_pods, seed, 0.1))
    pred = np.ascontiguousarray(hot["pred"])
    sched = np.ascontiguousarray((hot["sched"] & ~np.uint32(0xFFFF0000)) | (cls.astype(np.uint32) << np.uint32(16)))
    due = np.zeros(n_pods, dtype=np.int64)
    table, deltas, harness = prog.table(), prog.delta_array(), prog.harness_struct()
    refcpu.soa_steps(table, deltas, harness, pred, sched, due, NOW0, 10**9, 3, seed, cores)  # warm-up: first matches
    steps, fired, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < sample_s:
        fired += refcpu.soa_steps(table, deltas, harness, pred, sched, due, NOW0 + (3 + steps) * 10**9, 10**9, 4, seed,
                                  cores)
        steps += 4
    dt = time.perf_counter() - t0
    return {"value": round(fired / dt, 1), "unit": "stage transitions/sec", "cores": cores, "kind": "port",
            "sample": f"{n_pods:,} C5-shaped pods x {steps} steps ({dt:.1f} s): the compiled pod-fast program over SoA "
                      f"columns (harness churn, match, pick, delay, fire, delta), {cores} threads; CPU {_cpu_model()}"}


def cpu_baseline_c3(sample_s: float, seed: int):
    """The reference-faithful matcher (refcpu: JSON re-parse + Match + Delay, 1 thread) over node
    objects with node-initialize + node-heartbeat (the C3 stage set), half of them Ready (the
    heartbeat matches, its jitter drawn), half fresh (node-initialize)."""
    import yaml
    from kwok_amd import workload as W
    from oracle import refcpu
    lc = refcpu.Lifecycle([yaml.safe_load(open(p)) for p in W.stage_paths(W.NODE_FAST + W.NODE_HEARTBEAT)])
    objs = []
    for i in range(20000):
        o = W.node_object(f"node-{i}")
        if i % 2:
            o["status"]["phase"] = "Running"
            o["status"]["conditions"] = [{"type": "Ready", "status": "True"}]
        objs.append(json.dumps(o, separators=(",", ":")).encode())
    lc.match_batch(objs[:2000], NOW0, seed, 0)
    t0, n, reps = time.perf_counter(), 0, 0
    while time.perf_counter() - t0 < sample_s:
        lc.match_batch(objs, NOW0, seed, reps + 1)
        n += len(objs)
        reps += 1
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 1), "unit": "node transitions/sec (upper bound: matches/sec)", "cores": 1,
            "kind": "port",
            "sample": f"{len(objs)} node JSON objects x {reps} passes ({dt:.1f} s): JSON re-parse + Match + Delay "
                      f"(node-initialize + node-heartbeat), 1 thread; CPU {_cpu_model()}"}


def cpu_baseline_c4(sample_s: float, seed: int):
    """The oracle's usage restatement (oracle/usage_ref: getResourceUsage + the
    usage-from-annotation expression + the Quantity parse, per container, 1 thread) over a C4
    sample: container usage evaluations per second, as a scrape would evaluate them."""
    import yaml
    from kwok_amd import workload as W
    from oracle import usage_ref
    docs = [d for d in yaml.safe_load_all(open(os.path.join(ROOT, "kwok_amd", "metrics", "usage-from-annotation.yaml")))
            if d]
    pods = W.make_cluster("C4", 100, 5000, seed=seed).pods.materialize()
    t0, n, reps = time.perf_counter(), 0, 0
    while time.perf_counter() - t0 < sample_s:
        for p in pods:
            for c in p["spec"]["containers"]:
                usage_ref.container_usage(docs, p, c["name"], "cpu")
                usage_ref.container_usage(docs, p, c["name"], "memory")
                n += 1
        reps += 1
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 1), "unit": "container usage evaluations/sec", "cores": 1, "kind": "port",
            "sample": f"{len(pods)} C4 pods x {reps} passes ({dt:.1f} s): cpu + memory usage per container "
                      f"(ResourceUsage lookup, usage-from-annotation, Quantity parse), 1 thread; CPU {_cpu_model()}"}


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
    ap.add_argument("--nodes", type=int, default=1_000_000, help="nodes in total (strong) or per GPU (weak)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="strong")
    ap.add_argument("--config", choices=("C1", "C2", "C3", "C4", "C5"), default="C5",
                    help="BASELINE.json configuration; C5 is the headline line, C1-C4 run on one GPU")
    ap.add_argument("--pods-per-node", type=int, default=100)
    ap.add_argument("--job-frac", type=float, default=0.1)
    ap.add_argument("--seed", type=int, default=0x6B776F6B)
    ap.add_argument("--dt-ms", type=int, default=1000, help="simulated time per step")
    ap.add_argument("--report-every", type=int, default=10, help="steps per reporting interval (aggregates + RCCL)")
    ap.add_argument("--cpu-sample-s", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC child passes (traffic null)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--hbm-nodes", type=int, default=1_000_000, help="nodes of the C2-mix HBM working-set run (0: off)")
    ap.add_argument("--hbm-state", default="auto", choices=("auto", "u32", "wide"),
                    help="pod state format of the C2-mix run (auto: the fused 8-byte records)")
    ap.add_argument("--hbm-steps", type=int, default=10)
    ap.add_argument("--hbm-only", action="store_true", help="diagnostic: only the C2-mix HBM working-set run")
    ap.add_argument("--hbm-warmup", type=int, default=12)
    ap.add_argument("--pcie-steps", type=int, default=10)
    ap.add_argument("--metrics-pods", type=int, default=0,
                    help="diagnostic: only the Metric-CR evaluation leg at this many pods (100 per node; C4 shape, "
                         "metrics-resource.yaml), e.g. 100000000 for the single-GPU C5 size")
    ap.add_argument("--emit-steps", type=int, default=5, help="device patch emission steps after the timed run (0: off)")
    ap.add_argument("--no-harness", action="store_true", help="diagnostic: no churn (steady state is an idle sweep)")
    ap.add_argument("--wide-state", action="store_true", help="diagnostic: force the 8-byte device state format")
    ap.add_argument("--tune-q16", type=int, default=0, help="diagnostic: the 2-byte sweep's q (KWK_TUNE_SWEEP16) for the "
                    "pod engine (0: default)")
    ap.add_argument("--tune-fsm-kernel", type=int, default=-1,
                    help="diagnostic: the table-only kernel field of KWK_TUNE_SWEEP16 for the pod engine (-1: default)")
    ap.add_argument("--tune-priority", type=int, default=1,
                    help="1 (default): the pod engine's stream at the device's greatest priority, the node engine's at "
                         "the least (the node step fills in around the pod path: sweep 49.1-49.6 -> 48.3-48.5 us, r4zg; round 6: the PCIe-inclusive leg 3.9-4.0e10 vs 2.1-2.7e10 with 0, "
                         "profiles/r6/r6bg_r6bh_priority_ab.txt); 0: both default")
    ap.add_argument("--fuse-steps", type=int, default=4, choices=(0, 1, 2, 4),
                    help="KWK_TUNE_FUSE_STEPS for the pod engine: up to 4 (default) or 2 steps per 1-byte sweep "
                         "launch, 0 / 1 one step per launch")
    ap.add_argument("--tune-compact-small", type=int, default=-1,
                    help="diagnostic: KWK_TUNE_COMPACT_SMALL for the pod engine (-1: default)")
    ap.add_argument("--tail-handback", type=int, default=-1, choices=(-1, 0, 1),
                    help="diagnostic: KWK_TUNE_TAIL_HANDBACK for both engines (-1: default, 1)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL over xGMI); gloo to rehearse ranks sharing a GPU")
    ap.add_argument("--pcie-handback", choices=("bits", "packed16", "packed", "rec"), default="bits",
                    help="the PCIe-inclusive leg's hand-back format (default: the fewest bytes per transition)")
    ap.add_argument("--handback", choices=("packed16", "bits", "packed", "rec"), default="packed16",
                    help="fired hand-back per step: 2-byte records where the sweep has them (kwk_fired_compact_packed16: "
                         "the 1-byte sweep's {offset, stage, flags} + records per segment; other engines 4-byte), "
                         "packed 4-byte records (kwk_fired_compact_packed, 27-bit slot | 5-bit stage) or 8-byte "
                         "kwk_fired_rec (kwk_fired_compact)")
    ap.add_argument("--collective", choices=("torch", "native"), default="torch",
                    help="aggregate all-reduce: torch.distributed (default) or libkwok_comm (RCCL, no torch; N > 1)")
    args = ap.parse_args()

    if args.config != "C5":
        from kwok_amd import build as kbuild
        from kwok_amd import configs
        if not os.path.exists(kbuild.OUT):
            kbuild.build()
        r = configs.run(args.config, args.steps, args.warmup, args.seed)
        if args.config == "C4":  # the Metric CR on the same cluster size
            r["metric_cr"] = configs.run_metrics(10_000, 1_000_000, scrapes=10, warmup=3, seed=args.seed)
        roof = r.pop("roofline", None)
        cpu = None
        if not args.no_cpu_baseline:
            cpu = {"C1": lambda: cpu_baseline(args.cpu_sample_s / 2, args.seed),
                   "C2": lambda: cpu_baseline_c2(args.cpu_sample_s / 2, args.seed),
                   "C3": lambda: cpu_baseline_c3(args.cpu_sample_s / 2, args.seed),
                   "C4": lambda: cpu_baseline_c4(args.cpu_sample_s / 2, args.seed)}[args.config]()
        line = {"metric": r.pop("metric"), "value": round(r.pop("value"), 1), "n_gpus": 1, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(r.pop("ms_per_step"), 4), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None,
                "dtype": ({1: "u8", 2: "u16", 4: "u32", 8: "u32x2"}.get(r.get("state_bytes_per_object"), "u32") + "/i64"
                          if args.config != "C4" else "f64"),
                "data": "synthetic (seeded kwokctl-shaped objects), cache-resident working set",
                "config": {"workload": r.pop("workload")}, "roofline": roof, "cpu_baseline": cpu, "detail": r}
        print(json.dumps(line), flush=True)
        return

    if args.metrics_pods:
        from kwok_amd import build as kbuild
        from kwok_amd import configs
        if not os.path.exists(kbuild.OUT):
            kbuild.build()
        n = args.metrics_pods
        print(json.dumps(configs.run_metrics(max(1, n // args.pods_per_node), n, scrapes=5, warmup=2, seed=args.seed,
                                             sample_every=9973 if n > 10_000_000 else 97, copy=n <= 10_000_000)),
              flush=True)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:  # ranks beyond the visible GPUs share them (a rehearsal with --dist-backend gloo)
        import torch
        local_rank %= max(1, torch.cuda.device_count())
    weak = args.scaling == "weak"
    if args.hbm_only:
        from kwok_amd import build as kbuild
        if not os.path.exists(kbuild.OUT):
            kbuild.build()
        print(json.dumps(measure_hbm_working_set(args, local_rank)), flush=True)
        return

    # PMC child passes first, while this process has not touched the GPU (N=1 only)
    traffic, pmc_err = None, "not collected (N>1, --no-pmc or --no-harness)"
    if world == 1 and not args.pmc_child and not args.no_pmc and not args.no_harness:
        log("PMC passes (FETCH_SIZE, WRITE_SIZE) as child processes")
        traffic, pmc_err = pmc_traffic(args)

    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group(args.dist_backend)

    from kwok_amd import build as kbuild
    if rank == 0 and not os.path.exists(kbuild.OUT):
        kbuild.build()

    t_setup = time.perf_counter()
    nlo, nhi = node_range(args.nodes, rank, world, weak)
    log(f"rank {rank}: nodes [{nlo}, {nhi}), pods [{nlo * args.pods_per_node}, {nhi * args.pods_per_node})")
    pods, nodes, (pvars, pidx) = build_engines(nlo, nhi, args.pods_per_node, local_rank, args.seed, args.job_frac,
                                               wide_state=args.wide_state)
    configure_usage(pods, pvars, pidx, nhi - nlo, args.pods_per_node)
    setup_s = time.perf_counter() - t_setup
    if args.no_harness:
        pods.set_harness(False)
    if args.tune_q16 or args.tune_fsm_kernel >= 0:
        from kwok_amd.host import abi
        pods.set_tuning(abi.TUNE_SWEEP16, abi.sweep16_shape(q=args.tune_q16 or 4,
                                                            kernel=2 if args.tune_fsm_kernel < 0 else args.tune_fsm_kernel))
    if args.tune_priority:
        from kwok_amd.host import abi
        pods.set_tuning(abi.TUNE_STREAM_PRIORITY, 1)
        nodes.set_tuning(abi.TUNE_STREAM_PRIORITY, 2)
    from kwok_amd.host import abi
    pods.set_tuning(abi.TUNE_FUSE_STEPS, args.fuse_steps)
    if args.tune_compact_small >= 0:
        from kwok_amd.host import abi
        pods.set_tuning(abi.TUNE_COMPACT_SMALL, args.tune_compact_small)
    if args.tail_handback >= 0:
        for e in (pods, nodes):
            e.set_tuning(abi.TUNE_TAIL_HANDBACK, args.tail_handback)
    dt = args.dt_ms * 10**6
    reporter = Reporter(pods, nodes, dist, f"cuda:{local_rank}" if dist is not None else None, args.collective, local_rank)
    report_every = 0 if args.pmc_child else args.report_every

    log(f"setup {setup_s:.1f} s; warmup {args.warmup} steps")
    run_steps(pods, nodes, args.seed, dt, 0, args.warmup, handback=args.handback)
    if report_every and args.warmup:
        # the warm-up covers one reporting interval too: its one-time work (the aggregate and count
        # buffers' allocation, the masks' upload, occupancy queries, the communicator's first
        # collective) stays out of the timed region like the steps' own
        reporter.collect(NOW0 + (args.warmup - 1) * dt)
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
    # HIP events (each idles the stream ~5 us) bracket sampled pod sweeps inside the timed region
    # at N = 1 (the roofline line); with several ranks they are sampled after it (below), so the
    # scaling runs time the steps alone
    agg, _ = run_steps(pods, nodes, args.seed, dt, args.warmup, args.warmup + args.steps,
                       ev_base=0 if world == 1 else None, reporter=reporter, report_every=report_every,
                       handback=args.handback)
    pods.sync()
    nodes.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    agg_dict = agg.result().as_dict() if agg is not None else None  # the last interval's all-reduced aggregates
    s1p, s1n = pods.stats(), nodes.stats()
    pod_kernel = pods.last_sweep()
    pod_n_stages = len(pods.p.stages)
    n_ev = (args.steps + EV_EVERY - 1) // EV_EVERY
    if world > 1:  # sampled after the timed region (the same steps continued)
        k0 = args.warmup + args.steps
        run_steps(pods, nodes, args.seed, dt, k0, k0 + args.steps, ev_base=0, handback=args.handback)
        pods.sync()
        nodes.sync()
    sweep_ms = [pods.event_elapsed_ms(2 * i, 2 * i + 1) for i in range(n_ev)]

    fired = (s1p["fired"] - s0p["fired"]) + (s1n["fired"] - s0n["fired"])
    pbytes, plines = sweep_bytes(s0p, s1p)
    per_stage = {k: s1p["fired_per_stage"][k] - s0p["fired_per_stage"][k] for k in s1p["fired_per_stage"]}
    per_stage.update({k: s1n["fired_per_stage"][k] - s0n["fired_per_stage"][k] for k in s1n["fired_per_stage"]})

    total_fired, max_s = float(fired), elapsed
    if dist is not None:
        import torch
        t = torch.tensor([float(fired)], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(t)  # RCCL over xGMI
        tm = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        total_fired, max_s = t.item(), tm.item()

    if args.pmc_child:
        pods.close()
        nodes.close()
        return

    # the bytes of one sampled launch (the first of a reporting interval: fused_first steps): one more
    # such launch after the timed region, alone between two stats reads (the timed launches share the
    # stats counters; their average over the 4-, 2- and 1-step launches would understate it)
    fused_first = 1
    if pod_kernel["kernel"] == abi.SWEEP_8:
        fused_first = args.fuse_steps if args.fuse_steps >= 2 and len(pods.p.stages) <= 4 else 1
        while fused_first > max(1, report_every or args.steps):
            fused_first >>= 1
    k0 = args.warmup + args.steps
    sa = pods.stats()
    pods.step_n_pair(nodes, fused_first, NOW0 + k0 * dt, dt, args.seed, k0, HANDBACK[args.handback])
    pods.sync()
    nodes.sync()
    first_bytes, first_lines = sweep_bytes(sa, pods.stats())

    # PCIe-inclusive rate: the same steps with every fired record copied to pinned host memory
    pcie = None
    if args.pcie_steps > 0 and world == 1:
        from kwok_amd.host.engine import PinnedBuffer
        pod_list = {"bits": 2, "packed16": 2, "packed": 4, "rec": 8}[args.pcie_handback] * pods.capacity + 64
        node_list = (8 if args.pcie_handback == "rec" else 4) * nodes.capacity + 64
        pin = [tuple(PinnedBuffer(n) for n in (pod_list, node_list, 4 * (pods.capacity // 512 + 64)))
               for _ in range(args.pcie_steps)]
        pods.fired_keep(args.pcie_steps)
        nodes.fired_keep(args.pcie_steps)
        k0 = args.warmup + args.steps
        # one untimed call first: the copy streams, events and ring slots are created at the first use
        run_steps(pods, nodes, args.seed, dt, k0, k0 + args.pcie_steps, pinned=pin, handback=args.pcie_handback)
        k0 += args.pcie_steps
        pods.sync()
        nodes.sync()
        s2p, s2n = pods.stats(), nodes.stats()
        t1 = time.perf_counter()
        _, n_host = run_steps(pods, nodes, args.seed, dt, k0, k0 + args.pcie_steps, pinned=pin,
                              handback=args.pcie_handback)
        wall = time.perf_counter() - t1
        s3p, s3n = pods.stats(), nodes.stats()
        nf = (s3p["fired"] - s2p["fired"]) + (s3n["fired"] - s2n["fired"])
        assert n_host == nf, (n_host, nf)
        pcie = {"value": round(nf / wall, 1), "unit": "stage transitions/sec", "steps": args.pcie_steps,
                "fired_records_to_host_per_step": nf / args.pcie_steps, "ms_per_step": round(wall / args.pcie_steps * 1e3, 4),
                "n_host_equals_fired": True,
                "note": "one kwk_step_n_pair call on the fused path (pod launches of up to 4 steps), then every "
                        "step's fired lists copied into kwk_alloc_host buffers by kwk_fired_fetch_step from the "
                        "engines' hand-back rings (each copy overlaps the later steps): " + {
                    "packed16": "pods' 2-byte records (2 B per transition + 4 B per 2048-slot segment), nodes' "
                                "4-byte packed records",
                    "bits": "pods' byte-sparse fired maps + 2-bit stage codes (kwk_fired_compact_bits, ~1.1 B per "
                            "transition at 10 % firing), nodes' 4-byte packed records",
                    "packed": "4-byte packed records",
                    "rec": "kwk_fired_rec, 8 B per transition"}[args.pcie_handback]}
        pods.fired_keep(0)
        nodes.fired_keep(0)
        for x in pin:
            for p in x:
                p.close()
        k_after = k0 + args.pcie_steps
    else:
        k_after = args.warmup + args.steps
    patch_emit = None
    if args.emit_steps > 0 and world == 1:
        log("device patch emission run")
        patch_emit = measure_patch_emit(pods, pvars, pidx, args, dt, k_after)
    del pidx
    if reporter.comm is not None:
        reporter.comm.close()
    pods.close()
    nodes.close()

    hbm = None
    if rank == 0 and world == 1 and args.hbm_nodes > 0 and not args.no_harness:
        log("HBM working-set run: C2 stage mix at 100M pods")
        hbm = measure_hbm_working_set(args, local_rank)
        if not args.no_cpu_baseline:
            hbm["cpu_baseline"] = cpu_baseline_c2(args.cpu_sample_s / 2, args.seed)

    if rank == 0:
        value = total_fired / max_s
        pod_kernel_s = statistics.mean(sweep_ms) / 1e3
        # the engine fuses the 1-byte pod sweep when its program allows (pod-fast: <= 4 stages, no delayed
        # stage) — decided from the engine, not from the last launch's steps (a 1-step tail launch)
        fuse_max = (args.fuse_steps if (args.fuse_steps >= 2 and int(s1p["state_bytes"]) == 1 and pod_n_stages <= 4)
                    else 1)
        launches = sweep_launches(args.steps, report_every, fuse_max)
        spl = args.steps / launches  # steps per pod sweep launch (mean)
        achieved = first_bytes / pod_kernel_s / 1e9  # the sampled launches' bytes / their duration
        sb = int(s1p["state_bytes"])
        tr = None if traffic is None else traffic["read"] + traffic["write"]
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": tr,
                "traffic_note": (f"rocprofv3 PMC child passes of this workload ({traffic['launches']} pod-sweep launches): "
                                 f"FETCH_SIZE x 2 = {traffic['read']} B read + WRITE_SIZE = {traffic['write']} B written "
                                 "per launch" if traffic else f"null: {pmc_err}"),
                "kernel": SWEEP_NAMES.get(pod_kernel["kernel"], "?") + (" persistent" if pod_kernel["persistent"] else "")
                          + " (pods)",
                "bytes_per_launch": int(first_bytes), "state_bytes_per_object": sb,
                "steps_per_launch": fused_first, "launches": launches,
                "mean_bytes_per_launch": int(pbytes / launches), "mean_steps_per_launch": round(spl, 3),
                "launch_note": "avg_launch_us = the sampled launches (the first of each reporting interval: "
                               f"{fused_first} step(s)); bytes_per_launch = the bytes of one such launch, counted "
                               "alone after the timed region (mean_bytes_per_launch: the timed region's bytes over "
                               "all its launches of every size)",
                "avg_launch_us": round(pod_kernel_s * 1e6, 2),
                # the same count with state writes as the whole 128-byte lines the sweep stores
                "line_bytes_per_launch": int(first_lines),
                "line_frac": round(first_lines / pod_kernel_s / 1e9 / HBM_PEAK_GBS, 4)}
        if tr:
            roof["traffic_GBps"] = round(tr / pod_kernel_s / 1e9, 1)
        cpu = None
        log(f"timed {args.steps} steps in {max_s:.3f} s")
        cpu_soa = None
        if not args.no_cpu_baseline and world == 1:  # the CPU leg runs on rank 0 at N=1 only
            cpu = cpu_baseline(args.cpu_sample_s, args.seed)
            cpu_soa = cpu_baseline_soa(args.cpu_sample_s / 2, args.seed)
        total_nodes = args.nodes * world if weak else args.nodes
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "stage transitions/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(max_s / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
            "dtype": {1: "u8", 2: "u16", 4: "u32", 8: "u32x2"}[sb] + "/i64",
            "data": "synthetic (seeded kwokctl-shaped pods/nodes; pod-fast + node-fast/heartbeat stages)",
            "config": {"workload": f"C5: {total_nodes:,} nodes / {total_nodes * args.pods_per_node:,} pods in total "
                                   f"over {world} GPU(s), pod-fast + node-initialize/heartbeat, harness churn "
                                   "(Succeeded -> delete -> re-create), 10% Job-owned; per step: sweep + fired "
                                   f"hand-back (device compaction into {HANDBACK_NAMES[args.handback]}"
                                   f" records); every {args.report_every} steps: phase "
                                   "histograms + cluster usage + per-stage counts all-reduced over RCCL",
                       "nodes": total_nodes, "pods": total_nodes * args.pods_per_node,
                       "nodes_per_gpu": nhi - nlo, "parallelism": f"node-shard{world}", "sim_dt_ms": args.dt_ms},
            "roofline": roof,
            "cpu_baseline": cpu,
            "cpu_baseline_soa": cpu_soa,
            "pcie_inclusive": pcie,
            "patch_emit": patch_emit,
            "hbm_working_set": hbm,
            "aggregates": agg_dict,
            "detail": {"transitions_per_step": total_fired / args.steps, "per_stage_rank0": per_stage,
                       "pod_sweep_us_mean": round(statistics.mean(sweep_ms) * 1e3, 2),
                       "pod_sweep_us_median": round(statistics.median(sweep_ms) * 1e3, 2),
                       "pod_sweep_launches_timed": len(sweep_ms),
                       "pod_sweep_events": "inside the timed region" if world == 1 else
                                           "after the timed region (the same steps continued)",
                       "setup_s": round(setup_s, 1)},
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
