"""Isolated timing of the reporting-interval kernels at the C5 shard size (100M pods, 1M nodes):
kwk_usage (usage_kernel), kwk_count (count_kernel) and kwk_fired_compact (hand-back), each
launched alone on the pod engine's stream and timed with HIP events on that stream.

    python tools/agg_bench.py [--nodes 1000000] [--reps 10]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def timed(eng, fn, reps):
    out = []
    for r in range(reps):
        eng.event_record(0)
        fn()
        eng.event_record(1)
        eng.sync()
        out.append(eng.event_elapsed_ms(0, 1) * 1e3)
    return {"mean_us": round(statistics.mean(out), 2), "min_us": round(min(out), 2), "reps": reps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--pods-per-node", type=int, default=100)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--lib", default="", help="engine library to load (a tools/variants.py build)")
    ap.add_argument("--usage-only", action="store_true", help="the default usage kernel only (PMC passes)")
    args = ap.parse_args()
    if args.lib:
        from kwok_amd.host import abi
        abi.LIB_PATH = os.path.abspath(args.lib)
    pods, nodes, (pvars, pidx) = bench.build_engines(0, args.nodes, args.pods_per_node, 0, 0x6B776F6B, 0.1)
    bench.configure_usage(pods, pvars, pidx, args.nodes, args.pods_per_node)
    for k in range(6):  # steady-state churn
        pods.step(bench.NOW0 + k * 10**9, 1, k)
    pods.sync()
    from kwok_amd.host.cluster import phase_masks
    pm = [0] + list(phase_masks(pods.p, values=("Running", "Succeeded", "Failed")).values())
    t = [bench.NOW0 + 10**10]
    res = {"pods": args.nodes * args.pods_per_node}

    def usage():
        t[0] += 10**9
        pods.usage(t[0])
    res["usage"] = timed(pods, usage, args.reps)
    if args.usage_only:
        print(json.dumps(res), flush=True)
        pods.close()
        nodes.close()
        return
    res["count"] = timed(pods, lambda: pods.count(pm), args.reps)
    res["fired_compact"] = timed(pods, pods.fired_compact, args.reps)
    res["aggregate"] = timed(pods, lambda: pods.aggregate(pm, t[0], usage=True), args.reps)
    print(json.dumps(res), flush=True)
    pods.close()
    nodes.close()


if __name__ == "__main__":
    main()
