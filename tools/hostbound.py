"""Is the per-rank step host-bound at the N = 8 shard size?  Times the host side of
kwk_step_n_pair (the call's own duration: launches and events enqueued) against the wall time
of the same steps including the device (call + synchronise), at a given node count.

    python tools/hostbound.py [--nodes 125000] [--steps 10] [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=125_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import bench
    pods, nodes, _ = bench.build_engines(0, a.nodes, 100, 0, 0x6B776F6B, 0.1)
    dt = 10**9
    k = 0
    for _ in range(3):  # warm-up
        pods.step_n_pair(nodes, a.steps, bench.NOW0 + k * dt, dt, 0x6B776F6B, k, "packed16")
        k += a.steps
    pods.sync()
    nodes.sync()
    host, wall = [], []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        pods.step_n_pair(nodes, a.steps, bench.NOW0 + k * dt, dt, 0x6B776F6B, k, "packed16")
        t1 = time.perf_counter()
        pods.sync()
        nodes.sync()
        t2 = time.perf_counter()
        host.append((t1 - t0) / a.steps * 1e6)
        wall.append((t2 - t0) / a.steps * 1e6)
        k += a.steps
    host.sort()
    wall.sort()
    print(json.dumps({"nodes": a.nodes, "steps_per_call": a.steps, "host_us_per_step_median": round(host[len(host) // 2], 2),
                      "wall_us_per_step_median": round(wall[len(wall) // 2], 2),
                      "host_us_per_step_min": round(host[0], 2), "wall_us_per_step_min": round(wall[0], 2)}))
    pods.close()
    nodes.close()


if __name__ == "__main__":
    main()
