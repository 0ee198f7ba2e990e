"""Would a HIP graph shorten the N = 8 shard step?  Times the pod engine's kwk_step_n at the shard
size (125k nodes / 12.5M pods, 2-byte hand-back, folded) launched directly against the same
10-step sequence captured once on the engine's stream (hipStreamBeginCapture / EndCapture) and
replayed as one graph.  The replays repeat the captured steps' clock and step indices, so the
device state does not advance like a run's — a timing probe of the launch path only (no results
are checked).  Pods only: the node engine's stream is not captured.

    python tools/graph_probe.py [--nodes 125000] [--steps 10] [--reps 30]
"""
from __future__ import annotations

import argparse
import ctypes as C
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
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    import bench
    hip = C.CDLL("libamdhip64.so")
    pods, nodes, _ = bench.build_engines(0, a.nodes, 100, 0, 0x6B776F6B, 0.1)
    nodes.close()
    dt, seed = 10**9, 0x6B776F6B
    k = 0
    for _ in range(3):  # warm-up (allocates the fold buffers before any capture)
        pods.step_n(a.steps, bench.NOW0 + k * dt, dt, seed, k, "packed16")
        k += a.steps
    pods.sync()
    direct = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        pods.step_n(a.steps, bench.NOW0 + k * dt, dt, seed, k, "packed16")
        pods.sync()
        direct.append((time.perf_counter() - t0) / a.steps * 1e6)
        k += a.steps
    s = C.c_void_p(pods.stream_handle())
    graph, exe = C.c_void_p(), C.c_void_p()
    assert hip.hipStreamBeginCapture(s, 2) == 0  # hipStreamCaptureModeRelaxed
    pods.step_n(a.steps, bench.NOW0 + k * dt, dt, seed, k, "packed16")
    assert hip.hipStreamEndCapture(s, C.byref(graph)) == 0
    n_nodes = C.c_size_t(0)
    hip.hipGraphGetNodes(graph, None, C.byref(n_nodes))
    assert hip.hipGraphInstantiate(C.byref(exe), graph, None, None, C.c_size_t(0)) == 0
    for _ in range(3):
        assert hip.hipGraphLaunch(exe, s) == 0
    pods.sync()
    replay = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        assert hip.hipGraphLaunch(exe, s) == 0
        pods.sync()
        replay.append((time.perf_counter() - t0) / a.steps * 1e6)
    hip.hipGraphExecDestroy(exe)
    hip.hipGraphDestroy(graph)
    direct.sort()
    replay.sort()
    print(json.dumps({"nodes": a.nodes, "steps_per_call": a.steps, "graph_nodes": n_nodes.value,
                      "direct_us_per_step_median": round(direct[len(direct) // 2], 2),
                      "graph_us_per_step_median": round(replay[len(replay) // 2], 2),
                      "direct_us_per_step_min": round(direct[0], 2), "graph_us_per_step_min": round(replay[0], 2)}))
    pods.close()


if __name__ == "__main__":
    main()
