import sys, numpy as np
sys.path.insert(0, "/root/repo")
import bench
pods, nodes, _ = bench.build_engines(0, 40000, 100, 0, 0x6B776F6B, 0.1, mix="general")
n = pods.capacity
prev = None
for k in range(16):
    pods.step(bench.NOW0 + k * 500 * 10**6, 0x6B776F6B, k)
    pods.fired_compact()
    hot, _ = pods.read()
    st = hot["sched"] & 0xFF
    pend = st != 0xFF
    alive = (hot["sched"] & (1 << 8)) != 0
    if prev is not None:
        ph, pp = prev
        due_w = np.sum(pend & ((hot["due"] != ph["due"]) | ~pp))
        chg = np.sum((hot["pred"] != ph["pred"]) | (hot["sched"] != ph["sched"]))
        # lines: 16 dues per 128 B, 32 words per 128 B
        dl = np.zeros(n, bool); dl[pend & ((hot["due"] != ph["due"]) | ~pp)] = True
        due_lines = dl[: n // 16 * 16].reshape(-1, 16).any(1).mean()
        cl = np.zeros(n, bool); cl[(hot["pred"] != ph["pred"]) | (hot["sched"] != ph["sched"])] = True
        st_lines = cl[: n // 32 * 32].reshape(-1, 32).any(1).mean()
        pl = pp[: n // 16 * 16].reshape(-1, 16).any(1).mean()
        print(f"step {k}: pending {pend.mean():.3f} (due-read lines {pl:.3f}) due writes {due_w/n:.3f} (lines {due_lines:.3f}) changed words {chg/n:.3f} (lines {st_lines:.3f}) fired {pods.stats()['fired']}")
    prev = (hot.copy(), pend.copy())
pods.close(); nodes.close()
