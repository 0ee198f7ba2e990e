"""Summaries of rocprofv3 rocpd databases (ROCm 7.2 writes SQLite `run_results.db`).

    python tools/rocpd_summary.py stats <db> [out.csv]        # kernel-trace --stats table
    python tools/rocpd_summary.py pmc <db> [kernel-substring]  # per-kernel counter means per dispatch
    python tools/rocpd_summary.py window <db> <kernel-substring> <first> <count> [stride]
                                                           # mean duration of dispatches first, first+stride, ...
    python tools/rocpd_summary.py timeline <db> <kernel-substring> <nth> <span>
                                                           # every dispatch from the nth launch of a kernel to
                                                           # the (nth + span)th: offsets, durations, gaps

`stats` reproduces rocprofv3's kernel_stats.csv columns (Name, Calls, TotalDurationNs,
AverageNs, Percentage, MinNs, MaxNs).  `pmc` sums each counter over its dimensions
(SE / XCD instances) per dispatch and prints the mean over dispatches of each kernel.
"""
from __future__ import annotations

import csv
import sqlite3
import statistics
import sys
from collections import defaultdict


def stats(db: str, out: str | None = None):
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration from kernels").fetchall()
    by = defaultdict(list)
    for name, d in rows:
        by[name].append(int(d))
    total = sum(sum(v) for v in by.values()) or 1
    table = []
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        table.append([name, len(v), sum(v), round(sum(v) / len(v), 3), round(100.0 * sum(v) / total, 4), min(v), max(v),
                      round(statistics.pstdev(v), 3)])
    hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"]
    f = open(out, "w", newline="") if out else sys.stdout
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(hdr)
    w.writerows(table)
    if out:
        f.close()
    return table


def pmc(db: str, kernel: str = ""):
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection").fetchall()
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> sum
    for disp, name, cn, v in rows:
        if kernel in name:
            per[(name, disp)][cn] += float(v)
    agg = defaultdict(lambda: defaultdict(list))
    for (name, _), cs in per.items():
        for cn, v in cs.items():
            agg[name][cn].append(v)
    out = {}
    for name, cs in agg.items():
        out[name] = {cn: (statistics.mean(v), len(v)) for cn, v in cs.items()}
    return out


def window(db: str, kernel: str, first: int, count: int, stride: int = 1):
    """Durations (ns) of one kernel's dispatches in launch order, [first, first + count) with a
    stride: e.g. the timed launches of bench.py (after its warm-up steps; every EV_EVERY-th one is
    the launch its HIP events sampled)."""
    c = sqlite3.connect(db)
    d = [int(v) for n, v in c.execute("select name, duration from kernels order by start") if kernel in n]
    sel = d[first:first + count:stride]
    return {"kernel": kernel, "dispatches": len(d), "selected": len(sel), "mean_ns": statistics.mean(sel),
            "median_ns": statistics.median(sel), "min_ns": min(sel), "max_ns": max(sel), "durations_ns": sel}


def _short(name: str) -> str:
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("((")[0].split("(")[0][:60] if "(" in n else n[:60]


def timeline(db: str, kernel: str, nth: int, span: int):
    """The dispatches from the nth dispatch of `kernel` to the (nth + span)th, in start order:
    offset from the first start, duration and the idle gap before each (ns) — what one step's
    kernels cost back to back, launch gaps included."""
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, \"end\" from kernels order by start").fetchall()
    hits = [i for i, r in enumerate(rows) if kernel in r[0]]
    i0, i1 = hits[nth], hits[min(nth + span, len(hits) - 1)]
    t0, prev = rows[i0][1], rows[i0][1]
    out = []
    for name, s, e in rows[i0:i1 + 1]:
        out.append((int(s - t0), int(e - s), int(max(0, s - prev)), _short(name)))
        prev = max(prev, e)
    busy = sum(d for _, d, _, _ in out[:-1])
    return out, int(rows[i1][1] - t0), busy


if __name__ == "__main__":
    if sys.argv[1] == "timeline":
        rows, wall, busy = timeline(sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]))
        for off, dur, gap, name in rows:
            print(f"{off / 1e3:9.2f} us  dur {dur / 1e3:8.2f}  gap {gap / 1e3:6.2f}  {name}")
        print(f"wall {wall / 1e3:.2f} us (first to last start), kernels busy {busy / 1e3:.2f} us")
    elif sys.argv[1] == "window":
        import json
        print(json.dumps(window(sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]),
                                int(sys.argv[6]) if len(sys.argv) > 6 else 1)))
    elif sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
    else:
        for name, cs in pmc(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "").items():
            print(name)
            for cn, (m, n) in sorted(cs.items()):
                print(f"  {cn:24s} mean {m:.6g} over {n} dispatches")
