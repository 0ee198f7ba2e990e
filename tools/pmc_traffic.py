"""HBM traffic per pod-sweep launch from rocprofv3 --pmc passes (bench.py runs them itself as child
processes; this script summarises such a run) -> profiles/pmc_traffic.json.

FETCH_SIZE / WRITE_SIZE (KiB per dispatch) are summed over the PMC dimensions per dispatch.
Only the pod engine's sweep launches count: in the churn run they are the harness
instantiation (`<true`); in the no-harness run pods and nodes share one instantiation, so
the pod launches are the large ones (>= 30 % of the largest steady-state dispatch; the node
sweep moves ~1 % of the pod sweep's bytes).  The first `skip` launches (warm-up transients:
the initial pod-ready of every pod) are dropped.

The guide's x2 FETCH_SIZE correction is stated for 16-B-per-lane reads; it is checked here
on the no-harness run, whose pod launches read exactly the state stream (bytes_per_launch of
that bench run):
    read_factor = bytes_per_launch(idle) / FETCH_SIZE(idle)
    traffic     = FETCH_SIZE(churn) * read_factor + WRITE_SIZE(churn) * 1024
    python tools/pmc_traffic.py gpurun_out/<tag> [profiles/pmc_traffic.json]
"""
import json
import os
import sqlite3
import statistics
import sys
from collections import defaultdict

CHURN = "<true"    # harness instantiation: pods only
IDLE = "<false"    # pods and nodes


def pod_dispatches(db, counter, tag, skip=3, shared=False):
    c = sqlite3.connect(db)
    per = defaultdict(float)
    for disp, name, cn, v in c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection"):
        if "sweep" in name and tag in name and cn == counter:
            per[disp] += float(v)
    vals = [per[d] for d in sorted(per)]
    if not vals:
        raise SystemExit(f"{db}: no {counter} for sweep kernels {tag}")
    if shared:  # pods and nodes in one instantiation: the pod launches are the large ones
        big = max(vals[skip:] or vals)
        vals = [v for v in vals[skip:] if v >= 0.3 * big]
    else:
        vals = vals[skip:]
    return statistics.mean(vals), len(vals)


def main(d, out):
    bench_idle = json.loads(open(os.path.join(d, "bench_noharness.json")).read().strip().splitlines()[-1])
    bench = json.loads(open(os.path.join(d, "bench.json")).read().strip().splitlines()[-1])
    idle_bytes = bench_idle["roofline"]["bytes_per_launch"]
    fi, ni = pod_dispatches(os.path.join(d, "pmc_fetch_idle", "run_results.db"), "FETCH_SIZE", IDLE, shared=True)
    fh, nf = pod_dispatches(os.path.join(d, "pmc_fetch", "run_results.db"), "FETCH_SIZE", CHURN)
    wh, nw = pod_dispatches(os.path.join(d, "pmc_write", "run_results.db"), "WRITE_SIZE", CHURN)
    factor = idle_bytes / (fi * 1024.0)
    res = {"source": d, "kernel": bench["roofline"]["kernel"] + " (churn)",
           "state_bytes_per_object": bench["roofline"].get("state_bytes_per_object"),
           "fetch_kib": fh, "write_kib": wh,
           "read_factor_calibrated_on_idle_sweep": round(factor, 4), "idle_fetch_kib": fi,
           "idle_bytes_per_launch": idle_bytes, "hbm_read_bytes_per_launch": int(fh * 1024 * factor),
           "hbm_write_bytes_per_launch": int(wh * 1024),
           "hbm_bytes_per_launch": int(fh * 1024 * factor + wh * 1024),
           "algorithmic_bytes_per_launch": bench["roofline"]["bytes_per_launch"],
           "dispatches": [ni, nf, nw]}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_traffic.json")
