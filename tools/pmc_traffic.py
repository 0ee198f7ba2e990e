"""HBM traffic per sweep launch from a tools/gpu_profile.sh run -> profiles/pmc_traffic.json.

FETCH_SIZE / WRITE_SIZE (KiB per dispatch) are summed over the PMC dimensions per dispatch.
The guide's x2 FETCH_SIZE correction is calibrated for 16-B-per-lane reads; the sweep reads
4 or 8 B per lane, so the read counter is calibrated here on the no-harness run, whose
launches read exactly the state stream (bytes_per_launch of that bench run):
    read_factor = bytes_per_launch(idle) / FETCH_SIZE(idle)
    traffic     = FETCH_SIZE(churn) * read_factor + WRITE_SIZE(churn) * 1024
    python tools/pmc_traffic.py gpurun_out/<tag> [profiles/pmc_traffic.json]
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rocpd_summary import pmc  # noqa: E402

KERNEL = "sweep_kernel<true"
IDLE_KERNEL = "sweep_kernel<false"


def mean_of(db, counter, kernel, skip=4):
    import sqlite3
    from collections import defaultdict
    c = sqlite3.connect(db)
    per = defaultdict(float)
    for disp, name, cn, v in c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection"):
        if kernel in name and cn == counter:
            per[disp] += float(v)
    vals = [per[d] for d in sorted(per)][skip:]  # drop warm-up dispatches
    return statistics.mean(vals), len(vals)


def main(d, out):
    bench_idle = json.loads(open(os.path.join(d, "bench_noharness.json")).read().strip().splitlines()[-1])
    idle_bytes = bench_idle["roofline"]["bytes_per_launch"]
    fi, _ = mean_of(os.path.join(d, "pmc_fetch_idle", "run_results.db"), "FETCH_SIZE", IDLE_KERNEL)
    fh, nf = mean_of(os.path.join(d, "pmc_fetch", "run_results.db"), "FETCH_SIZE", KERNEL)
    wh, nw = mean_of(os.path.join(d, "pmc_write", "run_results.db"), "WRITE_SIZE", KERNEL)
    factor = idle_bytes / (fi * 1024.0)
    res = {"source": d, "kernel": "sweep_kernel (pods, churn)", "fetch_kib": fh, "write_kib": wh,
           "read_factor_calibrated_on_idle_sweep": round(factor, 4), "idle_fetch_kib": fi,
           "idle_bytes_per_launch": idle_bytes, "hbm_read_bytes_per_launch": int(fh * 1024 * factor),
           "hbm_write_bytes_per_launch": int(wh * 1024),
           "hbm_bytes_per_launch": int(fh * 1024 * factor + wh * 1024), "dispatches": [nf, nw]}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_traffic.json")
