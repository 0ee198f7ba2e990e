"""Diagnostic (tools only): time the fused-format load of the 100M-pod C2 engine twice in one
process, so a kernel trace shows whether dw_fold_kernel's long first dispatch is the kernel or
the state upload it follows."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kwok_amd import workload as W  # noqa: E402
from kwok_amd.host.compiler import HarnessSpec, KindProgram  # noqa: E402
from kwok_amd.host.engine import Engine, Ingest  # noqa: E402
from kwok_amd.host.stages import load_stage_files  # noqa: E402

n_nodes = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
pvars, pidx = W.c2_pod_variants(0, n_nodes * 100, seed=0x6B776F6B, job_frac=0.1)
prog = KindProgram(load_stage_files(*W.stage_paths(W.POD_GENERAL + W.POD_CHAOS)), HarnessSpec())
prog.explore(pvars)
ing = Ingest(prog)
hot, dels, rec, cls = ing.variant_columns(pvars, pidx)
eng = Engine(prog, capacity=len(pidx), max_records=max(1, len(ing.records)) + 16)
eng.load_stages()
eng.set_harness(True)
for i in range(3):
    t = time.perf_counter()
    eng.load(hot, dels, rec, cls, ing.record_array())
    eng.sync()
    print(f"load {i}: {time.perf_counter() - t:.3f} s", flush=True)
eng.close()
