# Fused-record (dw) format: its parity tests first, then the full GPU suite, the bench, a C2 kernel trace.
# Usage: bash tools/gpu_r3o.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3o}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "dw or c2_mini or fused_due or c2_word_sweep or c2_mix" > $O/p1.log 2>&1 || { tail -40 $O/p1.log; exit 1; }
tail -2 $O/p1.log
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "
import json;d=json.loads(open('$O/bench.json').read());r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_us'],r['frac'],r['traffic'],r['line_frac']);print(json.dumps(d.get('hbm_working_set')))"
echo "gpu_r3o $T done"
