# Selected + full GPU tests, the driver's bench, a C5-only kernel trace.  Usage: bash tools/gpu_r3l.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3l}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "c1_mini or handback or byte or c5_persistent or aggregate" > $O/p1.log 2>&1 || { tail -40 $O/p1.log; exit 1; }
tail -2 $O/p1.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "
import json;d=json.loads(open('$O/bench.json').read());r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_us'],r['frac'],r['traffic'],r['line_frac']);print(d['detail'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --hbm-nodes 0 --pcie-steps 0 > $O/prof_bench.json 2> $O/prof_bench.err || { tail -30 $O/prof_bench.err; exit 1; }
cd $R && python tools/rocpd_summary.py stats $(find $O/prof -name '*.db' | head -1) $O/kernel_stats.csv && cut -c1-150 $O/kernel_stats.csv | head -12
echo "gpu_r3l $T done"
