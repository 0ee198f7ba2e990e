# Final round-3 build: all GPU tests, the driver's bench, kernel trace of the driver's bench command.
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3y}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "
import json;d=json.loads(open('$O/bench.json').read());r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_us'],r['frac'],r['traffic'],r['line_frac']);h=d['hbm_working_set'];print(h['kernel'],h['avg_launch_us'],h['frac'],h['line_frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail -30 $O/prof_bench.err; exit 1; }
cd $R && python tools/rocpd_summary.py stats $(find $O/prof -name '*.db' | head -1) $O/kernel_stats.csv && cut -c1-150 $O/kernel_stats.csv | head -14
echo "gpu_r3y $T done"
