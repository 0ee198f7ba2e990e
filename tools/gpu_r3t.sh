# Round-3 evidence after the fused records: all GPU tests, the driver's bench, C2 PMC traffic per format,
# a kernel trace of the C2 run.  Usage: bash tools/gpu_r3t.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3t}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "
import json;d=json.loads(open('$O/bench.json').read());r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_us'],r['frac'],r['traffic'],r['line_frac']);print(json.dumps(d.get('hbm_working_set'))[:600])"
cd /tmp && export TMPDIR=/tmp
for st in auto u32; do
  H="$R/bench.py --hbm-only --hbm-steps 4 --hbm-warmup 12 --hbm-state $st"
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/c2fetch_$st -o run -- python3 $H > $O/c2fetch_$st.log 2>&1 || { tail -20 $O/c2fetch_$st.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/c2write_$st -o run -- python3 $H > $O/c2write_$st.log 2>&1 || { tail -20 $O/c2write_$st.log; exit 1; }
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/c2trace -o run -- python3 $R/bench.py --hbm-only --hbm-steps 10 --hbm-warmup 12 > $O/c2trace.log 2>&1 || { tail -20 $O/c2trace.log; exit 1; }
cd $R
for st in auto u32; do
  for c in fetch write; do python tools/rocpd_summary.py pmc $(find $O/c2${c}_$st -name '*.db' | head -1) sweepw > $O/c2${c}_$st.txt; done
done
python tools/rocpd_summary.py stats $(find $O/c2trace -name '*.db' | head -1) $O/c2_kernel_stats.csv && cut -c1-150 $O/c2_kernel_stats.csv | head -6
tail -n +1 $O/c2*_*.txt | cut -c1-200
echo "gpu_r3t $T done"
