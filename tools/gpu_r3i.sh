# 1-byte tests, the bench, and the C5 SQ LDS pass.  Usage: bash tools/gpu_r3i.sh <tag> [full]
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3i}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "c1_mini or byte or c5_persistent or empty_after or scale_prop" > $O/p1.log 2>&1 || { tail -40 $O/p1.log; exit 1; }
tail -2 $O/p1.log
if [ "$2" = full ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "
import json;d=json.loads(open('$O/bench.json').read());r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_us'],r['frac'],r['traffic'],r['line_frac']);print(d['detail'])"
cd /tmp && export TMPDIR=/tmp
S2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
timeout -s KILL 150 rocprofv3 --pmc $S2 -d $O/c5sq2 -o run -- python3 $R/bench.py --pmc-child --steps 6 --warmup 4 --no-cpu-baseline > $O/c5sq2.log 2>&1 || { tail -20 $O/c5sq2.log; exit 1; }
cd $R && python tools/rocpd_summary.py pmc $(find $O/c5sq2 -name '*.db' | head -1) sweep8
echo "gpu_r3i $T done"
