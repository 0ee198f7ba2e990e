# SQ counter passes over the C5 pod sweep (sweep8_kernel) and the C2 working set (sweepw_kernel),
# plus any extra GPU test selection given as $2.  Usage: bash tools/gpu_sq8.sh <tag> ["pytest -k expr"]
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-sq8}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
if [ -n "$2" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$2" > $O/pytest_sel.log 2>&1 || { tail -40 $O/pytest_sel.log; exit 1; }
  tail -3 $O/pytest_sel.log
fi
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --pmc-child --steps 6 --warmup 4 --no-cpu-baseline"
H="$R/bench.py --hbm-only --hbm-steps 4 --hbm-warmup 12"
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
S2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
timeout -s KILL 150 rocprofv3 --pmc $S1 -d $O/c5sq1 -o run -- python3 $B > $O/c5sq1.log 2>&1 || { tail -20 $O/c5sq1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc $S2 -d $O/c5sq2 -o run -- python3 $B > $O/c5sq2.log 2>&1 || { tail -20 $O/c5sq2.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc $S1 -d $O/c2sq1 -o run -- python3 $H > $O/c2sq1.log 2>&1 || { tail -20 $O/c2sq1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc $S2 -d $O/c2sq2 -o run -- python3 $H > $O/c2sq2.log 2>&1 || { tail -20 $O/c2sq2.log; exit 1; }
cd $R
for d in c5sq1 c5sq2; do python tools/rocpd_summary.py pmc $(find $O/$d -name '*.db' | head -1) sweep8 ; done > $O/c5_sq.txt
for d in c2sq1 c2sq2; do python tools/rocpd_summary.py pmc $(find $O/$d -name '*.db' | head -1) sweepw ; done > $O/c2_sq.txt
cat $O/c5_sq.txt $O/c2_sq.txt
echo "gpu_sq8 $T done"
