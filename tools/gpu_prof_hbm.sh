# Kernel-trace + SQ / traffic counters of the C2-mix HBM working-set run (sweepw_kernel).
# Usage: bash tools/gpu_prof_hbm.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-hbm}; O=$R/gpurun_out/$T
mkdir -p $O && cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --hbm-only --hbm-steps 10 > $O/hbm.json 2> $O/hbm.err || { tail -20 $O/hbm.err; exit 1; }
cat $O/hbm.json
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $O/pmc_sq -o run -- python3 $R/bench.py --hbm-only --hbm-steps 4 --hbm-warmup 12 > $O/pmc_sq.log 2>&1 || { tail -20 $O/pmc_sq.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -- python3 $R/bench.py --hbm-only --hbm-steps 4 --hbm-warmup 12 > $O/pmc_fetch.log 2>&1 || { tail -20 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -- python3 $R/bench.py --hbm-only --hbm-steps 4 --hbm-warmup 12 > $O/pmc_write.log 2>&1 || { tail -20 $O/pmc_write.log; exit 1; }
echo "gpu_prof_hbm $T done"
