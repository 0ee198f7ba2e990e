# second SQ pass over the C2-mix word sweep (instruction classes, LDS).  Usage: bash tools/gpu_prof_hbm_sq2.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-hbmsq2}; O=$R/gpurun_out/$T
mkdir -p $O && cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_SALU -d $O/pmc_sq2 -o run -- python3 $R/bench.py --hbm-only --hbm-steps 4 --hbm-warmup 12 > $O/pmc_sq2.log 2>&1 || { tail -20 $O/pmc_sq2.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $O/pmc_sq1 -o run -- python3 $R/bench.py --hbm-only --hbm-steps 4 --hbm-warmup 12 > $O/pmc_sq1.log 2>&1 || { tail -20 $O/pmc_sq1.log; exit 1; }
echo "sq2 $T done"
