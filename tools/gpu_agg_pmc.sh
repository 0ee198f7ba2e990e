# PMC passes over the isolated reporting-interval kernels.  Usage: bash tools/gpu_agg_pmc.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-aggpmc}; O=$R/gpurun_out/$T
mkdir -p $O && cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/agg_bench.py --reps 4 > $O/agg.json 2> $O/agg.err || { tail -20 $O/agg.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU -d $O/pmc_sq -o run -- python3 $R/tools/agg_bench.py --reps 4 > $O/pmc_sq.log 2>&1 || { tail -20 $O/pmc_sq.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM -d $O/pmc_lds -o run -- python3 $R/tools/agg_bench.py --reps 4 > $O/pmc_lds.log 2>&1 || { tail -20 $O/pmc_lds.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -- python3 $R/tools/agg_bench.py --reps 4 > $O/pmc_fetch.log 2>&1 || { tail -20 $O/pmc_fetch.log; exit 1; }
echo "agg pmc $T done"
