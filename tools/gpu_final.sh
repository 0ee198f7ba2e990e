# The round's evidence: the driver's bench command, a kernel trace of the same command (timed
# launches summarised), PMC traffic of the C2 working set.  Usage: bash tools/gpu_final.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-final}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail -30 $O/prof_bench.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_hbm -o run -- python3 $R/bench.py --hbm-only --hbm-steps 4 --hbm-warmup 12 > $O/pmc_fetch_hbm.log 2>&1 || { tail -20 $O/pmc_fetch_hbm.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_hbm -o run -- python3 $R/bench.py --hbm-only --hbm-steps 4 --hbm-warmup 12 > $O/pmc_write_hbm.log 2>&1 || { tail -20 $O/pmc_write_hbm.log; exit 1; }
echo "gpu_final $T done"
