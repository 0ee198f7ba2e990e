# bench + rocprofv3 kernel-trace stats + FETCH/WRITE/SQ PMC passes of the default build.
# Usage: bash tools/gpu_profile.sh <tag> [extra bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-prof}; shift; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 300 python -u bench.py "$@" > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 200 python -u bench.py --no-harness --no-cpu-baseline > $O/bench_noharness.json 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline "$@" > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -- python3 $R/bench.py --no-cpu-baseline --steps 6 --warmup 4 > $O/pmc_fetch.log 2>&1 || { tail -20 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -- python3 $R/bench.py --no-cpu-baseline --steps 6 --warmup 4 > $O/pmc_write.log 2>&1 || { tail -20 $O/pmc_write.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $O/pmc_sq -o run -- python3 $R/bench.py --no-cpu-baseline --steps 6 --warmup 4 > $O/pmc_sq.log 2>&1 || { tail -20 $O/pmc_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_idle -o run -- python3 $R/bench.py --no-cpu-baseline --no-harness --steps 6 --warmup 4 > $O/pmc_fetch_idle.log 2>&1 || { tail -20 $O/pmc_fetch_idle.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_idle -o run -- python3 $R/bench.py --no-cpu-baseline --no-harness --steps 6 --warmup 4 > $O/pmc_write_idle.log 2>&1 || { tail -20 $O/pmc_write_idle.log; exit 1; }
echo profile done
