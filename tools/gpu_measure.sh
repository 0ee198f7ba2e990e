set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r1a
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r1a/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r1a/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r1a/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/r1a/bench.json 2> gpurun_out/r1a/bench.err || { cat gpurun_out/r1a/bench.err; exit 1; }
cat gpurun_out/r1a/bench.json
timeout -k 10 200 python -u bench.py --no-harness --no-cpu-baseline > gpurun_out/r1a/bench_noharness.json 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r1a/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/r1a/prof_bench.log 2>&1 || { tail -20 $R/gpurun_out/r1a/prof_bench.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/r1a/pmc_fetch -o run -- python3 $R/bench.py --no-cpu-baseline --steps 4 --warmup 2 > $R/gpurun_out/r1a/pmc_fetch.log 2>&1 || { tail -20 $R/gpurun_out/r1a/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/r1a/pmc_write -o run -- python3 $R/bench.py --no-cpu-baseline --steps 4 --warmup 2 > $R/gpurun_out/r1a/pmc_write.log 2>&1 || { tail -20 $R/gpurun_out/r1a/pmc_write.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $R/gpurun_out/r1a/pmc_sq -o run -- python3 $R/bench.py --no-cpu-baseline --steps 4 --warmup 2 > $R/gpurun_out/r1a/pmc_sq.log 2>&1 || { tail -20 $R/gpurun_out/r1a/pmc_sq.log; exit 1; }
find $R/gpurun_out/r1a -name '*.csv' | head -50
