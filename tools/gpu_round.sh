# GPU tests, the driver's bench command and a kernel-trace profile of it.
# Usage: bash tools/gpu_round.sh <tag> [tests|bench|prof ...]   (default: tests bench prof)
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r2}; shift; O=$R/gpurun_out/$T
STEPS=${*:-tests bench prof}
mkdir -p $O && cd $R
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
        || { tail -40 $O/pytest_gpu.log; exit 1; }
      tail -3 $O/pytest_gpu.log ;;
    bench)
      timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err \
        || { tail -30 $O/bench.err; exit 1; }
      cat $O/bench.json ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err \
        || { tail -30 $O/prof_bench.err; exit 1; }
      cd $R
      find $O/prof -name '*kernel_stats.csv' -exec head -12 {} \; ;;
  esac
done
echo "gpu_round $T done"
