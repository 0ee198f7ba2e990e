# Round-3 evidence of HEAD: GPU tests, the driver's bench command, a kernel trace of it.
# Usage: bash tools/gpu_r3e.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3e}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail -30 $O/prof_bench.err; exit 1; }
cd $R
find $O/prof -name '*kernel_stats.csv' -exec head -14 {} \;
echo "gpu_r3e $T done"
