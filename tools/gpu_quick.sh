# GPU tests (optionally -k), the isolated aggregate bench and the driver bench.  Usage: bash tools/gpu_quick.sh <tag> [k-expr]
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-quick}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
K=${2:+-k "$2"}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread $K > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u tools/agg_bench.py > $O/agg.json 2> $O/agg.err || { tail -20 $O/agg.err; exit 1; }
cat $O/agg.json
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
