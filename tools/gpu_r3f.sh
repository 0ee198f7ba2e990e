# sweep8 rework: the 1-byte tests first, then every GPU test, then the driver's bench command.
# Usage: bash tools/gpu_r3f.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3f}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "c1_mini or byte or c5_persistent or empty_after" > $O/p1.log 2>&1 || { tail -40 $O/p1.log; exit 1; }
tail -3 $O/p1.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
echo "gpu_r3f $T done"
