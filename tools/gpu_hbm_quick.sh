# word-sweep parity tests + the C2-mix HBM working-set line.  Usage: bash tools/gpu_hbm_quick.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-hbmq}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "general or chaos or c2 or wide or u32 or formats" > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --hbm-only > $O/hbm.json 2> $O/hbm.err || { tail -20 $O/hbm.err; exit 1; }
cat $O/hbm.json
