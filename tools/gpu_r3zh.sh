# The fused records' load / read / step test at 4M pods.  Usage: bash tools/gpu_r3zh.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3zh}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "fused_records_load" > $O/p1.log 2>&1 || { tail -40 $O/p1.log; exit 1; }
tail -3 $O/p1.log
echo "gpu_r3zh $T done"
