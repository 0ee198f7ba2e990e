# The word-sweep tile loop against the oracle.  Usage: bash tools/gpu_r3za.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3za}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread -k "tile_loop or c2_mini or fused_due" > $O/p1.log 2>&1 || { tail -40 $O/p1.log; exit 1; }
grep -E "PASSED|FAILED" $O/p1.log | cut -c1-150; tail -1 $O/p1.log
echo "gpu_r3za $T done"
