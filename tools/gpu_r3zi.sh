# C2 PMC traffic of the final fused word sweep (FETCH_SIZE, WRITE_SIZE passes).  Usage: bash tools/gpu_r3zi.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3zi}; O=$R/gpurun_out/$T
mkdir -p $O && cd /tmp && export TMPDIR=/tmp
H="$R/bench.py --hbm-only --hbm-steps 4 --hbm-warmup 12 --hbm-state auto"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/c2fetch_auto -o run -- python3 $H > $O/c2fetch_auto.log 2>&1 || { tail -20 $O/c2fetch_auto.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/c2write_auto -o run -- python3 $H > $O/c2write_auto.log 2>&1 || { tail -20 $O/c2write_auto.log; exit 1; }
tail -1 $O/c2write_auto.log
echo "gpu_r3zi $T done"
