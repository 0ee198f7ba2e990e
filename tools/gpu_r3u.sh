# C1-C4 bench lines (round 3 build: fused records for C2, kwk_tick_n for C3).  Usage: bash tools/gpu_r3u.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3u}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
for c in C1 C2 C3 C4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 >> $O/configs_C1_C4.jsonl 2> $O/config_$c.err || { tail -30 $O/config_$c.err; exit 1; }
  tail -1 $O/configs_C1_C4.jsonl | cut -c1-400
done
echo "gpu_r3u $T done"
