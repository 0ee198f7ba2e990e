# C1-C4 single-GPU runs of bench.py --config.  Usage: bash tools/gpu_configs.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-cfg}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
for c in C1 C2 C4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 50 --warmup 10 > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  tail -1 $O/bench_$c.json | cut -c1-400
done
timeout -k 10 300 python -u bench.py --config C3 --steps 2000 --warmup 100 > $O/bench_C3.json 2> $O/bench_C3.err || { tail -20 $O/bench_C3.err; exit 1; }
tail -1 $O/bench_C3.json | cut -c1-600
