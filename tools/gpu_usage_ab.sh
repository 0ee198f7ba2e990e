# Same-box A/B of the usage kernel: rocprof kernel stats of bench.py with the in-tree library,
# then with tools/build/libkwok_engine_head.so (git HEAD) in its place.
# Usage: bash tools/gpu_usage_ab.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-uab}; O=$R/gpurun_out/$T
mkdir -p $O && cd /tmp && export TMPDIR=/tmp
for v in cur head; do
  if [ $v = head ]; then cp $R/tools/build/libkwok_engine_head.so $R/kwok_amd/lib/libkwok_engine.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $O/$v.json 2> $O/$v.err \
    || { tail -30 $O/$v.err; exit 1; }
  echo "== $v"; find $O/$v -name '*kernel_stats.csv' -exec grep -h 'usage\|sweep16\|compact' {} \;
done
