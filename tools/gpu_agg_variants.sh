# reporting-interval kernels (tools/agg_bench.py) with tools/variants.py builds, alternating on one box.
# Usage: bash tools/gpu_agg_variants.sh <tag> <variants...>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-aggv}; shift; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
for v in "$@"; do
  timeout -k 10 300 python -u tools/agg_bench.py --reps 10 --lib tools/build/libkwok_engine_$v.so > $O/$v.json 2>>$O/err.log || { tail -20 $O/err.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$v.json')); print('$v', 'usage', d['usage'], 'count', d['count'], 'aggregate', d['aggregate'])"
done
