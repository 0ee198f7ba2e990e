# C5 bench lines (pod sweep timing only) for several argument sets on one box.
# Usage: bash tools/gpu_bench_args.sh <tag> "<args 1>" "<args 2>" ...
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-args}; O=$R/gpurun_out/$T
shift
mkdir -p $O && cd $R
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --hbm-nodes 0 --pcie-steps 0 $a \
    > $O/b$i.json 2>>$O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b$i.json')); print('[$a]', d['value'], 'sweep us mean/median', d['detail']['pod_sweep_us_mean'], d['detail']['pod_sweep_us_median'], 'ms/step', d['ms_per_step'])"
done
