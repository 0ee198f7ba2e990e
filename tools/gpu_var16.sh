# C5 pod-sweep cost isolation of the table-only 2-byte sweep (tools/variants.py builds, wrong
# results on purpose).  Usage: bash tools/gpu_var16.sh <tag> <variants...>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-var16}; O=$R/gpurun_out/$T
shift
mkdir -p $O && cd $R
for v in "$@"; do
  timeout -k 10 200 python -u tools/variants.py child $v --c5 --steps 20 > $O/$v.json 2>>$O/err.log || { tail -20 $O/err.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$v.json')); print('$v', d['value'], 'sweep us mean/median', d['detail']['pod_sweep_us_mean'], d['detail']['pod_sweep_us_median'], 'ms/step', d['ms_per_step'])"
done
