# 2-byte sweep A/B on one box: parity subset, then C5 bench lines alternating the pod engine's
# KWK_TUNE_FSM_KERNEL (0 = general sweep16_kernel, 1 / 2 = table-only kernel, prefetch depth).
# Usage: bash tools/gpu_ab16.sh <tag> [variants...]
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-ab16}; O=$R/gpurun_out/$T
shift; V=${@:-0 2 1 0 2 1}
mkdir -p $O && cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_scale_properties.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -k "pod_fast or sweep16 or node_fast or empty" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
i=0
for v in $V; do
  i=$((i+1))
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --hbm-nodes 0 --pcie-steps 0 \
    --tune-fsm-kernel $v > $O/b${i}_$v.json 2>>$O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b${i}_$v.json')); print('fsm_kernel', $v, d['value'], 'sweep us mean/median', d['detail']['pod_sweep_us_mean'], d['detail']['pod_sweep_us_median'], 'ms/step', d['ms_per_step'])"
done
