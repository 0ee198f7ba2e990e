# GPU parity + sweep-variant timing (one gpurun call).  Usage: bash tools/gpu_variants.sh <tag>
# Variant libraries are built beforehand into kwok_amd/lib/variants/ (tools/build_variants.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-var}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
fi
run() {  # name, env assignments...   (BARGS: extra bench args)
  n=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 40 $BARGS > $O/bench_$n.json 2> $O/bench_$n.err || { cat $O/bench_$n.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$n.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$n', '%.4g'%d['value'], r['avg_launch_us'], r['achieved'], r['bytes_per_launch'], r.get('state_bytes_per_object'), 'node_ms', d['detail']['node_kernel_ms_per_step'])"
}
run q2_persist KWOK_SWEEP_Q16=2
for lib in kwok_amd/lib/variants/*.so; do
  [ -e "$lib" ] && run $(basename $lib .so) KWOK_ENGINE_LIB=$R/$lib
done
for lib in kwok_amd/lib/variants/*.so; do
  [ -e "$lib" ] && BARGS=--no-harness run idle_$(basename $lib .so) KWOK_ENGINE_LIB=$R/$lib
done
BARGS=--no-harness run idle_q2_persist KWOK_SWEEP_Q16=2
run q2_persist_again KWOK_SWEEP_Q16=2
echo variants done
