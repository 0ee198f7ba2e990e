# Same-box A/B of the driver's bench command: the in-tree library against
# tools/build/libkwok_engine_head.so (git HEAD), alternating.  Usage: bash tools/gpu_bench_ab.sh <tag> [rounds]
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-bab}; N=${2:-2}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
cp kwok_amd/lib/libkwok_engine.so $O/cur.so
for i in $(seq 1 $N); do
  for v in cur head; do
    if [ $v = head ]; then cp tools/build/libkwok_engine_head.so kwok_amd/lib/libkwok_engine.so; else cp $O/cur.so kwok_amd/lib/libkwok_engine.so; fi
    timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $O/${v}_$i.json 2> $O/${v}_$i.err || { tail -20 $O/${v}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${v}_$i.json')); print('$v', $i, d['value'], 'ms/step', d['ms_per_step'], 'sweep us', d['detail']['pod_sweep_us_mean'], d['detail']['pod_sweep_us_median'])"
  done
done
rm -f $O/cur.so
