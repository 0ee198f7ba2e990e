# retry GPU tests + the bench at the per-rank shard sizes of N = 8 / 4 / 2 (strong scaling) on one GPU
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/shards; mkdir -p $O && cd $R
timeout -k 10 200 python -u -m pytest tests/test_retry.py -m gpu -q --timeout 120 --timeout-method thread > $O/retry.log 2>&1 || { tail -30 $O/retry.log; exit 1; }
tail -2 $O/retry.log
for n in 125000 250000 500000; do
  timeout -k 10 200 python -u bench.py --nodes $n --no-cpu-baseline --no-pmc --hbm-nodes 0 --pcie-steps 0 --steps 40 --warmup 5 > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$n.json')); print($n, d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
