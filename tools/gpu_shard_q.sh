# the bench at the per-rank shard sizes of N = 8 / 4 (strong scaling) with each 2-byte tile shape
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/shardq; mkdir -p $O && cd $R
for n in 125000 250000; do for q in 1 2 4; do
  timeout -k 10 200 python -u bench.py --nodes $n --tune-q16 $q --no-cpu-baseline --no-pmc --hbm-nodes 0 --pcie-steps 0 --steps 40 --warmup 5 > $O/b_${n}_$q.json 2> $O/b_${n}_$q.err || { tail -20 $O/b_${n}_$q.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_${n}_$q.json')); print($n, $q, d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done; done
