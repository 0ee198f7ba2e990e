# 2 ranks sharing the box's GPU over gloo: the N>1 bench path (node shards, DeviceReport all-reduce).
# Usage: bash tools/gpu_dist_rehearsal.sh <tag> [nproc]
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-dist}; N=${2:-2}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29561 \
  bench.py --gpus $N --steps 6 --warmup 2 --nodes 200000 --dist-backend gloo --no-cpu-baseline --no-pmc --hbm-nodes 0 \
  --pcie-steps 0 --report-every 3 > $O/bench_dist.json 2> $O/bench_dist.err || { tail -30 $O/bench_dist.err; exit 1; }
cat $O/bench_dist.json
timeout -k 10 200 python -u bench.py --gpus 1 --steps 6 --warmup 2 --nodes 200000 --no-cpu-baseline --no-pmc --hbm-nodes 0 \
  --pcie-steps 0 --report-every 3 > $O/bench_one.json 2> $O/bench_one.err || { tail -30 $O/bench_one.err; exit 1; }
cat $O/bench_one.json
