# kernel timeline of a small-shard C5 bench (125k nodes = the N = 8 strong-scaling shard)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/probe_small; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --hbm-nodes 0 --pcie-steps 0 --nodes 125000 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
echo done
