set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/probe1; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-pmc --no-cpu-baseline --hbm-nodes 0 --pcie-steps 0 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 $f | head -20
