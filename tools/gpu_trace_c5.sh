# Kernel trace of the C5 step alone (no C2 working set, no PCIe leg): per-step kernel composition.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-c5trace}
mkdir -p $O && cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --hbm-nodes 0 --pcie-steps 0 > $O/prof_bench.json 2> $O/prof_bench.err || { tail -30 $O/prof_bench.err; exit 1; }
cd $R && python tools/rocpd_summary.py stats $(find $O/prof -name '*.db' | head -1) $O/kernel_stats.csv && cut -c1-160 $O/kernel_stats.csv | head -20
echo "trace done"
