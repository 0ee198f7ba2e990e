# Kernel trace of tools/agg_bench.py (the reporting kernels alone, no concurrent engine) at a
# given node count: usage, count, hand-back and kwk_aggregate each timed in isolation.
#   bash tools/agg_trace.sh <tag> [nodes]        outputs under gpurun_out/<tag>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$1; N=${2:-125000}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/agg -o run -- python3 $R/tools/agg_bench.py --nodes $N --reps 10 \
  > $O/agg.json 2> $O/agg.err || { tail -20 $O/agg.err; exit 1; }
cd $R && python tools/rocpd_summary.py stats $(find $O/agg -name '*.db' | head -1) $O/agg_kernel_stats.csv && cut -c1-170 $O/agg_kernel_stats.csv | head -12 && cat $O/agg.json
