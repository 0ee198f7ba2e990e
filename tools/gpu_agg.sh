# isolated reporting-interval kernels + kernel-trace stats.  Usage: bash tools/gpu_agg.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-agg}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 300 python -u tools/agg_bench.py > $O/agg.json 2> $O/agg.err || { tail -20 $O/agg.err; exit 1; }
cat $O/agg.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/agg_bench.py > $O/prof_agg.json 2> $O/prof_agg.err || { tail -20 $O/prof_agg.err; exit 1; }
echo agg done
