# HIP API + kernel trace of a short C5 run (which host calls sit between the reporting kernels).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-hiptrace}
mkdir -p $O && cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d $O/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --hbm-nodes 0 --pcie-steps 0 > $O/b.json 2> $O/b.err || { tail -30 $O/b.err; exit 1; }
ls -la $O/prof
echo "hiptrace done"
