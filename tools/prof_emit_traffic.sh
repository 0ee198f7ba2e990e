# FETCH_SIZE / WRITE_SIZE passes over the patch emitter (and the counter list of the box): bash tools/prof_emit_traffic.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5e; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/$O/avail.txt 2>&1 || true
E="$GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 2 --warmup 2 --no-pmc --no-cpu-baseline --hbm-nodes 0 --pcie-steps 0 --emit-steps 3"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/$O/f -o run -- python3 $E > $GRAFT_REPO_ROOT/$O/f.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/$O/w -o run -- python3 $E > $GRAFT_REPO_ROOT/$O/w.log 2>&1
