# SQ counter passes over the C5 pod sweep (one rocprofv3 --pmc pass each, short bench child).
# Usage: bash tools/gpu_sq16.sh <tag> [extra bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-sq16}; shift; O=$R/gpurun_out/$T
mkdir -p $O && cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --pmc-child --steps 6 --warmup 4 $*"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $O/sq1 -o run -- python3 $B > $O/sq1.log 2>&1 || { tail -20 $O/sq1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -d $O/sq2 -o run -- python3 $B > $O/sq2.log 2>&1 || { tail -20 $O/sq2.log; exit 1; }
cd $R
for d in sq1 sq2; do python tools/rocpd_summary.py pmc $(find $O/$d -name '*.db' | head -1) sweep16 ; done
