# SQ passes of the C5 pod sweep and the C2 word-sweep cost isolation (record / deletion-column loads).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r3h}
mkdir -p $O && cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --pmc-child --steps 6 --warmup 4 --no-cpu-baseline"
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
S2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
timeout -s KILL 150 rocprofv3 --pmc $S1 -d $O/c5sq1 -o run -- python3 $B > $O/c5sq1.log 2>&1 || { tail -20 $O/c5sq1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc $S2 -d $O/c5sq2 -o run -- python3 $B > $O/c5sq2.log 2>&1 || { tail -20 $O/c5sq2.log; exit 1; }
cd $R
for d in c5sq1 c5sq2; do python tools/rocpd_summary.py pmc $(find $O/$d -name '*.db' | head -1) sweep8 ; done > $O/c5_sq.txt
cat $O/c5_sq.txt
timeout -k 10 600 python tools/variants.py run base w_norec w_nodel w_nophase2 > $O/variants.jsonl 2> $O/variants.err || { tail -20 $O/variants.err; exit 1; }
python -c "
import json
for l in open('$O/variants.jsonl'):
    d=json.loads(l); print(d['variant'], d.get('avg_launch_us'), d.get('transitions_per_s'))"
echo "gpu_r3h done"
