# Word sweep tiles per workgroup (fused records and 4-byte words), same box.  Usage: bash tools/gpu_r3q.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3q}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 250 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "c2_mini or fused_due" > $O/p1.log 2>&1 || { tail -40 $O/p1.log; exit 1; }
tail -2 $O/p1.log
timeout -k 10 600 python -u tools/variants.py run base tpb2 tpb4 w_nophase2 tpb4_nophase2 --steps 10 > $O/v_dw.jsonl 2> $O/v.err || { tail -30 $O/v.err; exit 1; }
timeout -k 10 400 python -u tools/variants.py run base tpb2 tpb4 --steps 10 --state u32 > $O/v_u32.jsonl 2>> $O/v.err || { tail -30 $O/v.err; exit 1; }
python -c "
import json
for f in ('$O/v_dw.jsonl','$O/v_u32.jsonl'):
    for l in open(f):
        d=json.loads(l); print(d['variant'], d['state'], d['avg_launch_us'], d['frac'], d['line_frac'], d['transitions_per_step'])"
echo "gpu_r3q $T done"
