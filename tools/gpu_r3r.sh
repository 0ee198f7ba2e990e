# Word sweep: tiles per workgroup with the next tile's stream in flight (early / late), same box.
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3r}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 250 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "c2_mini or fused_due or count_phase" > $O/p1.log 2>&1 || { tail -40 $O/p1.log; exit 1; }
tail -2 $O/p1.log
timeout -k 10 700 python -u tools/variants.py run base tpb4 tpb4_late tpb8 tpb8_late --steps 10 > $O/v_dw.jsonl 2> $O/v.err || { tail -30 $O/v.err; exit 1; }
timeout -k 10 500 python -u tools/variants.py run base tpb4 tpb4_late tpb8_late --steps 10 --state u32 > $O/v_u32.jsonl 2>> $O/v.err || { tail -30 $O/v.err; exit 1; }
python -c "
import json
for f in ('$O/v_dw.jsonl','$O/v_u32.jsonl'):
    for l in open(f):
        d=json.loads(l); print(d['variant'], d['state'], d['avg_launch_us'], d['frac'], d['line_frac'], d['transitions_per_step'])"
echo "gpu_r3r $T done"
