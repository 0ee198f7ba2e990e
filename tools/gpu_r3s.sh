# Word sweep: the three-kind work list (heavy items with a value record last) against the two-kind one,
# per format, same box; then the GPU tests the word sweep touches.  Usage: bash tools/gpu_r3s.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3s}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "c2_word or c2_mini or fused_due or count_phase or weight_edge or chaos_weights or c2_mix" > $O/p1.log 2>&1 || { tail -40 $O/p1.log; exit 1; }
tail -2 $O/p1.log
timeout -k 10 500 python -u tools/variants.py run base nosort base --steps 10 > $O/v_dw.jsonl 2> $O/v.err || { tail -30 $O/v.err; exit 1; }
timeout -k 10 500 python -u tools/variants.py run base nosort base --steps 10 --state u32 > $O/v_u32.jsonl 2>> $O/v.err || { tail -30 $O/v.err; exit 1; }
python -c "
import json
for f in ('$O/v_dw.jsonl','$O/v_u32.jsonl'):
    for l in open(f):
        d=json.loads(l); print(d['variant'], d['state'], d['avg_launch_us'], d['frac'], d['line_frac'], d['transitions_per_step'])"
echo "gpu_r3s $T done"
