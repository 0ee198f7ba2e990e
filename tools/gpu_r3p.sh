# C2 fused-record variants vs the split-due words on one box.  Usage: bash tools/gpu_r3p.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3p}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 600 python -u tools/variants.py run base dw_q4 w_nophase2 dw_q4_nophase2 --steps 10 > $O/variants_dw.jsonl 2> $O/variants_dw.err || { tail -30 $O/variants_dw.err; exit 1; }
timeout -k 10 200 python -u tools/variants.py run base --steps 10 --state u32 > $O/variants_u32.jsonl 2>> $O/variants_dw.err || { tail -30 $O/variants_dw.err; exit 1; }
python -c "
import json
for f in ('$O/variants_dw.jsonl','$O/variants_u32.jsonl'):
    for l in open(f):
        d=json.loads(l); print(d['variant'], d['state'], d['avg_launch_us'], d['frac'], d['line_frac'], d['transitions_per_step'])"
echo "gpu_r3p $T done"
