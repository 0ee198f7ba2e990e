# C5 pod sweep: sweep8 with a shared invalid-id row (6 workgroups per CU fit in LDS) and a VGPR cap.
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3x}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 700 python -u tools/variants.py run base s8_inv s8_lb6 base s8_inv s8_lb6 --c5 --steps 20 > $O/v_c5.jsonl 2> $O/v.err || { tail -30 $O/v.err; exit 1; }
python -c "
import json
for l in open('$O/v_c5.jsonl'):
    d=json.loads(l); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'])"
echo "gpu_r3x $T done"
