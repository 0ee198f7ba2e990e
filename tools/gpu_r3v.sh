# Word sweep capped at 5 waves per SIMD, per format, same box.  Usage: bash tools/gpu_r3v.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3v}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 500 python -u tools/variants.py run base lb5 base lb5 --steps 10 > $O/v_dw.jsonl 2> $O/v.err || { tail -30 $O/v.err; exit 1; }
timeout -k 10 500 python -u tools/variants.py run base lb5 --steps 10 --state u32 > $O/v_u32.jsonl 2>> $O/v.err || { tail -30 $O/v.err; exit 1; }
python -c "
import json
for f in ('$O/v_dw.jsonl','$O/v_u32.jsonl'):
    for l in open(f):
        d=json.loads(l); print(d['variant'], d['state'], d['avg_launch_us'], d['frac'], d['line_frac'], d['transitions_per_step'])"
echo "gpu_r3v $T done"
