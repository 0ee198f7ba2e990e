# Fused word sweep: 5 (default) / 6 waves per SIMD, 8 / 16 tiles per workgroup, same box.
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3w}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 600 python -u tools/variants.py run base lb6 tpb16 base lb6 tpb16 --steps 10 > $O/v_dw.jsonl 2> $O/v.err || { tail -30 $O/v.err; exit 1; }
python -c "
import json
for l in open('$O/v_dw.jsonl'):
    d=json.loads(l); print(d['variant'], d['state'], d['avg_launch_us'], d['frac'], d['line_frac'], d['transitions_per_step'])"
echo "gpu_r3w $T done"
