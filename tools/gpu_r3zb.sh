# C5 pod sweep: two id passes per loop step (working tree) against the committed engine, alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3zb}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread -k "c1_mini" > $O/p1.log 2>&1 || { tail -40 $O/p1.log; exit 1; }
tail -1 $O/p1.log
timeout -k 10 700 python -u tools/variants.py run id8b1 id8b4 id8b1 id8b4 id8b1 id8b4 id8b1 id8b4 --c5 --steps 30 > $O/v_c5.jsonl 2> $O/v.err || { tail -30 $O/v.err; exit 1; }
python -c "
import json
for l in open('$O/v_c5.jsonl'):
    d=json.loads(l); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'])"
echo "gpu_r3zb $T done"
