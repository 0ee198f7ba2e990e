# C2 word sweep: deferred-store batches (base: 4 passes) against HEAD and 2 / 1 pass batches.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r3k}
mkdir -p $O && cd $R
timeout -k 10 900 python tools/variants.py run head base w_batch2 w_batch1 head base > $O/variants.jsonl 2> $O/variants.err || { tail -20 $O/variants.err; exit 1; }
python -c "
import json
for l in open('$O/variants.jsonl'):
    d=json.loads(l); print(d['variant'], d.get('avg_launch_us'), d.get('transitions_per_s'), d.get('frac'))"
echo "gpu_r3k done"
