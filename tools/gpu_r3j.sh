# C5 pod-sweep floors of the 1-byte sweep: the kernel's own read + rewrite stream and read stream.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r3j}
mkdir -p $O && cd $R
timeout -k 10 600 python tools/variants.py run base s8_stream s8_read --c5 --steps 20 > $O/c5_variants.jsonl 2> $O/c5_variants.err || { tail -20 $O/c5_variants.err; exit 1; }
python -c "
import json
for l in open('$O/c5_variants.jsonl'):
    l=l.strip()
    if not l.startswith('{'): continue
    d=json.loads(l); print(d['detail']['pod_sweep_us_mean'], d['detail']['pod_sweep_us_median'], d['roofline']['traffic'] if d.get('roofline') else None, d['ms_per_step'])"
echo "gpu_r3j done"
