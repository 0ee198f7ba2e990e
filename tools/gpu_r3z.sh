# The bench with the reporting path warmed up, twice; the two-rank bench test.  Usage: bash tools/gpu_r3z.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r3z}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread -k "dist_bench or c5_aggregates" > $O/p1.log 2>&1 || { tail -40 $O/p1.log; exit 1; }
tail -2 $O/p1.log
for i in 1 2; do
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --hbm-nodes 0 > $O/bench$i.json 2> $O/bench$i.err || { tail -30 $O/bench$i.err; exit 1; }
python -c "
import json;d=json.loads(open('$O/bench$i.json').read());r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_us'],r['frac'])"
done
echo "gpu_r3z $T done"
