# Sweep variants that also need an env switch.  Usage: bash tools/gpu_qvariants.sh <tag> name:lib:ENV=V ...
# (lib "-" = the default build).  Prints tag, transitions/s, us per pod sweep, algorithmic GB/s.
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-qvar}; shift; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
for spec in "$@" ; do
  n=${spec%%:*}; rest=${spec#*:}; lib=${rest%%:*}; ev=${rest#*:}
  L=""; [ "$lib" != "-" ] && L="KWOK_ENGINE_LIB=$R/kwok_amd/lib/variants/libkwok_$lib.so"
  for mode in churn idle; do
    B=""; [ $mode = idle ] && B=--no-harness
    env $L $ev timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 40 $B > $O/${mode}_$n.json 2> $O/${mode}_$n.err || { cat $O/${mode}_$n.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/${mode}_$n.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$mode', '$n', '%.4g'%d['value'], r['avg_launch_us'], r['achieved'])"
  done
done
echo qvariants done
