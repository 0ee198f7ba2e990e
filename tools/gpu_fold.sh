set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/fold; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/fold_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
cat $O/probe.log | tail -4
cd $R && python -c "
import sqlite3,glob
db=glob.glob('$O/prof/**/*.db',recursive=True)[0]
c=sqlite3.connect(db)
for n,s,e in c.execute('select name,start,end from kernels order by start'):
    print('%10.3f ms  %s'%((e-s)/1e6, n[:80]))
"
