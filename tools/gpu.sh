# The one GPU runner (replaces round 1-3's per-call scripts; see profiles/r*/README.md for what
# each call produced).  Runs on the gpurun box from the repo root; every GPU step has its own
# time limit and the steps are chained: the first failing step ends the call.
#
# Usage: bash tools/gpu.sh <tag> <step> [<step> ...]      outputs under gpurun_out/<tag>/
#   tests[=<pytest -k expr>]   GPU test suite (or a selection; '+' between names: any of them)
#   smoke                      __graft_entry__.smoke()
#   bench[=<bench.py args>]    the driver's bench command (default --gpus 1 --steps 20 --warmup 5)
#   prof                       kernel trace + stats of the driver's bench command (kernel_stats.csv)
#   timeline[=<bench args>]    kernel trace of the C5 bench (timed steps only): one reporting interval's dispatches and
#                              gaps (from pod sweep launch TL_N, 2, for TL_SPAN, 3, launches: fused groups 4 + 4 + 2)
#   agg                        the reporting kernels alone at C5 (tools/agg_bench.py) + SQ passes over usage
#   configs                    bench.py --config C1..C4 lines (configs_C1_C4.jsonl)
#   c2prof                     C2 working set: kernel trace + FETCH_SIZE / WRITE_SIZE passes
#   sq                         SQ counter passes over the C5 pod sweep and the C2 word sweep
#   shards                     the bench at the per-rank shard sizes of N = 8 / 4 / 2 (strong scaling:
#                              125k / 250k / 500k nodes) + a kernel trace of the 125k-node shard
#   dist                       2 ranks sharing the GPU over gloo (the N > 1 bench path) vs one rank
#   ab=<so>                    same-box A/B of the bench: in-tree engine vs tools/ab/<so>, alternating x2
#   abshard=<so>               the same A/B at the N = 8 shard size (125k nodes / 12.5M pods)
#   abemit=<so>                same-box A/B of the patch emitter: in-tree libkwok_emit.so vs tools/ab/<so>
#   emitprof                   the patch emitter alone: kernel trace + SQ / TA counter passes over its write kernel
#   variants=<a,b,...>         tools/variants.py build + run of those variants (cost-isolation builds, built on the box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; shift; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
TRACE() { cd /tmp && export TMPDIR=/tmp; }
B1="--gpus 1 --steps 20 --warmup 5"
for step in "$@"; do
  name=${step%%=*}; arg=""; [ "$name" != "$step" ] && arg=${step#*=}
  echo "== $name $arg"
  case $name in
    tests)
      K=(); [ -n "$arg" ] && K=(-k "${arg//+/ or }")  # tests=a+b selects a or b
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
        > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
      tail -2 $O/pytest_gpu.log ;;
    smoke)
      timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 500 python -u bench.py ${arg:-$B1} > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
      python -c "
import json;d=json.loads(open('$O/bench.json').read().splitlines()[-1]);r=d['roofline'];print(d['value'],d['ms_per_step'],r.get('avg_launch_us'),r['frac'],r['traffic'],r.get('line_frac'))
h=d.get('hbm_working_set') or {};print('hbm',h.get('kernel'),h.get('avg_launch_us'),h.get('frac'),h.get('line_frac'));print('pcie',d.get('pcie_inclusive'))" ;;
    prof)
      TRACE
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py $B1 --no-pmc --no-cpu-baseline \
        > $O/prof_bench.json 2> $O/prof_bench.err || { tail -30 $O/prof_bench.err; exit 1; }
      cd $R && python tools/rocpd_summary.py stats $(find $O/prof -name '*.db' | head -1) $O/kernel_stats.csv && cut -c1-150 $O/kernel_stats.csv | head -14 ;;
    timeline)  # kernel trace of the C5 timed steps only; every dispatch of 10 steps with its gap
      TRACE
      timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl -o run -- python3 $R/bench.py $B1 --no-pmc --no-cpu-baseline \
        --hbm-nodes 0 --pcie-steps 0 --emit-steps 0 $arg > $O/tl_bench.json 2> $O/tl_bench.err || { tail -30 $O/tl_bench.err; exit 1; }
      cd $R && python tools/rocpd_summary.py timeline $(find $O/tl -name '*.db' | head -1) sweep8 ${TL_N:-2} ${TL_SPAN:-3} > $O/timeline.txt \
        && cat $O/timeline.txt ;;
    agg)  # the reporting kernels alone at C5 (tools/agg_bench.py) + SQ passes over them
      timeout -k 10 300 python -u tools/agg_bench.py > $O/agg.json 2> $O/agg.err || { tail -30 $O/agg.err; exit 1; }
      cat $O/agg.json
      TRACE
      S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
      S2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
      for p in 1 2; do
        S=S$p
        timeout -s KILL 200 rocprofv3 --pmc ${!S} -d $O/aggsq$p -o run -- python3 $R/tools/agg_bench.py --reps 3 --usage-only > $O/aggsq$p.log 2>&1 || { tail -20 $O/aggsq$p.log; exit 1; }
      done
      cd $R
      for d in aggsq1 aggsq2; do python tools/rocpd_summary.py pmc $(find $O/$d -name '*.db' | head -1) usage_fast; done > $O/agg_sq.txt
      cat $O/agg_sq.txt ;;
    configs)
      for c in C1 C2 C3 C4; do
        timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 >> $O/configs_C1_C4.jsonl 2> $O/config_$c.err || { tail -30 $O/config_$c.err; exit 1; }
        tail -1 $O/configs_C1_C4.jsonl | cut -c1-300
      done ;;
    metrics)
      # the Metric CR at C4 size (bench --config C4's metric_cr) and at 100M pods (--metrics-pods), plus a
      # kernel trace of the 100M leg
      timeout -k 10 400 python -u bench.py --config C4 --steps 20 --warmup 5 > $O/c4_metrics.json 2> $O/c4_metrics.err \
        || { tail -30 $O/c4_metrics.err; exit 1; }
      python -c "import json,sys; d=json.load(open('$O/c4_metrics.json'))['detail']['metric_cr']; print(json.dumps(d)[:900])"
      timeout -k 10 600 python -u bench.py --metrics-pods ${arg:-100000000} > $O/metrics_100m.json 2> $O/metrics_100m.err \
        || { tail -30 $O/metrics_100m.err; exit 1; }
      cut -c1-900 $O/metrics_100m.json
      TRACE
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/metrics_prof -o run -- python -u $R/bench.py \
        --metrics-pods ${arg:-100000000} > $O/metrics_prof.log 2>&1 || { tail -30 $O/metrics_prof.log; exit 1; }
      cd $R && python tools/rocpd_summary.py stats $(find $O/metrics_prof -name '*.db' | head -1) $O/metrics_kernel_stats.csv \
        && cut -c1-150 $O/metrics_kernel_stats.csv | head -12 ;;
    c2prof)
      TRACE
      H="$R/bench.py --hbm-only --hbm-steps 4 --hbm-warmup 12"
      timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/c2fetch -o run -- python3 $H > $O/c2fetch.log 2>&1 || { tail -20 $O/c2fetch.log; exit 1; }
      timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/c2write -o run -- python3 $H > $O/c2write.log 2>&1 || { tail -20 $O/c2write.log; exit 1; }
      timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/c2trace -o run -- python3 $R/bench.py --hbm-only --hbm-steps 10 --hbm-warmup 12 \
        > $O/c2trace.log 2>&1 || { tail -20 $O/c2trace.log; exit 1; }
      cd $R
      for c in fetch write; do python tools/rocpd_summary.py pmc $(find $O/c2$c -name '*.db' | head -1) sweepw > $O/c2$c.txt; done
      python tools/rocpd_summary.py stats $(find $O/c2trace -name '*.db' | head -1) $O/c2_kernel_stats.csv && cut -c1-150 $O/c2_kernel_stats.csv | head -6
      cut -c1-200 $O/c2fetch.txt $O/c2write.txt ;;
    sq)
      TRACE
      B="$R/bench.py --pmc-child --steps 6 --warmup 4 --no-cpu-baseline"
      H="$R/bench.py --hbm-only --hbm-steps 4 --hbm-warmup 12"
      S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
      S2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
      for p in 1 2; do
        S=S$p
        timeout -s KILL 150 rocprofv3 --pmc ${!S} -d $O/c5sq$p -o run -- python3 $B > $O/c5sq$p.log 2>&1 || { tail -20 $O/c5sq$p.log; exit 1; }
        timeout -s KILL 200 rocprofv3 --pmc ${!S} -d $O/c2sq$p -o run -- python3 $H > $O/c2sq$p.log 2>&1 || { tail -20 $O/c2sq$p.log; exit 1; }
      done
      cd $R
      for d in c5sq1 c5sq2; do python tools/rocpd_summary.py pmc $(find $O/$d -name '*.db' | head -1) sweep8; done > $O/c5_sq.txt
      for d in c2sq1 c2sq2; do python tools/rocpd_summary.py pmc $(find $O/$d -name '*.db' | head -1) sweepw; done > $O/c2_sq.txt
      cat $O/c5_sq.txt $O/c2_sq.txt ;;
    emitprof)  # the patch emitter alone: kernel trace (size / scan / write split) + SQ and TA passes over emit_write
      TRACE
      E="$R/bench.py --gpus 1 --steps 2 --warmup 2 --no-pmc --no-cpu-baseline --hbm-nodes 0 --pcie-steps 0 --emit-steps 3"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/emit_trace -o run -- python3 $E > $O/emit_trace.json 2> $O/emit_trace.err \
        || { tail -20 $O/emit_trace.err; exit 1; }
      S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
      S2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
      S3="TA_BUSY_avr TA_FLAT_WRITE_WAVEFRONTS_sum"
      for p in 1 2 3; do
        S=S$p
        timeout -s KILL 150 rocprofv3 --pmc ${!S} -d $O/emsq$p -o run -- python3 $E > $O/emsq$p.log 2>&1 || { tail -20 $O/emsq$p.log; break; }
      done
      cd $R && python tools/rocpd_summary.py stats $(find $O/emit_trace -name '*.db' | head -1) $O/emit_kernel_stats.csv \
        && cut -c1-150 $O/emit_kernel_stats.csv | grep -i emit
      for d in emsq1 emsq2 emsq3; do [ -d $O/$d ] && python tools/rocpd_summary.py pmc $(find $O/$d -name '*.db' | head -1) emit_write; done \
        > $O/emit_sq.txt; cat $O/emit_sq.txt ;;
    shards)
      S="--no-cpu-baseline --no-pmc --hbm-nodes 0 --pcie-steps 0 --steps 40 --warmup 5"
      for n in 125000 250000 500000; do
        timeout -k 10 200 python -u bench.py --nodes $n $S > $O/shard_$n.json 2> $O/shard_$n.err || { tail -20 $O/shard_$n.err; exit 1; }
        python -c "import json; d=json.load(open('$O/shard_$n.json')); print($n, d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
      done
      TRACE
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/shard_prof -o run -- python3 $R/bench.py --nodes 125000 $S \
        > $O/shard_prof.json 2> $O/shard_prof.err || { tail -30 $O/shard_prof.err; exit 1; }
      cd $R && python tools/rocpd_summary.py stats $(find $O/shard_prof -name '*.db' | head -1) $O/shard_kernel_stats.csv \
        && cut -c1-150 $O/shard_kernel_stats.csv | head -14 ;;
    shardtune)  # the 125k-node shard under pod-sweep grid / hand-back tunings: "<label>:<bench args>;..."
      S="--nodes 125000 --no-cpu-baseline --no-pmc --hbm-nodes 0 --pcie-steps 0 --steps 40 --warmup 5"
      IFS=';' read -ra V <<< "${arg:-base:}"
      for i in 1 2; do
        for v in "${V[@]}"; do
          l=${v%%:*}; x=${v#*:}
          timeout -k 10 200 python -u bench.py $S $x > $O/st_${l}_$i.json 2> $O/st_${l}_$i.err || { tail -20 $O/st_${l}_$i.err; exit 1; }
          python -c "import json; d=json.load(open('$O/st_${l}_$i.json')); print('$l', $i, d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
        done
      done ;;
    ab2)  # same-box A/B of C5 bench variants by flags, alternating x2: "<label>:<bench args>;..."
      IFS=';' read -ra V <<< "$arg"
      for i in 1 2; do
        for v in "${V[@]}"; do
          l=${v%%:*}; x=${v#*:}
          timeout -k 10 200 python -u bench.py $B1 --no-pmc --no-cpu-baseline --hbm-nodes 0 --pcie-steps 0 --emit-steps 0 $x \
            > $O/ab_${l}_$i.json 2> $O/ab_${l}_$i.err || { tail -20 $O/ab_${l}_$i.err; exit 1; }
          python -c "import json; d=json.load(open('$O/ab_${l}_$i.json')); print('$l', $i, d['value'], 'ms/step', d['ms_per_step'], 'sweep us', d['detail']['pod_sweep_us_mean'])"
        done
      done ;;
    dist)
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 \
        bench.py --gpus 2 --steps 6 --warmup 2 --nodes 200000 --dist-backend gloo --no-cpu-baseline --no-pmc --hbm-nodes 0 \
        --pcie-steps 0 --report-every 3 > $O/bench_dist.json 2> $O/bench_dist.err || { tail -30 $O/bench_dist.err; exit 1; }
      cut -c1-300 $O/bench_dist.json ;;
    ab)
      cp kwok_amd/lib/libkwok_engine.so $O/cur.so
      for i in 1 2; do
        for v in cur other; do
          if [ $v = other ]; then cp tools/ab/$arg kwok_amd/lib/libkwok_engine.so; else cp $O/cur.so kwok_amd/lib/libkwok_engine.so; fi
          timeout -k 10 200 python -u bench.py $B1 --no-pmc --no-cpu-baseline > $O/${v}_$i.json 2> $O/${v}_$i.err \
            || { cp $O/cur.so kwok_amd/lib/libkwok_engine.so; tail -20 $O/${v}_$i.err; exit 1; }
          python -c "import json; d=json.load(open('$O/${v}_$i.json')); print('$v', $i, d['value'], 'ms/step', d['ms_per_step'], 'sweep us', d['detail']['pod_sweep_us_mean'])"
        done
      done
      cp $O/cur.so kwok_amd/lib/libkwok_engine.so && rm -f $O/cur.so ;;
    abshard)  # same-box A/B at the N = 8 shard size (125k nodes): in-tree engine vs tools/ab/<so>, alternating x2
      cp kwok_amd/lib/libkwok_engine.so $O/cur.so
      S="--nodes 125000 --no-cpu-baseline --no-pmc --hbm-nodes 0 --pcie-steps 0 --emit-steps 0 --steps 40 --warmup 5"
      for i in 1 2; do
        for v in cur other; do
          if [ $v = other ]; then cp tools/ab/$arg kwok_amd/lib/libkwok_engine.so; else cp $O/cur.so kwok_amd/lib/libkwok_engine.so; fi
          timeout -k 10 200 python -u bench.py $S > $O/sh_${v}_$i.json 2> $O/sh_${v}_$i.err \
            || { cp $O/cur.so kwok_amd/lib/libkwok_engine.so; tail -20 $O/sh_${v}_$i.err; exit 1; }
          python -c "import json; d=json.load(open('$O/sh_${v}_$i.json')); print('$v', $i, d['value'], 'ms/step', d['ms_per_step'], 'sweep us', d['detail']['pod_sweep_us_mean'])"
        done
      done
      cp $O/cur.so kwok_amd/lib/libkwok_engine.so && rm -f $O/cur.so ;;
    abusage)  # same-box A/B of the C5 usage kernel alone (tools/agg_bench.py --usage-only): in-tree engine vs tools/ab/<so>
      for i in 1 2; do
        for v in cur other; do
          L=kwok_amd/lib/libkwok_engine.so; [ $v = other ] && L=tools/ab/$arg
          timeout -k 10 200 python -u tools/agg_bench.py --usage-only --reps 10 --lib $L > $O/usage_${v}_$i.json 2> $O/usage_${v}_$i.err \
            || { tail -20 $O/usage_${v}_$i.err; exit 1; }
          echo "$v $i $(cat $O/usage_${v}_$i.json)"
        done
      done ;;
    abemit)  # same-box A/B of the patch emitter: in-tree libkwok_emit.so vs tools/ab/<so>[,<so>...], each
             # variant first checked by tests/test_gpu_emit.py, then alternating x2
      L=kwok_amd/lib/libkwok_emit.so; cp $L $O/cur_emit.so
      for v in ${arg//,/ }; do
        cp tools/ab/$v $L
        timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_emit.py \
          > $O/emit_test_$v.log 2>&1 || { cp $O/cur_emit.so $L; tail -30 $O/emit_test_$v.log; exit 1; }
        echo "$v: $(tail -1 $O/emit_test_$v.log)"
      done
      for i in 1 2; do
        for v in cur ${arg//,/ }; do
          if [ $v = cur ]; then cp $O/cur_emit.so $L; else cp tools/ab/$v $L; fi
          timeout -k 10 200 python -u bench.py --gpus 1 --steps 5 --warmup 3 --no-pmc --no-cpu-baseline --hbm-nodes 0 --pcie-steps 0 \
            --emit-steps 8 > $O/emit_${v}_$i.json 2> $O/emit_${v}_$i.err || { cp $O/cur_emit.so $L; tail -20 $O/emit_${v}_$i.err; exit 1; }
          python -c "import json; e=json.load(open('$O/emit_${v}_$i.json'))['patch_emit']; print('$v', $i, e['patches_per_s'], 'us', e['avg_emit_us'], 'GBps', e['written_GBps'])"
        done
      done
      cp $O/cur_emit.so $L && rm -f $O/cur_emit.so ;;
    emittrace)  # kernel trace of the emitter per variant: in-tree libkwok_emit.so and tools/ab/<so>[,<so>...]
      TRACE
      L=$R/kwok_amd/lib/libkwok_emit.so; cp $L $O/cur_emit.so
      E="$R/bench.py --gpus 1 --steps 2 --warmup 2 --no-pmc --no-cpu-baseline --hbm-nodes 0 --pcie-steps 0 --emit-steps 3"
      for v in cur ${arg//,/ }; do
        if [ $v = cur ]; then cp $O/cur_emit.so $L; else cp $R/tools/ab/$v $L; fi
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/et_$v -o run -- python3 $E > $O/et_$v.json 2> $O/et_$v.err \
          || { cp $O/cur_emit.so $L; tail -20 $O/et_$v.err; exit 1; }
        (cd $R && python tools/rocpd_summary.py stats $(find $O/et_$v -name '*.db' | head -1) $O/et_${v}_stats.csv) > /dev/null \
          && echo "== $v" && grep -i emit $O/et_${v}_stats.csv | cut -c1-160
      done
      cp $O/cur_emit.so $L && rm -f $O/cur_emit.so ;;
    abagg)  # same-box A/B of the reporting kernels alone (tools/agg_bench.py): in-tree engine vs tools/ab/<so>, x2
      for i in 1 2; do
        for v in cur $arg; do
          L=""; [ $v != cur ] && L="--lib tools/ab/$v"
          timeout -k 10 300 python -u tools/agg_bench.py $L > $O/agg_${v}_$i.json 2> $O/agg_${v}_$i.err || { tail -20 $O/agg_${v}_$i.err; exit 1; }
          echo "$v $i $(tail -1 $O/agg_${v}_$i.json | cut -c1-400)"
        done
      done ;;
    variants)
      V=$(echo $arg | tr ',' ' ')
      timeout -k 10 600 python -u tools/variants.py build ${V//--*/} > $O/variants_build.log 2>&1 || { tail -30 $O/variants_build.log; exit 1; }
      timeout -k 10 900 python -u tools/variants.py run $V > $O/variants.jsonl 2> $O/variants.err || { tail -30 $O/variants.err; exit 1; }
      cut -c1-300 $O/variants.jsonl ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
  cd $R
done
echo "gpu.sh $T done"
