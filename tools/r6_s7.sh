#!/bin/bash
# Round 6, session 7 (A/B experiment): the split persistent dataflow on
# CU-masked streams -- bit-identity and status first, then interleaved c3 benches, then rocprofv3
# kernel times and SQ / TCC counters of both schedules.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; O=gpurun_out/r6s7; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python tools/flow2_check.py > $O/check_default.txt 2>$O/check_default.err || { tail -3 $O/check_default.err; exit 1; }
RSP_FLOW2=18 timeout -k 10 120 python tools/flow2_check.py > $O/check_flow2.txt 2>$O/check_flow2.err || { echo "flow2 check failed"; tail -5 $O/check_flow2.err; exit 1; }
diff $O/check_default.txt $O/check_flow2.txt > /dev/null && echo "flow2 bit-identical" || { echo "flow2 DIFFERS"; diff $O/check_default.txt $O/check_flow2.txt | head; exit 1; }
for rep in 1 2; do
  for n in 0 16 18 20; do
    RSP_FLOW2=$n timeout -k 10 200 python bench.py --steps 20 --warmup 2 --cpu-seconds 0 > $O/bench_f${n}_${rep}.log 2>&1 || { echo "bench $n failed"; tail -3 $O/bench_f${n}_${rep}.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('flow2', sys.argv[2], d['value'], d['ms_per_step'], {k: v['avg_us'] for k, v in r.get('kernels', {}).items()})" $O/bench_f${n}_${rep}.log $n
  done
done
for n in 0 18; do
  (cd /tmp && RSP_FLOW2=$n timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof_f$n -o run -- python3 $ROOT/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-profile > $ROOT/$O/prof_f$n.log 2>&1) || { echo "rocprof $n failed"; exit 1; }
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    (cd /tmp && RSP_FLOW2=$n timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $ROOT/$O/pmc_f$n/g$i -o run -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-profile > $ROOT/$O/pmc_f${n}_g$i.log 2>&1)
    rc=$?; echo "flow2=$n pmc group $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
