#!/bin/bash
# Round 6, session 8: SQ / TCC counters and kernel times of the split persistent dataflow
# (RSP_FLOW2=18) beside the default schedule's (session 7 has the default's).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; O=gpurun_out/r6s7; mkdir -p $O
export TMPDIR=/tmp
n=18
(cd /tmp && RSP_FLOW2=$n timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof_f$n -o run -- python3 $ROOT/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-profile > $ROOT/$O/prof_f$n.log 2>&1) || { echo "rocprof failed"; tail -3 $ROOT/$O/prof_f$n.log; exit 1; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  (cd /tmp && RSP_FLOW2=$n timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $ROOT/$O/pmc_f$n/g$i -o run -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-profile > $ROOT/$O/pmc_f${n}_g$i.log 2>&1)
  rc=$?; echo "flow2=$n pmc group $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
