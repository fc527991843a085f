#!/bin/bash
# Hardware-counter passes (one rocprofv3 --pmc run per counter group, kernel-trace only).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/pmc"
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS="--steps ${PMC_STEPS:-2} --warmup 1 ${BENCH_ARGS:-}"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE GRBM_COUNT" ${EXTRA_GROUPS:-}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/g$i" -o run -- \
      python3 "$ROOT/bench.py" $ARGS --cpu-seconds 0 --no-profile > "$OUT/g$i.log" 2>&1
  rc=$?; echo "group $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/g$i.log"; exit $rc; fi
done
