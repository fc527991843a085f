#!/bin/bash
# Library-variant sweep: one bench per variant (kernel times via HIP events).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out/ablate
for v in ${VARIANTS:-base}; do
  lib="$ROOT/radar-signal-process_amd/lib/librsp.so"; [ $v != base ] && lib="$ROOT/radar-signal-process_amd/lib/ablate/librsp_$v.so"
  for st in ${STREAMS:-1 2}; do
    RSP_LIB=$lib timeout -k 10 200 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --streams $st ${BENCH_ARGS:-} > gpurun_out/ablate/${v}_s$st.json 2>/dev/null || exit $?
  done
  echo "$v done"
done
