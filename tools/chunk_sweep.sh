#!/bin/bash
# bench.py over chunk sizes x stream counts (kernel times via sampled HIP events).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out/chunks
for c in ${CHUNKS:-2 4 8 16 32}; do
  for st in ${STREAMS:-1 2 3}; do
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --chunk $c --streams $st ${BENCH_ARGS:-} > gpurun_out/chunks/c${c}_s$st.json 2>/dev/null || exit $?
  done
  echo "chunk $c done"
done
