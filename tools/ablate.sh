#!/bin/bash
# PC-kernel ablation builds + chunk-size sweep; one bench per variant (kernel times via HIP events).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out/ablate
for cfg in "1 16" "2 16" "2 32" "2 64" "3 32" "2 128" "4 32"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --streams $1 --chunk $2 > gpurun_out/ablate/s$1_c$2.json 2>/dev/null || exit $?
  echo "streams $1 chunk $2 done"
done
