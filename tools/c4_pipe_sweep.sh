#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for v in "" "--streams 2 --chunk 16" "--streams 2 --chunk 8" "--streams 1 --chunk 16"; do
  timeout -k 10 200 python bench.py --config c4 --steps 20 --cpu-seconds 0 $v > gpurun_out/c4s.log 2>&1 || { echo "fail $v"; tail -3 gpurun_out/c4s.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/c4s.log').read().strip().splitlines()[-1]); print(repr(sys.argv[1]), d['value'], d['ms_per_step'])" "$v"
done
done
