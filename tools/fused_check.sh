#!/bin/bash
# Fused-chain GPU session: its parity tests, then the c3 bench with the fused chain and with
# the chunked pipeline.  Every GPU step has its own limit; a failure ends the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/fused_tests.log 2>&1
rc=$?; echo "fused tests rc=$rc"; tail -15 gpurun_out/fused_tests.log
[ $rc -eq 0 ] || exit $rc
for f in 1 0; do
  timeout -k 10 180 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --fused $f ${BENCH_ARGS:-} \
      > gpurun_out/bench_fused$f.log 2>&1
  rc=$?; echo "bench fused=$f rc=$rc"; tail -2 gpurun_out/bench_fused$f.log | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
done
