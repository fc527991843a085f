#!/bin/bash
# Round 6, session 4: GPU tests (flow removal, range concat), host fresh-output breakdown.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; O=gpurun_out/r6s4; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "concat" > $O/pytest_concat.log 2>&1
rc=$?; echo "concat test rc=$rc"; tail -15 $O/pytest_concat.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for pf in 1 0 1; do
  RSP_PREFAULT=$pf timeout -k 10 120 python tools/host_fresh_probe.py > $O/host_fresh_pf$pf.json 2>&1 || exit 1
  tail -1 $O/host_fresh_pf$pf.json
done
