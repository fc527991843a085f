#!/bin/bash
# Round 6, session 9: the new GPU tests (prefaulted new outputs, window stream with range concat).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; O=gpurun_out/r6s9; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_hostpath.py tests/test_gpu_window.py -x -v --timeout 120 --timeout-method thread -k "prefault or concat" > $O/pytest_new.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "PASS|FAIL|Error" $O/pytest_new.log | tail -8; exit $rc
