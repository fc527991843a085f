#!/bin/bash
# One GPU session: parity tests, short bench, rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; a crash/timeout (not a plain test failure) ends the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
if [ "${SKIP_PYTEST:-0}" != "1" ]; then
  timeout -k 10 ${PYTEST_LIMIT:-900} python -m pytest tests -m gpu -q --timeout 300 -rf ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
  if fatal $rc; then exit $rc; fi
fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds ${CPU_SECONDS:-5} ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${PROFILE:-1}" = "1" ]; then
  rm -rf "$ROOT/gpurun_out/prof"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --cpu-seconds 0 --no-profile ${BENCH_ARGS:-} > "$ROOT/gpurun_out/prof.log" 2>&1)
  rc=$?; echo "rocprof rc=$rc"; tail -3 "$ROOT/gpurun_out/prof.log"
  find "$ROOT/gpurun_out/prof" -name "*stats*" | head
fi
if [ "${PMC:-0}" = "1" ]; then
  bash "$ROOT/tools/pmc.sh"
fi
