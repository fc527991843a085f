#!/bin/bash
# Bench sweep on the GPU box: each argument is one quoted set of bench.py flags; prints the
# value and the single-pipeline per-kernel times of each (env: STEPS, SKIP_TESTS).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-1}" != "1" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 240 python bench.py --steps ${STEPS:-10} --warmup 2 --cpu-seconds 0 $args > gpurun_out/sweep_$i.log 2>&1 \
    || { echo "bench '$args' rc=$?"; tail -3 gpurun_out/sweep_$i.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], '|', d['value'], {k: v['avg_us'] for k, v in r.get('kernels', {}).items()})" gpurun_out/sweep_$i.log "$args"
done
