#!/bin/bash
# GPU check after a kernel change: the whole -m gpu suite, stage times, the c3 bench (3 runs).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
NS="${NS:-64 256}" timeout -k 10 120 python tools/stage_times.py 2>&1 | grep -v amdgpu.ids || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 2 --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/bench_$i.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], {k: v['avg_us'] for k, v in r.get('kernels', {}).items()})" gpurun_out/bench_$i.log
done
