#!/bin/bash
# GPU check after a kernel change: the whole -m gpu suite, stage times, the c3 bench.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
NS="${NS:-64 256}" timeout -k 10 120 python tools/stage_times.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || exit $?
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], {k: v['avg_us'] for k, v in r.get('kernels', {}).items()})" gpurun_out/bench.log
