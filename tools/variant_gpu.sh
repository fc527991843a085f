#!/bin/bash
# GPU check of a library variant (lib/ablate/librsp_$V.so): the -m gpu suite, stage times, bench.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
export RSP_LIB="$ROOT/radar-signal-process_amd/lib/ablate/librsp_$V.so"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:-} > gpurun_out/pytest_$V.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_$V.log
[ $rc -eq 0 ] || [ "${IGNORE_TESTS:-0}" = 1 ] || exit $rc
NS="${NS:-64 256}" timeout -k 10 120 python tools/stage_times.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/bench_$V.log 2>&1 || exit $?
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], {k: v['avg_us'] for k, v in r.get('kernels', {}).items()})" gpurun_out/bench_$V.log
