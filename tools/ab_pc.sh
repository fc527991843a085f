#!/bin/bash
# A/B of library variants (tools/build_variant.sh NAME FLAGS): optional parity subset
# (PYTEST_K), PC alone (tools/pc_bench.py), then the c3 bench (or BENCH_ARGS), per variant.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  lib="$ROOT/radar-signal-process_amd/lib/librsp.so"; [ $v != lib ] && lib="$ROOT/radar-signal-process_amd/lib/ablate/librsp_$v.so"
  echo "== $v"
  if [ -n "${PYTEST_K:-}" ]; then
    RSP_LIB=$lib timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$PYTEST_K" \
      > gpurun_out/ab/pytest_$v.log 2>&1; rc=$?; tail -1 gpurun_out/ab/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
  fi
  RSP_LIB=$lib timeout -k 10 120 python tools/pc_bench.py --cpis ${CPIS:-16 64} --iters 20 ${PC_ARGS:-} 2>&1 | grep -v amdgpu.ids || exit 1
  for i in $(seq ${BENCH_REPS:-1}); do
    RSP_LIB=$lib timeout -k 10 200 python bench.py --steps 10 --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/ab/$v.json 2>/dev/null || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], {k: v['avg_us'] for k, v in r.get('kernels', {}).items()})" gpurun_out/ab/$v.json
  done
done
