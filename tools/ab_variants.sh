#!/bin/bash
# A/B of library variants (tools/build_variant.sh NAME FLAGS): stage times + 2 bench runs each.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS}; do
  export RSP_LIB="$ROOT/radar-signal-process_amd/lib/ablate/librsp_$v.so"
  echo "== $v"
  NS="${NS:-64}" timeout -k 10 120 python tools/stage_times.py 2>&1 | grep -v amdgpu.ids || exit 1
  for i in 1 2; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 2 --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/bench_$v.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], {k: v['avg_us'] for k, v in r.get('kernels', {}).items()})" gpurun_out/bench_$v.log
  done
done
