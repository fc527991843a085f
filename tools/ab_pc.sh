#!/bin/bash
# A/B of library variants: stage times (PC alone, MTD alone) + the c3 bench, per variant.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out/ab
for v in ${VARIANTS:-base}; do
  lib="$ROOT/radar-signal-process_amd/lib/librsp.so"; [ $v != base ] && lib="$ROOT/radar-signal-process_amd/lib/ablate/librsp_$v.so"
  echo "== $v"
  NS="${NS:-64 256}" RSP_LIB=$lib timeout -k 10 120 python tools/stage_times.py || exit $?
  RSP_LIB=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/ab/$v.json 2>/dev/null || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], {k: v['avg_us'] for k, v in r.get('kernels', {}).items()})" gpurun_out/ab/$v.json
done
