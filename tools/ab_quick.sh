#!/bin/bash
# A/B of library variants x env settings on c3 and c5: 2 bench runs each (bench line + per-kernel µs).
#   VARIANTS="base x4" ENVS="RSP_FLAG_MEMSET=0 RSP_FLAG_MEMSET=1" CONFIGS="c3 c5" tools/ab_quick.sh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${CONFIGS:-c3}; do
  for v in ${VARIANTS}; do
    for e in ${ENVS:-NONE=0}; do
      export RSP_LIB="$ROOT/radar-signal-process_amd/lib/ablate/librsp_$v.so"
      for i in ${REPS:-1 2}; do
        env "$e" timeout -k 10 200 python bench.py --config $cfg --steps ${STEPS:-20} --warmup 2 --cpu-seconds 0 > gpurun_out/ab_${cfg}_${v}.log 2>&1 || exit $?
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], {k: v['avg_us'] for k, v in r.get('kernels', {}).items()})" gpurun_out/ab_${cfg}_${v}.log "$cfg $v $e"
      done
    done
  done
done
