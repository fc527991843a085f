#!/bin/bash
# A/B of the overlap-save threshold for 8192-point matched filters (c4): the whole-row 8192-point
# transform (2 workgroups per CU) against 3 blocks of 4096 points (4 per CU).  Not bit-identical
# (different fp32 summation), so parity runs through the GPU tests with the variant installed.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in ${VARIANTS:-head ols4k}; do
    RSP_LIB="$ROOT/radar-signal-process_amd/lib/ablate/librsp_$v.so" timeout -k 10 200 python bench.py --config ${CFG:-c4} --steps 20 --cpu-seconds 0 > gpurun_out/ab_${CFG:-c4}_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab_${CFG:-c4}_$v.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], {k: v['avg_us'] for k, v in r.get('kernels', {}).items()})" gpurun_out/ab_${CFG:-c4}_$v.log "${CFG:-c4} $v"
  done
done
