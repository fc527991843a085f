#!/bin/bash
# A/B of library variants (tools/build_variant.sh NAME FLAGS): bitwise output digest per
# variant (tools/lib_digest.py), then bench runs interleaved across variants (REPS rounds,
# default warmup) for each config.
#   VARIANTS="base new" CONFIGS="c3 c5" REPS=2 tools/ab2.sh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${DIGEST:-1}" = 1 ]; then
  for v in ${VARIANTS}; do
    RSP_LIB="$ROOT/radar-signal-process_amd/lib/ablate/librsp_$v.so" timeout -k 10 180 python tools/lib_digest.py > gpurun_out/digest_$v.txt 2>&1 || { echo "digest $v failed"; tail -5 gpurun_out/digest_$v.txt; exit 1; }
    echo "== digest $v"; grep -v "^lib" gpurun_out/digest_$v.txt | grep -v amdgpu.ids
  done
fi
for cfg in ${CONFIGS:-c3}; do
  for i in $(seq ${REPS:-2}); do
    for v in ${VARIANTS}; do
      RSP_LIB="$ROOT/radar-signal-process_amd/lib/ablate/librsp_$v.so" timeout -k 10 200 python bench.py --config $cfg --steps ${STEPS:-20} --cpu-seconds 0 > gpurun_out/ab_${cfg}_${v}.log 2>&1 || { echo "bench $cfg $v failed"; tail -5 gpurun_out/ab_${cfg}_${v}.log; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], {k: v['avg_us'] for k, v in r.get('kernels', {}).items()})" gpurun_out/ab_${cfg}_${v}.log "$cfg $v"
    done
  done
done
