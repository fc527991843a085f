#!/bin/bash
# PC diagnostics on the GPU: the hand-written HBM ceiling, then tools/pc_bench.py on the
# diagnostic builds of tools/build_variant.sh (VARIANTS="base l2in ...").
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${CEILING:-1}" = 1 ]; then
  timeout -k 10 150 tools/micro/hbm_ceiling ${CEIL_GIB:-2} > gpurun_out/hbm_ceiling.txt 2>&1 || exit $?
  grep BEST gpurun_out/hbm_ceiling.txt | tail -6
fi
for v in ${VARIANTS:-base}; do
  echo "== $v"
  RSP_LIB="$ROOT/radar-signal-process_amd/lib/ablate/librsp_$v.so" timeout -k 10 120 \
    python tools/pc_bench.py --cpis ${CPIS:-16 64} --iters 20 ${PC_ARGS:-} 2>&1 | grep -v amdgpu.ids || exit 1
done
