#!/bin/bash
# Range-stage placement A/B (dev knobs RSP_RANGE_MODE / RSP_RANGE_GROUP, rsp_capi.cpp
# run_chain_body; RSP_HITS_LPR, rsp_kernels.hip launch_cfar_hits): digests per mode, then
# interleaved bench runs.  A mode is M[:G[:L]] (range mode, group size, lanes per hit region;
# L 0 = the library's rule).
#   MODES="0 2:16 2:16:16" CONFIGS="c3 c5 c4" REPS=2
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
for m in ${MODES:-0 1}; do
  IFS=: read -r M G L <<< "$m"; export RSP_RANGE_MODE=$M RSP_RANGE_GROUP=${G:-16} RSP_HITS_LPR=${L:-0}
  timeout -k 10 180 python tools/lib_digest.py > gpurun_out/digest_range$m.txt 2>&1 || { echo "digest $m failed"; tail -5 gpurun_out/digest_range$m.txt; exit 1; }
  echo "== digest mode $m"; grep -v "^lib" gpurun_out/digest_range$m.txt | grep -v amdgpu.ids
done
for cfg in ${CONFIGS:-c3 c5 c4}; do
  for i in $(seq ${REPS:-2}); do
    for m in ${MODES:-0 1}; do
      IFS=: read -r M G L <<< "$m"; export RSP_RANGE_MODE=$M RSP_RANGE_GROUP=${G:-16} RSP_HITS_LPR=${L:-0}
      timeout -k 10 200 python bench.py --config $cfg --steps ${STEPS:-20} --cpu-seconds 0 > gpurun_out/rab_${cfg}_$m.log 2>&1 || { echo "bench $cfg $m failed"; tail -5 gpurun_out/rab_${cfg}_$m.log; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], {k: (v['avg_us'], v['launches_per_step']) for k, v in r.get('kernels', {}).items()})" gpurun_out/rab_${cfg}_$m.log "$cfg mode$m"
    done
  done
done
