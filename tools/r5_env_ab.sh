#!/bin/bash
# Interleaved A/B of dev environment knobs: VAR=NAME VALUES="0 1 2" CONFIGS="c4 c3" REPS=2;
# digests per value first (tools/lib_digest.py), then bench runs.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
for v in ${VALUES}; do
  env "$VAR=$v" timeout -k 10 180 python tools/lib_digest.py > gpurun_out/digest_${VAR}_$v.txt 2>&1 || { echo "digest $v failed"; tail -5 gpurun_out/digest_${VAR}_$v.txt; exit 1; }
done
for v in ${VALUES}; do
  diff <(grep -v "^lib\|amdgpu" gpurun_out/digest_${VAR}_${VALUES%% *}.txt) <(grep -v "^lib\|amdgpu" gpurun_out/digest_${VAR}_$v.txt) > /dev/null \
    && echo "digest $VAR=$v identical" || echo "digest $VAR=$v DIFFERS"
done
for cfg in ${CONFIGS:-c3}; do
  for i in $(seq ${REPS:-2}); do
    for v in ${VALUES}; do
      env "$VAR=$v" timeout -k 10 200 python bench.py --config $cfg --steps ${STEPS:-20} --cpu-seconds 0 > gpurun_out/eab_${cfg}_$v.log 2>&1 || { echo "bench $cfg $v failed"; tail -5 gpurun_out/eab_${cfg}_$v.log; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], {k: (v['avg_us'], v['launches_per_step']) for k, v in r.get('kernels', {}).items()})" gpurun_out/eab_${cfg}_$v.log "$cfg $VAR=$v"
    done
  done
done
