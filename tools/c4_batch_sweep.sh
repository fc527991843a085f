#!/bin/bash
# window-mode / c5 batch sweep: CONFIG batch streams chunk triples from SWEEP (windows/s or CPI/s)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out/c4sweep
IFS=';' read -ra CASES <<< "${SWEEP:-c4 32 0 0;c4 128 0 0}"
for cfg in "${CASES[@]}"; do
  set -- $cfg
  f=gpurun_out/c4sweep/$1_b$2_s$3_c$4.json
  timeout -k 10 300 python bench.py --config $1 --batch $2 --streams $3 --chunk $4 --steps ${STEPS:-6} --cpu-seconds 0 \
      --no-profile > $f 2>/dev/null || { echo "fail $cfg"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $f "$cfg"
done
