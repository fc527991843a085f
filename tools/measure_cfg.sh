#!/bin/bash
# Measurement session for one bench config (run on the GPU box from the repo root):
#   1. bench.py line (throughput + single-pipeline per-kernel pass)
#   2. rocprofv3 --kernel-trace --stats of the same command (--no-profile) + trace summary
#   3. PMC passes (HBM bytes; SQ groups with SQ=1), one rocprofv3 --pmc run per group,
#      summarised to gpurun_out/<cfg>/pmc.json (bytes per CPI over the whole run)
# Usage: tools/measure_cfg.sh c3 [extra bench args]      (env: STEPS, PMC_STEPS, SQ=1)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"
CFG=$1; shift
EXTRA="$*"
OUT="$ROOT/gpurun_out/$CFG"; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-10}
timeout -k 10 300 python bench.py --config $CFG --steps $STEPS --cpu-seconds ${CPU_SECONDS:-10} $EXTRA \
    > "$OUT/bench.log" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -5 "$OUT/bench.err"; exit 1; }
tail -1 "$OUT/bench.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$CFG', d['value'], d['unit'], 'ms/step', d['ms_per_step'], 'frac', r['frac'], {k: (v['avg_us'], v.get('frac')) for k, v in r.get('kernels', {}).items()})"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/bench.py" --config $CFG --steps 5 --cpu-seconds 0 --no-profile $EXTRA > "$OUT/prof.log" 2>&1) \
    || { echo "rocprof rc=$?"; tail -3 "$OUT/prof.log"; exit 1; }
python tools/trace_summary.py "$OUT/prof/run_kernel_trace.csv" --steps 5 --warmup-from "$OUT/prof.log" --json "$OUT/trace.json" > /dev/null
python -c "import json; d=json.load(open('$OUT/trace.json')); print('trace span ms/step', d['span_ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
python tools/lane_overlap.py "$OUT/prof/run_kernel_trace.csv" --steps 5 --warmup-from "$OUT/prof.log" --json "$OUT/overlap.json" > /dev/null || true
# the same on ONE pipeline (--streams 1): kernels do not overlap, so rocprof's per-kernel averages
# are comparable with bench.py's single-pipeline per-kernel entries
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof1" -o run -- \
    python3 "$ROOT/bench.py" --config $CFG --steps 5 --cpu-seconds 0 --no-profile --streams 1 $EXTRA > "$OUT/prof1.log" 2>&1) \
    || { echo "rocprof (1 pipeline) rc=$?"; tail -3 "$OUT/prof1.log"; exit 1; }
python tools/trace_summary.py "$OUT/prof1/run_kernel_trace.csv" --steps 5 --warmup-from "$OUT/prof1.log" --json "$OUT/trace_1lane.json" > /dev/null
python -c "import json; d=json.load(open('$OUT/trace_1lane.json')); print('1-pipeline trace', d['span_ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
[ "${PMC:-1}" = "1" ] || exit 0
PSTEPS=${PMC_STEPS:-2}
PGROUPS=("FETCH_SIZE" "WRITE_SIZE")
if [ "${SQ:-0}" = "1" ]; then
  PGROUPS+=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
           "GRBM_GUI_ACTIVE GRBM_COUNT")
fi
i=0
for grp in "${PGROUPS[@]}"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/pmc/g$i" -o run -- \
      python3 "$ROOT/bench.py" --config $CFG --steps $PSTEPS --warmup 1 --cpu-seconds 0 --no-profile $EXTRA > "$OUT/pmc_g$i.log" 2>&1)
  rc=$?; echo "pmc group $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || { tail -3 "$OUT/pmc_g$i.log"; exit $rc; }
done
UNITS=$(tail -1 "$OUT/bench.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(c['batch_per_gpu'] * (c['windows_per_pair'] or 1) * ($PSTEPS + 1))")
python tools/pmc_summary.py "$OUT/pmc" --json "$OUT/pmc.json" --units-total $UNITS > "$OUT/pmc.txt"
python -c "import json; d=json.load(open('$OUT/pmc.json')); print('pmc bytes/unit', d.get('bytes_per_unit'), {k: (v['hbm_bytes_per_launch'], v.get('valu_frac')) for k, v in d['kernels'].items()})"
