#!/bin/bash
# Ingest measurement session: bench lines and rocprofv3 --kernel-trace --stats
# for all-DDC capture frames and for frames mixing DDC / ADC / 24-bit DBF PRTs.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
for kind in ddc mix; do
  OUT="$ROOT/gpurun_out/ingest_$kind"; rm -rf "$OUT"; mkdir -p "$OUT"
  FLAG=""; [ $kind = mix ] && FLAG="--ingest-mix"
  timeout -k 10 240 python bench.py --config ingest --steps 20 --cpu-seconds 5 $FLAG > "$OUT/bench.log" 2> "$OUT/bench.err" \
      || { echo "bench $kind rc=$?"; tail -5 "$OUT/bench.err"; exit 1; }
  tail -1 "$OUT/bench.log" | cut -c1-260
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python3 "$ROOT/bench.py" --config ingest --steps 10 --cpu-seconds 0 $FLAG > "$OUT/prof.log" 2>&1) \
      || { echo "rocprof $kind rc=$?"; tail -3 "$OUT/prof.log"; exit 1; }
  python - "$OUT/prof/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("  %-60s calls %6s avg %8.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
