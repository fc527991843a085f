#!/bin/bash
# Copy one measure_cfg.sh session (gpurun_out/<cfg>) into profiles/<round>/<cfg>: the bench
# line, the rocprofv3 --stats summary, the trace summary and the PMC summary; and install the
# PMC summary as profiles/pmc_<tag>.json, the file bench.py reads its `traffic` from.
# Usage: tools/save_profile.sh r02/final c3 v2_P128_R4096
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
dst="$ROOT/profiles/$1/$2"; src="$ROOT/gpurun_out/$2"
mkdir -p "$dst"
cp "$src/bench.log" "$src/trace.json" "$src/pmc.json" "$src/pmc.txt" "$dst/"
[ -f "$src/overlap.json" ] && cp "$src/overlap.json" "$dst/"
cp "$src/prof/run_kernel_stats.csv" "$dst/kernel_stats.csv"
if [ -f "$src/prof1/run_kernel_stats.csv" ]; then
  cp "$src/prof1/run_kernel_stats.csv" "$dst/kernel_stats_1pipeline.csv"; cp "$src/trace_1lane.json" "$dst/"
fi
cp "$src/pmc.json" "$ROOT/profiles/pmc_$3.json"
echo "saved $2 -> profiles/$1/$2, profiles/pmc_$3.json"
