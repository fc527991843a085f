#!/bin/bash
# Kernel trace of the chain (2 pipelines) for a library variant, and how its lanes overlap
# (tools/lane_overlap.py).  Usage: V=<variant|lib> CFG=c3 tools/overlap_probe.sh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"
export TMPDIR=/tmp
V=${V:-lib}; CFG=${CFG:-c3}
lib="$ROOT/radar-signal-process_amd/lib/librsp.so"; [ $V != lib ] && lib="$ROOT/radar-signal-process_amd/lib/ablate/librsp_$V.so"
OUT="$ROOT/gpurun_out/overlap_${V}_$CFG"; rm -rf "$OUT"; mkdir -p "$OUT"
(cd /tmp && RSP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/bench.py" --config $CFG --steps 5 --cpu-seconds 0 --no-profile ${BENCH_ARGS:-} > "$OUT/prof.log" 2>&1) \
    || { echo "rocprof rc=$?"; tail -3 "$OUT/prof.log"; exit 1; }
python tools/lane_overlap.py "$OUT/prof/run_kernel_trace.csv" --steps 5 --warmup-from "$OUT/prof.log" --json "$OUT/overlap.json"
