#!/bin/bash
# Instruction-cache hits / misses per kernel (one rocprofv3 --pmc pass of 2 SQC counters) for
# the c3 bench on a library variant.  Usage: V=<variant|lib> tools/icache_probe.sh [bench args]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"
export TMPDIR=/tmp
V=${V:-lib}
lib="$ROOT/radar-signal-process_amd/lib/librsp.so"; [ $V != lib ] && lib="$ROOT/radar-signal-process_amd/lib/ablate/librsp_$V.so"
OUT="$ROOT/gpurun_out/icache_$V"; rm -rf "$OUT"; mkdir -p "$OUT"
(cd /tmp && RSP_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --kernel-trace --output-format csv \
    -d "$OUT/pmc" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-seconds 0 --no-profile --lane-steps 0 "$@" \
    > "$OUT/log" 2>&1) || { echo "rocprof rc=$?"; tail -3 "$OUT/log"; exit 1; }
python3 - "$OUT/pmc/run_counter_collection.csv" <<'PY'
import csv, collections, sys
sys.path.insert(0, "tools")
from pmc_summary import short
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = short(r["Kernel_Name"]); acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQC_ICACHE_HITS": n[k] += 1
for k, c in acc.items():
    h, m = c.get("SQC_ICACHE_HITS", 0), c.get("SQC_ICACHE_MISSES", 0)
    print("%-16s dispatches %4d  icache hits/disp %12.0f  misses/disp %10.0f  miss rate %.4f" % (k, n[k], h / max(n[k], 1), m / max(n[k], 1), m / max(h + m, 1)))
PY
