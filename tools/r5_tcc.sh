#!/bin/bash
# L2 (TCC) hit rates per kernel for library variants (round 5, VERDICT r4 item 1b: does CPI-to-XCD
# affinity let the MTD read its PC rows from the XCD's L2?).  One rocprofv3 --pmc pass per variant
# over a short c3 run; VARIANTS="head xcd" CHUNK=16.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/tcc"; rm -rf "$OUT"; mkdir -p "$OUT"
for v in ${VARIANTS:-head xcd}; do
  (cd /tmp && RSP_LIB="$ROOT/radar-signal-process_amd/lib/ablate/librsp_$v.so" timeout -s KILL 120 rocprofv3 \
      --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d "$OUT/$v" -o run -- \
      python3 "$ROOT/bench.py" --config c3 --steps 2 --warmup 1 --cpu-seconds 0 --no-profile --chunk ${CHUNK:-16} \
      > "$OUT/$v.log" 2>&1)
  rc=$?; echo "tcc $v rc=$rc"; [ $rc -eq 0 ] || { tail -3 "$OUT/$v.log"; exit $rc; }
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys, collections
out = sys.argv[1]
res = {}
for d in sorted(glob.glob(os.path.join(out, "*"))):
    if not os.path.isdir(d):
        continue
    acc = collections.defaultdict(collections.Counter)
    for f in glob.glob(os.path.join(d, "run_counter_collection.csv")) + glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            k = "pc" if "pc_mf_kernel" in n else ("mtd" if "mtd_kernel" in n else ("cfar" if "cfar" in n else None))
            if k:
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    res[os.path.basename(d)] = {k: {"hit_rate": round(c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4),
                                    "hits": c["TCC_HIT_sum"], "misses": c["TCC_MISS_sum"]} for k, c in acc.items()}
json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
PY
