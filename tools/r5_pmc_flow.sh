#!/bin/bash
# SQ counters of the dataflow kernel against the chunked schedule (round 5):
# one rocprofv3 --pmc pass per counter group and schedule, summed over every dispatch of a
# 3-step c3 run (warm-up included) and divided by the CPIs processed.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/pmcflow"; rm -rf "$OUT"; mkdir -p "$OUT"
PG=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
        "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
        "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_GROUPS:-})
for f in ${FLOWS:-0 1}; do
  i=0
  for grp in "${PG[@]}"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/f$f/g$i" -o run -- \
        python3 "$ROOT/bench.py" --config c3 --steps 2 --warmup 1 --cpu-seconds 0 --no-profile --flow $f > "$OUT/f${f}_g$i.log" 2>&1)
    rc=$?; echo "flow $f group $i rc=$rc"; [ $rc -eq 0 ] || { tail -3 "$OUT/f${f}_g$i.log"; exit $rc; }
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys, collections
out = sys.argv[1]
res = {}
for fd in sorted(glob.glob(os.path.join(out, "f*"))):
    if not os.path.isdir(fd):
        continue
    tot = collections.Counter()
    for f in glob.glob(os.path.join(fd, "g*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
    cpis = 3 * 1024
    per = {k: v / cpis for k, v in tot.items()}
    if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
        per["hbm_bytes"] = (2 * per["FETCH_SIZE"] + per["WRITE_SIZE"]) * 1024
    if per.get("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in per:
                per[k + "_frac"] = per[k] / per["SQ_WAVE_CYCLES"]
    res[os.path.basename(fd)] = {k: round(v, 4) for k, v in sorted(per.items())}
json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
PY
