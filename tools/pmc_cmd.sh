#!/bin/bash
# rocprofv3 --pmc passes over an arbitrary python command (one counter group per pass).
#   GROUPS_FILE=... OUT=gpurun_out/pmcX bash tools/pmc_cmd.sh tools/pc_bench.py --cpis 256
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/${OUT:-gpurun_out/pmc_cmd}"
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
script="$ROOT/$1"; shift
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  (cd /tmp && timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/g$i" -o run -- \
      python3 "$script" "$@" > "$OUT/g$i.log" 2>&1)
  rc=$?; echo "group $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/g$i.log"; exit $rc; fi
done < "${GROUPS_FILE:-$ROOT/tools/pmc_groups.txt}"
