#!/bin/bash
# Run one gpurun call; when nothing ran because no box or GPU slot was free (gpurun exit code 3:
# nothing charged), wait and submit the same call again, up to 15 times.  Any other outcome --
# success, a failing command, a refusal -- ends the loop.
for i in $(seq 1 15); do
  out=$(/usr/local/graft/bin/gpurun "$@" 2>&1); rc=$?
  if [ $rc -eq 3 ] || echo "$out" | grep -q "no free box right now"; then echo "[retry $i: no box/slot]"; sleep 120; continue; fi
  echo "$out" | tail -40; exit $rc
done
echo "gave up: no box"; exit 3
