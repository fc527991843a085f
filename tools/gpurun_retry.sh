#!/bin/bash
# Run one gpurun call; when the pool has no free box (nothing ran, nothing charged), wait and
# submit the same call again, up to 12 times.  Any other outcome ends the loop.
for i in $(seq 1 12); do
  out=$(/usr/local/graft/bin/gpurun "$@" 2>&1); rc=$?
  if echo "$out" | grep -q "no free box right now"; then echo "[retry $i: no box]"; sleep 150; continue; fi
  echo "$out" | tail -40; exit $rc
done
echo "gave up: no box"; exit 3
