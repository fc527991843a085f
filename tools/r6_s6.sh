#!/bin/bash
# Round 6, session 6: host prefault on the caller's NUMA node (A/B: THP/NUMA placement and release
# cost of fresh outputs; the fresh/reused breakdown); then the c2 / c4 / c5 measurement sessions.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; O=gpurun_out/r6s6; mkdir -p $O
export TMPDIR=/tmp
g++ -O2 -pthread tools/micro/prefault_probe.cpp -o $O/prefault_probe && timeout -k 10 120 $O/prefault_probe 100 3 > $O/prefault_probe.txt 2>&1; head -8 $O/prefault_probe.txt; tail -4 $O/prefault_probe.txt
for rep in 1 2; do
  for nm in 1 0; do
    RSP_PREFAULT_NUMA=$nm timeout -k 10 120 python tools/host_thp_probe.py > $O/thp_numa${nm}_$rep.json 2>$O/thp.err || { tail -3 $O/thp.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('numa', sys.argv[2], d['caller_cpu_node'], [(r['numa_kib'], r['release_ms']) for r in d['library']][1:3], 'numpy', [r['release_ms'] for r in d['numpy_fill']][1:3])" $O/thp_numa${nm}_$rep.json $nm
    RSP_PREFAULT_NUMA=$nm timeout -k 10 120 python tools/host_fresh_probe.py > $O/fresh_numa${nm}_$rep.json 2>&1 || exit 1
    tail -1 $O/fresh_numa${nm}_$rep.json
  done
done
for c in c2 c4 c5; do
  SQ=1 bash tools/measure_cfg.sh $c || exit 1
done
