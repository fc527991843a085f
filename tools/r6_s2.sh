#!/bin/bash
# Round 6, session 2: GPU tests after the flow removal; CU-mask census v2; host-path prefault A/B;
# CU-split schedule A/B at c3 (digests first, then interleaved benches).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; O=gpurun_out/r6s2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 tools/micro/cumask_probe 20 4 > $O/cumask_probe.txt 2>&1 || { echo "probe failed"; tail -5 $O/cumask_probe.txt; exit 1; }
grep -E "more than one|mask bits|co-residency|per xcc" $O/cumask_probe.txt | head -20
timeout -k 10 200 python tools/lib_digest.py > $O/digest_default.txt 2>&1 || exit 1
RSP_CU_SPLIT=20 timeout -k 10 200 python tools/lib_digest.py > $O/digest_split20.txt 2>&1 || exit 1
diff <(grep -v "^lib" $O/digest_default.txt) <(grep -v "^lib" $O/digest_split20.txt) > /dev/null && echo "digests: split20 identical" || echo "digests: split20 DIFFER"
for rep in 1 2; do
  for sp in 0 16 20 24; do
    RSP_CU_SPLIT=$sp timeout -k 10 200 python bench.py --steps 20 --warmup 2 --cpu-seconds 0 --no-profile > $O/split${sp}_$rep.log 2>&1 || { echo "bench split $sp failed"; tail -3 $O/split${sp}_$rep.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('split', sys.argv[2], d['value'])" $O/split${sp}_$rep.log $sp
  done
done
for cfg in "1 1" "1 0" "0 1"; do
  set -- $cfg
  RSP_PREFAULT=$1 RSP_PREFAULT_HUGE=$2 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --host-path --no-profile > $O/host_pf$1_h$2.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); h=d['host_path']; print('host', sys.argv[2], {k: v['value'] for k, v in h.items() if isinstance(v, dict)})" $O/host_pf$1_h$2.log "pf=$1 huge=$2"
done
