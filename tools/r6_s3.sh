#!/bin/bash
# Round 6, session 3: c4 flag memset beside the PC (A/B, digests first); the CU split with
# per-kernel times; host-path diagnostics (fault throughput on the box, trace of fresh vs reused).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; O=gpurun_out/r6s3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/lib_digest.py > $O/digest_side.txt 2>&1 || { tail -3 $O/digest_side.txt; exit 1; }
RSP_FLAG_MEMSET_SIDE=0 timeout -k 10 200 python tools/lib_digest.py > $O/digest_lane.txt 2>&1 || exit 1
diff <(grep -v "^lib" $O/digest_side.txt) <(grep -v "^lib" $O/digest_lane.txt) > /dev/null && echo "digests: side == lane" || echo "digests: side DIFFERS"
for rep in 1 2 3; do
  for sd in 1 0; do
    RSP_FLAG_MEMSET_SIDE=$sd timeout -k 10 200 python bench.py --config c4 --steps 20 --cpu-seconds 0 --no-profile > $O/c4_side${sd}_$rep.log 2>&1 || { tail -3 $O/c4_side${sd}_$rep.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c4 side', sys.argv[2], d['value'])" $O/c4_side${sd}_$rep.log $sd
  done
done
RSP_CU_SPLIT=20 timeout -k 10 200 python bench.py --steps 20 --warmup 2 --cpu-seconds 0 > $O/split20_kernels.log 2>&1 || exit 1
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('split20', d['value'], {k: v['avg_us'] for k, v in r['kernels'].items()})" $O/split20_kernels.log
g++ -O2 -pthread tools/micro/prefault_probe.cpp -o $O/prefault_probe && timeout -k 10 120 $O/prefault_probe 100 3 > $O/prefault_probe.txt 2>&1; cat $O/prefault_probe.txt
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag 2>&1 | tee $O/thp.txt
python - <<'PY' 2>&1 | tee $O/alloc_cost.txt
import time, numpy as np
n, Ro, V = 32, 4096, 128
for rep in range(3):
    t0 = time.perf_counter(); k = 0
    while time.perf_counter() - t0 < 1.0:
        o = (np.empty((n, Ro, V), np.float32), np.empty((n, Ro, V), np.uint8), np.empty((n, Ro, V), np.uint8))
        del o; k += 1
    t1 = time.perf_counter(); k2 = 0
    while time.perf_counter() - t1 < 1.0:
        o = (np.empty((n, Ro, V), np.float32), np.empty((n, Ro, V), np.uint8), np.empty((n, Ro, V), np.uint8))
        for a in o: a.reshape(-1)[::4096 // a.itemsize] = 0
        del o; k2 += 1
    print("empty+free %.3f ms; empty+touch+free %.3f ms" % ((t1 - t0) / k * 1e3, (time.perf_counter() - t1) / k2 * 1e3))
PY
for pf in 1 0; do
  RSP_HOST_TRACE=1 RSP_PREFAULT=$pf timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --host-path --no-profile > $O/host_trace_pf$pf.log 2> $O/host_trace_pf$pf.err || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); h=d['host_path']; print('host pf', sys.argv[2], {k: v['value'] for k, v in h.items() if isinstance(v, dict)})" $O/host_trace_pf$pf.log $pf
done
