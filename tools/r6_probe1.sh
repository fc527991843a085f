#!/bin/bash
# Round 6, session 1: CU-mask census + co-residency probe; the c3 bench; the host path with and
# without the output prefault (RSP_PREFAULT=0).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 120 tools/micro/cumask_probe 20 4 > gpurun_out/r6/cumask_probe.txt 2>&1 || { echo "probe rc=$?"; tail -5 gpurun_out/r6/cumask_probe.txt; exit 1; }
tail -12 gpurun_out/r6/cumask_probe.txt
timeout -k 10 200 python bench.py --steps 20 --warmup 2 --cpu-seconds 0 > gpurun_out/r6/bench_head.log 2>&1 || exit $?
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], {k: (v['avg_us'], v['frac_alg']) for k, v in r['kernels'].items()})" gpurun_out/r6/bench_head.log
for pf in 1 0 1 0; do
  RSP_PREFAULT=$pf timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --host-path --no-profile > gpurun_out/r6/host_pf$pf.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); h=d['host_path']; print('host pf=$pf', {k: v['value'] for k, v in h.items() if isinstance(v, dict)})" gpurun_out/r6/host_pf$pf.log
done
