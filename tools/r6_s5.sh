#!/bin/bash
# Round 6, session 5: THP probe of fresh host outputs; the -m gpu suite + smoke; the default bench
# line (the driver's command); the c3 measurement session (bench, rocprofv3 x2, PMC incl. SQ).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; O=gpurun_out/r6s5; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python tools/host_thp_probe.py > $O/host_thp_probe.json 2>$O/host_thp_probe.err || { tail -3 $O/host_thp_probe.err; exit 1; }
cat $O/host_thp_probe.json
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench rc=$?"; tail -3 $O/bench_default.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('default', d['value'], d['ms_per_step'], r['frac'], r.get('dominant_kernel'), r.get('dominant_frac_alg'), d['cpu_baseline']['value'])" $O/bench_default.json
SQ=1 bash tools/measure_cfg.sh c3 || exit 1
