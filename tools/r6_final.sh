#!/bin/bash
# Round 6, final validation of the committed tree: the -m gpu suite, smoke(), the driver's default
# bench command, and a rocprofv3 --kernel-trace --stats pass of that same command.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; O=gpurun_out/r6final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench rc=$?"; tail -3 $O/bench_default.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('default', d['value'], d['ms_per_step'], r['frac'], r.get('dominant_kernel'), r.get('dominant_frac_alg'), {k: (v['avg_us'], v.get('frac_alg')) for k, v in r['kernels'].items()})" $O/bench_default.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof -o run -- python3 $ROOT/bench.py --cpu-seconds 0 > $ROOT/$O/prof.log 2>&1) || { echo "rocprof failed"; tail -3 $ROOT/$O/prof.log; exit 1; }
head -5 $O/prof/run_kernel_stats.csv | cut -c1-150
