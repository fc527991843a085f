#!/bin/bash
# Round-4 measurement sessions on the GPU box (one gpurun call each, < 20 min):
#   tools/r4_session.sh tests   -- the whole -m gpu suite + smoke()
#   tools/r4_session.sh c3 c4   -- tools/measure_cfg.sh per config (bench line, rocprofv3 --stats on
#                                  2 and 1 pipelines, PMC incl. the SQ groups)
#   tools/r4_session.sh extras  -- host path (batch 32 and 1), ingest, prefilter, measure bench lines
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
for what in "$@"; do
  case $what in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
          > gpurun_out/pytest_gpu.log 2>&1; rc=$?
      echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/smoke.log; exit 1; }
      tail -1 gpurun_out/smoke.log ;;
    extras)
      timeout -k 10 240 python bench.py --steps 5 --cpu-seconds 0 --host-path --lane-steps 0 > gpurun_out/host_c3.log 2>&1 || { echo host failed; exit 1; }
      tail -1 gpurun_out/host_c3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('host', json.dumps(d.get('host_path')))"
      for c in ingest prefilter measure; do
        timeout -k 10 200 python bench.py --config $c --steps 20 --cpu-seconds 0 > gpurun_out/bench_$c.log 2>&1 || { echo "$c failed"; exit 1; }
        tail -1 gpurun_out/bench_$c.log | cut -c1-300
      done ;;
    *)
      SQ=${SQ:-1} bash tools/measure_cfg.sh $what || exit $? ;;
  esac
done
