#!/bin/bash
# Round-5 GPU sessions (one gpurun call each; every GPU step has its own time limit and a
# failure ends the script):
#   tools/r5_session.sh tests           -- the whole -m gpu suite + smoke()
#   tools/r5_session.sh probe           -- tools/micro/handoff_probe (hand-off cost)
#   VARIANTS="base new" tools/r5_session.sh digest   -- bitwise output digests per library variant
#   VARIANTS="base new" CONFIGS="c3" REPS=2 tools/r5_session.sh ab   -- interleaved bench A/B
#   tools/r5_session.sh c3 c5           -- tools/measure_cfg.sh per config (bench, rocprofv3, PMC)
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
    probe)
      timeout -k 10 90 tools/micro/handoff_probe ${PROBE_ROUNDS:-64} > gpurun_out/handoff_probe.txt 2>&1; rc=$?
      cat gpurun_out/handoff_probe.txt; [ $rc -eq 0 ] || exit $rc ;;
    # (flowtest / flowab: round 5's dataflow-kernel cases; the kernel left the product in round 6)
    digest)
      DIGEST=1 CONFIGS=none REPS=0 bash tools/ab2.sh || exit $? ;;
    ab)
      DIGEST=0 bash tools/ab2.sh || exit $? ;;
    *)
      SQ=${SQ:-1} bash tools/measure_cfg.sh $what || exit $? ;;
  esac
done
