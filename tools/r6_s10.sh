#!/bin/bash
# Round 6, session 10: after the PC LDS-DMA variant left the source -- output digests against the
# round-6 reference digests (tools/r6_digest_ref.txt, session 3's build), then the -m gpu suite.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; O=gpurun_out/r6s10; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/lib_digest.py > $O/digest.txt 2>$O/digest.err || { tail -3 $O/digest.err; exit 1; }
diff <(grep -v "^lib" tools/r6_digest_ref.txt) <(grep -v "^lib" $O/digest.txt) && echo "digests identical" || { echo "digests DIFFER"; exit 1; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; exit $rc
