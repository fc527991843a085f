#!/bin/bash
# Round-4 verification + extras session: bitwise digests of the committed product ("head")
# against the working build ("new"), interleaved c3/c4 runs of both, the whole -m gpu suite on the
# working build, then the host-path / ingest / prefilter / measure bench lines and c2.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS="head new" CONFIGS="c3 c4" REPS=2 timeout -k 10 600 tools/ab2.sh || exit $?
SQ=0 bash tools/r4_session.sh tests extras c2
