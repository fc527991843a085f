#!/bin/bash
# Round-4 third A/B session: the MTD LDS-DMA variant (and PC + MTD DMA together) against the
# product at c3, c4, c5 (bit-identity digests first, then two interleaved rounds).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS="${VARIANTS:-base mdma both}" CONFIGS="${CONFIGS:-c3 c4 c5}" REPS=${REPS:-2} timeout -k 10 1050 tools/ab2.sh
