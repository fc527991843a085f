#!/bin/bash
# Round-4 second A/B session: DMA probe (offsets > 64 KiB), variant localisation, host-path probe,
# digests + interleaved c3 / c4 / c5 bench runs of the LDS-DMA variants.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
M=gpurun_out/micro; mkdir -p $M
hipcc -O3 --offload-arch=gfx950 tools/micro/lds_dma_probe.hip -o $M/lds_dma_probe 2>/dev/null || { echo "build failed"; exit 1; }
timeout -k 10 60 $M/lds_dma_probe > gpurun_out/lds_dma_probe.txt 2>&1 || { echo "probe failed"; exit 1; }
grep "LDS-DMA to" gpurun_out/lds_dma_probe.txt
timeout -k 10 300 python tools/variant_diff.py base dma1 dma2 mdma 2>&1 | grep -v amdgpu.ids || { echo "vdiff failed"; exit 1; }
timeout -k 10 300 python tools/host_probe.py > gpurun_out/host_probe.txt 2>&1 || { echo "host probe failed"; tail -3 gpurun_out/host_probe.txt; exit 1; }
cat gpurun_out/host_probe.txt | grep -v amdgpu.ids
VARIANTS="${VARIANTS:-base dma1 dma2 mdma}" CONFIGS="${CONFIGS:-c3 c4}" REPS=${REPS:-1} timeout -k 10 780 tools/ab2.sh
