#!/bin/bash
# Round-4 first GPU session: primitives (LDS-DMA range check, HBM ceiling, PCIe), the new GPU
# tests (host pipeline, ingest types, device guard), the host-path bench, and the PC LDS-DMA A/B
# (bit-identity digests, then interleaved bench runs).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
# the microbenchmarks are built here (their binaries do not travel)
M=gpurun_out/micro; mkdir -p $M
hipcc -O3 --offload-arch=gfx950 tools/micro/lds_dma_probe.hip -o $M/lds_dma_probe 2>/dev/null &&
hipcc -O3 --offload-arch=gfx950 tools/micro/hbm_ceiling.hip -o $M/hbm_ceiling 2>/dev/null &&
g++ -O3 -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tools/micro/pcie_probe.cpp -L/opt/rocm/lib -lamdhip64 \
    -lpthread -o $M/pcie_probe || { echo "micro build failed"; exit 1; }
timeout -k 10 60 $M/lds_dma_probe > gpurun_out/lds_dma_probe.txt 2>&1 || { echo "probe failed"; exit 1; }
cat gpurun_out/lds_dma_probe.txt
timeout -k 10 120 $M/pcie_probe 256 > gpurun_out/pcie_probe.txt 2>&1 || { echo "pcie failed"; exit 1; }
cat gpurun_out/pcie_probe.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_hostpath.py \
    tests/test_gpu_ingest.py tests/test_gpu_dist.py > gpurun_out/pytest_new.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 5 --cpu-seconds 0 --host-path --lane-steps 0 > gpurun_out/host_c3.log 2>&1 || { echo "host bench failed"; tail -5 gpurun_out/host_c3.log; exit 1; }
tail -1 gpurun_out/host_c3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['value'], 'host', json.dumps(d.get('host_path')))"
timeout -k 10 240 $M/hbm_ceiling 2 > gpurun_out/hbm_ceiling.txt 2>&1 || { echo "ceiling failed"; exit 1; }
tail -1 gpurun_out/hbm_ceiling.txt
timeout -k 10 120 python tools/mall_probe.py > gpurun_out/mall_probe.txt 2>&1 || { echo "mall probe failed"; exit 1; }
grep cpis gpurun_out/mall_probe.txt
VARIANTS="${VARIANTS:-base dma1 dma2 mdma}" CONFIGS="${CONFIGS:-c3}" REPS=${REPS:-2} timeout -k 10 700 tools/ab2.sh
