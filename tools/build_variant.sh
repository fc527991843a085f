#!/bin/bash
# Build a flag variant of librsp for A/B runs on the GPU (tools/ab_pc.sh VARIANTS=...):
#   tools/build_variant.sh NAME "-DFOO=1 -DBAR"   ->  radar-signal-process_amd/lib/ablate/librsp_NAME.so
# The flags reach the kernels and the host code (dev-only -D switches of either).
# KSRC=dir: take rsp_kernels.hip / rsp_capi.cpp (and the headers next to them) from dir instead
# of csrc (e.g. a `git show` of an older commit for a bit-identity A/B).
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"; P="$ROOT/radar-signal-process_amd"
name=$1; flags=${2:-}
make -s -C "$P" build/rsp_ingest.o build/rsp_measure.o build/rsp_prefilter.o
mkdir -p "$P/build/ablate" "$P/lib/ablate"
S="${KSRC:-$P/csrc}"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics $flags -c "$S/rsp_kernels.hip" -o "$P/build/ablate/k_$name.o"
g++ -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include $flags -c "$S/rsp_capi.cpp" -o "$P/build/ablate/c_$name.o"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 "$P/build/ablate/k_$name.o" "$P/build/rsp_ingest.o" "$P/build/rsp_measure.o" \
    "$P/build/rsp_prefilter.o" "$P/build/ablate/c_$name.o" -o "$P/lib/ablate/librsp_$name.so"
echo "built lib/ablate/librsp_$name.so ($flags)"
