#!/bin/bash
# Build a flag variant of librsp for A/B runs on the GPU (tools/ab_variants.sh VARIANTS=...):
#   tools/build_variant.sh NAME "-DFOO=1 -DBAR"   ->  radar-signal-process_amd/lib/ablate/librsp_NAME.so
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"; P="$ROOT/radar-signal-process_amd"
name=$1; flags=${2:-}
make -s -C "$P" build/rsp_capi.o build/rsp_ingest.o build/rsp_measure.o build/rsp_prefilter.o
mkdir -p "$P/build/ablate" "$P/lib/ablate"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics $flags -c "$P/csrc/rsp_kernels.hip" -o "$P/build/ablate/k_$name.o"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 "$P/build/ablate/k_$name.o" "$P/build/rsp_ingest.o" "$P/build/rsp_measure.o" \
    "$P/build/rsp_prefilter.o" "$P/build/rsp_capi.o" -o "$P/lib/ablate/librsp_$name.so"
echo "built lib/ablate/librsp_$name.so ($flags)"
