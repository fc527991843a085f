// Probe of gfx950's v_permlane16_swap / v_permlane32_swap lane semantics (builtins), used by
// the quad-lane FFT passes: prints, for each lane, which source lane's value each operand holds.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(int* out) {
    const int lane = threadIdx.x;
    unsigned a = 1000 + lane, b = 2000 + lane;
    auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    out[lane] = (int)r[0];
    out[64 + lane] = (int)r[1];
    auto q = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    out[128 + lane] = (int)q[0];
    out[192 + lane] = (int)q[1];
}

int main() {
    int* d;
    int h[256];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    for (int k = 0; k < 4; ++k) {
        printf("%s %s:", k < 2 ? "swap16" : "swap32", k % 2 ? "src " : "vdst");
        for (int l = 0; l < 64; l += 4) printf(" %d", h[64 * k + l]);
        printf("\n");
    }
    hipFree(d);
    return 0;
}
