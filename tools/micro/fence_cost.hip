// Cost of agent-scope release (buffer_wbl2 sc1) / acquire (buffer_inv sc1) fences on gfx950
// for a dataflow kernel: each workgroup writes a 32 KB item, then (optionally) fences and bumps
// a counter; the acquire variant also re-reads a 32 KB L2-resident table after each fence.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int MODE>   // 0: no fence; 1: release per item; 2: release + acquire per item
__global__ __launch_bounds__(256) void items(float4* out, const float4* table, unsigned* ctr, int nitems,
                                             float* sink) {
    float acc = 0.f;
    for (int it = blockIdx.x; it < nitems; it += gridDim.x) {
        float4* o = out + (size_t)it * 2048;   // 32 KB per item
#pragma unroll
        for (int k = 0; k < 8; ++k) o[threadIdx.x + 256 * k] = make_float4(it, k, 1.f, 2.f);
        if (MODE >= 1) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __syncthreads();
            if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (MODE >= 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += table[threadIdx.x + 256 * k].x;   // 32 KB table, L2-resident
    }
    if (acc == 12345.f) *sink = acc;
}

int main() {
    const int nitems = 16384;   // 512 MB written
    float4 *out, *table;
    unsigned* ctr;
    float* sink;
    hipMalloc(&out, (size_t)nitems * 2048 * sizeof(float4));
    hipMalloc(&table, 2048 * sizeof(float4));
    hipMalloc(&ctr, 4);
    hipMalloc(&sink, 4);
    hipMemset(table, 0, 2048 * sizeof(float4));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
        for (int mode = 0; mode < 3; ++mode) {
            const int grid = 256 * 4;
            for (int w = 0; w < 2; ++w) {
                hipEventRecord(e0);
                if (mode == 0) hipLaunchKernelGGL(items<0>, dim3(grid), dim3(256), 0, 0, out, table, ctr, nitems, sink);
                if (mode == 1) hipLaunchKernelGGL(items<1>, dim3(grid), dim3(256), 0, 0, out, table, ctr, nitems, sink);
                if (mode == 2) hipLaunchKernelGGL(items<2>, dim3(grid), dim3(256), 0, 0, out, table, ctr, nitems, sink);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
            }
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            printf("mode %d (%s): %.1f us, %.2f TB/s written, %.2f us per item-round\n", mode,
                   mode == 0 ? "no fence" : mode == 1 ? "release" : "release+acquire", ms * 1e3,
                   (double)nitems * 32768 / (ms * 1e-3) / 1e12, ms * 1e3 / ((double)nitems / grid));
        }
    }
    return hipGetLastError() != hipSuccess;
}
