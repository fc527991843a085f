// Range-check behaviour of 16-byte buffer loads on gfx950, to VGPRs and LDS-DMA
// (buffer_load_dwordx4 ... lds), when num_records cuts a 16-byte access in half (an odd
// count of complex fp32 elements, 8 B each): does the in-range half arrive?
//   hipcc -O3 --offload-arch=gfx950 tools/micro/lds_dma_probe.hip -o tools/micro/lds_dma_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void probe(const int* __restrict__ src, int* __restrict__ out, uint32_t nrec) {
    __shared__ __attribute__((aligned(16))) int lds[64 * 4];
    for (int i = threadIdx.x; i < 256; i += 64) lds[i] = -1;
    __syncthreads();
    const auto r = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, (int)nrec, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, threadIdx.x * 16, 0, 0, 0);
    const v4i v = __builtin_amdgcn_raw_buffer_load_b128(r, threadIdx.x * 16, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int k = 0; k < 4; ++k) {
        out[threadIdx.x * 4 + k] = lds[threadIdx.x * 4 + k];
        out[256 + threadIdx.x * 4 + k] = v[k];
    }
}

// LDS-DMA destinations beyond 64 KiB (M0 carries the full LDS byte address?): one wave DMAs
// 1 KiB to each of several offsets of a 160 KiB dynamic LDS and reads it back.
__global__ void probe_hi(const int* __restrict__ src, int* __restrict__ out, const uint32_t* offs, int n) {
    extern __shared__ __attribute__((aligned(16))) int dyn[];
    const auto r = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 4096, 0x00020000);
    for (int i = 0; i < n; ++i) {
        for (int k = threadIdx.x; k < 256; k += 64) dyn[offs[i] / 4 + k] = -7;
        __syncthreads();
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)((char*)dyn + offs[i]), 16,
                                                 threadIdx.x * 16, 0, 0, 0);
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        for (int k = threadIdx.x; k < 256; k += 64) out[i * 256 + k] = dyn[offs[i] / 4 + k];
        __syncthreads();
    }
}

int main() {
    int *src, *out;
    hipMalloc(&src, 4096);
    hipMalloc(&out, 4096);
    int h[1024];
    for (int i = 0; i < 256; ++i) h[i] = i + 1;
    hipMemcpy(src, h, 1024, hipMemcpyHostToDevice);
    for (uint32_t nrec : {1024u, 1000u, 1016u, 1020u, 1012u}) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, src, out, nrec);
        hipMemcpy(h, out, 2048, hipMemcpyDeviceToHost);
        printf("num_records %u:", nrec);
        // the last dwords before and after the cut, LDS-DMA then VGPR
        const int lo = (int)nrec / 4 - 4, hi = (int)nrec / 4 + 4;
        printf("\n  lds :");
        for (int i = lo; i < hi && i < 256; ++i) printf(" [%d]=%d", i, h[i]);
        printf("\n  vgpr:");
        for (int i = lo; i < hi && i < 256; ++i) printf(" [%d]=%d", i, h[256 + i]);
        printf("\n");
    }
    {
        const uint32_t h_offs[6] = {0u, 34816u, 65024u, 69632u, 100000u, 162816u};
        uint32_t* d_offs;
        int* d_out;
        (void)hipMalloc(&d_offs, sizeof(h_offs));
        (void)hipMalloc(&d_out, 6 * 1024);
        (void)hipMemcpy(d_offs, h_offs, sizeof(h_offs), hipMemcpyHostToDevice);
        (void)hipFuncSetAttribute((const void*)probe_hi, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
        hipLaunchKernelGGL(probe_hi, dim3(1), dim3(64), 163840, 0, src, d_out, d_offs, 6);
        int hh[6 * 256];
        (void)hipMemcpy(hh, d_out, sizeof(hh), hipMemcpyDeviceToHost);
        for (int i = 0; i < 6; ++i) {
            int bad = 0;
            for (int k = 0; k < 256; ++k) bad += hh[i * 256 + k] != k + 1;
            printf("LDS-DMA to byte offset %6u: %s (%d of 256 dwords wrong)\n", h_offs[i], bad ? "WRONG" : "ok", bad);
        }
    }
    return 0;
}
