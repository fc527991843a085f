// Latency of the primitives a one-CPI host call (the MEX path: 4 MiB of C64 in, 2 MiB of RDM
// out per 128 x 4096 CPI) is built from, on the GPU box:
//   * a single pinned hipMemcpyAsync of S bytes, H2D and D2H: wall time from issue to
//     hipEventSynchronize's return, and the event-timed transfer;
//   * the same with a spin on hipEventQuery instead of hipEventSynchronize;
//   * hipStreamSynchronize / hipEventSynchronize on work that is already done;
//   * kernels that read the input straight from pinned host memory, or write the output
//     straight into it (zero-copy over PCIe), against the DMA;
//   * an empty kernel's launch-to-sync round trip.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/host_latency_probe.hip -o tools/micro/host_latency_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

__global__ void empty_kernel() {}

// dst[i] = src[i] over n uint4, grid-stride (src or dst may be pinned host memory)
__global__ void __launch_bounds__(256) copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// float -> double widening written straight into pinned host memory (the RDM's MATLAB type)
__global__ void __launch_bounds__(256) widen_kernel(const float4* __restrict__ src, double4* __restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = src[i];
        dst[i] = make_double4(v.x, v.y, v.z, v.w);
    }
}

int main() {
    CK(hipSetDevice(0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const size_t maxb = 16u << 20;
    void *h, *d, *d2;
    CK(hipHostMalloc(&h, maxb, hipHostMallocDefault));
    CK(hipMalloc(&d, maxb));
    CK(hipMalloc(&d2, maxb));
    memset(h, 1, maxb);
    CK(hipMemset(d, 0, maxb));
    const int N = 40;
    // warm up
    for (int i = 0; i < 5; ++i) {
        CK(hipMemcpyAsync(d, h, maxb, hipMemcpyHostToDevice, st));
        CK(hipMemcpyAsync(h, d, maxb, hipMemcpyDeviceToHost, st));
        empty_kernel<<<1, 64, 0, st>>>();
    }
    CK(hipStreamSynchronize(st));

    {
        std::vector<double> w;
        for (int i = 0; i < N; ++i) {
            const double t0 = now_us();
            empty_kernel<<<1, 64, 0, st>>>();
            CK(hipStreamSynchronize(st));
            w.push_back(now_us() - t0);
        }
        printf("empty kernel launch + hipStreamSynchronize            %8.1f us\n", median(w));
        w.clear();
        for (int i = 0; i < N; ++i) {
            const double t0 = now_us();
            CK(hipStreamSynchronize(st));
            w.push_back(now_us() - t0);
        }
        printf("hipStreamSynchronize, idle stream                     %8.1f us\n", median(w));
        CK(hipEventRecord(a, st));
        CK(hipEventSynchronize(a));
        w.clear();
        for (int i = 0; i < N; ++i) {
            const double t0 = now_us();
            CK(hipEventSynchronize(a));
            w.push_back(now_us() - t0);
        }
        printf("hipEventSynchronize, completed event                  %8.1f us\n", median(w));
        w.clear();
        for (int i = 0; i < N; ++i) {
            const double t0 = now_us();
            CK(hipEventRecord(b, st));
            w.push_back(now_us() - t0);
        }
        printf("hipEventRecord (issue)                                %8.1f us\n", median(w));
        CK(hipStreamSynchronize(st));
    }

    for (size_t S : {(size_t)256 << 10, (size_t)1 << 20, (size_t)2 << 20, (size_t)4 << 20, (size_t)8 << 20}) {
        for (int dir = 0; dir < 2; ++dir) {
            for (int spin = 0; spin < 2; ++spin) {
                std::vector<double> w, g, iss;
                for (int i = 0; i < N; ++i) {
                    const double t0 = now_us();
                    CK(hipEventRecord(a, st));
                    if (dir == 0) CK(hipMemcpyAsync(d, h, S, hipMemcpyHostToDevice, st));
                    else CK(hipMemcpyAsync(h, d, S, hipMemcpyDeviceToHost, st));
                    CK(hipEventRecord(b, st));
                    const double t1 = now_us();
                    if (spin) {
                        while (hipEventQuery(b) == hipErrorNotReady) {
                        }
                    } else {
                        CK(hipEventSynchronize(b));
                    }
                    w.push_back(now_us() - t0);
                    iss.push_back(t1 - t0);
                    float ms;
                    CK(hipEventElapsedTime(&ms, a, b));
                    g.push_back(ms * 1e3);
                }
                printf("%s %5zu KiB pinned, %s: wall %7.1f us (issue %5.1f), events %7.1f us = %5.1f GB/s\n",
                       dir ? "D2H" : "H2D", S >> 10, spin ? "spin " : "esync", median(w), median(iss), median(g),
                       S / median(g) * 1e-3);
            }
        }
    }
    // 4 pieces of S/4 back to back vs one copy, H2D (the current one-CPI input staging)
    for (size_t S : {(size_t)4 << 20}) {
        for (int pieces : {1, 2, 4, 8}) {
            std::vector<double> w;
            for (int i = 0; i < N; ++i) {
                const double t0 = now_us();
                for (int p = 0; p < pieces; ++p)
                    CK(hipMemcpyAsync((char*)d + p * (S / pieces), (char*)h + p * (S / pieces), S / pieces,
                                      hipMemcpyHostToDevice, st));
                CK(hipEventRecord(b, st));
                CK(hipEventSynchronize(b));
                w.push_back(now_us() - t0);
            }
            printf("H2D %5zu KiB in %d pieces: wall %7.1f us\n", S >> 10, pieces, median(w));
        }
    }
    // zero-copy kernels: read pinned host -> device, device -> pinned host, widen f32 -> f64 into host
    for (size_t S : {(size_t)2 << 20, (size_t)4 << 20}) {
        for (int grid : {64, 256, 1024}) {
            std::vector<double> r, wr, wd;
            for (int i = 0; i < N; ++i) {
                double t0 = now_us();
                copy_kernel<<<grid, 256, 0, st>>>((const uint4*)h, (uint4*)d, S / 16);
                CK(hipStreamSynchronize(st));
                r.push_back(now_us() - t0);
                t0 = now_us();
                copy_kernel<<<grid, 256, 0, st>>>((const uint4*)d, (uint4*)h, S / 16);
                CK(hipStreamSynchronize(st));
                wr.push_back(now_us() - t0);
                t0 = now_us();
                widen_kernel<<<grid, 256, 0, st>>>((const float4*)d, (double4*)h, S / 16);   // S bytes of f32 -> 2S into host
                CK(hipStreamSynchronize(st));
                wd.push_back(now_us() - t0);
            }
            printf("zero-copy %5zu KiB grid %4d: kernel read host %7.1f us, write host %7.1f us, widen->host (2x bytes) %7.1f us\n",
                   S >> 10, grid, median(r), median(wr), median(wd));
        }
    }
    CK(hipHostFree(h));
    CK(hipFree(d));
    CK(hipFree(d2));
    return 0;
}
