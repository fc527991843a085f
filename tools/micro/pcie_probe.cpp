// Host <-> device copy primitives on the GPU box, for the pipelined host path of
// rsp_pc_mtd_cfar (MATLAB's buffers are pageable): pageable vs pinned hipMemcpyAsync rates in
// each direction, the cost of hipHostRegister on a fresh pageable buffer, and multi-threaded
// host memcpy (pageable -> pinned staging) rates.
//   g++ -O3 -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tools/micro/pcie_probe.cpp \
//       -L/opt/rocm/lib -lamdhip64 -lpthread -o tools/micro/pcie_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void par_copy(void* dst, const void* src, size_t n, int T) {
    if (T <= 1) {
        memcpy(dst, src, n);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (n / T + 4095) & ~(size_t)4095;
    for (int t = 0; t < T; ++t) {
        const size_t a = (size_t)t * per;
        if (a >= n) break;
        const size_t b = a + per < n ? a + per : n;
        th.emplace_back([=] { memcpy((char*)dst + a, (const char*)src + a, b - a); });
    }
    for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
    const size_t MB = 1 << 20;
    const size_t n = (argc > 1 ? atoi(argv[1]) : 256) * MB;
    void *d, *pin;
    CK(hipMalloc(&d, n));
    CK(hipHostMalloc(&pin, n, 0));
    char* page = (char*)malloc(n);
    memset(page, 1, n);
    memset(pin, 1, n);
    hipStream_t s;
    CK(hipStreamCreate(&s));
    auto rate = [&](const char* name, auto fn) {
        fn();
        CK(hipStreamSynchronize(s));
        double best = 1e30;
        for (int r = 0; r < 5; ++r) {
            const double t0 = now();
            fn();
            CK(hipStreamSynchronize(s));
            const double t = now() - t0;
            best = t < best ? t : best;
        }
        printf("%-40s %8.2f GB/s  (%.2f ms per %zu MB)\n", name, n / best / 1e9, best * 1e3, n / MB);
        fflush(stdout);
    };
    rate("H2D pageable", [&] { CK(hipMemcpyAsync(d, page, n, hipMemcpyHostToDevice, s)); });
    rate("H2D pinned", [&] { CK(hipMemcpyAsync(d, pin, n, hipMemcpyHostToDevice, s)); });
    rate("D2H pageable", [&] { CK(hipMemcpyAsync(page, d, n, hipMemcpyDeviceToHost, s)); });
    rate("D2H pinned", [&] { CK(hipMemcpyAsync(pin, d, n, hipMemcpyDeviceToHost, s)); });
    hipStream_t s2;
    CK(hipStreamCreate(&s2));
    rate("H2D + D2H pinned, two streams (sum)", [&] {
        CK(hipMemcpyAsync(d, pin, n / 2, hipMemcpyHostToDevice, s));
        CK(hipMemcpyAsync((char*)pin + n / 2, (char*)d + n / 2, n / 2, hipMemcpyDeviceToHost, s2));
        CK(hipStreamSynchronize(s2));
    });
    for (int T : {1, 2, 4, 8, 16}) {
        char name[64];
        snprintf(name, sizeof(name), "memcpy pageable->pinned, %d threads", T);
        rate(name, [&] { par_copy(pin, page, n, T); });
        snprintf(name, sizeof(name), "memcpy pinned->pageable, %d threads", T);
        rate(name, [&] { par_copy(page, pin, n, T); });
    }
    // hipHostRegister of a fresh (never registered) pageable buffer, as a MATLAB array would be
    for (size_t sz : {8 * MB, 64 * MB, n}) {
        char* fresh = (char*)malloc(sz);
        memset(fresh, 2, sz);
        const double t0 = now();
        CK(hipHostRegister(fresh, sz, hipHostRegisterDefault));
        const double t1 = now();
        void* dp = nullptr;
        CK(hipHostGetDevicePointer(&dp, fresh, 0));
        CK(hipMemcpyAsync(d, fresh, sz, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        const double t2 = now();
        CK(hipHostUnregister(fresh));
        const double t3 = now();
        printf("hipHostRegister %4zu MB: register %.2f ms, first H2D %.2f ms (%.1f GB/s), unregister %.2f ms\n",
               sz / MB, (t1 - t0) * 1e3, (t2 - t1) * 1e3, sz / (t2 - t1) / 1e9, (t3 - t2) * 1e3);
        free(fresh);
    }
    printf("hardware threads: %u\n", std::thread::hardware_concurrency());
    return 0;
}
