// Host-only probe: how fast can fresh anonymous memory (a caller's new output array) be faulted
// in?  mmap N MiB, then fault it in with T threads over 2 MiB blocks: madvise(MADV_POPULATE_WRITE),
// a memset, or one locked `or 0` per page (a write fault that keeps the contents); with or without
// MADV_HUGEPAGE first.
// Usage: prefault_probe [MiB=100] [reps=5]
#include <sys/mman.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? atoi(argv[1]) : 100;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const size_t bytes = mib << 20, blk = 2u << 20;
    for (int mode = 0; mode < 5; ++mode) {   // 0 populate, 1 hugepage + populate, 2 memset, 3 touch, 4 hugepage + touch
        for (int T : {1, 2, 4, 8}) {
            double best = 1e9, unmap_best = 1e9;
            for (int r = 0; r < reps; ++r) {
                char* p = (char*)mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
                if (p == MAP_FAILED) return 1;
                if (mode == 1 || mode == 4) madvise(p, bytes, MADV_HUGEPAGE);
                std::atomic<size_t> next{0};
                const double t0 = now();
                std::vector<std::thread> th;
                for (int t = 0; t < T; ++t)
                    th.emplace_back([&] {
                        for (;;) {
                            const size_t i = next.fetch_add(1);
                            if (i * blk >= bytes) break;
                            const size_t n = bytes - i * blk < blk ? bytes - i * blk : blk;
                            if (mode == 2) {
                                memset(p + i * blk, 1, n);
                            } else if (mode >= 3) {   // one locked `or 0` per page: a write fault, contents kept
                                for (size_t o = 0; o < n; o += 4096) __atomic_fetch_or(p + i * blk + o, (char)0, __ATOMIC_RELAXED);
                            } else {
                                madvise(p + i * blk, n, MADV_POPULATE_WRITE);
                            }
                        }
                    });
                for (auto& x : th) x.join();
                const double dt = now() - t0;
                best = dt < best ? dt : best;
                const double u0 = now();
                munmap(p, bytes);
                const double du = now() - u0;
                unmap_best = du < unmap_best ? du : unmap_best;
            }
            printf("%-22s threads %d: %7.2f ms  (%.1f GB/s), munmap %.2f ms\n",
                   mode == 0 ? "populate" : mode == 1 ? "hugepage+populate" : mode == 2 ? "memset first touch" : mode == 3 ? "touch (lock or 0)" : "hugepage+touch", T, best * 1e3,
                   bytes / best / 1e9, unmap_best * 1e3);
        }
    }
    return 0;
}
