// CPU check of rsp::CopyPool (radar-signal-process_amd/csrc/rsp_hostpool.h), driven by
// tests/test_hostpool.py: every conversion against a scalar loop, over thread counts, sizes
// either side of the split threshold and misaligned destinations, with many back-to-back jobs
// (the spin / block hand-off) -- exit 0 and "ok" on success.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "rsp_hostpool.h"

static int fails = 0;
#define CHECK(c, ...)                    \
    do {                                 \
        if (!(c)) {                      \
            fprintf(stderr, __VA_ARGS__); \
            fprintf(stderr, "\n");       \
            ++fails;                     \
        }                                \
    } while (0)

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 20;
    // a job issued right after construction, before the workers have started (a worker must
    // not skip the first generation: that hung the caller)
    for (int k = 0; k < 200; ++k) {
        rsp::CopyPool fresh(8);
        std::vector<uint8_t> a(1 << 21, (uint8_t)k), b(1 << 21);
        fresh.copy(b.data(), a.data(), a.size());
        CHECK(b[12345] == (uint8_t)k && b.back() == (uint8_t)k, "fresh pool copy %d", k);
    }
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> u(-1e6, 1e6);
    for (int threads : {1, 3, 8}) {
        rsp::CopyPool pool(threads);
        for (size_t n : {(size_t)1, (size_t)1000, (size_t)131071, (size_t)131072, (size_t)400001, (size_t)1 << 20}) {
            for (int off : {0, 1, 3}) {
                std::vector<double> src(2 * n + 8), dsrc(n + 8);
                std::vector<float> fsrc(n + 8), f(2 * n + 8);
                std::vector<uint8_t> bsrc(n + 8);
                std::vector<double> d(n + 8);
                for (auto& x : src) x = u(rng) * (rng() % 7 == 0 ? 1e-40 : 1.0);   // incl. float subnormals / zero
                for (size_t i = 0; i < n + 8; ++i) {
                    fsrc[i] = (float)u(rng);
                    bsrc[i] = (uint8_t)(rng() & 1);
                    dsrc[i] = u(rng);
                }
                for (int r = 0; r < rounds; ++r) {
                    pool.narrow_c128(f.data() + off, src.data(), n);
                    for (size_t i = 0; i < 2 * n; ++i)
                        if (f[off + i] != (float)src[i] && !(std::isnan(f[off + i]) && std::isnan(src[i]))) {
                            CHECK(false, "narrow_c128 t%d n%zu off%d i%zu", threads, n, off, i);
                            break;
                        }
                    pool.narrow_f64(f.data() + off, dsrc.data(), n);
                    CHECK(std::memcmp(f.data() + off, std::vector<float>(dsrc.begin(), dsrc.begin() + n).data(), n * 4) == 0,
                          "narrow_f64 t%d n%zu off%d", threads, n, off);
                    pool.widen_f32(d.data() + off, fsrc.data(), n);
                    bool ok = true;
                    for (size_t i = 0; i < n && ok; ++i) ok = d[off + i] == (double)fsrc[i];
                    CHECK(ok, "widen_f32 t%d n%zu off%d", threads, n, off);
                    pool.widen_u8(d.data() + off, bsrc.data(), n);
                    ok = true;
                    for (size_t i = 0; i < n && ok; ++i) ok = d[off + i] == (double)bsrc[i];
                    CHECK(ok, "widen_u8 t%d n%zu off%d", threads, n, off);
                    pool.copy(f.data() + off, fsrc.data(), n * 4);
                    CHECK(std::memcmp(f.data() + off, fsrc.data(), n * 4) == 0, "copy t%d n%zu off%d", threads, n, off);
                }
            }
        }
    }
    if (fails) {
        fprintf(stderr, "%d failures\n", fails);
        return 1;
    }
    printf("ok\n");
    return 0;
}
