// CPU check of rsp::CopyPool (radar-signal-process_amd/csrc/rsp_hostpool.h), driven by
// tests/test_hostpool.py: every conversion against a scalar loop, over thread counts, sizes
// either side of the split threshold and misaligned destinations, with many back-to-back jobs
// (the spin / block hand-off) -- exit 0 and "ok" on success.
#include <sys/mman.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
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
    // rsp::Prefaulter (the host calls' output prefault): fresh anonymous ranges at unaligned
    // offsets, some bytes written before the job (their contents must survive the faulting), two
    // copier threads that wait() per piece and then write it, and jobs abandoned early (end()
    // before every block was waited for).  Every byte ends as the copier or the early writer left it.
    for (int threads : {1, 4}) {
        for (bool huge : {false, true}) {
            rsp::Prefaulter pf(threads, huge);
            for (int job = 0; job < (rounds > 4 ? 12 : 4); ++job) {
                const size_t sizes[3] = {(size_t)(5u << 20) + 4097u, (size_t)(1u << 20) + 13u, (size_t)(3u << 20) + 1u};
                char* maps[3];
                char* base[3];
                std::vector<std::pair<void*, size_t>> ranges;
                for (int r = 0; r < 3; ++r) {
                    maps[r] = (char*)mmap(nullptr, sizes[r] + 8192, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
                    CHECK(maps[r] != MAP_FAILED, "mmap");
                    base[r] = maps[r] + 8 + 512 * r + job;   // unaligned starts
                    // an early writer: every 7th page's first bytes before the job begins
                    for (size_t o = 0; o < sizes[r]; o += 7 * 4096) base[r][o] = (char)(0x5a + r);
                    ranges.push_back({base[r], sizes[r]});
                }
                const bool abandon = job % 3 == 2;
                pf.begin(ranges);
                auto copier = [&](int r) {
                    const size_t piece = 700000 + 1000 * (size_t)r;
                    const size_t lim = abandon ? sizes[r] / 3 : sizes[r];
                    for (size_t o = 0; o < lim; o += piece) {
                        const size_t n = lim - o < piece ? lim - o : piece;
                        pf.wait(base[r] + o, n);
                        std::memset(base[r] + o, (char)(r + 1), n);
                    }
                };
                std::thread t0([&] { copier(0); copier(2); });
                std::thread t1([&] { copier(1); });
                t0.join();
                t1.join();
                pf.end();
                for (int r = 0; r < 3; ++r) {
                    const size_t lim = abandon ? sizes[r] / 3 : sizes[r];
                    bool ok = true;
                    for (size_t o = 0; o < sizes[r] && ok; o += 997)
                        ok = o < lim ? base[r][o] == (char)(r + 1)
                                     : (base[r][o] == ((o % (7 * 4096)) == 0 ? (char)(0x5a + r) : (char)0));
                    CHECK(ok, "prefault t%d huge%d job%d range%d", threads, (int)huge, job, r);
                    munmap(maps[r], sizes[r] + 8192);
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
