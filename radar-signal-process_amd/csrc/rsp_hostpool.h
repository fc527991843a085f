// rsp_hostpool.h -- host-side helpers of the pipelined host-buffer entry points
// (rsp_pc_mtd_cfar / rsp_pc_mtd with MATLAB's pageable arrays): a small persistent thread pool
// for the pageable <-> pinned staging copies.  One memcpy thread moves 20-30 GB/s of host DRAM,
// 8 threads ~130 GB/s (profiles/r04/probe1/pcie_probe.txt), against ~57 GB/s of PCIe Gen5 DMA
// per direction, so each staging piece is split over the pool.
//
// A one-CPI call (the MEX granularity) runs the pool ~8 times for ~1 MiB each, so the hand-off
// itself is on the critical path: a condition-variable wake costs several microseconds per
// worker.  Workers therefore spin on the job generation for kSpinUs after their last part before
// they block, and the caller spins on the pending count while the parts run.  The conversions
// write with streaming (non-temporal) stores: the destination -- pinned staging or the caller's
// fresh output array -- is not read back by this thread, so the store skips the cache line fill.
#pragma once
#include <emmintrin.h>
#include <sys/mman.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace rsp {

class CopyPool {
public:
    // Thread creation can throw (std::system_error / bad_alloc): the threads already started are
    // stopped and joined before the exception leaves, so no joinable std::thread is destroyed.
    explicit CopyPool(int threads) : n_(threads < 1 ? 1 : threads) {
        try {
            workers_.reserve((size_t)n_);
            for (int i = 1; i < n_; ++i) workers_.emplace_back([this, i] { loop(i); });
        } catch (...) {
            stop_all();
            throw;
        }
    }
    ~CopyPool() { stop_all(); }
    int threads() const { return n_; }

    // memcpy(dst, src, bytes) split into n_ page-aligned parts; the caller runs part 0 and
    // returns when every part is done.  Small copies stay on the calling thread.
    void copy(void* dst, const void* src, size_t bytes) {
        char* d = (char*)dst;
        const char* sp = (const char*)src;
        run(bytes, 4096, [=](size_t a, size_t b) { std::memcpy(d + a, sp + a, b - a); });
    }

    // complex double -> complex float (MATLAB's C128 echo -> the chain's C64), `n` complex
    // samples: cvtpd2ps rounds to nearest-even under the default MXCSR exactly as the (float)
    // cast (cvtsd2ss) and the GPU's v_cvt_f32_f64, so the chain sees the same samples as when it
    // converts on the device.
    void narrow_c128(float* dst, const double* src, size_t n) {
        run(n, 512, [=](size_t a, size_t b) { narrow_nt(dst + 2 * a, src + 2 * a, 2 * (b - a)); });
    }

    // MATLAB's output types: float RDM cells and 0/1 flag bytes widened to double (exact), and
    // a real double input narrowed to float (round to nearest, as the (float) cast on the GPU)
    void widen_f32(double* dst, const float* src, size_t n) {
        run(n, 1024, [=](size_t a, size_t b) {
            double* d = dst + a;
            const float* s = src + a;
            size_t m = b - a, i = 0;
            for (; i < m && ((uintptr_t)(d + i) & 15u) != 0; ++i) d[i] = (double)s[i];
            for (; i + 4 <= m; i += 4) {
                const __m128 v = _mm_loadu_ps(s + i);
                _mm_stream_pd(d + i, _mm_cvtps_pd(v));
                _mm_stream_pd(d + i + 2, _mm_cvtps_pd(_mm_movehl_ps(v, v)));
            }
            for (; i < m; ++i) d[i] = (double)s[i];
            _mm_sfence();
        });
    }
    void narrow_f64(float* dst, const double* src, size_t n) {
        run(n, 1024, [=](size_t a, size_t b) { narrow_nt(dst + a, src + a, b - a); });
    }
    void widen_u8(double* dst, const uint8_t* src, size_t n) {
        run(n, 4096, [=](size_t a, size_t b) {
            double* d = dst + a;
            const uint8_t* s = src + a;
            size_t m = b - a, i = 0;
            for (; i < m && ((uintptr_t)(d + i) & 15u) != 0; ++i) d[i] = (double)s[i];
            for (; i + 2 <= m; i += 2) _mm_stream_pd(d + i, _mm_set_pd((double)s[i + 1], (double)s[i]));
            for (; i < m; ++i) d[i] = (double)s[i];
            _mm_sfence();
        });
    }

    // fn(begin, end) over [0, n) in n_ parts aligned to `align` elements; the caller runs part 0
    void run(size_t n, size_t align, const std::function<void(size_t, size_t)>& fn) {
        if (n_ == 1 || n * 8 < (size_t)kMinSplit) {
            fn(0, n);
            return;
        }
        size_t per = (n + n_ - 1) / n_;
        per = (per + align - 1) / align * align;
        fn_ = &fn;
        n_items_ = n;
        per_ = per;
        pending_.store(n_ - 1, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> g(m_);
            gen_.fetch_add(1, std::memory_order_release);   // publishes fn_ / n_items_ / per_
        }
        if (sleepers_.load(std::memory_order_acquire) > 0) cv_.notify_all();
        part(0);
        for (unsigned spins = 0; pending_.load(std::memory_order_acquire) != 0; ++spins) {
            _mm_pause();
            if ((spins & 0xffffu) == 0xffffu) std::this_thread::yield();   // a descheduled worker
        }
    }

private:
    static constexpr int kMinSplit = 1 << 20;
    static constexpr int kSpinUs = 200;   // workers spin this long after a part before blocking

    // count doubles -> floats, streaming stores where the destination is 16-byte aligned
    static void narrow_nt(float* d, const double* s, size_t m) {
        size_t i = 0;
        for (; i < m && ((uintptr_t)(d + i) & 15u) != 0; ++i) d[i] = (float)s[i];
        for (; i + 4 <= m; i += 4) {
            const __m128 lo = _mm_cvtpd_ps(_mm_loadu_pd(s + i));
            const __m128 hi = _mm_cvtpd_ps(_mm_loadu_pd(s + i + 2));
            _mm_stream_ps(d + i, _mm_movelh_ps(lo, hi));
        }
        for (; i < m; ++i) d[i] = (float)s[i];
        _mm_sfence();
    }

    void stop_all() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_.store(true, std::memory_order_release);
        }
        cv_.notify_all();
        for (auto& w : workers_)
            if (w.joinable()) w.join();
        workers_.clear();
    }
    void part(int i) {
        const size_t a = (size_t)i * per_;
        if (a >= n_items_) return;
        const size_t b = a + per_ < n_items_ ? a + per_ : n_items_;
        (*fn_)(a, b);
    }
    void loop(int i) {
        // (generation 0, not the current value: a worker that starts after the first run() was
        // published must still take that job)
        uint64_t seen = 0;
        for (;;) {
            // spin phase: a new job usually follows within microseconds during a call
            const auto t0 = std::chrono::steady_clock::now();
            for (unsigned spins = 0; gen_.load(std::memory_order_acquire) == seen && !stop_.load(std::memory_order_acquire);
                 ++spins) {
                _mm_pause();
                if ((spins & 255u) == 255u &&
                    std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(kSpinUs))
                    break;
            }
            if (gen_.load(std::memory_order_acquire) == seen && !stop_.load(std::memory_order_acquire)) {
                std::unique_lock<std::mutex> lk(m_);
                sleepers_.fetch_add(1, std::memory_order_acq_rel);
                cv_.wait(lk, [&] { return stop_.load(std::memory_order_acquire) || gen_.load(std::memory_order_acquire) != seen; });
                sleepers_.fetch_sub(1, std::memory_order_acq_rel);
            }
            if (stop_.load(std::memory_order_acquire)) return;
            seen = gen_.load(std::memory_order_acquire);
            part(i);
            pending_.fetch_sub(1, std::memory_order_acq_rel);
        }
    }
    int n_;
    std::vector<std::thread> workers_;
    std::mutex m_;
    std::condition_variable cv_;
    std::atomic<bool> stop_{false};
    std::atomic<uint64_t> gen_{0};
    std::atomic<int> pending_{0};
    std::atomic<int> sleepers_{0};
    const std::function<void(size_t, size_t)>* fn_ = nullptr;
    size_t n_items_ = 0, per_ = 0;
};

// Prefault of the caller's output arrays while the call's input staging, DMA and chain run.
// A caller that hands in new arrays (numpy.empty / mxCreateUninitNumericMatrix of ~100 MB:
// fresh anonymous mappings) pays one page fault and one page zeroing per 4 KiB the first time
// the copy threads write there -- 32 CPIs per call at c3 ran at 1.9k CPI/s with new arrays
// against 5.7k with reused ones.  Here `threads` dedicated workers walk the
// output ranges in 2 MiB-aligned blocks, in order, from the start of the call, and fault each
// page in by a write that keeps its contents (a locked `or 0` of one byte per page, inside the
// range); the ranges' whole 2 MiB extents are first advised MADV_HUGEPAGE (`huge`), so one
// fault maps and zeroes 2 MiB.  Before the copy threads write a host range, wait() makes sure
// its blocks are done, faulting any block no worker has claimed yet itself, so the delivery is
// never slower than faulting in place.  Host probe (tools/micro/prefault_probe.cpp, 100 MiB of
// fresh memory, the GPU box): per-page touch 6.8 / 14.9 GB/s on 1 / 4 threads, with MADV_HUGEPAGE
// 25 / 74-77 GB/s (MADV_POPULATE_WRITE: 16-38 GB/s); in this container populate does not scale
// at all (2.4-2.7 GB/s), the touch does.  The same probe times the release: munmap of that memory
// costs 4.6 / 7.3 / 9.0 ms on the box when 1 / 4 / 8 threads faulted it -- the caller's cost of
// freeing new arrays, which no prefault removes.
class Prefaulter {
public:
    static constexpr size_t kBlock = 2u << 20;
    Prefaulter(int threads, bool huge) : n_(threads < 1 ? 1 : threads), huge_(huge) {
        try {
            workers_.reserve((size_t)n_);
            for (int i = 0; i < n_; ++i) workers_.emplace_back([this] { loop(); });
        } catch (...) {
            stop_all();
            throw;
        }
    }
    ~Prefaulter() { stop_all(); }

    // Begin faulting in `ranges` (host pointer, bytes) in order.  The previous job must be done
    // (end() was called).
    void begin(const std::vector<std::pair<void*, size_t>>& ranges) {
        blocks_.clear();
        for (const auto& r : ranges) {
            const uintptr_t a = (uintptr_t)r.first, e = a + r.second;
            if (huge_) {   // the range's whole 2 MiB extents (advice only: errors are ignored)
                const uintptr_t h0 = (a + kBlock - 1) & ~(uintptr_t)(kBlock - 1), h1 = e & ~(uintptr_t)(kBlock - 1);
                if (h1 > h0) (void)madvise((void*)h0, (size_t)(h1 - h0), MADV_HUGEPAGE);
            }
            for (uintptr_t b = a; b < e;) {
                const uintptr_t nb = (b & ~(uintptr_t)(kBlock - 1)) + kBlock;
                blocks_.push_back({b, nb < e ? nb : e});
                b = nb;
            }
        }
        state_.reset(new std::atomic<int>[blocks_.size() ? blocks_.size() : 1]);
        for (size_t i = 0; i < blocks_.size(); ++i) state_[i].store(0, std::memory_order_relaxed);
        next_.store(0, std::memory_order_relaxed);
        cancel_.store(false, std::memory_order_relaxed);
        active_.store(n_, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> g(m_);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
    }
    // Every block overlapping [p, p + n) is populated when this returns.
    void wait(const void* p, size_t n) {
        const uintptr_t a = (uintptr_t)p, e = a + n;
        for (size_t i = 0; i < blocks_.size(); ++i) {
            if (blocks_[i].e <= a || blocks_[i].a >= e) continue;
            int expect = 0;
            if (state_[i].compare_exchange_strong(expect, 1, std::memory_order_acq_rel)) {
                populate(blocks_[i]);   // no worker had it: populate it here
                state_[i].store(2, std::memory_order_release);
            }
            while (state_[i].load(std::memory_order_acquire) != 2) _mm_pause();
        }
    }
    // The job is over (done, or abandoned on an error): workers stop claiming, and this returns
    // once none of them still touches the ranges -- the caller may then free its arrays.
    void end() {
        cancel_.store(true, std::memory_order_release);
        while (active_.load(std::memory_order_acquire) != 0) _mm_pause();
    }

private:
    struct Blk {
        uintptr_t a, e;
    };
    // one write fault per page of [b.a, b.e), contents kept: a locked `or 0` of the block's first
    // byte and of each later page's first byte (all inside the caller's range)
    static void populate(const Blk& b) {
        for (uintptr_t q = b.a; q < b.e; q = (q & ~(uintptr_t)4095) + 4096)
            __atomic_fetch_or((char*)q, (char)0, __ATOMIC_RELAXED);
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || gen_.load(std::memory_order_acquire) != seen; });
                if (stop_) return;
                seen = gen_.load(std::memory_order_acquire);
            }
            for (;;) {
                if (cancel_.load(std::memory_order_acquire)) break;
                const size_t i = next_.fetch_add(1, std::memory_order_acq_rel);
                if (i >= blocks_.size()) break;
                int expect = 0;
                if (!state_[i].compare_exchange_strong(expect, 1, std::memory_order_acq_rel)) continue;
                populate(blocks_[i]);
                state_[i].store(2, std::memory_order_release);
            }
            active_.fetch_sub(1, std::memory_order_acq_rel);
        }
    }
    void stop_all() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& w : workers_)
            if (w.joinable()) w.join();
        workers_.clear();
    }
    int n_;
    std::vector<std::thread> workers_;
    std::mutex m_;
    std::condition_variable cv_;
    bool stop_ = false;
    std::atomic<uint64_t> gen_{0};
    std::vector<Blk> blocks_;
    std::unique_ptr<std::atomic<int>[]> state_;   // per block: 0 free, 1 being populated, 2 done
    std::atomic<size_t> next_{0};
    std::atomic<bool> cancel_{false};
    std::atomic<int> active_{0};
    bool huge_;
};

}  // namespace rsp
