// rsp_hostpool.h -- host-side helpers of the pipelined host-buffer entry points
// (rsp_pc_mtd_cfar / rsp_pc_mtd with MATLAB's pageable arrays): a small persistent thread pool
// for the pageable <-> pinned staging copies.  One memcpy thread moves 20-30 GB/s of host DRAM,
// 8 threads ~130 GB/s (profiles/r04/probe1/pcie_probe.txt), against ~57 GB/s of PCIe Gen5 DMA
// per direction, so each staging piece is split over the pool.
#pragma once
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
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
    // samples: the (float) casts round to nearest-even exactly as the GPU's v_cvt_f32_f64, so the
    // chain sees the same samples as when it converts on the device.
    void narrow_c128(float* dst, const double* src, size_t n) {
        run(n, 512, [=](size_t a, size_t b) {
            for (size_t i = 2 * a; i < 2 * b; ++i) dst[i] = (float)src[i];
        });
    }

    // MATLAB's output types: float RDM cells and 0/1 flag bytes widened to double (exact), and
    // a real double input narrowed to float (round to nearest, as the (float) cast on the GPU)
    void widen_f32(double* dst, const float* src, size_t n) {
        run(n, 1024, [=](size_t a, size_t b) {
            for (size_t i = a; i < b; ++i) dst[i] = (double)src[i];
        });
    }
    void narrow_f64(float* dst, const double* src, size_t n) {
        run(n, 1024, [=](size_t a, size_t b) {
            for (size_t i = a; i < b; ++i) dst[i] = (float)src[i];
        });
    }
    void widen_u8(double* dst, const uint8_t* src, size_t n) {
        run(n, 4096, [=](size_t a, size_t b) {
            for (size_t i = a; i < b; ++i) dst[i] = (double)src[i];
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
        {
            std::lock_guard<std::mutex> g(m_);
            fn_ = &fn;
            n_items_ = n;
            per_ = per;
            pending_ = n_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        part(0);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return pending_ == 0; });
    }

private:
    static constexpr int kMinSplit = 1 << 20;
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
    void part(int i) {
        const size_t a = (size_t)i * per_;
        if (a >= n_items_) return;
        const size_t b = a + per_ < n_items_ ? a + per_ : n_items_;
        (*fn_)(a, b);
    }
    void loop(int i) {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            part(i);
            {
                std::lock_guard<std::mutex> g(m_);
                if (--pending_ == 0) done_.notify_one();
            }
        }
    }
    int n_;
    std::vector<std::thread> workers_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    bool stop_ = false;
    uint64_t gen_ = 0;
    int pending_ = 0;
    const std::function<void(size_t, size_t)>* fn_ = nullptr;
    size_t n_items_ = 0, per_ = 0;
};

}  // namespace rsp
