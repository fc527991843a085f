// rsp_hostpool.h -- host-side helpers of the pipelined host-buffer entry points
// (rsp_pc_mtd_cfar / rsp_pc_mtd with MATLAB's pageable arrays): a small persistent thread pool
// for the pageable <-> pinned staging copies.  One memcpy thread reads and writes host DRAM at
// ~10 GB/s, well below a PCIe Gen5 x16 DMA, so each staging piece is split over the pool.
#pragma once
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace rsp {

class CopyPool {
public:
    explicit CopyPool(int threads) : n_(threads < 1 ? 1 : threads) {
        for (int i = 1; i < n_; ++i) workers_.emplace_back([this, i] { loop(i); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& w : workers_) w.join();
    }
    int threads() const { return n_; }

    // memcpy(dst, src, bytes) split into n_ page-aligned parts; the caller runs part 0 and
    // returns when every part is done.  Small copies stay on the calling thread.
    void copy(void* dst, const void* src, size_t bytes) {
        if (n_ == 1 || bytes < (size_t)kMinSplit) {
            std::memcpy(dst, src, bytes);
            return;
        }
        size_t per = (bytes + n_ - 1) / n_;
        per = (per + 4095) & ~(size_t)4095;
        {
            std::lock_guard<std::mutex> g(m_);
            dst_ = (char*)dst;
            src_ = (const char*)src;
            bytes_ = bytes;
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
    void part(int i) {
        const size_t a = (size_t)i * per_;
        if (a >= bytes_) return;
        const size_t b = a + per_ < bytes_ ? a + per_ : bytes_;
        std::memcpy(dst_ + a, src_ + a, b - a);
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
    char* dst_ = nullptr;
    const char* src_ = nullptr;
    size_t bytes_ = 0, per_ = 0;
};

}  // namespace rsp
