// copy_pool.hpp — persistent host threads for staging copies (pinned <-> caller memory).
//
// Host-buffer calls (SEC_F_HOST) gather the caller's chunks / blocks into pinned
// slabs and scatter results back; one core's memcpy (~10 GB/s) would cap the
// end-to-end rate well below PCIe Gen5, so copies are cut into <= 1 MiB pieces
// and spread over a few threads (the calling thread works too).
#pragma once
#include <stddef.h>
#include <string.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

namespace sec {

struct CopyJob {
    void *dst;
    const void *src;  // nullptr: zero-fill dst (a decode block's bytes past its avail)
    size_t len;
};

inline void copy_or_zero(void *dst, const void *src, size_t len)
{
    if (src)
        memcpy(dst, src, len);
    else
        memset(dst, 0, len);
}

class CopyPool {
public:
    explicit CopyPool(int nthreads)
    {
        for (int i = 0; i < nthreads; ++i)
            threads_.emplace_back([this] { worker(); });
    }
    ~CopyPool()
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : threads_)
            t.join();
    }
    CopyPool(const CopyPool &) = delete;
    CopyPool &operator=(const CopyPool &) = delete;

    // Runs every job; returns when all bytes are copied.
    void run(const std::vector<CopyJob> &jobs)
    {
        size_t total = 0;
        for (const auto &j : jobs)
            total += j.len;
        if (threads_.empty() || total < kInline) {
            for (const auto &j : jobs)
                if (j.len)  // memcpy's pointers must be valid even for 0 bytes
                    copy_or_zero(j.dst, j.src, j.len);
            return;
        }
        {
            // workers only touch pieces_ while counted in active_, so it is rebuilt
            // with none of them inside drain()
            std::unique_lock<std::mutex> lk(mu_);
            done_cv_.wait(lk, [this] { return active_ == 0; });
            pieces_.clear();
            for (const auto &j : jobs)
                for (size_t o = 0; o < j.len; o += kPiece) {
                    const size_t n = j.len - o < kPiece ? j.len - o : kPiece;
                    pieces_.push_back(CopyJob{(char *)j.dst + o, j.src ? (const char *)j.src + o : nullptr, n});
                }
            next_.store(0);
            left_.store(pieces_.size());
            ++gen_;
        }
        cv_.notify_all();
        drain();
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [this] { return left_.load() == 0 && active_ == 0; });
    }

private:
    static constexpr size_t kPiece = (size_t)1 << 20;
    static constexpr size_t kInline = (size_t)4 << 20;

    void drain()
    {
        for (;;) {
            const size_t i = next_.fetch_add(1);
            if (i >= pieces_.size())
                return;
            copy_or_zero(pieces_[i].dst, pieces_[i].src, pieces_[i].len);
            if (left_.fetch_sub(1) == 1) {
                std::lock_guard<std::mutex> lk(mu_);
                done_cv_.notify_all();
            }
        }
    }

    void worker()
    {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_)
                    return;
                seen = gen_;
                ++active_;
            }
            drain();
            {
                std::lock_guard<std::mutex> lk(mu_);
                --active_;
            }
            done_cv_.notify_all();
        }
    }

    std::vector<std::thread> threads_;
    std::vector<CopyJob> pieces_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::atomic<size_t> next_{0}, left_{0};
    uint64_t gen_ = 0;
    int active_ = 0;
    bool stop_ = false;
};

}  // namespace sec
