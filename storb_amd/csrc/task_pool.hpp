// task_pool.hpp — persistent host threads for the piece work around an encode call
// (sec_encode_pieces): the data pieces' copies and SHA-1 piece ids run on these threads while
// the calling thread drives the GPU, the parity pieces' right after.  Unlike CopyPool (one
// blocking batch of copies at a time) tasks are queued asynchronously in groups, and the
// thread that waits on a group runs queued tasks itself until the group is done.
//
// SHA-1 is OpenSSL's (libcrypto's EVP, the implementation CPython's hashlib uses, with the
// SHA extensions where the CPU has them), so a piece id is byte for byte
// hashlib.sha1(piece).hexdigest() (/root/reference/storb/util/piece.py:54-68).
#pragma once
#include <openssl/evp.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

namespace sec {

// SHA-1 of a `len`-byte message whose first `avail` bytes are at p and the rest zero (zfec's
// padded last data block hashed as the piece it becomes).  False on an OpenSSL failure.
inline bool sha1_padded(const uint8_t *p, size_t avail, size_t len, uint8_t out[20])
{
    static const EVP_MD *md = EVP_sha1();
    EVP_MD_CTX *c = EVP_MD_CTX_new();
    if (!c)
        return false;
    bool ok = EVP_DigestInit_ex(c, md, nullptr) == 1;
    if (ok && avail)
        ok = EVP_DigestUpdate(c, p, avail < len ? avail : len) == 1;
    static const uint8_t zeros[4096] = {};
    for (size_t z = avail < len ? len - avail : 0; ok && z > 0;) {
        const size_t n = z < sizeof(zeros) ? z : sizeof(zeros);
        ok = EVP_DigestUpdate(c, zeros, n) == 1;
        z -= n;
    }
    unsigned int olen = 0;
    if (ok)
        ok = EVP_DigestFinal_ex(c, out, &olen) == 1 && olen == 20;
    EVP_MD_CTX_free(c);
    return ok;
}

class TaskPool {
public:
    struct Group {
        std::atomic<int64_t> left{0};
        std::atomic<bool> failed{false};
    };

    explicit TaskPool(int nthreads)
    {
        for (int i = 0; i < nthreads; ++i)
            threads_.emplace_back([this] { worker(); });
    }
    ~TaskPool()
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : threads_)
            t.join();
    }
    TaskPool(const TaskPool &) = delete;
    TaskPool &operator=(const TaskPool &) = delete;

    // f returns false on failure (recorded in the group)
    void submit(Group &g, std::function<bool()> f)
    {
        g.left.fetch_add(1);
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.emplace_back(&g, std::move(f));
        }
        cv_.notify_one();
    }

    // Runs queued tasks (of any group) until g's are all done; true when none failed.
    bool wait(Group &g)
    {
        while (g.left.load() > 0) {
            std::pair<Group *, std::function<bool()>> t;
            {
                std::unique_lock<std::mutex> lk(mu_);
                if (q_.empty()) {
                    done_cv_.wait(lk, [&] { return g.left.load() == 0 || !q_.empty(); });
                    continue;
                }
                t = std::move(q_.front());
                q_.pop_front();
            }
            run(t);
        }
        return !g.failed.load();
    }

private:
    void run(std::pair<Group *, std::function<bool()>> &t)
    {
        if (!t.second())
            t.first->failed.store(true);
        if (t.first->left.fetch_sub(1) == 1) {
            std::lock_guard<std::mutex> lk(mu_);
            done_cv_.notify_all();
        }
    }

    void worker()
    {
        for (;;) {
            std::pair<Group *, std::function<bool()>> t;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
                if (stop_ && q_.empty())
                    return;
                t = std::move(q_.front());
                q_.pop_front();
            }
            run(t);
        }
    }

    std::vector<std::thread> threads_;
    std::deque<std::pair<Group *, std::function<bool()>>> q_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    bool stop_ = false;
};

}  // namespace sec
