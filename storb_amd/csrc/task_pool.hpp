// task_pool.hpp — the library's host threads: one pool per process (per thread count), shared by
// every context, for the host work around the GPU calls:
//  - sec_encode_pieces: the data pieces' copies and SHA-1 piece ids run on these threads while
//    the calling thread drives the GPU, the parity pieces' right after;
//  - the staged host paths: gathers into / scatters out of the pinned slabs and the decode's host
//    joins (run_copies: a batch of copies cut into <= 1 MiB tasks; one core's memcpy, ~10 GB/s,
//    would cap the end-to-end rate well below PCIe Gen5).
// Tasks are queued in groups; a thread that waits on a group runs queued tasks itself until the
// group is done, so a caller never idles while its own work is queued.  The pool is sized from
// the CPUs this process may actually use (affinity mask and cgroup quota, as storb_amd/piece.py
// _usable_cpus), and shared: a validator calling from a thread pool (one context per thread)
// gets one set of threads, not one per context.
//
// SHA-1 is OpenSSL's (libcrypto's EVP, the implementation CPython's hashlib uses, with the
// SHA extensions where the CPU has them), so a piece id is byte for byte
// hashlib.sha1(piece).hexdigest() (/root/reference/storb/util/piece.py:54-68).
#pragma once
#include <openssl/evp.h>
#include <sched.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <new>
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

class TaskPool {
public:
    struct Group {
        std::atomic<int64_t> left{0};
        std::atomic<bool> failed{false};
    };

    explicit TaskPool(int nthreads)
    {
        for (int i = 0; i < nthreads; ++i) {
            try {
                threads_.emplace_back([this] { worker(); });
            } catch (...) {  // fewer threads (none: callers run every task themselves in wait)
                break;
            }
        }
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

    int threads() const { return (int)threads_.size(); }

    // f returns false on failure (recorded in the group).  When the task cannot be queued (no
    // memory for its closure or queue node) it runs here, now: submit never throws, so the
    // extern "C" entry points above it cannot terminate the process on std::bad_alloc, and no
    // queued task is left pointing into a frame that unwound.
    template <class F>
    void submit(Group &g, const F &f) noexcept
    {
        g.left.fetch_add(1);
        try {
            std::function<bool()> fn(f);  // a copy: f stays whole for the fallback
            {
                std::lock_guard<std::mutex> lk(mu_);
                q_.emplace_back(&g, std::move(fn));
            }
            cv_.notify_one();
        } catch (...) {
            finish(g, run_inline(f));
        }
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

    // Every job's bytes, cut into <= 1 MiB tasks (a small batch runs on the calling thread);
    // returns when all are copied.  Safe from any number of threads at once.
    void run_copies(const std::vector<CopyJob> &jobs)
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
        Group g;
        for (const auto &j : jobs)
            for (size_t o = 0; o < j.len; o += kPiece) {
                const size_t n = j.len - o < kPiece ? j.len - o : kPiece;
                void *d = (char *)j.dst + o;
                const void *s = j.src ? (const char *)j.src + o : nullptr;
                submit(g, [d, s, n] {
                    copy_or_zero(d, s, n);
                    return true;
                });
            }
        wait(g);
    }

private:
    static constexpr size_t kPiece = (size_t)1 << 20;
    static constexpr size_t kInline = (size_t)4 << 20;

    template <class F>
    static bool run_inline(const F &f)
    {
        try {
            return f();
        } catch (...) {
            return false;
        }
    }

    void finish(Group &g, bool ok)
    {
        if (!ok)
            g.failed.store(true);
        if (g.left.fetch_sub(1) == 1) {
            std::lock_guard<std::mutex> lk(mu_);
            done_cv_.notify_all();
        }
    }

    void run(std::pair<Group *, std::function<bool()>> &t)
    {
        bool ok;
        try {
            ok = t.second();
        } catch (...) {
            ok = false;
        }
        finish(*t.first, ok);
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

// The cgroup CPU quota (v2 cpu.max "quota period", else v1 cfs_quota_us / cfs_period_us),
// rounded up; 0 when unlimited or unknown.
inline int cgroup_cpus()
{
    long long q = -1, p = 0;
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char qs[32] = {0};
        if (fscanf(f, "%31s %lld", qs, &p) == 2 && strcmp(qs, "max") != 0)
            q = atoll(qs);
        fclose(f);
    } else {
        FILE *fq = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r");
        FILE *fp = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r");
        if (fq && fp && (fscanf(fq, "%lld", &q) != 1 || fscanf(fp, "%lld", &p) != 1))
            q = -1;
        if (fq)
            fclose(fq);
        if (fp)
            fclose(fp);
    }
    if (q <= 0 || p <= 0)
        return 0;
    return (int)std::max(1LL, (q + p - 1) / p);
}

// CPUs this process may run on: the affinity mask, capped by the cgroup quota
inline int usable_cpus()
{
    int n = 0;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0)
        n = CPU_COUNT(&set);
    if (n <= 0)
        n = (int)std::max(1u, std::thread::hardware_concurrency());
    const int q = cgroup_cpus();
    return q > 0 ? std::min(n, q) : n;
}

// The default pool size: half the usable CPUs (the calling threads work too), at most 7.
// SEC_POOL_DIV / SEC_POOL_RESERVE / SEC_POOL_MAX (build knobs, A/B): min(MAX, usable / DIV -
// RESERVE).  Round 6 measured all but two of a 16-CPU quota (14 threads): the 1 GiB upload
// stream +17 to +49 %, but C5 end to end from pinned memory 47.3 -> 36.0 GiB/s (more runnable
// threads than the quota: the cgroup is throttled), profiles/r06_pool_threads_ab.txt.
#ifndef SEC_POOL_DIV
#define SEC_POOL_DIV 2
#endif
#ifndef SEC_POOL_RESERVE
#define SEC_POOL_RESERVE 0
#endif
#ifndef SEC_POOL_MAX
#define SEC_POOL_MAX 7
#endif
inline int default_pool_threads()
{
    return std::min(SEC_POOL_MAX, std::max(1, usable_cpus() / SEC_POOL_DIV - SEC_POOL_RESERVE));
}

// The process's pool of `nthreads` threads, created on first use and shared by every holder; it
// ends with its last holder.
inline std::shared_ptr<TaskPool> shared_pool(int nthreads)
{
    static std::mutex mu;
    static std::map<int, std::weak_ptr<TaskPool>> pools;
    std::lock_guard<std::mutex> lk(mu);
    std::weak_ptr<TaskPool> &w = pools[nthreads];
    std::shared_ptr<TaskPool> p = w.lock();
    if (!p) {
        p = std::make_shared<TaskPool>(nthreads);
        w = p;
    }
    return p;
}

}  // namespace sec
