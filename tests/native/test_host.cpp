// Host-side unit test of libstorbec's C++ helpers (no HIP): GF matrices, the staging copy
// pool, and the task pool + SHA-1 of sec_encode_pieces.  Built by tests/test_native_host.py
// with g++ under AddressSanitizer + UBSan and, separately, ThreadSanitizer (the pools' threads).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <memory>
#include <random>
#include <thread>
#include <vector>

#include "gf_host.hpp"
#include "task_pool.hpp"

static int fails = 0;
#define EXPECT(c)                                                        \
    do {                                                                 \
        if (!(c)) {                                                      \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                     \
        }                                                                \
    } while (0)

static void test_matrices()
{
    const sec::Gf &g = sec::gf();
    const std::vector<uint8_t> e = sec::encode_matrix(4, 6);
    const uint8_t want[8] = {0x77, 0x40, 0x38, 0x0e, 0xc7, 0xa7, 0x0d, 0x6c};
    EXPECT(memcmp(e.data() + 16, want, 8) == 0);
    for (int k : {1, 2, 5, 10, 32, 64}) {
        const int m = std::min(256, k + k / 2 + 1);
        const std::vector<uint8_t> enc = sec::encode_matrix(k, m);
        // any k rows (here: the last k) form an invertible matrix whose inverse is exact
        std::vector<int> idx;
        for (int i = 0; i < k; ++i)
            idx.push_back(m - k + i);
        std::vector<int> perm;
        sec::normalise_slots(k, idx, perm);
        for (int i = 0; i < k; ++i)
            EXPECT(idx[i] >= k || idx[i] == i);
        std::vector<uint8_t> minv;
        EXPECT(sec::decode_matrix(k, m, idx, minv));
        for (int r = 0; r < k; ++r)
            for (int c = 0; c < k; ++c) {
                uint8_t s = 0;
                for (int t = 0; t < k; ++t) {
                    const uint8_t a = idx[r] < k ? (uint8_t)(t == r) : enc[(size_t)idx[r] * k + t];
                    s ^= g.mul(a, minv[(size_t)t * k + c]);
                }
                EXPECT(s == (r == c ? 1 : 0));
            }
    }
}

static void test_copy_pool()
{
    std::mt19937_64 rng(7);
    sec::TaskPool pool(5);
    for (int round = 0; round < 40; ++round) {
        const int njobs = 1 + (int)(rng() % 40);
        std::vector<std::vector<char>> src(njobs), dst(njobs);
        std::vector<sec::CopyJob> jobs;
        for (int j = 0; j < njobs; ++j) {
            const size_t n = rng() % (round % 3 == 0 ? 64 : (3 << 20));
            src[j].resize(n);
            dst[j].assign(n, 0);
            for (size_t i = 0; i < n; i += 4096)
                src[j][i] = (char)rng();
            jobs.push_back(sec::CopyJob{dst[j].data(), src[j].data(), n});
        }
        pool.run_copies(jobs);
        for (int j = 0; j < njobs; ++j)
            EXPECT(src[j] == dst[j]);
    }
}

// copies from several threads at once through one shared pool (contexts of one process share it)
static void test_shared_pool_concurrent()
{
    std::shared_ptr<sec::TaskPool> a = sec::shared_pool(4), b = sec::shared_pool(4);
    EXPECT(a.get() == b.get());
    EXPECT(sec::shared_pool(3).get() != a.get());
    EXPECT(sec::usable_cpus() >= 1);
    EXPECT(sec::default_pool_threads() >= 1 && sec::default_pool_threads() <= 7 &&
           sec::default_pool_threads() <= std::max(1, sec::usable_cpus() / 2));
    std::vector<std::thread> th;
    std::atomic<int> bad{0};
    for (int t = 0; t < 6; ++t)
        th.emplace_back([&, t] {
            std::mt19937_64 rng(100 + t);
            for (int round = 0; round < 6; ++round) {
                const size_t n = (5u << 20) + rng() % (3u << 20);
                std::vector<char> src(n), dst(n, 0), zero(n, 1);
                for (size_t i = 0; i < n; i += 512)
                    src[i] = (char)rng();
                a->run_copies({sec::CopyJob{dst.data(), src.data(), n}, sec::CopyJob{zero.data(), nullptr, n}});
                if (dst != src || zero != std::vector<char>(n, 0))
                    ++bad;
            }
        });
    for (auto &x : th)
        x.join();
    EXPECT(bad.load() == 0);
}

static void test_task_pool_sha1()
{
    // known answers (FIPS 180-1): "abc", and the empty message
    uint8_t d[20];
    const uint8_t abc[20] = {0xa9, 0x99, 0x3e, 0x36, 0x47, 0x06, 0x81, 0x6a, 0xba, 0x3e,
                             0x25, 0x71, 0x78, 0x50, 0xc2, 0x6c, 0x9c, 0xd0, 0xd8, 0x9d};
    EXPECT(sec::sha1_padded((const uint8_t *)"abc", 3, 3, d) && memcmp(d, abc, 20) == 0);
    const uint8_t empty[20] = {0xda, 0x39, 0xa3, 0xee, 0x5e, 0x6b, 0x4b, 0x0d, 0x32, 0x55,
                               0xbf, 0xef, 0x95, 0x60, 0x18, 0x90, 0xaf, 0xd8, 0x07, 0x09};
    EXPECT(sec::sha1_padded(nullptr, 0, 0, d) && memcmp(d, empty, 20) == 0);
    // the padded form equals the hash of the explicitly zero-padded bytes, from many threads
    std::mt19937_64 rng(11);
    sec::TaskPool pool(6);
    for (int round = 0; round < 8; ++round) {
        const int n = 1 + (int)(rng() % 64);
        std::vector<std::vector<uint8_t>> msg(n);
        std::vector<size_t> avail(n);
        std::vector<uint8_t> got((size_t)n * 20), want((size_t)n * 20);
        for (int i = 0; i < n; ++i) {
            const size_t len = rng() % (round % 2 ? 70000 : 300);
            avail[i] = len ? rng() % (len + 1) : 0;
            msg[i].assign(len, 0);
            for (size_t b = 0; b < avail[i]; ++b)
                msg[i][b] = (uint8_t)rng();
            EXPECT(sec::sha1_padded(msg[i].data(), len, len, &want[(size_t)i * 20]));
        }
        sec::TaskPool::Group g1, g2;
        for (int i = 0; i < n; ++i) {
            sec::TaskPool::Group &g = i % 2 ? g1 : g2;
            const uint8_t *p = msg[i].data();
            const size_t av = avail[i], len = msg[i].size();
            uint8_t *o = &got[(size_t)i * 20];
            pool.submit(g, [=] { return sec::sha1_padded(p, av, len, o); });
        }
        EXPECT(pool.wait(g1));
        EXPECT(pool.wait(g2));
        EXPECT(got == want);
    }
    sec::TaskPool::Group gf;  // a failing task is reported, the rest still run
    std::atomic<int> ran{0};
    for (int i = 0; i < 20; ++i)
        pool.submit(gf, [&ran, i] { ++ran; return i != 7; });
    EXPECT(!pool.wait(gf));
    EXPECT(ran.load() == 20);
}

int main()
{
    test_matrices();
    test_copy_pool();
    test_shared_pool_concurrent();
    test_task_pool_sha1();
    if (fails)
        return 1;
    printf("native host tests ok\n");
    return 0;
}
