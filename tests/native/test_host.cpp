// Host-side unit test of libstorbec's C++ helpers (no HIP): GF matrices and the
// staging copy pool.  Built by tests/test_native_host.py with g++ under
// AddressSanitizer + UBSan and, separately, ThreadSanitizer (the pool's threads).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "copy_pool.hpp"
#include "gf_host.hpp"

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
    sec::CopyPool pool(5);
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
        pool.run(jobs);
        for (int j = 0; j < njobs; ++j)
            EXPECT(src[j] == dst[j]);
    }
}

int main()
{
    test_matrices();
    test_copy_pool();
    if (fails)
        return 1;
    printf("native host tests ok\n");
    return 0;
}
