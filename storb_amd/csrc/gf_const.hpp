// gf_const.hpp — GF(2^8) / 0x11D and zfec's systematic encode matrix as compile-time values,
// for the kernels whose coefficients are template constants (kernels_xb.hip, kernels_bs.hip).
// The run-time tables (gf_host.hpp) and the oracle (oracle/fec_oracle.c build_enc_matrix)
// compute the same matrix; SURVEY.md Appendix A restates zfec's construction.
#pragma once
#include <stdint.h>

namespace gfc {

struct Gf {
    uint8_t exp[512];
    uint8_t log[256];
};

constexpr Gf make_gf()
{
    Gf t{};
    uint32_t v = 1;
    for (int e = 0; e < 255; ++e) {
        t.exp[e] = (uint8_t)v;
        t.exp[e + 255] = (uint8_t)v;
        t.log[v] = (uint8_t)e;
        v <<= 1;
        if (v & 0x100)
            v ^= 0x11D;
    }
    t.exp[510] = t.exp[0];
    t.exp[511] = t.exp[1];
    return t;
}
inline constexpr Gf kGf = make_gf();
constexpr uint32_t gmul(uint32_t a, uint32_t b) { return (a && b) ? kGf.exp[kGf.log[a] + kGf.log[b]] : 0u; }
constexpr uint32_t ginv(uint32_t a) { return kGf.exp[255 - kGf.log[a]]; }
// zfec's evaluation points: p_0 = 0, p_i = alpha^(i-1)
constexpr uint32_t point(int i) { return i == 0 ? 0u : kGf.exp[(i - 1) % 255]; }

// Parity rows of zfec's encode matrix: c[r][j] = L_j(p_{k+r}), the Lagrange basis polynomial of
// point j over points 0..k-1 (the closed form of _invert_vdm + _matmul; SURVEY.md Appendix A,
// oracle/fec_oracle.c build_enc_matrix).
template <int K, int M>
struct EncMatrix {
    uint8_t c[M - K][K];
    constexpr EncMatrix() : c{}
    {
        uint32_t den[K] = {};  // prod over i != j of (p_j - p_i)
        for (int j = 0; j < K; ++j) {
            uint32_t d = 1;
            for (int i = 0; i < K; ++i)
                if (i != j)
                    d = gmul(d, point(j) ^ point(i));
            den[j] = d;
        }
        for (int r = 0; r < M - K; ++r) {
            const uint32_t P = point(K + r);
            uint32_t N = 1;  // prod over all i < K of (P - p_i)
            for (int i = 0; i < K; ++i)
                N = gmul(N, P ^ point(i));
            for (int j = 0; j < K; ++j)
                c[r][j] = (uint8_t)gmul(gmul(N, ginv(P ^ point(j))), ginv(den[j]));
        }
    }
};
// zfec(4,6) and (2,3) rows as restated in SURVEY.md Appendix A (and tests/golden)
static_assert(EncMatrix<4, 6>().c[0][0] == 0x77 && EncMatrix<4, 6>().c[0][3] == 0x0e, "zfec(4,6) row 0");
static_assert(EncMatrix<4, 6>().c[1][0] == 0xc7 && EncMatrix<4, 6>().c[1][3] == 0x6c, "zfec(4,6) row 1");
static_assert(EncMatrix<2, 3>().c[0][0] == 0x03 && EncMatrix<2, 3>().c[0][1] == 0x02, "zfec(2,3)");

template <int K, int M>
struct Matrix {
    static constexpr EncMatrix<K, M> v{};
};

}  // namespace gfc
