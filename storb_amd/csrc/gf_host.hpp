// gf_host.hpp — host-side GF(2^8) matrix arithmetic for the C ABI.
//
// O(k^3) set-up work only (the byte streams never touch the CPU):
//   * the systematic encode matrix zfec's fec_new builds (zfec 1.6.0.0, called
//     via easyfec.Encoder at /root/reference/storb/util/piece.py:129): seed
//     rows tmp[0] = [1,0..0], tmp[r][c] = alpha^((r-1)c mod 255), then
//     enc[k..m-1] = tmp[k..m-1] * inv(tmp[0..k-1])
//   * the decode matrix zfec's fec_decode inverts (easyfec.Decoder at
//     piece.py:196): row i = e_i for a primary in its own slot, enc[idx[i]]
//     for a secondary.
#pragma once
#include <stdint.h>
#include <string.h>

#include <vector>

namespace sec {

struct Gf {
    uint8_t exp[510];
    int log[256];
    uint8_t inv[256];
    Gf()
    {
        unsigned v = 1;
        for (int e = 0; e < 255; ++e) {
            exp[e] = exp[e + 255] = (uint8_t)v;
            log[v] = e;
            v <<= 1;
            if (v & 0x100)
                v ^= 0x11D;
        }
        log[0] = -1;
        inv[0] = 0;
        for (int a = 1; a < 256; ++a)
            inv[a] = exp[255 - log[a]];
    }
    uint8_t mul(uint8_t a, uint8_t b) const { return (a && b) ? exp[log[a] + log[b]] : 0; }
};

inline const Gf &gf()
{
    static const Gf g;
    return g;
}

// In-place inverse of a k x k row-major matrix; false if singular.
inline bool gf_invert(std::vector<uint8_t> &a, int k)
{
    const Gf &g = gf();
    std::vector<uint8_t> inv((size_t)k * k, 0);
    for (int i = 0; i < k; ++i)
        inv[(size_t)i * k + i] = 1;
    for (int c = 0; c < k; ++c) {
        int piv = c;
        while (piv < k && a[(size_t)piv * k + c] == 0)
            ++piv;
        if (piv == k)
            return false;
        if (piv != c)
            for (int t = 0; t < k; ++t) {
                std::swap(a[(size_t)piv * k + t], a[(size_t)c * k + t]);
                std::swap(inv[(size_t)piv * k + t], inv[(size_t)c * k + t]);
            }
        const uint8_t s = g.inv[a[(size_t)c * k + c]];
        for (int t = 0; t < k; ++t) {
            a[(size_t)c * k + t] = g.mul(a[(size_t)c * k + t], s);
            inv[(size_t)c * k + t] = g.mul(inv[(size_t)c * k + t], s);
        }
        for (int r = 0; r < k; ++r) {
            const uint8_t f = a[(size_t)r * k + c];
            if (r == c || f == 0)
                continue;
            for (int t = 0; t < k; ++t) {
                a[(size_t)r * k + t] ^= g.mul(f, a[(size_t)c * k + t]);
                inv[(size_t)r * k + t] ^= g.mul(f, inv[(size_t)c * k + t]);
            }
        }
    }
    a.swap(inv);
    return true;
}

// Full m x k encode matrix (identity on top).
inline std::vector<uint8_t> encode_matrix(int k, int m)
{
    const Gf &g = gf();
    std::vector<uint8_t> seed((size_t)m * k, 0), enc((size_t)m * k, 0);
    seed[0] = 1;
    for (int r = 1; r < m; ++r)
        for (int c = 0; c < k; ++c)
            seed[(size_t)r * k + c] = g.exp[((r - 1) * c) % 255];
    std::vector<uint8_t> top(seed.begin(), seed.begin() + (size_t)k * k);
    gf_invert(top, k);  // Vandermonde on distinct points: never singular
    for (int i = 0; i < k; ++i)
        enc[(size_t)i * k + i] = 1;
    for (int r = k; r < m; ++r)
        for (int c = 0; c < k; ++c) {
            uint8_t s = 0;
            for (int t = 0; t < k; ++t)
                s ^= g.mul(seed[(size_t)r * k + t], top[(size_t)t * k + c]);
            enc[(size_t)r * k + c] = s;
        }
    return enc;
}

// zfec _fecmodule.c normalisation: each primary moved into its own slot.
// perm[i] = caller's position of the block now in slot i.
inline void normalise_slots(int k, std::vector<int> &idx, std::vector<int> &perm)
{
    perm.resize(k);
    for (int i = 0; i < k; ++i)
        perm[i] = i;
    int i = 0;
    while (i < k) {
        if (idx[i] >= k || idx[i] == i) {
            ++i;
        } else {
            const int c = idx[i];
            std::swap(idx[i], idx[c]);
            std::swap(perm[i], perm[c]);
        }
    }
}

// zfec's evaluation points: p_0 = 0, p_i = alpha^(i-1) (the seed rows above)
inline uint8_t point(int i) { return i == 0 ? 0 : gf().exp[(i - 1) % 255]; }

// Scalings of the syndrome decode's Cauchy solve (kernels_bs.hip).  zfec's parity row r is the
// Lagrange basis at x_r = p_{k+r}: c[r][j] = a_r b_j / (x_r + y_j) with y_j = p_j,
// a_r = prod_{i<k} (x_r + y_i), b_j = 1 / prod_{i<k, i!=j} (y_j + y_i).  For the present parity
// rows S (ascending) and the lost data rows L (ascending), |S| = |L| = e, the e x e system
// A = c[S][L] = D_a C D_b has C a Cauchy matrix, whose inverse is again one up to diagonals, so
//     A^-1[l][r] = z_l c[r][l] w_r,
//     w_r = prod_{l in L} (x_r + y_l) / prod_{r' in S, r' != r} (x_r + x_r') / a_r^2,
//     z_l = prod_{r in S} (x_r + y_l) / prod_{l' in L, l' != l} (y_l + y_l') / b_l^2.
// Checked against a Gauss-Jordan inverse for every shape (tests/test_cauchy.py restates it).
inline void cauchy_scales(int k, const std::vector<int> &S, const std::vector<int> &Lost, std::vector<uint8_t> &w,
                          std::vector<uint8_t> &z)
{
    const Gf &g = gf();
    auto div = [&](uint8_t a, uint8_t b) { return g.mul(a, g.inv[b]); };
    const size_t e = S.size();
    w.assign(e, 0);
    z.assign(e, 0);
    for (size_t q = 0; q < e; ++q) {
        const uint8_t x = point(k + S[q]);
        uint8_t num = 1, den = 1, a = 1;
        for (int l : Lost)
            num = g.mul(num, x ^ point(l));
        for (size_t q2 = 0; q2 < e; ++q2)
            if (q2 != q)
                den = g.mul(den, x ^ point(k + S[q2]));
        for (int i = 0; i < k; ++i)
            a = g.mul(a, x ^ point(i));
        w[q] = div(div(num, den), g.mul(a, a));
    }
    for (size_t t = 0; t < e; ++t) {
        const uint8_t y = point(Lost[t]);
        uint8_t num = 1, den = 1, binv = 1;  // binv = 1 / b_l
        for (int r : S)
            num = g.mul(num, point(k + r) ^ y);
        for (size_t t2 = 0; t2 < e; ++t2)
            if (t2 != t)
                den = g.mul(den, y ^ point(Lost[t2]));
        for (int i = 0; i < k; ++i)
            if (i != Lost[t])
                binv = g.mul(binv, y ^ point(i));
        z[t] = g.mul(div(num, den), g.mul(binv, binv));
    }
}

// Multiplication by c on bit planes (kernels_bs.hip scale_planes): byte s = c * alpha^s, so
// plane t of c * x is the XOR of the planes s of x whose byte s has bit t set.
inline uint64_t scale_mask(uint8_t c)
{
    uint64_t m = 0;
    for (int s = 0; s < 8; ++s)
        m |= (uint64_t)gf().mul(c, (uint8_t)(1u << s)) << (8 * s);
    return m;
}

// Inverse of zfec's decode matrix for normalised slot indices.
inline bool decode_matrix(int k, int m, const std::vector<int> &idx, std::vector<uint8_t> &minv)
{
    const std::vector<uint8_t> enc = encode_matrix(k, m);
    minv.assign((size_t)k * k, 0);
    for (int i = 0; i < k; ++i) {
        if (idx[i] < k)
            minv[(size_t)i * k + i] = 1;
        else
            memcpy(&minv[(size_t)i * k], &enc[(size_t)idx[i] * k], k);
    }
    return gf_invert(minv, k);
}

}  // namespace sec
