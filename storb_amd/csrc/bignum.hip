// bignum.hip — RSA-2048 modular arithmetic on CDNA4 for storb's APDP proofs of data
// possession (F4: /root/reference/storb/challenge/__init__.py:304-350 generate_tag,
// :352-399 issue_challenge, :401-463 generate_proof, :465-528 verify_proof;
// DEFAULT_RSA_KEY_SIZE = 2048 at storb/constants.py:26).
//
// One wave = one integer: lane j holds 32-bit limb j (little-endian limbs), so a 64-lane
// wavefront is one RSA-2048 residue, and a 1024-bit CRT half (mod p or q) uses lanes 0..31
// with lanes 32..63 zero.  Montgomery multiplication (R = 2^(32*ROWS)) runs as ROWS row
// steps: the row's limb a_i is broadcast with v_readlane, every lane does two
// 32x32->64 multiply-adds (a_i*b_j and m*n_j), and the running sum moves down one lane
// per row (DPP wave_shl:1).  Carries stay redundant per lane and are resolved once per
// product with two wave ballots (generate / propagate masks; carry-lookahead done as
// 64-bit integer arithmetic on the masks).  The work is integer-multiply issue bound, not
// memory bound.
//
// Where the key owner holds p and q (the validator: tags and verification) exponentiations
// by secret-sized exponents run as two 1024-bit halves (CRT): half the rows per product
// and half the exponent bits.  g^X for tags and g^s for challenges use a fixed-base table
// of g^(v * 256^k) (255 products instead of ~2.6k).
#include <hip/hip_runtime.h>

#include "bignum.hpp"

using u8 = uint8_t;
using u32 = uint32_t;
using u64 = uint64_t;

namespace {

__device__ __forceinline__ u32 lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

__device__ __forceinline__ u32 bcast(u32 x, u32 i) { return __builtin_amdgcn_readlane(x, i); }

__device__ __forceinline__ u64 ballot(bool p) { return __ballot(p); }

// lane j <- x[j+1]; lane 63 <- 0 (DPP wave_shl:1; the lane without a source keeps `old`)
__device__ __forceinline__ u32 down1(u32 x) { return (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xf, 0xf, false); }

// lane j <- x[j-1]; lane 0 <- 0 (DPP wave_shr:1)
__device__ __forceinline__ u32 up1(u32 x) { return (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, false); }

// lane j <- x[j+32] for j < 32, 0 above: the high 1024 bits as a 1024-bit integer
__device__ __forceinline__ u32 high_half(u32 x, u32 l)
{
    const u32 y = (u32)__builtin_amdgcn_ds_bpermute((int)(((l + 32) & 63) << 2), (int)x);
    return l < 32 ? y : 0u;
}

// Carry-in mask of a multi-limb add: limb j generates (G) or propagates (P) a carry
// (never both).  *out = carry out of limb 63.
__device__ __forceinline__ u64 carry_in(u64 G, u64 P, bool *out)
{
    const u64 X = G << 1;
    const u64 S = X + P;
    *out = (S < X) || (G >> 63);
    return S ^ P;
}

// limb-vector + one carry bit per limb position already folded into `u` (64-bit sums
// whose high words are 0 or 1): normalise to 32-bit limbs, return the carry out.
__device__ __forceinline__ u32 resolve(u64 u, u32 l, u32 *t)
{
    u32 v = (u32)u;
    bool co;
    const u64 C = carry_in(ballot((u >> 32) != 0), ballot(v == 0xFFFFFFFFu), &co);
    *t = v + (u32)((C >> l) & 1u);
    return co ? 1u : 0u;
}

// a >= n, where `top` is a's limb 64
__device__ __forceinline__ bool geq(u32 a, u32 n, u32 top)
{
    if (top)
        return true;
    const u64 ne = ballot(a != n);
    if (!ne)
        return true;
    const u32 h = 63 - (u32)__builtin_clzll(ne);
    return bcast(a, h) > bcast(n, h);
}

// (a - n) mod 2^2048
__device__ __forceinline__ u32 sub_n(u32 a, u32 n, u32 l)
{
    bool dummy;
    const u64 B = carry_in(ballot(a < n), ballot(a == n), &dummy);
    return a - n - (u32)((B >> l) & 1u);
}

// Final step of a Montgomery product: value = t + sum_j c_j 2^32(j+1) < 2n.
__device__ __forceinline__ u32 mont_finish(u32 t, u32 c, u32 n, u32 l)
{
    u32 top = bcast(c, 63);
    top += resolve((u64)t + up1(c), l, &t);
    if (geq(t, n, top))
        t = sub_n(t, n, l);
    return t;
}

#ifndef SEC_BN_MM
#define SEC_BN_MM 3
#endif

// Montgomery product a*b*R^-1 mod n, R = 2^(32*ROWS), for a < R, b < n (result < n).
// ROWS = 64 (RSA-2048) or 32 (a 1024-bit CRT half; limbs 32..63 of a, b, n are zero).
//
// Row i adds a_i*b + m*n (m making limb 0 vanish) and shifts down one limb.  Lane j keeps
// t_j plus carry bits owed to limb j+1, kept as the carry-outs of its own add chain (k1,
// k2) rather than normalised each row: the next row's add chain takes them back as
// carry-ins.  p2 = m*n_j + p1_j (the whole first product as the 64-bit addend) may carry
// out of 64 bits; that bit belongs to limb j+1 after the shift (the next lane: the carry
// mask shifted left by one).
#if SEC_BN_MM == 3
// Hand-scheduled rows: 7 VALU + 5 SALU each (the compiler's rendering of the same
// arithmetic in C++ spends ~16 VALU, mostly moves that rebuild 64-bit operand pairs).
// Hard registers, so the pair {t, 0} (v[40:41]) is the first product's addend without a
// copy:
//   v[40:41] {t, 0}   v[42:43] p1   v[44:45] p2   v47 carry bit of p2 from lane j-1
//   s40 a_i   s41 m   s[42:43] p2 carry-outs (K)   s[44:45] K << 1
//   vcc, s[48:49] the two add-chain carries (k1, k2)   s[50:51] scratch
//   s[52:53] p1's (always zero) carry-out   s[54:55] lane-63 mask
// The shifted limb comes in as the DPP operand of the first add (wave_shl:1; lane 63
// reads 0 under bound_ctrl).  Lane 63's K lands in k2's bit 63 one row later (before
// k2 is next read): the value is < 2n < 2^2049 after every row, so at most one of the
// position-64 bits (k1, k2, K of lane 63) is set.
// Hazards: >= 1 wait state between mad1's write of v42 and v_readlane of it (the two
// SALU ops of the lane-63 merge); >= 2 between mad2's write of v44 and its DPP read
// (s_lshl + v_cndmask).
#define SEC_BN_IRP32 "0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22,23,24,25,26,27,28,29,30,31"
#define SEC_BN_IRP64 \
    SEC_BN_IRP32 ",32,33,34,35,36,37,38,39,40,41,42,43,44,45,46,47,48,49,50,51,52,53,54,55,56,57,58,59,60,61,62,63"
#define SEC_BN_ROWS_ASM(LIST)                                                                                    \
    asm volatile("v_mov_b32 v40, 0\n"                                                                           \
                 "v_mov_b32 v41, 0\n"                                                                           \
                 "s_mov_b64 vcc, 0\n"                                                                           \
                 "s_mov_b64 s[48:49], 0\n"                                                                      \
                 "s_mov_b64 s[42:43], 0\n"                                                                      \
                 "s_mov_b32 s54, 0\n"                                                                           \
                 "s_mov_b32 s55, 0x80000000\n"                                                                  \
                 ".irp i, " LIST "\n"                                                                           \
                 "v_readlane_b32 s40, %[a], \\i\n"                                                              \
                 "v_mad_u64_u32 v[42:43], s[52:53], s40, %[b], v[40:41]\n"                                      \
                 "s_and_b64 s[50:51], s[42:43], s[54:55]\n"                                                     \
                 "s_or_b64 s[48:49], s[48:49], s[50:51]\n"                                                      \
                 "v_readlane_b32 s41, v42, 0\n"                                                                 \
                 "s_mul_i32 s41, s41, %[n0]\n"                                                                  \
                 "v_mad_u64_u32 v[44:45], s[42:43], s41, %[n], v[42:43]\n"                                      \
                 "s_lshl_b64 s[44:45], s[42:43], 1\n"                                                           \
                 "v_cndmask_b32_e64 v47, 0, 1, s[44:45]\n"                                                      \
                 "v_addc_co_u32_dpp v40, vcc, v44, v45, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
                 "v_addc_co_u32_e64 v40, s[48:49], v40, v47, s[48:49]\n"                                        \
                 ".endr\n"                                                                                      \
                 "s_and_b64 s[50:51], s[42:43], s[54:55]\n"                                                     \
                 "s_or_b64 s[48:49], s[48:49], s[50:51]\n"                                                      \
                 "v_mov_b32 %[t], v40\n"                                                                        \
                 "s_mov_b64 %[k1], vcc\n"                                                                       \
                 "s_mov_b64 %[k2], s[48:49]\n"                                                                  \
                 : [t] "=v"(t), [k1] "=s"(k1), [k2] "=s"(k2)                                                    \
                 : [a] "v"(a), [b] "v"(b), [n] "v"(n), [n0] "s"(n0inv)                                          \
                 : "v40", "v41", "v42", "v43", "v44", "v45", "v47", "s40", "s41", "s42", "s43", "s44", "s45",   \
                   "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "vcc")

template <int ROWS>
__device__ __forceinline__ u32 mont_mul(u32 a, u32 b, u32 n, u32 n0inv, u32 l)
{
    static_assert(ROWS == 64 || ROWS == 32, "RSA-2048 or a 1024-bit CRT half");
    n0inv = __builtin_amdgcn_readfirstlane(n0inv);  // uniform by construction; SGPR for the asm
    u32 t;
    u64 k1, k2;
    if constexpr (ROWS == 64)
        SEC_BN_ROWS_ASM(SEC_BN_IRP64);
    else
        SEC_BN_ROWS_ASM(SEC_BN_IRP32);
    const u32 c = (u32)((k1 >> l) & 1u) + (u32)((k2 >> l) & 1u);
    return mont_finish(t, c, n, l);
}
#else
// The same product in plain C++ (A/B reference for the asm rows).
template <int ROWS>
__device__ u32 mont_mul(u32 a, u32 b, u32 n, u32 n0inv, u32 l)
{
    u32 t = 0, c = 0;  // value = sum t_j 2^32j + sum c_j 2^32(j+1), c_j <= 3
#pragma unroll 8
    for (u32 i = 0; i < (u32)ROWS; ++i) {
        const u32 ai = bcast(a, i);
        const u64 p1 = (u64)ai * b + t;
        const u32 m = bcast((u32)p1, 0) * n0inv;
        const u64 p2 = (u64)m * n + (u32)p1;  // limb 0 of p2 is 0 mod 2^32
        const u64 s = (u64)down1((u32)p2) + (p1 >> 32) + (p2 >> 32) + c;
        t = (u32)s;
        c = (u32)(s >> 32);
    }
    return mont_finish(t, c, n, l);
}
#endif

// (a + x) mod n for a < n and x < 2^bits (so a + x < 3n: n has its top bit set)
__device__ u32 add_mod(u32 a, u32 x, u32 n, u32 l)
{
    u32 t;
    u32 top = resolve((u64)a + x, l, &t);
    for (int k = 0; k < 2; ++k)
        if (geq(t, n, top)) {
            t = sub_n(t, n, l);  // exact mod 2^2048 even when top == 1
            top = 0;
        }
    return t;
}

// One modulus as the kernels read it (lane l's limbs of sec::BnKey).
struct Mod {
    u32 n, r2, one, n0inv;
};

__device__ __forceinline__ Mod load_mod(const sec::BnKey *k, u32 l) { return Mod{k->n[l], k->r2[l], k->one[l], k->n0inv}; }

template <int ROWS>
__device__ __forceinline__ u32 mmul(const Mod &M, u32 a, u32 b, u32 l)
{
    return mont_mul<ROWS>(a, b, M.n, M.n0inv, l);
}

// 4-bit fixed-window exponentiation in Montgomery form; the exponent's nibbles come from
// `nib(i)` for i = nnib-1 .. 0 (most significant first).  tab: 16 x 64 u32 of LDS.
// Two mont_mul call sites only (table, then one loop for squarings and products): each
// inlined product is ~1k instructions, so call sites are kept few for the I-cache.
template <int ROWS, class Nib>
__device__ u32 mont_pow(const Mod &M, u32 base_m, u32 l, u32 nnib, Nib nib, u32 *tab)
{
    tab[l] = M.one;
    tab[64 + l] = base_m;
    u32 x = base_m;
#pragma unroll 1
    for (u32 w = 2; w < 16; ++w) {
        x = mmul<ROWS>(M, x, base_m, l);
        tab[w * 64 + l] = x;
    }
    u32 i = nnib, r = M.one;
    while (i > 0) {  // leading zero nibbles cost nothing
        const u32 v = nib(--i);
        if (v) {
            r = tab[v * 64 + l];
            break;
        }
    }
#pragma unroll 1
    for (; i > 0; --i) {
        const u32 v = nib(i - 1);
        const u32 ops = v ? 5u : 4u;  // 4 squarings, then the table product
#pragma unroll 1
        for (u32 s = 0; s < ops; ++s)
            r = mmul<ROWS>(M, r, s < 4 ? r : tab[v * 64 + l], l);
    }
    return r;
}

// Fixed-base power g^e from the comb table T[k][v] = g^(v * 256^k) (Montgomery form,
// entry (k, v) at (k * 256 + v) * 64 u32): one product per nonzero exponent byte.
// `byte(k)` = byte k of e counted from the least significant, k < nbytes <= 256.  The
// next entry is loaded before the current product so its latency hides under it.
// k0 / k1: the byte range [k0, k1) this call multiplies (the whole exponent by default).
template <class Byte>
__device__ u32 fixed_pow(const Mod &M, const u32 *__restrict__ table, u32 nbytes, Byte byte, u32 l, u32 k0 = 0,
                         u32 k1 = ~0u)
{
    k1 = k1 < nbytes ? k1 : nbytes;
    u32 r = M.one;
    bool started = false;
    u32 v = k0 < k1 ? byte(k0) : 0u;
    u32 e = v ? table[((u64)k0 * 256 + v) * 64 + l] : 0u;
#pragma unroll 1
    for (u32 k = k0; k < k1; ++k) {
        const u32 cv = v, ce = e;
        if (k + 1 < k1) {
            v = byte(k + 1);
            e = v ? table[((u64)(k + 1) * 256 + v) * 64 + l] : 0u;
        }
        if (cv) {
            r = started ? mmul<64>(M, r, ce, l) : ce;
            started = true;
        }
    }
    return r;
}

// limb l of an nbytes-long big-endian integer (nbytes a multiple of 4, <= 256)
__device__ __forceinline__ u32 load_be(const u8 *be, u32 nbytes, u32 l)
{
    if (4 * l >= nbytes)
        return 0u;
    const u8 *p = be + nbytes - 4 - 4 * l;
    return (u32)p[0] << 24 | (u32)p[1] << 16 | (u32)p[2] << 8 | (u32)p[3];
}

__device__ __forceinline__ u32 load_be_limb(const u8 *be, u32 l) { return load_be(be, 256, l); }

__device__ __forceinline__ void store_be_limb(u8 *be, u32 l, u32 v)
{
    u8 *p = be + 252 - 4 * l;
    p[0] = (u8)(v >> 24);
    p[1] = (u8)(v >> 16);
    p[2] = (u8)(v >> 8);
    p[3] = (u8)v;
}

// byte k (from the least significant) of the integer held one limb per lane
__device__ __forceinline__ u32 limb_byte(u32 x, u32 k) { return (bcast(x, k / 4) >> (8 * (k % 4))) & 0xFFu; }

// nibble k (from the least significant) of the integer held one limb per lane
__device__ __forceinline__ u32 limb_nib(u32 x, u32 k) { return (bcast(x, k / 8) >> (4 * (k % 8))) & 15u; }

// limb j of the big-endian integer formed by bytes [start, start+len) of a message
// whose bytes at or beyond `avail` read as zero (len <= 256)
__device__ __forceinline__ u32 chunk_limb(const u8 *p, uint64_t start, uint32_t len, uint64_t avail, u32 l)
{
    const int64_t end = (int64_t)start + len - 4 * (int64_t)l;  // exclusive end of this limb's bytes
    u32 v = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int64_t pos = end - 4 + b;
        const u32 byte = (pos >= (int64_t)start && (uint64_t)pos < avail) ? (u32)p[pos] : 0u;
        v = (v << 8) | byte;
    }
    return v;
}

// int.from_bytes(msg, "big") mod n: Horner over 256-byte chunks from the most
// significant, r <- r * 2^2048 + chunk  (r * 2^2048 = mont_mul(r, R^2)).
__device__ u32 reduce_msg(const Mod &M, const u8 *p, uint64_t len, uint64_t avail, u32 l)
{
    u32 r = 0;
    if (len == 0)
        return r;
    const uint64_t nch = (len + 255) / 256;
    const uint32_t first = (uint32_t)(len - 256 * (nch - 1));
    uint64_t off = 0;
#pragma unroll 1
    for (uint64_t c = 0; c < nch; ++c) {
        const uint32_t clen = c == 0 ? first : 256u;
        const u32 x = chunk_limb(p, off, clen, avail, l);
        if (c > 0)
            r = mmul<64>(M, r, M.r2, l);
        r = add_mod(r, x, M.n, l);
        off += clen;
    }
    return r;
}

// x (any value < 2^2048, plain) mod a 1024-bit half h, in h's Montgomery form:
// (hi * 2^1024 + lo) mod h with hi * 2^1024 = mont_mul(hi, R_h^2), then * R_h.
__device__ u32 to_half_m(const Mod &H, u32 x, u32 l)
{
    const u32 hi = high_half(x, l), lo = l < 32 ? x : 0u;
    const u32 r = add_mod(mmul<32>(H, hi, H.r2, l), lo, H.n, l);
    return mmul<32>(H, r, H.r2, l);
}

// CRT: x^e mod n from (x mod p)^ep and (x mod q)^eq recombined as tp * cp + tq * cq mod n
// (cp = q * (q^-1 mod p), cq = p * (p^-1 mod q), Montgomery form mod n in the key).
// One half (h = 0: p, 1: q): (x mod h)^e_h times its weight; x plain (< 2^2048), `nib`:
// 4-bit digits of e_h.  The two halves' results add up to x^e mod n.
template <class Nib>
__device__ u32 crt_half(const sec::TagKey *__restrict__ tk, const Mod &N, u32 x, u32 h, u32 nnib, Nib nib, u32 *tab,
                        u32 l)
{
    const Mod H = load_mod(h ? &tk->q : &tk->p, l);
    const u32 rm = mont_pow<32>(H, to_half_m(H, x, l), l, nnib, nib, tab);
    const u32 t = mmul<32>(H, rm, l == 0 ? 1u : 0u, l);  // plain, < h
    return mmul<64>(N, t, h ? tk->cq_m[l] : tk->cp_m[l], l);
}

// ---- kernels (one wave per integer unless stated) ---------------------------------

// BnKey from a big-endian modulus of `bits` (2048 or 1024, top bit set, odd):
// R mod n = 2^bits - n, R^2 mod n by `bits` modular doublings.
__global__ __launch_bounds__(64) void sec_bn_setup_kernel(const u8 *__restrict__ n_be, u32 n0inv, u32 bits,
                                                          sec::BnKey *key)
{
    const u32 l = lane_id();
    const u32 n = load_be(n_be, bits / 8, l);
    u32 one;
    {  // 0 - n mod 2^2048, then cut to 2^bits
        bool dummy;
        const u64 B = carry_in(ballot(0u < n), ballot(n == 0u), &dummy);
        one = 0u - n - (u32)((B >> l) & 1u);
        if (32 * l >= bits)
            one = 0;
    }
    u32 r2 = one;
    for (u32 i = 0; i < bits; ++i)
        r2 = add_mod(r2, r2, n, l);
    key->n[l] = n;
    key->one[l] = one;
    key->r2[l] = r2;
    if (l == 0) {
        key->n0inv = n0inv;
        key->bits = bits;
    }
}

// generate_tag's constants: g, fdh in Montgomery form; d, dp, dq plain
__global__ __launch_bounds__(64) void sec_tag_setup_kernel(const u8 *__restrict__ g_be, const u8 *__restrict__ fdh_be,
                                                           const u8 *__restrict__ d_be, const u8 *__restrict__ dp_be,
                                                           const u8 *__restrict__ dq_be, sec::TagKey *tk)
{
    const u32 l = lane_id();
    const Mod N = load_mod(&tk->k, l);
    tk->g_m[l] = mmul<64>(N, load_be_limb(g_be, l), N.r2, l);
    tk->fdh_m[l] = mmul<64>(N, load_be_limb(fdh_be, l), N.r2, l);
    tk->d[l] = load_be_limb(d_be, l);
    tk->dp[l] = dp_be ? load_be(dp_be, 128, l) : 0u;
    tk->dq[l] = dq_be ? load_be(dq_be, 128, l) : 0u;
}

// CRT recombination constants cp, cq (plain big-endian mod n) into Montgomery form
__global__ __launch_bounds__(64) void sec_crt_setup_kernel(const u8 *__restrict__ cp_be, const u8 *__restrict__ cq_be,
                                                           sec::TagKey *tk)
{
    const u32 l = lane_id();
    const Mod N = load_mod(&tk->k, l);
    tk->cp_m[l] = mmul<64>(N, load_be_limb(cp_be, l), N.r2, l);
    tk->cq_m[l] = mmul<64>(N, load_be_limb(cq_be, l), N.r2, l);
}

// Fixed-base table, step 1 (one wave): T[k][1] = g^(256^k) for k < 256 by 8 squarings per
// step, and T[k][0] = 1.
__global__ __launch_bounds__(64) void sec_gtab_base_kernel(const sec::TagKey *__restrict__ tk, u32 *table)
{
    const u32 l = lane_id();
    const Mod N = load_mod(&tk->k, l);
    u32 G = tk->g_m[l];
#pragma unroll 1
    for (u32 k = 0; k < 256; ++k) {
        table[(k * 256 + 1) * 64 + l] = G;
        table[(k * 256) * 64 + l] = N.one;
        if (k + 1 < 256)
#pragma unroll 1
            for (int s = 0; s < 8; ++s)
                G = mmul<64>(N, G, G, l);
    }
}

// Fixed-base table, step 2 (one wave per k): T[k][v] = T[k][v-1] * T[k][1] for v < 256
__global__ __launch_bounds__(64) void sec_gtab_fill_kernel(const sec::TagKey *__restrict__ tk, u32 *table)
{
    const u32 l = lane_id();
    const u32 k = blockIdx.x;
    const Mod N = load_mod(&tk->k, l);
    const u32 G = table[(k * 256 + 1) * 64 + l];
    u32 x = G;
#pragma unroll 1
    for (u32 v = 2; v < 256; ++v) {
        x = mmul<64>(N, x, G, l);
        table[(k * 256 + v) * 64 + l] = x;
    }
}

// P_j = R^(j * S) mod n in Montgomery form: Q = (R in Montgomery form)^S, P_j = Q^j
__global__ __launch_bounds__(64) void sec_bn_rpow_kernel(const sec::BnKey *__restrict__ key, u32 j0, u32 *P)
{
    __shared__ u32 tab[16 * 64];
    const u32 l = lane_id();
    const u32 j = j0 + blockIdx.x;
    const Mod N = load_mod(key, l);
    const u32 Q = mont_pow<64>(N, N.r2, l, 8, [](u32 k) { return (sec::kSegChunks >> (4 * k)) & 15u; }, tab);
    P[(u64)j * 64 + l] = mont_pow<64>(N, Q, l, 8, [j](u32 k) { return (j >> (4 * k)) & 15u; }, tab);
}

// One segment of one message: its bytes as an integer mod n, times R^(j S) (its weight
// in the message), plain limbs into partials.
__global__ __launch_bounds__(64) void sec_bn_reduce_seg_kernel(const sec::BnKey *__restrict__ key,
                                                               const u32 *__restrict__ P, const u8 *base0,
                                                               const sec::MsgDesc *__restrict__ msgs,
                                                               const sec::SegDesc *__restrict__ segs, u32 nsegs,
                                                               u32 *partials)
{
    const u32 b = blockIdx.x;
    if (b >= nsegs)
        return;
    const u32 l = lane_id();
    const sec::SegDesc sd = segs[b];
    const sec::MsgDesc m = msgs[sd.msg];
    const Mod N = load_mod(key, l);
    const u64 seg = (u64)sec::kSegChunks * 256;
    const u64 end = m.len - (u64)sd.j * seg;
    const u64 start = end > seg ? end - seg : 0;
    const u64 avail = m.avail > start ? m.avail - start : 0;
    u32 r = reduce_msg(N, base0 + m.off + start, end - start, avail, l);
    if (sd.j)
        r = mmul<64>(N, r, P[(u64)sd.j * 64 + l], l);
    partials[(u64)b * 64 + l] = r;
}

// message value mod n = sum of its segments' partial residues
__device__ __forceinline__ u32 combine(const Mod &N, const u32 *__restrict__ partials, sec::SegInfo si, u32 l)
{
    u32 acc = 0;
#pragma unroll 1
    for (u32 s = 0; s < si.count; ++s)
        acc = add_mod(acc, partials[(u64)(si.first + s) * 64 + l], N.n, l);
    return acc;
}

__global__ __launch_bounds__(64) void sec_bn_reduce_sum_kernel(const sec::BnKey *__restrict__ key,
                                                               const sec::SegInfo *__restrict__ info, u32 nmsgs,
                                                               const u32 *__restrict__ partials, u8 *out)
{
    const u32 i = blockIdx.x;
    if (i >= nmsgs)
        return;
    const u32 l = lane_id();
    store_be_limb(out + (u64)i * 256, l, combine(load_mod(key, l), partials, info[i], l));
}

// out_i = bases_i ^ exps_i mod n; bases < 2^2048 (256 B big-endian), exps fixed-width big-endian
__global__ __launch_bounds__(64) void sec_bn_modexp_kernel(const sec::BnKey *__restrict__ key, const u8 *bases,
                                                           const u8 *exps, u32 exp_bytes, u32 count, u8 *out)
{
    __shared__ u32 tab[16 * 64];
    const u32 i = blockIdx.x;
    if (i >= count)
        return;
    const u32 l = lane_id();
    const Mod N = load_mod(key, l);
    const u32 bm = mmul<64>(N, load_be_limb(bases + (u64)i * 256, l), N.r2, l);
    const u8 *e = exps + (u64)i * exp_bytes;
    auto nib = [&](u32 k) -> u32 {  // nibble k counted from the least significant
        const u8 byte = e[exp_bytes - 1 - k / 2];
        return (k & 1) ? (u32)(byte >> 4) : (u32)(byte & 15);
    };
    const u32 r = mont_pow<64>(N, bm, l, 2 * exp_bytes, nib, tab);
    store_be_limb(out + (u64)i * 256, l, mmul<64>(N, r, l == 0 ? 1u : 0u, l));
}

// CRT exponentiation with per-item exponents ep (mod p-1) and eq (mod q-1), exp_bytes each.
// Two waves per item: wave 0 the p half, wave 1 the q half, summed through LDS.
__global__ __launch_bounds__(128) void sec_bn_crt_modexp_kernel(const sec::TagKey *__restrict__ tk, const u8 *bases,
                                                                const u8 *exps_p, const u8 *exps_q, u32 exp_bytes,
                                                                u32 count, u8 *out)
{
    __shared__ u32 tab[2][16 * 64];
    __shared__ u32 part[64];
    const u32 i = blockIdx.x;
    if (i >= count)
        return;
    const u32 l = lane_id(), w = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);  // wave-uniform
    const Mod N = load_mod(&tk->k, l);
    const u8 *e = (w ? exps_q : exps_p) + (u64)i * exp_bytes;
    auto nib = [&](u32 k) -> u32 {
        const u8 byte = e[exp_bytes - 1 - k / 2];
        return (k & 1) ? (u32)(byte >> 4) : (u32)(byte & 15);
    };
    const u32 y = crt_half(tk, N, load_be_limb(bases + (u64)i * 256, l), w, 2 * exp_bytes, nib, tab[w], l);
    if (w)
        part[l] = y;
    __syncthreads();
    if (!w)
        store_be_limb(out + (u64)i * 256, l, add_mod(y, part[l], N.n, l));
}

// out_i = a_i * b_i mod n: (a_i R) * b_i * R^-1
__global__ __launch_bounds__(64) void sec_bn_mulmod_kernel(const sec::BnKey *__restrict__ key, const u8 *a,
                                                           const u8 *b, u32 count, u8 *out)
{
    const u32 i = blockIdx.x;
    if (i >= count)
        return;
    const u32 l = lane_id();
    const Mod N = load_mod(key, l);
    const u32 am = mmul<64>(N, load_be_limb(a + (u64)i * 256, l), N.r2, l);
    store_be_limb(out + (u64)i * 256, l, mmul<64>(N, load_be_limb(b + (u64)i * 256, l), am, l));
}

// g^e mod n through the fixed-base table (issue_challenge's g_s = g^s); e: exp_bytes <= 256
__global__ __launch_bounds__(64) void sec_apdp_gpow_kernel(const sec::TagKey *__restrict__ tk, const u32 *table,
                                                           const u8 *exps, u32 exp_bytes, u32 count, u8 *out)
{
    const u32 i = blockIdx.x;
    if (i >= count)
        return;
    const u32 l = lane_id();
    const Mod N = load_mod(&tk->k, l);
    const u8 *e = exps + (u64)i * exp_bytes;
    const u32 r = fixed_pow(N, table, exp_bytes, [&](u32 k) -> u32 { return e[exp_bytes - 1 - k]; }, l);
    store_be_limb(out + (u64)i * 256, l, mmul<64>(N, r, l == 0 ? 1u : 0u, l));
}

// APDP generate_tag for one piece: X = piece mod n (summed from its segments' residues);
// tag = (fdh * g^X)^d mod n.  Two waves per piece: each multiplies half of g^X's
// fixed-base table entries (combined through LDS), then with a CRT key each raises to d
// mod one factor and the halves are summed through LDS; without CRT wave 0 does the d
// power alone.
__global__ __launch_bounds__(128) void sec_apdp_tag_kernel(const sec::TagKey *__restrict__ tk, const u32 *table,
                                                           const sec::SegInfo *__restrict__ info, u32 nmsgs,
                                                           const u32 *__restrict__ partials, u8 *tags)
{
    __shared__ u32 tab[2][16 * 64];
    __shared__ u32 part[2][64];
    const u32 i = blockIdx.x;
    if (i >= nmsgs)
        return;
    const u32 l = lane_id(), w = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);  // wave-uniform
    const Mod N = load_mod(&tk->k, l);
    const u32 X = combine(N, partials, info[i], l);  // the piece mod n (segments reduced before)
    part[w][l] = fixed_pow(N, table, 256, [&](u32 k) { return limb_byte(X, k); }, l, 128 * w, 128 * w + 128);
    __syncthreads();
    const u32 gx = mmul<64>(N, part[0][l], part[1][l], l);
    const u32 base_m = mmul<64>(N, tk->fdh_m[l], gx, l);
    if (tk->crt) {
        const u32 dh = w ? tk->dq[l] : tk->dp[l];
        const u32 y = crt_half(
            tk, N, mmul<64>(N, base_m, l == 0 ? 1u : 0u, l), w, 256, [&](u32 k) { return limb_nib(dh, k); }, tab[w],
            l);
        __syncthreads();  // both waves are done reading part[] for gx
        if (w)
            part[1][l] = y;
        __syncthreads();
        if (!w)
            store_be_limb(tags + (u64)i * 256, l, add_mod(y, part[1][l], N.n, l));
    } else if (!w) {
        const u32 d = tk->d[l];
        const u32 r = mont_pow<64>(N, base_m, l, 512, [&](u32 k) { return limb_nib(d, k); }, tab[0]);
        store_be_limb(tags + (u64)i * 256, l, mmul<64>(N, r, l == 0 ? 1u : 0u, l));
    }
}

}  // namespace

int sec_launch_bn_setup(const uint8_t *n_be, uint32_t n0inv, uint32_t bits, sec::BnKey *key, void *stream)
{
    hipLaunchKernelGGL(sec_bn_setup_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, n_be, n0inv, bits, key);
    return hipGetLastError();
}

int sec_launch_tag_setup(const uint8_t *g_be, const uint8_t *fdh_be, const uint8_t *d_be, const uint8_t *dp_be,
                         const uint8_t *dq_be, sec::TagKey *tk, uint32_t *table, void *stream)
{
    hipLaunchKernelGGL(sec_tag_setup_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, g_be, fdh_be, d_be, dp_be,
                       dq_be, tk);
    hipLaunchKernelGGL(sec_gtab_base_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, tk, table);
    hipLaunchKernelGGL(sec_gtab_fill_kernel, dim3(256), dim3(64), 0, (hipStream_t)stream, tk, table);
    return hipGetLastError();
}

int sec_launch_crt_setup(const uint8_t *cp_be, const uint8_t *cq_be, sec::TagKey *tk, void *stream)
{
    hipLaunchKernelGGL(sec_crt_setup_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, cp_be, cq_be, tk);
    return hipGetLastError();
}

int sec_launch_bn_rpow(const sec::BnKey *key, uint32_t j0, uint32_t j1, uint32_t *P, void *stream)
{
    if (j1 <= j0)
        return hipSuccess;
    hipLaunchKernelGGL(sec_bn_rpow_kernel, dim3(j1 - j0), dim3(64), 0, (hipStream_t)stream, key, j0, P);
    return hipGetLastError();
}

int sec_launch_bn_reduce(const sec::BnKey *key, const uint32_t *P, const uint8_t *base0, const sec::MsgDesc *msgs,
                         uint32_t nmsgs, const sec::SegDesc *segs, uint32_t nsegs, const sec::SegInfo *info,
                         uint8_t *partials, uint8_t *out, void *stream)
{
    if (nmsgs == 0)
        return hipSuccess;
    hipLaunchKernelGGL(sec_bn_reduce_seg_kernel, dim3(nsegs), dim3(64), 0, (hipStream_t)stream, key, P, base0, msgs,
                       segs, nsegs, (u32 *)partials);
    hipLaunchKernelGGL(sec_bn_reduce_sum_kernel, dim3(nmsgs), dim3(64), 0, (hipStream_t)stream, key, info, nmsgs,
                       (const u32 *)partials, out);
    return hipGetLastError();
}

int sec_launch_bn_modexp(const sec::BnKey *key, const uint8_t *bases, const uint8_t *exps, uint32_t exp_bytes,
                         uint32_t count, uint8_t *out, void *stream)
{
    if (count == 0)
        return hipSuccess;
    hipLaunchKernelGGL(sec_bn_modexp_kernel, dim3(count), dim3(64), 0, (hipStream_t)stream, key, bases, exps,
                       exp_bytes, count, out);
    return hipGetLastError();
}

int sec_launch_bn_crt_modexp(const sec::TagKey *tk, const uint8_t *bases, const uint8_t *exps_p,
                             const uint8_t *exps_q, uint32_t exp_bytes, uint32_t count, uint8_t *out, void *stream)
{
    if (count == 0)
        return hipSuccess;
    hipLaunchKernelGGL(sec_bn_crt_modexp_kernel, dim3(count), dim3(128), 0, (hipStream_t)stream, tk, bases, exps_p,
                       exps_q, exp_bytes, count, out);
    return hipGetLastError();
}

int sec_launch_bn_mulmod(const sec::BnKey *key, const uint8_t *a, const uint8_t *b, uint32_t count, uint8_t *out,
                         void *stream)
{
    if (count == 0)
        return hipSuccess;
    hipLaunchKernelGGL(sec_bn_mulmod_kernel, dim3(count), dim3(64), 0, (hipStream_t)stream, key, a, b, count, out);
    return hipGetLastError();
}

int sec_launch_apdp_gpow(const sec::TagKey *tk, const uint32_t *table, const uint8_t *exps, uint32_t exp_bytes,
                         uint32_t count, uint8_t *out, void *stream)
{
    if (count == 0)
        return hipSuccess;
    hipLaunchKernelGGL(sec_apdp_gpow_kernel, dim3(count), dim3(64), 0, (hipStream_t)stream, tk, table, exps,
                       exp_bytes, count, out);
    return hipGetLastError();
}

int sec_launch_apdp_tag(const sec::TagKey *tk, const uint32_t *table, const uint32_t *P, const uint8_t *base0,
                        const sec::MsgDesc *msgs, uint32_t nmsgs, const sec::SegDesc *segs, uint32_t nsegs,
                        const sec::SegInfo *info, uint8_t *partials, uint8_t *tags, void *stream)
{
    if (nmsgs == 0)
        return hipSuccess;
    hipLaunchKernelGGL(sec_bn_reduce_seg_kernel, dim3(nsegs), dim3(64), 0, (hipStream_t)stream, &tk->k, P, base0,
                       msgs, segs, nsegs, (u32 *)partials);
    hipLaunchKernelGGL(sec_apdp_tag_kernel, dim3(nmsgs), dim3(128), 0, (hipStream_t)stream, tk, table, info, nmsgs,
                       (const u32 *)partials, tags);
    return hipGetLastError();
}
