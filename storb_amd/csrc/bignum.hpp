// bignum.hpp — device structs and launchers for the RSA-2048 APDP kernels (bignum.hip).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "kernels.hpp"

namespace sec {

constexpr int kBnLimbs = 64;  // 2048 bits = one 32-bit limb per lane of a wave
constexpr int kBnBytes = 256;
constexpr size_t kGTabWords = (size_t)256 * 256 * kBnLimbs;  // fixed-base table: 256 bytes x 256 values
constexpr uint32_t kSegChunks = 32;  // segmented reductions: 32 x 256 B = 8 KiB per wave

// Segment j of message `msg`: bytes [len - (j+1) * 8 KiB, len - j * 8 KiB) (clipped at 0),
// i.e. counted from the least significant end of the big-endian integer.
struct SegDesc {
    uint32_t msg, j;
};
// A message's segments are entries first .. first+count-1 of the segment list.
struct SegInfo {
    uint32_t first, count;
};

// Per-modulus Montgomery constants, limbs little-endian; derived on the device by
// sec_bn_setup from n alone (R = 2^bits).  A 1024-bit CRT half keeps limbs 32..63 zero.
struct BnKey {
    uint32_t n[kBnLimbs];
    uint32_t r2[kBnLimbs];   // R^2 mod n
    uint32_t one[kBnLimbs];  // R mod n (Montgomery 1)
    uint32_t n0inv;          // -n^-1 mod 2^32
    uint32_t bits;           // 2048 or 1024
    uint32_t pad[kBnLimbs - 2];
};

// A modulus plus, for the key owner, APDP tag constants (generate_tag,
// storb/challenge/__init__.py:304-350) and the CRT halves (p, q).
struct TagKey {
    BnKey k;                   // n
    BnKey p, q;                // CRT halves (valid when crt != 0)
    uint32_t g_m[kBnLimbs];    // g in Montgomery form
    uint32_t fdh_m[kBnLimbs];  // full_domain_hash(prf(key, 0)) in Montgomery form
    uint32_t d[kBnLimbs];      // RSA private exponent (plain limbs)
    uint32_t dp[kBnLimbs];     // d reduced for p (limbs 0..31), used when crt != 0
    uint32_t dq[kBnLimbs];     // d reduced for q
    uint32_t cp_m[kBnLimbs];   // q * (q^-1 mod p), Montgomery form mod n
    uint32_t cq_m[kBnLimbs];   // p * (p^-1 mod q), Montgomery form mod n
    uint32_t crt;              // tags use CRT: p, q, cp, cq, dp and dq are all set
    uint32_t pad[kBnLimbs - 1];
};

}  // namespace sec

extern "C++" {
// All big-endian inputs are device memory.  bits = 2048 (n, 256 B) or 1024 (p / q, 128 B).
int sec_launch_bn_setup(const uint8_t *n_be, uint32_t n0inv, uint32_t bits, sec::BnKey *key, void *stream);
// g, fdh, d: 256 B; dp, dq: 128 B or NULL.  Also builds the fixed-base table of g
// (kGTabWords u32, T[k][v] = g^(v * 256^k) in Montgomery form).
int sec_launch_tag_setup(const uint8_t *g_be, const uint8_t *fdh_be, const uint8_t *d_be, const uint8_t *dp_be,
                         const uint8_t *dq_be, sec::TagKey *tk, uint32_t *table, void *stream);
int sec_launch_crt_setup(const uint8_t *cp_be, const uint8_t *cq_be, sec::TagKey *tk, void *stream);
// P_j = R^(j * kSegChunks) mod n in Montgomery form, for j in [j0, j1) (one wave each).
int sec_launch_bn_rpow(const sec::BnKey *key, uint32_t j0, uint32_t j1, uint32_t *P, void *stream);
// int.from_bytes(message, "big") mod n per message, 256 B big-endian each: one wave per
// segment into `partials` (256 B per segment), then one wave per message sums them.
int sec_launch_bn_reduce(const sec::BnKey *key, const uint32_t *P, const uint8_t *base0, const sec::MsgDesc *msgs,
                         uint32_t nmsgs, const sec::SegDesc *segs, uint32_t nsegs, const sec::SegInfo *info,
                         uint8_t *partials, uint8_t *out, void *stream);
int sec_launch_bn_modexp(const sec::BnKey *key, const uint8_t *bases, const uint8_t *exps, uint32_t exp_bytes,
                         uint32_t count, uint8_t *out, void *stream);
int sec_launch_bn_crt_modexp(const sec::TagKey *tk, const uint8_t *bases, const uint8_t *exps_p,
                             const uint8_t *exps_q, uint32_t exp_bytes, uint32_t count, uint8_t *out, void *stream);
int sec_launch_bn_mulmod(const sec::BnKey *key, const uint8_t *a, const uint8_t *b, uint32_t count, uint8_t *out,
                         void *stream);
int sec_launch_apdp_gpow(const sec::TagKey *tk, const uint32_t *table, const uint8_t *exps, uint32_t exp_bytes,
                         uint32_t count, uint8_t *out, void *stream);
int sec_launch_apdp_tag(const sec::TagKey *tk, const uint32_t *table, const uint32_t *P, const uint8_t *base0,
                        const sec::MsgDesc *msgs, uint32_t nmsgs, const sec::SegDesc *segs, uint32_t nsegs,
                        const sec::SegInfo *info, uint8_t *partials, uint8_t *tags, void *stream);
}
