// bignum.hpp — device structs and launchers for the 2048-bit APDP kernels (bignum.hip).
#pragma once
#include <stdint.h>

#include "kernels.hpp"

namespace sec {

constexpr int kBnLimbs = 64;    // 2048 bits = one 32-bit limb per lane of a wave
constexpr int kBnBytes = 256;

// Per-modulus Montgomery constants, limbs little-endian; derived on the device by
// sec_bn_setup from n alone (R = 2^2048).
struct BnKey {
    uint32_t n[kBnLimbs];
    uint32_t r2[kBnLimbs];   // R^2 mod n
    uint32_t one[kBnLimbs];  // R mod n (Montgomery 1)
    uint32_t n0inv;          // -n^-1 mod 2^32
    uint32_t pad[kBnLimbs - 1];
};

// APDP tag constants (generate_tag, storb/challenge/__init__.py:304-350).
struct TagKey {
    BnKey k;
    uint32_t g_m[kBnLimbs];    // g in Montgomery form
    uint32_t fdh_m[kBnLimbs];  // full_domain_hash(prf(key, 0)) in Montgomery form
    uint32_t d[kBnLimbs];      // RSA private exponent (plain limbs)
};

}  // namespace sec

extern "C++" {
// key_be: big-endian modulus (and for tags g, fdh, d), 256 bytes each, device memory
int sec_launch_bn_setup(const uint8_t *n_be, uint32_t n0inv, sec::BnKey *key, void *stream);
int sec_launch_tag_setup(const uint8_t *g_be, const uint8_t *fdh_be, const uint8_t *d_be, sec::TagKey *tk,
                         void *stream);
int sec_launch_bn_reduce(const sec::BnKey *key, const uint8_t *base0, const sec::MsgDesc *msgs, uint32_t nmsgs,
                         uint8_t *out, void *stream);
int sec_launch_bn_modexp(const sec::BnKey *key, const uint8_t *bases, const uint8_t *exps, uint32_t exp_bytes,
                         uint32_t count, uint8_t *out, void *stream);
int sec_launch_bn_mulmod(const sec::BnKey *key, const uint8_t *a, const uint8_t *b, uint32_t count, uint8_t *out,
                         void *stream);
int sec_launch_apdp_tag(const sec::TagKey *tk, const uint8_t *base0, const sec::MsgDesc *msgs, uint32_t nmsgs,
                        uint8_t *tags, void *stream);
}
