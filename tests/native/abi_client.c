/*
 * abi_client.c — a plain C caller of libstorbec.so through include/storb_ec.h only: the shape
 * a cgo / JNI / FFI binding of storb's erasure-coding path takes, with no
 * Python and no HIP headers.  TEST INFRASTRUCTURE: it links the CPU oracle
 * (oracle/fec_oracle.c) as the checker; tests/test_abi_client.py builds and runs it.
 *
 * Cases, all bit-exact against the oracle:
 *   1. host buffers (SEC_F_HOST): one encode batch over every policy shape, C4's RS(10,4) and
 *      C5's RS(8,3), ragged and padded sizes, then a decode batch with erasures (reassembled
 *      bytes == the source) and a recover-only batch (== the lost blocks);
 *   2. device buffers: sec_malloc / sec_memcpy, the same encode on device pointers with a
 *      padded parity stride, and a decode whose padded block k-1 is read in place
 *      (sec_decode_batch_ex, avail = B - padlen);
 *   3. zfec's preconditions as error codes (sec_strerror names each one).
 * Prints "abi_client ok: ..." and exits 0, or prints the first mismatch and exits 1.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "storb_ec.h"

long fo_easy_encode(int k, int m, const uint8_t *data, size_t n, uint8_t *out); /* oracle */

#define CHECK(call)                                                                      \
    do {                                                                                 \
        int rc_ = (call);                                                                \
        if (rc_ != SEC_OK) {                                                             \
            fprintf(stderr, "%s:%d %s -> %d (%s) %s\n", __FILE__, __LINE__, #call, rc_,    \
                    sec_strerror(rc_), rc_ == SEC_EHIP ? sec_last_hip_error() : "");     \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint8_t next_byte(void)
{
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (uint8_t)(rng >> 24);
}

typedef struct {
    int k, m;
    size_t n;
} shape_t;

static const shape_t kCases[] = {
    {1, 2, 7},          {2, 3, 300001},     {4, 6, 1 << 20},      {4, 6, 65536 + 3},
    {8, 12, 1 << 22},   {8, 12, 4000 * 8 - 5}, {16, 24, 1 << 23}, {16, 24, 16 * 2047 + 9},
    {32, 48, 1 << 22},  {32, 48, 32 * 100 - 1}, {64, 96, 1 << 23}, {64, 96, 64 * 5000 + 63},
    {10, 14, 65536},    {8, 11, 1234567},   {3, 256, 10000},
};
#define NCASES ((int)(sizeof(kCases) / sizeof(kCases[0])))

static size_t blk(const shape_t *s) { return (s->n + (size_t)s->k - 1) / (size_t)s->k; }

int main(void)
{
    int ndev = 0;
    CHECK(sec_device_count(&ndev));
    if (ndev < 1) {
        fprintf(stderr, "no device\n");
        return 1;
    }
    sec_ctx *ctx = NULL;
    CHECK(sec_ctx_create(0, &ctx));

    /* ---- 1. host buffers ---------------------------------------------------------- */
    size_t in_total = 0, par_total = 0;
    for (int i = 0; i < NCASES; ++i) {
        in_total += kCases[i].n;
        par_total += (size_t)(kCases[i].m - kCases[i].k) * blk(&kCases[i]);
    }
    uint8_t *in = (uint8_t *)malloc(in_total), *par = (uint8_t *)malloc(par_total);
    for (size_t i = 0; i < in_total; ++i)
        in[i] = next_byte();
    sec_enc_chunk enc[NCASES];
    memset(enc, 0, sizeof(enc));
    size_t io = 0, po = 0;
    for (int i = 0; i < NCASES; ++i) {
        const size_t B = blk(&kCases[i]);
        enc[i].in_off = io;
        enc[i].n = kCases[i].n;
        enc[i].parity_off = po;
        enc[i].parity_stride = B;
        enc[i].k = kCases[i].k;
        enc[i].m = kCases[i].m;
        io += kCases[i].n;
        po += (size_t)(kCases[i].m - kCases[i].k) * B;
    }
    CHECK(sec_encode_batch(ctx, enc, NCASES, in, par, SEC_F_HOST));

    /* oracle: every block of every case */
    uint8_t **want = (uint8_t **)malloc(sizeof(*want) * NCASES);
    for (int i = 0; i < NCASES; ++i) {
        const size_t B = blk(&kCases[i]);
        want[i] = (uint8_t *)malloc((size_t)kCases[i].m * B);
        if (fo_easy_encode(kCases[i].k, kCases[i].m, in + enc[i].in_off, kCases[i].n, want[i]) != (long)B) {
            fprintf(stderr, "oracle encode failed on case %d\n", i);
            return 1;
        }
        if (memcmp(par + enc[i].parity_off, want[i] + (size_t)kCases[i].k * B,
                   (size_t)(kCases[i].m - kCases[i].k) * B) != 0) {
            fprintf(stderr, "host encode mismatch: case %d zfec(%d,%d) n=%zu\n", i, kCases[i].k, kCases[i].m,
                    kCases[i].n);
            return 1;
        }
    }

    /* decode: data blocks 0, 2, 4, ... lost (as many as there are parity blocks), the
     * survivors passed in reverse order; blocks come from the oracle's full block set */
    size_t nslots = 0;
    for (int i = 0; i < NCASES; ++i)
        nslots += (size_t)kCases[i].k;
    int32_t *sn = (int32_t *)malloc(sizeof(int32_t) * nslots);
    uint64_t *offs = (uint64_t *)malloc(sizeof(uint64_t) * nslots);
    sec_dec_chunk dec[NCASES], rec[NCASES];
    memset(dec, 0, sizeof(dec));
    memset(rec, 0, sizeof(rec));
    size_t slot = 0, oo = 0, ro = 0;
    for (int i = 0; i < NCASES; ++i) {
        const int k = kCases[i].k, m = kCases[i].m;
        const size_t B = blk(&kCases[i]);
        int lost[256] = {0}, e = 0;
        for (int j = 0; j < k && e < m - k; j += 2) {
            lost[j] = 1;
            ++e;
        }
        int keep[256], nk = 0;
        for (int s = 0; s < m && nk < k; ++s)
            if (s >= k || !lost[s])
                keep[nk++] = s;
        for (int q = 0; q < k; ++q) {
            const int s = keep[k - 1 - q];
            sn[slot + q] = s;
            offs[slot + q] = (uint64_t)(uintptr_t)(want[i] + (size_t)s * B);
        }
        dec[i].out_off = oo;
        dec[i].B = B;
        dec[i].padlen = (size_t)k * B - kCases[i].n;
        dec[i].slot0 = slot;
        dec[i].k = k;
        dec[i].m = m;
        rec[i] = dec[i];
        rec[i].out_off = ro;
        slot += (size_t)k;
        oo += kCases[i].n;
        ro += (size_t)e * B;
    }
    uint8_t *out = (uint8_t *)malloc(in_total), *rout = (uint8_t *)malloc(ro ? ro : 1);
    CHECK(sec_decode_batch(ctx, dec, NCASES, sn, offs, NULL, out, SEC_F_HOST));
    if (memcmp(out, in, in_total) != 0) {
        fprintf(stderr, "host decode mismatch\n");
        return 1;
    }
    CHECK(sec_decode_batch(ctx, rec, NCASES, sn, offs, NULL, rout, SEC_F_HOST | SEC_F_RECOVER));
    for (int i = 0; i < NCASES; ++i) {
        const size_t B = blk(&kCases[i]);
        size_t o = rec[i].out_off;
        for (int j = 0, e = 0; j < kCases[i].k && e < kCases[i].m - kCases[i].k; j += 2, ++e, o += B)
            if (memcmp(rout + o, want[i] + (size_t)j * B, B) != 0) {
                fprintf(stderr, "recover-only mismatch: case %d block %d\n", i, j);
                return 1;
            }
    }

    /* ---- 2. device buffers ---------------------------------------------------------- */
    const int k = 10, m = 14, nch = 64;
    const size_t n = 65536, B = (n + k - 1) / k, ps = B + 64, padlen = (size_t)k * B - n;
    uint8_t *dsrc = NULL, *dpar = NULL, *dout = NULL;
    CHECK(sec_malloc(ctx, nch * n, (void **)&dsrc));
    CHECK(sec_malloc(ctx, (size_t)nch * (m - k) * ps, (void **)&dpar));
    CHECK(sec_malloc(ctx, nch * n, (void **)&dout));
    CHECK(sec_memcpy(ctx, dsrc, in, nch * n, 0));
    sec_enc_chunk de[64];
    memset(de, 0, sizeof(de));
    for (int c = 0; c < nch; ++c) {
        de[c].in_off = (uint64_t)c * n;
        de[c].n = n;
        de[c].parity_off = (uint64_t)c * (m - k) * ps;
        de[c].parity_stride = ps;
        de[c].k = k;
        de[c].m = m;
    }
    CHECK(sec_encode_batch(ctx, de, nch, dsrc, dpar, 0));
    uint8_t *hpar = (uint8_t *)malloc((size_t)nch * (m - k) * ps), *full = (uint8_t *)malloc((size_t)m * B);
    CHECK(sec_memcpy(ctx, hpar, dpar, (size_t)nch * (m - k) * ps, 1));
    for (int c = 0; c < nch; ++c) {
        fo_easy_encode(k, m, in + (size_t)c * n, n, full);
        for (int r = 0; r < m - k; ++r)
            if (memcmp(hpar + (size_t)c * (m - k) * ps + (size_t)r * ps, full + (size_t)(k + r) * B, B) != 0) {
                fprintf(stderr, "device encode mismatch: chunk %d row %d\n", c, r);
                return 1;
            }
    }
    /* decode in place: blocks {0, 2, 5, 7} lost, block 9 (padded) read from the chunk buffer */
    const int keep[10] = {1, 3, 4, 6, 8, 9, 10, 11, 12, 13};
    int32_t dsn[640];
    uint64_t doffs[640], davail[640];
    sec_dec_chunk dd[64];
    memset(dd, 0, sizeof(dd));
    for (int c = 0; c < nch; ++c) {
        for (int q = 0; q < k; ++q) {
            const int s = keep[q];
            dsn[c * k + q] = s;
            doffs[c * k + q] = s < k ? (uint64_t)(uintptr_t)(dsrc + (size_t)c * n + (size_t)s * B)
                                     : (uint64_t)(uintptr_t)(dpar + (size_t)c * (m - k) * ps + (size_t)(s - k) * ps);
            davail[c * k + q] = s == k - 1 ? B - padlen : B;
        }
        dd[c].out_off = (uint64_t)c * n;
        dd[c].B = B;
        dd[c].padlen = padlen;
        dd[c].slot0 = (uint64_t)c * k;
        dd[c].k = k;
        dd[c].m = m;
    }
    CHECK(sec_decode_batch_ex(ctx, dd, nch, dsn, doffs, davail, NULL, dout, 0)); /* absolute addresses */
    uint8_t *hout = (uint8_t *)malloc(nch * n);
    CHECK(sec_memcpy(ctx, hout, dout, nch * n, 1));
    if (memcmp(hout, in, nch * n) != 0) {
        fprintf(stderr, "device decode mismatch\n");
        return 1;
    }

    /* ---- 3. preconditions ------------------------------------------------------------ */
    sec_enc_chunk bad = enc[0];
    bad.k = 0;
    if (sec_encode_batch(ctx, &bad, 1, in, par, SEC_F_HOST) != SEC_EKM) {
        fprintf(stderr, "k = 0 not refused with SEC_EKM\n");
        return 1;
    }
    sec_dec_chunk bd = dec[2];
    int32_t dup[4] = {0, 0, 4, 5};
    uint64_t doff4[4] = {offs[dec[2].slot0], offs[dec[2].slot0 + 1], offs[dec[2].slot0 + 2], offs[dec[2].slot0 + 3]};
    bd.slot0 = 0;
    if (sec_decode_batch(ctx, &bd, 1, dup, doff4, NULL, out, SEC_F_HOST) != SEC_EDUPSHARE) {
        fprintf(stderr, "duplicate sharenum not refused with SEC_EDUPSHARE\n");
        return 1;
    }
    int32_t big[4] = {0, 1, 2, 6};
    if (sec_decode_batch(ctx, &bd, 1, big, doff4, NULL, out, SEC_F_HOST) != SEC_ESHARENUM) {
        fprintf(stderr, "sharenum >= m not refused with SEC_ESHARENUM\n");
        return 1;
    }

    CHECK(sec_free(ctx, dsrc));
    CHECK(sec_free(ctx, dpar));
    CHECK(sec_free(ctx, dout));
    sec_ctx_destroy(ctx);
    printf("abi_client ok: %d host chunks (encode, decode, recover-only), %d device chunks RS(10,4), "
           "precondition codes; abi %d\n", NCASES, nch, sec_abi_version());
    for (int i = 0; i < NCASES; ++i)
        free(want[i]);
    free(want);
    free(in);
    free(par);
    free(sn);
    free(offs);
    free(out);
    free(rout);
    free(hpar);
    free(full);
    free(hout);
    return 0;
}
