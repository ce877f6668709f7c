/*
 * fec_oracle.c — CPU restatement of zfec 1.6.0.0's Reed–Solomon code
 * (Rizzo's fec.c as wrapped by zfec/_fecmodule.c + zfec/easyfec.py).
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle and the timed
 * CPU baseline ("kind": "port") for bench.py.  Only tests/, the
 * __graft_entry__.smoke() checker and bench.py's cpu_baseline leg may load
 * it.  The product path (storb_amd/, libstorbec.so) never links it.
 *
 * PARITY STATUS: "parity unpinned" against real zfec bytes.  zfec is the
 * third-party dependency on the reference path (pinned zfec==1.6.0.0 at
 * /root/reference/uv.lock:1088-1091, imported at
 * /root/reference/storb/util/piece.py:8) and is neither vendored under
 * /root/reference nor installed in this image, and the reference's own tests
 * (storb/util/piece_test.py:48-125) hold no known-answer vectors — only
 * round-trip identity.  This restatement is pinned by (a) those round-trip
 * tests, (b) two independent constructions of the encode matrix (Lagrange /
 * Vandermonde-inverse below vs. Gauss–Jordan in oracle/zfec_ref.py), and
 * (c) the matrix rows restated in SURVEY.md Appendix A.
 *
 * Algorithm (published zfec / Rizzo 1997 "Effective erasure codes"):
 *   field     GF(2^8), primitive polynomial x^8+x^4+x^3+x^2+1 (0x11D), alpha=2
 *   matrix    rows 0..k-1 = identity; row r>=k, col j = L_j(x_r) where L_j is
 *             the Lagrange basis on points x_0=0, x_i=alpha^(i-1) (i>=1);
 *             this equals tmp[k..m-1] * inv(tmp[0..k-1]) with
 *             tmp[0]=[1,0..0], tmp[r][c]=alpha^((r-1)*c mod 255)
 *   encode    fecs[r][i] = XOR_j mul(enc[r][j], src[j][i]), in STRIDE-byte
 *             blocks (zfec fec_encode / addmul)
 *   decode    rows: e_i for a primary present in slot i, enc[index[i]] for a
 *             secondary; invert (Gauss–Jordan); each missing primary i is
 *             XOR_c Minv[i][c] * in[c] (zfec fec_decode)
 *   easyfec   B = ceil(n/k); k slices of B, the last zero-padded; decode
 *             joins the k primaries and strips padlen (easyfec.py).
 * All code below is written from that description; no zfec source is
 * present in this environment.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define FO_STRIDE 8192 /* zfec fec.c STRIDE: addmul blocking */

static uint8_t fo_exp[510];
static int fo_log[256];
static uint8_t fo_inv[256];
static uint8_t fo_mul[256][256]; /* 64 KiB product table, as zfec's gf_mul_table */
static int fo_ready = 0;

/* GF(2^8) tables: exp doubled so exp[a+b] needs no reduction. */
void fo_init(void)
{
    if (fo_ready)
        return;
    unsigned v = 1;
    for (int e = 0; e < 255; ++e) {
        fo_exp[e] = (uint8_t)v;
        fo_exp[e + 255] = (uint8_t)v;
        fo_log[v] = e;
        v <<= 1;
        if (v & 0x100)
            v ^= 0x11D;
    }
    fo_log[0] = 255; /* sentinel, as zfec */
    fo_inv[0] = 0;
    for (int a = 1; a < 256; ++a)
        fo_inv[a] = fo_exp[255 - fo_log[a]];
    for (int a = 0; a < 256; ++a)
        for (int b = 0; b < 256; ++b)
            fo_mul[a][b] = (a && b) ? fo_exp[fo_log[a] + fo_log[b]] : 0;
    fo_ready = 1;
}

static inline uint8_t gmul(uint8_t a, uint8_t b) { return fo_mul[a][b]; }

uint8_t fo_gf_mul(uint8_t a, uint8_t b) { fo_init(); return gmul(a, b); }
uint8_t fo_gf_exp(int e) { fo_init(); return fo_exp[e % 255]; }

/* point x_r used by row r of zfec's Vandermonde seed matrix */
static uint8_t fo_point(int r) { return r == 0 ? 0 : fo_exp[(r - 1) % 255]; }

/*
 * Encode matrix, m x k (row-major), via Lagrange basis polynomials:
 * L_j(x) = prod_{t!=j} (x - x_t) / prod_{t!=j} (x_j - x_t)  (minus == plus).
 * Returns 0, or -1 on bad (k, m).
 */
int fo_encode_matrix(int k, int m, uint8_t *enc)
{
    fo_init();
    if (k < 1 || m < k || m > 256)
        return -1;
    memset(enc, 0, (size_t)m * k);
    for (int i = 0; i < k; ++i)
        enc[i * k + i] = 1;
    for (int r = k; r < m; ++r) {
        uint8_t xr = fo_point(r);
        for (int j = 0; j < k; ++j) {
            uint8_t num = 1, den = 1, xj = fo_point(j);
            for (int t = 0; t < k; ++t) {
                if (t == j)
                    continue;
                uint8_t xt = fo_point(t);
                num = gmul(num, (uint8_t)(xr ^ xt));
                den = gmul(den, (uint8_t)(xj ^ xt));
            }
            enc[r * k + j] = gmul(num, fo_inv[den]);
        }
    }
    return 0;
}

/* In-place Gauss–Jordan inverse of a k x k matrix.  0 ok, -1 singular. */
int fo_invert(uint8_t *a, int k)
{
    fo_init();
    uint8_t *w = (uint8_t *)malloc((size_t)k * 2 * k);
    if (!w)
        return -1;
    for (int r = 0; r < k; ++r) {
        memcpy(w + (size_t)r * 2 * k, a + (size_t)r * k, k);
        memset(w + (size_t)r * 2 * k + k, 0, k);
        w[(size_t)r * 2 * k + k + r] = 1;
    }
    for (int c = 0; c < k; ++c) {
        int piv = -1;
        for (int r = c; r < k; ++r)
            if (w[(size_t)r * 2 * k + c]) { piv = r; break; }
        if (piv < 0) { free(w); return -1; }
        if (piv != c)
            for (int t = 0; t < 2 * k; ++t) {
                uint8_t s = w[(size_t)c * 2 * k + t];
                w[(size_t)c * 2 * k + t] = w[(size_t)piv * 2 * k + t];
                w[(size_t)piv * 2 * k + t] = s;
            }
        uint8_t iv = fo_inv[w[(size_t)c * 2 * k + c]];
        for (int t = 0; t < 2 * k; ++t)
            w[(size_t)c * 2 * k + t] = gmul(w[(size_t)c * 2 * k + t], iv);
        for (int r = 0; r < k; ++r) {
            uint8_t f = w[(size_t)r * 2 * k + c];
            if (r == c || !f)
                continue;
            for (int t = 0; t < 2 * k; ++t)
                w[(size_t)r * 2 * k + t] ^= gmul(f, w[(size_t)c * 2 * k + t]);
        }
    }
    for (int r = 0; r < k; ++r)
        memcpy(a + (size_t)r * k, w + (size_t)r * 2 * k + k, k);
    free(w);
    return 0;
}

/* dst[i] ^= c * src[i]  — zfec addmul, through the 64 KiB table row */
static void addmul(uint8_t *dst, const uint8_t *src, uint8_t c, size_t sz)
{
    if (c == 0)
        return;
    const uint8_t *row = fo_mul[c];
    for (size_t i = 0; i < sz; ++i)
        dst[i] ^= row[src[i]];
}

/*
 * zfec fec_encode: for each requested secondary block number (>= k), write
 * XOR_j enc[num][j] * src[j] into fecs[i], STRIDE bytes at a time.
 */
int fo_encode(int k, int m, const uint8_t *enc, const uint8_t *const *src,
              uint8_t *const *fecs, const unsigned *block_nums, size_t nb, size_t sz)
{
    fo_init();
    for (size_t i = 0; i < nb; ++i)
        if (block_nums[i] < (unsigned)k || block_nums[i] >= (unsigned)m)
            return -1;
    for (size_t off = 0; off < sz; off += FO_STRIDE) {
        size_t len = sz - off < FO_STRIDE ? sz - off : FO_STRIDE;
        for (size_t i = 0; i < nb; ++i) {
            const uint8_t *row = enc + (size_t)block_nums[i] * k;
            memset(fecs[i] + off, 0, len);
            for (int j = 0; j < k; ++j)
                addmul(fecs[i] + off, src[j] + off, row[j], len);
        }
    }
    return 0;
}

/*
 * zfec decode matrix for slot indices `index` (already normalised so that a
 * primary p sits at slot p): row i = e_i if index[i] < k else enc[index[i]];
 * inverted in place into `dm` (k x k).
 */
int fo_decode_matrix(int k, const uint8_t *enc, const unsigned *index, uint8_t *dm)
{
    for (int i = 0; i < k; ++i) {
        if (index[i] < (unsigned)k) {
            memset(dm + (size_t)i * k, 0, k);
            dm[(size_t)i * k + i] = 1;
        } else {
            memcpy(dm + (size_t)i * k, enc + (size_t)index[i] * k, k);
        }
    }
    return fo_invert(dm, k);
}

/* zfec fec_decode: fills outpkts[0..e-1] with the missing primaries in row order. */
int fo_decode(int k, int m, const uint8_t *enc, const uint8_t *const *inpkts,
              uint8_t *const *outpkts, const unsigned *index, size_t sz)
{
    fo_init();
    for (int i = 0; i < k; ++i) {
        if (index[i] >= (unsigned)m)
            return -1;
        if (index[i] < (unsigned)k && index[i] != (unsigned)i)
            return -2; /* primary not in its own slot */
    }
    uint8_t *dm = (uint8_t *)malloc((size_t)k * k);
    if (!dm || fo_decode_matrix(k, enc, index, dm)) {
        free(dm);
        return -3;
    }
    int outix = 0;
    for (int row = 0; row < k; ++row) {
        if (index[row] < (unsigned)k)
            continue;
        memset(outpkts[outix], 0, sz);
        for (int c = 0; c < k; ++c)
            addmul(outpkts[outix], inpkts[c], dm[(size_t)row * k + c], sz);
        ++outix;
    }
    free(dm);
    return 0;
}

/* ---- easyfec-level wrappers (zfec/easyfec.py + _fecmodule.c checks) ---- */

/*
 * easyfec.Encoder(k,m).encode(data): out receives m blocks of B=ceil(n/k)
 * bytes back to back (the k data slices, last zero-padded, then m-k parity).
 * Returns B, or -1 bad (k,m), -2 unequal slices (zfec "Input blocks are
 * required to be all the same length").
 */
long fo_easy_encode(int k, int m, const uint8_t *data, size_t n, uint8_t *out)
{
    fo_init();
    if (k < 1 || m < k || m > 256)
        return -1;
    size_t B = (n + k - 1) / k;
    if (k > 1 && (size_t)(k - 1) * B > n)
        return -2;
    for (int j = 0; j < k; ++j) {
        size_t lo = (size_t)j * B, len = lo < n ? (n - lo < B ? n - lo : B) : 0;
        memcpy(out + (size_t)j * B, data + lo, len);
        memset(out + (size_t)j * B + len, 0, B - len);
    }
    if (m == k || B == 0)
        return (long)B;
    uint8_t *enc = (uint8_t *)malloc((size_t)m * k);
    const uint8_t **src = (const uint8_t **)malloc(sizeof(*src) * k);
    uint8_t **fecs = (uint8_t **)malloc(sizeof(*fecs) * (m - k));
    unsigned *nums = (unsigned *)malloc(sizeof(*nums) * (m - k));
    fo_encode_matrix(k, m, enc);
    for (int j = 0; j < k; ++j)
        src[j] = out + (size_t)j * B;
    for (int r = k; r < m; ++r) {
        fecs[r - k] = out + (size_t)r * B;
        nums[r - k] = (unsigned)r;
    }
    fo_encode(k, m, enc, src, fecs, nums, (size_t)(m - k), B);
    free(enc); free(src); free(fecs); free(nums);
    return (long)B;
}

/*
 * easyfec.Decoder(k,m).decode(blocks, sharenums, padlen): blocks is k
 * pointers of B bytes, out receives k*B - padlen bytes.
 * Returns 0, -1 bad (k,m), -3 sharenum >= m, -4 duplicate sharenum,
 * -5 singular, -6 padlen > k*B.
 */
int fo_easy_decode(int k, int m, const uint8_t *const *blocks, const int *sharenums,
                   size_t B, size_t padlen, uint8_t *out)
{
    fo_init();
    if (k < 1 || m < k || m > 256)
        return -1;
    if (padlen > (size_t)k * B)
        return -6;
    const uint8_t **slot = (const uint8_t **)calloc(k, sizeof(*slot));
    unsigned *index = (unsigned *)calloc(k, sizeof(*index));
    unsigned char seen[256] = {0};
    int rc = 0;
    /* _fecmodule.c Decoder_decode: validate, then move each primary to its own slot */
    for (int i = 0; i < k; ++i) {
        if (sharenums[i] < 0 || sharenums[i] >= m) { rc = -3; goto done; }
        if (seen[sharenums[i]]) { rc = -4; goto done; }
        seen[sharenums[i]] = 1;
        slot[i] = blocks[i];
        index[i] = (unsigned)sharenums[i];
    }
    for (int i = 0; i < k; ++i) {
        while (index[i] < (unsigned)k && index[i] != (unsigned)i) {
            unsigned t = index[i];
            const uint8_t *tb = slot[i];
            index[i] = index[t]; slot[i] = slot[t];
            index[t] = t; slot[t] = tb;
        }
    }
    {
        int e = 0;
        for (int i = 0; i < k; ++i)
            e += index[i] >= (unsigned)k;
        uint8_t *rec = (uint8_t *)malloc(e ? (size_t)e * B : 1);
        uint8_t **outp = (uint8_t **)malloc(sizeof(*outp) * (e ? e : 1));
        for (int i = 0; i < e; ++i)
            outp[i] = rec + (size_t)i * B;
        if (e) {
            uint8_t *enc = (uint8_t *)malloc((size_t)m * k);
            fo_encode_matrix(k, m, enc);
            if (fo_decode(k, m, enc, slot, outp, index, B))
                rc = -5;
            free(enc);
        }
        if (!rc) {
            size_t total = (size_t)k * B - padlen, w = 0;
            int outix = 0;
            for (int i = 0; i < k && w < total; ++i) {
                const uint8_t *srcb = index[i] < (unsigned)k ? slot[i] : outp[outix];
                if (index[i] >= (unsigned)k)
                    ++outix;
                size_t len = total - w < B ? total - w : B;
                memcpy(out + w, srcb, len);
                w += len;
            }
        }
        free(rec); free(outp);
    }
done:
    free(slot); free(index);
    return rc;
}
