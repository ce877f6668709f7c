/*
 * storb_ec.h — C ABI of libstorbec.so, the MI355X (gfx950) Reed–Solomon engine
 * behind storb's chunk-and-shard path.
 *
 * Boundary.  In the reference the path crosses into native code at zfec's
 * CPython extension:
 *   zfec.easyfec.Encoder(k, m).encode(chunk)         /root/reference/storb/util/piece.py:129-130
 *   zfec.easyfec.Decoder(k, m).decode(b, s, padlen)  /root/reference/storb/util/piece.py:196-197
 * (zfec 1.6.0.0, /root/reference/uv.lock:1088-1091; import at piece.py:8).
 * This header replaces that extension with plain C entry points (no torch or
 * HIP types in any signature) that a ctypes / cffi / cgo binding can bind
 * directly; storb_amd/_lib.py is the ctypes binding, INTEGRATION.md shows it.
 *
 * Conventions (zfec's, kept on purpose):
 *   k = data blocks, m = TOTAL blocks (data + parity), 1 <= k <= m <= 256
 *   B = ceil(n / k) bytes per block; padlen = k*B - n; the last data block
 *   is zero-padded to B (easyfec).  Block numbers 0..k-1 are primaries
 *   (systematic: the chunk bytes themselves), k..m-1 are secondaries.
 *
 * Ownership.  The caller owns every buffer passed in; the library never frees
 * caller memory.  Device scratch, coefficient tables, pinned staging and
 * streams belong to the sec_ctx and are reused across calls.
 *
 * Threading.  One sec_ctx per (device, host thread).  Calls on different
 * contexts are independent; a context must not be used from two threads at
 * once.
 *
 * Errors.  Every int-returning function returns SEC_OK (0) or a negative
 * SEC_E* code; sec_strerror() names it.  The zfec preconditions map as
 * follows (zfec raises zfec.Error for each; storb_amd.easyfec raises
 * storb_amd.easyfec.Error with the same message text).
 */
#ifndef STORB_EC_H
#define STORB_EC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SEC_ABI_VERSION 1

enum sec_status {
    SEC_OK = 0,
    SEC_EINVAL = -1,     /* NULL pointer / negative count / bad flag                  */
    SEC_EKM = -2,        /* 1 <= k <= m <= 256 violated (zfec Encoder/Decoder init)    */
    SEC_EBLOCKLEN = -3,  /* blocks not all the same length (easyfec short middle slice) */
    SEC_ENBLOCKS = -4,   /* decode given other than exactly k blocks                   */
    SEC_ESHARENUM = -5,  /* sharenum < 0 or >= m                                       */
    SEC_EDUPSHARE = -6,  /* duplicate sharenum                                         */
    SEC_EPADLEN = -7,    /* padlen > k*B                                               */
    SEC_ESIZE = -8,      /* block size B >= 2^31 bytes                                 */
    SEC_ENODEV = -9,     /* no HIP device / bad device ordinal                         */
    SEC_EHIP = -10,      /* HIP runtime error; sec_last_hip_error() has the text       */
    SEC_ENOMEM = -11,    /* device / pinned allocation failed                          */
    SEC_ESINGULAR = -12, /* decode matrix singular (cannot happen for valid inputs)    */
    SEC_EMODULUS = -13,  /* bignum modulus not an odd 2048-bit integer                 */
    SEC_ENOTAG = -14,    /* APDP call on a key without sec_bn_key_set_tag              */
    SEC_ENOCRT = -15     /* CRT call on a key without sec_bn_key_set_crt               */
};

/* flags for sec_encode_batch / sec_decode_batch */
#define SEC_F_HOST 1u  /* in/out/blocks are HOST pointers; the call returns when the
                          results are back in host memory.  When every buffer of an
                          encode / decode lies in pinned memory mapped at the same address
                          on the device (sec_host_alloc, sec_host_register, hipHostMalloc),
                          the kernels read and write it directly over PCIe: no staging
                          copy.  Pageable buffers of a large call (context option SEC_REGISTER_MIN
                          bytes, default 4 MiB, in ranges of >= 1 MiB on average) are page-locked
                          for the call and used the same way; otherwise (or if locking
                          fails) they are staged through pinned slabs and device scratch.
                          sec_ctx_host_paths counts which path each call took        */
#define SEC_F_ASYNC 2u /* device pointers only: return once enqueued on the context
                          stream (sec_sync() waits)                                  */
#define SEC_F_RECOVER 4u /* decode only, recover-only: write just the chunk's missing
                          primaries, i.e. what zfec's fec_decode itself produces: the
                          e = (primaries absent from the chunk's k blocks) recovered
                          blocks, B bytes each (block k-1 with its zero padding), in
                          increasing block number at out + out_off + r*B.  Present
                          primaries are not copied; a chunk with e = 0 writes nothing  */
#define SEC_F_STAGED 8u /* SEC_F_HOST only: never page-lock pageable buffers for this call
                          (they are staged; persistently pinned ones stay zero-copy).
                          Page-locking takes the process's memory-map lock, so it stalls
                          while other threads fault in or free memory: one 8 MiB encode
                          beside storb's piece copies took 6.4 ms locked, 0.55 ms staged */
#define SEC_F_GPU_PARITY_IDS 16u /* sec_encode_pieces with digests only: the parity pieces'
                          SHA-1 ids come from the GPU (sec_sha1_kernel on the parity while it
                          is device-resident, one lane per piece, sub-batches of up to
                          SEC_SLAB_BYTES_DIGEST input bytes) while the host threads hash the
                          data pieces; without it the host threads hash every piece  */

typedef struct sec_ctx sec_ctx;

/* One chunk to encode: the easyfec.Encoder(k, m).encode(chunk) of piece.py:129-130. */
typedef struct sec_enc_chunk {
    uint64_t in_off;        /* byte offset of the chunk in `in`                       */
    uint64_t n;             /* chunk bytes (EncodedChunk.original_chunk_size)         */
    uint64_t parity_off;    /* byte offset in `parity` of block k (first secondary)   */
    uint64_t parity_stride; /* bytes from one secondary block to the next (>= B)      */
    int32_t k;              /* data blocks                                            */
    int32_t m;              /* total blocks                                           */
} sec_enc_chunk;

/* One chunk to reassemble: the easyfec.Decoder(k, m).decode(blocks, sharenums,
 * padlen) of piece.py:196-197.  The chunk's k blocks are entries
 * slot0 .. slot0+k-1 of the call's sharenums[] / block_offs[] arrays. */
typedef struct sec_dec_chunk {
    uint64_t out_off; /* byte offset in `out` of the k*B - padlen reassembled bytes    */
    uint64_t B;       /* block size (EncodedChunk.chunk_size)                          */
    uint64_t padlen;  /* EncodedChunk.padlen                                           */
    uint64_t slot0;   /* first index into sharenums[] / block_offs[]                   */
    int32_t k;
    int32_t m;
} sec_dec_chunk;

/* ---- library / device ------------------------------------------------- */
int sec_abi_version(void);
const char *sec_strerror(int status);
const char *sec_last_hip_error(void);          /* thread-local text of the last SEC_EHIP */
int sec_device_count(int *count);              /* SEC_ENODEV when the HIP runtime has none */

/* ---- context ------------------------------------------------------------ */
int sec_ctx_create(int device, sec_ctx **out);
void sec_ctx_destroy(sec_ctx *ctx);
/* Launch on an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream);
 * NULL restores the context's own stream, which is created blocking (ordered with
 * the legacy NULL stream, torch's default stream).  Producers on any other stream
 * must be ordered by the caller (or the context switched onto their stream). */
int sec_ctx_set_stream(sec_ctx *ctx, void *hip_stream);
int sec_sync(sec_ctx *ctx);
/* HIP-event timing of the hot kernels: when enabled every batch call records an
 * event pair around its encode / decode kernels on the launch stream. */
int sec_ctx_set_timing(sec_ctx *ctx, int enable);
/* Waits for recorded pairs, returns the summed milliseconds and launch count of
 * kind 0 = encode, 1 = decode, 2 = SHA-1, 3 = bignum (APDP), and clears them. */
int sec_timing_collect(sec_ctx *ctx, int kind, double *total_ms, int64_t *launches);

/* ---- context options --------------------------------------------------------
 * The library picks kernels, tile widths and host paths by measured rules and reads no
 * environment variable.  A test or an A/B tool that must force another choice sets it on
 * its own context; the context's cached plans are dropped, so the next call is planned
 * with it.  Names (e.g. "SEC_SYN": -1 cost rule, 0 direct decode, 1 syndrome path;
 * "SEC_BS"; "SEC_REGISTER_MIN": bytes, 0 = never page-lock) are listed by
 * sec_option_name(0, 1, ...) up to NULL; their meaning is documented in api.cpp (enum Opt).
 * Only options that force a shipped path or size the host pipeline exist (round 5 archived
 * the A/B-only ones with their kernels).
 * No zfec counterpart: the reference has no tuning surface on this path.
 * SEC_EINVAL for an unknown name or a value out of the option's range. */
int sec_ctx_set_option(sec_ctx *ctx, const char *name, int64_t value);
/* The context's value (NULL ctx: the library default). */
int sec_ctx_get_option(sec_ctx *ctx, const char *name, int64_t *value);
const char *sec_option_name(int index);

/* ---- choosing the blocks to decode from (host logic, no device needed) ---------------
 * A caller holding n > k blocks of a chunk (storb's validator fetches every data and parity
 * piece: validator.py:1556-1604, 1631) passes their sharenums; pick[0..k) receives the
 * positions of the k blocks to hand to sec_decode_batch(_ex): every present primary, then
 * parity rows from as few of the decode kernels' row groups as possible (the cheapest decode;
 * any k distinct blocks give the same bytes).  Replaces the reference's `pieces[:k]`
 * (storb/util/piece.py:189-191).  Out-of-range and repeated sharenums are never chosen;
 * SEC_ENBLOCKS when fewer than k distinct valid ones are present. */
int sec_decode_choose(int k, int m, int64_t n, const int32_t *sharenums, int32_t *pick);

/* ---- matrices (host arithmetic, no device needed) ------------------------ */
/* Rows k..m-1 of zfec's systematic encode matrix ((m-k)*k bytes, row-major). */
int sec_encode_matrix(int k, int m, uint8_t *out_rows);
/* zfec decode matrix for the given k sharenums: slots normalised as
 * _fecmodule.c does (each primary moved to its own slot), rows built, inverted.
 * out: k*k bytes of the inverse; out_index (nullable): k normalised sharenums. */
int sec_decode_matrix(int k, int m, const int32_t *sharenums, uint8_t *out, int32_t *out_index);

/* ---- the hot path ----------------------------------------------------------
 * Encode: for every chunk, parity block r (r = k..m-1) is written at
 * parity + parity_off + (r-k)*parity_stride, B bytes.  Data blocks are not
 * written: they are the chunk bytes themselves (systematic code); the zero
 * padding of the last data block is synthesised, never read from `in`.
 */
int sec_encode_batch(sec_ctx *ctx, const sec_enc_chunk *chunks, int64_t nchunks,
                     const uint8_t *in, uint8_t *parity, unsigned flags);

/* Decode + reassemble: for every chunk, its k blocks are at
 * blocks + block_offs[slot0 + i] (B bytes each) with block numbers
 * sharenums[slot0 + i]; the chunk's k*B - padlen bytes are written at
 * out + out_off.  Present primaries are copied, missing ones recovered.
 * `blocks` may be NULL, in which case block_offs are absolute addresses.
 * Every block must have B readable bytes here; sec_decode_batch_ex lifts that.
 * SEC_F_RECOVER: recover-only output instead (see the flag).
 * Aliasing: a chunk's output range must not overlap any block of any chunk in
 * the call (no in-place reassembly).  The kernels read blocks while other
 * workgroups write `out`, and a SEC_F_HOST call joins present primaries on the
 * host while the device writes the recovered rows, so an overlap gives
 * unspecified bytes.  The library does not check this. */
int sec_decode_batch(sec_ctx *ctx, const sec_dec_chunk *chunks, int64_t nchunks,
                     const int32_t *sharenums, const uint64_t *block_offs,
                     const uint8_t *blocks, uint8_t *out, unsigned flags);

/* sec_decode_batch with a readable length per block: block_avail[slot0 + i] bytes
 * of block i exist at its address and bytes [avail, B) read as zero (values
 * above B count as B; block_avail NULL = every block has B).  This is zfec's
 * padded last data block read in place from the chunk buffer: avail = B - padlen
 * (the same mechanism as sec_msg.avail).  Nothing past a block's avail is read. */
int sec_decode_batch_ex(sec_ctx *ctx, const sec_dec_chunk *chunks, int64_t nchunks,
                        const int32_t *sharenums, const uint64_t *block_offs,
                        const uint64_t *block_avail, const uint8_t *blocks, uint8_t *out,
                        unsigned flags);

/* ---- piece ids: SHA-1 (piece_hash, /root/reference/storb/util/piece.py:54-68) ----
 * A message is `len` bytes at `addr`, of which the first `avail` exist in
 * memory and the rest read as zero (so zfec's zero-padded last data block can
 * be hashed in place).  digests: 20 bytes per message, in order.
 * Device mode: addr / digests are device memory.  SEC_F_HOST: both are host
 * memory (messages are staged through pinned slabs).                        */
typedef struct sec_msg {
    uint64_t addr;
    uint64_t len;
    uint64_t avail;
} sec_msg;

int sec_sha1_batch(sec_ctx *ctx, const sec_msg *msgs, int64_t nmsgs, uint8_t *digests, unsigned flags);

/* Encode + the SHA-1 of every one of the chunk's m blocks (the piece ids the
 * validator computes right after encode, validator.py:1081), while data and
 * parity are still on the device.  Block j of chunk c gets digest slot
 * M_c + j with M_c = sum of m over chunks before c; digests (20 B per slot)
 * live where the parity does (device, or host with SEC_F_HOST). */
int sec_encode_digest_batch(sec_ctx *ctx, const sec_enc_chunk *chunks, int64_t nchunks,
                            const uint8_t *in, uint8_t *parity, uint8_t *digests, unsigned flags);

/* ---- pieces: easyfec's Encoder.encode output in the caller's piece buffers -------------------
 * Replaces zfec.easyfec.Encoder(k, m).encode(chunk) at /root/reference/storb/util/piece.py:
 * 129-130 (k slices copied out of the chunk, the last zero-padded, then the m - k parity
 * blocks), writing every one of chunk c's m pieces to its own host buffer pieces[M_c + j]
 * (B = ceil(n / k) bytes each; M_c = sum of m over chunks before c), and, when digests is not
 * NULL, each piece's SHA-1 (20 bytes at digests + 20 (M_c + j): storb's piece id,
 * hashlib.sha1(piece), piece.py:54-68 / validator.py:1081).  Host memory only (SEC_F_HOST
 * required; SEC_F_STAGED as for sec_encode_batch); chunks[c].parity_off / parity_stride are
 * ignored (the parity goes through a context-owned pinned scratch).  The data pieces are copied
 * and hashed on the context's host threads while the calling thread runs the GPU encode, the
 * parity pieces right after it; the call returns when every piece and digest is written.
 * Preconditions and errors as sec_encode_batch; SEC_EINVAL for a NULL piece buffer of a
 * non-empty chunk.  Flags: SEC_F_HOST (required), SEC_F_STAGED, SEC_F_GPU_PARITY_IDS. */
int sec_encode_pieces(sec_ctx *ctx, const sec_enc_chunk *chunks, int64_t nchunks, const uint8_t *in,
                      uint8_t *const *pieces, uint8_t *digests, unsigned flags);

/* ---- APDP proofs of data possession: 2048-bit modular arithmetic ----------
 * Replaces the gmpy2 calls of storb's ChallengeSystem
 * (/root/reference/storb/challenge/__init__.py:304-350 generate_tag,
 * :401-463 generate_proof, :465-528 verify_proof; gmpy2 2.2.1,
 * /root/reference/uv.lock).  Integers cross the boundary as 256-byte big-endian
 * strings (int.to_bytes(256, "big")).  The modulus is an RSA-2048 modulus:
 * odd, exactly 2048 bits (DEFAULT_RSA_KEY_SIZE, storb/constants.py:26);
 * anything else is SEC_EMODULUS.  Results are fully reduced (< n).
 * Device mode: every data pointer is device memory; SEC_F_HOST: host memory. */
typedef struct sec_bn_key sec_bn_key;

int sec_bn_key_create(sec_ctx *ctx, const uint8_t n_be[256], sec_bn_key **out);
void sec_bn_key_destroy(sec_bn_key *key);
/* The key owner's factors (the validator's RSA key): n = p*q with p, q odd and exactly
 * 1024 bits (128 B big-endian each), cp = q*(q^-1 mod p) and cq = p*(p^-1 mod q) (256 B,
 * mod n).  Enables sec_bn_crt_modexp_batch and CRT tags.  The caller guarantees
 * n = p*q; p or q not odd 1024-bit integers give SEC_EMODULUS. */
int sec_bn_key_set_crt(sec_ctx *ctx, sec_bn_key *key, const uint8_t p_be[128], const uint8_t q_be[128],
                       const uint8_t cp_be[256], const uint8_t cq_be[256]);
/* generate_tag's per-key constants: g, fdh = full_domain_hash(prf(prf_key, 0)) (each taken
 * mod n) and the private exponent d (< 2^2048), 256 B each.  dp, dq (128 B each, or both
 * NULL): exponents for p and q congruent to d mod p-1 and q-1, nonzero when d is (e.g.
 * (d-1) mod (p-1) + 1); given with a CRT key, tags run as two 1024-bit halves.  Builds the
 * key's 16 MiB fixed-base table of g (sec_apdp_gpow_batch, tags).  Host memory. */
int sec_bn_key_set_tag(sec_ctx *ctx, sec_bn_key *key, const uint8_t g_be[256], const uint8_t fdh_be[256],
                       const uint8_t d_be[256], const uint8_t *dp_be, const uint8_t *dq_be);

/* out[i] = int.from_bytes(message i, "big") mod n (256 B each); messages as in
 * sec_sha1_batch (bytes past `avail` read as zero).  block_int of
 * generate_tag / generate_proof. */
int sec_bn_reduce_batch(sec_ctx *ctx, const sec_bn_key *key, const sec_msg *msgs, int64_t nmsgs,
                        uint8_t *out, unsigned flags);
/* out[i] = bases[i] ^ exps[i] mod n.  bases: 256 B each (any value < 2^2048);
 * exps: exp_bytes each, big-endian (1 <= exp_bytes <= 4096). */
int sec_bn_modexp_batch(sec_ctx *ctx, const sec_bn_key *key, const uint8_t *bases,
                        const uint8_t *exps, uint32_t exp_bytes, int64_t count, uint8_t *out,
                        unsigned flags);
/* out[i] = bases[i] ^ e[i] mod n by CRT, given exps_p[i] / exps_q[i] (exp_bytes each,
 * big-endian, 1 <= exp_bytes <= 4096) congruent to e[i] mod p-1 / q-1 and nonzero when
 * e[i] is (e.g. (e-1) mod (p-1) + 1): exact for every base, including multiples of p or
 * q.  Needs sec_bn_key_set_crt. */
int sec_bn_crt_modexp_batch(sec_ctx *ctx, const sec_bn_key *key, const uint8_t *bases,
                            const uint8_t *exps_p, const uint8_t *exps_q, uint32_t exp_bytes,
                            int64_t count, uint8_t *out, unsigned flags);
/* out[i] = g ^ exps[i] mod n from the fixed-base table (issue_challenge's g_s,
 * challenge/__init__.py:387); exps: exp_bytes each, 1 <= exp_bytes <= 256.  Needs
 * sec_bn_key_set_tag. */
int sec_apdp_gpow_batch(sec_ctx *ctx, const sec_bn_key *key, const uint8_t *exps, uint32_t exp_bytes,
                        int64_t count, uint8_t *out, unsigned flags);
/* out[i] = a[i] * b[i] mod n (256 B each, any values < 2^2048). */
int sec_bn_mulmod_batch(sec_ctx *ctx, const sec_bn_key *key, const uint8_t *a, const uint8_t *b,
                        int64_t count, uint8_t *out, unsigned flags);
/* APDP tags, fused per message: X = message mod n; tag = (fdh * g^X)^d mod n
 * (generate_tag's tag_value), g^X from the fixed-base table, the d power by CRT when
 * the key has it.  Needs sec_bn_key_set_tag; 256 B per tag. */
int sec_apdp_tag_batch(sec_ctx *ctx, const sec_bn_key *key, const sec_msg *msgs, int64_t nmsgs,
                       uint8_t *tags, unsigned flags);

/* ---- memory helpers for hosts without a device allocator ----------------- */
int sec_malloc(sec_ctx *ctx, size_t bytes, void **dptr);
int sec_free(sec_ctx *ctx, void *dptr);
int sec_host_alloc(sec_ctx *ctx, size_t bytes, void **hptr); /* pinned */
int sec_host_free(sec_ctx *ctx, void *hptr);                 /* ctx may be NULL */
/* Page-lock an existing host buffer (hipHostRegister) so SEC_F_HOST calls on it take the
 * zero-copy path; unregister (ctx may be NULL) before freeing it. */
int sec_host_register(sec_ctx *ctx, void *hptr, size_t bytes);
int sec_host_unregister(sec_ctx *ctx, void *hptr);
/* SEC_F_HOST encode / decode calls so far on this context: zero-copy on the caller's pinned
 * buffers, zero-copy on pages the call locked itself, and staged. */
int sec_ctx_host_paths(sec_ctx *ctx, int64_t *zero_copy, int64_t *registered, int64_t *staged);
/* Pinned staging memory of the whole process (all contexts): bytes lent to host-mode calls in
 * progress, and idle bytes the library keeps for the next call (at most 512 MiB; the rest is
 * freed).  A context holds none between calls: its slabs and parity scratch are borrowed per
 * call from one process-wide pool.  Either pointer may be NULL. */
int sec_host_pinned_bytes(int64_t *loaned, int64_t *idle);
/* Chunks with a lost data block decoded so far on this context, by method: `syndrome` (the
 * wide-decode path: bit-sliced syndromes of the present parity rows, then the e x e solve) and
 * `direct` (the decode matrix rows over all k blocks).  Which one a chunk takes is the library's
 * choice (cost estimate; context option SEC_SYN = 0 / 1 turns the syndrome path off / forces
 * it where it applies); the bytes are the same. */
int sec_ctx_decode_paths(sec_ctx *ctx, int64_t *syndrome, int64_t *direct);
/* The same chunks by kernel: the one-wave fused syndrome kernel, `pair` (always 0 since round 5:
 * the one-kernel wave pair for parity rows of both groups of zfec(64,96) lost its A/B and is no
 * longer built; the slot stays for ABI stability), the two syndrome kernels (syndromes through
 * device scratch), the direct decode (syndrome = fused + two_kernel). */
int sec_ctx_decode_methods(sec_ctx *ctx, int64_t *fused, int64_t *pair, int64_t *two_kernel, int64_t *direct);
/* kind: 0 host->device, 1 device->host, 2 device->device; synchronous on the ctx stream */
int sec_memcpy(sec_ctx *ctx, void *dst, const void *src, size_t bytes, int kind);
int sec_memset(sec_ctx *ctx, void *dptr, int value, size_t bytes);
/* Host-to-host copies on the context's copy threads (the caller's thread takes part): dst[i] <-
 * src[i] for len[i] bytes, src 0 = zero-fill.  The Python layer joins a reassembled chunk's rows
 * (present pieces and recovered rows) into its output object with this instead of a
 * single-threaded b"".join (easyfec's join, /root/reference/storb/util/piece.py:196-197). */
typedef struct sec_copy {
    uint64_t dst;
    uint64_t src;
    uint64_t len;
} sec_copy;
int sec_host_copy(sec_ctx *ctx, const sec_copy *jobs, int64_t njobs);

#ifdef __cplusplus
}
#endif
#endif /* STORB_EC_H */
