// kernels.hip — CDNA4 (gfx950) kernels for GF(2^8) Reed–Solomon encode / decode.
//
// What they compute is zfec's fec_encode / fec_decode (restated in
// oracle/fec_oracle.c; called from /root/reference/storb/util/piece.py:129-130
// and :196-197 through zfec.easyfec):
//     out_r[t] = XOR_j  c_rj * in_j[t]        over GF(2^8) / 0x11D
//
// How.  The work is byte-wise and HBM-bound (a few VALU ops per byte, no
// matrix shape), so there is no MFMA and no LDS in the hot loop:
//   * multiplication by a constant c is GF(2)-linear in the byte x, so with
//     x = lo3 | mid3 << 3 | hi2 << 6
//         c*x = c*lo3  ^  c*(mid3 << 3)  ^  c*(hi2 << 6)
//     and each term is an 8- (or 4-) entry byte table: exactly what one
//     v_perm_b32 looks up for 4 bytes at once (its 8-byte source = the table,
//     its selector = the 3-bit fields).  So one coefficient costs 3 v_perm +
//     2 XOR per dword, and the 3 selectors of an input dword are shared by all
//     output rows.  The tables (5 dwords per coefficient) are wave-uniform and
//     arrive through scalar loads.
//   * the tables themselves are expanded on the device from the coefficient
//     bytes by sec_expand_tables, which stages the GF(2^8) exp/log tables in
//     LDS and forms every product as exp[log c + log v].
//   * each lane streams 16 B (global_load_dwordx4) per block per u-step, so a
//     wave reads one coalesced 1 KiB run from each of the k blocks; block
//     starts that are not 16 B aligned (B % 16 != 0) use the hardware's
//     unaligned dwordx4 access; the last data block's zero padding is
//     synthesised by the byte-granular tail kernels (at most padlen positions per
//     chunk), never read.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "kernels.hpp"

using u8 = uint8_t;
using u32 = uint32_t;
using u64 = uint64_t;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(1)));  // byte-aligned 16 B access

namespace {

struct GfTables {
    u8 exp[512];
    u8 log[256];
};

constexpr GfTables make_gf()
{
    GfTables t{};
    u32 v = 1;
    for (int e = 0; e < 255; ++e) {
        t.exp[e] = (u8)v;
        t.exp[e + 255] = (u8)v;
        t.log[v] = (u8)e;
        v <<= 1;
        if (v & 0x100)
            v ^= 0x11D;
    }
    t.exp[510] = t.exp[0];
    t.exp[511] = t.exp[1];
    t.log[0] = 255;  // sentinel; products with 0 are special-cased
    return t;
}

__constant__ GfTables c_gf = make_gf();

// ---- table expansion: coefficient byte -> 5 v_perm tables ---------------
__global__ __launch_bounds__(256) void sec_expand_tables(const u8 *__restrict__ coef, u32 ncoef,
                                                         u32 *__restrict__ tabs)
{
    __shared__ u8 s_exp[512];
    __shared__ u8 s_log[256];
    for (u32 i = threadIdx.x; i < 512; i += blockDim.x)
        s_exp[i] = c_gf.exp[i];
    for (u32 i = threadIdx.x; i < 256; i += blockDim.x)
        s_log[i] = c_gf.log[i];
    __syncthreads();
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ncoef)
        return;
    const u32 c = coef[i];
    const u32 lc = s_log[c];
    auto mul = [&](u32 v) -> u32 { return (c && v) ? (u32)s_exp[lc + s_log[v]] : 0u; };
    auto pack = [&](u32 a, u32 b, u32 cc, u32 d) { return mul(a) | mul(b) << 8 | mul(cc) << 16 | mul(d) << 24; };
    u32 *o = tabs + (u64)i * sec::kTabDwords;
    o[0] = pack(0, 1, 2, 3);                      // c * lo3,        lo3 = 0..3
    o[1] = pack(4, 5, 6, 7);                      //                 lo3 = 4..7
    o[2] = pack(0 << 3, 1 << 3, 2 << 3, 3 << 3);  // c * (mid3<<3), mid3 = 0..3
    o[3] = pack(4 << 3, 5 << 3, 6 << 3, 7 << 3);  //                 mid3 = 4..7
    o[4] = pack(0 << 6, 1 << 6, 2 << 6, 3 << 6);  // c * (hi2<<6),   hi2 = 0..3
}

// gfx950's three-input bitwise op (v_bitop3_b32, truth table as the immediate).  The
// compiler does not form it from C: a 4-term XOR took 3 v_xor_b32 (GF accumulation, SHA-1
// message schedule) and SHA-1's Maj 2 ops.  Only symmetric tables are used (0x96 = XOR3,
// 0xE8 = Maj), so the operand order of the table does not matter.
__device__ __forceinline__ u32 xor3(u32 a, u32 b, u32 c)
{
    u32 r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// Ch(b, c, d) = (b & c) | (~b & d); written as C the compiler folded it into the round's
// additions as 3 ops (sub, and, and_or)
__device__ __forceinline__ u32 bfi(u32 b, u32 c, u32 d)
{
    u32 r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(c), "v"(d));
    return r;
}
__device__ __forceinline__ u32 maj(u32 a, u32 b, u32 c)
{
    u32 r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe8" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// ---- the multiply-accumulate ------------------------------------------------
template <int U>
struct Sel {  // the 3 v_perm selectors of each dword of x: bits 0-2, 3-5, 6-7 of every byte
    u32 s0[U][4], s1[U][4], s2[U][4];
    __device__ __forceinline__ explicit Sel(const u32x4 (&x)[U])
    {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const u32 v = x[u][w];
                s0[u][w] = v & 0x07070707u;
                s1[u][w] = (v >> 3) & 0x07070707u;
                s2[u][w] = (v >> 6) & 0x03030303u;
            }
    }
};
__device__ __forceinline__ u32 perm(u32 hi, u32 lo, u32 sel) { return __builtin_amdgcn_perm(hi, lo, sel); }

// SEC_LDS_TAB: v_perm is VOP3, which reads at most one SGPR, so with every table dword in
// SGPRs (scalar loads) one source of perm(c[1], c[0]) and of perm(c[3], c[2]) is first copied
// into a VGPR: 2 v_mov per coefficient and wave, 0.5 per dword and row at U = 1 (8 % of C4's
// encode VALU).  With the knob on, each wave keeps dwords 1 and 3 of its batch's coefficients
// in its own slice of LDS (filled by vector loads at the batch's start; the same wave writes
// and reads it, so no barrier), and the products read them with one ds_read_b64 per
// coefficient instead of the two v_mov.
// SEC_LDS_TAB = 0 off, 1 every tile kernel, 2 (default) the encode kernels of 8-row groups
// only.  Against the SGPR-only build (profiles/r02_ldstab.jsonl, one process per shape):
// encode of 8-row groups zfec(16,24) +4 %, (32,48) +1 %, (64,96) +5 %; but C2 encode -6 %,
// C4 -3 %, C5 -6 %, and the wide decodes -35 % (VGPR spills), so it stays off there.
#ifndef SEC_LDS_TAB
#define SEC_LDS_TAB 2
#endif
template <int R, bool DEC>
__host__ __device__ constexpr bool lds_tab() { return SEC_LDS_TAB == 1 || (SEC_LDS_TAB == 2 && !DEC && R == 8); }
using u32x2 = uint2;

// SEC_PROBE_NOGF (build knob, calibration only; never the product): every GF product replaced by
// the block itself (acc ^= x), so a variant library moves exactly the product kernels' bytes with
// the same tiles and descriptors but no field arithmetic -- the access pattern's own ceiling
// (tools/c5_classes.py --lib).  Its outputs are not Reed-Solomon parity.
#ifndef SEC_PROBE_NOGF
#define SEC_PROBE_NOGF 0
#endif

// acc[r] ^= coefficient(r) * x for one block: 3 v_perm + 2 XOR per dword and row
// (t: the block's first row's 5 table dwords; v: its dwords 1 and 3 in LDS, SEC_LDS_TAB only)
template <int R, int U, bool LT = false>
__device__ __forceinline__ void gf_mac(u32x4 (&acc)[R][U], const u32x4 (&x)[U], const u32 *__restrict__ t,
                                       const u32x2 *v)
{
    if constexpr (SEC_PROBE_NOGF) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u)
                acc[r][u] ^= x[u];
        return;
    }
    const Sel<U> s(x);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const u32 *c = t + r * 5;
        u32 c1 = c[1], c3 = c[3];
        if constexpr (LT) {
            const u32x2 h = v[r];
            c1 = h.x;
            c3 = h.y;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int w = 0; w < 4; ++w)
                acc[r][u][w] = xor3(acc[r][u][w], perm(c1, c[0], s.s0[u][w]), perm(c3, c[2], s.s1[u][w])) ^
                               perm(c[4], c[4], s.s2[u][w]);
    }
}

// In the k <= 16 kernels blocks go to gf_mac2 in pairs only for row groups of <= 4 rows: with 8 rows the second
// block's selectors cost registers, and zfec(16,24) measured encode -14 %, decode -42 %
// (C4 encode +12 %, C2 +1 %; profiles/r01_sweep_xor3.jsonl)
// The wide-k (W) kernels load smaller batches (SEC_WIDE_BATCH), which leaves the registers
// to pair blocks for 8-row groups too: zfec(32,48) / (64,96) encode +11 %, decode +7-10 %
// (profiles/r01_sweep_wide_pair.jsonl).
#ifndef SEC_PAIR_ROWS
#define SEC_PAIR_ROWS 4
#endif
#ifndef SEC_WIDE_PAIR_ROWS
#define SEC_WIDE_PAIR_ROWS 8
#endif
template <int R, bool W>
__host__ __device__ constexpr bool kPairRows() { return R <= (W ? SEC_WIDE_PAIR_ROWS : SEC_PAIR_ROWS); }

// Two blocks at once: the 6 products of a dword and row go into acc by 3 XOR3s, so 3 v_perm
// + 1.5 XOR per dword, row and block (a 4-term XOR chain in C took 3 v_xor_b32 per block)
template <int R, int U, bool LT = false>
__device__ __forceinline__ void gf_mac2(u32x4 (&acc)[R][U], const u32x4 (&x)[U], const u32 *__restrict__ t,
                                        const u32x2 *v, const u32x4 (&y)[U], const u32 *__restrict__ q,
                                        const u32x2 *vq)
{
    if constexpr (SEC_PROBE_NOGF) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u)
                acc[r][u] ^= x[u] ^ y[u];
        return;
    }
    const Sel<U> s(x), z(y);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const u32 *c = t + r * 5, *d = q + r * 5;
        u32 c1 = c[1], c3 = c[3], d1 = d[1], d3 = d[3];
        if constexpr (LT) {
            const u32x2 h = v[r], g = vq[r];
            c1 = h.x;
            c3 = h.y;
            d1 = g.x;
            d3 = g.y;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                u32 a = xor3(acc[r][u][w], perm(c1, c[0], s.s0[u][w]), perm(c3, c[2], s.s1[u][w]));
                a = xor3(a, perm(c[4], c[4], s.s2[u][w]), perm(d1, d[0], z.s0[u][w]));
                acc[r][u][w] = xor3(a, perm(d3, d[2], z.s1[u][w]), perm(d[4], d[4], z.s2[u][w]));
            }
    }
}

// SEC_LDS_TAB: this wave's LDS slice, filled by its active lanes with dwords 1 and 3 of the tables of blocks
// j0 .. j0 + KB - 1 (those < k), rows 0 .. R - 1 (tj: row 0 of block 0, tstep: dwords per
// block), entry c * R + r.  The launch passes (lanes / 64) * KB * R * 8 bytes of dynamic LDS.
template <int KB, int R, bool LT>
__device__ __forceinline__ const u32x2 *wave_tabs(const u32 *__restrict__ tj, u32 tstep, u32 j0, u32 k)
{
    extern __shared__ u32x2 s_vt[];
    u32x2 *vt = s_vt + (threadIdx.x >> 6) * (KB * R);
    if constexpr (LT && R > 0) {
        // the wave's active lanes share the fill (lanes past a tile's `valid` never get here)
        const u64 live = __builtin_amdgcn_read_exec();
        const u32 rank = __builtin_amdgcn_mbcnt_hi((u32)(live >> 32), __builtin_amdgcn_mbcnt_lo((u32)live, 0u));
        const u32 nlive = (u32)__builtin_popcountll(live);
        for (u32 i = rank; i < (u32)(KB * R); i += nlive) {
            const u32 c = i / R, r = i % R;
            if (j0 + c < k) {
                const u32 *src = tj + (j0 + c) * tstep + r * sec::kTabDwords;
                vt[i] = u32x2{src[1], src[3]};
            }
        }
    }
    return vt;
}
// Dynamic LDS bytes of a tile launch (0 without SEC_LDS_TAB)
template <int KB, int R, bool DEC>
constexpr u32 lds_tab_bytes(u32 lanes) { return lds_tab<R, DEC>() ? lanes / 64 * KB * R * 8 : 0; }

// Build knobs (A/B variants are compiled as separate libraries by tools/sweep.py):
//   SEC_NT_LOAD / SEC_NT_STORE  nontemporal (streaming) global loads / stores: every
//                               byte is touched once, so keeping it out of the caches
//                               measured +11% on encode, +4% on decode (r01 sweep)
//   SEC_ENC_BATCH / SEC_DEC_BATCH  16-byte vectors per lane loaded as one batch (all
//                               issued before any arithmetic): KB = this / U blocks (slots)
//                               per batch.  Decode batching: C2 +4 %, RS(8,3) +6.6 %, C4 +2 %
//                               (r01 sweep_dec_batch); encode: C2 +3.5 %, C4 +9 %
//   SEC_ENC_ST / SEC_DEC_ST     store cache policy of the encode / decode kernels:
//                               0 plain, 1 nt, 2 "nt sc1" (write-through, line dropped from
//                               L2), 3 "sc0 sc1".  The asm forms end in s_nop 1: a store of
//                               more than 8 bytes reads its data VGPRs after issue, and the
//                               compiler, blind to the asm, may overwrite them at once
#ifndef SEC_NT_LOAD
#define SEC_NT_LOAD 1
#endif
#ifndef SEC_NT_STORE
#define SEC_NT_STORE 1
#endif
#ifndef SEC_ENC_ST
#define SEC_ENC_ST SEC_NT_STORE
#endif
#ifndef SEC_DEC_ST
#define SEC_DEC_ST SEC_NT_STORE
#endif
#ifndef SEC_DEC_BATCH
#define SEC_DEC_BATCH sec::kBatchVecs
#endif
//   SEC_DEC_LATE                decode: store a batch's present primaries after its GF work
//                               (1) or as each slot arrives (0): C4 decode +5 %, C2 / C5
//                               within noise (profiles/r01_sweep_declate.jsonl)
#ifndef SEC_DEC_LATE
#define SEC_DEC_LATE 1
#endif
#ifndef SEC_ENC_BATCH
#define SEC_ENC_BATCH sec::kBatchVecs
#endif
//   SEC_WIDE_BATCH              vectors per batch in the wide-k (W) kernels, which loop over
//                               batches; default: the encode / decode batch
#ifndef SEC_WIDE_BATCH
#define SEC_WIDE_BATCH 8
#endif
//   (Rounds 1-5 also tried, and archived: a compile-time k for single-shape workloads, VGPR caps
//   through amdgpu_waves_per_eu, LDS padding to cap the decode's workgroups per CU.)
// Blocks (slots) per batch of a tile kernel: KB * U = the batch's 16 B vectors per lane
template <int U, bool W, bool DEC>
constexpr int batch_blocks()
{
    constexpr int v = (W && SEC_WIDE_BATCH > 0) ? SEC_WIDE_BATCH : (DEC ? SEC_DEC_BATCH : SEC_ENC_BATCH);
    return v / U > 0 ? v / U : 1;
}

__device__ __forceinline__ u32x4 load16(const u8 *p)
{
#if SEC_NT_LOAD
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4_u *>(p));
#else
    return *reinterpret_cast<const u32x4_u *>(p);
#endif
}
template <int POL>
__device__ __forceinline__ void store16(u8 *p, u32x4 v)
{
    if constexpr (POL == 0)
        *reinterpret_cast<u32x4_u *>(p) = v;
    else if constexpr (POL == 1)
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4_u *>(p));
    else if constexpr (POL == 2)
        asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// GF(2^8) product of one byte through the same 5-dword table (tail kernels)
__device__ __forceinline__ u32 gf_mul_byte(const u32 *__restrict__ t, u32 x)
{
    return (__builtin_amdgcn_perm(t[1], t[0], x & 7u) ^ __builtin_amdgcn_perm(t[3], t[2], (x >> 3) & 7u) ^
            __builtin_amdgcn_perm(t[4], t[4], x >> 6)) & 0xFFu;
}

// ---- encode ----------------------------------------------------------------
// Tile = (chunk, t0, r0): lanes cover t0 + 16*lane + 4096*u.  Every position handled here
// is < `valid` (all k blocks fully readable there, including the last, shorter data
// block); a lane's 16 bytes are clamped to end at `valid`, so the last lane of a ragged
// chunk overlaps its neighbour (identical bytes written twice) instead of taking a
// byte-granular path.  Positions in [valid, B) — at most padlen of them — are computed
// byte by byte by the chunk's last tile (Tile::ntail, encode_ragged) after its main work.
template <int R, int U, bool W>
__device__ __forceinline__ void encode_main(const u8 *__restrict__ in, u8 *__restrict__ par, const sec::EncDesc &d,
                                            const sec::Tile &tl, const u32 *__restrict__ tabs, u32 t);
template <int R>
__device__ __forceinline__ void encode_ragged(const u8 *__restrict__ in, u8 *__restrict__ par, const sec::EncDesc &d,
                                           const sec::Tile &tl, const u32 *__restrict__ tabs);

template <int R, int U, bool W>
__global__ __launch_bounds__(sec::max_lanes(R, U)) void sec_encode_kernel(const u8 *__restrict__ in, u8 *__restrict__ par,
                                                         const sec::EncDesc *__restrict__ descs,
                                                         const sec::Tile *__restrict__ tiles,
                                                         const u32 *__restrict__ tabs)
{
    const sec::Tile tl = tiles[blockIdx.x];
    const sec::EncDesc d = descs[tl.chunk];
    const u32 t = tl.t0 + threadIdx.x * sec::kLaneBytes;
    if (t < d.valid)
        encode_main<R, U, W>(in, par, d, tl, tabs, t);
    if (tl.ntail)
        encode_ragged<R>(in, par, d, tl, tabs);
}

template <int R, int U, bool W>
__device__ __forceinline__ void encode_main(const u8 *__restrict__ in, u8 *__restrict__ par, const sec::EncDesc &d,
                                            const sec::Tile &tl, const u32 *__restrict__ tabs, u32 t)
{
    const u32 B = d.B, k = d.k, valid = d.valid;
    const u32 step = blockDim.x * sec::kLaneBytes;  // bytes one u-step of the workgroup covers
    u32 pos[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        pos[u] = min(t + u * step, valid - sec::kLaneBytes);
    const u8 *row = in + d.in_off;
    u8 *dst = par + d.par_off + (u64)tl.r0 * d.par_stride;
    const u32 *tj = tabs + d.tab + tl.r0 * sec::kTabDwords;
    const u32 tstep = d.p * sec::kTabDwords;

    u32x4 acc[R][U];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc[r][u] = u32x4{0u, 0u, 0u, 0u};

    // Blocks go in batches of KB: every load of a batch is issued before any arithmetic and
    // the batch is consumed in order (counted waits), so a lane keeps KB * U = SEC_ENC_BATCH
    // loads in flight; C2 (k = 4) and C4 (k = 10) are one batch.  A one-block-ahead prefetch
    // loop compiled to a full wait at its head (the next block's load included): one load in
    // flight per lane and u-step, C2 -3.5 %, C4 -9 % (profiles/r01_sweep_enc_batch.jsonl).
    constexpr int KB = batch_blocks<U, W, false>();
    auto batch = [&](u32 j0) {
        constexpr bool LT = lds_tab<R, false>();
        const u32x2 *vt = wave_tabs<KB, R, LT>(tj, tstep, j0, k);
        u32x4 xs[KB][U];
#pragma unroll
        for (int c = 0; c < KB; ++c)
            if (j0 + c < k) {
#pragma unroll
                for (int u = 0; u < U; ++u)
                    xs[c][u] = load16(row + (u64)(j0 + c) * B + pos[u]);
            }
        if constexpr (kPairRows<R, W>()) {
#pragma unroll
            for (int c = 0; c < KB; c += 2) {
                if (c + 1 < KB && j0 + c + 1 < k)
                    gf_mac2<R, U, LT>(acc, xs[c], tj + (j0 + c) * tstep, vt + c * R, xs[c + 1],
                                  tj + (j0 + c + 1) * tstep, vt + (c + 1) * R);
                else if (j0 + c < k)
                    gf_mac<R, U, LT>(acc, xs[c], tj + (j0 + c) * tstep, vt + c * R);
            }
        } else {
#pragma unroll
            for (int c = 0; c < KB; ++c)
                if (j0 + c < k)
                    gf_mac<R, U, LT>(acc, xs[c], tj + (j0 + c) * tstep, vt + c * R);
        }
    };
    // W (wide k, U = 1 only): k > KB, several batches.  A separate instantiation: merely
    // compiling this loop into the k <= KB kernel cost C4 15 % (registers; r01 sweep_wide).
    if constexpr (W) {
#pragma unroll 1
        for (u32 j0 = 0; j0 < k; j0 += KB)
            batch(j0);
    } else {
        batch(0);  // the plan guarantees k <= KB here
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u)
            store16<SEC_ENC_ST>(dst + (u64)r * d.par_stride + pos[u], acc[r][u]);
}

// Lane of the workgroup that takes ragged position i first: the lanes past the tile's main
// range (idle there) come first, then the wrap reaches the busy ones.
__device__ __forceinline__ u32 ragged_lane0(u32 valid, u32 t0)
{
    const u32 used = min(blockDim.x, (valid - t0 + sec::kLaneBytes - 1) / sec::kLaneBytes);
    return (threadIdx.x + blockDim.x - used) % blockDim.x;
}

// The chunk's ragged end [valid, valid + ntail), byte by byte, for this tile's R parity rows:
// blocks 0..k-2 are full there and block k-1 is zero padding, so it contributes nothing.
// Each lane issues its bytes' loads kBatch at a time before using any (a loop of dependent
// single-byte loads costs one memory latency per block).
constexpr u32 kBatch = 16;

template <int R>
__device__ __forceinline__ void encode_ragged(const u8 *__restrict__ in, u8 *__restrict__ par, const sec::EncDesc &d,
                                              const sec::Tile &tl, const u32 *__restrict__ tabs)
{
    const u8 *src = in + d.in_off;
    const u32 nblk = d.k - 1;
    for (u32 i = ragged_lane0(d.valid, tl.t0); i < tl.ntail; i += blockDim.x) {
        const u32 tp = d.valid + i;
        u32 acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r)
            acc[r] = 0;
        for (u32 j0 = 0; j0 < nblk; j0 += kBatch) {
            u32 x[kBatch];
#pragma unroll
            for (u32 q = 0; q < kBatch; ++q)
                x[q] = j0 + q < nblk ? (u32)src[(u64)(j0 + q) * d.B + tp] : 0u;
#pragma unroll
            for (u32 q = 0; q < kBatch; ++q)
                if (j0 + q < nblk) {
                    const u32 *tj = tabs + d.tab + ((j0 + q) * d.p + tl.r0) * sec::kTabDwords;
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        acc[r] ^= gf_mul_byte(tj + r * sec::kTabDwords, x[q]);
                }
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
            par[d.par_off + (u64)(tl.r0 + r) * d.par_stride + tp] = (u8)acc[r];
    }
}

// One thread per (chunk, position) of the chunks too small for a tile (valid < 16):
// all p parity bytes at that position, the last block's padding read as zero.
__global__ __launch_bounds__(256) void sec_encode_tail(const u8 *__restrict__ in, u8 *__restrict__ par,
                                                       const sec::EncDesc *__restrict__ descs,
                                                       const sec::TailItem *__restrict__ items, u32 nitems,
                                                       const u32 *__restrict__ tabs)
{
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nitems)
        return;
    const sec::TailItem it = items[i];
    const sec::EncDesc d = descs[it.chunk];
    const u8 *src = in + d.in_off + it.t;
    for (u32 r = 0; r < d.p; ++r) {
        u32 acc = 0;
        for (u32 j = 0; j < d.k; ++j) {
            const u32 x = (j + 1 < d.k || it.t < d.valid) ? (u32)src[(u64)j * d.B] : 0u;
            acc ^= gf_mul_byte(tabs + d.tab + (j * d.p + r) * sec::kTabDwords, x);
        }
        par[d.par_off + (u64)r * d.par_stride + it.t] = (u8)acc;
    }
}

// ---- decode + reassemble -----------------------------------------------------
// Slot c of a chunk holds block number idx[c]; primaries sit in their own slot
// (zfec's normalisation).  Present primaries are copied to their output row;
// the R missing rows of this tile's row group are XOR_c Minv[row][c] * slot_c.
// Positions are < valid = min(the last output row's length, every slot's avail), so every
// row is writable and every slot readable there; the rest is decode_ragged's (Tile::ntail),
// which reads a slot's bytes past its avail as zero (zfec's padded block k-1 read in place).
// Recover-only decodes (SEC_F_RECOVER) use the same kernels: no copies (row = none) and the
// recovered rows go to output rows 0..e-1.
template <int R, int U, bool W, int KBX>
__device__ __forceinline__ void decode_main(const u8 *__restrict__ blocks, u8 *__restrict__ out,
                                            const sec::DecDesc &d, const sec::Tile &tl, u32 t,
                                            const u32 *__restrict__ tabs, const sec::DecSlots sl);
template <int R>
__device__ __forceinline__ void decode_ragged(const u8 *__restrict__ blocks, u8 *__restrict__ out, const sec::DecDesc &d,
                                           const sec::Tile &tl, const u32 *__restrict__ tabs,
                                           const sec::DecSlots sl);

// KBX > 0: slots per load batch fixed at KBX (the plan sends only chunks with k <= KBX; fewer
// live registers, more waves): recover-only and copy-free decodes, see api.cpp dec_small_kb
template <int R, int U, bool W, int KBX>
__global__ __launch_bounds__(sec::max_lanes(R, U)) void sec_decode_kernel(const u8 *__restrict__ blocks, u8 *__restrict__ out,
                                                         const sec::DecDesc *__restrict__ descs,
                                                         const sec::Tile *__restrict__ tiles,
                                                         const u32 *__restrict__ tabs,
                                                         const sec::DecSlots sl)
{
    const sec::Tile tl = tiles[blockIdx.x];
    const sec::DecDesc d = descs[tl.chunk];
    const u32 t = tl.t0 + threadIdx.x * sec::kLaneBytes;
    if (t < d.valid)
        decode_main<R, U, W, KBX>(blocks, out, d, tl, t, tabs, sl);
    if (tl.ntail)
        decode_ragged<R>(blocks, out, d, tl, tabs, sl);
}

// The chunk's ragged end [valid, valid + ntail), byte by byte: the present primaries' bytes
// (row group 0) and this tile's R recovered rows, wherever the output row still has bytes.
// Every slot's byte is loaded once, kBatch slots at a time, and feeds the copy and all R rows.
template <int R>
__device__ __forceinline__ void decode_ragged(const u8 *__restrict__ blocks, u8 *__restrict__ out, const sec::DecDesc &d,
                                              const sec::Tile &tl, const u32 *__restrict__ tabs,
                                              const sec::DecSlots sl)
{
    for (u32 i = ragged_lane0(d.valid, tl.t0); i < tl.ntail; i += blockDim.x) {
        const u32 tp = d.valid + i;
        u8 *dst = out + d.out_off + tp;
        u32 acc[R > 0 ? R : 1];
#pragma unroll
        for (int r = 0; r < R; ++r)
            acc[r] = 0;
        for (u32 c0 = 0; c0 < d.k; c0 += kBatch) {
            u32 x[kBatch];
#pragma unroll
            for (u32 q = 0; q < kBatch; ++q)
                x[q] = (c0 + q < d.k && tp < sl.avail[d.slot0 + c0 + q]) ? (u32)blocks[sl.off[d.slot0 + c0 + q] + tp] : 0u;
#pragma unroll
            for (u32 q = 0; q < kBatch; ++q)
                if (c0 + q < d.k) {
                    const u32 c = c0 + q;
                    const u32 orow = sl.row[d.slot0 + c];
                    if (tl.r0 == 0 && orow != 0xFFFFFFFFu && (u64)orow * d.B + tp < d.n)
                        dst[(u64)orow * d.B] = (u8)x[q];
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        acc[r] ^= gf_mul_byte(tabs + d.tab + (c * d.e + tl.r0 + r) * sec::kTabDwords, x[q]);
                }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const u32 orow = sl.miss[d.slot0 + tl.r0 + r];
            if ((u64)orow * d.B + tp < d.n)
                dst[(u64)orow * d.B] = (u8)acc[r];
        }
    }
}

template <int R, int U, bool W, int KBX>
__device__ __forceinline__ void decode_main(const u8 *__restrict__ blocks, u8 *__restrict__ out,
                                            const sec::DecDesc &d, const sec::Tile &tl, u32 t,
                                            const u32 *__restrict__ tabs,
                                                         const sec::DecSlots sl)
{
    const u32 B = d.B, k = d.k, valid = d.valid;
    const u32 step = blockDim.x * sec::kLaneBytes;  // bytes one u-step of the workgroup covers
    u32 pos[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        pos[u] = min(t + u * step, valid - sec::kLaneBytes);
    u8 *dst = out + d.out_off;
    const bool copies = tl.r0 == 0;  // row group 0 also copies the present primaries
    const u32 *tj = tabs + d.tab + tl.r0 * sec::kTabDwords;
    const u32 tstep = d.e * sec::kTabDwords;

    u32x4 acc[R > 0 ? R : 1][U];
#pragma unroll
    for (int r = 0; r < (R > 0 ? R : 1); ++r)
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc[r][u] = u32x4{0u, 0u, 0u, 0u};

    // Slots go in batches of KB, as in encode_main: every load of a batch before any store
    // or arithmetic, then the batch in order — each present primary copied to its output
    // row, every slot fed to the R accumulators.  C2 / C4 are one batch (all loads in flight).
    constexpr int KB = KBX > 0 ? KBX : batch_blocks<U, W, true>();
    auto batch = [&](u32 c0) {
        constexpr bool LT = lds_tab<R, true>();
        const u32x2 *vt = wave_tabs<KB, R, LT>(tj, tstep, c0, k);
        // the batch's block offsets in one go (the plan pads sl.off by kBatchVecs entries): one
        // offset loaded and waited for per slot would put KB scalar round trips before the last load
        u64 so[KB];
        const u64 *sop = sl.off + d.slot0 + c0;
#pragma unroll
        for (int c = 0; c < KB; ++c)
            so[c] = sop[c];
        u32x4 xs[KB][U];
#pragma unroll
        for (int c = 0; c < KB; ++c)
            if (c0 + c < k) {
                const u8 *s = blocks + so[c];
#pragma unroll
                for (int u = 0; u < U; ++u)
                    xs[c][u] = load16(s + pos[u]);
            }
        if constexpr (SEC_DEC_LATE) {  // slots in pairs (gf_mac2)
            if constexpr (R > 0 && kPairRows<R, W>()) {
#pragma unroll
                for (int c = 0; c < KB; c += 2) {
                    if (c + 1 < KB && c0 + c + 1 < k)
                        gf_mac2<R, U, LT>(acc, xs[c], tj + (c0 + c) * tstep, vt + c * R, xs[c + 1],
                                      tj + (c0 + c + 1) * tstep, vt + (c + 1) * R);
                    else if (c0 + c < k)
                        gf_mac<R, U, LT>(acc, xs[c], tj + (c0 + c) * tstep, vt + c * R);
                }
            } else if constexpr (R > 0) {
#pragma unroll
                for (int c = 0; c < KB; ++c)
                    if (c0 + c < k)
                        gf_mac<R, U, LT>(acc, xs[c], tj + (c0 + c) * tstep, vt + c * R);
            }
        } else {
#pragma unroll
            for (int c = 0; c < KB; ++c)
                if (c0 + c < k) {
                    const u32 orow = sl.row[d.slot0 + c0 + c];
                    if (copies && orow != 0xFFFFFFFFu) {
                        u8 *o = dst + (u64)orow * B;
#pragma unroll
                        for (int u = 0; u < U; ++u)
                            store16<SEC_DEC_ST>(o + pos[u], xs[c][u]);
                    }
                    if constexpr (R > 0)
                        gf_mac<R, U, LT>(acc, xs[c], tj + (c0 + c) * tstep, vt + c * R);
                }
        }
        if (SEC_DEC_LATE)  // the batch's copies after its arithmetic
#pragma unroll
            for (int c = 0; c < KB; ++c)
                if (c0 + c < k) {
                    const u32 orow = sl.row[d.slot0 + c0 + c];
                    if (copies && orow != 0xFFFFFFFFu) {
                        u8 *o = dst + (u64)orow * B;
#pragma unroll
                        for (int u = 0; u < U; ++u)
                            store16<SEC_DEC_ST>(o + pos[u], xs[c][u]);
                    }
                }
    };
    if constexpr (W) {  // wide k: several batches (see encode_main)
#pragma unroll 1
        for (u32 c0 = 0; c0 < k; c0 += KB)
            batch(c0);
    } else {
        batch(0);  // the plan guarantees k <= KB here
    }
    if constexpr (R > 0) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            u8 *o = dst + (u64)sl.miss[d.slot0 + tl.r0 + r] * B;
#pragma unroll
            for (int u = 0; u < U; ++u)
                store16<SEC_DEC_ST>(o + pos[u], acc[r][u]);
        }
    }
}

// One thread per (chunk, position) outside the main kernel's range: copies and
// recovered bytes for every output row that is still inside the chunk there.
__global__ __launch_bounds__(256) void sec_decode_tail(const u8 *__restrict__ blocks, u8 *__restrict__ out,
                                                       const sec::DecDesc *__restrict__ descs,
                                                       const sec::TailItem *__restrict__ items, u32 nitems,
                                                       const u32 *__restrict__ tabs,
                                                       const sec::DecSlots sl)
{
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nitems)
        return;
    const sec::TailItem it = items[i];
    const sec::DecDesc d = descs[it.chunk];
    u8 *dst = out + d.out_off + it.t;
    auto slot_byte = [&](u32 c) -> u32 {  // bytes past the slot's avail read as zero
        return it.t < sl.avail[d.slot0 + c] ? (u32)blocks[sl.off[d.slot0 + c] + it.t] : 0u;
    };
    for (u32 c = 0; c < d.k; ++c) {
        const u32 orow = sl.row[d.slot0 + c];
        if (orow != 0xFFFFFFFFu && (u64)orow * d.B + it.t < d.n)
            dst[(u64)orow * d.B] = (u8)slot_byte(c);
    }
    for (u32 r = 0; r < d.e; ++r) {
        const u32 orow = sl.miss[d.slot0 + r];
        if ((u64)orow * d.B + it.t >= d.n)
            continue;
        u32 acc = 0;
        for (u32 c = 0; c < d.k; ++c)
            acc ^= gf_mul_byte(tabs + d.tab + (c * d.e + r) * sec::kTabDwords, slot_byte(c));
        dst[(u64)orow * d.B] = (u8)acc;
    }
}

// ---- SHA-1 of pieces (storb piece ids, /root/reference/storb/util/piece.py:54-68) ----
// One lane per message: SHA-1 is a sequential chain of 64-byte compressions, so a
// message cannot be split; the kernel is latency-bound on each lane's round chain
// and wants many messages in flight.  Words are loaded 16 B at a time (unaligned
// allowed) and byte-swapped to SHA-1's big-endian order.
__device__ __forceinline__ u32 rotl(u32 x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }

// FIPS 180-4 SHA-1 compression: per round rotl(a, 5), f (v_bfi / XOR3 / Maj), two add3 and
// rotl(b, 30); per scheduled word XOR3, XOR and a rotate.
__device__ __forceinline__ void sha1_compress(u32 (&h)[5], u32 (&w)[16])
{
    u32 a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#pragma unroll
    for (int t = 0; t < 80; ++t) {
        u32 wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = rotl(xor3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
            w[t & 15] = wt;
        }
        u32 f, k;
        if (t < 20) {
            f = bfi(b, c, d);
            k = 0x5A827999u;
        } else if (t < 40) {
            f = xor3(b, c, d);
            k = 0x6ED9EBA1u;
        } else if (t < 60) {
            f = maj(b, c, d);
            k = 0x8F1BBCDCu;
        } else {
            f = xor3(b, c, d);
            k = 0xCA62C1D6u;
        }
        const u32 tmp = rotl(a, 5) + f + (e + k + wt);
        e = d;
        d = c;
        c = rotl(b, 30);
        b = a;
        a = tmp;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
    h[4] += e;
}

// byte i of the message: real below `avail`, zero from there to `len`
// Blocks are loaded SEC_SHA1_DEPTH ahead of their compression (a ring of registers), so a
// block's load latency overlaps earlier blocks' round chains.  Interleaved in-process A/B
// against the plain loop (tools/sha1_ab.py, profiles/r02_sha1_prefetch_ab.jsonl; HIP-event
// kernel times, median of 7 rounds, spread under 2 %): 1.14x on C4's 114688 pieces of
// 6554 B (1.75 waves per SIMD) and 1.26-1.37x on every other shape measured (C2's 6144
// pieces of 256 KiB, 4096 x 1 MiB, 16384 x 64 KiB, 65536 x 16 KiB, 32768 x 6554 B), so it
// is used for every launch.  (Round 1 kept the plain loop for >= 65536 messages on wall-time
// numbers that were dominated by launch and sync time.)  SEC_SHA1_PF = 0 forces it off (A/B).
#ifndef SEC_SHA1_PF
#define SEC_SHA1_PF 1
#endif
#ifndef SEC_SHA1_DEPTH
#define SEC_SHA1_DEPTH 2
#endif
__device__ __forceinline__ u32 msg_byte(const u8 *p, uint64_t i, uint64_t avail) { return i < avail ? p[i] : 0u; }

template <bool PF>
__global__ __launch_bounds__(64) void sec_sha1_kernel(const u8 *__restrict__ base0, const u8 *__restrict__ base1,
                                                      const sec::MsgDesc *__restrict__ msgs, u32 nmsgs,
                                                      u8 *__restrict__ digests)
{
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nmsgs)
        return;
    const sec::MsgDesc m = msgs[i];
    const u8 *p = (m.base ? base1 : base0) + m.off;
    u32 h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    u32 w[16];
    const uint64_t nfull = m.len / 64;
    // PF: the next block's four 16 B loads are issued before this block's compression, so
    // with one wave per SIMD their latency overlaps the round chain
    const uint64_t nfast = PF ? min(nfull, m.avail / 64) : 0;  // blocks wholly inside the real bytes
    // SEC_SHA1_DEPTH blocks ahead (1 or 2), in a ring of registers walked by an unrolled loop
    constexpr int D = SEC_SHA1_DEPTH;
    u32x4 nx[D][4];
#pragma unroll
    for (int d = 0; d < D; ++d)
        if ((uint64_t)d < nfast) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                nx[d][q] = *reinterpret_cast<const u32x4_u *>(p + d * 64 + 16 * q);
        }
    for (uint64_t b0 = 0; b0 < nfast; b0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const uint64_t blk = b0 + d;
            if (blk < nfast) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    w[4 * q + 0] = __builtin_bswap32(nx[d][q].x);
                    w[4 * q + 1] = __builtin_bswap32(nx[d][q].y);
                    w[4 * q + 2] = __builtin_bswap32(nx[d][q].z);
                    w[4 * q + 3] = __builtin_bswap32(nx[d][q].w);
                }
                if (blk + D < nfast) {
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        nx[d][q] = *reinterpret_cast<const u32x4_u *>(p + (blk + D) * 64 + 16 * q);
                }
                sha1_compress(h, w);
            }
        }
    }
    for (uint64_t blk = nfast; blk < nfull; ++blk) {
        const uint64_t o = blk * 64;
        if (o + 64 <= m.avail) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const u32x4 v = *reinterpret_cast<const u32x4_u *>(p + o + 16 * q);
                w[4 * q + 0] = __builtin_bswap32(v.x);
                w[4 * q + 1] = __builtin_bswap32(v.y);
                w[4 * q + 2] = __builtin_bswap32(v.z);
                w[4 * q + 3] = __builtin_bswap32(v.w);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                u32 x = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    x = (x << 8) | msg_byte(p, o + 4 * q + b, m.avail);
                w[q] = x;
            }
        }
        sha1_compress(h, w);
    }
    // final block(s): remaining bytes, 0x80, zeros, 64-bit big-endian bit length
    const uint64_t o = nfull * 64;
    const u32 rem = (u32)(m.len - o);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        u32 x = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const u32 pos = 4 * q + b;
            const u32 byte = pos < rem ? msg_byte(p, o + pos, m.avail) : (pos == rem ? 0x80u : 0u);
            x = (x << 8) | byte;
        }
        w[q] = x;
    }
    const uint64_t bits = m.len * 8;
    if (rem >= 56) {
        sha1_compress(h, w);
#pragma unroll
        for (int q = 0; q < 16; ++q)
            w[q] = 0;
    }
    w[14] = (u32)(bits >> 32);
    w[15] = (u32)bits;
    sha1_compress(h, w);
    u32 *out = reinterpret_cast<u32 *>(digests + (uint64_t)i * 20);
#pragma unroll
    for (int q = 0; q < 5; ++q)
        out[q] = __builtin_bswap32(h[q]);
}

// SHA-1 with the message schedule on a second wave (few, long messages: the latency-bound
// regime, e.g. C2's 6144 pieces of 256 KiB are 96 waves, one per SIMD at most).  A workgroup is
// two waves for the same 64 messages: wave 1 loads each block (prefetched), byte-swaps it and
// expands the 80 schedule words W_t + K_t into LDS; wave 0 runs only the 80 rounds from LDS
// (rotl 5, f, add3, add, rotl 30: 5 VALU per round, 405 per block against 597 with the
// schedule inline), one block behind, the two buffers handed over by one s_barrier per block.
// Blocks past a message's real bytes (zfec's zero padding) and the final padded block(s) go
// through sha1_compress on wave 0 afterwards, as in sec_sha1_kernel.
constexpr u32 kShaK[4] = {0x5A827999u, 0x6ED9EBA1u, 0x8F1BBCDCu, 0xCA62C1D6u};

__device__ __forceinline__ void sha1_rounds_wk(u32 (&h)[5], const u32x4 (&vs)[20])
{
    u32 a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#pragma unroll
    for (int q = 0; q < 20; ++q) {
        const u32x4 v = vs[q];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int t = 4 * q + j;
            const u32 f = t < 20 ? bfi(b, c, d) : t < 40 ? xor3(b, c, d) : t < 60 ? maj(b, c, d) : xor3(b, c, d);
            const u32 tmp = rotl(a, 5) + f + e + v[j];
            e = d;
            d = c;
            c = rotl(b, 30);
            b = a;
            a = tmp;
        }
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
    h[4] += e;
}

// one block's 80 words from LDS into registers (left to the scheduler, the reads went out two
// at a time, each pair waited for a few rounds later: 1.06x over the one-lane kernel, not 1.26x)
__device__ __forceinline__ void sha1_fetch_wk(u32x4 (&vs)[20], const u32x4 *__restrict__ wk, u32 lane)
{
#pragma unroll
    for (int q = 0; q < 20; ++q)
        vs[q] = wk[q * 64 + lane];
}

// W_t + K_t of one block (16 big-endian words in w) into wk[t / 4][lane][t % 4]
__device__ __forceinline__ void sha1_schedule_wk(u32 (&w)[16], u32x4 *__restrict__ wk, u32 lane)
{
#pragma unroll
    for (int q = 0; q < 20; ++q) {
        u32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int t = 4 * q + j;
            u32 wt;
            if (t < 16) {
                wt = w[t];
            } else {
                wt = rotl(xor3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
                w[t & 15] = wt;
            }
            v[j] = wt + kShaK[t / 20];
        }
        wk[q * 64 + lane] = v;
    }
}

__global__ __launch_bounds__(128) void sec_sha1_split_kernel(const u8 *__restrict__ base0, const u8 *__restrict__ base1,
                                                              const sec::MsgDesc *__restrict__ msgs, u32 nmsgs,
                                                              u8 *__restrict__ digests)
{
    __shared__ u32x4 s_wk[2][20 * 64];  // two blocks' W + K, [t / 4][lane]
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u32 i = blockIdx.x * 64 + lane;
    const bool live = i < nmsgs;
    sec::MsgDesc m{};
    if (live)
        m = msgs[i];
    const u8 *p = (m.base ? base1 : base0) + m.off;
    const uint64_t nfast = live ? min(m.len / 64, m.avail / 64) : 0;  // blocks wholly inside the real bytes
    // the workgroup walks the longest message's blocks (shorter ones idle, masked)
    uint64_t nmax = nfast;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
        nmax = max(nmax, (uint64_t)__shfl_xor((unsigned long long)nmax, o, 64));
    u32 h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    // Two LDS buffers, one barrier per block: before barrier j wave 1 has written block j into
    // buffer j & 1, and wave 0 has finished block j - 1 (buffer (j - 1) & 1, which wave 1 fills
    // next).  (Three buffers with block j + 1 read into registers during block j measured
    // 1.22-1.25x over the one-lane kernel against 1.23-1.26x for this form.)
    if (wave == 1) {  // the schedule, one block ahead of wave 0; loads two blocks ahead of that
        u32x4 nx[2][4];
#pragma unroll
        for (int d = 0; d < 2; ++d)
            if ((uint64_t)d < nfast) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    nx[d][q] = *reinterpret_cast<const u32x4_u *>(p + d * 64 + 16 * q);
            }
        for (uint64_t b0 = 0; b0 < nmax; b0 += 2) {
#pragma unroll
            for (int d = 0; d < 2; ++d) {
                const uint64_t blk = b0 + d;
                if (blk >= nmax)
                    break;
                if (blk < nfast) {
                    u32 w[16];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        w[4 * q + 0] = __builtin_bswap32(nx[d][q].x);
                        w[4 * q + 1] = __builtin_bswap32(nx[d][q].y);
                        w[4 * q + 2] = __builtin_bswap32(nx[d][q].z);
                        w[4 * q + 3] = __builtin_bswap32(nx[d][q].w);
                    }
                    if (blk + 2 < nfast) {
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            nx[d][q] = *reinterpret_cast<const u32x4_u *>(p + (blk + 2) * 64 + 16 * q);
                    }
                    sha1_schedule_wk(w, s_wk[d], lane);
                }
                __syncthreads();  // barrier blk
            }
        }
        __syncthreads();  // barrier nmax, wave 0's last (both waves take nmax + 1 barriers)
        return;
    }
    __syncthreads();  // barrier 0: block 0 is in buffer 0
    for (uint64_t blk = 0; blk < nmax; ++blk) {
        if (blk < nfast) {
            u32x4 v[20];
            sha1_fetch_wk(v, s_wk[blk & 1], lane);
            __builtin_amdgcn_sched_barrier(0);  // all 20 reads out before the first round
            sha1_rounds_wk(h, v);
        }
        __syncthreads();  // barrier blk + 1: block blk + 1 is in its buffer, buffer blk & 1 free
    }
    if (!live)
        return;
    u32 w[16];
    const uint64_t nfull = m.len / 64;
    for (uint64_t blk = nfast; blk < nfull; ++blk) {
        const uint64_t o = blk * 64;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            u32 x = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b)
                x = (x << 8) | msg_byte(p, o + 4 * q + b, m.avail);
            w[q] = x;
        }
        sha1_compress(h, w);
    }
    const uint64_t o = nfull * 64;
    const u32 rem = (u32)(m.len - o);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        u32 x = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const u32 pos = 4 * q + b;
            const u32 byte = pos < rem ? msg_byte(p, o + pos, m.avail) : (pos == rem ? 0x80u : 0u);
            x = (x << 8) | byte;
        }
        w[q] = x;
    }
    const uint64_t bits = m.len * 8;
    if (rem >= 56) {
        sha1_compress(h, w);
#pragma unroll
        for (int q = 0; q < 16; ++q)
            w[q] = 0;
    }
    w[14] = (u32)(bits >> 32);
    w[15] = (u32)bits;
    sha1_compress(h, w);
    u32 *out = reinterpret_cast<u32 *>(digests + (uint64_t)i * 20);
#pragma unroll
    for (int q = 0; q < 5; ++q)
        out[q] = __builtin_bswap32(h[q]);
}

// Timing events for the next launch (sec_launch_events): the kernel's own dispatch records
// them (hipExtLaunchKernelGGL), so timing adds no marker packets between kernels.  Two event
// records per launch around back-to-back kernels cost the bench 3-5 % of its rate.
// The start event goes to the first launch after sec_launch_events, the stop event to every
// launch until the next call (the last record of an event is the one timed).
thread_local hipEvent_t t_start = nullptr, t_stop = nullptr;
thread_local int t_launched = 0;

template <class K, class... A>
hipError_t launch_shm(K kernel, dim3 grid, dim3 block, u32 shm, hipStream_t s, A... args)
{
    hipEvent_t a = t_start;
    t_start = nullptr;
    ++t_launched;
    hipExtLaunchKernelGGL(kernel, grid, block, shm, s, a, t_stop, 0, args...);
    return hipGetLastError();
}
template <class K, class... A>
hipError_t launch(K kernel, dim3 grid, dim3 block, hipStream_t s, A... args)
{
    return launch_shm(kernel, grid, block, 0, s, args...);
}

template <int R, int U, bool W>
hipError_t launch_enc(const u8 *in, u8 *par, const sec::EncDesc *descs, const sec::Tile *tiles, u32 ntiles,
                      const u32 *tabs, u32 lanes, hipStream_t s)
{
    return launch_shm(sec_encode_kernel<R, U, W>, dim3(ntiles), dim3(lanes),
                      lds_tab_bytes<batch_blocks<U, W, false>(), R, false>(lanes), s, in, par, descs, tiles, tabs);
}

template <int R, int U, bool W, int KBX>
hipError_t launch_dec(const u8 *blocks, u8 *out, const sec::DecDesc *descs, const sec::Tile *tiles, u32 ntiles,
                      const u32 *tabs, sec::DecSlots sl, u32 lanes, hipStream_t s)
{
    constexpr int KB = KBX > 0 ? KBX : batch_blocks<U, W, true>();
    return launch_shm(sec_decode_kernel<R, U, W, KBX>, dim3(ntiles), dim3(lanes),
                      lds_tab_bytes<KB, R, true>(lanes), s, blocks, out, descs, tiles, tabs, sl);
}

template <int U, bool W>
hipError_t dispatch_enc(int rows, const u8 *in, u8 *par, const sec::EncDesc *d, const sec::Tile *t, u32 nt,
                        const u32 *tabs, u32 lanes, hipStream_t s)
{
    switch (rows) {
    case 1: return launch_enc<1, U, W>(in, par, d, t, nt, tabs, lanes, s);
    case 2: return launch_enc<2, U, W>(in, par, d, t, nt, tabs, lanes, s);
    case 3: return launch_enc<3, U, W>(in, par, d, t, nt, tabs, lanes, s);
    case 4: return launch_enc<4, U, W>(in, par, d, t, nt, tabs, lanes, s);
    case 5: return launch_enc<5, U, W>(in, par, d, t, nt, tabs, lanes, s);
    case 6: return launch_enc<6, U, W>(in, par, d, t, nt, tabs, lanes, s);
    case 7: return launch_enc<7, U, W>(in, par, d, t, nt, tabs, lanes, s);
    case 8: return launch_enc<8, U, W>(in, par, d, t, nt, tabs, lanes, s);
    default: return hipErrorInvalidValue;
    }
}

template <int U, bool W, int KBX = 0>
hipError_t dispatch_dec(int rows, const u8 *b, u8 *o, const sec::DecDesc *d, const sec::Tile *t, u32 nt,
                        const u32 *tabs, sec::DecSlots sl, u32 lanes, hipStream_t s)
{
    switch (rows) {
    case 0: return launch_dec<0, U, W, KBX>(b, o, d, t, nt, tabs, sl, lanes, s);
    case 1: return launch_dec<1, U, W, KBX>(b, o, d, t, nt, tabs, sl, lanes, s);
    case 2: return launch_dec<2, U, W, KBX>(b, o, d, t, nt, tabs, sl, lanes, s);
    case 3: return launch_dec<3, U, W, KBX>(b, o, d, t, nt, tabs, sl, lanes, s);
    case 4: return launch_dec<4, U, W, KBX>(b, o, d, t, nt, tabs, sl, lanes, s);
    case 5: return launch_dec<5, U, W, KBX>(b, o, d, t, nt, tabs, sl, lanes, s);
    case 6: return launch_dec<6, U, W, KBX>(b, o, d, t, nt, tabs, sl, lanes, s);
    case 7: return launch_dec<7, U, W, KBX>(b, o, d, t, nt, tabs, sl, lanes, s);
    case 8: return launch_dec<8, U, W, KBX>(b, o, d, t, nt, tabs, sl, lanes, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

void sec_next_launch_events(void **start, void **stop)
{
    *start = t_start;
    t_start = nullptr;
    *stop = t_stop;
    ++t_launched;
}

int sec_launch_events(void *start, void *stop)
{
    const int n = t_launched;
    t_start = (hipEvent_t)start;
    t_stop = (hipEvent_t)stop;
    t_launched = 0;
    return n;
}

int sec_launch_expand(const uint8_t *coef, uint32_t ncoef, uint32_t *tabs, void *stream)
{
    if (ncoef == 0)
        return hipSuccess;
    return launch(sec_expand_tables, dim3((ncoef + 255) / 256), dim3(256), (hipStream_t)stream, coef, ncoef, tabs);
}

int sec_launch_encode(int rows, int U, int wide, int lanes, const uint8_t *in, uint8_t *par,
                      const sec::EncDesc *descs, const sec::Tile *tiles, uint32_t ntiles, const uint32_t *tabs,
                      void *stream)
{
    if (ntiles == 0)
        return hipSuccess;
    if (lanes < 64 || lanes % 64 || lanes > sec::max_lanes(rows, U) || (wide && U != 1))
        return hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
    if (wide)
        return dispatch_enc<1, true>(rows, in, par, descs, tiles, ntiles, tabs, (u32)lanes, s);
    if (U != 1)  // U > 1 tiles measured slower (profiles/r01_sweep_u.jsonl) and are not built
        return hipErrorInvalidValue;
    return dispatch_enc<1, false>(rows, in, par, descs, tiles, ntiles, tabs, (u32)lanes, s);
}

int sec_launch_encode_tail(const uint8_t *in, uint8_t *par, const sec::EncDesc *descs, const sec::TailItem *items,
                           uint32_t nitems, const uint32_t *tabs, void *stream)
{
    if (nitems == 0)
        return hipSuccess;
    return launch(sec_encode_tail, dim3((nitems + 255) / 256), dim3(256), (hipStream_t)stream, in, par, descs, items,
                  nitems, tabs);
}

int sec_launch_decode(int rows, int U, int wide, int lanes, const uint8_t *blocks, uint8_t *out,
                      const sec::DecDesc *descs, const sec::Tile *tiles, uint32_t ntiles, const uint32_t *tabs,
                      sec::DecSlots sl, void *stream, int kb)
{
    if (ntiles == 0)
        return hipSuccess;
    if (lanes < 64 || lanes % 64 || lanes > sec::max_lanes(rows, U) || (wide && U != 1))
        return hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
    const u32 L = (u32)lanes;
    if (kb) {  // small load batches: U = 1 tiles of chunks with k <= kb only
        if (U != 1 || wide)
            return hipErrorInvalidValue;
        if (kb == 4)
            return dispatch_dec<1, false, 4>(rows, blocks, out, descs, tiles, ntiles, tabs, sl, L, s);
        return hipErrorInvalidValue;
    }
    if (wide)
        return dispatch_dec<1, true>(rows, blocks, out, descs, tiles, ntiles, tabs, sl, L, s);
    if (U != 1)
        return hipErrorInvalidValue;
    return dispatch_dec<1, false>(rows, blocks, out, descs, tiles, ntiles, tabs, sl, L, s);
}

int sec_launch_sha1(const uint8_t *base0, const uint8_t *base1, const sec::MsgDesc *msgs, uint32_t nmsgs,
                    uint8_t *digests, void *stream, int split)
{
    if (nmsgs == 0)
        return hipSuccess;
    if (split)
        return launch(sec_sha1_split_kernel, dim3((nmsgs + 63) / 64), dim3(128), (hipStream_t)stream, base0, base1,
                      msgs, nmsgs, digests);
    if (SEC_SHA1_PF)
        return launch(sec_sha1_kernel<true>, dim3((nmsgs + 63) / 64), dim3(64), (hipStream_t)stream, base0, base1, msgs,
                      nmsgs, digests);
    return launch(sec_sha1_kernel<false>, dim3((nmsgs + 63) / 64), dim3(64), (hipStream_t)stream, base0, base1, msgs,
                  nmsgs, digests);
}

int sec_launch_decode_tail(const uint8_t *blocks, uint8_t *out, const sec::DecDesc *descs,
                           const sec::TailItem *items, uint32_t nitems, const uint32_t *tabs, sec::DecSlots sl,
                           void *stream)
{
    if (nitems == 0)
        return hipSuccess;
    return launch(sec_decode_tail, dim3((nitems + 255) / 256), dim3(256), (hipStream_t)stream, blocks, out, descs,
                  items, nitems, tabs, sl);
}
