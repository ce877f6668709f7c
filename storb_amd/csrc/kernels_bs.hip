// kernels_bs.hip — bit-sliced encode with the zfec matrix fixed at compile time, for the
// shapes whose v_perm encode is VALU-bound: C4's RS(10,4) = zfec(10,14) and the policy's
// zfec(8,12), (16,24), (32,48), (64,96), plus C5's RS(8,3).
//
// Multiplication by a constant c is GF(2)-linear on a byte's 8 bits: bit i of c*x is the XOR
// of the bits s of x for which bit i of c*alpha^s is set (an 8-bit mask per (c, i), a
// compile-time constant here).  So a lane turns 32 bytes of a block into 8 bit planes (one
// dword per bit position, an 8x8 bit transpose of each byte column: 48 VALU for 8 dwords),
// and every parity row's output plane i is
//     acc[r][i] ^= lo[mask & 15] ^ hi[mask >> 4]        (one XOR3)
// where lo / hi are the XORs of the subsets of planes 0..3 / 4..7 (at most 11 + 11 VALU per
// block, only the subsets some row uses survive compilation).  The parity planes are
// transposed back (the transpose is its own inverse) and stored.  Per input dword:
//     6 (transpose) + <= 2.75 (subsets) + p (rows) + 6 p / k (transpose out)
// against 5 + 4.5 p .. 5 p for sec_encode_kernel's v_perm rows and 35 + 22 + p for
// sec_encode_xb_kernel: C4 15.8 instead of 25, zfec(16,24) 19.8 instead of ~45, (32,48) 27.8
// instead of 69.
//
// Layout.  A wave covers 2048 positions of a chunk: lane l owns the 16 bytes at s + 16 l and
// the 16 at s + 1024 + 16 l of every block (each load instruction is one coalesced 1 KiB
// run).  A workgroup of `lanes` lanes covers lanes / 64 consecutive wave spans.  In the
// chunk's last span a piece that would run past B is moved back to end at B (it recomputes
// and stores bytes a neighbour also stores, identical), so the kernel covers all of [0, B) of
// every chunk with B >= 16, the ragged end included: block k-1's bytes past `valid` (zfec's
// zero padding) read as zero.  Parity rows [R0, R0 + NR) per launch; (64,96)'s 32 rows take
// two launches of 16 (256 accumulator
// dwords would not fit a lane's registers).  Loads stream through a ring of D blocks in
// flight.  Results are zfec's fec_encode (restated in oracle/fec_oracle.c;
// /root/reference/storb/util/piece.py:129-130).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <utility>

#include "gf_const.hpp"
#include "kernels.hpp"

namespace {

using u8 = uint8_t;
using u32 = uint32_t;
using u64 = uint64_t;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(1)));

constexpr u32 kSpan = 2048;  // positions per wave

// mask of the input bits s that feed bit i of c * x
constexpr u32 plane_mask(u32 c, int i)
{
    u32 m = 0;
    for (int s = 0; s < 8; ++s)
        if ((gfc::gmul(c, 1u << s) >> i) & 1u)
            m |= 1u << s;
    return m;
}
static_assert(plane_mask(1, 3) == 8 && plane_mask(2, 0) == 0x80 && plane_mask(2, 1) == 0x01, "plane masks");

__device__ __forceinline__ u32 xor3(u32 a, u32 b, u32 c)
{
    u32 r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// (m & x) | (~m & y), as one v_bfi_b32 (opaque to the compiler: left to itself it folded the
// transpose's masks into the later XORs and issued 1.4x the instructions)
__device__ __forceinline__ u32 bfi(u32 m, u32 x, u32 y)
{
    u32 r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(m), "v"(x), "v"(y));
    return r;
}

// Swap the bits of a at (MK << S) with the bits of b at MK: one 2x2 block step of an 8x8 bit
// transpose applied to each byte column of rows a and b (4 VALU).
template <int S, u32 MK>
__device__ __forceinline__ void swap_bits(u32 &a, u32 &b)
{
    constexpr u32 HI = MK << S;
    const u32 na = bfi(HI, b << S, a);
    const u32 nb = bfi(MK, a >> S, b);
    a = na;
    b = nb;
}

// x[i] byte q bit b  <->  x[b] byte q bit i  (an involution)
__device__ __forceinline__ void transpose8(u32 (&x)[8])
{
    swap_bits<4, 0x0F0F0F0Fu>(x[0], x[4]);
    swap_bits<4, 0x0F0F0F0Fu>(x[1], x[5]);
    swap_bits<4, 0x0F0F0F0Fu>(x[2], x[6]);
    swap_bits<4, 0x0F0F0F0Fu>(x[3], x[7]);
    swap_bits<2, 0x33333333u>(x[0], x[2]);
    swap_bits<2, 0x33333333u>(x[1], x[3]);
    swap_bits<2, 0x33333333u>(x[4], x[6]);
    swap_bits<2, 0x33333333u>(x[5], x[7]);
    swap_bits<1, 0x55555555u>(x[0], x[1]);
    swap_bits<1, 0x55555555u>(x[2], x[3]);
    swap_bits<1, 0x55555555u>(x[4], x[5]);
    swap_bits<1, 0x55555555u>(x[6], x[7]);
}

// Block loads: nontemporal (streaming) in the one-group kernels, where every byte is read
// once; cached in the interleaved two-group kernel, whose second group reads the blocks again
// from L2 (measured: (64,96) +5-8 % cached, (16,24) -5 %, (32,48) even; r02_bs_ab.jsonl run 4).
// SEC_BS_NT_LOAD (build knob, A/B): 0 = cached loads everywhere.
#ifndef SEC_BS_NT_LOAD
#define SEC_BS_NT_LOAD 1
#endif
template <bool NT>
__device__ __forceinline__ u32x4 ld16(const u8 *p)
{
    if constexpr (NT && SEC_BS_NT_LOAD)
        return __builtin_nontemporal_load(reinterpret_cast<const u32x4_u *>(p));
    else
        return *reinterpret_cast<const u32x4_u *>(p);
}

// 16 bytes at base + off of which the first `avail - off` exist; the rest read as zero
template <bool NT>
__device__ __forceinline__ u32x4 ld16_avail(const u8 *base, u32 off, u32 avail)
{
    if (off + 16 <= avail)
        return ld16<NT>(base + off);
    u32 w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < 16; ++b)
        if (off + b < avail)
            w[b >> 2] |= (u32)base[off + b] << (8 * (b & 3));
    return u32x4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ void st16(u8 *p, u32 a, u32 b, u32 c, u32 d)
{
    __builtin_nontemporal_store(u32x4{a, b, c, d}, reinterpret_cast<u32x4_u *>(p));
}

// acc (= or ^=) the output plane whose input mask is MSK
template <u32 MSK, bool FIRST>
__device__ __forceinline__ void upd(u32 &acc, const u32 (&lo)[16], const u32 (&hi)[16])
{
    constexpr u32 l = MSK & 15, h = MSK >> 4;
    if constexpr (FIRST) {
        if constexpr (l && h)
            acc = lo[l] ^ hi[h];
        else if constexpr (l)
            acc = lo[l];
        else if constexpr (h)
            acc = hi[h];
        else
            acc = 0;
    } else {
        if constexpr (l && h)
            acc = xor3(acc, lo[l], hi[h]);
        else if constexpr (l)
            acc ^= lo[l];
        else if constexpr (h)
            acc ^= hi[h];
    }
}

// XORs of every subset of v[0..3] (s[S] for S = 1..15; those no row reads are dead code)
__device__ __forceinline__ void subsets(u32 v0, u32 v1, u32 v2, u32 v3, u32 (&s)[16])
{
    s[0] = 0;
    s[1] = v0;
    s[2] = v1;
    s[4] = v2;
    s[8] = v3;
    s[3] = v0 ^ v1;
    s[5] = v0 ^ v2;
    s[6] = v1 ^ v2;
    s[9] = v0 ^ v3;
    s[10] = v1 ^ v3;
    s[12] = v2 ^ v3;
    s[7] = s[3] ^ v2;
    s[11] = s[3] ^ v3;
    s[13] = s[5] ^ v3;
    s[14] = s[6] ^ v3;
    s[15] = s[7] ^ v3;
}

template <int K, int M, int R0, int J, bool FIRST, int... Q>
__device__ __forceinline__ void block_rows(std::integer_sequence<int, Q...>, u32 (&acc)[sizeof...(Q)],
                                           const u32 (&lo)[16], const u32 (&hi)[16])
{
    (upd<plane_mask(gfc::Matrix<K, M>::v.c[R0 + Q / 8][J], Q % 8), FIRST>(acc[Q], lo, hi), ...);
}

// the lane's two 16-byte pieces of a block: at pa and pb
template <bool NT>
__device__ __forceinline__ void load_block(u32 (&x)[8], const u8 *blk, u32 pa, u32 pb, u32 avail, bool last)
{
    u32x4 a, b;
    if (!last) {
        a = ld16<NT>(blk + pa);
        b = ld16<NT>(blk + pb);
    } else {
        a = ld16_avail<NT>(blk, pa, avail);
        b = ld16_avail<NT>(blk, pb, avail);
    }
    x[0] = a.x;
    x[1] = a.y;
    x[2] = a.z;
    x[3] = a.w;
    x[4] = b.x;
    x[5] = b.y;
    x[6] = b.z;
    x[7] = b.w;
}

template <int K, int M, int R0, int NR, int D, bool NT, int J>
__device__ __forceinline__ void one_block(u32 (&acc)[NR * 8], u32 (&ring)[D][8], const u8 *src, u64 B, u32 pa,
                                          u32 pb, u32 valid)
{
    u32 x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        x[i] = ring[J % D][i];
    if constexpr (J + D < K)
        load_block<NT>(ring[J % D], src + (u64)(J + D) * B, pa, pb, valid, J + D == K - 1);
    transpose8(x);
    u32 lo[16], hi[16];
    subsets(x[0], x[1], x[2], x[3], lo);
    subsets(x[4], x[5], x[6], x[7], hi);
    block_rows<K, M, R0, J, J == 0>(std::make_integer_sequence<int, NR * 8>{}, acc, lo, hi);
}

template <int K, int M, int R0, int NR, int D, bool NT, int... Js>
__device__ __forceinline__ void all_blocks(std::integer_sequence<int, Js...>, u32 (&acc)[NR * 8], u32 (&ring)[D][8],
                                           const u8 *src, u64 B, u32 pa, u32 pb, u32 valid)
{
    (one_block<K, M, R0, NR, D, NT, Js>(acc, ring, src, B, pa, pb, valid), ...);
}

// SEC_BS_WAVES (build knob, A/B): minimum waves per SIMD (amdgpu_waves_per_eu, a VGPR cap)
#if defined(SEC_BS_WAVES) && SEC_BS_WAVES > 0
#define SEC_BS_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(SEC_BS_WAVES)))
#else
#define SEC_BS_WAVES_ATTR
#endif

// One wave's span of one tile: rows [R0, R0 + NR) of the chunk's parity over the lane's pieces.
template <int K, int M, int R0, int NR, int D, bool NT>
__device__ __forceinline__ void bs_span(const u8 *__restrict__ in, u8 *__restrict__ par, const sec::EncDesc &d, u32 s)
{
    static_assert(D >= 1 && D <= K, "ring depth");
    const u32 B = d.B;
    // a piece past the chunk's end moves back to end at B: it recomputes (and stores) bytes
    // its neighbour also stores, identical, instead of taking a byte path
    const u32 lane = (threadIdx.x & 63) * 16;
    const u32 pa = min(s + lane, B - 16), pb = min(s + 1024 + lane, B - 16);
    const u8 *src = in + d.in_off;

    u32 ring[D][8];
#pragma unroll
    for (int j = 0; j < D; ++j)
        load_block<NT>(ring[j], src + (u64)j * B, pa, pb, d.valid, j == K - 1);
    u32 acc[NR * 8];
    all_blocks<K, M, R0, NR, D, NT>(std::make_integer_sequence<int, K>{}, acc, ring, src, B, pa, pb, d.valid);

    u8 *dst = par + d.par_off;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        u32 y[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            y[i] = acc[r * 8 + i];
        transpose8(y);
        u8 *o = dst + (u64)(R0 + r) * d.par_stride;
        st16(o + pa, y[0], y[1], y[2], y[3]);
        st16(o + pb, y[4], y[5], y[6], y[7]);
    }
}

// Rows [R0, R0 + NR) of every tile.
template <int K, int M, int R0, int NR, int D>
__global__ __launch_bounds__(256) SEC_BS_WAVES_ATTR void sec_encode_bs_kernel(const u8 *__restrict__ in, u8 *__restrict__ par,
                                                            const sec::EncDesc *__restrict__ descs,
                                                            const sec::Tile *__restrict__ tiles)
{
    const sec::Tile tl = tiles[blockIdx.x];
    const sec::EncDesc d = descs[tl.chunk];
    const u32 s = tl.t0 + (threadIdx.x >> 6) * kSpan;
    if (s >= d.B)
        return;
    bs_span<K, M, R0, NR, D, true>(in, par, d, s);
}

// Two row groups in one launch, the tile's r0 picking one: the plan puts a run of 8 tiles of
// group 0 and the same 8 positions of group 1 next in the launch, so each pair lands on one
// XCD (workgroup b runs on XCD b % 8) at about the same time and the second reads the blocks
// from that XCD's L2 instead of HBM.
template <int K, int M, int NR, int D>
__global__ __launch_bounds__(256) SEC_BS_WAVES_ATTR void sec_encode_bs2_kernel(const u8 *__restrict__ in, u8 *__restrict__ par,
                                                             const sec::EncDesc *__restrict__ descs,
                                                             const sec::Tile *__restrict__ tiles)
{
    const sec::Tile tl = tiles[blockIdx.x];
    const sec::EncDesc d = descs[tl.chunk];
    const u32 s = tl.t0 + (threadIdx.x >> 6) * kSpan;
    if (s >= d.B)
        return;
    if (tl.r0 == 0)
        bs_span<K, M, 0, NR, D, false>(in, par, d, s);
    else
        bs_span<K, M, NR, NR, D, false>(in, par, d, s);
}

// ---- decode, phase 1: syndromes of the present parity rows (wide decodes) -------------------
// A decode that lost e data blocks and holds e parity rows S instead: for a parity row r in S,
//     s_r = p_r ^ XOR_{present j} c[r][j] * d_j  =  XOR_{lost j} c[r][j] * d_j,
// so the lost blocks are A^-1 s with A = c[S][lost] (e x e).  Phase 1 is this kernel: the
// bit-sliced encode of the PRESENT data blocks (the matrix c at compile time, a block the chunk
// lacks skipped by a wave-uniform branch), XORed with the present parity rows and stored as e
// syndrome rows.  While it has each present data block in registers it also stores it to its
// output row (the copy half of a reassembly).  Phase 2 applies the run-time e x e inverse with
// sec_decode_kernel (api.cpp).  Per input dword this costs the bit-sliced rows (6 + 2.75 + NR +
// 6 NR / 64 VALU) instead of ceil(e / 8) v_perm row groups over all k blocks (5 + 36 VALU each),
// and reads the k blocks once instead of once per 8-row group.
//
// Items 0..K-1 of a chunk are its data blocks, K..K+NR-1 the parity rows R0.. of this tile's
// group; one ring of D items in flight serves both.  Results are zfec's fec_decode (restated in
// oracle/fec_oracle.c; /root/reference/storb/util/piece.py:196-197).

// The lane's two 16-byte pieces of an item.  Only data block K-1 may be short (avail < B: zfec's
// padded last block read in place; the plan sends chunks whose other slots are shorter to the
// direct decode), so only that item carries the byte path.
template <bool SHORT>
__device__ __forceinline__ void load_item(u32 (&x)[8], const u8 *blk, u32 pa, u32 pb, u32 avail)
{
    u32x4 a, b;
    if (!SHORT || pb + 16 <= avail) {  // pb >= pa: the whole lane is inside
        a = ld16<true>(blk + pa);
        b = ld16<true>(blk + pb);
    } else {
        a = ld16_avail<true>(blk, pa, avail);
        b = ld16_avail<true>(blk, pb, avail);
    }
    x[0] = a.x;
    x[1] = a.y;
    x[2] = a.z;
    x[3] = a.w;
    x[4] = b.x;
    x[5] = b.y;
    x[6] = b.z;
    x[7] = b.w;
}

// 16 bytes to o + off, only those below `lim` (the rare short end: a byte loop, not unrolled,
// so it costs neither code nor registers in the common path)
__device__ __forceinline__ void st16_clamped(u8 *o, u32 off, u32 lim, u32 a, u32 b, u32 c, u32 d)
{
    if (off + 16 <= lim) {
        st16(o + off, a, b, c, d);
        return;
    }
#pragma clang loop vectorize(disable) unroll(disable)
    for (u32 i = 0; off + i < lim; ++i) {
        const u32 w = i < 4 ? a : i < 8 ? b : i < 12 ? c : d;
        o[off + i] = (u8)(w >> (8 * (i & 3)));
    }
}

struct SynCtx {
    const u8 *blocks;
    const uint64_t *off;
    const uint32_t *avail;
    u32 slot0, pa, pb;
    uint64_t dmask, pmask;
};

template <int K, int NR, int R0>
__device__ __forceinline__ bool item_present(const SynCtx &c, int J)
{
    return J < K ? ((c.dmask >> J) & 1) : ((c.pmask >> (R0 + J - K)) & 1);
}

template <int K, int NR, int R0, int J>
__device__ __forceinline__ void load_syn_item(u32 (&x)[8], const SynCtx &c)
{
    constexpr u32 slot = J < K ? (u32)J : (u32)(K + R0 + J - K);
    load_item<J == K - 1>(x, c.blocks + c.off[c.slot0 + slot], c.pa, c.pb, J == K - 1 ? c.avail[c.slot0 + slot] : 0u);
}

template <int K, int NR, int R0, int... Js>
__device__ __forceinline__ void load_syn_first(std::integer_sequence<int, Js...>, u32 (&ring)[sizeof...(Js)][8],
                                               const SynCtx &c)
{
    ((item_present<K, NR, R0>(c, Js) ? load_syn_item<K, NR, R0, Js>(ring[Js], c) : void()), ...);
}

template <int K, int M, int R0, int NR, int D, int J>
__device__ __forceinline__ void syn_item(u32 (&acc)[NR * 8], u32 (&ring)[D][8], const SynCtx &c, u8 *orow0, u32 B,
                                         u32 last, bool copies, u8 *syn, u32 &q)
{
    constexpr int NI = K + NR;
    const bool here = item_present<K, NR, R0>(c, J);
    u32 x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        x[i] = ring[J % D][i];
    if constexpr (J + D < NI)
        if (item_present<K, NR, R0>(c, J + D))
            load_syn_item<K, NR, R0, J + D>(ring[J % D], c);
    if (!here)
        return;
    if constexpr (J < K) {
        if (copies) {  // the present primary's bytes to its output row (row K-1 clamps to `last`)
            u8 *o = orow0 + (u64)J * B;
            if constexpr (J == K - 1) {
                st16_clamped(o, c.pa, last, x[0], x[1], x[2], x[3]);
                st16_clamped(o, c.pb, last, x[4], x[5], x[6], x[7]);
            } else {
                st16(o + c.pa, x[0], x[1], x[2], x[3]);
                st16(o + c.pb, x[4], x[5], x[6], x[7]);
            }
        }
        transpose8(x);
        u32 lo[16], hi[16];
        subsets(x[0], x[1], x[2], x[3], lo);
        subsets(x[4], x[5], x[6], x[7], hi);
        block_rows<K, M, R0, J, false>(std::make_integer_sequence<int, NR * 8>{}, acc, lo, hi);
    } else {  // parity row R0 + r: syndrome = its bytes ^ the present blocks' contribution
        constexpr int r = J - K;
        u32 y[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            y[i] = acc[r * 8 + i];
        transpose8(y);
        u8 *o = syn + (u64)q * B;
        st16(o + c.pa, y[0] ^ x[0], y[1] ^ x[1], y[2] ^ x[2], y[3] ^ x[3]);
        st16(o + c.pb, y[4] ^ x[4], y[5] ^ x[5], y[6] ^ x[6], y[7] ^ x[7]);
        ++q;
    }
}

template <int K, int M, int R0, int NR, int D, int... Js>
__device__ __forceinline__ void syn_items(std::integer_sequence<int, Js...>, u32 (&acc)[NR * 8], u32 (&ring)[D][8],
                                          const SynCtx &c, u8 *orow0, u32 B, u32 last, bool copies, u8 *syn, u32 &q)
{
    (syn_item<K, M, R0, NR, D, Js>(acc, ring, c, orow0, B, last, copies, syn, q), ...);
}

template <int K, int M, int R0, int NR, int D>
__device__ __forceinline__ void syn_span(const u8 *__restrict__ blocks, u8 *__restrict__ out, u8 *__restrict__ syn,
                                         const sec::SynDesc &d, const sec::SynSlots &sl, u32 s, bool copies)
{
    const u32 B = d.B;
    const u32 lane = (threadIdx.x & 63) * 16;
    SynCtx c{blocks, sl.off, sl.avail, d.slot0, min(s + lane, B - 16), min(s + 1024 + lane, B - 16), d.dmask, d.pmask};
    u32 ring[D][8];
    load_syn_first<K, NR, R0>(std::make_integer_sequence<int, D>{}, ring, c);
    u32 acc[NR * 8];
#pragma unroll
    for (int i = 0; i < NR * 8; ++i)
        acc[i] = 0;
    // syndrome row of this group's first present parity row: the present rows below R0
    u32 q = (u32)__builtin_popcountll(d.pmask & ((1ull << R0) - 1ull));
    syn_items<K, M, R0, NR, D>(std::make_integer_sequence<int, K + NR>{}, acc, ring, c, out + d.out_off, B, d.last,
                               copies, syn + d.syn_off, q);
}

// The syndromes go to `syn`; sec_decode_kernel then solves for the lost blocks (api.cpp).
template <int K, int M, int NR, int D>
__global__ __launch_bounds__(256) void sec_syndrome_bs_kernel(const u8 *__restrict__ blocks, u8 *__restrict__ out,
                                                              u8 *__restrict__ syn,
                                                              const sec::SynDesc *__restrict__ descs,
                                                              const sec::Tile *__restrict__ tiles,
                                                              const sec::SynSlots sl)
{
    const sec::Tile tl = tiles[blockIdx.x];
    const sec::SynDesc d = descs[tl.chunk];
    const u32 s = tl.t0 + (threadIdx.x >> 6) * kSpan;
    if (s >= d.B)
        return;
    const bool copies = tl.ntail & 1;  // the chunk's first touched row group copies the primaries
    if constexpr (M - K <= NR) {
        syn_span<K, M, 0, NR, D>(blocks, out, syn, d, sl, s, copies);
    } else {
        static_assert(M - K == 2 * NR, "two row groups");
        if (tl.r0 == 0)
            syn_span<K, M, 0, NR, D>(blocks, out, syn, d, sl, s, copies);
        else
            syn_span<K, M, NR, NR, D>(blocks, out, syn, d, sl, s, copies);
    }
}

template <int K, int M, int R0, int NR, int D>
hipError_t launch_bs(int lanes, const u8 *in, u8 *par, const sec::EncDesc *d, const sec::Tile *t, u32 nt,
                     hipStream_t s)
{
    void *a = nullptr, *b = nullptr;
    sec_next_launch_events(&a, &b);  // kernel timing (sec_ctx_set_timing) rides on the dispatch
    if constexpr (R0 < 0)
        hipExtLaunchKernelGGL((sec_encode_bs2_kernel<K, M, NR, D>), dim3(nt), dim3(lanes), 0, s, (hipEvent_t)a,
                              (hipEvent_t)b, 0, in, par, d, t);
    else
        hipExtLaunchKernelGGL((sec_encode_bs_kernel<K, M, R0, NR, D>), dim3(nt), dim3(lanes), 0, s, (hipEvent_t)a,
                              (hipEvent_t)b, 0, in, par, d, t);
    return hipGetLastError();
}

// Shapes: (k, m, rows per launch).  Ring depths from the register budget (8 NR accumulators
// + 8 D ring dwords per lane) and A/Bs: zfec(16,24) keeps 10 of its 16 blocks in flight
// (182 VGPRs; +2-8 % over 4 on 1 and 16 MiB chunks), C4 5 (10: -2 %), the 16-row groups 2;
// SEC_BS_RING (build knob, A/B) sets one depth for every shape.
#ifdef SEC_BS_RING
#define RING_K(k, d) (SEC_BS_RING < (k) ? SEC_BS_RING : (k))
#else
#define RING_K(k, d) (d)
#endif
struct BsShape {
    int k, m, nr;
};
// 6: (32,48) in two groups of 8 rows (A/B against shape 3's one pass of 16)
constexpr BsShape kShapes[] = {{10, 14, 4}, {8, 12, 4}, {16, 24, 8}, {32, 48, 16}, {64, 96, 16}, {8, 11, 3}, {32, 48, 8}};
constexpr int kNShapes = (int)(sizeof(kShapes) / sizeof(kShapes[0]));

}  // namespace

int sec_bs_shape(int k, int m, int rows)
{
    for (int i = 0; i < kNShapes; ++i)
        if (kShapes[i].k == k && kShapes[i].m == m && (rows == 0 || kShapes[i].nr == rows))
            return i;
    return -1;
}

int sec_bs_groups(int shape) { return (kShapes[shape].m - kShapes[shape].k + kShapes[shape].nr - 1) / kShapes[shape].nr; }

int sec_bs_rows(int shape) { return kShapes[shape].nr; }

uint32_t sec_bs_span() { return kSpan; }

int sec_launch_encode_bs(int shape, int group, int lanes, const uint8_t *in, uint8_t *par, const sec::EncDesc *descs,
                         const sec::Tile *t, uint32_t ntiles, void *stream)
{
    if (ntiles == 0)
        return hipSuccess;
    if (lanes < 64 || lanes > 256 || lanes % 64 || shape < 0 || shape >= kNShapes)
        return hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
    // group -1: both row groups in one launch (sec_encode_bs2_kernel), tiles carry r0
    switch (shape * 4 + group + 1) {
    case 1: return launch_bs<10, 14, 0, 4, RING_K(10, 5)>(lanes, in, par, descs, t, ntiles, s);
    case 5: return launch_bs<8, 12, 0, 4, RING_K(8, 4)>(lanes, in, par, descs, t, ntiles, s);
    case 9: return launch_bs<16, 24, 0, 8, RING_K(16, 10)>(lanes, in, par, descs, t, ntiles, s);
    case 13: return launch_bs<32, 48, 0, 16, RING_K(32, 2)>(lanes, in, par, descs, t, ntiles, s);
    case 16: return launch_bs<64, 96, -1, 16, RING_K(64, 2)>(lanes, in, par, descs, t, ntiles, s);
    case 17: return launch_bs<64, 96, 0, 16, RING_K(64, 2)>(lanes, in, par, descs, t, ntiles, s);
    case 18: return launch_bs<64, 96, 16, 16, RING_K(64, 2)>(lanes, in, par, descs, t, ntiles, s);
    case 21: return launch_bs<8, 11, 0, 3, RING_K(8, 4)>(lanes, in, par, descs, t, ntiles, s);
    case 24: return launch_bs<32, 48, -1, 8, RING_K(32, 4)>(lanes, in, par, descs, t, ntiles, s);
    case 25: return launch_bs<32, 48, 0, 8, RING_K(32, 4)>(lanes, in, par, descs, t, ntiles, s);
    case 26: return launch_bs<32, 48, 8, 8, RING_K(32, 4)>(lanes, in, par, descs, t, ntiles, s);
    default: return hipErrorInvalidValue;
    }
}

namespace {
template <int K, int M, int NR, int D>
hipError_t launch_syn(int lanes, const u8 *blocks, u8 *out, u8 *syn, const sec::SynDesc *d, const sec::Tile *t, u32 nt,
                      sec::SynSlots sl, hipStream_t s)
{
    void *a = nullptr, *b = nullptr;
    sec_next_launch_events(&a, &b);
    hipExtLaunchKernelGGL((sec_syndrome_bs_kernel<K, M, NR, D>), dim3(nt), dim3(lanes), 0, s, (hipEvent_t)a,
                          (hipEvent_t)b, 0, blocks, out, syn, d, t, sl);
    return hipGetLastError();
}
}  // namespace

int sec_syn_shape(int k, int m)
{
    const int sh = sec_bs_shape(k, m);
    return sh == 6 ? -1 : sh;  // (32,48) in 8-row groups is an encode A/B only
}

int sec_launch_syndrome_bs(int shape, int lanes, const uint8_t *blocks, uint8_t *out, uint8_t *syn,
                           const sec::SynDesc *descs, const sec::Tile *t, uint32_t ntiles, sec::SynSlots sl,
                           void *stream)
{
    if (ntiles == 0)
        return hipSuccess;
    if (lanes < 64 || lanes > 256 || lanes % 64)
        return hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
    switch (shape) {  // ring depths as the encode's (kernels' register budgets are alike)
    case 0: return launch_syn<10, 14, 4, RING_K(10, 5)>(lanes, blocks, out, syn, descs, t, ntiles, sl, s);
    case 1: return launch_syn<8, 12, 4, RING_K(8, 4)>(lanes, blocks, out, syn, descs, t, ntiles, sl, s);
    case 2: return launch_syn<16, 24, 8, RING_K(16, 10)>(lanes, blocks, out, syn, descs, t, ntiles, sl, s);
    case 3: return launch_syn<32, 48, 16, RING_K(32, 2)>(lanes, blocks, out, syn, descs, t, ntiles, sl, s);
    case 4: return launch_syn<64, 96, 16, RING_K(64, 2)>(lanes, blocks, out, syn, descs, t, ntiles, sl, s);
    case 5: return launch_syn<8, 11, 3, RING_K(8, 4)>(lanes, blocks, out, syn, descs, t, ntiles, sl, s);
    default: return hipErrorInvalidValue;
    }
}

