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
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "libstorbec is written for gfx950 (MI355X) only: 16-byte global_load_lds, v_bitop3, 64+ KiB LDS"
#endif
#include <hip/hip_runtime.h>

#include <type_traits>
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

// Block loads: nontemporal (streaming) in the one-group encode kernels, where every byte is read
// once; cached elsewhere (the zfec(64,96) encode and the decode phases, whose blocks a second
// wave or group reads again from L2; measured (64,96) +5-8 % cached, (16,24) -5 %, (32,48) even;
// r02_bs_ab.jsonl run 4).
template <bool NT>
__device__ __forceinline__ u32x4 ld16(const u8 *p)
{
    if constexpr (NT)
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

// ---- loads through an LDS ring filled by global_load_lds (k >= 32; see phase 1 below) --------
#ifndef SEC_FUSED_LDS_RING
#define SEC_FUSED_LDS_RING 8
#endif

template <int D, int W = 4>
struct LdsRing {
    u32x4 v[W][D][2][64];  // [wave of the workgroup][slot][half][lane]
};

template <int N>
__device__ __forceinline__ void wait_vm()
{
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

template <int K>
using Phase1Lds = std::conditional_t<(K >= 32), LdsRing<SEC_FUSED_LDS_RING>, char>;  // the LDS ring of k >= 32

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

    u32 acc[NR * 8];
    u32 ring[D][8];
#pragma unroll
    for (int j = 0; j < D; ++j)
        load_block<NT>(ring[j], src + (u64)j * B, pa, pb, d.valid, j == K - 1);
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
        // (pieces clamped to B - 16 repeat a neighbour's store; skipping them measured neutral on
        // C4, r03_c4_skip_dup_ab.jsonl)
        st16(o + pa, y[0], y[1], y[2], y[3]);
        st16(o + pb, y[4], y[5], y[6], y[7]);
    }
}

// Rows [R0, R0 + NR) of every tile.
template <int K, int M, int R0, int NR, int D>
__global__ __launch_bounds__(256) void sec_encode_bs_kernel(const u8 *__restrict__ in, u8 *__restrict__ par,
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

// ---- zfec(64,96) encode: both row groups of a span in one two-wave workgroup ----------------
// The interleaved kernel above runs each 16-row group as its own wave, so both waves of a span
// transpose all 64 blocks and form their plane subsets: 70 of each block's 198 VALU are done
// twice, and the kernel is VALU-bound (SQ_ACTIVE_INST_VALU 51 % of each wave's cycles at two
// waves per SIMD, i.e. the SIMD's VALU nearly saturated; profiles/r06_pmc_enc.json).  Here wave g
// (group g) loads, transposes and forms the subsets of the blocks j = 2i + g only, publishes the
// 30 subset XORs through LDS, and takes the other wave's for the blocks 2i + 1 - g: 163 VALU per
// block instead of 198, one barrier per pair of blocks, each block read from HBM once (no L2
// re-read).  LDS: two steps of both waves' 8 x 16 bytes per lane, 32 KiB per workgroup.
// Against the interleaved one-group-per-wave launch it replaced: 4.09 / 3.85 / 4.37 TB/s on
// 1 MiB / 256 MiB / 64 MiB ragged chunks against 3.81 / 3.73 / 3.78; publishing the 8 transposed
// planes instead (the taker forming the subsets) 3.27 / 3.09 / 3.32 (profiles/r06_enc_ab.jsonl;
// both archived: tools/archive/README.md).

struct PairXchg {
    u32x4 v[2][2][8][64];  // [step & 1][publishing wave][dword quad][lane]
};

__device__ __forceinline__ void barrier_lds()
{
    // own LDS stores done, then the workgroup barrier; no vmcnt wait (the loads in flight stay)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int K, int M, int G, int NR, int D, int I>
__device__ __forceinline__ void pair_step(u32 (&acc)[NR * 8], u32 (&ring)[D][8], PairXchg &xb, const u8 *src, u64 B,
                                          u32 pa, u32 pb, u32 valid)
{
    constexpr int J = 2 * I + G, O = 2 * I + 1 - G;  // own block, the other wave's block
    const u32 l = threadIdx.x & 63;
    u32 x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        x[i] = ring[I % D][i];
    if constexpr (I + D < K / 2)
        load_block<true>(ring[I % D], src + (u64)(2 * (I + D) + G) * B, pa, pb, valid, 2 * (I + D) + G == K - 1);
    transpose8(x);
    u32x4(&mine)[8][64] = xb.v[I & 1][G];
    u32x4(&theirs)[8][64] = xb.v[I & 1][1 - G];
    u32 lo[16], hi[16];
    subsets(x[0], x[1], x[2], x[3], lo);
    subsets(x[4], x[5], x[6], x[7], hi);
    mine[0][l] = u32x4{lo[1], lo[2], lo[3], lo[4]};
    mine[1][l] = u32x4{lo[5], lo[6], lo[7], lo[8]};
    mine[2][l] = u32x4{lo[9], lo[10], lo[11], lo[12]};
    mine[3][l] = u32x4{lo[13], lo[14], lo[15], hi[1]};
    mine[4][l] = u32x4{hi[2], hi[3], hi[4], hi[5]};
    mine[5][l] = u32x4{hi[6], hi[7], hi[8], hi[9]};
    mine[6][l] = u32x4{hi[10], hi[11], hi[12], hi[13]};
    mine[7][l] = u32x4{hi[14], hi[15], 0u, 0u};
    block_rows<K, M, G * NR, J, I == 0>(std::make_integer_sequence<int, NR * 8>{}, acc, lo, hi);
    barrier_lds();  // both waves' step-I subsets are in LDS (and both finished reading step I-1's)
    u32 lo2[16], hi2[16];
    const u32x4 t0 = theirs[0][l], t1 = theirs[1][l], t2 = theirs[2][l], t3 = theirs[3][l], t4 = theirs[4][l],
                t5 = theirs[5][l], t6 = theirs[6][l], t7 = theirs[7][l];
    lo2[0] = hi2[0] = 0;
    lo2[1] = t0.x, lo2[2] = t0.y, lo2[3] = t0.z, lo2[4] = t0.w;
    lo2[5] = t1.x, lo2[6] = t1.y, lo2[7] = t1.z, lo2[8] = t1.w;
    lo2[9] = t2.x, lo2[10] = t2.y, lo2[11] = t2.z, lo2[12] = t2.w;
    lo2[13] = t3.x, lo2[14] = t3.y, lo2[15] = t3.z, hi2[1] = t3.w;
    hi2[2] = t4.x, hi2[3] = t4.y, hi2[4] = t4.z, hi2[5] = t4.w;
    hi2[6] = t5.x, hi2[7] = t5.y, hi2[8] = t5.z, hi2[9] = t5.w;
    hi2[10] = t6.x, hi2[11] = t6.y, hi2[12] = t6.z, hi2[13] = t6.w;
    hi2[14] = t7.x, hi2[15] = t7.y;
    block_rows<K, M, G * NR, O, false>(std::make_integer_sequence<int, NR * 8>{}, acc, lo2, hi2);
}

template <int K, int M, int G, int NR, int D, int... Is>
__device__ __forceinline__ void pair_steps(std::integer_sequence<int, Is...>, u32 (&acc)[NR * 8], u32 (&ring)[D][8],
                                           PairXchg &xb, const u8 *src, u64 B, u32 pa, u32 pb, u32 valid)
{
    (pair_step<K, M, G, NR, D, Is>(acc, ring, xb, src, B, pa, pb, valid), ...);
}

template <int K, int M, int G, int NR, int D>
__device__ __forceinline__ void bs_pair_span(const u8 *__restrict__ in, u8 *__restrict__ par, const sec::EncDesc &d,
                                             u32 s, PairXchg &xb)
{
    static_assert(K % 2 == 0 && D >= 1 && D <= K / 2, "pair encode shape");
    const u32 B = d.B;
    const u32 lane = (threadIdx.x & 63) * 16;
    const u32 pa = min(s + lane, B - 16), pb = min(s + 1024 + lane, B - 16);
    const u8 *src = in + d.in_off;
    u32 ring[D][8];
#pragma unroll
    for (int j = 0; j < D; ++j)
        load_block<true>(ring[j], src + (u64)(2 * j + G) * B, pa, pb, d.valid, 2 * j + G == K - 1);
    u32 acc[NR * 8];
    pair_steps<K, M, G, NR, D>(std::make_integer_sequence<int, K / 2>{}, acc, ring, xb, src, B, pa, pb, d.valid);
    u8 *dst = par + d.par_off;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        u32 y[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            y[i] = acc[r * 8 + i];
        transpose8(y);
        u8 *o = dst + (u64)(G * NR + r) * d.par_stride;
        st16(o + pa, y[0], y[1], y[2], y[3]);
        st16(o + pb, y[4], y[5], y[6], y[7]);
    }
}

// One span per workgroup (tile t0), wave g = row group g.
template <int K, int M, int NR, int D>
__global__ __launch_bounds__(128) void sec_encode_bs_pair_kernel(const u8 *__restrict__ in, u8 *__restrict__ par,
                                                                 const sec::EncDesc *__restrict__ descs,
                                                                 const sec::Tile *__restrict__ tiles)
{
    static_assert(M - K == 2 * NR, "two row groups");
    const sec::Tile tl = tiles[blockIdx.x];
    const sec::EncDesc d = descs[tl.chunk];
    if (tl.t0 >= d.B)  // the whole workgroup: both waves leave before any barrier
        return;
    __shared__ PairXchg xb;
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) < 64)
        bs_pair_span<K, M, 0, NR, D>(in, par, d, tl.t0, xb);
    else
        bs_pair_span<K, M, 1, NR, D>(in, par, d, tl.t0, xb);
}

// ---- decode: syndromes of the present parity rows, then a Cauchy solve (wide decodes) --------
// A decode that lost e data blocks L and holds e parity rows S instead: for a parity row r in S,
//     s_r = p_r ^ XOR_{present j} c[r][j] * d_j  =  XOR_{l in L} c[r][l] * d_l,
// so the lost blocks are A^-1 s with A = c[S][L] (e x e).  zfec's parity rows are a Cauchy
// matrix up to diagonal scalings (c[r][j] = a_r b_j / (x_r + y_j) on its evaluation points), and
// so is A^-1:  A^-1[l][r] = z_l c[r][l] w_r  (gf_host.hpp cauchy_scales).  Both phases therefore
// apply compile-time matrices on bit planes, with run-time diagonal scalings in between:
//   phase 1 (sec_syndrome_bs_kernel): the bit-sliced encode of the PRESENT data blocks (a block
//     the chunk lacks skipped by a wave-uniform branch) XORed with the present parity rows,
//     scaled by w_r and stored as bit planes (no transpose back).  While it has each present data
//     block in registers it also stores it to its output row (the copy half of a reassembly);
//   phase 2 (sec_solve_bs_kernel): the transposed parity matrix c[S][l] over the scaled
//     syndromes for the lost rows l of one 16-row group, scaled by z_l and transposed back.
// Per input dword phase 1 costs 6 + 2.75 + NR (bit-sliced rows) and 15 per syndrome; phase 2
// 2.75 per syndrome and row group plus 1 per (syndrome, lost row) and 14 per lost row, against
// ceil(e / 8) v_perm row groups over all k blocks (5 + 36 VALU each) for the direct decode.
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
    const uint64_t *wmask;  // masks + wq0
    u32 slot0, pa, pb, ua, ub;  // clamped (block) and unclamped (syndrome) lane positions
    uint64_t dmask, pmask, stride;
};

// a ^ (b & m), m wave-uniform (an SGPR holding 0 or ~0)
__device__ __forceinline__ u32 xor_and(u32 a, u32 b, u32 m)
{
    u32 r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x78" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}

// bit i of w as 0 / ~0
__device__ __forceinline__ u32 bitmask(u32 w, int i) { return (u32)((int32_t)(w << (31 - i)) >> 31); }

// y <- c * y on bit planes, m = scale_mask(c) (gf_host.hpp): byte s of m is c * alpha^s, so
// plane t of the product is the XOR of the planes s whose byte s has bit t set (64 VALU)
__device__ __forceinline__ void scale_planes(u32 (&y)[8], uint64_t m)
{
    const u32 w0 = (u32)m, w1 = (u32)(m >> 32);
    u32 o[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
        o[t] = y[0] & bitmask(w0, t);
#pragma unroll
    for (int s = 1; s < 8; ++s)
#pragma unroll
        for (int t = 0; t < 8; ++t)
            o[t] = xor_and(o[t], y[s], bitmask(s < 4 ? w0 : w1, 8 * (s & 3) + t));
#pragma unroll
    for (int t = 0; t < 8; ++t)
        y[t] = o[t];
}

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

// acc (8 planes) ^= c[PR][DL] * the input whose plane subsets are lo / hi, skipped when bit BIT
// of `lost` is clear (phase 2: data row DL not lost; phase 1: parity row PR absent).  The wave-uniform branch lives inside the asm statement, so the compiler sees
// straight-line code: as C++ branches (one per row and input) the same skips cost 50-100 VGPRs
// (one wave per SIMD); per block of 4 rows they fit but compute every row of a touched block.
template <int K, int M, int PR, int DL, int BIT = DL>
__device__ __forceinline__ void coef_planes_skip(u32 *a, const u32 (&lo)[16], const u32 (&hi)[16], uint64_t lost)
{
    constexpr uint32_t c = gfc::Matrix<K, M>::v.c[PR][DL];
    constexpr u32 m0 = plane_mask(c, 0), m1 = plane_mask(c, 1), m2 = plane_mask(c, 2), m3 = plane_mask(c, 3),
                  m4 = plane_mask(c, 4), m5 = plane_mask(c, 5), m6 = plane_mask(c, 6), m7 = plane_mask(c, 7);
    asm volatile("s_bitcmp1_b64 %8, %25\n\t"
                 "s_cbranch_scc0 1f\n\t"
                 "v_bitop3_b32 %0, %0, %9, %10 bitop3:0x96\n\t"
                 "v_bitop3_b32 %1, %1, %11, %12 bitop3:0x96\n\t"
                 "v_bitop3_b32 %2, %2, %13, %14 bitop3:0x96\n\t"
                 "v_bitop3_b32 %3, %3, %15, %16 bitop3:0x96\n\t"
                 "v_bitop3_b32 %4, %4, %17, %18 bitop3:0x96\n\t"
                 "v_bitop3_b32 %5, %5, %19, %20 bitop3:0x96\n\t"
                 "v_bitop3_b32 %6, %6, %21, %22 bitop3:0x96\n\t"
                 "v_bitop3_b32 %7, %7, %23, %24 bitop3:0x96\n"
                 "1:"
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
                 : "s"(lost), "v"(lo[m0 & 15]), "v"(hi[m0 >> 4]), "v"(lo[m1 & 15]), "v"(hi[m1 >> 4]),
                   "v"(lo[m2 & 15]), "v"(hi[m2 >> 4]), "v"(lo[m3 & 15]), "v"(hi[m3 >> 4]), "v"(lo[m4 & 15]),
                   "v"(hi[m4 >> 4]), "v"(lo[m5 & 15]), "v"(hi[m5 >> 4]), "v"(lo[m6 & 15]), "v"(hi[m6 >> 4]),
                   "v"(lo[m7 & 15]), "v"(hi[m7 >> 4]), "i"(BIT)
                 : "scc");
}

// data block J's contribution to the present parity rows R0 + r of the group
template <int K, int M, int R0, int J, int... Rs>
__device__ __forceinline__ void syn_rows(std::integer_sequence<int, Rs...>, u32 *acc, const u32 (&lo)[16],
                                         const u32 (&hi)[16], uint64_t pmask)
{
    (coef_planes_skip<K, M, R0 + Rs, J, R0 + Rs>(&acc[Rs * 8], lo, hi, pmask), ...);
}

// Item J's processing once its 8 dwords are in x: a present data block (copy to its output
// row, bit-sliced rows of the present parity rows) or a present parity row (its syndrome).
template <int K, int M, int R0, int NR, bool FUSED, int J>
__device__ __forceinline__ void syn_process(u32 (&acc)[NR * 8], u32 (&x)[8], const SynCtx &c, u8 *orow0, u32 B,
                                            u32 last, bool copies, u8 *syn, u32 &q)
{
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
        syn_rows<K, M, R0, J>(std::make_integer_sequence<int, NR>{}, acc, lo, hi, c.pmask);  // present rows only
    } else {  // parity row R0 + r: syndrome = its planes ^ the present blocks' contribution, * w
        constexpr int r = J - K;
        transpose8(x);
        u32 y[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            y[i] = acc[r * 8 + i] ^ x[i];
        scale_planes(y, c.wmask[q]);
        if constexpr (FUSED) {  // kept for the solve in the same wave
#pragma unroll
            for (int i = 0; i < 8; ++i)
                acc[r * 8 + i] = y[i];
        } else {
            u8 *o = syn + (u64)q * c.stride;
            st16(o + c.ua, y[0], y[1], y[2], y[3]);
            st16(o + c.ub, y[4], y[5], y[6], y[7]);
        }
        ++q;
    }
}

template <int K, int M, int R0, int NR, int D, bool FUSED, int J>
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
    syn_process<K, M, R0, NR, FUSED, J>(acc, x, c, orow0, B, last, copies, syn, q);
}

template <int K, int M, int R0, int NR, int D, bool FUSED, int... Js>
__device__ __forceinline__ void syn_items(std::integer_sequence<int, Js...>, u32 (&acc)[NR * 8], u32 (&ring)[D][8],
                                          const SynCtx &c, u8 *orow0, u32 B, u32 last, bool copies, u8 *syn, u32 &q)
{
    (syn_item<K, M, R0, NR, D, FUSED, Js>(acc, ring, c, orow0, B, last, copies, syn, q), ...);
}

// ---- phase 1's loads for k >= 32: an LDS ring filled by global_load_lds (no VGPRs) ----------
// Phase 1's items stream through a per-wave LDS ring of D slots (two 1 KiB halves each, one
// global_load_lds_dwordx4 per half: lane l's 16 bytes land at slot + 16 l), so D items are in
// flight without ring registers.  Against the register ring: +0-5 % reassembling, +7-16 %
// recover-only on zfec(32,48) / (64,96); the small-k shapes keep the register ring (LDS ring -8 %
// on (32,48) with 8 lost, -9 % (16,24), -20 % C4; the direct decode is chosen there anyway),
// r03_syn_ab_lds.jsonl.  The ring holds only the items a wave works on: the present data blocks
// but K-1 and the group's present parity rows, in item order ("ranks"), so D slots are D items of
// work ahead.  Rank r lies in slot r % D; its block address comes from a per-lane table (lane r:
// rank r) by a run-time readlane.  Past the last rank the refills re-read the last item (an L2
// hit) into the slot just consumed, so every consume issues exactly two loads and the wait is
// the compile-time s_waitcnt vmcnt(2 (D - 1)) whatever the erasure pattern: loads complete in
// order, so at most that many outstanding retires the slot's, whatever stores are in flight.
// Data block K-1 (possibly short: the byte path) is read into registers before any ring load,
// so every ring load is younger than it.  Round 6 put the ring in rank order (round 5 gave
// every item a slot, absent ones re-reading a present block): neutral, 573 / 544 us at 32 / 24
// lost against 567 / 545 (profiles/r06_phase_stats_*.csv).  Letting the waits count the wave's
// own stores (so the ring runs at its full depth in the copying wave) made it slower, 621 /
// 572 us (tools/archive/kernels_bs_r06_store_waits.diff), and so did one ring shared by the
// pair's two waves with each block read once, 606 / 621 us
// (tools/archive/kernels_bs_r06_syn_share.diff): the ring depth is not what holds phase 1 back.

struct RankRing {
    u64 a, b;  // lane r: the block address of rank r (a) and of rank 64 + r (b)
    u32 n;     // ranks
};

template <int K, int NR, int R0>
__device__ __forceinline__ bool ring_item(const SynCtx &c, u32 it)
{
    constexpr u32 NI = K + NR;
    if (it >= NI || it == (u32)K - 1)
        return false;
    return it < (u32)K ? ((c.dmask >> it) & 1) : ((c.pmask >> (R0 + it - K)) & 1);
}

template <int K, int NR, int R0, class Ring>
__device__ __forceinline__ RankRing rank_ring(Ring &ring, u32 w, const SynCtx &c)
{
    const u32 t = threadIdx.x & 63;
    const bool h0 = ring_item<K, NR, R0>(c, t), h1 = ring_item<K, NR, R0>(c, 64 + t);
    const u64 m0 = __builtin_amdgcn_ballot_w64(h0), m1 = __builtin_amdgcn_ballot_w64(h1);
    const u32 n0 = (u32)__builtin_popcountll(m0);
    auto below = [&](u64 m) { return __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u)); };
    auto addr = [&](u32 it) -> u64 {
        const u32 slot = it < (u32)K ? it : it + R0;
        return (u64)(uintptr_t)(c.blocks + c.off[c.slot0 + slot]);
    };
    // the table goes through slot 0 of the wave's ring (1 KiB = 128 addresses) before any load
    u64 *tbl = reinterpret_cast<u64 *>(&ring.v[w][0][0][0]);
    if (h0)
        tbl[below(m0)] = addr(t);
    if (h1)
        tbl[n0 + below(m1)] = addr(64 + t);
    RankRing rr{tbl[t], tbl[64 + t], n0 + (u32)__builtin_popcountll(m1)};
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read before the first loads overwrite it
    return rr;
}

// rank min(r, n - 1)'s two halves into `slot`
template <class Ring>
__device__ __forceinline__ void rank_issue(Ring &ring, u32 w, const RankRing &rr, const SynCtx &c, u32 r, u32 slot)
{
    r = min(r, rr.n - 1);
    const u64 v = r < 64 ? rr.a : rr.b;
    const u32 lo = __builtin_amdgcn_readlane((u32)v, r & 63), hi = __builtin_amdgcn_readlane((u32)(v >> 32), r & 63);
    const u8 *blk = reinterpret_cast<const u8 *>(((u64)hi << 32) | lo);
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(blk + c.pa),
                                     (__attribute__((address_space(3))) void *)&ring.v[w][slot][0][0], 16, 0, 0);
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(blk + c.pb),
                                     (__attribute__((address_space(3))) void *)&ring.v[w][slot][1][0], 16, 0, 0);
}

template <int K, int M, int R0, int NR, int D, bool FUSED, int J, class Ring>
__device__ __forceinline__ void syn_item_rank(u32 (&acc)[NR * 8], Ring &ring, u32 w, u32 (&xs)[8], const SynCtx &c,
                                              const RankRing &rr, u32 &p, u8 *orow0, u32 B, u32 last, bool copies,
                                              u8 *syn, u32 &q)
{
    if (!item_present<K, NR, R0>(c, J))
        return;
    u32 x[8];
    if constexpr (J == K - 1) {
        wait_vm<2 * D>();  // the ring's 2 D loads in flight are all younger than block K-1's
#pragma unroll
        for (int i = 0; i < 8; ++i)
            x[i] = xs[i];
    } else {
        wait_vm<2 * (D - 1)>();  // rank p has landed
        const u32 slot = p % D;
        const u32x4 a = ring.v[w][slot][0][threadIdx.x & 63], b = ring.v[w][slot][1][threadIdx.x & 63];
        x[0] = a.x;
        x[1] = a.y;
        x[2] = a.z;
        x[3] = a.w;
        x[4] = b.x;
        x[5] = b.y;
        x[6] = b.z;
        x[7] = b.w;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot is read before it is refilled
        rank_issue(ring, w, rr, c, p + D, slot);
        ++p;
    }
    syn_process<K, M, R0, NR, FUSED, J>(acc, x, c, orow0, B, last, copies, syn, q);
}

template <int K, int M, int R0, int NR, int D, bool FUSED, class Ring, int... Js>
__device__ __forceinline__ void syn_items_rank(std::integer_sequence<int, Js...>, u32 (&acc)[NR * 8], Ring &ring,
                                               u32 w, const SynCtx &c, u8 *orow0, u32 B, u32 last, bool copies,
                                               u8 *syn, u32 &q)
{
    u32 xs[8];
    if (item_present<K, NR, R0>(c, K - 1))
        load_syn_item<K, NR, R0, K - 1>(xs, c);
    asm volatile("" ::: "memory");  // block K-1's loads are issued before (older than) every ring load
    const RankRing rr = rank_ring<K, NR, R0>(ring, w, c);
#pragma unroll
    for (u32 r = 0; r < (u32)D; ++r)
        rank_issue(ring, w, rr, c, r, r);
    u32 p = 0;
    (syn_item_rank<K, M, R0, NR, D, FUSED, Js>(acc, ring, w, xs, c, rr, p, orow0, B, last, copies, syn, q), ...);
}

template <int K, int M, int R0, int NR, int D, class Ring>
__device__ __forceinline__ void syn_span(const u8 *__restrict__ blocks, u8 *__restrict__ out, u8 *__restrict__ syn,
                                         const sec::SynDesc &d, const sec::SynSlots &sl, u32 s, bool copies,
                                         Ring &lring)
{
    const u32 B = d.B;
    const u32 lane = (threadIdx.x & 63) * 16;
    SynCtx c{blocks,  sl.off,     sl.avail, sl.masks + d.wq0,     d.slot0,         min(s + lane, B - 16),
             min(s + 1024 + lane, B - 16), s + lane, s + 1024 + lane, d.dmask, d.pmask, sec::syn_stride(B)};
    u32 acc[NR * 8];
#pragma unroll
    for (int i = 0; i < NR * 8; ++i)
        acc[i] = 0;
    // syndrome row of this group's first present parity row: the present rows below R0
    u32 q = (u32)__builtin_popcountll(d.pmask & ((1ull << R0) - 1ull));
    if constexpr (K >= 32) {
        constexpr int DL = SEC_FUSED_LDS_RING;
        const u32 w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        syn_items_rank<K, M, R0, NR, DL, false>(std::make_integer_sequence<int, K + NR>{}, acc, lring, w, c,
                                                out + d.out_off, B, d.last, copies, syn + d.syn_off, q);
    } else {
        u32 ring[D][8];
        load_syn_first<K, NR, R0>(std::make_integer_sequence<int, D>{}, ring, c);
        syn_items<K, M, R0, NR, D, false>(std::make_integer_sequence<int, K + NR>{}, acc, ring, c, out + d.out_off,
                                          B, d.last, copies, syn + d.syn_off, q);
    }
}

// The scaled syndromes go to `syn` as bit planes; sec_solve_bs_kernel then solves for the lost
// blocks.
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
    __shared__ Phase1Lds<K> lring;     // one ring for both row-group variants
    if constexpr (M - K <= NR) {
        syn_span<K, M, 0, NR, D>(blocks, out, syn, d, sl, s, copies, lring);
    } else {
        static_assert(M - K == 2 * NR, "two row groups");
        if (tl.r0 == 0)
            syn_span<K, M, 0, NR, D>(blocks, out, syn, d, sl, s, copies, lring);
        else
            syn_span<K, M, NR, NR, D>(blocks, out, syn, d, sl, s, copies, lring);
    }
}

// Phase 1 of a chunk whose present parity rows lie in both groups (zfec(64,96)), both groups of a
// span in one workgroup of two waves (wave g: group g, one 8-slot LDS ring each, 32 KiB).  The
// tiles above run the groups as separate workgroups, so each group reads the span's data blocks
// from HBM (1.55 GB read per GiB decoded at e = 32 where the blocks are 1.07,
// profiles/r04_syn_pmc.json); here the two waves read them together and the second read hits L2.
template <int K, int M, int NR, int D>
__global__ __launch_bounds__(128) void sec_syndrome_bs_pair_kernel(
    const u8 *__restrict__ blocks, u8 *__restrict__ out, u8 *__restrict__ syn, const sec::SynDesc *__restrict__ descs,
    const sec::Tile *__restrict__ tiles, const sec::SynSlots sl)
{
    static_assert(K >= 32 && M - K == 2 * NR, "two row groups on the LDS ring");
    const sec::Tile tl = tiles[blockIdx.x];
    const sec::SynDesc d = descs[tl.chunk];
    if (tl.t0 >= d.B)
        return;
    // wave 0 copies the primaries (a run-time flag in both waves: a constant false lets the
    // compiler hoist wave 1's transposes and spill)
    const bool first = __builtin_amdgcn_readfirstlane(threadIdx.x) < 64, copies = (tl.ntail & 1) && first;
    __shared__ LdsRing<SEC_FUSED_LDS_RING, 2> lring;
    if (first)
        syn_span<K, M, 0, NR, D>(blocks, out, syn, d, sl, tl.t0, copies, lring);
    else
        syn_span<K, M, NR, NR, D>(blocks, out, syn, d, sl, tl.t0, copies, lring);
}

// ---- decode, phase 2: lost row l = z_l * XOR_{r in S} c[r][l] * (w_r s_r) ----------------------
struct SolveCtx {
    const u8 *syn;  // the chunk's syndrome rows
    uint64_t stride, pmask, lost;
    u32 ua, ub;
};

template <int J>
__device__ __forceinline__ void load_syndrome(u32 (&x)[8], const SolveCtx &c)
{
    const u32 q = (u32)__builtin_popcountll(c.pmask & ((1ull << J) - 1ull));
    const u8 *p = c.syn + (u64)q * c.stride;
    const u32x4 a = *reinterpret_cast<const u32x4 *>(p + c.ua), b = *reinterpret_cast<const u32x4 *>(p + c.ub);
    x[0] = a.x;
    x[1] = a.y;
    x[2] = a.z;
    x[3] = a.w;
    x[4] = b.x;
    x[5] = b.y;
    x[6] = b.z;
    x[7] = b.w;
}

// parity input J's contribution c[J][R0 + r] to every lost row r of the group
template <int K, int M, int R0, int NR, int J, int... Rs>
__device__ __forceinline__ void solve_rows(std::integer_sequence<int, Rs...>, u32 (&acc)[NR * 8], const u32 (&lo)[16],
                                           const u32 (&hi)[16], uint64_t lost)
{
    (coef_planes_skip<K, M, J, R0 + Rs>(&acc[Rs * 8], lo, hi, lost), ...);
}

template <int K, int M, int R0, int NR, int D, int J>
__device__ __forceinline__ void solve_item(u32 (&acc)[NR * 8], u32 (&ring)[D][8], const SolveCtx &c)
{
    constexpr int P = M - K;
    u32 x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        x[i] = ring[J % D][i];
    if constexpr (J + D < P)
        if ((c.pmask >> (J + D)) & 1)
            load_syndrome<J + D>(ring[J % D], c);
    if (!((c.pmask >> J) & 1))
        return;
    u32 lo[16], hi[16];
    subsets(x[0], x[1], x[2], x[3], lo);
    subsets(x[4], x[5], x[6], x[7], hi);
    solve_rows<K, M, R0, NR, J>(std::make_integer_sequence<int, NR>{}, acc, lo, hi, c.lost);
}

template <int K, int M, int R0, int NR, int D, int... Js>
__device__ __forceinline__ void solve_items(std::integer_sequence<int, Js...>, u32 (&acc)[NR * 8], u32 (&ring)[D][8],
                                            const SolveCtx &c)
{
    (solve_item<K, M, R0, NR, D, Js>(acc, ring, c), ...);
}

template <int K, int M, int R0, int NR, int D, int... Js>
__device__ __forceinline__ void solve_first(std::integer_sequence<int, Js...>, u32 (&ring)[D][8], const SolveCtx &c)
{
    ((((c.pmask >> Js) & 1) ? load_syndrome<Js>(ring[Js], c) : void()), ...);
}

// Where the recovered rows go: row l (reassembly; row K-1 clamps to `last`) or the l-th lost
// row in ascending order (recover-only) of the chunk at `out`, scaled by zmask[that rank].
struct OutCtx {
    u8 *out;
    const uint64_t *zmask;
    uint64_t lost;
    u32 B, last, recover, pa, pb;
};

// lost row R0 + r: scale by z, transpose back, store
template <int K, int R0, int NR, int r>
__device__ __forceinline__ void solve_out(u32 (&acc)[NR * 8], const OutCtx &o)
{
    constexpr int l = R0 + r;
    if (!((o.lost >> l) & 1))
        return;
    const u32 t = (u32)__builtin_popcountll(o.lost & ((1ull << l) - 1ull));
    u32 y[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        y[i] = acc[r * 8 + i];
    scale_planes(y, o.zmask[t]);
    transpose8(y);
    u8 *dst = o.out + (u64)(o.recover ? t : (u32)l) * o.B;
    if (l == K - 1 && !o.recover) {
        st16_clamped(dst, o.pa, o.last, y[0], y[1], y[2], y[3]);
        st16_clamped(dst, o.pb, o.last, y[4], y[5], y[6], y[7]);
    } else {
        st16(dst + o.pa, y[0], y[1], y[2], y[3]);
        st16(dst + o.pb, y[4], y[5], y[6], y[7]);
    }
}

template <int K, int R0, int NR, int... Rs>
__device__ __forceinline__ void solve_outs(std::integer_sequence<int, Rs...>, u32 (&acc)[NR * 8], const OutCtx &o)
{
    (solve_out<K, R0, NR, Rs>(acc, o), ...);
}

template <int K, int M, int R0, int NR, int D>
__device__ __forceinline__ void solve_span(const u8 *__restrict__ syn, u8 *__restrict__ out, const sec::SolveDesc &d,
                                           const uint64_t *__restrict__ masks, u32 s)
{
    constexpr int P = M - K;
    static_assert(D >= 1 && D <= P && R0 + NR <= K, "solve shape");
    const u32 B = d.B;
    const u32 lane = (threadIdx.x & 63) * 16;
    const SolveCtx c{syn + d.syn_off, sec::syn_stride(B), d.pmask, d.lost, s + lane, s + 1024 + lane};
    u32 ring[D][8];
    solve_first<K, M, R0, NR, D>(std::make_integer_sequence<int, D>{}, ring, c);
    u32 acc[NR * 8];
#pragma unroll
    for (int i = 0; i < NR * 8; ++i)
        acc[i] = 0;
    solve_items<K, M, R0, NR, D>(std::make_integer_sequence<int, P>{}, acc, ring, c);
    const OutCtx o{out + d.out_off, masks + d.zq0, d.lost, B, d.last, d.recover, min(s + lane, B - 16),
                   min(s + 1024 + lane, B - 16)};
    solve_outs<K, R0, NR>(std::make_integer_sequence<int, NR>{}, acc, o);
}

template <int K, int M, int NR, int D, int... Gs>
__device__ __forceinline__ void solve_group(std::integer_sequence<int, Gs...>, u32 r0, const u8 *__restrict__ syn,
                                            u8 *__restrict__ out, const sec::SolveDesc &d,
                                            const uint64_t *__restrict__ masks, u32 s)
{
    ((r0 == (u32)(Gs * NR) ? solve_span<K, M, Gs * NR, NR, D>(syn, out, d, masks, s) : void()), ...);
}

// Tiles carry the row group's first data row in r0 (groups of NR rows).
template <int K, int M, int NR, int D>
__global__ __launch_bounds__(256) void sec_solve_bs_kernel(const u8 *__restrict__ syn, u8 *__restrict__ out,
                                                           const sec::SolveDesc *__restrict__ descs,
                                                           const sec::Tile *__restrict__ tiles,
                                                           const uint64_t *__restrict__ masks)
{
    const sec::Tile tl = tiles[blockIdx.x];
    const sec::SolveDesc d = descs[tl.chunk];
    const u32 s = tl.t0 + (threadIdx.x >> 6) * kSpan;
    if (s >= d.B)
        return;
    static_assert(K % NR == 0 && K / NR <= 8, "row groups");
    solve_group<K, M, NR, D>(std::make_integer_sequence<int, K / NR>{}, tl.r0, syn, out, d, masks, s);
}

// ---- phase 2 with each span's syndromes staged in LDS once (k >= 32) ---------------------------
// sec_solve_bs_kernel's tiles are (span, 8-row group) pairs, each re-reading all e syndrome rows
// of its span: with e = 32 spread over 8 groups its PMC showed 1.44 GB read per GiB decoded where
// the syndromes are 0.54 (profiles/r04_syn_pmc.json).  Here a workgroup is one span and K / NR
// waves, wave w solving 8-row group w: the e rows (2 KiB each) come into LDS once by
// global_load_lds (spread over the waves), then every wave reads them from LDS.  LDS = e rounded
// up to 8 rows x 2 KiB (dynamic), at most 64 KiB.

// Every syndrome row lands before the first is solved.  Round 6 tried starting on each chunk of
// 8 rows once it had landed (a wave's own loads waited, then a barrier per chunk): 446 / 368 us at
// 32 / 24 lost against 409 / 330 (profiles/r06_phase_stats_*.csv; tools/archive/README.md).

template <int K, int M, int R0, int NR, int J>
__device__ __forceinline__ void solve_item_lds(u32 (&acc)[NR * 8], const u32x4 (*sy)[2][64], uint64_t pmask,
                                               uint64_t lost, u32 lane)
{
    if (!((pmask >> J) & 1))
        return;
    const u32 q = (u32)__builtin_popcountll(pmask & ((1ull << J) - 1ull));
    const u32x4 a = sy[q][0][lane], b = sy[q][1][lane];
    u32 lo[16], hi[16];
    subsets(a.x, a.y, a.z, a.w, lo);
    subsets(b.x, b.y, b.z, b.w, hi);
    solve_rows<K, M, R0, NR, J>(std::make_integer_sequence<int, NR>{}, acc, lo, hi, lost);
}

template <int K, int M, int R0, int NR, int... Js>
__device__ __forceinline__ void solve_span_lds(std::integer_sequence<int, Js...>, const u32x4 (*sy)[2][64],
                                               const sec::SolveDesc &d, const uint64_t *__restrict__ masks,
                                               u8 *__restrict__ out, u32 s, u32 lane)
{
    if (!((d.lost >> R0) & ((1ull << NR) - 1ull)))
        return;
    u32 acc[NR * 8];
#pragma unroll
    for (int i = 0; i < NR * 8; ++i)
        acc[i] = 0;
    (solve_item_lds<K, M, R0, NR, Js>(acc, sy, d.pmask, d.lost, lane), ...);
    const OutCtx o{out + d.out_off, masks + d.zq0, d.lost, d.B, d.last, d.recover, min(s + 16 * lane, d.B - 16),
                   min(s + 1024 + 16 * lane, d.B - 16)};
    solve_outs<K, R0, NR>(std::make_integer_sequence<int, NR>{}, acc, o);
}

template <int K, int M, int NR, int... Gs>
__device__ __forceinline__ void solve_groups_lds(std::integer_sequence<int, Gs...>, u32 w, const u32x4 (*sy)[2][64],
                                                 const sec::SolveDesc &d, const uint64_t *__restrict__ masks,
                                                 u8 *__restrict__ out, u32 s, u32 lane)
{
    ((w == (u32)Gs ? solve_span_lds<K, M, Gs * NR, NR>(std::make_integer_sequence<int, M - K>{}, sy, d, masks, out,
                                                        s, lane)
                   : void()),
     ...);
}

template <int K, int M, int NR>
__global__ __launch_bounds__(64 * (K / NR)) void sec_solve_bs_lds_kernel(const u8 *__restrict__ syn,
                                                                         u8 *__restrict__ out,
                                                                         const sec::SolveDesc *__restrict__ descs,
                                                                         const sec::Tile *__restrict__ tiles,
                                                                         const uint64_t *__restrict__ masks)
{
    static_assert(K % NR == 0 && NR <= 16, "row groups");
    extern __shared__ u32x4 sy_dyn[];
    auto sy = reinterpret_cast<u32x4 (*)[2][64]>(sy_dyn);
    const sec::Tile tl = tiles[blockIdx.x];
    const sec::SolveDesc d = descs[tl.chunk];
    const u32 s = tl.t0;
    if (s >= d.B)  // the whole workgroup (one span)
        return;
    constexpr u32 W = K / NR;
    const u32 w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const u8 *base = syn + d.syn_off + s + 16 * lane;  // rows hold whole spans: no clamping
    const u64 stride = sec::syn_stride(d.B);
    const u32 e = (u32)__builtin_popcountll(d.pmask);
    const u32 n = 2 * e;  // 1 KiB halves of the e rows
    for (u32 i = w; i < n; i += W)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(base + (u64)(i >> 1) * stride + (i & 1) * 1024),
                                         (__attribute__((address_space(3))) void *)&sy[i >> 1][i & 1][0], 16, 0, 0);
    wait_vm<0>();
    __syncthreads();
    solve_groups_lds<K, M, NR>(std::make_integer_sequence<int, W>{}, w, sy, d, masks, out, s, lane);
}

// ---- decode, both phases in one wave (e <= 16, the present parity rows in one group) ---------
// The scaled syndromes stay in the phase-1 accumulators (the compiler parks what does not fit
// in the 256 VGPRs in AGPRs: one wave per SIMD), so they never go through HBM: traffic is the
// decode's own (k blocks read, the chunk or the e rows written).
template <int K, int M, int RP0, int NRP, int NR2, int G, int... Js>
__device__ __forceinline__ void fused_group(std::integer_sequence<int, Js...>, const u32 (&sy)[NRP * 8],
                                            uint64_t pmask, const OutCtx &o)
{
    constexpr int R0 = G * NR2;
    if (!((o.lost >> R0) & ((1ull << NR2) - 1ull)))
        return;
    u32 acc[NR2 * 8];
#pragma unroll
    for (int i = 0; i < NR2 * 8; ++i)
        acc[i] = 0;
    auto one = [&](auto jc) {
        constexpr int r = decltype(jc)::value;
        if (!((pmask >> (RP0 + r)) & 1))
            return;
        u32 lo[16], hi[16];
        subsets(sy[r * 8 + 0], sy[r * 8 + 1], sy[r * 8 + 2], sy[r * 8 + 3], lo);
        subsets(sy[r * 8 + 4], sy[r * 8 + 5], sy[r * 8 + 6], sy[r * 8 + 7], hi);
        solve_rows<K, M, R0, NR2, RP0 + r>(std::make_integer_sequence<int, NR2>{}, acc, lo, hi, o.lost);
    };
    (one(std::integral_constant<int, Js>{}), ...);
    solve_outs<K, R0, NR2>(std::make_integer_sequence<int, NR2>{}, acc, o);
}

template <int K, int M, int RP0, int NRP, int NR2, int... Gs>
__device__ __forceinline__ void fused_groups(std::integer_sequence<int, Gs...>, const u32 (&sy)[NRP * 8],
                                             uint64_t pmask, const OutCtx &o)
{
    (fused_group<K, M, RP0, NRP, NR2, Gs>(std::make_integer_sequence<int, NRP>{}, sy, pmask, o), ...);
}

template <int K, int M, int RP0, int NRP, int NR2, int D>
__device__ __forceinline__ void fused_span(const u8 *__restrict__ blocks, u8 *__restrict__ out,
                                           const sec::SynDesc &d, const sec::SynSlots &sl, u32 s, bool copies,
                                           Phase1Lds<K> &lring)
{
    const u32 B = d.B;
    const u32 lane = (threadIdx.x & 63) * 16;
    SynCtx c{blocks,  sl.off,     sl.avail, sl.masks + d.wq0,     d.slot0,         min(s + lane, B - 16),
             min(s + 1024 + lane, B - 16), s + lane, s + 1024 + lane, d.dmask, d.pmask, 0};
    u32 acc[NRP * 8];
#pragma unroll
    for (int i = 0; i < NRP * 8; ++i)
        acc[i] = 0;
    u32 q = 0;  // every present parity row is in this group
    if constexpr (K >= 32) {
        constexpr int DL = SEC_FUSED_LDS_RING;
        const u32 w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        syn_items_rank<K, M, RP0, NRP, DL, true>(std::make_integer_sequence<int, K + NRP>{}, acc, lring, w, c,
                                                 out + d.out_off, B, d.last, copies, nullptr, q);
    } else {
        u32 ring[D][8];
        load_syn_first<K, NRP, RP0>(std::make_integer_sequence<int, D>{}, ring, c);
        syn_items<K, M, RP0, NRP, D, true>(std::make_integer_sequence<int, K + NRP>{}, acc, ring, c,
                                           out + d.out_off, B, d.last, copies, nullptr, q);
    }
    const uint64_t lost = ~d.dmask & (K >= 64 ? ~0ull : (1ull << K) - 1ull);
    const OutCtx o{out + d.out_off, sl.masks + d.zq0, lost, B, d.last, d.flags & 2u ? 1u : 0u, c.pa, c.pb};
    fused_groups<K, M, RP0, NRP, NR2>(std::make_integer_sequence<int, K / NR2>{}, acc, d.pmask, o);
}

// Tiles: r0 = the parity group's first row; ntail bit 0 = copy the present primaries.
template <int K, int M, int NRP, int NR2, int D>
__global__ __launch_bounds__(256) void sec_decode_bs_kernel(const u8 *__restrict__ blocks, u8 *__restrict__ out,
                                                            const sec::SynDesc *__restrict__ descs,
                                                            const sec::Tile *__restrict__ tiles, const sec::SynSlots sl)
{
    const sec::Tile tl = tiles[blockIdx.x];
    const sec::SynDesc d = descs[tl.chunk];
    const u32 s = tl.t0 + (threadIdx.x >> 6) * kSpan;
    if (s >= d.B)
        return;
    const bool copies = tl.ntail & 1;
    __shared__ Phase1Lds<K> lring;  // one ring for both row-group variants
    if constexpr (M - K <= NRP) {
        fused_span<K, M, 0, NRP, NR2, D>(blocks, out, d, sl, s, copies, lring);
    } else {
        static_assert(M - K == 2 * NRP, "two row groups");
        if (tl.r0 == 0)
            fused_span<K, M, 0, NRP, NR2, D>(blocks, out, d, sl, s, copies, lring);
        else
            fused_span<K, M, NRP, NRP, NR2, D>(blocks, out, d, sl, s, copies, lring);
    }
}

template <int K, int M, int R0, int NR, int D>
hipError_t launch_bs(int lanes, const u8 *in, u8 *par, const sec::EncDesc *d, const sec::Tile *t, u32 nt,
                     hipStream_t s)
{
    void *a = nullptr, *b = nullptr;
    sec_next_launch_events(&a, &b);  // kernel timing (sec_ctx_set_timing) rides on the dispatch
    if constexpr (R0 == -2)
        hipExtLaunchKernelGGL((sec_encode_bs_pair_kernel<K, M, NR, D>), dim3(nt), dim3(128), 0, s, (hipEvent_t)a,
                              (hipEvent_t)b, 0, in, par, d, t);
    else
        hipExtLaunchKernelGGL((sec_encode_bs_kernel<K, M, R0, NR, D>), dim3(nt), dim3(lanes), 0, s, (hipEvent_t)a,
                              (hipEvent_t)b, 0, in, par, d, t);
    return hipGetLastError();
}

// Shapes: (k, m, rows per launch).  Ring depths from the register budget (8 NR accumulators
// + 8 D ring dwords per lane) and A/Bs: zfec(16,24) keeps 10 of its 16 blocks in flight
// (182 VGPRs; +2-8 % over 4 on 1 and 16 MiB chunks), C4 5 (10: -2 %), the 16-row groups 2;
// own blocks in flight per wave of the pair kernel
#ifndef SEC_BS_PAIR_RING
#define SEC_BS_PAIR_RING 2
#endif
struct BsShape {
    int k, m, nr;
};
constexpr BsShape kShapes[] = {{10, 14, 4}, {8, 12, 4}, {16, 24, 8}, {32, 48, 16}, {64, 96, 16}, {8, 11, 3}};
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
    if (lanes < 64 || lanes > 256 || lanes % 64 || shape < 0 || shape >= kNShapes || (group != 0 && group != -2))
        return hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
    // group -2: both groups of a span in one two-wave workgroup (sec_encode_bs_pair_kernel, the
    // two-group zfec(64,96), one tile per span); 0: the one-group shapes
    if (group == -2)
        return shape == 4 ? launch_bs<64, 96, -2, 16, SEC_BS_PAIR_RING>(128, in, par, descs, t, ntiles, s)
                          : hipErrorInvalidValue;
    switch (shape * 4 + group + 1) {
    case 1: return launch_bs<10, 14, 0, 4, 5>(lanes, in, par, descs, t, ntiles, s);
    case 5: return launch_bs<8, 12, 0, 4, 4>(lanes, in, par, descs, t, ntiles, s);
    case 9: return launch_bs<16, 24, 0, 8, 10>(lanes, in, par, descs, t, ntiles, s);
    case 13: return launch_bs<32, 48, 0, 16, 2>(lanes, in, par, descs, t, ntiles, s);
    case 21: return launch_bs<8, 11, 0, 3, 4>(lanes, in, par, descs, t, ntiles, s);
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

// phase-2 rows per group: (10,14) 10, (8,*) 8, the rest 16
// (k >= 32 in groups of 8 rows; groups of 16, four waves per span: -9 % at 32 lost, +4-6 % on
// random 16-30 % losses, profiles/r06_syn_ab_rank_pipe_snr16.jsonl)
constexpr int solve_nr(int k) { return k <= 16 ? k : 8; }

template <int K, int M, int D>
hipError_t launch_solve(int lanes, const u8 *syn, u8 *out, const sec::SolveDesc *d, const sec::Tile *t, u32 nt,
                        const uint64_t *masks, hipStream_t s)
{
    void *a = nullptr, *b = nullptr;
    sec_next_launch_events(&a, &b);
    hipExtLaunchKernelGGL((sec_solve_bs_kernel<K, M, solve_nr(K), D>), dim3(nt), dim3(lanes), 0, s, (hipEvent_t)a,
                          (hipEvent_t)b, 0, syn, out, d, t, masks);
    return hipGetLastError();
}
}  // namespace

int sec_solve_rows(int shape) { return shape >= 0 && shape < kNShapes ? solve_nr(kShapes[shape].k) : 0; }

// Ring depths: the syndromes' 8-dword items, D of them in flight (SEC_SOLVE_RING, build knob;
// 4 against 2: +2-7 % on the two-kernel decodes, r03_syn_ab.jsonl)
#ifndef SEC_SOLVE_RING
#define SEC_SOLVE_RING 4
#endif
int sec_launch_solve_bs(int shape, int lanes, const uint8_t *syn, uint8_t *out, const sec::SolveDesc *descs,
                        const sec::Tile *t, uint32_t ntiles, const uint64_t *masks, void *stream)
{
    if (ntiles == 0)
        return hipSuccess;
    if (lanes < 64 || lanes > 256 || lanes % 64)
        return hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
    constexpr int R = SEC_SOLVE_RING;
    switch (shape) {
    case 0: return launch_solve<10, 14, R < 4 ? R : 4>(lanes, syn, out, descs, t, ntiles, masks, s);
    case 1: return launch_solve<8, 12, R < 4 ? R : 4>(lanes, syn, out, descs, t, ntiles, masks, s);
    case 2: return launch_solve<16, 24, R>(lanes, syn, out, descs, t, ntiles, masks, s);
    case 3: return launch_solve<32, 48, R>(lanes, syn, out, descs, t, ntiles, masks, s);
    case 4: return launch_solve<64, 96, R>(lanes, syn, out, descs, t, ntiles, masks, s);
    case 5: return launch_solve<8, 11, R < 3 ? R : 3>(lanes, syn, out, descs, t, ntiles, masks, s);
    default: return hipErrorInvalidValue;
    }
}

namespace {
// solve rows per group in the one-wave kernel: 8 (16 cost 282 VGPRs = one wave per SIMD, and a
// lone wave leaves the memory pipe idle while it solves: 0.8x the two-kernel path; 8 rows: 224)
constexpr int fused_nr(int k) { return k <= 10 ? k : 8; }

template <int K, int M, int NRP, int D>
hipError_t launch_fused(int lanes, const u8 *blocks, u8 *out, const sec::SynDesc *d, const sec::Tile *t, u32 nt,
                        sec::SynSlots sl, hipStream_t s)
{
    void *a = nullptr, *b = nullptr;
    sec_next_launch_events(&a, &b);
    hipExtLaunchKernelGGL((sec_decode_bs_kernel<K, M, NRP, fused_nr(K), D>), dim3(nt), dim3(lanes), 0, s,
                          (hipEvent_t)a, (hipEvent_t)b, 0, blocks, out, d, t, sl);
    return hipGetLastError();
}
}  // namespace

// fused kernel ring (SEC_FUSED_RING, build knob): 6 against 4 +0-4 % (r03_syn_ab.jsonl)
#ifndef SEC_FUSED_RING
#define SEC_FUSED_RING 6
#endif
int sec_launch_decode_bs(int shape, int lanes, const uint8_t *blocks, uint8_t *out, const sec::SynDesc *descs,
                         const sec::Tile *t, uint32_t ntiles, sec::SynSlots sl, void *stream)
{
    if (ntiles == 0)
        return hipSuccess;
    if (lanes < 64 || lanes > 256 || lanes % 64)
        return hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
    constexpr int R = SEC_FUSED_RING;
    switch (shape) {
    case 0: return launch_fused<10, 14, 4, R>(lanes, blocks, out, descs, t, ntiles, sl, s);
    case 1: return launch_fused<8, 12, 4, R>(lanes, blocks, out, descs, t, ntiles, sl, s);
    case 2: return launch_fused<16, 24, 8, R>(lanes, blocks, out, descs, t, ntiles, sl, s);
    case 3: return launch_fused<32, 48, 16, R>(lanes, blocks, out, descs, t, ntiles, sl, s);
    case 4: return launch_fused<64, 96, 16, R>(lanes, blocks, out, descs, t, ntiles, sl, s);
    case 5: return launch_fused<8, 11, 3, R>(lanes, blocks, out, descs, t, ntiles, sl, s);
    default: return hipErrorInvalidValue;
    }
}

int sec_solve_lds(int shape) { return shape == 3 || shape == 4; }  // zfec(32,48), (64,96)

int sec_launch_solve_bs_lds(int shape, int slots, const uint8_t *syn, uint8_t *out, const sec::SolveDesc *descs,
                            const sec::Tile *t, uint32_t ntiles, const uint64_t *masks, void *stream)
{
    if (ntiles == 0)
        return hipSuccess;
    if (slots < 1 || slots > 32)
        return hipErrorInvalidValue;
    const size_t lds = (size_t)slots * 2048;
    void *a = nullptr, *b = nullptr;
    sec_next_launch_events(&a, &b);
    hipStream_t s = (hipStream_t)stream;
    switch (shape) {
    case 3:
        if (slots > 16)
            return hipErrorInvalidValue;
        hipExtLaunchKernelGGL((sec_solve_bs_lds_kernel<32, 48, solve_nr(32)>), dim3(ntiles), dim3(64 * (32 / solve_nr(32))),
                              lds, s, (hipEvent_t)a, (hipEvent_t)b, 0, syn, out, descs, t, masks);
        break;
    case 4:
        hipExtLaunchKernelGGL((sec_solve_bs_lds_kernel<64, 96, solve_nr(64)>), dim3(ntiles), dim3(64 * (64 / solve_nr(64))),
                              lds, s, (hipEvent_t)a, (hipEvent_t)b, 0, syn, out, descs, t, masks);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

int sec_syn_pair(int shape) { return shape == 4; }  // zfec(64,96)

#ifndef SEC_SYN_RING
#define SEC_SYN_RING 4
#endif
int sec_syn_shape(int k, int m) { return sec_bs_shape(k, m); }

int sec_launch_syndrome_bs(int shape, int lanes, const uint8_t *blocks, uint8_t *out, uint8_t *syn,
                           const sec::SynDesc *descs, const sec::Tile *t, uint32_t ntiles, sec::SynSlots sl,
                           void *stream)
{
    if (ntiles == 0)
        return hipSuccess;
    if (lanes < 64 || lanes > 256 || lanes % 64)
        return hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
    switch (shape) {  // ring depths as the encode's (kernels' register budgets are alike); the
                      // 16-row groups' SEC_SYN_RING (build knob, A/B)
    case 0: return launch_syn<10, 14, 4, 5>(lanes, blocks, out, syn, descs, t, ntiles, sl, s);
    case 1: return launch_syn<8, 12, 4, 4>(lanes, blocks, out, syn, descs, t, ntiles, sl, s);
    case 2: return launch_syn<16, 24, 8, 10>(lanes, blocks, out, syn, descs, t, ntiles, sl, s);
    case 3: return launch_syn<32, 48, 16, SEC_SYN_RING>(lanes, blocks, out, syn, descs, t, ntiles, sl, s);
    case 4: return launch_syn<64, 96, 16, SEC_SYN_RING>(lanes, blocks, out, syn, descs, t, ntiles, sl, s);
    case 5: return launch_syn<8, 11, 3, 4>(lanes, blocks, out, syn, descs, t, ntiles, sl, s);
    default: return hipErrorInvalidValue;
    }
}

int sec_launch_syndrome_bs_pair(int shape, const uint8_t *blocks, uint8_t *out, uint8_t *syn, const sec::SynDesc *descs,
                                const sec::Tile *t, uint32_t ntiles, sec::SynSlots sl, void *stream)
{
    if (ntiles == 0)
        return hipSuccess;
    if (shape != 4)
        return hipErrorInvalidValue;
    void *a = nullptr, *b = nullptr;
    sec_next_launch_events(&a, &b);
    hipExtLaunchKernelGGL((sec_syndrome_bs_pair_kernel<64, 96, 16, SEC_SYN_RING>), dim3(ntiles), dim3(128), 0,
                          (hipStream_t)stream, (hipEvent_t)a, (hipEvent_t)b, 0, blocks, out, syn, descs, t, sl);
    return hipGetLastError();
}

