// kernels_mfma.hip — wide-k Reed–Solomon encode on the integer matrix cores (gfx950).
//
// For k = 32 * G the GF(2^8) encode is VALU-bound in sec_encode_kernel (3 v_perm + 1.5 XOR3
// + 0.5 v_mov per input dword and parity row).  Here it is bit-sliced instead:
// parity bit (rho, b) = XOR over input bits (j, s) of M[(rho, b)][(j, s)] x_j[s], with M the
// 0/1 matrix of gf_host.hpp's mfma_table, and the XOR is the parity of the integer dot product
// v_mfma_i32_32x32x32_i8 computes.  Per wave and group of 128 positions:
//   * lane (r, h) loads one dword (4 positions) of each of its 16 blocks 16h..16h+15;
//   * 4x4 byte transposes turn those into 4 dwords per position q (blocks on bytes);
//   * for bit s, (T >> s) & 0x01010101 is the B operand (K = bit s of 32 blocks, N = 32
//     positions); TILES accumulators of 32 rows (= 4 parity bytes) each;
//   * each lane's 16 accumulator registers hold two whole parity bytes (the table's row
//     order): their low bits are gathered with v_perm and folded into bytes, and each lane
//     stores one dword per parity row (4 positions).
// Positions covered: whole groups of 128 below the chunk's `valid` (every block readable);
// the rest goes to sec_encode_kernel's tiles (api.cpp).  Same results as zfec's fec_encode
// (restated in oracle/fec_oracle.c; /root/reference/storb/util/piece.py:129-130).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "kernels.hpp"

// Waves per SIMD the kernels are compiled for (register budget 512 / this): 2 lets one wave's
// MFMAs overlap another's VALU work and loads (A/B knob).
#ifndef SEC_MFMA_WAVES
#define SEC_MFMA_WAVES 2
#endif
// q steps unrolled (A/B knob): 1 keeps the step loop rolled (static indices by rotation);
// 4 unrolls it, which needs the 512-register budget of one wave per SIMD
#ifndef SEC_MFMA_QU
#define SEC_MFMA_QU 1
#endif

namespace {

using u8 = uint8_t;
using u32 = uint32_t;
using u64 = uint64_t;
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef u32 u32_u __attribute__((aligned(1)));

__device__ __forceinline__ u32 perm(u32 hi, u32 lo, u32 sel) { return __builtin_amdgcn_perm(hi, lo, sel); }

// rows x0..x3 (bytes = positions 0..3) -> columns t[q] (bytes = rows 0..3)
__device__ __forceinline__ void transpose4(u32 x0, u32 x1, u32 x2, u32 x3, u32 &t0, u32 &t1, u32 &t2, u32 &t3)
{
    const u32 a0 = perm(x1, x0, 0x06020400u), a1 = perm(x1, x0, 0x07030501u);
    const u32 a2 = perm(x3, x2, 0x06020400u), a3 = perm(x3, x2, 0x07030501u);
    t0 = perm(a2, a0, 0x05040100u);
    t2 = perm(a2, a0, 0x07060302u);
    t1 = perm(a3, a1, 0x05040100u);
    t3 = perm(a3, a1, 0x07060302u);
}

// Bit 0 of registers o..o+7 of each tile's accumulator (register o + b = bit b of that tile's
// parity byte) -> one dword whose byte t is tile t's parity byte.  Per bit b one v_perm pair
// gathers the four tiles' low bytes, then the planes are masked and shifted into place.
template <int TILES>
__device__ __forceinline__ u32 pack_tiles(const i32x16 (&a)[TILES], int o)
{
    u32 y = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const u32 a0 = (u32)a[0][o + b];
        const u32 a1 = TILES > 1 ? (u32)a[TILES > 1 ? 1 : 0][o + b] : 0u;
        const u32 a2 = TILES > 2 ? (u32)a[TILES > 2 ? 2 : 0][o + b] : 0u;
        const u32 a3 = TILES > 3 ? (u32)a[TILES > 3 ? 3 : 0][o + b] : 0u;
        const u32 g = perm(a1, a0, 0x0c0c0400u) | perm(a3, a2, 0x04000c0cu);  // low bytes of tiles 0..3
        y |= (g & 0x01010101u) << b;
    }
    return y;
}

template <int G, int TILES>
__global__ __launch_bounds__(256, SEC_MFMA_WAVES) void sec_encode_mfma_kernel(const u8 *__restrict__ in, u8 *__restrict__ par,
                                                              const sec::EncDesc *__restrict__ descs,
                                                              const sec::Tile *__restrict__ tiles,
                                                              const i32x4 *__restrict__ mtabs)
{
    constexpr int S = 8 * G, TMAX = G == 1 ? 4 : 2;
    const sec::Tile tl = tiles[blockIdx.x];
    const sec::EncDesc d = descs[tl.chunk];
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
    const u32 end = d.valid & ~(u32)(sec::kMfmaGroup - 1);
    const u32 rg = tl.r0 / (4 * TMAX);
    const i32x4 *at = mtabs + d.pad + (u64)rg * TMAX * S * 64;
    i32x4 A[TILES][S];
#pragma unroll
    for (int t = 0; t < TILES; ++t)
#pragma unroll
        for (int st = 0; st < S; ++st)
            A[t][st] = at[(t * S + st) * 64 + lane];
    const u8 *src = in + d.in_off + (u64)(16 * h) * d.B;
    u8 *dst = par + d.par_off;
    // software pipeline: the next group's 16 * G dword loads are in flight while this group's
    // transposes, MFMAs and packing run (with one or two waves per SIMD nothing else hides them)
    u32 x[G][16];
    auto load = [&](u32 pos) {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int jj = 0; jj < 16; ++jj)
                x[g][jj] = __builtin_nontemporal_load(
                    reinterpret_cast<const u32_u *>(src + (u64)(32 * g + jj) * d.B + pos));
    };
    u32 pos0 = tl.t0 + wave * sec::kMfmaGroup;
    if (pos0 + sec::kMfmaGroup <= end)
        load(pos0 + 4 * r);
    for (u32 gi = 0; gi < sec::kMfmaGroupsPerWave; ++gi) {
        if (pos0 + sec::kMfmaGroup > end)
            break;
        const u32 pos = pos0 + 4 * r;
        u32 T[G][4][4];  // [block group][position q][4 blocks]: bytes = blocks
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int v = 0; v < 4; ++v)
                transpose4(x[g][4 * v], x[g][4 * v + 1], x[g][4 * v + 2], x[g][4 * v + 3], T[g][0][v], T[g][1][v],
                           T[g][2][v], T[g][3][v]);
        const u32 next = pos0 + 4 * sec::kMfmaGroup;
        if (gi + 1 < sec::kMfmaGroupsPerWave && next + sec::kMfmaGroup <= end)
            load(next + 4 * r);
        // P[e][q]: byte t = parity row (t, h, e) at position pos + q.  The q loop stays rolled
        // (its body is the 8 * G * TILES MFMAs, their operands and the packing), walking T and P
        // by rotation so every index is static: unrolled (also with scheduling barriers between
        // the steps) the compiler kept every q's operands live and spilled.
        u32 P[2][4];
#pragma unroll SEC_MFMA_QU
        for (int q = 0; q < 4; ++q) {
            i32x16 acc[TILES];
#pragma unroll
            for (int t = 0; t < TILES; ++t)
                acc[t] = i32x16{};
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int s = 0; s < 8; ++s) {
                    // K = bit s of 16 blocks: a byte's low bit must be that bit, the bits above it
                    // may be anything.  The parity of an integer sum of products with 0/1 entries
                    // depends only on each term's low bit, so (T >> s) needs no mask.
                    const i32x4 b = {(int)(T[g][0][0] >> s), (int)(T[g][0][1] >> s), (int)(T[g][0][2] >> s),
                                     (int)(T[g][0][3] >> s)};
#pragma unroll
                    for (int t = 0; t < TILES; ++t)
                        acc[t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[t][8 * g + s], b, acc[t], 0, 0, 0);
                }
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                P[e][0] = P[e][1];
                P[e][1] = P[e][2];
                P[e][2] = P[e][3];
                P[e][3] = pack_tiles<TILES>(acc, 8 * e);
            }
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    T[g][0][v] = T[g][1][v];
                    T[g][1][v] = T[g][2][v];
                    T[g][2][v] = T[g][3][v];
                }
        }
        // P[e][q] has the tiles on its bytes; the stores want each tile's 4 positions in a dword
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            u32 Y[4];
            transpose4(P[e][0], P[e][1], P[e][2], P[e][3], Y[0], Y[1], Y[2], Y[3]);
#pragma unroll
            for (int t = 0; t < TILES; ++t) {
                const u32 rho = tl.r0 + 4 * t + 2 * h + e;
                if (rho < d.p)
                    __builtin_nontemporal_store(Y[t], reinterpret_cast<u32_u *>(dst + (u64)rho * d.par_stride + pos));
            }
        }
        pos0 = next;
    }
}

template <int G, int TILES>
hipError_t launch_mfma(const u8 *in, u8 *par, const sec::EncDesc *d, const sec::Tile *t, u32 nt, const void *mtabs,
                       hipStream_t s)
{
    void *a = nullptr, *b = nullptr;
    sec_next_launch_events(&a, &b);  // kernel timing (sec_ctx_set_timing) rides on the dispatch
    hipExtLaunchKernelGGL((sec_encode_mfma_kernel<G, TILES>), dim3(nt), dim3(256), 0, s, (hipEvent_t)a,
                          (hipEvent_t)b, 0, in, par, d, t, (const i32x4 *)mtabs);
    return hipGetLastError();
}

}  // namespace

int sec_launch_encode_mfma(int G, int tiles, const uint8_t *in, uint8_t *par, const sec::EncDesc *descs,
                           const sec::Tile *t, uint32_t ntiles, const void *mtabs, void *stream)
{
    if (ntiles == 0)
        return hipSuccess;
    hipStream_t s = (hipStream_t)stream;
    switch (G * 8 + tiles) {
    case 9: return launch_mfma<1, 1>(in, par, descs, t, ntiles, mtabs, s);
    case 10: return launch_mfma<1, 2>(in, par, descs, t, ntiles, mtabs, s);
    case 11: return launch_mfma<1, 3>(in, par, descs, t, ntiles, mtabs, s);
    case 12: return launch_mfma<1, 4>(in, par, descs, t, ntiles, mtabs, s);
    case 17: return launch_mfma<2, 1>(in, par, descs, t, ntiles, mtabs, s);
    case 18: return launch_mfma<2, 2>(in, par, descs, t, ntiles, mtabs, s);
    default: return hipErrorInvalidValue;
    }
}
