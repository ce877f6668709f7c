// kernels_xb.hip — encode for the zfec shapes with many parity rows ((64,96), (32,48): the
// reference policy's shapes for 16 GiB .. 1 TiB files), with the
// encode matrix fixed at compile time.
//
// sec_encode_kernel is VALU-bound on these shapes (profiles/r02_pmc_wide.json: 0.92-1.00 of
// the issue floor): every parity row costs 3 v_perm + 1.5 XOR3 per input dword, so p = 32
// rows cost ~150 VALU instructions per dword.  zfec's matrix depends only on (k, m), so here
// it is a constexpr and the products become XORs of a per-block basis:
//   * c * x = XOR over the bits b of c of (alpha^b * x)   (polynomial basis, alpha = 2);
//   * per input dword x the 8 products y_b = alpha^b * x (y_0 = x, then xtime: 5 VALU each);
//   * y_0..y_3 and y_4..y_7 combine into the XOR of every subset of each half ("lo" / "hi"
//     nibble combinations, at most 11 + 11 instructions, only those some row of this block
//     uses are kept by the compiler);
//   * parity row r then takes one XOR3: acc_r ^= lo[c_rj & 15] ^ hi[c_rj >> 4].
// Per input dword: 35 + <= 22 + p instructions (p = 32: <= 89, against ~150), shared by all
// p rows of the chunk in one pass (one read of the k blocks).  Each lane owns W consecutive
// dwords of every block; the k blocks stream through a ring of D loads in flight.
// Positions covered: [0, valid rounded down to 16) of each chunk (every block readable there);
// the rest goes to sec_encode_kernel's tiles (api.cpp add_xb_work).  Same results as zfec's
// fec_encode (restated in oracle/fec_oracle.c; /root/reference/storb/util/piece.py:129-130).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <utility>

#include "gf_const.hpp"
#include "kernels.hpp"

namespace {

using u8 = uint8_t;
using u32 = uint32_t;
using u64 = uint64_t;
typedef u32 u32_u __attribute__((aligned(1)));
typedef u32 u32x2 __attribute__((ext_vector_type(2)));
typedef u32x2 u32x2_u __attribute__((aligned(1)));

using gfc::Matrix;

// ---- device arithmetic --------------------------------------------------------------------
__device__ __forceinline__ u32 xor3(u32 a, u32 b, u32 c)
{
    u32 r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// (a & b) ^ c
__device__ __forceinline__ u32 and_xor(u32 a, u32 b, u32 c)
{
    u32 r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x6a" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// alpha * y for the 4 bytes of y: shift left, and 0x1D into every byte whose top bit fell out
// (a 2-entry v_perm lookup on that bit)
__device__ __forceinline__ u32 xtime(u32 y)
{
    const u32 h = (y >> 7) & 0x01010101u;
    return and_xor(y << 1, 0xFEFEFEFEu, __builtin_amdgcn_perm(0u, 0x00001D00u, h));
}

template <int W>
__device__ __forceinline__ void load_w(u32 (&x)[W], const u8 *p)
{
    if constexpr (W == 1) {
        x[0] = __builtin_nontemporal_load(reinterpret_cast<const u32_u *>(p));
    } else {
        static_assert(W == 2, "W = 1 or 2 dwords per lane");
        const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2_u *>(p));
        x[0] = v.x;
        x[1] = v.y;
    }
}
template <int W>
__device__ __forceinline__ void store_w(u8 *p, const u32 (&x)[W])
{
    if constexpr (W == 1)
        __builtin_nontemporal_store(x[0], reinterpret_cast<u32_u *>(p));
    else
        __builtin_nontemporal_store(u32x2{x[0], x[1]}, reinterpret_cast<u32x2_u *>(p));
}

// XOR of the subset S (4 bits, S >= 1) of v[0..3] (pair23 = v[2] ^ v[3]); resolved at compile
// time per coefficient, and a subset no row of the block uses is never computed
template <int S>
__device__ __forceinline__ u32 subset(const u32 (&v)[4], u32 pair23)
{
    if constexpr (S == 1 || S == 2 || S == 4 || S == 8)
        return v[S == 1 ? 0 : S == 2 ? 1 : S == 4 ? 2 : 3];
    else if constexpr (S == 12)
        return pair23;
    else if constexpr (S == 3 || S == 5 || S == 6 || S == 9 || S == 10)
        return v[S & 1 ? 0 : 1] ^ v[S == 3 ? 1 : S == 5 || S == 6 ? 2 : 3];
    else if constexpr (S == 7)
        return xor3(v[0], v[1], v[2]);
    else if constexpr (S == 11)
        return xor3(v[0], v[1], v[3]);
    else if constexpr (S == 13)
        return xor3(v[0], v[2], v[3]);
    else if constexpr (S == 14)
        return xor3(v[1], v[2], v[3]);
    else
        return xor3(v[0], v[1], pair23);  // 15
}

// Positions [0, xb_end(valid)) of a chunk go to this kernel.
__host__ __device__ constexpr u32 xb_end(u32 valid) { return valid / 16 * 16; }

constexpr int kRing = 8;  // blocks whose loads are in flight ahead of the one being combined

// Everything below is instantiated per (block J, row R): the coefficient is a template
// constant, so each row's update compiles to at most one XOR3 with no run-time branch.
template <int K, int M, int J, int R, int W>
__device__ __forceinline__ void row_update(u32 (&acc)[M - K][W], const u32 (&lo)[W][4], const u32 (&hi)[W][4],
                                           const u32 (&lo23)[W], const u32 (&hi23)[W])
{
    constexpr int c = Matrix<K, M>::v.c[R][J];
    constexpr int cl = c & 15, ch = c >> 4;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        if constexpr (cl && ch)
            acc[R][w] = xor3(acc[R][w], subset<cl ? cl : 1>(lo[w], lo23[w]), subset<ch ? ch : 1>(hi[w], hi23[w]));
        else if constexpr (cl)
            acc[R][w] ^= subset<cl ? cl : 1>(lo[w], lo23[w]);
        else if constexpr (ch)
            acc[R][w] ^= subset<ch ? ch : 1>(hi[w], hi23[w]);
    }
}

template <int K, int M, int J, int W, int... Rs>
__device__ __forceinline__ void block_rows(std::integer_sequence<int, Rs...>, u32 (&acc)[M - K][W], const u32 (&lo)[W][4],
                                           const u32 (&hi)[W][4], const u32 (&lo23)[W], const u32 (&hi23)[W])
{
    (row_update<K, M, J, Rs, W>(acc, lo, hi, lo23, hi23), ...);
}

template <int K, int M, int W, int J>
__device__ __forceinline__ void one_block(u32 (&acc)[M - K][W], u32 (&ring)[kRing][W], const u8 *src, u64 B)
{
    u32 x[W];
#pragma unroll
    for (int w = 0; w < W; ++w)
        x[w] = ring[J % kRing][w];
    if constexpr (J + kRing < K)
        load_w<W>(ring[J % kRing], src + (u64)(J + kRing) * B);
    u32 lo[W][4], hi[W][4], lo23[W], hi23[W];
#pragma unroll
    for (int w = 0; w < W; ++w) {
        lo[w][0] = x[w];
#pragma unroll
        for (int b = 1; b < 4; ++b)
            lo[w][b] = xtime(lo[w][b - 1]);
        hi[w][0] = xtime(lo[w][3]);
#pragma unroll
        for (int b = 1; b < 4; ++b)
            hi[w][b] = xtime(hi[w][b - 1]);
        lo23[w] = lo[w][2] ^ lo[w][3];
        hi23[w] = hi[w][2] ^ hi[w][3];
    }
    block_rows<K, M, J, W>(std::make_integer_sequence<int, M - K>{}, acc, lo, hi, lo23, hi23);
}

template <int K, int M, int W, int... Js>
__device__ __forceinline__ void all_blocks(std::integer_sequence<int, Js...>, u32 (&acc)[M - K][W],
                                           u32 (&ring)[kRing][W], const u8 *src, u64 B)
{
    (one_block<K, M, W, Js>(acc, ring, src, B), ...);
}

template <int K, int M, int W>
__global__ __launch_bounds__(256) void sec_encode_xb_kernel(const u8 *__restrict__ in, u8 *__restrict__ par,
                                                            const sec::EncDesc *__restrict__ descs,
                                                            const sec::Tile *__restrict__ tiles)
{
    constexpr int P = M - K;
    const sec::Tile tl = tiles[blockIdx.x];
    const sec::EncDesc d = descs[tl.chunk];
    const u32 t = tl.t0 + threadIdx.x * 4 * W;
    if (t + 4 * W > xb_end(d.valid))
        return;
    const u8 *src = in + d.in_off + t;
    const u64 B = d.B;

    u32 acc[P][W];
#pragma unroll
    for (int r = 0; r < P; ++r)
#pragma unroll
        for (int w = 0; w < W; ++w)
            acc[r][w] = 0;
    u32 ring[kRing][W];
#pragma unroll
    for (int j = 0; j < kRing && j < K; ++j)
        load_w<W>(ring[j], src + (u64)j * B);
    all_blocks<K, M, W>(std::make_integer_sequence<int, K>{}, acc, ring, src, B);
    u8 *dst = par + d.par_off + t;
#pragma unroll
    for (int r = 0; r < P; ++r)
        store_w<W>(dst + (u64)r * d.par_stride, acc[r]);
}

template <int K, int M, int W>
hipError_t launch_xb(const u8 *in, u8 *par, const sec::EncDesc *d, const sec::Tile *t, u32 nt, hipStream_t s)
{
    void *a = nullptr, *b = nullptr;
    sec_next_launch_events(&a, &b);  // kernel timing (sec_ctx_set_timing) rides on the dispatch
    hipExtLaunchKernelGGL((sec_encode_xb_kernel<K, M, W>), dim3(nt), dim3(256), 0, s, (hipEvent_t)a, (hipEvent_t)b, 0,
                          in, par, d, t);
    return hipGetLastError();
}

}  // namespace

int sec_xb_shape(int k, int m)
{
    if (k == 64 && m == 96)
        return 0;
    if (k == 32 && m == 48)
        return 1;
    return -1;
}

uint32_t sec_xb_end(uint32_t valid) { return xb_end(valid); }

int sec_launch_encode_xb(int shape, int W, const uint8_t *in, uint8_t *par, const sec::EncDesc *descs,
                         const sec::Tile *t, uint32_t ntiles, void *stream)
{
    if (ntiles == 0)
        return hipSuccess;
    hipStream_t s = (hipStream_t)stream;
    switch (shape * 4 + W) {
    case 1: return launch_xb<64, 96, 1>(in, par, descs, t, ntiles, s);
    case 2: return launch_xb<64, 96, 2>(in, par, descs, t, ntiles, s);
    case 5: return launch_xb<32, 48, 1>(in, par, descs, t, ntiles, s);
    case 6: return launch_xb<32, 48, 2>(in, par, descs, t, ntiles, s);
    default: return hipErrorInvalidValue;
    }
}
