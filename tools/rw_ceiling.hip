// rw_ceiling.hip — HBM ceilings for the EC kernels' traffic mixes, launches timed back to back.
//
// Not product code: a calibration tool ("remeasure hbm_study2's decode
// pattern back-to-back").  Each variant is timed as 20 back-to-back launches between two HIP
// events (the way bench.py times the product kernels), median of 7 such batches; prints one
// JSON object, GB/s of algorithmic bytes.  16 B per lane, nontemporal loads and stores, one
// 256-lane workgroup per 4 KiB * U of each stream, like the product kernels.
//   read        1 GiB of loads (XOR-reduced into one dword per workgroup, kept live)
//   write       1 GiB of stores
//   copy_U*     1 GiB -> 1 GiB (the 1:1 mix of a decode); copy_lanes* the same with 64- to
//               1024-lane workgroups (16 B per lane, one step)
//   enc         RS(4,2)-shaped: 4 blocks read, 2 written per 1 MiB chunk (2:1, C2 encode)
//   dec         RS(4,2) reassemble-shaped ({1,3} erased): blocks 0, 2 and both parity blocks
//               read, 4 rows written (1:1, C3 decode), copies stored after the recovered rows
//   dec_early   the same with the two copies stored before the recovered rows
//   rec         recover-only-shaped: 4 blocks read, 2 rows written (2:1, like enc, but the
//               reads come from two buffers as in a decode)
//   c4_*        C4-shaped encode traffic (8192 x 64 KiB, 10 blocks of 6554 B read, 4 written),
//               printed as its own line; c4_aligned_* with B = 6656 (128 B multiple);
//               c4_decode_*: C4 reassembly-shaped (10 slots read, the 64 KiB chunk written)
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef unsigned int u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned char u8;

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            return 1;                                                          \
        }                                                                      \
    } while (0)

__device__ __forceinline__ u32x4 ld(const u8 *p) { return __builtin_nontemporal_load((const u32x4 *)p); }
__device__ __forceinline__ void st(u8 *p, u32x4 v) { __builtin_nontemporal_store(v, (u32x4 *)p); }

constexpr size_t G = 1ull << 30, CH = 1u << 20, BB = CH / 4;

template <int U>
__global__ __launch_bounds__(256) void k_read(const u8 *__restrict__ in, u32 *__restrict__ sink)
{
    const u8 *p = in + (size_t)blockIdx.x * 4096 * U + threadIdx.x * 16;
    u32x4 a = {0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u)
        a ^= ld(p + u * 4096);
    const u32 v = a.x ^ a.y ^ a.z ^ a.w;
    if (v == 0x12345678u)  // practically never: keeps the loads live without a store per lane
        sink[blockIdx.x] = v;
}

template <int U>
__global__ __launch_bounds__(256) void k_write(u8 *__restrict__ out)
{
    u8 *p = out + (size_t)blockIdx.x * 4096 * U + threadIdx.x * 16;
    const u32x4 v = {blockIdx.x, threadIdx.x, 3u, 4u};
#pragma unroll
    for (int u = 0; u < U; ++u)
        st(p + u * 4096, v);
}

template <int U>
__global__ __launch_bounds__(1024) void k_copy(const u8 *__restrict__ in, u8 *__restrict__ out)
{
    const size_t o = (size_t)blockIdx.x * blockDim.x * 16 * U + threadIdx.x * 16;
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        x[u] = ld(in + o + u * blockDim.x * 16);
#pragma unroll
    for (int u = 0; u < U; ++u)
        st(out + o + u * blockDim.x * 16, x[u]);
}

__global__ __launch_bounds__(256) void k_enc(const u8 *__restrict__ in, u8 *__restrict__ par)
{
    constexpr u32 per = BB / 4096;
    const u32 chunk = blockIdx.x / per, t0 = (blockIdx.x % per) * 4096 + threadIdx.x * 16;
    const u8 *s = in + (size_t)chunk * CH + t0;
    u8 *d = par + (size_t)chunk * 2 * BB + t0;
    const u32x4 x0 = ld(s), x1 = ld(s + BB), x2 = ld(s + 2 * BB), x3 = ld(s + 3 * BB);
    st(d, x0 ^ x1 ^ x2 ^ x3);
    st(d + BB, x0 ^ (x1 << 1) ^ x2 ^ (x3 << 2));
}

template <bool EARLY, bool COPIES>
__global__ __launch_bounds__(256) void k_dec(const u8 *__restrict__ in, const u8 *__restrict__ par,
                                             u8 *__restrict__ out)
{
    constexpr u32 per = BB / 4096;
    const u32 chunk = blockIdx.x / per, t0 = (blockIdx.x % per) * 4096 + threadIdx.x * 16;
    const u8 *d = in + (size_t)chunk * CH + t0;
    const u8 *p = par + (size_t)chunk * 2 * BB + t0;
    const u32x4 x0 = ld(d), x2 = ld(d + 2 * BB), x4 = ld(p), x5 = ld(p + BB);
    if constexpr (COPIES) {
        u8 *w = out + (size_t)chunk * CH + t0;
        if (EARLY) {
            st(w, x0);
            st(w + 2 * BB, x2);
        }
        st(w + BB, x0 ^ x4 ^ x5);
        st(w + 3 * BB, x2 ^ x4 ^ (x5 << 1));
        if (!EARLY) {
            st(w, x0);
            st(w + 2 * BB, x2);
        }
    } else {  // recover-only: the two recovered rows, dense
        u8 *w = out + (size_t)chunk * 2 * BB + t0;
        st(w, x0 ^ x4 ^ x5);
        st(w + BB, x2 ^ x4 ^ (x5 << 1));
    }
}

// C4-shaped (8192 x 64 KiB, k = 10, 4 parity rows of B = 6554 B, blocks back to back so most
// are unaligned): the product's v_perm tiles (256 lanes, 4 KiB of each block, 2 per chunk,
// last lane clamped to end at `valid`), every block read, 4 rows written, XOR only.  BB_ = B;
// L = lanes per tile (tiles per chunk = ceil(valid / (16 L))).
typedef u32x4 u32x4_u __attribute__((aligned(1)));
template <u32 BB_, u32 L, u32 PS = BB_>
__global__ __launch_bounds__(1024) void k_c4(const u8 *__restrict__ in, u8 *__restrict__ par, u32 n)
{
    constexpr u32 per = (BB_ + 16 * L - 1) / (16 * L);
    const u32 valid = n - 9 * BB_;
    const u32 chunk = blockIdx.x / per;
    u32 t = (blockIdx.x % per) * 16 * L + threadIdx.x * 16;
    if (t >= valid + 15)
        return;
    t = t + 16 > valid ? valid - 16 : t;
    const u8 *s = in + (size_t)chunk * n + t;
    u8 *d = par + (size_t)chunk * 4 * PS + t;
    u32x4 x[10];
#pragma unroll
    for (int j = 0; j < 10; ++j)
        x[j] = __builtin_nontemporal_load((const u32x4_u *)(s + j * BB_));
    u32x4 a = x[0], b = x[1], c = x[2], e = x[3];
#pragma unroll
    for (int j = 4; j < 10; ++j) {
        a ^= x[j];
        b ^= x[j] << 1;
        c ^= x[j] << 2;
        e ^= x[j] << 3;
    }
    __builtin_nontemporal_store(a, (u32x4_u *)d);
    __builtin_nontemporal_store(b, (u32x4_u *)(d + PS));
    __builtin_nontemporal_store(c, (u32x4_u *)(d + 2 * PS));
    __builtin_nontemporal_store(e, (u32x4_u *)(d + 3 * PS));
}

// C4-decode-shaped: slots = data blocks {1,3,4,6,8,9} of the chunk (block 9 short: reads clamp
// to `valid`) and parity rows 0..3; all 10 output rows of the reassembled 64 KiB written (the
// 6 copies and 4 "recovered" rows, XOR only), 256-lane tiles of 4 KiB as the product's
template <u32 L>
__global__ __launch_bounds__(1024) void k_c4dec(const u8 *__restrict__ in, const u8 *__restrict__ par,
                                                u8 *__restrict__ out, u32 n)
{
    constexpr u32 BB_ = 6554, per = (BB_ + 16 * L - 1) / (16 * L);
    const u32 valid = n - 9 * BB_;
    const u32 chunk = blockIdx.x / per;
    u32 t = (blockIdx.x % per) * 16 * L + threadIdx.x * 16;
    if (t >= valid + 15)
        return;
    t = t + 16 > valid ? valid - 16 : t;
    const u8 *s = in + (size_t)chunk * n + t;
    const u8 *p = par + (size_t)chunk * 4 * BB_ + t;
    u8 *o = out + (size_t)chunk * n + t;
    constexpr int keep[6] = {1, 3, 4, 6, 8, 9};
    u32x4 x[10];
#pragma unroll
    for (int j = 0; j < 6; ++j)
        x[j] = __builtin_nontemporal_load((const u32x4_u *)(s + keep[j] * BB_));
#pragma unroll
    for (int r = 0; r < 4; ++r)
        x[6 + r] = __builtin_nontemporal_load((const u32x4_u *)(p + r * BB_));
    u32x4 a = x[6], b = x[7], c = x[8], e = x[9];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        a ^= x[j];
        b ^= x[j] << 1;
        c ^= x[j] << 2;
        e ^= x[j] << 3;
    }
#pragma unroll
    for (int j = 0; j < 6; ++j)
        __builtin_nontemporal_store(x[j], (u32x4_u *)(o + keep[j] * BB_));
    __builtin_nontemporal_store(a, (u32x4_u *)(o + 0 * BB_));
    __builtin_nontemporal_store(b, (u32x4_u *)(o + 2 * BB_));
    __builtin_nontemporal_store(c, (u32x4_u *)(o + 5 * BB_));
    __builtin_nontemporal_store(e, (u32x4_u *)(o + 7 * BB_));
}


// C5-shaped (RS(8,3) = zfec(8,11), data blocks {1,3,5} erased): chunks of
// 8 blocks of BB_ bytes back to back, 3 parity rows per chunk in their own buffer; slots = data
// blocks {0,2,4,6,7} + the 3 parity rows; all 8 rows of the chunk written (5 copies + 3
// "recovered", XOR only), 256-lane tiles of 4 KiB as the product's decode.  ENC: the encode's
// traffic instead (8 blocks read, 3 rows written).
template <u32 BB_, bool ENC>
__global__ __launch_bounds__(256) void k_c5(const u8 *__restrict__ in, u8 *__restrict__ par, u8 *__restrict__ out)
{
    constexpr u32 per = BB_ / 4096;
    const u32 chunk = blockIdx.x / per, t0 = (blockIdx.x % per) * 4096 + threadIdx.x * 16;
    const u8 *s = in + (size_t)chunk * 8 * BB_ + t0;
    u8 *p = par + (size_t)chunk * 3 * BB_ + t0;
    if constexpr (ENC) {
        u32x4 x[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            x[j] = ld(s + j * BB_);
        u32x4 a = x[0], b = x[0], c = x[0];
#pragma unroll
        for (int j = 1; j < 8; ++j) {
            a ^= x[j];
            b ^= x[j] << 1;
            c ^= x[j] << 2;
        }
        st(p, a);
        st(p + BB_, b);
        st(p + 2 * BB_, c);
    } else {
        constexpr int keep[5] = {0, 2, 4, 6, 7};
        u8 *o = out + (size_t)chunk * 8 * BB_ + t0;
        u32x4 x[8];
#pragma unroll
        for (int j = 0; j < 5; ++j)
            x[j] = ld(s + keep[j] * BB_);
#pragma unroll
        for (int r = 0; r < 3; ++r)
            x[5 + r] = ld(p + r * BB_);
        u32x4 a = x[5], b = x[6], c = x[7];
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            a ^= x[j];
            b ^= x[j] << 1;
            c ^= x[j] << 2;
        }
        st(o + 1 * BB_, a);
        st(o + 3 * BB_, b);
        st(o + 5 * BB_, c);
#pragma unroll
        for (int j = 0; j < 5; ++j)
            st(o + keep[j] * BB_, x[j]);
    }
}

// C5's decode traffic with zfec's own block boundaries (B not a multiple of 16, as in the bench's
// log-uniform chunk sizes): every row read and written at an unaligned address
typedef u32x4 u32x4_u1 __attribute__((aligned(1)));
__device__ __forceinline__ u32x4 ldu(const u8 *p) { return __builtin_nontemporal_load((const u32x4_u1 *)p); }
__device__ __forceinline__ void stu(u8 *p, u32x4 v) { __builtin_nontemporal_store(v, (u32x4_u1 *)p); }
template <u32 BB_>
__global__ __launch_bounds__(256) void k_c5u(const u8 *__restrict__ in, u8 *__restrict__ par, u8 *__restrict__ out)
{
    constexpr u32 per = (BB_ + 4095) / 4096;
    const u32 chunk = blockIdx.x / per, t0 = min((blockIdx.x % per) * 4096 + threadIdx.x * 16, BB_ - 16);
    const u8 *s = in + (size_t)chunk * 8 * BB_ + t0;
    const u8 *p = par + (size_t)chunk * 3 * BB_ + t0;
    constexpr int keep[5] = {0, 2, 4, 6, 7};
    u8 *o = out + (size_t)chunk * 8 * BB_ + t0;
    u32x4 x[8];
#pragma unroll
    for (int j = 0; j < 5; ++j)
        x[j] = ldu(s + keep[j] * BB_);
#pragma unroll
    for (int r = 0; r < 3; ++r)
        x[5 + r] = ldu(p + r * BB_);
    u32x4 a = x[5], b = x[6], c = x[7];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        a ^= x[j];
        b ^= x[j] << 1;
        c ^= x[j] << 2;
    }
    stu(o + 1 * BB_, a);
    stu(o + 3 * BB_, b);
    stu(o + 5 * BB_, c);
#pragma unroll
    for (int j = 0; j < 5; ++j)
        stu(o + keep[j] * BB_, x[j]);
}

// the same with separate row strides for the blocks read and the rows written (which side's
// misalignment costs what)
// XR: workgroup b runs logical tile (b / 64) * 64 + (b % 8) * 8 + (b / 8) % 8, so each XCD (b % 8)
// takes runs of 8 consecutive tiles of a row at about the same time: a 128-byte line that two
// neighbouring tiles' unaligned rows share is written within one XCD's L2
__device__ __forceinline__ void stu_plain(u8 *p, u32x4 v) { *(u32x4_u1 *)p = v; }
template <u32 BI, u32 BO, bool XR = false, u32 OFF = 0, bool NT = true>
__global__ __launch_bounds__(256) void k_c5m(const u8 *__restrict__ in, u8 *__restrict__ par, u8 *__restrict__ out)
{
    constexpr u32 BB_ = BI < BO ? BI : BO, per = (BB_ + 4095) / 4096;
    u32 bx = blockIdx.x;
    if constexpr (XR)
        if ((bx | 63u) < gridDim.x)  // (a partial last run of 64 keeps the plain order)
            bx = (bx & ~63u) + (bx % 8) * 8 + (bx / 8) % 8;
    const u32 chunk = bx / per, t0 = min((bx % per) * 4096 + threadIdx.x * 16, BB_ - 16);
    const u8 *s = in + (size_t)chunk * 8 * BI + t0;
    const u8 *p = par + (size_t)chunk * 3 * BI + t0;
    constexpr int keep[5] = {0, 2, 4, 6, 7};
    u8 *o = out + OFF + (size_t)chunk * 8 * BO + t0;
    u32x4 x[8];
#pragma unroll
    for (int j = 0; j < 5; ++j)
        x[j] = ldu(s + keep[j] * BI);
#pragma unroll
    for (int r = 0; r < 3; ++r)
        x[5 + r] = ldu(p + r * BI);
    u32x4 a = x[5], b = x[6], c = x[7];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        a ^= x[j];
        b ^= x[j] << 1;
        c ^= x[j] << 2;
    }
    NT ? stu(o + 1 * BO, a) : stu_plain(o + 1 * BO, a);
    NT ? stu(o + 3 * BO, b) : stu_plain(o + 3 * BO, b);
    NT ? stu(o + 5 * BO, c) : stu_plain(o + 5 * BO, c);
#pragma unroll
    for (int j = 0; j < 5; ++j)
        NT ? stu(o + keep[j] * BO, x[j]) : stu_plain(o + keep[j] * BO, x[j]);
}

// Unaligned rows written as aligned 16-byte segments: lane l stores the segment that starts in
// its own 16 bytes and ends in lane l + 1's (wave_shl:1 DPP, v_alignbyte by the row's uniform
// misalignment d); lanes 0 and 63 also store their own unaligned 16 bytes, which cover the
// wave's partial first and last segments (the overlaps rewrite identical bytes).  Waves not
// wholly inside the row keep plain unaligned stores.
__device__ __forceinline__ u32 shl1(u32 x) { return (u32)__builtin_amdgcn_mov_dpp((int)x, 0x130, 0xf, 0xf, false); }
template <int Q>
__device__ __forceinline__ u32x4 window(const u32 (&c)[8], u32 r)
{
    return u32x4{__builtin_amdgcn_alignbyte(c[Q + 1], c[Q], r), __builtin_amdgcn_alignbyte(c[Q + 2], c[Q + 1], r),
                 __builtin_amdgcn_alignbyte(c[Q + 3], c[Q + 2], r), __builtin_amdgcn_alignbyte(c[Q + 4], c[Q + 3], r)};
}
template <bool EDGES = true>
__device__ __forceinline__ void st_realigned(u8 *o, u32x4 v, bool whole_wave)
{
    const u32 d = __builtin_amdgcn_readfirstlane((u32)(uintptr_t)o) & 15u;  // (lane offsets are multiples of 16)
    if (!whole_wave || d == 0) {
        stu(o, v);
        return;
    }
    const u32 c[8] = {v.x, v.y, v.z, v.w, shl1(v.x), shl1(v.y), shl1(v.z), shl1(v.w)};
    const u32 sft = 16 - d, r = sft & 3;
    u32x4 w;
    switch (sft >> 2) {
    case 0: w = window<0>(c, r); break;
    case 1: w = window<1>(c, r); break;
    case 2: w = window<2>(c, r); break;
    default: w = window<3>(c, r); break;
    }
    const u32 lane = threadIdx.x & 63;
    if (lane < 63)
        st(o - d + 16, w);
    if (EDGES && (lane == 0 || lane == 63))
        stu(o, v);
}
template <u32 BB_, bool EDGES = true>
__global__ __launch_bounds__(256) void k_c5r(const u8 *__restrict__ in, u8 *__restrict__ par, u8 *__restrict__ out)
{
    constexpr u32 per = (BB_ + 4095) / 4096;
    const u32 chunk = blockIdx.x / per, traw = (blockIdx.x % per) * 4096 + threadIdx.x * 16;
    const u32 t0 = min(traw, BB_ - 16);
    const bool whole = ((blockIdx.x % per) * 4096 + (threadIdx.x & ~63u) * 16 + 1024) <= BB_;  // wave-uniform
    const u8 *s = in + (size_t)chunk * 8 * BB_ + t0;
    const u8 *p = par + (size_t)chunk * 3 * BB_ + t0;
    constexpr int keep[5] = {0, 2, 4, 6, 7};
    u8 *o = out + (size_t)chunk * 8 * BB_ + t0;
    u32x4 x[8];
#pragma unroll
    for (int j = 0; j < 5; ++j)
        x[j] = ldu(s + keep[j] * BB_);
#pragma unroll
    for (int r = 0; r < 3; ++r)
        x[5 + r] = ldu(p + r * BB_);
    u32x4 a = x[5], b = x[6], c = x[7];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        a ^= x[j];
        b ^= x[j] << 1;
        c ^= x[j] << 2;
    }
    st_realigned<EDGES>(o + 1 * BB_, a, whole);
    st_realigned<EDGES>(o + 3 * BB_, b, whole);
    st_realigned<EDGES>(o + 5 * BB_, c, whole);
#pragma unroll
    for (int j = 0; j < 5; ++j)
        st_realigned<EDGES>(o + keep[j] * BB_, x[j], whole);
}

template <class F>
double time_ms(F launch)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 5; ++i)
        launch();
    std::vector<float> t;
    for (int i = 0; i < 7; ++i) {
        (void)hipEventRecord(a);
        for (int r = 0; r < 20; ++r)
            launch();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        t.push_back(ms / 20);
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main()
{
    u8 *a, *b, *c;
    u32 *sink;
    CK(hipMalloc(&a, G));
    CK(hipMalloc(&b, G));
    CK(hipMalloc(&c, G));
    CK(hipMalloc(&sink, G / 4096 * 4));
    CK(hipMemset(a, 7, G));
    CK(hipMemset(b, 1, G));
    CK(hipMemset(c, 3, G));
    auto rate = [&](double bytes, double ms) { return bytes / (ms * 1e-3) / 1e9; };
    const dim3 blk(256);
    const double rd = rate(G, time_ms([&] { hipLaunchKernelGGL((k_read<1>), dim3(G / 4096), blk, 0, 0, a, sink); }));
    const double rd4 = rate(G, time_ms([&] { hipLaunchKernelGGL((k_read<4>), dim3(G / 16384), blk, 0, 0, a, sink); }));
    const double wr = rate(G, time_ms([&] { hipLaunchKernelGGL((k_write<1>), dim3(G / 4096), blk, 0, 0, c); }));
    const double wr4 = rate(G, time_ms([&] { hipLaunchKernelGGL((k_write<4>), dim3(G / 16384), blk, 0, 0, c); }));
    const double cp1 = rate(2.0 * G, time_ms([&] { hipLaunchKernelGGL((k_copy<1>), dim3(G / 4096), blk, 0, 0, a, c); }));
    const double cp2 = rate(2.0 * G, time_ms([&] { hipLaunchKernelGGL((k_copy<2>), dim3(G / 8192), blk, 0, 0, a, c); }));
    const double cp4 = rate(2.0 * G, time_ms([&] { hipLaunchKernelGGL((k_copy<4>), dim3(G / 16384), blk, 0, 0, a, c); }));
    const double cpl64 = rate(2.0 * G, time_ms([&] { hipLaunchKernelGGL((k_copy<1>), dim3(G / 1024), dim3(64), 0, 0, a, c); }));
    const double cpl128 = rate(2.0 * G, time_ms([&] { hipLaunchKernelGGL((k_copy<1>), dim3(G / 2048), dim3(128), 0, 0, a, c); }));
    const double cpl512 = rate(2.0 * G, time_ms([&] { hipLaunchKernelGGL((k_copy<1>), dim3(G / 8192), dim3(512), 0, 0, a, c); }));
    const double cpl1024 = rate(2.0 * G, time_ms([&] { hipLaunchKernelGGL((k_copy<1>), dim3(G / 16384), dim3(1024), 0, 0, a, c); }));
    const double en = rate(1.5 * G, time_ms([&] { hipLaunchKernelGGL(k_enc, dim3(G / 16384), blk, 0, 0, a, b); }));
    const double de = rate(2.0 * G, time_ms([&] { hipLaunchKernelGGL((k_dec<false, true>), dim3(G / 16384), blk, 0, 0, a, b, c); }));
    const double dee = rate(2.0 * G, time_ms([&] { hipLaunchKernelGGL((k_dec<true, true>), dim3(G / 16384), blk, 0, 0, a, b, c); }));
    const double re = rate(1.5 * G, time_ms([&] { hipLaunchKernelGGL((k_dec<false, false>), dim3(G / 16384), blk, 0, 0, a, b, c); }));
    // C4-shaped: algorithmic bytes = n read + 4 B written per chunk
    constexpr u32 NC4 = 8192;
    auto c4 = [&](auto kern, u32 BBv, u32 L, u32 n) {
        const u32 per = (BBv + 16 * L - 1) / (16 * L);
        return rate((double)NC4 * (n + 4.0 * BBv),
                    time_ms([&] { hipLaunchKernelGGL(kern, dim3(NC4 * per), dim3(L), 0, 0, a, b, n); }));
    };
    const double c4_256 = c4(k_c4<6554, 256>, 6554, 256, 65536);
    const double c4_448 = c4(k_c4<6554, 448>, 6554, 448, 65536);
    const double c4_64 = c4(k_c4<6554, 64>, 6554, 64, 65536);
    const double c4a_256 = c4(k_c4<6656, 256>, 6656, 256, 66560);  // B a multiple of 128 (aligned blocks)
    const double c4a_448 = c4(k_c4<6656, 448>, 6656, 448, 66560);
    const double c4p_256 = c4(k_c4<6554, 256, 6656>, 6554, 256, 65536);  // parity stride 6656: aligned writes
    const double c4p_448 = c4(k_c4<6554, 448, 6656>, 6554, 448, 65536);
    const double c4r_256 = c4(k_c4<6656, 256, 6554>, 6656, 256, 66560);  // aligned reads, unaligned writes
    // C4 decode-shaped: 10 slots of B read + n written per chunk (the product's algorithmic bytes)
    auto c4d = [&](auto kern, u32 L) {
        const u32 per = (6554 + 16 * L - 1) / (16 * L);
        return rate((double)NC4 * (10.0 * 6554 + 65536),
                    time_ms([&] { hipLaunchKernelGGL(kern, dim3(NC4 * per), dim3(L), 0, 0, a, b, c, 65536u); }));
    };
    // C5-shaped: algorithmic bytes per chunk: decode 8 B read + 8 B written, encode 8 B + 3 B
    auto c5 = [&](auto kern, u32 BBv, double per_chunk) {
        const u32 nch = (u32)(G / (8ull * BBv));
        return rate((double)nch * per_chunk * BBv,
                    time_ms([&] { hipLaunchKernelGGL(kern, dim3(nch * (BBv / 4096)), dim3(256), 0, 0, a, b, c); }));
    };
    printf("{\"c5_decode_B256K\": %.1f, \"c5_decode_B32K\": %.1f, \"c5_decode_B8K\": %.1f, \"c5_encode_B256K\": %.1f, "
           "\"c5_encode_B32K\": %.1f}\n",
           c5(k_c5<262144, false>, 262144, 16.0), c5(k_c5<32768, false>, 32768, 16.0), c5(k_c5<8192, false>, 8192, 16.0),
           c5(k_c5<262144, true>, 262144, 11.0), c5(k_c5<32768, true>, 32768, 11.0));
    auto c5u = [&](auto kern, u32 BBv) {
        const u32 nch = (u32)(G / (8ull * BBv + 4096));
        return rate((double)nch * 16.0 * BBv,
                    time_ms([&] { hipLaunchKernelGGL(kern, dim3(nch * ((BBv + 4095) / 4096)), dim3(256), 0, 0, a, b, c); }));
    };
    printf("{\"c5_decode_unaligned_B256K+6\": %.1f, \"c5_decode_unaligned_B32K+6\": %.1f, \"c5_decode_B256K_again\": %.1f}\n",
           c5u(k_c5u<262150>, 262150), c5u(k_c5u<32774>, 32774), c5(k_c5<262144, false>, 262144, 16.0));
    auto c5m = [&](auto kern, u32 BI, u32 BO) {
        const u32 BBv = BI < BO ? BI : BO, BMAX = BI < BO ? BO : BI;
        const u32 nch = (u32)(G / (8ull * BMAX + 4096));
        return rate((double)nch * 16.0 * BBv,
                    time_ms([&] { hipLaunchKernelGGL(kern, dim3(nch * ((BBv + 4095) / 4096)), dim3(256), 0, 0, a, b, c); }));
    };
    printf("{\"c5_decode_unaligned_reads_only_B256K\": %.1f, \"c5_decode_unaligned_writes_only_B256K\": %.1f, "
           "\"c5_decode_unaligned_reads_only_B32K\": %.1f, \"c5_decode_unaligned_writes_only_B32K\": %.1f}\n",
           c5m(k_c5m<262150, 262144>, 262150, 262144), c5m(k_c5m<262144, 262150>, 262144, 262150),
           c5m(k_c5m<32774, 32768>, 32774, 32768), c5m(k_c5m<32768, 32774>, 32768, 32774));
    printf("{\"c5_decode_unaligned_xcd_runs_B256K\": %.1f, \"c5_decode_unaligned_writes_only_xcd_runs_B256K\": %.1f, "
           "\"c5_decode_aligned_xcd_runs_B256K\": %.1f, \"c5_decode_unaligned_xcd_runs_B32K\": %.1f}\n",
           c5m(k_c5m<262150, 262150, true>, 262150, 262150), c5m(k_c5m<262144, 262150, true>, 262144, 262150),
           c5m(k_c5m<262144, 262144, true>, 262144, 262144), c5m(k_c5m<32774, 32774, true>, 32774, 32774));
    // unaligned rows with plain (write-back) stores, plain and XCD-run tile order: whether two
    // waves' / workgroups' partial sectors merge in L2 before they are written back
    printf("{\"c5_decode_unaligned_plain_st_B256K\": %.1f, \"c5_decode_unaligned_plain_st_xcd_runs_B256K\": %.1f, "
           "\"c5_decode_unaligned_nt_B256K\": %.1f, \"c5_decode_aligned_plain_st_B256K\": %.1f}\n",
           c5m(k_c5m<262150, 262150, false, 0, false>, 262150, 262150),
           c5m(k_c5m<262150, 262150, true, 0, false>, 262150, 262150),
           c5m(k_c5m<262150, 262150, false, 0, true>, 262150, 262150),
           c5m(k_c5m<262144, 262144, false, 0, false>, 262144, 262144));
    // aligned rows whose output base is shifted by 16 / 64 / 128 bytes: 16-byte aligned stores
    // whose 1 KiB wave runs start inside a 128-byte line (16, 64) or on one (128)
    printf("{\"c5_decode_out_shift16_B256K\": %.1f, \"c5_decode_out_shift64_B256K\": %.1f, "
           "\"c5_decode_out_shift128_B256K\": %.1f, \"c5_decode_out_shift0_B256K\": %.1f}\n",
           c5m(k_c5m<262144, 262144, false, 16>, 262144, 262144), c5m(k_c5m<262144, 262144, false, 64>, 262144, 262144),
           c5m(k_c5m<262144, 262144, false, 128>, 262144, 262144), c5m(k_c5m<262144, 262144, false, 0>, 262144, 262144));
    {
        // realigned stores: correctness against the plain unaligned kernel on the same inputs
        const u32 BBv = 262150, nch = (u32)(G / (8ull * BBv + 4096));
        hipLaunchKernelGGL(k_c5u<262150>, dim3(nch * ((BBv + 4095) / 4096)), dim3(256), 0, 0, a, b, c);
        std::vector<u8> ref(4 << 20), got(4 << 20);
        CK(hipMemcpy(ref.data(), c, ref.size(), hipMemcpyDeviceToHost));
        CK(hipMemset(c, 0x5a, (size_t)nch * 8 * BBv));
        hipLaunchKernelGGL(k_c5r<262150>, dim3(nch * ((BBv + 4095) / 4096)), dim3(256), 0, 0, a, b, c);
        CK(hipMemcpy(got.data(), c, got.size(), hipMemcpyDeviceToHost));
        printf("{\"c5_realigned_matches_unaligned\": %s, \"c5_decode_realigned_B256K+6\": %.1f, "
               "\"c5_decode_realigned_B32K+6\": %.1f, \"c5_decode_unaligned_B256K+6_again\": %.1f, "
               "\"c5_decode_realigned_no_edges_B256K+6\": %.1f, \"c5_decode_realigned_no_edges_B32K+6\": %.1f}\n",
               ref == got ? "true" : "false", c5u(k_c5r<262150>, 262150), c5u(k_c5r<32774>, 32774),
               c5u(k_c5u<262150>, 262150), c5u(k_c5r<262150, false>, 262150), c5u(k_c5r<32774, false>, 32774));
    }
    const double c4d_256 = c4d(k_c4dec<256>, 256);
    const double c4d_448 = c4d(k_c4dec<448>, 448);
    printf("{\"c4_decode_lanes256\": %.1f, \"c4_decode_lanes448\": %.1f}\n", c4d_256, c4d_448);
    printf("{\"c4_lanes256\": %.1f, \"c4_lanes448\": %.1f, \"c4_lanes64\": %.1f, \"c4_aligned_lanes256\": %.1f, "
           "\"c4_aligned_lanes448\": %.1f, \"c4_pstride6656_lanes256\": %.1f, \"c4_pstride6656_lanes448\": %.1f, "
           "\"c4_aligned_reads_only_lanes256\": %.1f}\n",
           c4_256, c4_448, c4_64, c4a_256, c4a_448, c4p_256, c4p_448, c4r_256);
    printf("{\"unit\": \"GB/s\", \"read_U1\": %.1f, \"read_U4\": %.1f, \"write_U1\": %.1f, \"write_U4\": %.1f, "
           "\"copy_U1\": %.1f, \"copy_U2\": %.1f, \"copy_U4\": %.1f, \"enc\": %.1f, \"dec\": %.1f, \"dec_early\": %.1f, "
           "\"rec\": %.1f, \"copy_lanes64\": %.1f, \"copy_lanes128\": %.1f, \"copy_lanes512\": %.1f, "
           "\"copy_lanes1024\": %.1f}\n", rd, rd4, wr, wr4, cp1, cp2, cp4, en, de, dee, re, cpl64, cpl128, cpl512, cpl1024);
    CK(hipDeviceSynchronize());
    return 0;
}
