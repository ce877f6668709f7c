// hbm_study2.hip — tile granularity study for the encode / decode access patterns (MI355X).
//
// Not product code: a calibration tool (follows hbm_study.hip).  Question: how many
// contiguous bytes should one workgroup read / write per burst, and does a persistent
// (grid-stride over tiles) schedule beat one workgroup per tile?  Prints JSON lines, GB/s of
// algorithmic bytes (HIP events, median of 15 after 3 warm-ups):
//   w_U*      1.5 GiB of nt stores, one 256-lane workgroup per 4 KiB * U (U u-steps of 4 KiB)
//   e_U*      RS(4,2) encode pattern on 1024 x 1 MiB chunks (4 blocks read, 2 written, XOR in
//             place of GF), tile = 4 KiB * U positions; _wc = wave-contiguous layout (each
//             wave owns 1 KiB * U contiguous positions instead of the workgroup interleave);
//             _xcd = XCD-contiguous tile order; _pers = 2048 persistent workgroups looping
//             over tiles with the next tile's first block prefetched
//   d_U*      RS(4,2) decode pattern ({1,3} erased: read blocks 0, 2 and both parity blocks,
//             write the 4 rows of the chunk), same tile / order variants
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef unsigned int u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned char u8;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                         \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

__device__ __forceinline__ u32x4 ld(const u8 *p) { return __builtin_nontemporal_load((const u32x4 *)p); }
__device__ __forceinline__ void st(u8 *p, u32x4 v) { __builtin_nontemporal_store(v, (u32x4 *)p); }

__device__ __forceinline__ u32 xcd_tile(u32 b, u32 n)
{
    const u32 q = n / 8, r = n % 8, x = b % 8;
    return x * q + min(x, r) + b / 8;
}

// byte offset of lane's u-th 16 B within a tile of U * 4 KiB
template <int U, bool WC>
__device__ __forceinline__ u32 lane_off(u32 u)
{
    if constexpr (WC)  // wave w owns [w * 1 KiB * U, (w + 1) * 1 KiB * U)
        return (threadIdx.x / 64) * 1024u * U + u * 1024u + (threadIdx.x % 64) * 16u;
    else  // workgroup interleave: u-step = 4 KiB
        return u * 4096u + threadIdx.x * 16u;
}

template <int U, bool XCD>
__global__ __launch_bounds__(256) void w_tile(u8 *out)
{
    const u32 t = XCD ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x;
    const u32x4 v = {1u, 2u, 3u, t};
    u8 *o = out + (size_t)t * 4096 * U;
#pragma unroll
    for (int u = 0; u < U; ++u)
        st(o + lane_off<U, false>(u), v);
}

constexpr size_t CH = 1u << 20, BB = CH / 4;

template <int U, bool WC>
__device__ __forceinline__ void enc_tile(const u8 *in, u8 *par, u32 tile)
{
    constexpr u32 per = BB / (4096 * U);  // tiles per chunk
    const u32 chunk = tile / per, t0 = (tile % per) * 4096 * U;
    const u8 *src = in + (size_t)chunk * CH + t0;
    u8 *dst = par + (size_t)chunk * 2 * BB + t0;
    u32x4 a0[U], a1[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        a0[u] = a1[u] = u32x4{0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u32x4 x = ld(src + j * BB + lane_off<U, WC>(u));
            a0[u] ^= x;
            a1[u] ^= (x << 1);
        }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        st(dst + lane_off<U, WC>(u), a0[u]);
        st(dst + BB + lane_off<U, WC>(u), a1[u]);
    }
}

template <int U, bool WC, bool XCD>
__global__ __launch_bounds__(256) void e_tile(const u8 *__restrict__ in, u8 *__restrict__ par)
{
    enc_tile<U, WC>(in, par, XCD ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x);
}

// persistent: workgroup g handles tiles g, g + G, g + 2G, ...
template <int U>
__global__ __launch_bounds__(256) void e_pers(const u8 *__restrict__ in, u8 *__restrict__ par, u32 ntiles)
{
    for (u32 t = blockIdx.x; t < ntiles; t += gridDim.x)
        enc_tile<U, false>(in, par, t);
}

template <int U, bool XCD>
__global__ __launch_bounds__(256) void d_tile(const u8 *__restrict__ in, const u8 *__restrict__ par, u8 *__restrict__ out)
{
    constexpr u32 per = BB / (4096 * U);
    const u32 tile = XCD ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x;
    const u32 chunk = tile / per, t0 = (tile % per) * 4096 * U;
    const u8 *d = in + (size_t)chunk * CH + t0;
    const u8 *p = par + (size_t)chunk * 2 * BB + t0;
    u8 *w = out + (size_t)chunk * CH + t0;
    u32x4 x0[U], x2[U], x4[U], x5[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const u32 o = lane_off<U, false>(u);
        x0[u] = ld(d + o);
        x2[u] = ld(d + 2 * BB + o);
        x4[u] = ld(p + o);
        x5[u] = ld(p + BB + o);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const u32 o = lane_off<U, false>(u);
        st(w + o, x0[u]);
        st(w + 2 * BB + o, x2[u]);
        st(w + BB + o, x0[u] ^ x4[u] ^ x5[u]);
        st(w + 3 * BB + o, x2[u] ^ x4[u] ^ (x5[u] << 1));
    }
}

template <class F>
double time_ms(F launch)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 3; ++i)
        launch();
    std::vector<float> t;
    for (int i = 0; i < 15; ++i) {
        (void)hipEventRecord(a);
        launch();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        t.push_back(ms);
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main()
{
    const size_t G = 1ull << 30, W = G + G / 2;
    u8 *a, *b, *c;
    CK(hipMalloc(&a, G));
    CK(hipMalloc(&b, G / 2));
    CK(hipMalloc(&c, W));
    CK(hipMemset(a, 7, G));
    CK(hipMemset(b, 1, G / 2));
    CK(hipMemset(c, 3, W));
    auto rate = [&](double bytes, double ms) { return bytes / (ms * 1e-3) / 1e9; };
#define WT(U, X) rate(W, time_ms([&] { hipLaunchKernelGGL((w_tile<U, X>), dim3(W / (4096 * U)), dim3(256), 0, 0, c); }))
    printf("{\"w_U1\": %.1f, \"w_U2\": %.1f, \"w_U4\": %.1f, \"w_U8\": %.1f, \"w_U16\": %.1f, \"w_U4_xcd\": %.1f, "
           "\"w_U8_xcd\": %.1f, \"w_U16_xcd\": %.1f}\n",
           WT(1, false), WT(2, false), WT(4, false), WT(8, false), WT(16, false), WT(4, true), WT(8, true),
           WT(16, true));
    fflush(stdout);
    const double EB = 1.5 * G;  // encode: 1 GiB read + 0.5 GiB written
#define ET(U, WC, X) rate(EB, time_ms([&] { hipLaunchKernelGGL((e_tile<U, WC, X>), dim3(G / (4096 * 4 * U)), dim3(256), 0, 0, a, b); }))
#define EP(U, NG) rate(EB, time_ms([&] { hipLaunchKernelGGL((e_pers<U>), dim3(NG), dim3(256), 0, 0, a, b, (u32)(G / (4096 * 4 * U))); }))
    printf("{\"e_U1\": %.1f, \"e_U2\": %.1f, \"e_U4\": %.1f, \"e_U8\": %.1f, \"e_U4_wc\": %.1f, \"e_U8_wc\": %.1f, "
           "\"e_U4_xcd\": %.1f, \"e_U8_xcd\": %.1f, \"e_U4_pers1024\": %.1f, \"e_U4_pers2048\": %.1f, "
           "\"e_U2_pers2048\": %.1f}\n",
           ET(1, false, false), ET(2, false, false), ET(4, false, false), ET(8, false, false), ET(4, true, false),
           ET(8, true, false), ET(4, false, true), ET(8, false, true), EP(4, 1024), EP(4, 2048), EP(2, 2048));
    fflush(stdout);
    const double DB = 2.0 * G;  // decode: 1 GiB read + 1 GiB written
#define DT(U, X) rate(DB, time_ms([&] { hipLaunchKernelGGL((d_tile<U, X>), dim3(G / (4096 * 4 * U)), dim3(256), 0, 0, a, b, c); }))
    printf("{\"d_U1\": %.1f, \"d_U2\": %.1f, \"d_U4\": %.1f, \"d_U8\": %.1f, \"d_U1_xcd\": %.1f, \"d_U2_xcd\": %.1f, "
           "\"d_U4_xcd\": %.1f, \"d_U8_xcd\": %.1f}\n",
           DT(1, false), DT(2, false), DT(4, false), DT(8, false), DT(1, true), DT(2, true), DT(4, true), DT(8, true));
    fflush(stdout);
    CK(hipDeviceSynchronize());
    return 0;
}
