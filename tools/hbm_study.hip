// hbm_study.hip — what store / load shapes reach the most HBM bandwidth on MI355X.
//
// Not product code: a calibration tool.  The encode and decode kernels sit at about the
// harmonic mean of the read ceiling and the write ceiling tools/stream_ceiling.hip measured
// (6.4 / 4.8 TB/s), so the write side is the lever.  This prints one JSON object per line,
// GB/s = bytes moved / kernel time (HIP events, median of 15 after 3 warm-ups), for:
//   w_*   1.5 GiB of stores in several shapes and cache policies
//   r_*   1.5 GiB of loads
//   c_*   1 GiB -> 1 GiB copies
//   e_*   the RS(4,2) encode pattern (1024 x 1 MiB chunks; 4 blocks read, 2 written; XOR in
//         place of the GF arithmetic) with the store shapes / workgroup orders that matter
// Shapes: "gs" = grid-stride over the whole buffer with 2048 workgroups; "tile" = one 256-lane
// workgroup per 16 KiB (4 u-steps of 4 KiB, as sec_encode_kernel<2,4>); "xcd" = tile order
// remapped so each XCD (workgroup id mod 8) walks one contiguous eighth of the buffer.
// Policies: plain, nt (__builtin_nontemporal_*), and inline-asm stores with sc0/sc1/nt bits.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef unsigned int u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                         \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

enum Pol { PLAIN = 0, NT = 1, SC01 = 2, NTSC1 = 3, SC1 = 4, NTSC01 = 5 };

template <int P>
__device__ __forceinline__ void st(void *p, u32x4 v)
{
    if constexpr (P == PLAIN)
        *(u32x4 *)p = v;
    else if constexpr (P == NT)
        __builtin_nontemporal_store(v, (u32x4 *)p);
    else if constexpr (P == SC01)
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (P == NTSC1)
        asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (P == SC1)
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else
        asm volatile("global_store_dwordx4 %0, %1, off nt sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

template <int P>
__device__ __forceinline__ u32x4 ld(const void *p)
{
    if constexpr (P == NT)
        return __builtin_nontemporal_load((const u32x4 *)p);
    else
        return *(const u32x4 *)p;
}

// tile index of this workgroup: identity, or XCD-contiguous (tiles of XCD x = one eighth)
template <bool XCD>
__device__ __forceinline__ u32 tile_id()
{
    if constexpr (!XCD)
        return blockIdx.x;
    const u32 per = gridDim.x / 8;  // grid is a multiple of 8
    return (blockIdx.x % 8) * per + blockIdx.x / 8;
}

// ---- writes ------------------------------------------------------------------
template <int P>
__global__ __launch_bounds__(256) void w_gs(unsigned char *out, size_t n16)
{
    const u32x4 v = {1u, 2u, 3u, blockIdx.x};
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
        st<P>(out + i * 16, v);
}

// one workgroup per 16 KiB: lane writes 16 B at t + 4096*u
template <int P, bool XCD>
__global__ __launch_bounds__(256) void w_tile(unsigned char *out)
{
    const u32x4 v = {1u, 2u, 3u, blockIdx.x};
    unsigned char *o = out + (size_t)tile_id<XCD>() * 16384 + threadIdx.x * 16;
#pragma unroll
    for (int u = 0; u < 4; ++u)
        st<P>(o + u * 4096, v);
}

// one dword per lane (256 B per wave instruction), grid-stride
__global__ __launch_bounds__(256) void w_gs_dword(u32 *out, size_t n4)
{
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
        __builtin_nontemporal_store((u32)i, out + i);
}

// ---- reads -------------------------------------------------------------------
template <int P>
__global__ __launch_bounds__(256) void r_gs(const unsigned char *in, u32x4 *sink, size_t n16)
{
    u32x4 a = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
        a ^= ld<P>(in + i * 16);
    if ((a.x ^ a.y ^ a.z ^ a.w) == 0x12345678u)
        sink[blockIdx.x] = a;
}

template <int P, bool XCD>
__global__ __launch_bounds__(256) void r_tile(const unsigned char *in, u32x4 *sink)
{
    const unsigned char *p = in + (size_t)tile_id<XCD>() * 16384 + threadIdx.x * 16;
    u32x4 a = {0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 4; ++u)
        a ^= ld<P>(p + u * 4096);
    if ((a.x ^ a.y ^ a.z ^ a.w) == 0x12345678u)
        sink[blockIdx.x] = a;
}

// ---- copies ------------------------------------------------------------------
template <int LP, int SP>
__global__ __launch_bounds__(256) void c_gs(const unsigned char *in, unsigned char *out, size_t n16)
{
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
        st<SP>(out + i * 16, ld<LP>(in + i * 16));
}

template <int LP, int SP, bool XCD>
__global__ __launch_bounds__(256) void c_tile(const unsigned char *in, unsigned char *out)
{
    const size_t o = (size_t)tile_id<XCD>() * 16384 + threadIdx.x * 16;
    u32x4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
        x[u] = ld<LP>(in + o + u * 4096);
#pragma unroll
    for (int u = 0; u < 4; ++u)
        st<SP>(out + o + u * 4096, x[u]);
}

// ---- RS(4,2) encode pattern ------------------------------------------------------
template <int SP, bool XCD>
__global__ __launch_bounds__(256) void e_rs42(const unsigned char *__restrict__ in, unsigned char *__restrict__ par)
{
    const u32 tid = tile_id<XCD>();
    const u32 chunk = tid >> 4, t0 = (tid & 15) * 16384;
    const size_t B = 262144;
    const unsigned char *src = in + (size_t)chunk * 1048576 + t0 + threadIdx.x * 16;
    unsigned char *dst = par + (size_t)chunk * 2 * B + t0 + threadIdx.x * 16;
    u32x4 a0[4], a1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
        a0[u] = a1[u] = u32x4{0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const u32x4 x = ld<NT>(src + j * B + u * 4096);
            a0[u] ^= x;
            a1[u] ^= (x << 1);
        }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        st<SP>(dst + u * 4096, a0[u]);
        st<SP>(dst + B + u * 4096, a1[u]);
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
    unsigned char *a, *b;
    u32x4 *sink;
    CK(hipMalloc(&a, 2 * G));
    CK(hipMalloc(&b, 2 * G));
    CK(hipMalloc(&sink, 1 << 22));
    CK(hipMemset(a, 7, 2 * G));
    CK(hipMemset(b, 1, 2 * G));
    const int gs = 2048;
    const u32 tiles_w = (u32)(W / 16384), tiles_c = (u32)(G / 16384);
    const double gb = 1e9;
    auto rate = [&](double bytes, double ms) { return bytes / (ms * 1e-3) / gb; };

    // writes
    printf("{\"w_gs_plain\": %.1f, \"w_gs_nt\": %.1f, \"w_gs_sc01\": %.1f, \"w_gs_ntsc1\": %.1f, \"w_gs_sc1\": %.1f, "
           "\"w_gs_ntsc01\": %.1f}\n",
           rate(W, time_ms([&] { hipLaunchKernelGGL(w_gs<PLAIN>, dim3(gs), dim3(256), 0, 0, b, W / 16); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL(w_gs<NT>, dim3(gs), dim3(256), 0, 0, b, W / 16); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL(w_gs<SC01>, dim3(gs), dim3(256), 0, 0, b, W / 16); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL(w_gs<NTSC1>, dim3(gs), dim3(256), 0, 0, b, W / 16); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL(w_gs<SC1>, dim3(gs), dim3(256), 0, 0, b, W / 16); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL(w_gs<NTSC01>, dim3(gs), dim3(256), 0, 0, b, W / 16); })));
    fflush(stdout);
    printf("{\"w_tile_plain\": %.1f, \"w_tile_nt\": %.1f, \"w_tile_nt_xcd\": %.1f, \"w_tile_plain_xcd\": %.1f, "
           "\"w_tile_ntsc1\": %.1f, \"w_tile_sc01\": %.1f, \"w_gs_dword_nt\": %.1f, \"memset\": %.1f, "
           "\"w_gs_nt_grid8192\": %.1f, \"w_gs_nt_grid1024\": %.1f}\n",
           rate(W, time_ms([&] { hipLaunchKernelGGL((w_tile<PLAIN, false>), dim3(tiles_w), dim3(256), 0, 0, b); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL((w_tile<NT, false>), dim3(tiles_w), dim3(256), 0, 0, b); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL((w_tile<NT, true>), dim3(tiles_w), dim3(256), 0, 0, b); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL((w_tile<PLAIN, true>), dim3(tiles_w), dim3(256), 0, 0, b); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL((w_tile<NTSC1, false>), dim3(tiles_w), dim3(256), 0, 0, b); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL((w_tile<SC01, false>), dim3(tiles_w), dim3(256), 0, 0, b); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL(w_gs_dword, dim3(gs), dim3(256), 0, 0, (u32 *)b, W / 4); })),
           rate(W, time_ms([&] { (void)hipMemsetD32Async((hipDeviceptr_t)b, 0x01020304u, W / 4, 0); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL(w_gs<NT>, dim3(8192), dim3(256), 0, 0, b, W / 16); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL(w_gs<NT>, dim3(1024), dim3(256), 0, 0, b, W / 16); })));
    fflush(stdout);
    // reads
    printf("{\"r_gs_plain\": %.1f, \"r_gs_nt\": %.1f, \"r_tile_plain\": %.1f, \"r_tile_nt\": %.1f, "
           "\"r_tile_nt_xcd\": %.1f}\n",
           rate(W, time_ms([&] { hipLaunchKernelGGL(r_gs<PLAIN>, dim3(gs), dim3(256), 0, 0, a, sink, W / 16); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL(r_gs<NT>, dim3(gs), dim3(256), 0, 0, a, sink, W / 16); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL((r_tile<PLAIN, false>), dim3(tiles_w), dim3(256), 0, 0, a, sink); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL((r_tile<NT, false>), dim3(tiles_w), dim3(256), 0, 0, a, sink); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL((r_tile<NT, true>), dim3(tiles_w), dim3(256), 0, 0, a, sink); })));
    fflush(stdout);
    // copies
    printf("{\"c_gs_plain\": %.1f, \"c_gs_nt\": %.1f, \"c_tile_plain\": %.1f, \"c_tile_nt\": %.1f, "
           "\"c_tile_nt_xcd\": %.1f, \"c_tile_ntld_sc01\": %.1f, \"c_tile_ntld_ntsc1\": %.1f, \"hipMemcpyD2D\": %.1f}\n",
           rate(2.0 * G, time_ms([&] { hipLaunchKernelGGL((c_gs<PLAIN, PLAIN>), dim3(gs), dim3(256), 0, 0, a, b, G / 16); })),
           rate(2.0 * G, time_ms([&] { hipLaunchKernelGGL((c_gs<NT, NT>), dim3(gs), dim3(256), 0, 0, a, b, G / 16); })),
           rate(2.0 * G, time_ms([&] { hipLaunchKernelGGL((c_tile<PLAIN, PLAIN, false>), dim3(tiles_c), dim3(256), 0, 0, a, b); })),
           rate(2.0 * G, time_ms([&] { hipLaunchKernelGGL((c_tile<NT, NT, false>), dim3(tiles_c), dim3(256), 0, 0, a, b); })),
           rate(2.0 * G, time_ms([&] { hipLaunchKernelGGL((c_tile<NT, NT, true>), dim3(tiles_c), dim3(256), 0, 0, a, b); })),
           rate(2.0 * G, time_ms([&] { hipLaunchKernelGGL((c_tile<NT, SC01, false>), dim3(tiles_c), dim3(256), 0, 0, a, b); })),
           rate(2.0 * G, time_ms([&] { hipLaunchKernelGGL((c_tile<NT, NTSC1, false>), dim3(tiles_c), dim3(256), 0, 0, a, b); })),
           rate(2.0 * G, time_ms([&] { (void)hipMemcpyAsync(b, a, G, hipMemcpyDeviceToDevice, 0); })));
    fflush(stdout);
    // encode pattern
    const u32 et = 1024 * 16;
    printf("{\"e_nt\": %.1f, \"e_nt_xcd\": %.1f, \"e_plain\": %.1f, \"e_sc01\": %.1f, \"e_ntsc1\": %.1f, "
           "\"e_sc1\": %.1f, \"e_ntsc01\": %.1f}\n",
           rate(W, time_ms([&] { hipLaunchKernelGGL((e_rs42<NT, false>), dim3(et), dim3(256), 0, 0, a, b); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL((e_rs42<NT, true>), dim3(et), dim3(256), 0, 0, a, b); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL((e_rs42<PLAIN, false>), dim3(et), dim3(256), 0, 0, a, b); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL((e_rs42<SC01, false>), dim3(et), dim3(256), 0, 0, a, b); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL((e_rs42<NTSC1, false>), dim3(et), dim3(256), 0, 0, a, b); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL((e_rs42<SC1, false>), dim3(et), dim3(256), 0, 0, a, b); })),
           rate(W, time_ms([&] { hipLaunchKernelGGL((e_rs42<NTSC01, false>), dim3(et), dim3(256), 0, 0, a, b); })));
    fflush(stdout);
    CK(hipDeviceSynchronize());
    return 0;
}
