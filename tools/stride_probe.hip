// stride_probe.hip — HBM read rate of S concurrent streams whose addresses differ by a fixed
// distance D, the way a decode tile reads several blocks of one chunk at the same offset.
// Not product code.  Question it answers: do blocks 512 KiB apart (C3's {1,3} erasure: data
// blocks 0 and 2 of a 1 MiB chunk read together) cost more than blocks 256 KiB apart?
//
// Layout: chunks of CH bytes back to back over 1 GiB; a workgroup of 256 lanes reads 4 KiB at
// offset t of S streams chunk + t + s * D (s < S), 16 B per lane, nontemporal, XOR-reduced.
// Also: the same S streams with a write of each stream to a second buffer (a 1:1 copy of S
// rows), which is the reassembling decode's mix.  20 launches per timing, median of 7.
// Prints one JSON object per (S, D): read GB/s and copy GB/s; first, hipMemcpyAsync's own
// device-to-device rate over the same 1 GiB (read + write bytes).
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef unsigned int u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned char u8;

__device__ __forceinline__ u32x4 ld(const u8 *p) { return __builtin_nontemporal_load((const u32x4 *)p); }
__device__ __forceinline__ void st(u8 *p, u32x4 v) { __builtin_nontemporal_store(v, (u32x4 *)p); }

constexpr size_t G = 1ull << 30;

template <int S>
__global__ __launch_bounds__(256) void k_read(const u8 *__restrict__ in, u32 *__restrict__ sink, size_t ch, size_t d,
                                              u32 per)
{
    const size_t chunk = blockIdx.x / per, t = (size_t)(blockIdx.x % per) * 4096 + threadIdx.x * 16;
    const u8 *p = in + chunk * ch + t;
    u32x4 a = {0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < S; ++s)
        a ^= ld(p + s * d);
    const u32 v = a.x ^ a.y ^ a.z ^ a.w;
    if (v == 0x12345678u)
        sink[blockIdx.x] = v;
}

template <int S>
__global__ __launch_bounds__(256) void k_copy(const u8 *__restrict__ in, u8 *__restrict__ out, size_t ch, size_t d,
                                              u32 per)
{
    const size_t chunk = blockIdx.x / per, t = (size_t)(blockIdx.x % per) * 4096 + threadIdx.x * 16;
    const size_t o = chunk * ch + t;
    u32x4 x[S];
#pragma unroll
    for (int s = 0; s < S; ++s)
        x[s] = ld(in + o + s * d);
#pragma unroll
    for (int s = 0; s < S; ++s)
        st(out + o + s * d, x[s]);
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

template <int S>
void run(const u8 *a, u8 *c, u32 *sink, size_t d)
{
    // a chunk holds S streams of `d` bytes (the blocks) ; the tiles cover the first d bytes of
    // each stream, so every byte of the buffer is read once
    const size_t ch = S * d, nch = G / ch;
    const u32 per = (u32)(d / 4096);
    const dim3 grid((u32)(nch * per)), blk(256);
    const double bytes = (double)nch * ch;
    const double rd = bytes / (time_ms([&] { hipLaunchKernelGGL(k_read<S>, grid, blk, 0, 0, a, sink, ch, d, per); }) * 1e-3) / 1e9;
    const double cp = 2 * bytes / (time_ms([&] { hipLaunchKernelGGL(k_copy<S>, grid, blk, 0, 0, a, c, ch, d, per); }) * 1e-3) / 1e9;
    printf("{\"streams\": %d, \"distance_KiB\": %zu, \"read_GBs\": %.1f, \"copy_GBs\": %.1f}\n", S, d >> 10, rd, cp);
    fflush(stdout);
}

int main()
{
    u8 *a, *c;
    u32 *sink;
    if (hipMalloc(&a, G) != hipSuccess || hipMalloc(&c, G) != hipSuccess || hipMalloc(&sink, G / 4096 * 4) != hipSuccess)
        return 1;
    (void)hipMemset(a, 7, G);
    (void)hipMemset(c, 3, G);
    {  // the runtime's own device-to-device copy (its blit kernel), for reference
        const double ms = time_ms([&] { (void)hipMemcpyAsync(c, a, G, hipMemcpyDeviceToDevice, 0); });
        printf("{\"hipMemcpyAsync_d2d_1GiB_GBs\": %.1f}\n", 2.0 * G / (ms * 1e-3) / 1e9);
        fflush(stdout);
    }
    const size_t K = 1024;
    for (size_t d : {64 * K, 128 * K, 256 * K, 384 * K, 512 * K, 640 * K, 1024 * K, 2048 * K}) {
        run<1>(a, c, sink, d);
        run<2>(a, c, sink, d);
        run<4>(a, c, sink, d);
    }
    return hipDeviceSynchronize() != hipSuccess;
}
