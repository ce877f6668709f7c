// stream_ceiling.hip — measured HBM ceilings for the access pattern of the RS kernels.
//
// Not product code: a calibration tool for DESIGN.md's roofline.  Prints one JSON line with
// GB/s (algorithmic bytes / kernel time, HIP events, median of 20 after 3 warm-ups) for:
//   copy      uint4 grid-stride copy, 1 GiB -> 1 GiB
//   read      uint4 grid-stride XOR-reduce of 1.5 GiB (one store per workgroup)
//   write     uint4 grid-stride fill of 1.5 GiB
//   rs42_xor  the encode kernel's exact pattern for 1024 x 1 MiB RS(4,2) chunks (4 coalesced
//             block streams read, 2 written, 16 KiB positions per 256-lane workgroup) with
//             the GF arithmetic replaced by XOR: the practical roof for sec_encode_kernel
//   rs42_xor_nt  the same with nontemporal loads and stores
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

__global__ __launch_bounds__(256) void k_copy(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        out[i] = in[i];
}

__global__ __launch_bounds__(256) void k_read(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, size_t n)
{
    u32x4 a = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        a ^= in[i];
    if ((a.x ^ a.y ^ a.z ^ a.w) == 0x12345678u)
        out[blockIdx.x] = a;
}

__global__ __launch_bounds__(256) void k_write(u32x4 *__restrict__ out, size_t n)
{
    const u32x4 v = {1, 2, 3, 4};
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        out[i] = v;
}

template <bool NT>
__global__ __launch_bounds__(256) void k_rs42(const unsigned char *__restrict__ in, unsigned char *__restrict__ par)
{
    // 16 tiles of 16 KiB positions per 1 MiB chunk (B = 256 KiB)
    const u32 chunk = blockIdx.x >> 4, t0 = (blockIdx.x & 15) * 16384;
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
            const u32x4 *p = (const u32x4 *)(src + j * B + u * 4096);
            u32x4 x = NT ? __builtin_nontemporal_load(p) : *p;
            a0[u] ^= x;
            a1[u] ^= (x << 1);
        }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        u32x4 *q0 = (u32x4 *)(dst + u * 4096), *q1 = (u32x4 *)(dst + B + u * 4096);
        if (NT) {
            __builtin_nontemporal_store(a0[u], q0);
            __builtin_nontemporal_store(a1[u], q1);
        } else {
            *q0 = a0[u];
            *q1 = a1[u];
        }
    }
}

typedef u32x4 u32x4_u __attribute__((aligned(1)));

// the encode pattern with every block start shifted by `off` bytes (unaligned 16 B lanes)
// SHIFT: 0 = hardware unaligned dwordx4, 1 = dword-aligned dwordx4 + dword + v_alignbyte
template <int SHIFT>
__global__ __launch_bounds__(256) void k_rs42_mis(const unsigned char *__restrict__ in, unsigned char *__restrict__ par,
                                                  int off, int soff)
{
    const u32 chunk = blockIdx.x >> 4, t0 = (blockIdx.x & 15) * 16384;
    const size_t B = 262144;
    const unsigned char *src = in + (size_t)chunk * 1048576 + t0 + threadIdx.x * 16 + off;
    unsigned char *dst = par + (size_t)chunk * 2 * B + t0 + threadIdx.x * 16 + soff;
    u32x4 a0[4], a1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
        a0[u] = a1[u] = u32x4{0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const unsigned char *p = src + j * B + u * 4096;
            u32x4 x;
            if (SHIFT == 0) {
                x = __builtin_nontemporal_load((const u32x4_u *)p);
            } else {
                const unsigned r = (unsigned)((size_t)p & 3);
                const u32 *q = (const u32 *)(p - r);
                u32x4 w = __builtin_nontemporal_load((const u32x4 __attribute__((aligned(4))) *)q);
                u32 e = __builtin_nontemporal_load(q + 4);
                x.x = __builtin_amdgcn_alignbyte(w.y, w.x, r);
                x.y = __builtin_amdgcn_alignbyte(w.z, w.y, r);
                x.z = __builtin_amdgcn_alignbyte(w.w, w.z, r);
                x.w = __builtin_amdgcn_alignbyte(e, w.w, r);
            }
            a0[u] ^= x;
            a1[u] ^= (x << 1);
        }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        __builtin_nontemporal_store(a0[u], (u32x4_u *)(dst + u * 4096));
        __builtin_nontemporal_store(a1[u], (u32x4_u *)(dst + B + u * 4096));
    }
}

__global__ __launch_bounds__(256) void k_copy_nt(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        __builtin_nontemporal_store(__builtin_nontemporal_load(in + i), out + i);
}

// the decode kernel's pattern for 1024 x 1 MiB RS(4,2) with data {1,3} erased: read data
// blocks {0,2} (chunk buffer) and parity {4,5} (parity buffer), write the 4 rows of the
// reassembled chunk (copies + XOR in place of GF), nontemporal
__global__ __launch_bounds__(256) void k_dec42(const unsigned char *__restrict__ in, const unsigned char *__restrict__ par,
                                               unsigned char *__restrict__ out)
{
    const u32 chunk = blockIdx.x >> 4, t0 = (blockIdx.x & 15) * 16384;
    const size_t B = 262144;
    const size_t o = t0 + threadIdx.x * 16;
    const unsigned char *d = in + (size_t)chunk * 1048576 + o;
    const unsigned char *p = par + (size_t)chunk * 2 * B + o;
    unsigned char *w = out + (size_t)chunk * 1048576 + o;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const u32x4 x0 = __builtin_nontemporal_load((const u32x4 *)(d + u * 4096));
        const u32x4 x2 = __builtin_nontemporal_load((const u32x4 *)(d + 2 * B + u * 4096));
        const u32x4 x4 = __builtin_nontemporal_load((const u32x4 *)(p + u * 4096));
        const u32x4 x5 = __builtin_nontemporal_load((const u32x4 *)(p + B + u * 4096));
        __builtin_nontemporal_store(x0, (u32x4 *)(w + u * 4096));
        __builtin_nontemporal_store(x2, (u32x4 *)(w + 2 * B + u * 4096));
        __builtin_nontemporal_store(x0 ^ x4 ^ x5, (u32x4 *)(w + B + u * 4096));
        __builtin_nontemporal_store(x2 ^ x4 ^ (x5 << 1), (u32x4 *)(w + 3 * B + u * 4096));
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
    for (int i = 0; i < 20; ++i) {
        (void)hipEventRecord(a);
        launch();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main()
{
    const size_t G = 1ull << 30;
    unsigned char *a, *b;
    CK(hipMalloc(&a, 2 * G));
    CK(hipMalloc(&b, 2 * G));
    CK(hipMemset(a, 7, 2 * G));
    CK(hipMemset(b, 1, 2 * G));
    const int grid = 256 * 8;
    double ms_copy = time_ms([&] { hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, (u32x4 *)a, (u32x4 *)b, G / 16); });
    double ms_read = time_ms([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, (u32x4 *)a, (u32x4 *)b, (G + G / 2) / 16); });
    double ms_write = time_ms([&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, (u32x4 *)b, (G + G / 2) / 16); });
    double ms_rs = time_ms([&] { hipLaunchKernelGGL(k_rs42<false>, dim3(1024 * 16), dim3(256), 0, 0, a, b); });
    double ms_rsnt = time_ms([&] { hipLaunchKernelGGL(k_rs42<true>, dim3(1024 * 16), dim3(256), 0, 0, a, b); });
    double mis[6];
    const int offs[6][3] = {{2, 0, 0}, {4, 0, 0}, {8, 0, 0}, {2, 0, 1}, {0, 2, 0}, {0, 4, 0}};
    for (int i = 0; i < 6; ++i) {
        const int o = offs[i][0], so = offs[i][1];
        if (offs[i][2])
            mis[i] = time_ms([&] { hipLaunchKernelGGL(k_rs42_mis<1>, dim3(1024 * 16), dim3(256), 0, 0, a, b, o, so); });
        else
            mis[i] = time_ms([&] { hipLaunchKernelGGL(k_rs42_mis<0>, dim3(1024 * 16), dim3(256), 0, 0, a, b, o, so); });
    }
    const double ms_copy_nt = time_ms([&] { hipLaunchKernelGGL(k_copy_nt, dim3(grid), dim3(256), 0, 0, (u32x4 *)a, (u32x4 *)b, G / 16); });
    const double ms_dec = time_ms([&] { hipLaunchKernelGGL(k_dec42, dim3(1024 * 16), dim3(256), 0, 0, a, a + G, b); });
    CK(hipDeviceSynchronize());
    const double gb = 1e9;
    printf("{\"copy_nt_GBs\": %.1f, \"dec42_xor_nt_GBs\": %.1f}\n", 2.0 * G / (ms_copy_nt * 1e-3) / gb,
           2.0 * G / (ms_dec * 1e-3) / gb);
    printf("{\"rs42_nt_read_off2_GBs\": %.1f, \"read_off4_GBs\": %.1f, \"read_off8_GBs\": %.1f, "
           "\"read_off2_alignbyte_GBs\": %.1f, \"write_off2_GBs\": %.1f, \"write_off4_GBs\": %.1f}\n",
           1.5 * G / (mis[0] * 1e-3) / gb, 1.5 * G / (mis[1] * 1e-3) / gb, 1.5 * G / (mis[2] * 1e-3) / gb,
           1.5 * G / (mis[3] * 1e-3) / gb, 1.5 * G / (mis[4] * 1e-3) / gb, 1.5 * G / (mis[5] * 1e-3) / gb);
    printf("{\"copy_GBs\": %.1f, \"read_GBs\": %.1f, \"write_GBs\": %.1f, \"rs42_xor_GBs\": %.1f, "
           "\"rs42_xor_nt_GBs\": %.1f, \"rs42_xor_ms\": %.4f}\n",
           2.0 * G / (ms_copy * 1e-3) / gb, 1.5 * G / (ms_read * 1e-3) / gb, 1.5 * G / (ms_write * 1e-3) / gb,
           1.5 * G / (ms_rs * 1e-3) / gb, 1.5 * G / (ms_rsnt * 1e-3) / gb, ms_rs);
    return 0;
}
