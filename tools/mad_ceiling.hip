// mad_ceiling.hip — measured integer-multiply ceilings of an MI355X, the roofline of the
// APDP bignum kernels (bignum.hip), whose work is 32x32->64-bit multiply-adds.
//
// Not product code: a calibration tool for DESIGN.md.  Prints one JSON line with the
// sustained rate (lane-operations per second; HIP events, median of 10 after 2 warm-ups,
// 8192 workgroups x 256 lanes, 8 independent chains per lane) of:
//   mad_u64_u32   v_mad_u64_u32 (acc64 = a * b + acc64)
//   mul_lo_u32    v_mul_lo_u32 (+ one v_xor per mul, to defeat strength reduction)
//   add_u32       v_add_u32 (a plain full-rate VALU op, for scale)
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef unsigned int u32;
typedef unsigned long long u64;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                         \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

constexpr int kChains = 8;
constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void k_mad(u32 seed, u64 *out)
{
    u64 acc[kChains];
    u32 a[kChains];
    const u32 b = seed ^ threadIdx.x;
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
        acc[c] = c;
        a[c] = seed * (c + 3) + blockIdx.x;
    }
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int c = 0; c < kChains; ++c)
            acc[c] = (u64)(u32)acc[c] * (b ^ a[c]) + acc[c];  // nonlinear: no closed form
    }
    u64 r = 0;
#pragma unroll
    for (int c = 0; c < kChains; ++c)
        r ^= acc[c];
    if (r == 0x123456789ull)
        out[threadIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_mul(u32 seed, u32 *out)
{
    u32 acc[kChains];
    const u32 b = seed ^ threadIdx.x;
#pragma unroll
    for (int c = 0; c < kChains; ++c)
        acc[c] = seed * (c + 3) + blockIdx.x;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int c = 0; c < kChains; ++c)
            acc[c] = (acc[c] * b) ^ (u32)i;  // the xor blocks b^8 strength reduction
    }
    u32 r = 0;
#pragma unroll
    for (int c = 0; c < kChains; ++c)
        r ^= acc[c];
    if (r == 0x12345u)
        out[threadIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_add(u32 seed, u32 *out)
{
    u32 acc[kChains];
    const u32 b = seed ^ threadIdx.x;
#pragma unroll
    for (int c = 0; c < kChains; ++c)
        acc[c] = seed * (c + 3) + blockIdx.x;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int c = 0; c < kChains; ++c)
            acc[c] = (acc[c] + b) ^ (u32)(c + 1);  // the xor keeps the adds from folding into one
    }
    u32 r = 0;
#pragma unroll
    for (int c = 0; c < kChains; ++c)
        r ^= acc[c];
    if (r == 0x12345u)
        out[threadIdx.x] = r;
}

template <class F>
int time_kernel(F launch, double *ms_med)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> v;
    for (int r = 0; r < 12; ++r) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r >= 2)
            v.push_back(ms);
    }
    std::sort(v.begin(), v.end());
    *ms_med = v[v.size() / 2];
    return 0;
}

int main()
{
    const int blocks = 8192;
    u64 *o64;
    u32 *o32;
    CK(hipMalloc(&o64, 256 * sizeof(u64)));
    CK(hipMalloc(&o32, 256 * sizeof(u32)));
    const double ops = (double)blocks * 256 * kChains * kIters;
    double t_mad, t_mul, t_add;
    if (time_kernel([&] { hipLaunchKernelGGL(k_mad, dim3(blocks), dim3(256), 0, 0, 12345u, o64); }, &t_mad) ||
        time_kernel([&] { hipLaunchKernelGGL(k_mul, dim3(blocks), dim3(256), 0, 0, 12345u, o32); }, &t_mul) ||
        time_kernel([&] { hipLaunchKernelGGL(k_add, dim3(blocks), dim3(256), 0, 0, 12345u, o32); }, &t_add))
        return 1;
    CK(hipGetLastError());
    printf("{\"mad_u64_u32_per_s\": %.4g, \"mul_lo_u32_per_s\": %.4g, \"add_u32_per_s\": %.4g, "
           "\"note\": \"lane-ops/s, 8192x256 lanes, 8 independent chains, median of 10\"}\n",
           ops / (t_mad * 1e-3), ops / (t_mul * 1e-3), 2 * ops / (t_add * 1e-3));
    return 0;
}
