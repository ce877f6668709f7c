// mfma_i8_probe.hip — checks the lane maps of v_mfma_i32_32x32x32_i8 on gfx950 with exact
// integer data (cdna_hip_programming.md: "Other dtypes: check the map with exact integer data").
// Not product code.  Hypothesis (the bf16 32x32x16 map with 16 elements per lane):
//   lane l, r = l & 31, h = l >> 5, element j = 0..15 of the 16-byte operand:
//     A[row r][k = 16h + j],  B[k = 16h + j][col r]
//   D (16 x i32 per lane): col = l & 31, row = (reg & 3) + 8 * (reg >> 2) + 4h
// Prints "ok" when D equals the host product under that map, else the first mismatches.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

__host__ __device__ inline int aval(int row, int k) { return ((row * 7 + k * 3) % 11) - 5; }
__host__ __device__ inline int bval(int k, int col) { return ((k * 5 + col * 2 + 1) % 13) - 6; }

__global__ void probe(int *out)
{
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    unsigned a[4], b[4];
    for (int v = 0; v < 4; ++v) {
        unsigned x = 0, y = 0;
        for (int e = 0; e < 4; ++e) {
            const int j = 4 * v + e;
            x |= (unsigned)(aval(r, 16 * h + j) & 0xFF) << (8 * e);
            y |= (unsigned)(bval(16 * h + j, r) & 0xFF) << (8 * e);
        }
        a[v] = x;
        b[v] = y;
    }
    const i32x4 A = {(int)a[0], (int)a[1], (int)a[2], (int)a[3]};
    const i32x4 B = {(int)b[0], (int)b[1], (int)b[2], (int)b[3]};
    i32x16 c = {};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, B, c, 0, 0, 0);
    for (int reg = 0; reg < 16; ++reg)
        out[l * 16 + reg] = c[reg];
}

int main()
{
    int *d;
    (void)hipMalloc(&d, 64 * 16 * sizeof(int));
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    int h[64 * 16];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int reg = 0; reg < 16; ++reg) {
            const int col = l & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (l >> 5);
            int want = 0;
            for (int k = 0; k < 32; ++k)
                want += aval(row, k) * bval(k, col);
            if (want != h[l * 16 + reg] && bad++ < 8)
                printf("lane %d reg %d: got %d want %d\n", l, reg, h[l * 16 + reg], want);
        }
    printf(bad ? "mismatches: %d\n" : "ok\n", bad);
    return bad != 0;
}
