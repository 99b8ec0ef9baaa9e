// Operand / result lane layout of v_mfma_f32_16x16x32_f16 and v_mfma_f32_16x16x16_f16 on gfx950,
// as the 16x16 sweep (st_kmeans_nd.hip) assumes it:
//   A: lane l holds A[m = l & 15][k = KW*(l >> 4) + e], e < KW (KW = 8 for x32, 4 for x16)
//   B: lane l holds B[k = KW*(l >> 4) + e][n = l & 15]
//   D: lane l holds D[m = 4*(l >> 4) + i][n = l & 15], i < 4
// Integer-valued operands: every product and sum is exact, so the check is bitwise.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k(const _Float16 *A, const _Float16 *B, float *out) {
    // A: 16 x 48 row-major, B: 48 x 16 row-major; K = 32 (x32) + 16 (x16)
    const int l = threadIdx.x, n = l & 15, q = l >> 4;
    f16x8 a8, b8;
    f16x4 a4, b4;
    for (int e = 0; e < 8; ++e) {
        a8[e] = A[n * 48 + 8 * q + e];
        b8[e] = B[(8 * q + e) * 16 + n];
    }
    for (int e = 0; e < 4; ++e) {
        a4[e] = A[n * 48 + 32 + 4 * q + e];
        b4[e] = B[(32 + 4 * q + e) * 16 + n];
    }
    f32x4 acc = {};
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, acc, 0, 0, 0);
    for (int i = 0; i < 4; ++i) out[(4 * q + i) * 16 + n] = acc[i];
}

int main() {
    _Float16 a[16 * 48], b[48 * 16];
    float Af[16][48], Bf[48][16];
    for (int i = 0; i < 16; ++i)
        for (int kk = 0; kk < 48; ++kk) { Af[i][kk] = (float)((i * 7 + kk * 3) % 13 - 6); a[i * 48 + kk] = (_Float16)Af[i][kk]; }
    for (int kk = 0; kk < 48; ++kk)
        for (int j = 0; j < 16; ++j) { Bf[kk][j] = (float)((kk * 5 + j * 11) % 9 - 4); b[kk * 16 + j] = (_Float16)Bf[kk][j]; }
    _Float16 *dA, *dB; float *dO;
    (void)hipMalloc(&dA, sizeof a); (void)hipMalloc(&dB, sizeof b); (void)hipMalloc(&dO, 256 * 4);
    (void)hipMemcpy(dA, a, sizeof a, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, b, sizeof b, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dO);
    float o[256];
    (void)hipMemcpy(o, dO, sizeof o, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            float s = 0;
            for (int kk = 0; kk < 48; ++kk) s += Af[i][kk] * Bf[kk][j];
            if (s != o[i * 16 + j]) ++bad;
        }
    printf("16x16x32 + 16x16x16 layout: %s (%d mismatches of 256)\n", bad ? "MISMATCH" : "ok", bad);
    return bad != 0;
}
