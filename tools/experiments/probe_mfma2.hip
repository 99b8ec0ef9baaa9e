// Chained f16 MFMAs with operands bit_cast from uint4 loads, results read through VALU ops.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k(const uint4 *A, const uint4 *B, float *out, float *out2) {
    const int l = threadIdx.x;
    f32x16 acc = {};
    for (int s = 0; s < 3; ++s) {
        const f16x8 a = __builtin_bit_cast(f16x8, A[s * 64 + l]);
        const f16x8 b = __builtin_bit_cast(f16x8, B[s * 64 + l]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    }
    float m1 = __builtin_inff(), m2 = __builtin_inff();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        out[l * 16 + r] = acc[r];
        const float key = __builtin_bit_cast(float, (__builtin_bit_cast(uint32_t, acc[r]) & ~0xFu) | (uint32_t)r);
        m2 = __builtin_amdgcn_fmed3f(m1, m2, key);
        m1 = fminf(m1, key);
    }
    out2[l * 2] = m1;
    out2[l * 2 + 1] = m2;
}

int main() {
    // A[i][k] = (i*3 + k) % 7 - 3, B[k][j] = (k*5 + j) % 11 - 5, K = 48 (3 steps of 16)
    static uint16_t a[3 * 64 * 8], b[3 * 64 * 8];
    float Af[32][48], Bf[48][32];
    for (int i = 0; i < 32; ++i) for (int kk = 0; kk < 48; ++kk) Af[i][kk] = (float)((i * 3 + kk) % 7 - 3);
    for (int kk = 0; kk < 48; ++kk) for (int j = 0; j < 32; ++j) Bf[kk][j] = (float)((kk * 5 + j) % 11 - 5);
    for (int s = 0; s < 3; ++s)
        for (int l = 0; l < 64; ++l)
            for (int e = 0; e < 8; ++e) {
                const int kk = 16 * s + 8 * (l >> 5) + e;
                _Float16 av = (_Float16)Af[l & 31][kk], bv = (_Float16)Bf[kk][l & 31];
                memcpy(&a[(s * 64 + l) * 8 + e], &av, 2);
                memcpy(&b[(s * 64 + l) * 8 + e], &bv, 2);
            }
    uint4 *dA, *dB; float *dO, *dO2;
    (void)hipMalloc(&dA, sizeof a); (void)hipMalloc(&dB, sizeof b);
    (void)hipMalloc(&dO, 64 * 16 * 4); (void)hipMalloc(&dO2, 64 * 2 * 4);
    (void)hipMemcpy(dA, a, sizeof a, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, b, sizeof b, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dO, dO2);
    float o[64 * 16], o2[128];
    (void)hipMemcpy(o, dO, sizeof o, hipMemcpyDeviceToHost);
    (void)hipMemcpy(o2, dO2, sizeof o2, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int q = 0; q < 16; ++q) {
            const int row = (q & 3) + 8 * (q >> 2) + 4 * (l >> 5), col = l & 31;
            float want = 0;
            for (int kk = 0; kk < 48; ++kk) want += Af[row][kk] * Bf[kk][col];
            if (o[l * 16 + q] != want) {
                if (bad < 6) printf("lane %d reg %d got %g want %g\n", l, q, o[l * 16 + q], want);
                ++bad;
            }
        }
    printf("chained f16: %d mismatches; lane0 m1=%g m2=%g\n", bad, o2[0], o2[1]);
    return 0;
}
