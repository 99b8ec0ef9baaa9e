// Probe the operand/result lane layout of v_mfma_f32_32x32x16_{f16,bf16} on gfx950.
// A[i][k] = i*16 + k (exact), B[k][j] = (k == (j % 16)) -> C[i][j] = A[i][j%16] = i*16 + j%16.
// Operands are packed with the ASSUMED map (lane l: A[l&31][8(l>>5)+e], B[8(l>>5)+e][l&31]);
// each output register is decoded back to (i, j%16) and compared with the assumed C map.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k(float *out, int use_bf16) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    f32x16 acc = {};
    if (use_bf16) {
        bf16x8 a, b;
        for (int e = 0; e < 8; ++e) {
            const int kk = 8 * h + e;
            a[e] = (__bf16)(float)(r * 16 + kk);
            b[e] = (__bf16)(float)((kk == (r % 16)) ? 1 : 0);
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    } else {
        f16x8 a, b;
        for (int e = 0; e < 8; ++e) {
            const int kk = 8 * h + e;
            a[e] = (_Float16)(float)(r * 16 + kk);
            b[e] = (_Float16)(float)((kk == (r % 16)) ? 1 : 0);
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    }
    for (int q = 0; q < 16; ++q) out[l * 16 + q] = acc[q];
}

int main() {
    float *d, h[64 * 16];
    hipMalloc(&d, sizeof h);
    for (int bf = 0; bf < 2; ++bf) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, bf);
        hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int l = 0; l < 64; ++l)
            for (int q = 0; q < 16; ++q) {
                const int row = (q & 3) + 8 * (q >> 2) + 4 * (l >> 5), col = l & 31;
                const float want = row * 16 + (col % 16);
                if (h[l * 16 + q] != want) {
                    if (bad < 8) printf("%s lane %d reg %d: got %g (i=%d,k=%d) want %g\n", bf ? "bf16" : "f16", l, q,
                                        h[l * 16 + q], (int)h[l * 16 + q] / 16, (int)h[l * 16 + q] % 16, want);
                    ++bad;
                }
            }
        printf("%s: %d mismatches\n", bf ? "bf16" : "f16", bad);
    }
    return 0;
}
