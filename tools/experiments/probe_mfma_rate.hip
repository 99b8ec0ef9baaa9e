// MFMA issue rate and held clock per f16 instruction shape on random operands (DVFS probe).
// Every wave keeps its operands in registers and issues NACC independent accumulation chains;
// the in-kernel clock is d(s_memtime) / d(s_memrealtime) x 100 MHz (MI355X_MICROARCH.md DVFS (6)).
//   hipcc --offload-arch=gfx950 -O3 tools/experiments/probe_mfma_rate.hip -o tools/var/probe_mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ inline uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}
__device__ inline _Float16 rnd(uint32_t s) { return (_Float16)((float)(hash(s) & 0xffff) / 65536.0f - 0.5f); }

// KIND 0: 32x32x16 x3 chain (K=48, the sweep's slot); 1: 16x16x32 x2 (K=64); 2: 16x16x32 + 16x16x16 (K=48);
// 3: 16x16x16 alone; 4: 32x32x8 alone; 5: 16x16x32 alone; 6: 32x32x16 alone
template <int KIND>
__global__ __launch_bounds__(256) void k(int iters, float *out, uint64_t *stamps) {
    const uint32_t seed = (blockIdx.x * 256 + threadIdx.x) * 97;
    f16x8 a8[4], b8[4];
    f16x4 a4[4], b4[4];
    for (int i = 0; i < 4; ++i)
        for (int e = 0; e < 8; ++e) {
            a8[i][e] = rnd(seed + i * 8 + e);
            b8[i][e] = rnd(seed + 1000 + i * 8 + e);
            if (e < 4) { a4[i][e] = rnd(seed + 2000 + i * 4 + e); b4[i][e] = rnd(seed + 3000 + i * 4 + e); }
        }
    f32x16 c16[4] = {};
    f32x4 c4[8] = {};
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (KIND == 0) {
                c16[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8[0], b8[j], f32x16{}, 0, 0, 0);
                c16[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8[1], b8[(j + 1) & 3], c16[j], 0, 0, 0);
                c16[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8[2], b8[(j + 2) & 3], c16[j], 0, 0, 0);
            } else if (KIND == 1) {
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    c4[2 * j + q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8[q], b8[j], c4[2 * j + q], 0, 0, 0);
                    c4[2 * j + q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8[q + 1], b8[(j + 1) & 3], c4[2 * j + q], 0, 0, 0);
                }
            } else if (KIND == 2) {
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    c4[2 * j + q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8[q], b8[j], c4[2 * j + q], 0, 0, 0);
                    c4[2 * j + q] = __builtin_amdgcn_mfma_f32_16x16x16f16(a4[q], b4[j], c4[2 * j + q], 0, 0, 0);
                }
            } else if (KIND == 3) {
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    c4[2 * j + q] = __builtin_amdgcn_mfma_f32_16x16x16f16(a4[q], b4[j], c4[2 * j + q], 0, 0, 0);
            } else if (KIND == 4) {
                c16[j] = __builtin_amdgcn_mfma_f32_32x32x8f16(a4[0], b4[j], c16[j], 0, 0, 0);
            } else if (KIND == 5) {
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    c4[2 * j + q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8[q], b8[j], c4[2 * j + q], 0, 0, 0);
            } else {
                c16[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8[0], b8[j], c16[j], 0, 0, 0);
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    for (int j = 0; j < 4; ++j)
        for (int r = 0; r < 16; ++r) s += c16[j][r];
    for (int j = 0; j < 8; ++j)
        for (int r = 0; r < 4; ++r) s += c4[j][r];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        stamps[blockIdx.x * 2] = t1 - t0;
        stamps[blockIdx.x * 2 + 1] = r1 - r0;
    }
}

template <int KIND>
void run(const char *name, double flops_per_iter_wave, int mfma_per_iter, int iters) {
    const int nblk = 256 * 4;
    float *out; uint64_t *st;
    (void)hipMalloc(&out, nblk * 256 * 4);
    (void)hipMalloc(&st, nblk * 16);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k<KIND>, dim3(nblk), dim3(256), 0, 0, iters, out, st);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k<KIND>, dim3(nblk), dim3(256), 0, 0, iters, out, st);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint64_t> h(nblk * 2);
    (void)hipMemcpy(h.data(), st, nblk * 16, hipMemcpyDeviceToHost);
    double cyc = 0, rt = 0;
    for (int b = 0; b < nblk; ++b) { cyc += h[2 * b]; rt += h[2 * b + 1]; }
    cyc /= nblk; rt /= nblk;
    const double ghz = cyc / rt * 0.1;
    const double waves = nblk * 4.0;
    const double tf = flops_per_iter_wave * iters * waves / (ms * 1e-3) / 1e12;
    // SIMD cycles per MFMA from the wall time at the held clock (1,024 SIMDs)
    const double mfmas = (double)mfma_per_iter * iters * waves / 1024.0;
    printf("%-30s %8.2f ms  %7.1f TFLOP/s  clock %.3f GHz  %.2f cyc/MFMA/SIMD\n", name, ms, tf, ghz,
           ms * 1e-3 * ghz * 1e9 / mfmas);
    (void)hipFree(out); (void)hipFree(st);
}

int main() {
    const int it = 60000;
    for (int rep = 0; rep < 2; ++rep) {
        run<0>("32x32x16 x3 chain (K48)", 4 * 3 * 32768.0, 12, it);
        run<1>("16x16x32 x2 (K64)", 8 * 2 * 16384.0, 16, it);
        run<2>("16x16x32 + 16x16x16 (K48)", 8 * (16384.0 + 8192.0), 16, it);
        run<3>("16x16x16 f16 (legacy)", 8 * 8192.0, 8, it);
        run<4>("32x32x8 f16 (legacy)", 4 * 16384.0, 4, it);
        run<5>("16x16x32 f16", 8 * 16384.0, 8, it);
        run<6>("32x32x16 f16", 4 * 32768.0, 4, it);
    }
    return 0;
}
