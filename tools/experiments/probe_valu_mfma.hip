// Cost of VALU fillers beside MFMAs (the sweep epilogue's budget): SIMD cycles per 16x16x48
// pair (v_mfma_f32_16x16x32_f16 + v_mfma_f32_16x16x16_f16) and per 32x32x48 slot
// (3 x v_mfma_f32_32x32x16_f16) with NV v_min3_f32 per pair / slot, at WPS waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/experiments/probe_valu_mfma.hip -o tools/var/probe_valu_mfma
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

template <int SHAPE, int NV>
__global__ __launch_bounds__(64) void k(int iters, float *out, uint64_t *stamps) {
    const uint32_t seed = (blockIdx.x * 64 + threadIdx.x) * 97;
    f16x8 a8[2], b8[8];
    f16x4 a4[2], b4[8];
    for (int i = 0; i < 8; ++i)
        for (int e = 0; e < 8; ++e) {
            b8[i][e] = rnd(seed + 1000 + i * 8 + e);
            if (e < 4) b4[i][e] = rnd(seed + 3000 + i * 4 + e);
            if (i < 2) { a8[i][e] = rnd(seed + i * 8 + e); if (e < 4) a4[i][e] = rnd(seed + 2000 + i * 4 + e); }
        }
    f32x4 c4[8];
    f32x16 c16[4];
    for (int i = 0; i < 8; ++i) c4[i] = f32x4{1e30f, 1e30f, 1e30f, 1e30f};
    for (int i = 0; i < 4; ++i)
        for (int r = 0; r < 16; ++r) c16[i][r] = 1e30f;
    float mn[8];
    for (int i = 0; i < 8; ++i) mn[i] = 1e30f;
    // one 16-row sub-tile (SHAPE 0) / one centroid tile over 4 point tiles (SHAPE 1)
    auto sub16 = [&](const f16x8 &x8, const f16x4 &x4) {
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            if (i < 8) {
                if (NV >= 1) mn[i] = fminf(fminf(mn[i], c4[i][0]), c4[i][1]);
                if (NV >= 2) mn[i] = fminf(fminf(mn[i], c4[i][2]), c4[i][3]);
                if (NV >= 3) mn[i] = fminf(fminf(mn[i], c4[i][1]), c4[i][3]);
                if (NV >= 4) mn[i] = fminf(fminf(mn[i], c4[i][0]), c4[i][2]);
                c4[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(x8, b8[i], f32x4{}, 0, 0, 0);
            }
            if (i >= 2) c4[i - 2] = __builtin_amdgcn_mfma_f32_16x16x16f16(x4, b4[i - 2], c4[i - 2], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    auto tile32 = [&](const f16x8 &x0, const f16x8 &x1, const f16x8 &x2) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int td = (t + 1) & 3;
            f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x0, b8[t], f32x16{}, 0, 0, 0);
            float m = mn[td];
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                m = fminf(fminf(m, c16[td][(2 * q) & 15]), c16[td][(2 * q + 1) & 15]);
                if (q == (NV + 2) / 3 - 1) {
                    __builtin_amdgcn_sched_barrier(0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x1, b8[t + 4], acc, 0, 0, 0);
                }
                if (q == 2 * (NV + 2) / 3 - 1) {
                    __builtin_amdgcn_sched_barrier(0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x2, b8[(t + 2) & 7], acc, 0, 0, 0);
                }
            }
            if (NV < 1) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x1, b8[t + 4], acc, 0, 0, 0);
            if (NV < 2) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x2, b8[(t + 2) & 7], acc, 0, 0, 0);
            mn[td] = m;
            c16[t] = acc;
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    // SHAPE 2: the 16-value minimum of the previous slot's scores as a depth-3 tree of 8 ops,
    // spread over the slot's three MFMAs (3 + 3 + 2)
    auto tile32t = [&](const f16x8 &x0, const f16x8 &x1, const f16x8 &x2) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int td = (t + 1) & 3;
            const f32x16 &c = c16[td];
            f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x0, b8[t], f32x16{}, 0, 0, 0);
            const float u0 = fminf(fminf(c[0], c[1]), c[2]);
            const float u1 = fminf(fminf(c[3], c[4]), c[5]);
            const float u2 = fminf(fminf(c[6], c[7]), c[8]);
            __builtin_amdgcn_sched_barrier(0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x1, b8[t + 4], acc, 0, 0, 0);
            const float u3 = fminf(fminf(c[9], c[10]), c[11]);
            const float u4 = fminf(fminf(c[12], c[13]), c[14]);
            const float v0 = fminf(fminf(u0, u1), u2);
            __builtin_amdgcn_sched_barrier(0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x2, b8[(t + 2) & 7], acc, 0, 0, 0);
            const float v1 = fminf(fminf(u3, u4), c[15]);
            mn[td] = fminf(fminf(mn[td], v0), v1);
            c16[t] = acc;
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
        if (SHAPE == 0) {
            sub16(a8[0], a4[0]);
            sub16(a8[1], a4[1]);
        } else if (SHAPE == 1) {
            tile32(a8[0], a8[1], b8[7]);
            tile32(a8[1], a8[0], b8[6]);
        } else {
            tile32t(a8[0], a8[1], b8[7]);
            tile32t(a8[1], a8[0], b8[6]);
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    for (int i = 0; i < 8; ++i) s += c4[i][0] + c4[i][3] + mn[i];
    for (int i = 0; i < 4; ++i) s += c16[i][0] + c16[i][15];
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        stamps[blockIdx.x * 2] = t1 - t0;
        stamps[blockIdx.x * 2 + 1] = r1 - r0;
    }
}

template <int SHAPE, int NV>
void run(int wps, int iters) {
    const int nblk = 1024 * wps;  // one wave per block: wps waves per SIMD
    float *out; uint64_t *st;
    (void)hipMalloc(&out, nblk * 64 * 4);
    (void)hipMalloc(&st, nblk * 16);
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL((k<SHAPE, NV>), dim3(nblk), dim3(64), 0, 0, iters, out, st);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k<SHAPE, NV>), dim3(nblk), dim3(64), 0, 0, iters, out, st);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint64_t> h(nblk * 2);
    (void)hipMemcpy(h.data(), st, nblk * 16, hipMemcpyDeviceToHost);
    double cyc = 0, rt = 0;
    for (int b = 0; b < nblk; ++b) { cyc += h[2 * b]; rt += h[2 * b + 1]; }
    cyc /= nblk; rt /= nblk;
    const double ghz = cyc / rt * 0.1;
    // units per SIMD: SHAPE 0 = 8 pairs / iter, SHAPE 1 = 4 slots / iter
    const double units = (SHAPE == 0 ? 16.0 : 8.0) * iters * wps;
    const double flops = (SHAPE == 0 ? 16.0 * 16 * 16 * 48 * 2 : 8.0 * 32 * 32 * 48 * 2) * iters * nblk;
    const char *nm = SHAPE == 0 ? "16x16 pair" : SHAPE == 1 ? "32x32 slot, chain" : "32x32 slot, tree";
    printf("%s NV=%d waves/SIMD=%d: %.2f ms, clock %.3f GHz, %.1f cyc per %s (MFMA floor %s), %.0f TFLOP/s(K48)\n",
           nm, NV, wps, ms, ghz, ms * 1e-3 * ghz * 1e9 / units,
           SHAPE == 0 ? "pair" : "slot", SHAPE == 0 ? "32" : "96", flops / (ms * 1e-3) / 1e12);
    (void)hipFree(out); (void)hipFree(st);
}

int main() {
    const int it = 20000;
    for (int wps = 1; wps <= 2; ++wps) {
        run<0, 1>(wps, it); run<0, 2>(wps, it);
        run<1, 3>(wps, it); run<1, 8>(wps, it);
        run<2, 8>(wps, it);
    }
    return 0;
}
