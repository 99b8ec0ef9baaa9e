// The fused fix-up's memory pattern alone: 10M point rows of 48 floats (192 B) read in a random
// order (the decided points grouped by tile-half are a random permutation of the points), one
// float written per row, against the same rows read in order.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

// one lane per row: 12 x 16-B loads
__global__ void k_lane_row(const f32x4 *__restrict__ rows, const uint32_t *__restrict__ idx, uint32_t n,
                           float *__restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const f32x4 *r = rows + (uint64_t)idx[i] * 12;
    f32x4 s = r[0];
#pragma unroll
    for (int q = 1; q < 12; ++q) s += r[q];
    out[i] = s.x + s.y + s.z + s.w;
}

// 16 lanes per row (12 active): one 16-B load each
__global__ void k_group_row(const f32x4 *__restrict__ rows, const uint32_t *__restrict__ idx, uint32_t n,
                            float *__restrict__ out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t i = (uint32_t)(t >> 4), q = t & 15;
    if (i >= n) return;
    f32x4 v = q < 12 ? rows[(uint64_t)idx[i] * 12 + q] : f32x4{0, 0, 0, 0};
    float s = v.x + v.y + v.z + v.w;
    for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 16);
    if (q == 0) out[i] = s;
}

int main() {
    const uint32_t n = 10000000;
    std::vector<uint32_t> perm(n), seq(n);
    std::iota(seq.begin(), seq.end(), 0u);
    perm = seq;
    std::shuffle(perm.begin(), perm.end(), std::mt19937(7));
    f32x4 *rows;
    uint32_t *dperm, *dseq;
    float *out;
    hipMalloc(&rows, (size_t)n * 192);
    hipMemset(rows, 0, (size_t)n * 192);
    hipMalloc(&dperm, 4ull * n);
    hipMalloc(&dseq, 4ull * n);
    hipMalloc(&out, 4ull * n);
    hipMemcpy(dperm, perm.data(), 4ull * n, hipMemcpyHostToDevice);
    hipMemcpy(dseq, seq.data(), 4ull * n, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int kind = 0; kind < 2; ++kind)
        for (int order = 0; order < 2; ++order) {
            const uint32_t *ix = order ? dperm : dseq;
            float best = 1e9f;
            for (int rep = 0; rep < 6; ++rep) {
                hipEventRecord(a);
                if (kind == 0)
                    hipLaunchKernelGGL(k_lane_row, dim3((n + 255) / 256), dim3(256), 0, 0, rows, ix, n, out);
                else
                    hipLaunchKernelGGL(k_group_row, dim3((unsigned)(((uint64_t)n * 16 + 255) / 256)), dim3(256), 0, 0,
                                       rows, ix, n, out);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                if (rep) best = std::min(best, ms);
            }
            printf("%s %s: %.3f ms = %.2f TB/s of 192-B rows\n", kind ? "16 lanes/row" : "lane/row",
                   order ? "random" : "in order", best, n * 192.0 / best / 1e9);
        }
    return 0;
}
