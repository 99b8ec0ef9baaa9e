// Probe: rocPRIM's radix_sort_pairs on n (u32 key < 2^bits, u32 value) pairs -- the Morton
// level-0 shape -- timed with HIP events, to compare with the library's 8-bit LSD passes.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/experiments/probe_sort.hip -o tools/var/probe_sort
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 10000000;
    const int bits = argc > 2 ? atoi(argv[2]) : 30;
    std::vector<uint32_t> hk(n), hv(n);
    uint64_t s = 88172645463325252ull;
    for (size_t i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        hk[i] = (uint32_t)s & ((1u << bits) - 1u);
        hv[i] = (uint32_t)i;
    }
    uint32_t *k0, *k1, *v0, *v1;
    CK(hipMalloc(&k0, n * 4)); CK(hipMalloc(&k1, n * 4)); CK(hipMalloc(&v0, n * 4)); CK(hipMalloc(&v1, n * 4));
    CK(hipMemcpy(k0, hk.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(v0, hv.data(), n * 4, hipMemcpyHostToDevice));
    size_t tb = 0;
    CK(rocprim::radix_sort_pairs(nullptr, tb, k0, k1, v0, v1, n, 0, bits));
    void *tmp;
    CK(hipMalloc(&tmp, tb));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float best = 1e9f;
    for (int r = 0; r < 12; ++r) {
        CK(hipEventRecord(a, 0));
        CK(rocprim::radix_sort_pairs(tmp, tb, k0, k1, v0, v1, n, 0, bits));
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        if (r >= 2 && ms < best) best = ms;
    }
    std::vector<uint32_t> ok(n), ov(n);
    CK(hipMemcpy(ok.data(), k1, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ov.data(), v1, n * 4, hipMemcpyDeviceToHost));
    bool good = true;
    for (size_t i = 1; i < n && good; ++i)
        if (ok[i - 1] > ok[i] || (ok[i - 1] == ok[i] && ov[i - 1] > ov[i])) good = false;
    for (size_t i = 0; i < n && good; ++i) if (hk[ov[i]] != ok[i]) good = false;
    printf("rocprim radix_sort_pairs n=%zu bits=%d: %.1f us (temp %zu B) %s\n", n, bits, best * 1e3, tb,
           good ? "sorted+stable" : "WRONG");
    return good ? 0 : 2;
}
