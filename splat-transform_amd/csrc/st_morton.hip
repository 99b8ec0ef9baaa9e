// st_morton.hip -- generateOrdering (ordering.ts:4-110) on the device.
//
// The reference sorts `indices` by a 30-bit Morton key over the set's extents
// (stable), then recursively re-sorts every run of > 256 equal keys using that
// run's own extents.  Here every recursion level is one pass over all active
// segments at once:
//   extents   per segment, NaN-ignoring min/max + the segment's first element
//             (a NaN first element makes the JS extents NaN -> segment skipped)
//   keys      (segment rank << 30 | morton) computed in f64 exactly as JS
//   sort      stable LSD radix sort of (key, index) -- segments keep their
//             slots, their members are reordered in place
//   runs      equal-key runs > 256 inside sorted segments become next level
// Level 0 is a single segment over all n (u32 keys, 4 passes); deeper levels
// carry only the big buckets.  Non-finite or zero extents stop a segment
// exactly where ordering.ts:53-61 returns.
#include "st_internal.h"
#include "st_jsmath.h"

namespace st {
namespace {

__device__ inline uint32_t part1by2(uint32_t x) {
    x &= 0x000003ffu;
    x = (x ^ (x << 16)) & 0xff0000ffu;
    x = (x ^ (x << 8)) & 0x0300f00fu;
    x = (x ^ (x << 4)) & 0x030c30c3u;
    x = (x ^ (x << 2)) & 0x09249249u;
    return x;
}

// float -> monotone u32 (NaN never stored)
__device__ inline uint32_t fkey(float f) {
    uint32_t u = __builtin_bit_cast(uint32_t, f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float fkey_inv(uint32_t k) {
    uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
    return __builtin_bit_cast(float, u);
}

struct SegInfo {
    double mn[3];
    double mul[3];
    uint32_t ok;  // 1: keyed + sortable; 0: skipped (invalid / identical extents)
    uint32_t pad;
};

// expand segments (start,len) into element list: P[j] = position, S[j] = segment
__global__ __launch_bounds__(256) void k_expand(const uint32_t *__restrict__ seg_start,
                                                const uint32_t *__restrict__ seg_off, uint32_t nseg, uint64_t total,
                                                uint32_t *__restrict__ P, uint32_t *__restrict__ S) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += stride) {
        uint32_t lo = 0, hi = nseg;  // last seg with off <= j
        while (hi - lo > 1) {
            uint32_t mid = (lo + hi) >> 1;
            if (seg_off[mid] <= j) lo = mid; else hi = mid;
        }
        P[j] = seg_start[lo] + (uint32_t)(j - seg_off[lo]);
        S[j] = lo;
    }
}

__global__ void k_ext_init(uint32_t *ext, uint32_t nseg) {
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x) {
        for (int a = 0; a < 3; ++a) {
            ext[s * 6 + a] = 0xffffffffu;  // min key
            ext[s * 6 + 3 + a] = 0u;       // max key
        }
    }
}

// segmented NaN-ignoring min/max via ordered-int atomics; block-level pre-reduction
// when the whole block lies in one segment (the level-0 case).
__global__ __launch_bounds__(256) void k_ext(const float *__restrict__ x, const float *__restrict__ y,
                                             const float *__restrict__ z, const uint32_t *__restrict__ idx,
                                             const uint32_t *__restrict__ P, const uint32_t *__restrict__ S,
                                             uint64_t total, uint32_t *ext) {
    __shared__ uint32_t red[6][4];
    const uint64_t base = (uint64_t)blockIdx.x * 4096;
    if (base >= total) return;
    const uint64_t last = (base + 4096 < total ? base + 4096 : total) - 1;
    const bool one_seg = S[base] == S[last];
    const float *cols[3] = {x, y, z};
    uint32_t mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0, 0, 0};
    for (int r = 0; r < 16; ++r) {
        const uint64_t j = base + (uint64_t)r * 256 + threadIdx.x;
        if (j > last) break;
        const uint32_t row = idx[P[j]];
        const uint32_t s = S[j];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float v = cols[a][row];
            if (v == v) {
                const uint32_t k = fkey(v);
                if (one_seg) {
                    mn[a] = k < mn[a] ? k : mn[a];
                    mx[a] = k > mx[a] ? k : mx[a];
                } else {
                    atomicMin(&ext[s * 6 + a], k);
                    atomicMax(&ext[s * 6 + 3 + a], k);
                }
            }
        }
    }
    if (!one_seg) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            uint32_t t0 = __shfl_xor(mn[a], o, 64), t1 = __shfl_xor(mx[a], o, 64);
            mn[a] = t0 < mn[a] ? t0 : mn[a];
            mx[a] = t1 > mx[a] ? t1 : mx[a];
        }
        if (lane == 0) {
            red[a][w] = mn[a];
            red[3 + a][w] = mx[a];
        }
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int q = threadIdx.x;
        uint32_t v = red[q][0];
        for (int i = 1; i < 4; ++i) v = q < 3 ? (red[q][i] < v ? red[q][i] : v) : (red[q][i] > v ? red[q][i] : v);
        const uint32_t s = S[base];
        if (q < 3) atomicMin(&ext[s * 6 + q], v);
        else atomicMax(&ext[s * 6 + q], v);
    }
}

// ordering.ts:32-65 per segment
__global__ void k_seg_info(const float *__restrict__ x, const float *__restrict__ y, const float *__restrict__ z,
                           const uint32_t *__restrict__ idx, const uint32_t *__restrict__ seg_start,
                           const uint32_t *__restrict__ ext, uint32_t nseg, SegInfo *info) {
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x) {
        const uint32_t first = idx[seg_start[s]];
        const float f[3] = {x[first], y[first], z[first]};
        SegInfo si{};
        bool valid = true, all_zero = true;
        for (int a = 0; a < 3; ++a) {
            double len;
            if (f[a] != f[a] || ext[s * 6 + a] == 0xffffffffu) {
                len = __builtin_nan("");  // NaN first element -> extents NaN (ordering.ts:38-41)
            } else {
                const double lo = fkey_inv(ext[s * 6 + a]), hi = fkey_inv(ext[s * 6 + 3 + a]);
                len = hi - lo;
                si.mn[a] = lo;
            }
            if (!js::isfinite_(len)) valid = false;
            if (len != 0) all_zero = false;
            si.mul[a] = (len == 0) ? 0 : 1024 / len;
        }
        si.ok = (valid && !all_zero) ? 1u : 0u;
        info[s] = si;
    }
}

__device__ inline uint32_t axis_q(float v, double mn, double mul) {
    return js::to_uint32(js::min_(1023, ((double)v - mn) * mul));
}

template <typename K>
__global__ __launch_bounds__(256) void k_keys(const float *__restrict__ x, const float *__restrict__ y,
                                              const float *__restrict__ z, const uint32_t *__restrict__ idx,
                                              const uint32_t *__restrict__ P, const uint32_t *__restrict__ S,
                                              const SegInfo *__restrict__ info, uint64_t total, int single,
                                              K *__restrict__ keys, uint32_t *__restrict__ vals) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += stride) {
        const uint32_t p = single ? (uint32_t)j : P[j];
        const uint32_t s = single ? 0u : S[j];
        const uint32_t row = idx[p];
        const SegInfo &si = info[s];
        uint32_t m = 0;
        if (si.ok) {
            const uint32_t ix = axis_q(x[row], si.mn[0], si.mul[0]);
            const uint32_t iy = axis_q(y[row], si.mn[1], si.mul[1]);
            const uint32_t iz = axis_q(z[row], si.mn[2], si.mul[2]);
            m = (part1by2(iz) << 2) + (part1by2(iy) << 1) + part1by2(ix);
        }
        keys[j] = ((K)s << 30) | (K)m;
        vals[j] = row;
    }
}

__global__ __launch_bounds__(256) void k_scatter_back(const uint32_t *__restrict__ P, const uint32_t *__restrict__ vals,
                                                      uint64_t total, int single, uint32_t *__restrict__ idx) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += stride)
        idx[single ? (uint32_t)j : P[j]] = vals[j];
}

// run starts: flag[j] = 1 if j starts a run of equal keys
template <typename K>
__global__ __launch_bounds__(256) void k_run_flags(const K *__restrict__ keys, uint64_t total,
                                                   uint32_t *__restrict__ flag) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += stride)
        flag[j] = (j == 0 || keys[j] != keys[j - 1]) ? 1u : 0u;
}

__global__ __launch_bounds__(256) void k_run_starts(const uint32_t *__restrict__ flag,
                                                    const uint32_t *__restrict__ rid, uint64_t total,
                                                    uint32_t *__restrict__ run_start) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += stride)
        if (flag[j]) run_start[rid[j]] = (uint32_t)j;
}

// big runs of sortable segments -> flag; run_start[nruns] == total sentinel
template <typename K>
__global__ __launch_bounds__(256) void k_big_runs(const uint32_t *__restrict__ run_start, uint32_t nruns,
                                                  const K *__restrict__ keys, const SegInfo *__restrict__ info,
                                                  uint32_t *__restrict__ big) {
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < nruns; r += gridDim.x * blockDim.x) {
        const uint32_t len = run_start[r + 1] - run_start[r];
        const uint32_t s = (uint32_t)(keys[run_start[r]] >> 30);
        big[r] = (len > 256 && info[s].ok) ? 1u : 0u;
    }
}

__global__ __launch_bounds__(256) void k_emit_segs(const uint32_t *__restrict__ run_start, uint32_t nruns,
                                                   const uint32_t *__restrict__ big, const uint32_t *__restrict__ bpos,
                                                   const uint32_t *__restrict__ P, int single,
                                                   uint32_t *__restrict__ nstart, uint32_t *__restrict__ nlen) {
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < nruns; r += gridDim.x * blockDim.x) {
        if (!big[r]) continue;
        const uint32_t j = run_start[r];
        nstart[bpos[r]] = single ? j : P[j];
        nlen[bpos[r]] = run_start[r + 1] - j;
    }
}

__global__ void k_set_sentinel(uint32_t *a, uint32_t i, uint32_t v) { a[i] = v; }

}  // namespace

void morton_order_dev(st_ctx *c, const float *x, const float *y, const float *z, uint32_t *idx, uint64_t n) {
    if (n == 0) return;
    ST_REQUIRE(n < (1ull << 32) - 1, ST_ERR_ARG, "morton: n must be < 2^32-1");
    auto *h = static_cast<uint32_t *>(pinned(c, 64));
    // active segment list
    auto *seg_start = wsT<uint32_t>(c, "mo.seg_start", n / 257 + 2);
    auto *seg_len = wsT<uint32_t>(c, "mo.seg_len", n / 257 + 2);
    auto *nseg_start = wsT<uint32_t>(c, "mo.nseg_start", n / 257 + 2);
    auto *nseg_len = wsT<uint32_t>(c, "mo.nseg_len", n / 257 + 2);
    auto *seg_off = wsT<uint32_t>(c, "mo.seg_off", n / 257 + 3);
    uint32_t nseg = 1;
    {
        uint32_t one[2] = {0u, (uint32_t)n};
        ST_HIP(hipMemcpyAsync(seg_start, &one[0], 4, hipMemcpyHostToDevice, c->stream));
        ST_HIP(hipMemcpyAsync(seg_len, &one[1], 4, hipMemcpyHostToDevice, c->stream));
        ST_HIP(hipStreamSynchronize(c->stream));
    }
    uint64_t total = n;
    auto *P = wsT<uint32_t>(c, "mo.P", n);
    auto *S = wsT<uint32_t>(c, "mo.S", n);
    auto *flag = wsT<uint32_t>(c, "mo.flag", n + 1);
    auto *rid = wsT<uint32_t>(c, "mo.rid", n + 1);
    auto *vals = wsT<uint32_t>(c, "mo.vals", n);
    for (int level = 0; nseg > 0; ++level) {
        const bool single = (level == 0);
        if (!single) {
            scan_u32(c, seg_len, seg_off, nseg, seg_off + nseg);
            ST_HIP(hipMemcpyAsync(h, seg_off + nseg, 4, hipMemcpyDeviceToHost, c->stream));
            ST_HIP(hipStreamSynchronize(c->stream));
            total = h[0];
            hipLaunchKernelGGL(k_expand, dim3(grid_for(total, 256, 8192)), dim3(256), 0, c->stream, seg_start, seg_off,
                               nseg, total, P, S);
            ST_LAUNCH_CHECK();
        } else {
            // level 0: P = identity, S = 0 (only k_ext reads them)
            iota_u32(c, P, n);
            ST_HIP(hipMemsetAsync(S, 0, n * sizeof(uint32_t), c->stream));
        }
        auto *ext = wsT<uint32_t>(c, "mo.ext", (size_t)nseg * 6);
        auto *info = static_cast<SegInfo *>(ws(c, "mo.info", sizeof(SegInfo) * (size_t)nseg));
        hipLaunchKernelGGL(k_ext_init, dim3(grid_for(nseg, 256, 1024)), dim3(256), 0, c->stream, ext, nseg);
        hipLaunchKernelGGL(k_ext, dim3((unsigned)((total + 4095) / 4096)), dim3(256), 0, c->stream, x, y, z, idx, P, S,
                           total, ext);
        ST_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_seg_info, dim3(grid_for(nseg, 64, 1024)), dim3(64), 0, c->stream, x, y, z, idx, seg_start,
                           ext, nseg, info);
        ST_LAUNCH_CHECK();
        int seg_bits = 0;
        while ((1u << seg_bits) < nseg) ++seg_bits;
        const unsigned g = grid_for(total, 256, 8192);
        uint32_t nruns;
        if (seg_bits + 30 <= 32) {
            auto *keys = wsT<uint32_t>(c, "mo.k32", total + 1);
            hipLaunchKernelGGL(k_keys<uint32_t>, dim3(g), dim3(256), 0, c->stream, x, y, z, idx, P, S, info, total,
                               (int)single, keys, vals);
            ST_LAUNCH_CHECK();
            radix_sort_u32(c, keys, vals, total, 0, 30 + seg_bits, "mo.rs32");
            hipLaunchKernelGGL(k_scatter_back, dim3(g), dim3(256), 0, c->stream, P, vals, total, (int)single, idx);
            hipLaunchKernelGGL(k_run_flags<uint32_t>, dim3(g), dim3(256), 0, c->stream, keys, total, flag);
            ST_LAUNCH_CHECK();
            scan_u32(c, flag, rid, total, rid + total);
            ST_HIP(hipMemcpyAsync(h, rid + total, 4, hipMemcpyDeviceToHost, c->stream));
            ST_HIP(hipStreamSynchronize(c->stream));
            nruns = h[0];
            auto *run_start = wsT<uint32_t>(c, "mo.run_start", (size_t)nruns + 1);
            hipLaunchKernelGGL(k_run_starts, dim3(g), dim3(256), 0, c->stream, flag, rid, total, run_start);
            hipLaunchKernelGGL(k_set_sentinel, dim3(1), dim3(1), 0, c->stream, run_start, nruns, (uint32_t)total);
            auto *big = wsT<uint32_t>(c, "mo.big", (size_t)nruns + 1);
            hipLaunchKernelGGL(k_big_runs<uint32_t>, dim3(grid_for(nruns, 256, 8192)), dim3(256), 0, c->stream,
                               run_start, nruns, keys, info, big);
            ST_LAUNCH_CHECK();
            auto *bpos = wsT<uint32_t>(c, "mo.bpos", (size_t)nruns + 1);
            scan_u32(c, big, bpos, nruns, bpos + nruns);
            hipLaunchKernelGGL(k_emit_segs, dim3(grid_for(nruns, 256, 8192)), dim3(256), 0, c->stream, run_start,
                               nruns, big, bpos, P, (int)single, nseg_start, nseg_len);
            ST_LAUNCH_CHECK();
            ST_HIP(hipMemcpyAsync(h, bpos + nruns, 4, hipMemcpyDeviceToHost, c->stream));
        } else {
            auto *keys = wsT<uint64_t>(c, "mo.k64", total + 1);
            hipLaunchKernelGGL(k_keys<uint64_t>, dim3(g), dim3(256), 0, c->stream, x, y, z, idx, P, S, info, total,
                               (int)single, keys, vals);
            ST_LAUNCH_CHECK();
            radix_sort_u64(c, keys, vals, total, 0, 30 + seg_bits, "mo.rs64");
            hipLaunchKernelGGL(k_scatter_back, dim3(g), dim3(256), 0, c->stream, P, vals, total, (int)single, idx);
            hipLaunchKernelGGL(k_run_flags<uint64_t>, dim3(g), dim3(256), 0, c->stream, keys, total, flag);
            ST_LAUNCH_CHECK();
            scan_u32(c, flag, rid, total, rid + total);
            ST_HIP(hipMemcpyAsync(h, rid + total, 4, hipMemcpyDeviceToHost, c->stream));
            ST_HIP(hipStreamSynchronize(c->stream));
            nruns = h[0];
            auto *run_start = wsT<uint32_t>(c, "mo.run_start", (size_t)nruns + 1);
            hipLaunchKernelGGL(k_run_starts, dim3(g), dim3(256), 0, c->stream, flag, rid, total, run_start);
            hipLaunchKernelGGL(k_set_sentinel, dim3(1), dim3(1), 0, c->stream, run_start, nruns, (uint32_t)total);
            auto *big = wsT<uint32_t>(c, "mo.big", (size_t)nruns + 1);
            hipLaunchKernelGGL(k_big_runs<uint64_t>, dim3(grid_for(nruns, 256, 8192)), dim3(256), 0, c->stream,
                               run_start, nruns, keys, info, big);
            ST_LAUNCH_CHECK();
            auto *bpos = wsT<uint32_t>(c, "mo.bpos", (size_t)nruns + 1);
            scan_u32(c, big, bpos, nruns, bpos + nruns);
            hipLaunchKernelGGL(k_emit_segs, dim3(grid_for(nruns, 256, 8192)), dim3(256), 0, c->stream, run_start,
                               nruns, big, bpos, P, (int)single, nseg_start, nseg_len);
            ST_LAUNCH_CHECK();
            ST_HIP(hipMemcpyAsync(h, bpos + nruns, 4, hipMemcpyDeviceToHost, c->stream));
        }
        ST_HIP(hipStreamSynchronize(c->stream));
        nseg = h[0];
        std::swap(seg_start, nseg_start);
        std::swap(seg_len, nseg_len);
    }
}

}  // namespace st
