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
// Level 0 is a single segment over all n: block-partial extents (k_ext), keys
// plus the first digit's tile counts (k_keys0), and a 4-pass u32 sort that reads
// idx as its values and writes the order back into it.  Deeper levels carry only
// the big runs: segmented extents through per-block LDS slots (k_ext_seg), and
// only segments with usable extents are keyed and sorted -- non-finite or zero
// extents stop a segment exactly where ordering.ts:53-61 returns.
#include "st_internal.h"
#include "st_jsmath.h"
#include "st_typed.h"

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

// coordinate traits: float32 columns (the splat table) or float64 ones (the JS numbers of any
// other column type): extents as order-preserving integer keys of the coordinate's width
template <typename T>
struct MC;
template <>
struct MC<float> {
    using K = uint32_t;
    using V = float4;
    static constexpr K KMAX = 0xffffffffu;
    __device__ static K key(float f) { return fkey(f); }
    __device__ static double inv(K k) { return (double)fkey_inv(k); }
    __device__ static V pack(float a, float b, float c) { return make_float4(a, b, c, 0.0f); }
};
template <>
struct MC<double> {
    using K = unsigned long long;
    using V = double4;
    static constexpr K KMAX = ~0ull;
    __device__ static K key(double d) {
        const K u = __builtin_bit_cast(K, d);
        return (u >> 63) ? ~u : (u | (1ull << 63));
    }
    __device__ static double inv(K k) { return __builtin_bit_cast(double, (k >> 63) ? (k & ~(1ull << 63)) : ~k); }
    __device__ static V pack(double a, double b, double c) { return make_double4(a, b, c, 0.0); }
};

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

template <typename K>
__global__ void k_ext_init(K *ext, uint32_t nseg) {
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x) {
        for (int a = 0; a < 3; ++a) {
            ext[s * 6 + a] = ~(K)0;  // min key
            ext[s * 6 + 3 + a] = 0;  // max key
        }
    }
}

// level 0 (one segment, P = identity, S = 0 -- neither is read): each block leaves its six
// extents (NaN-ignoring min / max as ordered ints) in part[block]; k_ext_final reduces them
template <typename T>
__global__ __launch_bounds__(256) void k_ext(const T *__restrict__ x, const T *__restrict__ y,
                                             const T *__restrict__ z, const uint32_t *__restrict__ idx,
                                             uint64_t total, typename MC<T>::K *part) {
    using K = typename MC<T>::K;
    __shared__ K red[6][4];
    const uint64_t base = (uint64_t)blockIdx.x * 4096;
    if (base >= total) return;
    const uint64_t last = (base + 4096 < total ? base + 4096 : total) - 1;
    const T *cols[3] = {x, y, z};
    K mn[3] = {MC<T>::KMAX, MC<T>::KMAX, MC<T>::KMAX}, mx[3] = {0, 0, 0};
    // all 16 rows' indices, then all their coordinates, in flight before the first test
    uint32_t rows_[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint64_t j = base + (uint64_t)r * 256 + threadIdx.x;
        rows_[r] = idx[j > last ? last : j];
    }
    T vals_[16][3];
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
        for (int a = 0; a < 3; ++a) vals_[r][a] = cols[a][rows_[r]];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint64_t j = base + (uint64_t)r * 256 + threadIdx.x;
        if (j > last) break;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const T v = vals_[r][a];
            if (v == v) {
                const K k = MC<T>::key(v);
                mn[a] = k < mn[a] ? k : mn[a];
                mx[a] = k > mx[a] ? k : mx[a];
            }
        }
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            K t0 = __shfl_xor(mn[a], o, 64), t1 = __shfl_xor(mx[a], o, 64);
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
        K v = red[q][0];
        for (int i = 1; i < 4; ++i) v = q < 3 ? (red[q][i] < v ? red[q][i] : v) : (red[q][i] > v ? red[q][i] : v);
        part[(uint64_t)blockIdx.x * 6 + q] = v;
    }
}

// deeper levels: the segments are runs of > 256 elements, contiguous in P order, so the 4,096
// elements of a block touch at most 17 of them and a wave's 1,024 consecutive elements at most
// 5.  Lanes keep min / max for the wave's current segment while whole 64-element rows stay in
// it; on a change the wave reduces them by shuffles into the block's LDS slot of that segment
// (rows that straddle a boundary go to the slots lane by lane); the block then merges its
// slots into the global extents with one atomic per (segment, value).  (Per-element global
// atomics on a handful of addresses took 2.5 ms at 10M on a lattice input.)
constexpr int EXT_SLOTS = 4096 / 257 + 2;
template <typename T>
__global__ __launch_bounds__(256) void k_ext_seg(const T *__restrict__ x, const T *__restrict__ y,
                                                 const T *__restrict__ z, const uint32_t *__restrict__ idx,
                                                 const uint32_t *__restrict__ P, const uint32_t *__restrict__ S,
                                                 uint64_t total, typename MC<T>::K *ext,
                                                 typename MC<T>::V *__restrict__ cxyz) {
    using K = typename MC<T>::K;
    __shared__ K slot[EXT_SLOTS * 6];
    const uint64_t base = (uint64_t)blockIdx.x * 4096;
    if (base >= total) return;
    const uint64_t last = (base + 4096 < total ? base + 4096 : total) - 1;
    const uint32_t s0 = S[base], s1 = S[last];
    for (int i = threadIdx.x; i < EXT_SLOTS * 6; i += 256) slot[i] = (i % 6) < 3 ? MC<T>::KMAX : (K)0;
    __syncthreads();
    const T *cols[3] = {x, y, z};
    const int lane = threadIdx.x & 63;
    const uint64_t wb = base + (uint64_t)(threadIdx.x >> 6) * 1024;
    uint32_t seg_[16], pos_[16], rows_[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint64_t j = wb + (uint64_t)r * 64 + lane;
        const uint64_t jj = j > last ? last : j;
        seg_[r] = j > last ? 0xffffffffu : S[jj];
        pos_[r] = P[jj];
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) rows_[r] = idx[pos_[r]];
    T vals_[16][3];
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
        for (int a = 0; a < 3; ++a) vals_[r][a] = cols[a][rows_[r]];
    // the gathered coordinates, kept at their idx positions for the level's keys (coalesced
    // there: a segment's positions are contiguous), so x / y / z are gathered once per level
#pragma unroll
    for (int r = 0; r < 16; ++r)
        if (seg_[r] != 0xffffffffu) cxyz[pos_[r]] = MC<T>::pack(vals_[r][0], vals_[r][1], vals_[r][2]);
    auto take = [&](uint32_t s, const T *v) {  // one lane into its segment's slot
        const uint32_t q = s - s0;
        K *dst = q < (uint32_t)EXT_SLOTS ? &slot[q * 6] : &ext[(uint64_t)s * 6];
#pragma unroll
        for (int a = 0; a < 3; ++a)
            if (v[a] == v[a]) {
                atomicMin(&dst[a], MC<T>::key(v[a]));
                atomicMax(&dst[3 + a], MC<T>::key(v[a]));
            }
    };
    uint32_t cur = 0xffffffffu;  // wave-uniform
    K mn[3], mx[3];
    auto reset = [&] {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            mn[a] = MC<T>::KMAX;
            mx[a] = 0;
        }
    };
    auto flush = [&] {
        if (cur == 0xffffffffu) return;
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const K t0 = __shfl_xor(mn[a], o, 64), t1 = __shfl_xor(mx[a], o, 64);
                mn[a] = t0 < mn[a] ? t0 : mn[a];
                mx[a] = t1 > mx[a] ? t1 : mx[a];
            }
        if (lane == 0) {
            const uint32_t q = cur - s0;
            K *dst = q < (uint32_t)EXT_SLOTS ? &slot[q * 6] : &ext[(uint64_t)cur * 6];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                if (mn[a] != MC<T>::KMAX) atomicMin(&dst[a], mn[a]);
                if (mx[a] != 0) atomicMax(&dst[3 + a], mx[a]);
            }
        }
        cur = 0xffffffffu;
    };
    reset();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t s = seg_[r];
        const uint32_t sf = __builtin_amdgcn_readfirstlane(s);
        if (__ballot(s != sf) == 0ull) {  // the whole row lies in one segment (or past the end)
            if (sf == 0xffffffffu) continue;
            if (sf != cur) {
                flush();
                reset();
                cur = sf;
            }
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const T v = vals_[r][a];
                if (v == v) {
                    const K k = MC<T>::key(v);
                    mn[a] = k < mn[a] ? k : mn[a];
                    mx[a] = k > mx[a] ? k : mx[a];
                }
            }
        } else {
            flush();
            reset();
            if (s != 0xffffffffu) take(s, vals_[r]);
        }
    }
    flush();
    __syncthreads();
    const uint32_t used = (s1 - s0 + 1) * 6;
    for (uint32_t i = threadIdx.x; i < used && i < (uint32_t)EXT_SLOTS * 6; i += 256) {
        const K v = slot[i];
        const uint32_t q = i / 6, a = i % 6;
        if (a < 3) {
            if (v != MC<T>::KMAX) atomicMin(&ext[(uint64_t)(s0 + q) * 6 + a], v);
        } else if (v != 0) {
            atomicMax(&ext[(uint64_t)(s0 + q) * 6 + a], v);
        }
    }
}

// level 0: the six extents from the per-block partials
template <typename K>
__global__ __launch_bounds__(256) void k_ext_final(const K *__restrict__ part, uint32_t nb, K *ext) {
    __shared__ K red[6][4];
    K v[6] = {~(K)0, ~(K)0, ~(K)0, 0, 0, 0};
    for (uint32_t b = threadIdx.x; b < nb; b += 256)
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            const K t = part[(uint64_t)b * 6 + q];
            v[q] = q < 3 ? (t < v[q] ? t : v[q]) : (t > v[q] ? t : v[q]);
        }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        for (int o = 32; o > 0; o >>= 1) {
            const K t = __shfl_xor(v[q], o, 64);
            v[q] = q < 3 ? (t < v[q] ? t : v[q]) : (t > v[q] ? t : v[q]);
        }
        if (lane == 0) red[q][w] = v[q];
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int q = threadIdx.x;
        K r = red[q][0];
        for (int i = 1; i < 4; ++i) r = q < 3 ? (red[q][i] < r ? red[q][i] : r) : (red[q][i] > r ? red[q][i] : r);
        ext[q] = r;
    }
}

// segments that sort (info.ok), split by size: up to SMALL_SEG members sort inside one
// workgroup (k_seg_sort_small), larger ones go through the device-wide radix sort
constexpr uint32_t SMALL_SEG = 4096;
__global__ void k_seg_flags(const SegInfo *__restrict__ info, const uint32_t *__restrict__ seg_len, uint32_t nseg,
                            uint32_t *__restrict__ flag, uint32_t *__restrict__ mlen, uint32_t *__restrict__ sflag) {
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x) {
        const uint32_t ok = info[s].ok, len = seg_len[s];
        const uint32_t big = ok && len > SMALL_SEG;
        flag[s] = big;
        mlen[s] = big ? len : 0u;
        sflag[s] = ok && !big;
    }
}

// the small sorting segments: start, length, info
__global__ void k_seg_compact_small(const uint32_t *__restrict__ sflag, const uint32_t *__restrict__ spos,
                                    const uint32_t *__restrict__ seg_start, const uint32_t *__restrict__ seg_len,
                                    const SegInfo *__restrict__ info, uint32_t nseg, uint32_t *__restrict__ sstart,
                                    uint32_t *__restrict__ slen, SegInfo *__restrict__ sinfo) {
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x)
        if (sflag[s]) {
            const uint32_t q = spos[s];
            sstart[q] = seg_start[s];
            slen[q] = seg_len[s];
            sinfo[q] = info[s];
        }
}

// the sorting segments only (ordering.ts:53-61 returns before sorting the others): their
// starts, element offsets and infos, in order
__global__ void k_seg_compact(const uint32_t *__restrict__ flag, const uint32_t *__restrict__ pos,
                              const uint32_t *__restrict__ seg_start, const uint32_t *__restrict__ moff,
                              const SegInfo *__restrict__ info, uint32_t nseg, uint32_t *__restrict__ cstart,
                              uint32_t *__restrict__ coff, SegInfo *__restrict__ cinfo) {
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x)
        if (flag[s]) {
            const uint32_t q = pos[s];
            cstart[q] = seg_start[s];
            coff[q] = moff[s];
            cinfo[q] = info[s];
        }
}

// ordering.ts:32-65 per segment
// (level 0: seg_start null, the one segment starts at 0); also zeroes the level's big-run counts
template <typename T>
__global__ void k_seg_info(const T *__restrict__ x, const T *__restrict__ y, const T *__restrict__ z,
                           const uint32_t *__restrict__ idx, const uint32_t *__restrict__ seg_start,
                           const typename MC<T>::K *__restrict__ ext, uint32_t nseg, SegInfo *info,
                           uint32_t *bigcnt) {
    if (blockIdx.x == 0 && threadIdx.x < 2) bigcnt[threadIdx.x] = 0;  // big runs of both sort paths
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x) {
        const uint32_t first = idx[seg_start ? seg_start[s] : 0u];
        const T f[3] = {x[first], y[first], z[first]};
        SegInfo si{};
        bool valid = true, all_zero = true;
        for (int a = 0; a < 3; ++a) {
            double len;
            if (f[a] != f[a] || ext[s * 6 + a] == MC<T>::KMAX) {
                len = __builtin_nan("");  // NaN first element -> extents NaN (ordering.ts:38-41)
            } else {
                const double lo = MC<T>::inv(ext[s * 6 + a]), hi = MC<T>::inv(ext[s * 6 + 3 + a]);
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

template <typename T>
__device__ inline uint32_t axis_q(T v, double mn, double mul) {
    return js::to_uint32(js::min_(1023, ((double)v - mn) * mul));
}

template <typename K, typename T>
__global__ __launch_bounds__(256) void k_keys(const uint32_t *__restrict__ idx,
                                              const uint32_t *__restrict__ P, const uint32_t *__restrict__ S,
                                              const SegInfo *__restrict__ info, uint64_t total,
                                              const typename MC<T>::V *__restrict__ cxyz, K *__restrict__ keys,
                                              uint32_t *__restrict__ vals) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += stride) {
        const uint32_t p = P[j];
        const uint32_t s = S[j];
        const uint32_t row = idx[p];
        const SegInfo &si = info[s];
        uint32_t m = 0;
        if (si.ok) {
            const typename MC<T>::V v = cxyz[p];
            const uint32_t ix = axis_q(v.x, si.mn[0], si.mul[0]);
            const uint32_t iy = axis_q(v.y, si.mn[1], si.mul[1]);
            const uint32_t iz = axis_q(v.z, si.mn[2], si.mul[2]);
            m = (part1by2(iz) << 2) + (part1by2(iy) << 1) + part1by2(ix);
        }
        keys[j] = ((K)s << 30) | (K)m;
        vals[j] = row;
    }
}

// level 0: one segment, P = identity -- keys only (the sort takes idx itself as its values) and
// the first radix digit's count per sort tile (RADIX_TILE keys per workgroup), so the sort
// skips its first histogram pass
template <typename T>
__global__ __launch_bounds__(256) void k_keys0(const T *__restrict__ x, const T *__restrict__ y,
                                               const T *__restrict__ z, const uint32_t *__restrict__ idx,
                                               const SegInfo *__restrict__ info, uint64_t n,
                                               uint32_t *__restrict__ keys, uint32_t *__restrict__ hist,
                                               uint32_t ntiles) {
    constexpr int ROWS = RADIX_TILE / 256;
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const SegInfo si = info[0];
    const uint64_t base = (uint64_t)blockIdx.x * RADIX_TILE;
    uint32_t rows_[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
        const uint64_t j = base + (uint64_t)r * 256 + threadIdx.x;
        rows_[r] = j < n ? idx[j] : 0u;
    }
#pragma unroll 4
    for (int r = 0; r < ROWS; ++r) {
        const uint64_t j = base + (uint64_t)r * 256 + threadIdx.x;
        if (j >= n) break;
        const uint32_t row = rows_[r];
        uint32_t m = 0;
        if (si.ok) {
            const uint32_t ix = axis_q(x[row], si.mn[0], si.mul[0]);
            const uint32_t iy = axis_q(y[row], si.mn[1], si.mul[1]);
            const uint32_t iz = axis_q(z[row], si.mn[2], si.mul[2]);
            m = (part1by2(iz) << 2) + (part1by2(iy) << 1) + part1by2(ix);
        }
        keys[j] = m;
        atomicAdd(&h[m & 255u], 1u);
    }
    __syncthreads();
    hist[(uint64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// one workgroup per small segment (257..SMALL_SEG members, contiguous positions in idx): keys
// from the level's gathered coordinates, a stable 4-pass LSD radix sort with the elements in
// registers between passes (wave ballots rank each 64-element row, as the device-wide
// scatter does; LDS only for the reordering), the order written back into idx, and the
// segment's own runs of > 256 equal keys appended to the next level's list
template <typename T>
__global__ __launch_bounds__(256) void k_seg_sort_small(const uint32_t *__restrict__ sstart,
                                                        const uint32_t *__restrict__ slen,
                                                        const SegInfo *__restrict__ sinfo, uint32_t nsmall,
                                                        const typename MC<T>::V *__restrict__ cxyz,
                                                        uint32_t *__restrict__ idx,
                                                        uint32_t *__restrict__ ostart, uint32_t *__restrict__ olen,
                                                        uint32_t *__restrict__ ocnt) {
    constexpr int ROWS = SMALL_SEG / 256;
    __shared__ uint32_t kL[SMALL_SEG], vL[SMALL_SEG];
    __shared__ uint32_t wcount[4][256], wbase[4][256], dstart[256], wtot[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (uint32_t sg = blockIdx.x; sg < nsmall; sg += gridDim.x) {
        const uint32_t start = sstart[sg], len = slen[sg];
        const SegInfo si = sinfo[sg];
        // R rows of 64 per wave, wave w owning rows [w R, w R + R): contiguous element ranges per
        // wave keep the ranking stable, and no wave ranks rows past the segment's end
        const uint32_t R = ((len + 63) / 64 + 3) / 4;
        uint32_t k[ROWS], v[ROWS];
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            if ((uint32_t)r >= R) continue;
            const uint32_t e = (w * R + r) * 64 + lane;
            k[r] = 0u;
            v[r] = 0u;
            if (e < len) {
                const typename MC<T>::V cv = cxyz[start + e];
                const uint32_t ix = axis_q(cv.x, si.mn[0], si.mul[0]);
                const uint32_t iy = axis_q(cv.y, si.mn[1], si.mul[1]);
                const uint32_t iz = axis_q(cv.z, si.mn[2], si.mul[2]);
                k[r] = (part1by2(iz) << 2) + (part1by2(iy) << 1) + part1by2(ix);
                v[r] = idx[start + e];
            }
        }
        for (int pass = 0; pass < 4; ++pass) {
            const int shift = 8 * pass, bits = pass == 3 ? 6 : 8;
            for (int i = threadIdx.x; i < 4 * 256; i += 256) (&wcount[0][0])[i] = 0;
            __syncthreads();
            uint32_t off[ROWS], dg[ROWS];
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
                if ((uint32_t)r >= R) continue;
                const uint32_t e = (w * R + r) * 64 + lane;
                const bool valid = e < len;
                const uint32_t d = (k[r] >> shift) & 255u;
                dg[r] = d;
                uint64_t peers = __ballot(valid);
                for (int b = 0; b < bits; ++b) {
                    const bool bit = (d >> b) & 1u;
                    const uint64_t bb = __ballot(bit);
                    peers &= bit ? bb : ~bb;
                }
                const uint32_t before = valid ? wcount[w][d] : 0u;
                off[r] = before + (uint32_t)__popcll(peers & lt);
                if (valid && (peers & lt) == 0) wcount[w][d] = before + (uint32_t)__popcll(peers);
                __builtin_amdgcn_wave_barrier();
            }
            __syncthreads();
            {
                const int d = threadIdx.x;
                uint32_t tot = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    wbase[i][d] = tot;
                    tot += wcount[i][d];
                }
                uint32_t incl = tot;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t u = __shfl_up(incl, o, 64);
                    if (lane >= o) incl += u;
                }
                if (lane == 63) wtot[w] = incl;
                __syncthreads();
                uint32_t woff = 0;
                for (int i = 0; i < w; ++i) woff += wtot[i];
                dstart[d] = woff + incl - tot;
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
                if ((uint32_t)r >= R) continue;
                const uint32_t e = (w * R + r) * 64 + lane;
                if (e < len) {
                    const uint32_t lp = dstart[dg[r]] + wbase[w][dg[r]] + off[r];
                    kL[lp] = k[r];
                    vL[lp] = v[r];
                }
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
                if ((uint32_t)r >= R) continue;
                const uint32_t e = (w * R + r) * 64 + lane;
                if (e < len) {
                    k[r] = kL[e];
                    v[r] = vL[e];
                }
            }
            __syncthreads();
        }
        // kL holds the sorted keys: write the order, then the segment's own big runs
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            if ((uint32_t)r >= R) continue;
            const uint32_t e = (w * R + r) * 64 + lane;
            if (e < len) {
                idx[start + e] = v[r];
                if (e + 256 < len && kL[e + 256] == k[r] && (e == 0 || kL[e - 1] != k[r])) {
                    uint32_t end = e + 257;
                    while (end < len && kL[end] == k[r]) ++end;
                    const uint32_t slot = atomicAdd(ocnt, 1u);
                    ostart[slot] = start + e;
                    olen[slot] = end - e;
                }
            }
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_scatter_back(const uint32_t *__restrict__ P, const uint32_t *__restrict__ vals,
                                                      uint64_t total, uint32_t *__restrict__ idx) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += stride)
        idx[P[j]] = vals[j];
}





__global__ void k_set_sentinel(uint32_t *a, uint32_t i, uint32_t v) { a[i] = v; }

// Runs of equal keys longer than 256 (ordering.ts:90-104) without listing every run: j
// starts such a run iff it starts a run and keys[j + 256] == keys[j] (the keys are sorted).
// Their order in the next level's segment list is immaterial: a segment's rows go back to
// their own positions.
template <typename K>
__global__ __launch_bounds__(256) void k_big_starts(const K *__restrict__ keys, uint64_t total,
                                                    const SegInfo *__restrict__ info, uint32_t *__restrict__ starts,
                                                    uint32_t *__restrict__ count) {
    // a block's 4,096 positions hold at most 16 starts: ranked in LDS, appended with one
    // global atomic per block (one per start serialised on the counter: 0.23 ms at 20k runs)
    __shared__ uint32_t nloc, base;
    if (threadIdx.x == 0) nloc = 0;
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * 4096;
    uint32_t slot[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint64_t j = b0 + (uint64_t)r * 256 + threadIdx.x;
        slot[r] = 0xffffffffu;
        if (j + 256 < total) {
            const K k = keys[j];
            if (keys[j + 256] == k && (j == 0 || keys[j - 1] != k) && info[(uint32_t)(k >> 30)].ok)
                slot[r] = atomicAdd(&nloc, 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) base = nloc ? atomicAdd(count, nloc) : 0u;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r)
        if (slot[r] != 0xffffffffu) starts[base + slot[r]] = (uint32_t)(b0 + (uint64_t)r * 256 + threadIdx.x);
}

// end of each big run by binary search (first position past j whose key differs), then the
// next level's segment (start position in idx, length)
template <typename K>
__global__ __launch_bounds__(256) void k_big_segs(const K *__restrict__ keys, uint64_t total,
                                                  const uint32_t *__restrict__ starts, const uint32_t *__restrict__ count,
                                                  const uint32_t *__restrict__ P, int single,
                                                  uint32_t *__restrict__ nstart, uint32_t *__restrict__ nlen) {
    const uint32_t nb = *count;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += gridDim.x * blockDim.x) {
        const uint32_t j = starts[i];
        const K k = keys[j];
        uint64_t lo = (uint64_t)j + 257, hi = total;  // keys[j + 256] == k
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (keys[mid] == k) lo = mid + 1;
            else hi = mid;
        }
        nstart[i] = single ? j : P[j];
        nlen[i] = (uint32_t)(lo - j);
    }
}

template <typename T>
void morton_order_impl(st_ctx *c, const T *x, const T *y, const T *z, uint32_t *idx, uint64_t n) {
    using K = typename MC<T>::K;
    using V = typename MC<T>::V;
    if (n == 0) return;
    ST_REQUIRE(n < (1ull << 32) - 1, ST_ERR_ARG, "morton: n must be < 2^32-1");
    auto *h = static_cast<uint32_t *>(pinned(c, 64));
    // active segment list (level 0's single segment is implicit)
    auto *seg_start = wsT<uint32_t>(c, "mo.seg_start", n / 257 + 2);
    auto *seg_len = wsT<uint32_t>(c, "mo.seg_len", n / 257 + 2);
    auto *nseg_start = wsT<uint32_t>(c, "mo.nseg_start", n / 257 + 2);
    auto *nseg_len = wsT<uint32_t>(c, "mo.nseg_len", n / 257 + 2);
    auto *seg_off = wsT<uint32_t>(c, "mo.seg_off", n / 257 + 3);
    uint32_t nseg = 1;
    uint64_t total = n;
    auto *P = wsT<uint32_t>(c, "mo.P", n);
    auto *S = wsT<uint32_t>(c, "mo.S", n);
    auto *vals = wsT<uint32_t>(c, "mo.vals", n);
    auto *bigpos = wsT<uint32_t>(c, "mo.bigpos", n / 257 + 2);  // starts of runs longer than 256
    auto *bigcnt = wsT<uint32_t>(c, "mo.bigcnt", 2);  // [0] device-wide sort, [1] small segments
    auto *sm_start = wsT<uint32_t>(c, "mo.sm_start", n / 257 + 2);  // the small segments' big runs
    auto *sm_len = wsT<uint32_t>(c, "mo.sm_len", n / 257 + 2);
    V *cxyz = nullptr;  // deeper levels: x / y / z gathered by k_ext_seg, at idx positions
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
        }  // level 0: P = identity, S = 0, never materialised
        auto *ext = wsT<K>(c, "mo.ext", (size_t)nseg * 6);
        auto *info = static_cast<SegInfo *>(ws(c, "mo.info", sizeof(SegInfo) * (size_t)nseg));
        const unsigned eb = (unsigned)((total + 4095) / 4096);
        if (single) {
            auto *part = wsT<K>(c, "mo.extpart", (size_t)eb * 6);
            hipLaunchKernelGGL(k_ext<T>, dim3(eb), dim3(256), 0, c->stream, x, y, z, idx, total, part);
            hipLaunchKernelGGL(k_ext_final<K>, dim3(1), dim3(256), 0, c->stream, part, eb, ext);
        } else {
            if (!cxyz) cxyz = wsT<V>(c, "mo.cxyz", n);
            hipLaunchKernelGGL(k_ext_init<K>, dim3(grid_for(nseg, 256, 1024)), dim3(256), 0, c->stream, ext, nseg);
            hipLaunchKernelGGL(k_ext_seg<T>, dim3(eb), dim3(256), 0, c->stream, x, y, z, idx, P, S, total, ext, cxyz);
        }
        ST_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_seg_info<T>, dim3(grid_for(nseg, 64, 1024)), dim3(64), 0, c->stream, x, y, z, idx,
                           single ? nullptr : seg_start, ext, nseg, info, bigcnt);
        ST_LAUNCH_CHECK();
        bool large = true;  // the device-wide sort has members at this level
        if (!single) {
            // only segments with usable extents are keyed and sorted: the others keep their order
            // and never recurse (ordering.ts:53-61), so their members leave the level here.  Small
            // ones sort inside one workgroup each; large ones keep the device-wide sort below
            auto *flag = wsT<uint32_t>(c, "mo.flag", n / 257 + 2);
            auto *pos = wsT<uint32_t>(c, "mo.pos", n / 257 + 3);
            auto *mlen = wsT<uint32_t>(c, "mo.mlen", n / 257 + 2);
            auto *moff = wsT<uint32_t>(c, "mo.moff", n / 257 + 3);
            auto *sflag = wsT<uint32_t>(c, "mo.sflag", n / 257 + 2);
            auto *spos = wsT<uint32_t>(c, "mo.spos", n / 257 + 3);
            hipLaunchKernelGGL(k_seg_flags, dim3(grid_for(nseg, 256, 1024)), dim3(256), 0, c->stream, info, seg_len,
                               nseg, flag, mlen, sflag);
            ST_LAUNCH_CHECK();
            scan_u32(c, flag, pos, nseg, pos + nseg);
            scan_u32(c, mlen, moff, nseg, moff + nseg);
            scan_u32(c, sflag, spos, nseg, spos + nseg);
            ST_HIP(hipMemcpyAsync(h + 1, pos + nseg, 4, hipMemcpyDeviceToHost, c->stream));
            ST_HIP(hipMemcpyAsync(h + 2, moff + nseg, 4, hipMemcpyDeviceToHost, c->stream));
            ST_HIP(hipMemcpyAsync(h + 3, spos + nseg, 4, hipMemcpyDeviceToHost, c->stream));
            ST_HIP(hipStreamSynchronize(c->stream));
            const uint32_t kept = h[1], nsmall = h[3];
            if (kept == 0 && nsmall == 0) break;
            if (nsmall) {
                auto *sstart = wsT<uint32_t>(c, "mo.sstart", n / 257 + 2);
                auto *slen = wsT<uint32_t>(c, "mo.slen", n / 257 + 2);
                auto *sinfo = static_cast<SegInfo *>(ws(c, "mo.sinfo", sizeof(SegInfo) * (size_t)nsmall));
                hipLaunchKernelGGL(k_seg_compact_small, dim3(grid_for(nseg, 256, 1024)), dim3(256), 0, c->stream,
                                   sflag, spos, seg_start, seg_len, info, nseg, sstart, slen, sinfo);
                hipLaunchKernelGGL(k_seg_sort_small<T>, dim3(std::min<uint32_t>(nsmall, 4096)), dim3(256), 0, c->stream,
                                   sstart, slen, sinfo, nsmall, cxyz, idx, sm_start, sm_len, bigcnt + 1);
                ST_LAUNCH_CHECK();
            }
            large = kept > 0;
            if (large && kept < nseg) {
                auto *cstart = wsT<uint32_t>(c, "mo.cstart", n / 257 + 2);
                auto *cinfo = static_cast<SegInfo *>(ws(c, "mo.cinfo", sizeof(SegInfo) * (size_t)kept));
                hipLaunchKernelGGL(k_seg_compact, dim3(grid_for(nseg, 256, 1024)), dim3(256), 0, c->stream, flag, pos,
                                   seg_start, moff, info, nseg, cstart, seg_off, cinfo);
                total = h[2];
                nseg = kept;
                info = cinfo;
                // (seg_start is not read again this level: the next level's list comes from P)
                hipLaunchKernelGGL(k_expand, dim3(grid_for(total, 256, 8192)), dim3(256), 0, c->stream, cstart,
                                   seg_off, nseg, total, P, S);
                ST_LAUNCH_CHECK();
            }
        }
        int seg_bits = 0;
        while ((1u << seg_bits) < nseg) ++seg_bits;
        const unsigned g = grid_for(total, 256, 8192);
        if (!large) {
            // every sorting segment of this level was small
        } else if (single) {
            // keys + first digit counts, then the sort reads idx as its values and its last
            // (fourth) pass writes the ordered rows straight back into idx
            const uint32_t nt = radix_tiles(n);
            auto *keys = wsT<uint32_t>(c, "mo.k32", n + 1);
            auto *hist = wsT<uint32_t>(c, "mo.hist0", (size_t)256 * nt);
            hipLaunchKernelGGL(k_keys0<T>, dim3(nt), dim3(256), 0, c->stream, x, y, z, idx, info, n, keys, hist, nt);
            ST_LAUNCH_CHECK();
            radix_sort_u32_from(c, keys, idx, n, 0, 30, keys, idx, hist, "mo.rs32");
            hipLaunchKernelGGL(k_big_starts<uint32_t>, dim3((unsigned)((total + 4095) / 4096)), dim3(256), 0, c->stream, keys, total, info, bigpos,
                               bigcnt);
            hipLaunchKernelGGL(k_big_segs<uint32_t>, dim3(grid_for(total / 257 + 1, 256, 1024)), dim3(256), 0,
                               c->stream, keys, total, bigpos, bigcnt, P, 1, nseg_start, nseg_len);
            ST_LAUNCH_CHECK();
        } else if (seg_bits + 30 <= 32) {
            auto *keys = wsT<uint32_t>(c, "mo.k32", total + 1);
            hipLaunchKernelGGL((k_keys<uint32_t, T>), dim3(g), dim3(256), 0, c->stream, idx, P, S, info, total,
                               cxyz, keys, vals);
            ST_LAUNCH_CHECK();
            uint32_t *skeys = keys, *svals = vals;
            radix_sort_u32_inplace_or_swap(c, keys, vals, total, 0, 30 + seg_bits, "mo.rs32", &skeys, &svals);
            hipLaunchKernelGGL(k_scatter_back, dim3(g), dim3(256), 0, c->stream, P, svals, total, idx);
            hipLaunchKernelGGL(k_big_starts<uint32_t>, dim3((unsigned)((total + 4095) / 4096)), dim3(256), 0, c->stream, skeys, total, info, bigpos,
                               bigcnt);
            hipLaunchKernelGGL(k_big_segs<uint32_t>, dim3(grid_for(total / 257 + 1, 256, 1024)), dim3(256), 0,
                               c->stream, skeys, total, bigpos, bigcnt, P, 0, nseg_start, nseg_len);
            ST_LAUNCH_CHECK();
        } else {
            auto *keys = wsT<uint64_t>(c, "mo.k64", total + 1);
            hipLaunchKernelGGL((k_keys<uint64_t, T>), dim3(g), dim3(256), 0, c->stream, idx, P, S, info, total,
                               cxyz, keys, vals);
            ST_LAUNCH_CHECK();
            radix_sort_u64(c, keys, vals, total, 0, 30 + seg_bits, "mo.rs64");
            hipLaunchKernelGGL(k_scatter_back, dim3(g), dim3(256), 0, c->stream, P, vals, total, idx);
            hipLaunchKernelGGL(k_big_starts<uint64_t>, dim3((unsigned)((total + 4095) / 4096)), dim3(256), 0, c->stream, keys, total, info, bigpos,
                               bigcnt);
            hipLaunchKernelGGL(k_big_segs<uint64_t>, dim3(grid_for(total / 257 + 1, 256, 1024)), dim3(256), 0,
                               c->stream, keys, total, bigpos, bigcnt, P, 0, nseg_start, nseg_len);
            ST_LAUNCH_CHECK();
        }
        // next level: the device-wide sort's big runs, then the small segments' ones
        ST_HIP(hipMemcpyAsync(h + 4, bigcnt, 8, hipMemcpyDeviceToHost, c->stream));
        ST_HIP(hipStreamSynchronize(c->stream));
        const uint32_t nl = h[4], ns = h[5];
        if (ns) {
            ST_HIP(hipMemcpyAsync(nseg_start + nl, sm_start, 4ull * ns, hipMemcpyDeviceToDevice, c->stream));
            ST_HIP(hipMemcpyAsync(nseg_len + nl, sm_len, 4ull * ns, hipMemcpyDeviceToDevice, c->stream));
        }
        nseg = nl + ns;
        std::swap(seg_start, nseg_start);
        std::swap(seg_len, nseg_len);
    }
}

}  // namespace

void morton_order_dev(st_ctx *c, const float *x, const float *y, const float *z, uint32_t *idx, uint64_t n) {
    morton_order_impl<float>(c, x, y, z, idx, n);
}

void morton_order_dev_f64(st_ctx *c, const double *x, const double *y, const double *z, uint32_t *idx, uint64_t n) {
    morton_order_impl<double>(c, x, y, z, idx, n);
}

// generateOrdering over x / y / z columns of any type: ordering.ts:32-47 reads them as JS
// numbers, so float32 columns take the float32 path and any other type (or a mix) the float64
// one, whose values are the exact JS numbers of every type
void morton_order_tdev(st_ctx *c, const void *const xyz[3], const int32_t types[3], uint32_t *idx, uint64_t n) {
    if (types[0] == ST_PLY_FLOAT && types[1] == ST_PLY_FLOAT && types[2] == ST_PLY_FLOAT) {
        morton_order_impl<float>(c, static_cast<const float *>(xyz[0]), static_cast<const float *>(xyz[1]),
                                 static_cast<const float *>(xyz[2]), idx, n);
        return;
    }
    const double *d[3];
    for (int a = 0; a < 3; ++a) d[a] = as_f64_dev(c, TCol{const_cast<void *>(xyz[a]), types[a]}, n, "mo.f64." + std::to_string(a));
    morton_order_impl<double>(c, d[0], d[1], d[2], idx, n);
}

}  // namespace st
