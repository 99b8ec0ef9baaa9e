// st_kmeans.hip -- kmeans() on the --no-gpu semantics (k-means.ts:137-201).
//
// Parity target: labels = exact nearest centroid under the reference's f64
// distance with the KdTree's traversal tie-break (kd-tree.ts:22-71), means =
// f64 running sums in ascending point order (calcAverage, k-means.ts:41-63),
// empty clusters re-seeded from the caller's Math.random stream in ascending
// cluster order, labels from the last assign and centroids after the last
// update.
//
// Assign, D == 1: the KdTree over 1-D centroids is the implicit BST over the
//   stably sorted centroid values, so every point walks it exactly as
//   findNearest does (same pruning, same tie-break).
// Assign, D > 1 (SH palette, K up to 65,536): score(c) = |c|^2 - 2 p.c on the
//   matrix cores as a bf16x3 split GEMM (v_mfma_f32_32x32x16_bf16, K-dim
//   3*roundup(D+3,16)), a running top-2 per point in the epilogue, and a
//   rigorous per-point error bound W_p.  A point whose runner-up is > W_p
//   behind is decided; the rest (~1%) gather every centroid within W_p and
//   resolve them with the reference's exact f64 distance; exact ties go to a
//   KdTree traversal (st_kdtree.hip).
// Update: stable radix sort of (label, point) gives each cluster its members
//   in ascending order; 1-D clusters sum in parallel when an exactness
//   certificate proves every partial sum is representable (then any order
//   equals the sequential sum), otherwise sequentially.
#include "st_internal.h"
#include "st_jsmath.h"
#include "st_kmeans.h"

namespace st {
namespace km {

// ---------------------------------------------------------------------------
// common kernels

__global__ __launch_bounds__(256) void k_nonfinite(const float *const *cols, int d, uint64_t n, uint32_t *flag) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t bad = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        for (int c = 0; c < d; ++c) bad |= js::isfinitef_(cols[c][i]) ? 0u : 1u;
    if (__ballot(bad) != 0 && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
}

// the same test and max |x| in one pass: 4 rows per thread (float4), 8 columns' loads in
// flight, one atomic per workgroup
struct ScanCols {
    const float *p[64];
};
__global__ __launch_bounds__(256) void k_scan_cols(const ScanCols cp, int d, uint64_t n, uint32_t *flag,
                                                   uint32_t *amax_bits) {
    const uint64_t nq = n / 4;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t bad = 0;
    float m = 0.f;
    auto take = [&](float v) {
        bad |= js::isfinitef_(v) ? 0u : 1u;
        m = __builtin_fmaxf(m, __builtin_fabsf(v));
    };
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += stride) {
        int c = 0;
        for (; c + 8 <= d; c += 8) {
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = reinterpret_cast<const float4 *>(cp.p[c + u])[q];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                take(v[u].x);
                take(v[u].y);
                take(v[u].z);
                take(v[u].w);
            }
        }
        for (; c < d; ++c) {
            const float4 v = reinterpret_cast<const float4 *>(cp.p[c])[q];
            take(v.x);
            take(v.y);
            take(v.z);
            take(v.w);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < n % 4)
        for (int c = 0; c < d; ++c) take(cp.p[c][nq * 4 + threadIdx.x]);
    __shared__ uint32_t sb[4];
    __shared__ float sm[4];
    for (int o = 32; o > 0; o >>= 1) {
        bad |= __shfl_xor(bad, o, 64);
        m = __builtin_fmaxf(m, __shfl_xor(m, o, 64));
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sb[w] = bad;
        sm[w] = m;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        bad = sb[0] | sb[1] | sb[2] | sb[3];
        m = __builtin_fmaxf(__builtin_fmaxf(sm[0], sm[1]), __builtin_fmaxf(sm[2], sm[3]));
        if (bad) atomicOr(flag, 1u);
        atomicMax(amax_bits, __builtin_bit_cast(uint32_t, m));  // non-negative floats order as their bits
    }
}

// initializeCentroids1D (k-means.ts:23-39): linspace over [min, max] (keys from minmax_keys_dev)
__global__ void k_init1d(const uint32_t *mm, float *cen, int k) {
    const double m = fkey_inv_(mm[0]), M = fkey_inv_(mm[1]);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < k; i += gridDim.x * blockDim.x)
        cen[i] = (float)(m + (M - m) * i / (k - 1));
}

// centroids[c][i] = points[c][rows[i]]
__global__ __launch_bounds__(256) void k_gather_init(const float *const *cols, int d, const uint32_t *rows, int k,
                                                     float *cen) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < k; i += gridDim.x * blockDim.x) {
        const uint32_t r = rows[i];
        for (int c = 0; c < d; ++c) cen[(uint64_t)c * k + i] = cols[c][r];
    }
}

// initializeCentroids (k-means.ts:8-20) on the device: row floor(draw * n) of draw i is
// taken iff no earlier draw chose it, until k rows are taken.  first[row] = the earliest
// draw choosing it (first[] preset to ~0); draw i is a taking iff first[row_i] == i, and
// its rank among the takings (an exclusive scan) is its centroid slot.
__device__ inline uint32_t init_row(const double *draws, uint32_t i, uint64_t n) {  // ~0: outside the table
    const double f = __builtin_floor(draws[i] * (double)n);
    return (f >= 0.0 && f < (double)n) ? (uint32_t)f : 0xffffffffu;
}
__global__ __launch_bounds__(256) void k_init_first(const double *__restrict__ draws, uint32_t m, uint64_t n,
                                                    uint32_t *__restrict__ first, State *st) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const uint32_t r = init_row(draws, i, n);
        if (r < n)
            atomicMin(&first[r], i);
        else
            atomicOr(&st->err, ERR_INIT_WINDOW);  // a draw outside [0, 1): the host loop reports it
    }
}
__global__ __launch_bounds__(256) void k_init_flags(const double *__restrict__ draws, uint32_t m, uint64_t n,
                                                    const uint32_t *__restrict__ first, uint32_t *__restrict__ flags) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const uint32_t r = init_row(draws, i, n);
        flags[i] = (r < n && first[r] == i) ? 1u : 0u;
    }
}
__global__ __launch_bounds__(256) void k_init_select(const double *__restrict__ draws, uint32_t m, uint64_t n, int k,
                                                     const uint32_t *__restrict__ flags, const uint32_t *__restrict__ pos,
                                                     uint32_t *__restrict__ rows, State *st) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        if (!flags[i] || pos[i] >= (uint32_t)k) continue;
        rows[pos[i]] = init_row(draws, i, n);
        if (pos[i] == (uint32_t)k - 1) st->cursor = (uint64_t)i + 1;  // draws consumed
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && pos[m] < (uint32_t)k) st->err |= ERR_INIT_WINDOW;
}

// out[c][i] = the local row rows[i] - offset of column c where this rank holds it, bit
// pattern 0 elsewhere (an integer SUM over the ranks then assembles every row exactly)
__global__ __launch_bounds__(256) void k_gather_owned(const float *const *cols, int d, uint64_t n_local,
                                                      uint64_t offset, const uint32_t *__restrict__ rows, int k,
                                                      float *__restrict__ out) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < k; i += gridDim.x * blockDim.x) {
        const uint64_t r = rows[i];
        const bool mine = r >= offset && r - offset < n_local;
        for (int c = 0; c < d; ++c) out[(uint64_t)c * k + i] = mine ? cols[c][r - offset] : 0.0f;
    }
}

// ---------------------------------------------------------------------------
// update: cluster boundaries in the label-sorted member list
__global__ __launch_bounds__(256) void k_bounds(const uint32_t *__restrict__ sorted_labels, uint64_t n, int k,
                                                uint32_t *__restrict__ start) {
    // start[c] = first position with label >= c ; start[k] = n
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c <= k; c += gridDim.x * blockDim.x) {
        uint64_t lo = 0, hi = n;
        while (lo < hi) {
            uint64_t mid = (lo + hi) >> 1;
            if (sorted_labels[mid] < (uint32_t)c) lo = mid + 1; else hi = mid;
        }
        start[c] = (uint32_t)lo;
    }
}

// re-seed empty clusters (k-means.ts:174-178): the j-th empty cluster (ascending)
// takes draw cursor+j; rank comes from an exclusive scan of the empty flags
__global__ __launch_bounds__(256) void k_empty_flags(const uint32_t *start, int k, uint32_t *flags) {
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < k; c += gridDim.x * blockDim.x)
        flags[c] = (start[c + 1] == start[c]) ? 1u : 0u;
}

__global__ __launch_bounds__(256) void k_reseed(const float *const *cols, int d, uint64_t n, int k,
                                                const uint32_t *flags, const uint32_t *rank, const double *draws,
                                                uint64_t ndraws, State *st, float *cen) {
    const uint64_t cursor = st->cursor;
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < k; c += gridDim.x * blockDim.x) {
        if (!flags[c]) continue;
        const uint64_t di = cursor + rank[c];
        if (di >= ndraws) {
            atomicOr(&st->err, ERR_DRAWS);
            continue;
        }
        const double dr = draws[di];
        if (!(dr >= 0.0 && dr < 1.0)) {  // a Math.random draw outside [0, 1): no row to read
            atomicOr(&st->err, ERR_DRAW_RANGE);
            continue;
        }
        const uint64_t row = (uint64_t)__builtin_floor(dr * (double)n);
        for (int j = 0; j < d; ++j) cen[(uint64_t)j * k + c] = cols[j][row];
    }
}

__global__ void k_advance_cursor(State *st, const uint32_t *total_empty) { st->cursor += *total_empty; }

// k_reseed_small from member counts for any k: one 1,024-thread workgroup, each thread a run of
// consecutive clusters (the j-th empty cluster in ascending order takes draw cursor + j)
constexpr int RC_T = 1024;
__global__ __launch_bounds__(RC_T) void k_reseed_counts(const float *const *cols, int d, uint64_t n, int k,
                                                        const uint32_t *__restrict__ counts,
                                                        const double *__restrict__ draws, uint64_t ndraws, State *st,
                                                        float *__restrict__ cen) {
    __shared__ uint32_t wsum[RC_T / 64];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int per = (k + RC_T - 1) / RC_T;
    const int a = min(k, t * per), b = min(k, a + per);
    uint32_t mine = 0;
    for (int c = a; c < b; ++c) mine += counts[c] == 0u ? 1u : 0u;
    uint32_t incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t off = 0, total = 0;
    for (int i = 0; i < RC_T / 64; ++i) {
        if (i < w) off += wsum[i];
        total += wsum[i];
    }
    const uint64_t cursor = st->cursor;
    uint32_t rank = off + incl - mine;
    for (int c = a; c < b && mine; ++c) {
        if (counts[c] != 0u) continue;
        const uint64_t di = cursor + rank++;
        if (di >= ndraws) {
            atomicOr(&st->err, ERR_DRAWS);
            continue;
        }
        const double dr = draws[di];
        if (!(dr >= 0.0 && dr < 1.0)) {
            atomicOr(&st->err, ERR_DRAW_RANGE);
            continue;
        }
        const uint64_t row = (uint64_t)__builtin_floor(dr * (double)n);
        for (int j = 0; j < d; ++j) cen[(uint64_t)j * k + c] = cols[j][row];
    }
    __syncthreads();  // every thread has read st->cursor
    if (t == 0) st->cursor = cursor + total;
}

__global__ __launch_bounds__(256) void k_empty_flags_cnt(const uint32_t *counts, int k, uint32_t *flags) {
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < k; c += gridDim.x * blockDim.x)
        flags[c] = counts[c] == 0u ? 1u : 0u;
}

// the three steps above in one workgroup for k <= RS1_MAX (the 1-D codebooks, k = 256):
// empty flags, their exclusive scan in LDS, the re-seeds, the cursor
constexpr int RS1_T = 1024, RS1_MAX = 4096;
__global__ __launch_bounds__(RS1_T) void k_reseed_small(const float *const *cols, int d, uint64_t n, int k,
                                                        const uint32_t *__restrict__ start,
                                                        const double *__restrict__ draws, uint64_t ndraws, State *st,
                                                        float *__restrict__ cen) {
    constexpr int PER = RS1_MAX / RS1_T;
    __shared__ uint32_t wsum[RS1_T / 64];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t f[PER], mine = 0;
#pragma unroll
    for (int u = 0; u < PER; ++u) {  // thread t owns clusters t*PER .. t*PER+PER-1 (ascending)
        const int c = t * PER + u;
        f[u] = (c < k && start[c + 1] == start[c]) ? 1u : 0u;
        mine += f[u];
    }
    uint32_t incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t off = 0, total = 0;
    for (int i = 0; i < RS1_T / 64; ++i) {
        if (i < w) off += wsum[i];
        total += wsum[i];
    }
    const uint64_t cursor = st->cursor;
    uint32_t rank = off + incl - mine;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        if (!f[u]) continue;
        const int c = t * PER + u;
        const uint64_t di = cursor + rank++;
        if (di >= ndraws) {
            atomicOr(&st->err, ERR_DRAWS);
            continue;
        }
        const double dr = draws[di];
        if (!(dr >= 0.0 && dr < 1.0)) {
            atomicOr(&st->err, ERR_DRAW_RANGE);
            continue;
        }
        const uint64_t row = (uint64_t)__builtin_floor(dr * (double)n);
        for (int j = 0; j < d; ++j) cen[(uint64_t)j * k + c] = cols[j][row];
    }
    __syncthreads();  // every thread has read st->cursor
    if (t == 0) st->cursor = cursor + total;
}

}  // namespace km

using namespace km;

// ---------------------------------------------------------------------------
void check_finite(st_ctx *c, const float *const *cols, const float *const *dcols, int d, uint64_t n) {
    auto *flag = wsT<uint32_t>(c, "km.nf", 2);  // [0] non-finite seen, [1] max |x| bits
    ST_HIP(hipMemsetAsync(flag, 0, 8, c->stream));
    bool wide = d <= 64;
    ScanCols sc{};
    for (int j = 0; wide && j < d; ++j) {
        sc.p[j] = cols[j];
        wide = ((uintptr_t)cols[j] & 15u) == 0;
    }
    if (wide)
        hipLaunchKernelGGL(k_scan_cols, dim3(grid_for((n + 3) / 4, 256, 1024)), dim3(256), 0, c->stream, sc, d, n,
                           flag, flag + 1);
    else
        hipLaunchKernelGGL(k_nonfinite, dim3(grid_for(n, 256, 4096)), dim3(256), 0, c->stream, dcols, d, n, flag);
    ST_LAUNCH_CHECK();
    auto *h = static_cast<uint32_t *>(pinned(c, 16));
    ST_HIP(hipMemcpyAsync(h, flag, 8, hipMemcpyDeviceToHost, c->stream));
    ST_HIP(hipStreamSynchronize(c->stream));
    ST_REQUIRE(h[0] == 0, ST_ERR_NONFINITE,
               "kmeans: non-finite point (the reference's KdTree returns index -1 and k-means.ts:131 throws)");
    c->km_absmax = wide ? __builtin_bit_cast(float, h[1]) : -1.0f;
}

// reseed + cursor bookkeeping shared by both update paths
void reseed_empty(st_ctx *c, const float *const *dcols, int d, uint64_t n, int k, const uint32_t *start,
                  const double *ddraws, uint64_t ndraws, State *dstate, float *cen) {
    if (k <= RS1_MAX) {
        hipLaunchKernelGGL(k_reseed_small, dim3(1), dim3(RS1_T), 0, c->stream, dcols, d, n, k, start, ddraws, ndraws,
                           dstate, cen);
        ST_LAUNCH_CHECK();
        return;
    }
    auto *flags = wsT<uint32_t>(c, "km.eflags", (size_t)k + 1);
    auto *rank = wsT<uint32_t>(c, "km.erank", (size_t)k + 1);
    hipLaunchKernelGGL(k_empty_flags, dim3(grid_for(k, 256, 1024)), dim3(256), 0, c->stream, start, k, flags);
    scan_u32(c, flags, rank, (uint64_t)k, rank + k);
    hipLaunchKernelGGL(k_reseed, dim3(grid_for(k, 256, 1024)), dim3(256), 0, c->stream, dcols, d, n, k, flags, rank,
                       ddraws, ndraws, dstate, cen);
    hipLaunchKernelGGL(k_advance_cursor, dim3(1), dim3(1), 0, c->stream, dstate, rank + k);
    ST_LAUNCH_CHECK();
}

void reseed_empty_counts(st_ctx *c, const float *const *dcols, int d, uint64_t n, int k, const uint32_t *counts,
                         const double *ddraws, uint64_t ndraws, State *dstate, float *cen) {
    if (k <= RC_T * 256) {
        hipLaunchKernelGGL(k_reseed_counts, dim3(1), dim3(RC_T), 0, c->stream, dcols, d, n, k, counts, ddraws, ndraws,
                           dstate, cen);
        ST_LAUNCH_CHECK();
        return;
    }
    auto *flags = wsT<uint32_t>(c, "km.eflags", (size_t)k + 1);
    auto *rank = wsT<uint32_t>(c, "km.erank", (size_t)k + 1);
    hipLaunchKernelGGL(k_empty_flags_cnt, dim3(grid_for(k, 256, 1024)), dim3(256), 0, c->stream, counts, k, flags);
    scan_u32(c, flags, rank, (uint64_t)k, rank + k);
    hipLaunchKernelGGL(k_reseed, dim3(grid_for(k, 256, 1024)), dim3(256), 0, c->stream, dcols, d, n, k, flags, rank,
                       ddraws, ndraws, dstate, cen);
    hipLaunchKernelGGL(k_advance_cursor, dim3(1), dim3(1), 0, c->stream, dstate, rank + k);
    ST_LAUNCH_CHECK();
}

void bounds_from_sorted(st_ctx *c, const uint32_t *sorted_labels, uint64_t n, int k, uint32_t *start) {
    hipLaunchKernelGGL(k_bounds, dim3(grid_for((uint64_t)k + 1, 256, 1024)), dim3(256), 0, c->stream, sorted_labels,
                       n, k, start);
    ST_LAUNCH_CHECK();
}

void member_sort(st_ctx *c, const uint32_t *labels, uint64_t n, int k, uint32_t *sorted_labels, uint32_t *members,
                 uint32_t *start) {
    int bits = 1;
    while ((1ull << bits) < (uint64_t)k) ++bits;
    radix_sort_u32_iota(c, labels, n, 0, bits, sorted_labels, members, "km.ms");
    bounds_from_sorted(c, sorted_labels, n, k, start);
}

// initializeCentroids (k-means.ts:8-20) on the host: k distinct rows by rejection on the
// Math.random stream; returns the draws consumed
static uint64_t init_rows_host(const double *draws, uint64_t ndraws, uint64_t n, int k, std::vector<uint32_t> &rows) {
    rows.resize(k);
    std::vector<uint8_t> chosen(n, 0);
    uint64_t cur = 0;
    for (int i = 0; i < k; ++i) {
        uint64_t cand;
        do {
            ST_REQUIRE(cur < ndraws, ST_ERR_DRAWS, "kmeans: Math.random draws exhausted during initialisation");
            cand = (uint64_t)std::floor(draws[cur++] * (double)n);
            ST_REQUIRE(cand < n, ST_ERR_ARG, "kmeans: Math.random draws must lie in [0, 1)");
        } while (chosen[cand]);
        chosen[cand] = 1;
        rows[i] = (uint32_t)cand;
    }
    return cur;
}

// the same on the device over the first m draws of ddraws (already uploaded): rows (k, device),
// the draws consumed in st->cursor, or ERR_INIT_WINDOW in st->err when the window holds fewer
// than k distinct rows (or a draw outside [0, 1)); unset rows stay 0
static void init_rows_dev(st_ctx *c, const double *ddraws, uint32_t m, uint64_t n, int k, uint32_t *drows,
                          State *dstate) {
    auto *first = wsT<uint32_t>(c, "km.ifirst", n);
    auto *flags = wsT<uint32_t>(c, "km.iflags", m);
    auto *pos = wsT<uint32_t>(c, "km.ipos", (size_t)m + 1);
    ST_HIP(hipMemsetAsync(first, 0xff, n * sizeof(uint32_t), c->stream));
    ST_HIP(hipMemsetAsync(drows, 0, (size_t)k * sizeof(uint32_t), c->stream));
    const unsigned g = grid_for(m, 256, 1024);
    hipLaunchKernelGGL(k_init_first, dim3(g), dim3(256), 0, c->stream, ddraws, m, n, first, dstate);
    hipLaunchKernelGGL(k_init_flags, dim3(g), dim3(256), 0, c->stream, ddraws, m, n, first, flags);
    scan_u32(c, flags, pos, m, pos + m);
    hipLaunchKernelGGL(k_init_select, dim3(g), dim3(256), 0, c->stream, ddraws, m, n, k, flags, pos, drows, dstate);
    ST_LAUNCH_CHECK();
}
// draws the device init looks at: with n >= 4k the k-th distinct row comes after about
// n ln(n / (n - k)) <= 1.151 k draws
static uint64_t init_window(uint64_t ndraws, int k) { return std::min<uint64_t>(ndraws, (uint64_t)k + k / 4 + 4096); }

void kmeans_init_rows(st_ctx *c, const double *draws, uint64_t ndraws, uint64_t n, int k, uint32_t *rows,
                      uint64_t *used) {
    ST_REQUIRE(n < (1ull << 31) && k > 0 && (uint64_t)k <= n, ST_ERR_ARG, "kmeans init: need 0 < k <= n < 2^31");
    if (n >= 4 * (uint64_t)k && ndraws > 0 && !getenv("ST_KM_HOST_INIT")) {
        const uint32_t m = (uint32_t)init_window(ndraws, k);
        auto *ddraws = wsT<double>(c, "km.idraws", m);
        auto *dstate = static_cast<State *>(ws(c, "km.istate", sizeof(State)));
        State hs{};
        ST_HIP(hipMemcpyAsync(dstate, &hs, sizeof(State), hipMemcpyHostToDevice, c->stream));
        ST_HIP(hipMemcpyAsync(ddraws, draws, m * sizeof(double), hipMemcpyHostToDevice, c->stream));
        init_rows_dev(c, ddraws, m, n, k, rows, dstate);
        ST_HIP(hipMemcpyAsync(&hs, dstate, sizeof(State), hipMemcpyDeviceToHost, c->stream));
        ST_HIP(hipStreamSynchronize(c->stream));
        if (!(hs.err & ERR_INIT_WINDOW)) {
            *used = hs.cursor;
            return;
        }
    }
    std::vector<uint32_t> hrows;
    *used = init_rows_host(draws, ndraws, n, k, hrows);
    ST_HIP(hipMemcpyAsync(rows, hrows.data(), sizeof(uint32_t) * k, hipMemcpyHostToDevice, c->stream));
    ST_HIP(hipStreamSynchronize(c->stream));  // hrows is released on return
}

void gather_owned_rows(st_ctx *c, const float *const *cols, int d, uint64_t n_local, uint64_t offset,
                       const uint32_t *rows, int k, float *out) {
    ST_REQUIRE(d > 0 && d <= 4096 && k > 0, ST_ERR_ARG, "gather rows: bad shape");
    auto **dcols = wsT<const float *>(c, "km.gcols", (size_t)d);
    ST_HIP(hipMemcpyAsync(dcols, cols, sizeof(float *) * d, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(k_gather_owned, dim3(grid_for(k, 256, 1024)), dim3(256), 0, c->stream, dcols, d, n_local,
                       offset, rows, k, out);
    ST_LAUNCH_CHECK();
}

uint64_t kmeans_dev(st_ctx *c, const float *const *cols, int d, uint64_t n, int k, int iters, const double *draws,
                    uint64_t ndraws, float *cen, uint32_t *labels, bool host_init, const double *const *sum64) {
    ST_REQUIRE(n < (1ull << 31), ST_ERR_ARG, "kmeans: n must be < 2^31 per device");
    if (n < (uint64_t)k) {  // k-means.ts:139-144
        for (int j = 0; j < d; ++j)
            ST_HIP(hipMemcpyAsync(cen + (uint64_t)j * n, cols[j], n * sizeof(float), hipMemcpyDeviceToDevice,
                                  c->stream));
        iota_u32(c, labels, n);
        return 0;
    }
    auto **dcols = wsT<const float *>(c, "km.cols", (size_t)d);
    ST_HIP(hipMemcpyAsync(dcols, cols, sizeof(float *) * d, hipMemcpyHostToDevice, c->stream));
    if (d > 1) c->kn_stats = st_ctx::KnStats{};
    const bool finite_known = c->km_finite_known && d == 1;
    c->km_finite_known = false;
    if (!finite_known) check_finite(c, cols, dcols, d, n);
    mark(c, "km.check");

    // Math.random stream: uploaded once, consumed on device in reference order
    auto *dstate = static_cast<State *>(ws(c, "km.state", sizeof(State)));
    State hs{};
    uint64_t init_used = 0;
    uint32_t dev_init_m = 0;  // > 0: initializeCentroids runs on the device over this many draws
    if (d == 1) {
        auto *mm = wsT<uint32_t>(c, "km.mm", 2);
        minmax_keys_dev(c, cols, 1, n, mm);  // finite input (checked above): keys of min and max
        hipLaunchKernelGGL(k_init1d, dim3(grid_for(k, 256, 256)), dim3(256), 0, c->stream, mm, cen, k);
        ST_LAUNCH_CHECK();
    } else if (!host_init && !getenv("ST_KM_HOST_INIT") && n >= 4 * (uint64_t)k && ndraws > 0) {
        // initializeCentroids on the device over a window of the draws (init_rows_dev); a window
        // too short sets ERR_INIT_WINDOW and the call reruns with the host's loop
        dev_init_m = (uint32_t)init_window(ndraws, k);
    } else {
        // initializeCentroids by the host's loop; the rows are then gathered on the device
        std::vector<uint32_t> rows;
        init_used = init_rows_host(draws, ndraws, n, k, rows);
        auto *drows = wsT<uint32_t>(c, "km.initrows", (size_t)k);
        ST_HIP(hipMemcpyAsync(drows, rows.data(), sizeof(uint32_t) * k, hipMemcpyHostToDevice, c->stream));
        hipLaunchKernelGGL(k_gather_init, dim3(grid_for(k, 256, 1024)), dim3(256), 0, c->stream, dcols, d, drows, k,
                           cen);
        ST_LAUNCH_CHECK();
    }
    hs.cursor = init_used;
    ST_HIP(hipMemcpyAsync(dstate, &hs, sizeof(State), hipMemcpyHostToDevice, c->stream));
    // re-seeds consume at most k draws per iteration: upload only that window of the stream
    const uint64_t window = std::min<uint64_t>(ndraws, std::max<uint64_t>(init_used, dev_init_m) +
                                                           (uint64_t)k * (uint64_t)iters);
    auto *ddraws = wsT<double>(c, "km.draws", window ? window : 1);
    if (window) ST_HIP(hipMemcpyAsync(ddraws, draws, window * sizeof(double), hipMemcpyHostToDevice, c->stream));
    const uint64_t ndraws_all = ndraws;
    ndraws = window;
    if (dev_init_m) {
        // rows a short window leaves unset stay 0: the discarded run still reads inside the table
        auto *drows = wsT<uint32_t>(c, "km.initrows", (size_t)k);
        init_rows_dev(c, ddraws, dev_init_m, n, k, drows, dstate);
        hipLaunchKernelGGL(k_gather_init, dim3(grid_for(k, 256, 1024)), dim3(256), 0, c->stream, dcols, d, drows, k,
                           cen);
        ST_LAUNCH_CHECK();
    }
    mark(c, "km.init");

    if (d == 1)
        kmeans1d_loop(c, cols[0], dcols, n, k, iters, ddraws, ndraws, dstate, cen, labels);
    else
        kmeansnd_loop(c, cols, dcols, d, n, k, iters, ddraws, ndraws, dstate, cen, labels, sum64);

    ST_HIP(hipMemcpyAsync(&hs, dstate, sizeof(State), hipMemcpyDeviceToHost, c->stream));
    ST_HIP(hipStreamSynchronize(c->stream));
    if (hs.err & ERR_INIT_WINDOW)  // the device window held fewer than k distinct rows
        return kmeans_dev(c, cols, d, n, k, iters, draws, ndraws_all, cen, labels, true, sum64);
    if (hs.err & ERR_K1_MANY) {  // more uncertified 1-D clusters than the queued iteration takes
        const bool was = c->k1_sync;
        c->k1_sync = true;
        struct Reset {
            st_ctx *c;
            bool was;
            ~Reset() { c->k1_sync = was; }
        } reset{c, was};
        return kmeans_dev(c, cols, d, n, k, iters, draws, ndraws_all, cen, labels, host_init, sum64);
    }
    ST_REQUIRE(!(hs.err & ERR_DRAWS), ST_ERR_DRAWS, "kmeans: Math.random draws exhausted while re-seeding");
    ST_REQUIRE(!(hs.err & ERR_DRAW_RANGE), ST_ERR_ARG, "kmeans: a re-seed draw outside [0, 1)");
    ST_REQUIRE(!(hs.err & ERR_INTERNAL), ST_ERR_INTERNAL, "kmeans: internal consistency check failed");
    if (d > 1) kn_stats_publish(c);
    return hs.cursor;
}

void kn_stats_publish(st_ctx *c) {
    const auto &k_ = c->kn_stats;
    char buf[320];
    snprintf(buf, sizeof buf,
             "{\"assigns\": %llu, \"points\": %llu, \"pairs\": %llu, \"ambiguous\": %llu, \"overflow\": %llu, "
             "\"walked_overflow\": %llu, \"ties\": %llu}",
             (unsigned long long)k_.assigns, (unsigned long long)k_.points, (unsigned long long)k_.pairs,
             (unsigned long long)k_.ambiguous, (unsigned long long)k_.overflow, (unsigned long long)k_.walked_overflow,
             (unsigned long long)k_.ties);
    c->last_kn_stats = buf;
}

}  // namespace st
