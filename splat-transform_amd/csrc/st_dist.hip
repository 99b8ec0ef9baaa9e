// st_dist.hip -- multi-GPU building blocks.
//
// One process per GPU; the splat table is sharded in contiguous row ranges in
// rank order.  k-means needs one exchange per iteration: the per-cluster sums
// of calcAverage (k-means.ts:41-63).  The reference adds each cluster's members
// in ascending global point order into one f64, so the distributed update is
// exact in two regimes:
//   * certified (the common case): every value of the (cluster, dim) is a
//     multiple of 2^emin and sum|x| < 2^(emin+53), so every partial sum in any
//     order is exact -- each rank's partial sum and their allreduce are the
//     reference's value;
//   * otherwise the (cluster, dim) is "pending": its running sum is handed from
//     segment to segment in global order (st_dev_kmeans_seqsum on the owning
//     rank, a broadcast between ranks), replaying the sequential sum exactly.
// A segment is a contiguous range of a rank's points that is contiguous in the
// global order: the whole shard for N-D k-means, one column of the shard for
// cluster1d's column-major concatenation (write-sog.ts:56-99).
//
// The caller (splat-transform_amd/py/splat_dist.py) runs the collectives with
// torch.distributed (RCCL over xGMI, or gloo) between these calls.
#include <cmath>

#include "st_jsmath.h"
#include "st_kmeans.h"

namespace st {
namespace {

using namespace km;


// sort key of point i: (segment, label)
// (n < 2^31: 32-bit index arithmetic; the segment of i advances by a compare, not a division)
__global__ __launch_bounds__(256) void k_seg_keys(const uint32_t *labels, uint32_t n, uint32_t seg_len, int k,
                                                  const float *vals, uint32_t *keys, uint32_t *payload) {
    const uint32_t stride = gridDim.x * blockDim.x;
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;  // also an empty shard (seg_len = 0)
    uint32_t seg = i / seg_len, next = (seg + 1) * seg_len;
    for (; i < n; i += stride) {
        while (i >= next) {
            ++seg;
            next += seg_len;
        }
        keys[i] = seg * (uint32_t)k + labels[i];
        payload[i] = vals ? __builtin_bit_cast(uint32_t, vals[i]) : i;
    }
}

// N-D partials: one wave per (segment, cluster), lane = dimension; f64 sum, sum|x| and the
// smallest ulp exponent of the members.  The sum is used only where the certificate holds
// (every partial sum exact, in any order), so it is kept in 4 interleaved accumulators:
// a quarter of the dependent f64 add chain.  Layout [seg][dim][k].
__global__ __launch_bounds__(256) void k_partials_nd(const float *__restrict__ aos, int d,
                                                     const uint32_t *__restrict__ members,
                                                     const uint32_t *__restrict__ start, int k, int nseg,
                                                     double *__restrict__ sums, double *__restrict__ sabs,
                                                     int32_t *__restrict__ emin, uint32_t *__restrict__ counts) {
    const int lane = threadIdx.x & 63;
    const uint32_t sc = blockIdx.x * 4 + (threadIdx.x >> 6);  // seg * k + cluster
    if (sc >= (uint32_t)(nseg * k)) return;
    const uint32_t seg = sc / k, cl = sc % k;
    const uint32_t s0 = start[sc], s1 = start[sc + 1];
    if (lane == 0) counts[sc] = s1 - s0;
    if (lane >= d) return;
    const int ld = aos_ld(d);
    double sum[4] = {0, 0, 0, 0}, sa[4] = {0, 0, 0, 0};
    int em = 1 << 20;
    auto add = [&](float v, int a) {
        sum[a] += (double)v;
        sa[a] += (double)__builtin_fabsf(v);
        if (v != 0.0f) em = min(em, ulp_exp(v));
    };
    uint32_t j = s0;
    constexpr int U = 16;  // member rows in flight per wave
    for (; j + U <= s1; j += U) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = aos[(uint64_t)members[j + u] * ld + lane];
#pragma unroll
        for (int u = 0; u < U; ++u) add(v[u], u & 3);
    }
    for (; j < s1; ++j) add(aos[(uint64_t)members[j] * ld + lane], 0);
    const uint64_t o = ((uint64_t)seg * d + lane) * k + cl;
    sums[o] = (sum[0] + sum[1]) + (sum[2] + sum[3]);
    sabs[o] = (sa[0] + sa[1]) + (sa[2] + sa[3]);
    emin[o] = em;
}

// continue the sequential sums of the pending (cluster, dim) pairs over this rank's
// members of segment `seg`: one lane per pair
__global__ __launch_bounds__(64) void k_seqsum_nd(const float *__restrict__ aos, int d,
                                                  const uint32_t *__restrict__ members,
                                                  const uint32_t *__restrict__ start, int k, int seg,
                                                  const uint32_t *__restrict__ pairs, uint32_t npairs,
                                                  double *__restrict__ running) {
    const uint32_t p = blockIdx.x * 64 + threadIdx.x;
    if (p >= npairs) return;
    const uint32_t pair = pairs[p], cl = pair / d, dim = pair % d;
    const uint32_t sc = (uint32_t)seg * k + cl;
    const int ld = aos_ld(d);
    double s = running[p];
    uint32_t j = start[sc];
    const uint32_t e = start[sc + 1];
    constexpr int U = 8;  // loads in flight ahead of the ordered add chain
    for (; j + U <= e; j += U) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = aos[(uint64_t)members[j + u] * ld + dim];
#pragma unroll
        for (int u = 0; u < U; ++u) s += (double)v[u];
    }
    for (; j < e; ++j) s += (double)aos[(uint64_t)members[j] * ld + dim];
    running[p] = s;
}

// 1-D fallback: one wave per flagged pending cluster, lane 0 walks the contiguous values
__global__ __launch_bounds__(64) void k_seqsum_1d(const uint32_t *__restrict__ vals, const uint32_t *__restrict__ start,
                                                  int k, int seg, const uint32_t *__restrict__ pairs,
                                                  const uint32_t *__restrict__ flag, double *__restrict__ running) {
    if (threadIdx.x != 0 || !flag[blockIdx.x]) return;
    const uint32_t p = blockIdx.x;
    const uint32_t sc = (uint32_t)seg * k + pairs[p];
    uint32_t opaque0;  // keeps the loads on the vector path (see k_sum1d_seq)
    asm volatile("v_mov_b32 %0, 0" : "=v"(opaque0));
    const uint32_t *v = vals + opaque0;
    double s = running[p];
    uint32_t j = start[sc];
    const uint32_t e = start[sc + 1];
    for (; j + 8 <= e; j += 8) {
        uint32_t b[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) b[u] = v[j + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += (double)__builtin_bit_cast(float, b[u]);
    }
    for (; j < e; ++j) s += (double)__builtin_bit_cast(float, v[j]);
    running[p] = s;
}

// certified entries -> centroid; uncertified -> pending flag (empties untouched)
__global__ __launch_bounds__(256) void k_finish(int d, int k, const double *__restrict__ sums,
                                                const double *__restrict__ sabs, const int32_t *__restrict__ emin,
                                                const uint32_t *__restrict__ counts, float *__restrict__ cen,
                                                uint32_t *__restrict__ flags) {
    const uint32_t total = (uint32_t)d * k;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        const uint32_t dim = t / k, cl = t % k;
        const uint32_t cnt = counts[cl];
        uint32_t f = 0;
        if (cnt) {
            if (sum_is_exact(sabs[t], emin[t])) cen[t] = (float)(sums[t] / (double)cnt);
            else f = 1;
        }
        flags[cl * d + dim] = f;  // pair order: cluster-major
    }
}

__global__ __launch_bounds__(256) void k_compact_pairs(const uint32_t *flags, const uint32_t *pos, uint32_t total,
                                                       uint32_t *pairs) {
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x)
        if (flags[t]) pairs[pos[t]] = t;
}

__global__ __launch_bounds__(256) void k_average(int d, int k, const uint32_t *__restrict__ pairs, uint32_t npairs,
                                                 const double *__restrict__ running,
                                                 const uint32_t *__restrict__ counts, float *__restrict__ cen) {
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < npairs; p += gridDim.x * blockDim.x) {
        const uint32_t cl = pairs[p] / d, dim = pairs[p] % d;
        cen[(uint64_t)dim * k + cl] = (float)(running[p] / (double)counts[cl]);
    }
}

}  // namespace

// ---------------------------------------------------------------------------
void minmax_dev(st_ctx *c, const float *const *cols, int ncols, uint64_t n, double *lo, double *hi) {
    auto *mm = wsT<uint32_t>(c, "ds.mm", 2 * (size_t)ncols);
    std::vector<uint32_t> init(2 * ncols);
    minmax_keys_dev(c, cols, ncols, n, mm);
    ST_HIP(hipMemcpyAsync(init.data(), mm, init.size() * 4, hipMemcpyDeviceToHost, c->stream));
    ST_HIP(hipStreamSynchronize(c->stream));
    for (int a = 0; a < ncols; ++a) {
        lo[a] = init[2 * a] == 0xffffffffu ? HUGE_VAL : (double)fkey_inv_(init[2 * a]);
        hi[a] = init[2 * a + 1] == 0u ? -HUGE_VAL : (double)fkey_inv_(init[2 * a + 1]);
    }
}

void dist_prepare(st_ctx *c, const float *const *cols, int d, uint64_t n) {
    ST_REQUIRE(n < (1ull << 31), ST_ERR_ARG, "kmeans: n must be < 2^31 per device");
    auto **dcols = wsT<const float *>(c, "ds.cols", (size_t)d);
    ST_HIP(hipMemcpyAsync(dcols, cols, sizeof(float *) * d, hipMemcpyHostToDevice, c->stream));
    check_finite(c, cols, dcols, d, n);
    if (d > 1) nd_prepare(c, dcols, d, n);
}

void dist_assign(st_ctx *c, const float *const *cols, int d, uint64_t n, int k, const float *cen, uint32_t *labels) {
    if (d == 1) {
        assign1d(c, cols[0], n, k, cen, labels);
        return;
    }
    auto **dcols = wsT<const float *>(c, "ds.cols", (size_t)d);
    ST_HIP(hipMemcpyAsync(dcols, cols, sizeof(float *) * d, hipMemcpyHostToDevice, c->stream));
    auto *dstate = static_cast<State *>(ws(c, "ds.state", sizeof(State)));
    ST_HIP(hipMemsetAsync(dstate, 0, sizeof(State), c->stream));
    nd_assign(c, dcols, d, n, k, cen, labels, dstate);
}

void dist_assign_partials1d(st_ctx *c, const float *pts, uint64_t n, int nseg, int k, const float *cen,
                            uint32_t *labels, double *sums, double *sabs, int32_t *emin, uint32_t *counts) {
    ST_REQUIRE(n < (1ull << 31) && (uint64_t)nseg * k < (1ull << 31), ST_ERR_ARG, "kmeans partials: too large");
    assign_partials1d(c, pts, n, nseg, k, cen, labels, sums, sabs, emin, counts);
    c->ds_nseg = nseg;
    c->ds_k = k;
    c->ds_d = 1;
    c->ds_n = n;
    c->ds_pts = pts;
    c->ds_labels = labels;
    c->ds_sorted = false;
}

namespace {
// the (segment, label) member order of an N-D shard: payload = point indices, start = ranges
void member_order_nd(st_ctx *c, const uint32_t *labels, uint64_t n, int nseg, int k) {
    const uint64_t nk = (uint64_t)nseg * k;
    auto *keys = wsT<uint32_t>(c, "ds.keys", n);
    auto *payload = wsT<uint32_t>(c, "ds.payload", n);
    auto *start = wsT<uint32_t>(c, "ds.start", nk + 1);
    int bits = 1;
    while ((1ull << bits) < nk) ++bits;
    hipLaunchKernelGGL(k_seg_keys, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c->stream, labels, (uint32_t)n,
                       (uint32_t)(n / nseg), k, (const float *)nullptr, keys, payload);
    ST_LAUNCH_CHECK();
    radix_sort_u32(c, keys, payload, n, 0, bits, "ds.sort");
    bounds_from_sorted(c, keys, n, (int)nk, start);
}
}  // namespace

bool dist_assign_partials_nd(st_ctx *c, const float *const *dcols, int d, uint64_t n, int k, const float *cen,
                             uint32_t *labels, double *sums, double *sabs, int32_t *emin, uint32_t *counts) {
    ST_REQUIRE(d > 1 && n < (1ull << 31), ST_ERR_ARG, "kmeans partials: N-D shard of fewer than 2^31 points");
    auto *dstate = static_cast<State *>(ws(c, "ds.state", sizeof(State)));
    ST_HIP(hipMemsetAsync(dstate, 0, sizeof(State), c->stream));
    NdFused fz;
    fz.want = true;
    nd_assign(c, dcols, d, n, k, cen, labels, dstate, &fz);
    if (!fz.valid) return false;  // no fused fix-up (coinciding centroids, other shapes)
    nd_fused_partials(c, d, n, k, fz, labels, sums, sabs, emin, counts);
    c->ds_nseg = 1;
    c->ds_k = k;
    c->ds_d = d;
    c->ds_n = n;
    c->ds_labels = labels;
    c->ds_sorted = false;  // the member order is built only if a pending pair needs it
    return true;
}

void dist_partials(st_ctx *c, const float *const *cols, int d, uint64_t n, int nseg, int k, const uint32_t *labels,
                   double *sums, double *sabs, int32_t *emin, uint32_t *counts) {
    ST_REQUIRE(nseg >= 1 && n % (uint64_t)nseg == 0, ST_ERR_ARG, "kmeans partials: n must split into nseg segments");
    const uint64_t nk = (uint64_t)nseg * k;
    ST_REQUIRE(nk < (1ull << 31), ST_ERR_ARG, "kmeans partials: nseg * k too large");
    auto *keys = wsT<uint32_t>(c, "ds.keys", n);
    auto *payload = wsT<uint32_t>(c, "ds.payload", n);  // value bits (1-D) or point index (N-D)
    auto *start = wsT<uint32_t>(c, "ds.start", nk + 1);
    int bits = 1;
    while ((1ull << bits) < nk) ++bits;
    ST_REQUIRE(n < (1ull << 31), ST_ERR_ARG, "kmeans partials: n must be < 2^31 per device");
    if (d == 1 && k <= 256) {
        // stable by label inside each (contiguous) segment: one value-only counting pass per segment
        seg_label_sort1d(c, cols[0], labels, n, nseg, k, payload, start);
    } else {
        if (d == 1) {
            hipLaunchKernelGGL(k_seg_keys, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c->stream, labels, (uint32_t)n,
                               (uint32_t)(n / nseg), k, cols[0], keys, payload);
            ST_LAUNCH_CHECK();
            radix_sort_u32(c, keys, payload, n, 0, bits, "ds.sort");
            bounds_from_sorted(c, keys, n, (int)nk, start);
        } else {
            member_order_nd(c, labels, n, nseg, k);
        }
    }
    if (d == 1) {
        partials1d(c, payload, n, start, (int)nk, sums, sabs, emin, counts);
    } else {
        ST_REQUIRE(c->kn_n == n && c->kn_d == d, ST_ERR_ARG, "kmeans partials: point set not prepared");
        auto *aos = wsT<float>(c, "kn.aos", n * (size_t)aos_ld(d));
        hipLaunchKernelGGL(k_partials_nd, dim3((unsigned)((nk + 3) / 4)), dim3(256), 0, c->stream, aos, d, payload,
                           start, k, nseg, sums, sabs, emin, counts);
    }
    ST_LAUNCH_CHECK();
    c->ds_nseg = nseg;
    c->ds_k = k;
    c->ds_d = d;
    c->ds_n = n;
    c->ds_sorted = true;
}

void dist_seqsum(st_ctx *c, int d, int k, int seg, const uint32_t *pairs, uint32_t npairs, double *running,
                 const int32_t *emin, const double *sabs) {
    ST_REQUIRE(c->ds_d == d && c->ds_k == k && seg >= 0 && seg < c->ds_nseg, ST_ERR_ARG,
               "kmeans seqsum: no matching partials on this context");
    if (!npairs) return;
    const uint64_t n = c->ds_n, nk = (uint64_t)c->ds_nseg * k;
    auto *payload = wsT<uint32_t>(c, "ds.payload", n);
    auto *start = wsT<uint32_t>(c, "ds.start", nk + 1);
    if (d == 1) {
        if (!c->ds_sorted) {  // partials came from the accumulating assign: order the members now
            seg_label_sort1d(c, c->ds_pts, c->ds_labels, n, c->ds_nseg, k, payload, start);
            c->ds_sorted = true;
        }
        auto *flag = wsT<uint32_t>(c, "ds.sflag", npairs);
        seqsum1d(c, payload, n, start + (uint64_t)seg * k, k, pairs, npairs, running, emin, sabs, flag);
        hipLaunchKernelGGL(k_seqsum_1d, dim3(npairs), dim3(64), 0, c->stream, payload, start, k, seg, pairs, flag,
                           running);
    } else {
        if (!c->ds_sorted) {  // partials came from the fused fix-up: order the members now
            member_order_nd(c, c->ds_labels, n, c->ds_nseg, k);
            c->ds_sorted = true;
        }
        auto *aos = wsT<float>(c, "kn.aos", n * (size_t)aos_ld(d));
        hipLaunchKernelGGL(k_seqsum_nd, dim3((npairs + 63) / 64), dim3(64), 0, c->stream, aos, d, payload, start, k,
                           seg, pairs, npairs, running);
    }
    ST_LAUNCH_CHECK();
}

uint32_t dist_finish(st_ctx *c, int d, int k, const double *sums, const double *sabs, const int32_t *emin,
                     const uint32_t *counts, float *cen, uint32_t *pending) {
    const uint32_t total = (uint32_t)d * k;
    auto *flags = wsT<uint32_t>(c, "ds.flags", total);
    auto *pos = wsT<uint32_t>(c, "ds.pos", (size_t)total + 1);
    hipLaunchKernelGGL(k_finish, dim3(grid_for(total, 256, 4096)), dim3(256), 0, c->stream, d, k, sums, sabs, emin,
                       counts, cen, flags);
    ST_LAUNCH_CHECK();
    scan_u32(c, flags, pos, total, pos + total);
    hipLaunchKernelGGL(k_compact_pairs, dim3(grid_for(total, 256, 4096)), dim3(256), 0, c->stream, flags, pos, total,
                       pending);
    ST_LAUNCH_CHECK();
    auto *np = static_cast<uint32_t *>(pinned_slot(c, "ds.np", 4));
    ST_HIP(hipMemcpyAsync(np, pos + total, 4, hipMemcpyDeviceToHost, c->stream));
    ST_HIP(hipStreamSynchronize(c->stream));
    return *np;
}

void dist_average(st_ctx *c, int d, int k, const uint32_t *pairs, uint32_t npairs, const double *running,
                  const uint32_t *counts, float *cen) {
    if (!npairs) return;
    hipLaunchKernelGGL(k_average, dim3(grid_for(npairs, 256, 4096)), dim3(256), 0, c->stream, d, k, pairs, npairs,
                       running, counts, cen);
    ST_LAUNCH_CHECK();
}

}  // namespace st
