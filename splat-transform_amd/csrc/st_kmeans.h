// st_kmeans.h -- internal interfaces shared by the k-means translation units.
#pragma once

#include "st_internal.h"

namespace st {
namespace km {

enum : uint32_t {
    ERR_DRAWS = 1u,
    ERR_TIE = 2u,
    ERR_INTERNAL = 4u,
    ERR_INIT_WINDOW = 8u,
    ERR_DRAW_RANGE = 16u,
    ERR_K1_MANY = 32u,  // 1-D: more uncertified clusters than the queued path takes (rerun synchronised)
};

// device-resident k-means state (one per call)
struct State {
    uint64_t cursor;  // Math.random draws consumed so far
    uint32_t err;
    uint32_t amb;     // ambiguous points this iteration (D > 1)
    uint32_t ties;    // exact-distance ties this iteration (D > 1)
    uint32_t overflow;  // ambiguous points whose candidate list overflowed (exact scan of all K)
    uint32_t pairs;     // points whose candidates lie in two tile-halves (k_fixpair)
};

__host__ __device__ inline uint32_t fkey_(float f) {
    uint32_t u = __builtin_bit_cast(uint32_t, f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ inline float fkey_inv_(uint32_t k) {
    uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
    return __builtin_bit_cast(float, u);
}
// row stride of the f32 AoS copies of points and centroids (16-byte rows, zero padded)
__host__ __device__ inline int aos_ld(int d) { return (d + 3) & ~3; }

// exponent of the unit in the last place of an f32 (the value is a multiple of 2^ulp_exp)
__device__ inline int ulp_exp(float x) {
    const uint32_t e = (__builtin_bit_cast(uint32_t, x) >> 23) & 0xffu;
    return e == 0 ? -149 : (int)e - 150;
}
__device__ inline int ulp_exp(double x) {
    const uint32_t e = (uint32_t)(__builtin_bit_cast(uint64_t, x) >> 52) & 0x7ffu;
    return e == 0 ? -1074 : (int)e - 1075;
}
// certificate that every partial sum of a set of f32 values is exact in f64: all are
// multiples of 2^emin and |partial sums| <= sum|x| < 2^(emin + 53) (slack for sum|x|'s own rounding)
__host__ __device__ inline bool sum_is_exact(double sabs, int emin) {
    return sabs == 0.0 || sabs * (1.0 + 1.0e-6) < __builtin_ldexp(1.0, emin + 53);
}
// stable-sort key of a centroid coordinate under the comparator `a - b`
// (k-means / kd-tree sort callbacks): -0 and +0 compare equal
__host__ __device__ inline uint32_t sortkey_(float f) { return fkey_(f == 0.0f ? 0.0f : f); }

}  // namespace km

// shared by the 1-D and N-D loops
void reseed_empty(st_ctx *c, const float *const *dcols, int d, uint64_t n, int k, const uint32_t *start,
                  const double *ddraws, uint64_t ndraws, km::State *dstate, float *cen);
// the same from the clusters' member counts
void reseed_empty_counts(st_ctx *c, const float *const *dcols, int d, uint64_t n, int k, const uint32_t *counts,
                         const double *ddraws, uint64_t ndraws, km::State *dstate, float *cen);
// start[c] = first index with sorted_labels >= c, start[k] = n
void bounds_from_sorted(st_ctx *c, const uint32_t *sorted_labels, uint64_t n, int k, uint32_t *start);
void member_sort(st_ctx *c, const uint32_t *labels, uint64_t n, int k, uint32_t *sorted_labels, uint32_t *members,
                 uint32_t *start);

void kmeans1d_loop(st_ctx *c, const float *pts, const float *const *dcols, uint64_t n, int k, int iters,
                   const double *ddraws, uint64_t ndraws, km::State *dstate, float *cen, uint32_t *labels);
// (sum64: host array of device float64 columns whose values calcAverage sums instead of the
// float32 points -- the JS numbers of columns that are not float32)
void kmeansnd_loop(st_ctx *c, const float *const *cols, const float *const *dcols, int d, uint64_t n, int k,
                   int iters, const double *ddraws, uint64_t ndraws, km::State *dstate, float *cen, uint32_t *labels,
                   const double *const *sum64 = nullptr);

// step form of the loops (shared with the distributed step API, st_dist.hip)
void nd_prepare(st_ctx *c, const float *const *dcols, int d, uint64_t n);  // workspace: kn.pfrag/kn.pnorm/kn.aos
// the fix-up pass's share of the update (kmeansnd_loop): set by nd_assign when the fused
// fix-up ran (partials of the decided points; the other points' counts)
struct NdFused {
    bool want = false, valid = false;
    uint32_t npair = 0, namb = 0, nties_fix = 0, ncodes = 0;
};
// (settle: called once the centroids' duplicate-row check has synchronised the stream; true when
// it changed centroids, and the check runs again -- kmeansnd_loop's pending large-cluster sums)
void nd_assign(st_ctx *c, const float *const *dcols, int d, uint64_t n, int k, const float *cen, uint32_t *labels,
               km::State *dstate, NdFused *fz = nullptr, const std::function<bool()> &settle = {});
// after a fused nd_assign (fz.valid): the (dimension, cluster) partials of the shard -- f64 sum,
// sum|x|, smallest ulp exponent ([dim][k]) and counts -- from the fix-up's slices and the other
// points, without the member sort (the sharded writer's N-D update)
void nd_fused_partials(st_ctx *c, int d, uint64_t n, int k, const NdFused &fz, const uint32_t *labels, double *sums,
                       double *sabs, int32_t *emin, uint32_t *counts);
// returns true when it also wrote the update's (label, value bits) pairs into keys/vals
// (need_labels = false with keys: the labels are not written, only the pairs)
bool assign1d(st_ctx *c, const float *pts, uint64_t n, int k, const float *cen, uint32_t *labels,
              uint32_t *keys = nullptr, uint32_t *vals = nullptr, bool need_labels = true);
// the multi-GPU update's 1-D pieces (st_kmeans1d.hip's chunked kernels): per-(segment,
// cluster) partials of the label-sorted value bits (nk = nseg * k ranges of start), and the
// exact replay of the pending clusters' sums over one segment (start: that segment's k + 1
// bounds) from their running values; pflag[p] = 1 where the sequential chain must finish
void seg_label_sort1d(st_ctx *c, const float *pts, const uint32_t *labels, uint64_t n, int nseg, int k,
                      uint32_t *vals, uint32_t *start);
void partials1d(st_ctx *c, const uint32_t *vals, uint64_t n, const uint32_t *start, int nk, double *sums, double *sabs,
                int32_t *emin, uint32_t *counts);
// the labels and the same partials straight from the accumulating assign, segment by segment
// (n = nseg equal segments, k <= 256)
void assign_partials1d(st_ctx *c, const float *pts, uint64_t n, int nseg, int k, const float *cen, uint32_t *labels,
                       double *sums, double *sabs, int32_t *emin, uint32_t *counts);
void seqsum1d(st_ctx *c, const uint32_t *vals, uint64_t n, const uint32_t *start, int k, const uint32_t *pairs,
              uint32_t npairs, double *running, const int32_t *emin, const double *sabs, uint32_t *pflag);
// throws ST_ERR_NONFINITE on a non-finite value; also leaves max |x| in c->km_absmax
// (cols: host array of the device columns, dcols: the same array on the device)
void check_finite(st_ctx *c, const float *const *cols, const float *const *dcols, int d, uint64_t n);

// KdTree.findNearest for the points listed in tie_pts (exact-distance ties, candidate
// overflows): cen [d][k] for the tree, the row-major copies aos (points) / caos (centroids)
// with row stride ld (zero padded) for the distances (st_kdtree.hip)
// (tree_built: kd_build already ran on these centroids in this call)
void kd_resolve_ties(st_ctx *c, int d, int k, const float *cen, const float *aos, const float *caos, int ld,
                     const uint32_t *tie_pts, uint32_t nties, uint32_t *labels, bool tree_built = false);
// KdTree.build of cen [d][k]: the device array S[tree position] = centroid index (workspace kd.S)
const uint32_t *kd_build(st_ctx *c, int d, int k, const float *cen);

// coinciding centroids (identical rows, -0 == +0): one representative per distinct row
struct CenGroups {
    uint32_t kr = 0;        // distinct rows
    float *cen_r = nullptr;     // [d][kr] the representatives' rows (each group's lowest index)
    uint32_t *map_r2c = nullptr;  // [kr] representative slot -> centroid index
    uint32_t *grp = nullptr;      // [k] centroid -> its group's slot
};
// false when every row is distinct (nothing written); one host sync
bool cen_groups(st_ctx *c, int d, int k, const float *cen, CenGroups *g);
// labels[p] = slot of p's nearest distinct row (a unique minimum) -> the reference's centroid:
// the group's only member, or the member KdTree.findNearest meets first (a descent of the tree)
// (err: ERR_INTERNAL if a point's group is not found in the tree)
void kd_group_labels(st_ctx *c, int d, int k, const float *cen, const CenGroups &g, const float *aos, int ld,
                     uint64_t n, uint32_t *labels, uint32_t *err);

}  // namespace st
