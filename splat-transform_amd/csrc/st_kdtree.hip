// st_kdtree.hip -- the reference's KdTree tie-break for exact-distance ties.
//
// When two centroids are at exactly the same f64 distance from a point (e.g.
// a re-seeded centroid equal to another), the reference's answer is whichever
// KdTree.findNearest meets first (kd-tree.ts:39-68: nearer child first, strict
// `<`, prune on distance^2 >= best).  This file rebuilds that tree on the device
// and walks it for the (rare) tied points only.
//
// Tree build (kd-tree.ts:73-99): the recursion only permutes `indices` inside
// segments whose boundaries depend on K alone -- depth L sorts every segment of
// length >= 2 by axis L % D (stable), then splits [lo,hi) at mid = lo+(len>>1)
// (len 2: node lo, right child lo+1).  So each depth is one stable radix sort of
// (segment rank, coordinate) over the active positions; the segment layout is
// precomputed on the host per K.
// Walk: one thread per listed point over the implicit tree, the exact distance
// (row-major copies of points and centroids) computed at each visited node.
#include <memory>
#include <unordered_map>

#include "st_jsmath.h"
#include "st_kmeans.h"

namespace st {
namespace {

using namespace km;

struct Level {
    uint32_t count;      // active positions at this depth
    uint32_t seg_bits;   // bits of the segment rank
    uint32_t *pos;       // device: active positions (ascending)
    uint32_t *rank;      // device: segment rank of each active position
};

struct KdLayout {
    int k = 0;
    std::vector<Level> levels;
    uint8_t *depth = nullptr;  // device: the depth at which each position is a tree node
    std::vector<void *> allocs;
    ~KdLayout() {
        for (void *p : allocs) (void)hipFree(p);
    }
};

// host: the segment structure of KdTree.build for k centroids
std::unique_ptr<KdLayout> make_layout(int k) {
    auto L = std::make_unique<KdLayout>();
    L->k = k;
    std::vector<std::pair<uint32_t, uint32_t>> segs = {{0u, (uint32_t)k}}, next;
    std::vector<uint8_t> depth((size_t)k, 0);
    for (uint8_t dep = 0; !segs.empty(); ++dep) {
        std::vector<uint32_t> pos, rank;
        uint32_t r = 0;
        next.clear();
        for (auto s : segs) {
            const uint32_t len = s.second - s.first;
            if (len >= 2) {
                for (uint32_t p = s.first; p < s.second; ++p) {
                    pos.push_back(p);
                    rank.push_back(r);
                }
                ++r;
            }
            if (len == 1) {
                depth[s.first] = dep;
            } else if (len == 2) {
                // right child is a single leaf: nothing further to sort
                depth[s.first] = dep;
                depth[s.first + 1] = (uint8_t)(dep + 1);
            } else if (len >= 3) {
                const uint32_t mid = s.first + (len >> 1);
                depth[mid] = dep;
                next.push_back({s.first, mid});
                next.push_back({mid + 1, s.second});
            }
        }
        if (!pos.empty()) {
            Level lv{};
            lv.count = (uint32_t)pos.size();
            uint32_t bits = 0;
            while ((1u << bits) < r) ++bits;
            lv.seg_bits = bits;
            ST_HIP(hipMalloc(&lv.pos, pos.size() * 4));
            ST_HIP(hipMalloc(&lv.rank, rank.size() * 4));
            L->allocs.push_back(lv.pos);
            L->allocs.push_back(lv.rank);
            ST_HIP(hipMemcpy(lv.pos, pos.data(), pos.size() * 4, hipMemcpyHostToDevice));
            ST_HIP(hipMemcpy(lv.rank, rank.data(), rank.size() * 4, hipMemcpyHostToDevice));
            L->levels.push_back(lv);
        }
        segs.swap(next);
    }
    ST_HIP(hipMalloc(&L->depth, (size_t)k));
    L->allocs.push_back(L->depth);
    ST_HIP(hipMemcpy(L->depth, depth.data(), (size_t)k, hipMemcpyHostToDevice));
    return L;
}

__global__ __launch_bounds__(256) void k_level_keys(const float *__restrict__ cen, int k, int axis,
                                                    const uint32_t *__restrict__ S, const uint32_t *__restrict__ pos,
                                                    const uint32_t *__restrict__ rank, uint32_t m,
                                                    uint64_t *__restrict__ keys, uint32_t *__restrict__ vals) {
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m; j += gridDim.x * blockDim.x) {
        const uint32_t ci = S[pos[j]];
        keys[j] = ((uint64_t)rank[j] << 32) | sortkey_(cen[(uint64_t)axis * k + ci]);
        vals[j] = ci;
    }
}

__global__ __launch_bounds__(256) void k_level_scatter(const uint32_t *__restrict__ pos,
                                                       const uint32_t *__restrict__ vals, uint32_t m,
                                                       uint32_t *__restrict__ S) {
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m; j += gridDim.x * blockDim.x) S[pos[j]] = vals[j];
}

// calcDistance (kd-tree.ts:26-35): f64 differences of the f32 values, squares summed in
// dimension order (the zero padding of the rows adds +0)
__device__ inline double kd_dist(const float *__restrict__ crow, const float *__restrict__ prow, int ld) {
    const float4 *c4 = reinterpret_cast<const float4 *>(crow);
    const float4 *p4 = reinterpret_cast<const float4 *>(prow);
    double l = 0;
    for (int q = 0; q < ld / 4; ++q) {
        const float4 a = c4[q], b = p4[q];
        double v = (double)a.x - (double)b.x;
        l += v * v;
        v = (double)a.y - (double)b.y;
        l += v * v;
        v = (double)a.z - (double)b.z;
        l += v * v;
        v = (double)a.w - (double)b.w;
        l += v * v;
    }
    return l;
}

struct Frame {
    uint32_t lo, hi, depth;
};

__device__ inline void seg_split(uint32_t lo, uint32_t hi, uint32_t &node, uint32_t &llo, uint32_t &lhi,
                                 uint32_t &rlo, uint32_t &rhi) {
    const uint32_t len = hi - lo;
    if (len == 1) {
        node = lo;
        llo = lhi = rlo = rhi = 0;
    } else if (len == 2) {
        node = lo;
        llo = lhi = 0;
        rlo = lo + 1;
        rhi = lo + 2;
    } else {
        node = lo + (len >> 1);
        llo = lo;
        lhi = node;
        rlo = node + 1;
        rhi = hi;
    }
}

// KdTree.findNearest (kd-tree.ts:39-68) for one listed point per thread.  PRE = false: the
// splitting values through S and the exact distance computed at each visited node; PRE = true:
// both read from the tree-position layouts of k_tree_split / k_tree_dist (row t of dist)
template <bool PRE>
__global__ __launch_bounds__(256) void k_kd_walk(int d, const float *__restrict__ cen, int k,
                                                 const uint32_t *__restrict__ S, const float *__restrict__ aos,
                                                 const float *__restrict__ caos, int ld,
                                                 const float *__restrict__ split, const double *__restrict__ dist,
                                                 const uint32_t *__restrict__ tie_pts, uint32_t count,
                                                 uint32_t *__restrict__ labels) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count) return;
    const uint32_t p = tie_pts[t];
    const float *prow = aos + (uint64_t)p * ld;
    auto split_of = [&](uint32_t node, uint32_t depth) {
        const uint32_t axis = depth % (uint32_t)d;
        return PRE ? (double)split[node] : (double)cen[(uint64_t)axis * k + S[node]];
    };
    double mind = __builtin_inf();
    uint32_t mini = 0xffffffffu;
    Frame stack[64];
    int sp = 0;
    uint32_t clo = 0, chi = (uint32_t)k, cdepth = 0;
    bool descend = true;
    while (true) {
        if (descend) {
            while (chi > clo) {
                stack[sp++] = Frame{clo, chi, cdepth};
                uint32_t node, llo, lhi, rlo, rhi;
                seg_split(clo, chi, node, llo, lhi, rlo, rhi);
                const double distance = (double)prow[cdepth % (uint32_t)d] - split_of(node, cdepth);
                if (distance > 0) {
                    clo = rlo;
                    chi = rhi;
                } else {
                    clo = llo;
                    chi = lhi;
                }
                ++cdepth;
            }
        }
        if (sp == 0) break;
        const Frame f = stack[--sp];
        uint32_t node, llo, lhi, rlo, rhi;
        seg_split(f.lo, f.hi, node, llo, lhi, rlo, rhi);
        const double distance = (double)prow[f.depth % (uint32_t)d] - split_of(node, f.depth);
        const double thisd = PRE ? dist[(uint64_t)t * k + node] : kd_dist(caos + (uint64_t)S[node] * ld, prow, ld);
        if (thisd < mind) {
            mind = thisd;
            mini = S[node];
        }
        const uint32_t olo = (distance > 0) ? llo : rlo, ohi = (distance > 0) ? lhi : rhi;
        if (distance * distance < mind && ohi > olo) {
            clo = olo;
            chi = ohi;
            cdepth = f.depth + 1;
            descend = true;
        } else {
            descend = false;
        }
    }
    labels[p] = mini;
}

// ---- few walkers: every distance precomputed in tree order --------------------------
// After the equal rows have merged, a handful of points may each walk most of the tree
// (a duplicated row meets a coinciding centroid late): their splitting values and exact
// distances are laid out by tree position, so a visit is one load round instead of a chain
// through S and the 45-dim distance.
__global__ __launch_bounds__(256) void k_tree_split(const float *__restrict__ cen, int k, int d,
                                                    const uint32_t *__restrict__ S,
                                                    const uint8_t *__restrict__ depth, float *__restrict__ split) {
    for (uint32_t pos = blockIdx.x * blockDim.x + threadIdx.x; pos < (uint32_t)k; pos += gridDim.x * blockDim.x)
        split[pos] = cen[(uint64_t)(depth[pos] % d) * k + S[pos]];
}
__global__ __launch_bounds__(256) void k_tree_dist(const float *__restrict__ aos, const float *__restrict__ caos,
                                                   int ld, int k, const uint32_t *__restrict__ S,
                                                   const uint32_t *__restrict__ walkers, double *__restrict__ dist) {
    const uint32_t w = blockIdx.y;
    const float *prow = aos + (uint64_t)walkers[w] * ld;
    for (uint32_t pos = blockIdx.x * blockDim.x + threadIdx.x; pos < (uint32_t)k; pos += gridDim.x * blockDim.x)
        dist[(uint64_t)w * k + pos] = kd_dist(caos + (uint64_t)S[pos] * ld, prow, ld);
}
// ---- equal rows walk once ----------------------------------------------------------
// Duplicated points (e.g. all-zero SH rows) tie on every coinciding centroid and all take the
// same walk: the listed points are sorted by a hash of their row, a point whose row equals its
// predecessor's in that order takes its result, only the others walk.
__device__ inline uint64_t row_hash(const float *__restrict__ row, int ld) {
    uint64_t h = 0x9e3779b97f4a7c15ull;
    for (int i = 0; i < ld; ++i) {
        h ^= __builtin_bit_cast(uint32_t, row[i]);
        h *= 0xff51afd7ed558ccdull;
        h ^= h >> 33;
    }
    return h;
}

__global__ __launch_bounds__(256) void k_tie_hash(const float *__restrict__ aos, int ld,
                                                  const uint32_t *__restrict__ tie_pts, uint32_t nties,
                                                  uint64_t *__restrict__ keys, uint32_t *__restrict__ vals) {
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < nties; t += gridDim.x * blockDim.x) {
        keys[t] = row_hash(aos + (uint64_t)tie_pts[t] * ld, ld);
        vals[t] = t;
    }
}

// flag[j] = 1: position j of the hash order walks (first of its hash, or a row that differs
// from its predecessor's, bit for bit)
__global__ __launch_bounds__(256) void k_tie_flags(const uint64_t *__restrict__ keys, const uint32_t *__restrict__ vals,
                                                   const uint32_t *__restrict__ tie_pts, const float *__restrict__ aos,
                                                   int ld, uint32_t nties, uint32_t *__restrict__ flag) {
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < nties; j += gridDim.x * blockDim.x) {
        uint32_t f = 1u;
        if (j > 0 && keys[j] == keys[j - 1]) {
            const uint32_t *a = reinterpret_cast<const uint32_t *>(aos + (uint64_t)tie_pts[vals[j]] * ld);
            const uint32_t *b = reinterpret_cast<const uint32_t *>(aos + (uint64_t)tie_pts[vals[j - 1]] * ld);
            f = 0u;
            for (int i = 0; i < ld && !f; ++i) f = a[i] != b[i];
        }
        flag[j] = f;
    }
}

__global__ __launch_bounds__(256) void k_tie_compact(const uint32_t *__restrict__ flag, const uint32_t *__restrict__ pos,
                                                     const uint32_t *__restrict__ vals,
                                                     const uint32_t *__restrict__ tie_pts, uint32_t nties,
                                                     uint32_t *__restrict__ walkers) {
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < nties; j += gridDim.x * blockDim.x)
        if (flag[j]) walkers[pos[j]] = tie_pts[vals[j]];
}

// a point that did not walk takes the label of the nearest walker before it in hash order
__global__ __launch_bounds__(256) void k_tie_copy(const uint32_t *__restrict__ flag, const uint32_t *__restrict__ pos,
                                                  const uint32_t *__restrict__ vals,
                                                  const uint32_t *__restrict__ tie_pts, const uint32_t *__restrict__ walkers,
                                                  uint32_t nties, uint32_t *__restrict__ labels) {
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < nties; j += gridDim.x * blockDim.x)
        if (!flag[j]) labels[tie_pts[vals[j]]] = labels[walkers[pos[j] - 1]];
}

// ---- coinciding centroids ----------------------------------------------------------
// Duplicated input rows make the init (and re-seeds) draw several centroids with the same
// row.  They are at exactly the same distance from every point, so a point whose nearest row
// is such a group ties on all of its members and the reference's answer is the member its
// KdTree walk meets first.  The assign therefore sweeps one representative per distinct row
// (the group's lowest index) and settles a point that lands on a group of several with a
// descent of the reference's tree (k_group_descent) instead of a walk over it.
//
// Rows compare as the distance sees them: -0 and +0 are the same coordinate (every difference
// and square, and the tree's sort key, treat them alike).
__device__ inline uint32_t canon_bits(float x) { return __builtin_bit_cast(uint32_t, x == 0.0f ? 0.0f : x); }

// open-addressing table keyed by a 64-bit hash of the canonical row; the slot keeps the
// lowest index that inserted it
__global__ __launch_bounds__(256) void k_cen_hash(const float *__restrict__ cen, int d, int k,
                                                  unsigned long long *__restrict__ tkey, uint32_t *__restrict__ tval,
                                                  uint32_t tmask, uint32_t *__restrict__ gslot) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (uint32_t)k; i += gridDim.x * blockDim.x) {
        uint64_t h = 0x9e3779b97f4a7c15ull;
        for (int a = 0; a < d; ++a) {
            h ^= canon_bits(cen[(uint64_t)a * k + i]);
            h *= 0xff51afd7ed558ccdull;
            h ^= h >> 33;
        }
        h |= 1ull;  // 0 marks an empty slot
        uint32_t slot = (uint32_t)(h >> 17) & tmask;
        for (;;) {
            const unsigned long long prev = atomicCAS(&tkey[slot], 0ull, (unsigned long long)h);
            if (prev == 0ull || prev == h) {
                atomicMin(&tval[slot], i);
                gslot[i] = slot;
                break;
            }
            slot = (slot + 1) & tmask;
        }
    }
}

// rep[i] = the lowest index with i's row; a hash collision between different rows (a member
// whose row differs from its representative's) is reported and the caller keeps every centroid
__global__ __launch_bounds__(256) void k_cen_group(const float *__restrict__ cen, int d, int k,
                                                   const uint32_t *__restrict__ tval, const uint32_t *__restrict__ gslot,
                                                   uint32_t *__restrict__ rep, uint32_t *__restrict__ is_rep,
                                                   uint32_t *__restrict__ stat) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (uint32_t)k; i += gridDim.x * blockDim.x) {
        const uint32_t r = tval[gslot[i]];
        bool same = r <= i;
        for (int a = 0; a < d && same; ++a) same = canon_bits(cen[(uint64_t)a * k + i]) == canon_bits(cen[(uint64_t)a * k + r]);
        if (!same) atomicOr(&stat[1], 1u);
        rep[i] = r;
        is_rep[i] = r == i ? 1u : 0u;
        if (r != i) atomicAdd(&stat[0], 1u);
    }
}

// the representatives' rows as a [d][kr] centroid table; grp[i] = the slot of i's group
__global__ __launch_bounds__(256) void k_cen_compact(const float *__restrict__ cen, int d, int k,
                                                     const uint32_t *__restrict__ rep,
                                                     const uint32_t *__restrict__ rslot, uint32_t kr,
                                                     float *__restrict__ cen_r, uint32_t *__restrict__ map_r2c,
                                                     uint32_t *__restrict__ grp) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (uint32_t)k; i += gridDim.x * blockDim.x) {
        const uint32_t g = rslot[rep[i]];
        grp[i] = g;
        if (rep[i] == i) {
            map_r2c[g] = i;
            for (int a = 0; a < d; ++a) cen_r[(uint64_t)a * kr + g] = cen[(uint64_t)a * k + i];
        }
    }
}

// (group slot << 32 | tree position) of every centroid: sorted, each group's positions ascend
__global__ __launch_bounds__(256) void k_group_keys(const uint32_t *__restrict__ S, const uint32_t *__restrict__ grp,
                                                    int k, uint64_t *__restrict__ keys) {
    for (uint32_t pos = blockIdx.x * blockDim.x + threadIdx.x; pos < (uint32_t)k; pos += gridDim.x * blockDim.x)
        keys[pos] = ((uint64_t)grp[S[pos]] << 32) | pos;
}
__global__ __launch_bounds__(256) void k_group_starts(const uint64_t *__restrict__ keys, int k, uint32_t kr,
                                                      uint32_t *__restrict__ gstart, uint32_t *__restrict__ gpos) {
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < (uint32_t)k; j += gridDim.x * blockDim.x) {
        const uint32_t g = (uint32_t)(keys[j] >> 32);
        gpos[j] = (uint32_t)keys[j];
        if (j == 0 || (uint32_t)(keys[j - 1] >> 32) != g) gstart[g] = j;
        if (j == 0) gstart[kr] = (uint32_t)k;
    }
}

// labels[p] holds the slot of p's nearest distinct row (the unique minimum).  A group of one:
// its centroid.  A group of several: every member is at p's minimal distance and no other
// centroid is, so the reference's walk (kd-tree.ts:39-68) returns the first member it visits.
// Its pruning never skips a member before one is found (a subtree is skipped only when every
// node in it is at least the current best away), so that member is the first in the walk's
// visit order: at each node the near side's subtree, then the node, then the far side.  The
// descent follows that order, asking at each node whether the near subtree -- a contiguous
// range of tree positions -- holds a member (binary search in the group's sorted positions).
__global__ __launch_bounds__(256) void k_group_descent(int d, int k, const uint32_t *__restrict__ S,
                                                       const float *__restrict__ split,
                                                       const uint32_t *__restrict__ gstart,
                                                       const uint32_t *__restrict__ gpos,
                                                       const uint32_t *__restrict__ map_r2c,
                                                       const float *__restrict__ aos, int ld, uint64_t n,
                                                       uint32_t *__restrict__ labels, uint32_t *__restrict__ err) {
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t g = labels[p];
        const uint32_t s = gstart[g], e = gstart[g + 1];
        if (e - s == 1) {
            labels[p] = map_r2c[g];
            continue;
        }
        auto any_in = [&](uint32_t a, uint32_t b) {
            if (b <= a) return false;
            uint32_t lo = s, hi = e;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (gpos[mid] < a) lo = mid + 1;
                else hi = mid;
            }
            return lo < e && gpos[lo] < b;
        };
        const float *prow = aos + p * ld;
        uint32_t lo = 0, hi = (uint32_t)k, depth = 0, got = 0xffffffffu;
        while (hi > lo && depth < 64) {
            uint32_t node, llo, lhi, rlo, rhi;
            seg_split(lo, hi, node, llo, lhi, rlo, rhi);
            const double distance = (double)prow[depth % (uint32_t)d] - (double)split[node];
            const bool right = distance > 0;
            const uint32_t nlo = right ? rlo : llo, nhi = right ? rhi : lhi;
            if (any_in(nlo, nhi)) {
                lo = nlo, hi = nhi;
            } else if (any_in(node, node + 1)) {
                got = S[node];
                break;
            } else {
                lo = right ? llo : rlo, hi = right ? lhi : rhi;
            }
            ++depth;
        }
        if (got == 0xffffffffu) atomicOr(err, ERR_INTERNAL);  // cannot happen: the group is in the tree
        labels[p] = got;
    }
}

std::unordered_map<int64_t, std::unique_ptr<KdLayout>> &layouts() {
    static thread_local std::unordered_map<int64_t, std::unique_ptr<KdLayout>> m;
    return m;
}

KdLayout &layout_of(st_ctx *c, int k) {
    auto &L = layouts()[((int64_t)c->device << 32) | (uint32_t)k];
    if (!L) L = make_layout(k);
    return *L;
}

}  // namespace

// KdTree.build (kd-tree.ts:73-99) of the centroids cen [d][k]: S[tree position] = centroid
const uint32_t *kd_build(st_ctx *c, int d, int k, const float *cen) {
    KdLayout &L = layout_of(c, k);
    auto *S = wsT<uint32_t>(c, "kd.S", (size_t)k);
    auto *keys = wsT<uint64_t>(c, "kd.keys", (size_t)k);
    auto *vals = wsT<uint32_t>(c, "kd.vals", (size_t)k);
    iota_u32(c, S, (uint64_t)k);
    for (size_t lv = 0; lv < L.levels.size(); ++lv) {
        const Level &v = L.levels[lv];
        const int axis = (int)(lv % (size_t)d);
        hipLaunchKernelGGL(k_level_keys, dim3(grid_for(v.count, 256, 1024)), dim3(256), 0, c->stream, cen, k, axis, S,
                           v.pos, v.rank, v.count, keys, vals);
        ST_LAUNCH_CHECK();
        radix_sort_u64(c, keys, vals, v.count, 0, 32 + (int)v.seg_bits, "kd.rs");
        hipLaunchKernelGGL(k_level_scatter, dim3(grid_for(v.count, 256, 1024)), dim3(256), 0, c->stream, v.pos, vals,
                           v.count, S);
        ST_LAUNCH_CHECK();
    }
    return S;
}

bool cen_groups(st_ctx *c, int d, int k, const float *cen, CenGroups *out) {
    uint32_t tsize = 1024;
    while (tsize < 4u * (uint32_t)k) tsize <<= 1;
    auto *tkey = wsT<unsigned long long>(c, "cg.tkey", tsize);
    auto *tval = wsT<uint32_t>(c, "cg.tval", tsize);
    auto *gslot = wsT<uint32_t>(c, "cg.gslot", (size_t)k);
    auto *rep = wsT<uint32_t>(c, "cg.rep", (size_t)k);
    auto *is_rep = wsT<uint32_t>(c, "cg.isrep", (size_t)k + 1);
    auto *stat = wsT<uint32_t>(c, "cg.stat", 4);  // [0] non-representatives [1] collision [2] kr
    ST_HIP(hipMemsetAsync(tkey, 0, (size_t)tsize * 8, c->stream));
    ST_HIP(hipMemsetAsync(tval, 0xff, (size_t)tsize * 4, c->stream));
    ST_HIP(hipMemsetAsync(stat, 0, 16, c->stream));
    const unsigned g = grid_for((uint64_t)k, 256, 1024);
    hipLaunchKernelGGL(k_cen_hash, dim3(g), dim3(256), 0, c->stream, cen, d, k, tkey, tval, tsize - 1, gslot);
    hipLaunchKernelGGL(k_cen_group, dim3(g), dim3(256), 0, c->stream, cen, d, k, tval, gslot, rep, is_rep, stat);
    ST_LAUNCH_CHECK();
    auto *h = static_cast<uint32_t *>(pinned_slot(c, "cg.stat", 16));
    ST_HIP(hipMemcpyAsync(h, stat, 8, hipMemcpyDeviceToHost, c->stream));
    ST_HIP(hipStreamSynchronize(c->stream));
    if (h[0] == 0 || h[1] != 0) return false;  // all rows distinct (or a hash collision: keep all)
    auto *rslot = wsT<uint32_t>(c, "cg.rslot", (size_t)k + 1);
    scan_u32(c, is_rep, rslot, (uint64_t)k, rslot + k);
    const uint32_t kr = (uint32_t)k - h[0];
    out->kr = kr;
    out->cen_r = wsT<float>(c, "cg.cen", (size_t)kr * d);
    out->map_r2c = wsT<uint32_t>(c, "cg.map", kr);
    out->grp = wsT<uint32_t>(c, "cg.grp", (size_t)k);
    hipLaunchKernelGGL(k_cen_compact, dim3(g), dim3(256), 0, c->stream, cen, d, k, rep, rslot, kr, out->cen_r,
                       out->map_r2c, out->grp);
    ST_LAUNCH_CHECK();
    return true;
}

void kd_group_labels(st_ctx *c, int d, int k, const float *cen, const CenGroups &g, const float *aos, int ld,
                     uint64_t n, uint32_t *labels, uint32_t *err) {
    KdLayout &L = layout_of(c, k);
    const uint32_t *S = kd_build(c, d, k, cen);
    auto *split = wsT<float>(c, "kd.split", (size_t)k);
    auto *keys = wsT<uint64_t>(c, "cg.keys", (size_t)k);
    auto *vals = wsT<uint32_t>(c, "cg.vals", (size_t)k);
    auto *gstart = wsT<uint32_t>(c, "cg.gstart", (size_t)g.kr + 1);
    auto *gpos = wsT<uint32_t>(c, "cg.gpos", (size_t)k);
    const unsigned gk = grid_for((uint64_t)k, 256, 1024);
    hipLaunchKernelGGL(k_tree_split, dim3(gk), dim3(256), 0, c->stream, cen, k, d, S, L.depth, split);
    hipLaunchKernelGGL(k_group_keys, dim3(gk), dim3(256), 0, c->stream, S, g.grp, k, keys);
    ST_LAUNCH_CHECK();
    int bits = 0;
    while ((1u << bits) < g.kr) ++bits;
    radix_sort_u64(c, keys, vals, (uint64_t)k, 0, 32 + bits, "cg.rs");
    hipLaunchKernelGGL(k_group_starts, dim3(gk), dim3(256), 0, c->stream, keys, k, g.kr, gstart, gpos);
    hipLaunchKernelGGL(k_group_descent, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c->stream, d, k, S, split,
                       gstart, gpos, g.map_r2c, aos, ld, n, labels, err);
    ST_LAUNCH_CHECK();
}

void kd_resolve_ties(st_ctx *c, int d, int k, const float *cen, const float *aos, const float *caos, int ld,
                     const uint32_t *tie_pts, uint32_t nties, uint32_t *labels, bool tree_built) {
    KdLayout *L = &layout_of(c, k);
    const uint32_t *S = tree_built ? wsT<uint32_t>(c, "kd.S", (size_t)k) : kd_build(c, d, k, cen);
    // one thread per listed point, distances computed at the visited nodes only
    if (nties < 4096) {
        hipLaunchKernelGGL(k_kd_walk<false>, dim3((nties + 255) / 256), dim3(256), 0, c->stream, d, cen, k, S, aos,
                           caos, ld, (const float *)nullptr, (const double *)nullptr, tie_pts, nties, labels);
        ST_LAUNCH_CHECK();
        return;
    }
    auto *hk = wsT<uint64_t>(c, "kd.hkeys", nties);
    auto *hv = wsT<uint32_t>(c, "kd.hvals", nties);
    auto *flag = wsT<uint32_t>(c, "kd.flag", nties);
    auto *pos = wsT<uint32_t>(c, "kd.pos", (size_t)nties + 1);
    auto *walkers = wsT<uint32_t>(c, "kd.walkers", nties);
    const unsigned g = grid_for(nties, 256, 4096);
    hipLaunchKernelGGL(k_tie_hash, dim3(g), dim3(256), 0, c->stream, aos, ld, tie_pts, nties, hk, hv);
    ST_LAUNCH_CHECK();
    radix_sort_u64(c, hk, hv, nties, 0, 64, "kd.hs");
    hipLaunchKernelGGL(k_tie_flags, dim3(g), dim3(256), 0, c->stream, hk, hv, tie_pts, aos, ld, nties, flag);
    ST_LAUNCH_CHECK();
    scan_u32(c, flag, pos, nties, pos + nties);
    hipLaunchKernelGGL(k_tie_compact, dim3(g), dim3(256), 0, c->stream, flag, pos, hv, tie_pts, nties, walkers);
    ST_LAUNCH_CHECK();
    auto *hw = static_cast<uint32_t *>(pinned_slot(c, "kd.nwalk", 4));
    ST_HIP(hipMemcpyAsync(hw, pos + nties, 4, hipMemcpyDeviceToHost, c->stream));
    ST_HIP(hipStreamSynchronize(c->stream));
    const uint32_t nw = hw[0];
    if (nw <= 64) {
        auto *split = wsT<float>(c, "kd.split", (size_t)k);
        auto *tdist = wsT<double>(c, "kd.tdist", (size_t)nw * k);
        hipLaunchKernelGGL(k_tree_split, dim3(grid_for(k, 256, 1024)), dim3(256), 0, c->stream, cen, k, d, S, L->depth,
                           split);
        hipLaunchKernelGGL(k_tree_dist, dim3(grid_for(k, 256, 256), nw), dim3(256), 0, c->stream, aos, caos, ld, k, S,
                           walkers, tdist);
        hipLaunchKernelGGL(k_kd_walk<true>, dim3((nw + 255) / 256), dim3(256), 0, c->stream, d, cen, k, S, aos, caos,
                           ld, split, tdist, walkers, nw, labels);
    } else {
        hipLaunchKernelGGL(k_kd_walk<false>, dim3((nw + 255) / 256), dim3(256), 0, c->stream, d, cen, k, S, aos,
                           caos, ld, (const float *)nullptr, (const double *)nullptr, walkers, nw, labels);
    }
    hipLaunchKernelGGL(k_tie_copy, dim3(g), dim3(256), 0, c->stream, flag, pos, hv, tie_pts, walkers, nties, labels);
    ST_LAUNCH_CHECK();
}

}  // namespace st
