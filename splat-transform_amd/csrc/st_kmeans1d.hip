// st_kmeans1d.hip -- 1-D k-means (cluster1d's K=256 codebooks, write-sog.ts:56-99).
//
// Assign: the reference rebuilds a KdTree over the centroids every iteration
// (k-means.ts:104).  With one column every level sorts by the same key, so the
// tree is the implicit BST over the stably sorted centroid values: segment
// [lo,hi) has its node at lo+(len>>1) (len 2: node lo, right child lo+1).  Each
// point walks that tree exactly like KdTree.findNearest (kd-tree.ts:39-68):
// nearer child first, strict `<` on the f64 squared distance, prune when
// distance^2 >= best.  This reproduces the reference's tie-break bit-for-bit.
//
// Update: a stable sort by label lays each cluster's values out contiguously in
// ascending point order.  One workgroup per cluster sums them in f64: in
// parallel when every value is a multiple of 2^e and sum|x| < 2^(e+53) (then
// every partial sum is exact, so any order equals calcAverage's sequential
// sum), otherwise in the reference's order.
#include "st_jsmath.h"
#include "st_kmeans.h"
#include "st_replay.h"

namespace st {
namespace {

using namespace km;

constexpr int KD1_LDS = 4096;  // centroids kept in LDS up to this K

__global__ __launch_bounds__(256) void k_sortkeys(const float *cen, int k, uint32_t *keys, uint32_t *vals) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < k; i += gridDim.x * blockDim.x) {
        keys[i] = sortkey_(cen[i]);
        vals[i] = (uint32_t)i;
    }
}

struct Seg {
    uint32_t lo, hi;
};

// node / children of an implicit-tree segment
__device__ inline void seg_node(Seg s, uint32_t &node, Seg &left, Seg &right) {
    const uint32_t len = s.hi - s.lo;
    if (len == 1) {
        node = s.lo;
        left = right = Seg{0, 0};
    } else if (len == 2) {
        node = s.lo;
        left = Seg{0, 0};
        right = Seg{s.lo + 1, s.lo + 2};
    } else {
        const uint32_t mid = s.lo + (len >> 1);
        node = mid;
        left = Seg{s.lo, mid};
        right = Seg{mid + 1, s.hi};
    }
}

// KdTree.findNearest over the implicit tree (the reference's visit order and strict `<`)
template <typename V, typename I>
__device__ inline uint32_t kd1_walk(double p, int k, V val, I idx) {
    double mind = __builtin_inf();
    uint32_t mini = 0xffffffffu;
    Seg stack[24];
    int sp = 0;
    Seg cur{0, (uint32_t)k};
    bool descend = true;
    while (true) {
        if (descend) {
            // go down the `next` chain, remembering each frame
            while (cur.hi > cur.lo) {
                stack[sp++] = cur;
                uint32_t node;
                Seg l, r;
                seg_node(cur, node, l, r);
                const double distance = p - (double)val(node);
                cur = (distance > 0) ? r : l;
            }
        }
        if (sp == 0) break;
        const Seg f = stack[--sp];
        uint32_t node;
        Seg l, r;
        seg_node(f, node, l, r);
        const double cv = val(node);
        const double distance = p - cv;
        const double v = cv - p;
        const double thisd = 0.0 + v * v;
        if (thisd < mind) {
            mind = thisd;
            mini = idx(node);
        }
        const Seg other = (distance > 0) ? l : r;
        if (distance * distance < mind && other.hi > other.lo) {
            cur = other;
            descend = true;
        } else {
            descend = false;
        }
    }
    return mini;
}

template <bool LDS>
__global__ __launch_bounds__(256) void k_kd1_assign(const float *__restrict__ pts, uint64_t n,
                                                    const float *__restrict__ cen, const uint32_t *__restrict__ order,
                                                    int k, uint32_t *__restrict__ labels) {
    __shared__ float sv[LDS ? KD1_LDS : 1];
    __shared__ uint32_t si[LDS ? KD1_LDS : 1];
    if (LDS) {
        for (int i = threadIdx.x; i < k; i += blockDim.x) {
            const uint32_t o = order[i];
            si[i] = o;
            sv[i] = cen[o];
        }
        __syncthreads();
    }
    auto val = [&](uint32_t pos) -> float { return LDS ? sv[pos] : cen[order[pos]]; };
    auto idx = [&](uint32_t pos) -> uint32_t { return LDS ? si[pos] : order[pos]; };
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        labels[i] = kd1_walk((double)pts[i], k, val, idx);
}

// The same answer without the walk.  With one dimension every centroid is a value on a
// line, and the rounded distance (c - p)^2 is monotone in |c - p| on each side of p, so
// the minimum is reached at the last centroid <= p (L) or the first > p (R).  If it is
// reached there only -- the rounded distances of L, R and of their outer neighbours differ
// from it -- it is the unique minimum, which the KdTree walk finds in any visit order.
// Otherwise (duplicate centroid values, equal rounded distances) the point takes the walk.
// R is located through a uniform grid of KD1_CELLS cells over [c_min, c_max]: a monotone
// cell map puts every centroid of a smaller cell below p and of a larger one above it.
constexpr int KD1_CELLS = 1024;
__global__ __launch_bounds__(256) void k_kd1_assign_fast(const float *__restrict__ pts, uint64_t n,
                                                         const float *__restrict__ cen,
                                                         const uint32_t *__restrict__ order, int k,
                                                         uint32_t *__restrict__ labels, uint32_t *__restrict__ keys,
                                                         uint32_t *__restrict__ vals) {
    __shared__ float sv[KD1_LDS];
    __shared__ uint32_t si[KD1_LDS];
    __shared__ uint16_t cc[KD1_LDS];
    __shared__ uint32_t first[KD1_CELLS + 1];
    for (int i = threadIdx.x; i < k; i += blockDim.x) {
        const uint32_t o = order[i];
        si[i] = o;
        sv[i] = cen[o];
    }
    __syncthreads();
    const float lo = sv[0], hi = sv[k - 1];
    const float span = hi - lo;
    const float inv = (span > 0.f && span < __builtin_inff()) ? (float)KD1_CELLS / span : 0.f;
    auto cell = [&](float x) -> int {
        const float t = (x - lo) * inv;
        return (int)__builtin_fminf(__builtin_fmaxf(t, 0.f), (float)(KD1_CELLS - 1));
    };
    for (int i = threadIdx.x; i < k; i += blockDim.x) cc[i] = (uint16_t)cell(sv[i]);
    __syncthreads();
    for (int g = threadIdx.x; g <= KD1_CELLS; g += blockDim.x) {  // first[g] = #{i : cc[i] < g}
        int a = 0, b = k;
        while (a < b) {
            const int m = (a + b) >> 1;
            if ((int)cc[m] < g) a = m + 1;
            else b = m;
        }
        first[g] = (uint32_t)a;
    }
    __syncthreads();
    auto dist = [&](int pos, double p) {
        const double v = (double)sv[pos] - p;
        return 0.0 + v * v;
    };
    auto val = [&](uint32_t pos) -> float { return sv[pos]; };
    auto idx = [&](uint32_t pos) -> uint32_t { return si[pos]; };
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float pnext = i < n ? pts[i] : 0.f;  // the next point's value is in flight while this one is placed
    for (; i < n; i += stride) {
        const float pf = pnext;
        if (i + stride < n) pnext = pts[i + stride];
        const double p = pf;
        const int g = cell(pf);
        int u = (int)first[g];
        const int ue = (int)first[g + 1];
        while (u < ue && sv[u] <= pf) ++u;  // R = u: the first centroid > p
        const int L = u - 1, R = u;
        const double dl = L >= 0 ? dist(L, p) : __builtin_inf();
        const double dr = R < k ? dist(R, p) : __builtin_inf();
        const double m = __builtin_fmin(dl, dr);
        const bool tie = dl == dr || (L >= 1 && dist(L - 1, p) == m) || (R + 1 < k && dist(R + 1, p) == m);
        uint32_t lab;
        if (!tie) lab = si[dl < dr ? L : R];
        else lab = kd1_walk(p, k, val, idx);
        if (labels) labels[i] = lab;  // only the last iteration's labels are the result
        if (keys) {  // the member-sort pairs of the update (label, value bits)
            keys[i] = lab;
            vals[i] = __builtin_bit_cast(uint32_t, pf);
        }
    }
}

// ---- fused iteration for k <= 256 (cluster1d's codebooks) ------------------------------
// The member sort only has to lay each cluster's values out in ascending point order: the
// label is an 8-bit digit, so one counting-sort pass does it, and the cluster starts are
// the scanned digit counts.  Assign + tile histogram in one kernel (byte labels out), the
// scan of the (digit, tile) counts, then a scatter that moves 4-byte values only: 14 bytes
// per point against 36 for assign -> (label, value) pairs -> radix pass -> bounds.
constexpr int F1_T = 256, F1_ROWS = 16, F1_TILE = F1_T * F1_ROWS, F1_WAVES = F1_T / 64;

// k_kd1_assign_fast's bracket assign over one 4,096-point tile per workgroup; lab8 = labels
// as bytes, labels (if non-null) the u32 result, hist[d * ntiles + tile] = count of digit d
__global__ __launch_bounds__(F1_T) void k_kd1_assign_hist(const float *__restrict__ pts, uint64_t n,
                                                         const float *__restrict__ cen,
                                                         const uint32_t *__restrict__ order, int k,
                                                         uint32_t *__restrict__ labels, uint8_t *__restrict__ lab8,
                                                         uint32_t *__restrict__ hist, uint32_t ntiles) {
    __shared__ float sv[256];
    __shared__ uint32_t si[256];
    __shared__ uint16_t cc[256];
    __shared__ uint32_t first[KD1_CELLS + 1];
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    for (int i = threadIdx.x; i < k; i += blockDim.x) {
        const uint32_t o = order[i];
        si[i] = o;
        sv[i] = cen[o];
    }
    const uint64_t base = (uint64_t)blockIdx.x * F1_TILE;
    float pv[F1_ROWS];  // the tile's points in flight while the tables are built
#pragma unroll
    for (int r = 0; r < F1_ROWS; ++r) {
        const uint64_t i = base + (uint64_t)r * F1_T + threadIdx.x;
        pv[r] = i < n ? pts[i] : 0.f;
    }
    __syncthreads();
    const float lo = sv[0], hi = sv[k - 1];
    const float span = hi - lo;
    const float inv = (span > 0.f && span < __builtin_inff()) ? (float)KD1_CELLS / span : 0.f;
    auto cell = [&](float x) -> int {
        const float t = (x - lo) * inv;
        return (int)__builtin_fminf(__builtin_fmaxf(t, 0.f), (float)(KD1_CELLS - 1));
    };
    for (int i = threadIdx.x; i < k; i += blockDim.x) cc[i] = (uint16_t)cell(sv[i]);
    __syncthreads();
    for (int g = threadIdx.x; g <= KD1_CELLS; g += blockDim.x) {
        int a = 0, b = k;
        while (a < b) {
            const int m = (a + b) >> 1;
            if ((int)cc[m] < g) a = m + 1;
            else b = m;
        }
        first[g] = (uint32_t)a;
    }
    __syncthreads();
    auto dist = [&](int pos, double p) {
        const double v = (double)sv[pos] - p;
        return 0.0 + v * v;
    };
    auto val = [&](uint32_t pos) -> float { return sv[pos]; };
    auto idx = [&](uint32_t pos) -> uint32_t { return si[pos]; };
#pragma unroll
    for (int r = 0; r < F1_ROWS; ++r) {
        const uint64_t i = base + (uint64_t)r * F1_T + threadIdx.x;
        if (i >= n) break;
        const float pf = pv[r];
        const double p = pf;
        const int g = cell(pf);
        int u = (int)first[g];
        const int ue = (int)first[g + 1];
        while (u < ue && sv[u] <= pf) ++u;
        const int L = u - 1, R = u;
        const double dl = L >= 0 ? dist(L, p) : __builtin_inf();
        const double dr = R < k ? dist(R, p) : __builtin_inf();
        const double m = __builtin_fmin(dl, dr);
        const bool tie = dl == dr || (L >= 1 && dist(L - 1, p) == m) || (R + 1 < k && dist(R + 1, p) == m);
        const uint32_t lab = !tie ? si[dl < dr ? L : R] : kd1_walk(p, k, val, idx);
        lab8[i] = (uint8_t)lab;
        if (labels) labels[i] = lab;
        atomicAdd(&h[lab], 1u);
    }
    __syncthreads();
    hist[(uint64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// stable counting-sort pass on the byte labels moving the value bits only: each wave ranks its
// 1,024 points with ballots over the `bits` label bits, the tile is reordered by label in LDS
// and each label's run is stored contiguously at its scanned offset
template <typename L>
__global__ __launch_bounds__(F1_T) void k_lab_scatter(const L *__restrict__ lab8, const float *__restrict__ pts,
                                                      uint64_t n, int bits, const uint32_t *__restrict__ offs,
                                                      uint32_t ntiles, uint32_t *__restrict__ ovals) {
    __shared__ uint32_t wcount[F1_WAVES][256];
    __shared__ uint32_t wbase[F1_WAVES][256];
    __shared__ uint32_t goff[256];
    __shared__ uint32_t dstart[256];
    __shared__ uint32_t wtot[F1_WAVES];
    __shared__ uint32_t sval[F1_TILE];
    __shared__ uint8_t sdig[F1_TILE];
    for (int i = threadIdx.x; i < F1_WAVES * 256; i += F1_T) (&wcount[0][0])[i] = 0;
    goff[threadIdx.x] = offs[(uint64_t)threadIdx.x * ntiles + blockIdx.x];
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const uint64_t tbase = (uint64_t)blockIdx.x * F1_TILE;
    const uint64_t wb = tbase + (uint64_t)w * 64 * F1_ROWS;
    uint32_t v[F1_ROWS], off[F1_ROWS], dg[F1_ROWS];
#pragma unroll
    for (int r = 0; r < F1_ROWS; ++r) {
        const uint64_t e = wb + (uint64_t)r * 64 + lane;
        const bool valid = e < n;
        dg[r] = valid ? (uint32_t)lab8[e] : 0u;
        v[r] = valid ? __builtin_bit_cast(uint32_t, pts[e]) : 0u;
    }
#pragma unroll
    for (int r = 0; r < F1_ROWS; ++r) {
        const uint64_t e = wb + (uint64_t)r * 64 + lane;
        const bool valid = e < n;
        const uint32_t d = dg[r];
        uint64_t peers = __ballot(valid);
        for (int b = 0; b < bits; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint32_t rank = __popcll(peers & lt);
        const uint32_t before = valid ? wcount[w][d] : 0u;
        off[r] = before + rank;
        if (valid && (peers & lt) == 0) wcount[w][d] = before + (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    {
        const int d = threadIdx.x;
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < F1_WAVES; ++i) {
            wbase[i][d] = s;
            s += wcount[i][d];
        }
        uint32_t incl = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(incl, o, 64);
            if (lane >= o) incl += u;
        }
        if (lane == 63) wtot[w] = incl;
        __syncthreads();
        uint32_t woff = 0;
        for (int i = 0; i < w; ++i) woff += wtot[i];
        dstart[d] = woff + incl - s;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < F1_ROWS; ++r) {
        const uint64_t e = wb + (uint64_t)r * 64 + lane;
        if (e < n) {
            const uint32_t lp = dstart[dg[r]] + wbase[w][dg[r]] + off[r];
            sval[lp] = v[r];
            sdig[lp] = (uint8_t)dg[r];
        }
    }
    __syncthreads();
    const uint32_t cnt = (uint32_t)((n - tbase) < (uint64_t)F1_TILE ? (n - tbase) : (uint64_t)F1_TILE);
    for (uint32_t i = threadIdx.x; i < cnt; i += F1_T) {
        const uint32_t d = sdig[i];
        ovals[goff[d] + (i - dstart[d])] = sval[i];
    }
}

// cluster starts from the scanned (digit, tile) counts: start[c] = base + offs[c * ntiles],
// start[k] = base + n
__global__ void k_f1_starts(const uint32_t *__restrict__ offs, uint32_t ntiles, int k, uint64_t n,
                            uint32_t *__restrict__ start, uint32_t base = 0) {
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c <= k; c += gridDim.x * blockDim.x)
        start[c] = base + (c < k ? offs[(uint64_t)c * ntiles] : (uint32_t)n);
}

// tile histogram of given u32 labels (< 256): hist[d * ntiles + tile]
__global__ __launch_bounds__(F1_T) void k_lab_hist(const uint32_t *__restrict__ labels, uint64_t n,
                                                   uint32_t *__restrict__ hist, uint32_t ntiles) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * F1_TILE;
#pragma unroll 4
    for (int r = 0; r < F1_ROWS; ++r) {
        const uint64_t i = base + (uint64_t)r * F1_T + threadIdx.x;
        if (i < n) atomicAdd(&h[labels[i] & 255u], 1u);
    }
    __syncthreads();
    hist[(uint64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// pairs for the member sort: key = label, val = value bits (ascending point order kept)
__global__ __launch_bounds__(256) void k_pairs1d(const float *pts, const uint32_t *labels, uint64_t n,
                                                 uint32_t *keys, uint32_t *vals) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        keys[i] = labels[i];
        vals[i] = __builtin_bit_cast(uint32_t, pts[i]);
    }
}


// the sequential f64 sum of members [s0, s1) on the calling lane: the loads run PF x 16 bytes
// ahead of the dependent add chain
__device__ inline double seq_sum1d(const uint32_t *__restrict__ vals, uint32_t s0, uint32_t s1) {
    double s = 0;
    uint32_t j = s0;
    for (; j < s1 && (j & 3u); ++j) s += (double)__builtin_bit_cast(float, vals[j]);
    const uint32_t nq = (s1 - j) >> 2;
    // a zero the compiler cannot see keeps the (uniform) loads on the vector path: scalar
    // loads would each need an lgkmcnt(0) wait and serialise the chain
    uint32_t opaque0;
    asm volatile("v_mov_b32 %0, 0" : "=v"(opaque0));
    const uint4 *q = reinterpret_cast<const uint4 *>(vals + j) + opaque0;
    constexpr uint32_t PF = 16;
    uint4 buf[PF];
#pragma unroll
    for (uint32_t u = 0; u < PF; ++u) buf[u] = (u < nq) ? q[u] : make_uint4(0, 0, 0, 0);
    uint32_t i = 0;
    for (; i + PF <= nq; i += PF) {
#pragma unroll
        for (uint32_t u = 0; u < PF; ++u) {
            const uint4 v = buf[u];
            buf[u] = (i + u + PF < nq) ? q[i + u + PF] : make_uint4(0, 0, 0, 0);
            s += (double)__builtin_bit_cast(float, v.x);
            s += (double)__builtin_bit_cast(float, v.y);
            s += (double)__builtin_bit_cast(float, v.z);
            s += (double)__builtin_bit_cast(float, v.w);
        }
    }
#pragma unroll
    for (uint32_t u = 0; u < PF; ++u) {  // buf[u] holds quad i + u
        if (i + u < nq) {
            const uint4 v = buf[u];
            s += (double)__builtin_bit_cast(float, v.x);
            s += (double)__builtin_bit_cast(float, v.y);
            s += (double)__builtin_bit_cast(float, v.z);
            s += (double)__builtin_bit_cast(float, v.w);
        }
    }
    for (j += nq * 4; j < s1; ++j) s += (double)__builtin_bit_cast(float, vals[j]);
    return s;
}

// the sequential f64 sum of a flagged cluster (flag 2): one lane walks the members in order
__global__ __launch_bounds__(64) void k_sum1d_seq(const uint32_t *__restrict__ vals, const uint32_t *__restrict__ start,
                                                  const uint32_t *__restrict__ seq_flag, float *__restrict__ cen) {
    const int cl = blockIdx.x;
    if (seq_flag[cl] != 2u || threadIdx.x != 0) return;
    const uint32_t s0 = start[cl], s1 = start[cl + 1];
    cen[cl] = (float)(seq_sum1d(vals, s0, s1) / (double)(s1 - s0));
}

// ---- chunked update: every cluster's members split into SC_CH-member chunks ----------
// One workgroup per chunk instead of one per cluster: the clusters of a 1-D codebook are
// few (256) and uneven (the one straddling 0 can hold 1.5% of 30M points), so a
// per-cluster workgroup leaves the chip idle behind the largest cluster.
constexpr uint32_t SC_CH = 4096;  // members per chunk
constexpr uint32_t FL_CH = 512;   // members per chunk of the flagged clusters' replay
constexpr int SC_T = 256;         // threads per chunk (16 members each)

struct Chunk {
    uint32_t cl, begin, end, pad;
};

__global__ __launch_bounds__(256) void k_chunk_counts(const uint32_t *__restrict__ start, int k,
                                                      uint32_t *__restrict__ cnt) {
    for (int cl = blockIdx.x * blockDim.x + threadIdx.x; cl < k; cl += gridDim.x * blockDim.x)
        cnt[cl] = (start[cl + 1] - start[cl] + SC_CH - 1) / SC_CH;
}

__global__ __launch_bounds__(256) void k_chunk_list(const uint32_t *__restrict__ start, int k,
                                                    const uint32_t *__restrict__ first, Chunk *__restrict__ chunks) {
    for (int cl = blockIdx.x * blockDim.x + threadIdx.x; cl < k; cl += gridDim.x * blockDim.x) {
        const uint32_t s0 = start[cl], s1 = start[cl + 1];
        uint32_t o = first[cl];
        for (uint32_t b = s0; b < s1; b += SC_CH) chunks[o++] = Chunk{(uint32_t)cl, b, min(s1, b + SC_CH), 0u};
    }
}

// per-cluster accumulators of the certificate pass
struct SumAcc {
    double sum, sabs;
    int emin;
    int pad;
};

__global__ __launch_bounds__(256) void k_sumacc_init(SumAcc *acc, int k) {
    for (int cl = blockIdx.x * blockDim.x + threadIdx.x; cl < k; cl += gridDim.x * blockDim.x)
        acc[cl] = SumAcc{0.0, 0.0, 1 << 20, 0};
}

// chunk partials of sum, sum|x|, min ulp exponent.  Under the certificate every partial sum
// is exact, so the block reduction and the atomic order are immaterial; otherwise the sum
// is discarded (the replay below recomputes it).
__global__ __launch_bounds__(SC_T) void k_sum1d_chunks(const uint32_t *__restrict__ vals,
                                                      const Chunk *__restrict__ chunks,
                                                      const uint32_t *__restrict__ nchunks, SumAcc *acc) {
    if (blockIdx.x >= *nchunks) return;
    const Chunk ch = chunks[blockIdx.x];
    double sum = 0, sabs = 0;
    int emin = 1 << 20;
    for (uint32_t j = ch.begin + threadIdx.x; j < ch.end; j += SC_T) {
        const float x = __builtin_bit_cast(float, vals[j]);
        sum += (double)x;
        sabs += (double)__builtin_fabsf(x);
        if (x != 0.0f) emin = min(emin, ulp_exp(x));
    }
    __shared__ double rs[SC_T / 64], ra[SC_T / 64];
    __shared__ int re[SC_T / 64];
    for (int o = 32; o > 0; o >>= 1) {
        sum += __shfl_xor(sum, o, 64);
        sabs += __shfl_xor(sabs, o, 64);
        emin = min(emin, __shfl_xor(emin, o, 64));
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) {
        rs[w] = sum;
        ra[w] = sabs;
        re[w] = emin;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    sum = rs[0];
    sabs = ra[0];
    emin = re[0];
    for (int i = 1; i < SC_T / 64; ++i) {
        sum += rs[i];
        sabs += ra[i];
        emin = min(emin, re[i]);
    }
    atomicAdd(&acc[ch.cl].sum, sum);
    atomicAdd(&acc[ch.cl].sabs, sabs);
    atomicMin(&acc[ch.cl].emin, emin);
}

__global__ __launch_bounds__(256) void k_sum1d_final(const SumAcc *__restrict__ acc, const uint32_t *__restrict__ start,
                                                     int k, float *__restrict__ cen, uint32_t *__restrict__ seq_flag,
                                                     int32_t *__restrict__ emin_c, double *__restrict__ sabs_c) {
    for (int cl = blockIdx.x * blockDim.x + threadIdx.x; cl < k; cl += gridDim.x * blockDim.x) {
        const uint32_t cnt = start[cl + 1] - start[cl];
        if (cnt == 0) {  // empty: re-seeded separately
            seq_flag[cl] = 0;
            continue;
        }
        const SumAcc a = acc[cl];
        const bool exact = sum_is_exact(a.sabs, a.emin);
        seq_flag[cl] = exact ? 0u : 1u;
        emin_c[cl] = a.emin;
        sabs_c[cl] = a.sabs;
        if (exact) cen[cl] = (float)(a.sum / (double)cnt);
    }
}

// ---- chunked replay of the flagged clusters (the algorithm of st_replay.h) -----------
__device__ inline __int128 shfl_up_i128(__int128 v, int o) {
    const uint64_t lo = __shfl_up((uint64_t)v, o, 64), hi = __shfl_up((uint64_t)(v >> 64), o, 64);
    return (__int128)(((unsigned __int128)hi << 64) | lo);
}
// exclusive scan of one int128 per thread over an SC_T block
__device__ inline __int128 sc_exscan_i128(__int128 v, __int128 *total) {
    __shared__ __int128 ws[SC_T / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __int128 incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const __int128 u = shfl_up_i128(incl, o);
        if (lane >= o) incl += u;
    }
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    __int128 off = 0, tot = 0;
    for (int i = 0; i < SC_T / 64; ++i) {
        if (i < w) off += ws[i];
        tot += ws[i];
    }
    __syncthreads();
    *total = tot;
    return off + incl - v;
}
__device__ inline uint32_t sc_exscan_u32(uint32_t v, uint32_t *total) {
    __shared__ uint32_t ws[SC_T / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
    }
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (int i = 0; i < SC_T / 64; ++i) {
        if (i < w) off += ws[i];
        tot += ws[i];
    }
    __syncthreads();
    *total = tot;
    return off + incl - v;
}
// |running start| + sum|x| bounds every prefix of a cluster's chain; base (nullable) holds
// each cluster's running start (the multi-GPU segment chain), zero in the one-device loop
__device__ inline double rp_bound(const double *__restrict__ sabs_c, const double *__restrict__ base, int cl) {
    return sabs_c[cl] + (base ? __builtin_fabs(base[cl]) : 0.0);
}
__device__ inline __int128 rp_base(const double *__restrict__ base, int cl, int e_lo) {
    return base ? f64_units(base[cl], e_lo) : (__int128)0;
}
__device__ inline __int128 rp_margin(double sabs, int e_lo) {
    int e_top;
    __builtin_frexp(sabs, &e_top);
    return ((__int128)1) << max(e_top - 33 - e_lo, 0);
}

// A: exact chunk sums in units of 2^e_lo
__global__ __launch_bounds__(SC_T) void k_rp_sums(const uint32_t *__restrict__ vals, const Chunk *__restrict__ chunks,
                                                 const uint32_t *__restrict__ nchunks,
                                                 const uint32_t *__restrict__ seq_flag,
                                                 const int32_t *__restrict__ emin_c, __int128 *__restrict__ csum) {
    const uint32_t nch = *nchunks;
    for (uint32_t bi = blockIdx.x; bi < nch; bi += gridDim.x) {
        const Chunk ch = chunks[bi];
        if (seq_flag[ch.cl] != 1u) continue;  // uniform per workgroup
        const int e_lo = emin_c[ch.cl];
        __int128 local = 0;
        for (uint32_t j = ch.begin + threadIdx.x; j < ch.end; j += SC_T) local += f32_units(vals[j], e_lo);
        __int128 tot;
        sc_exscan_i128(local, &tot);
        if (threadIdx.x == 0) csum[bi] = tot;
    }
}

// B / D: one workgroup per flagged cluster scans its chunks in order (exclusive prefixes)
__global__ __launch_bounds__(SC_T) void k_rp_prefix(const uint32_t *__restrict__ first, int k,
                                                   uint32_t *__restrict__ seq_flag, const double *__restrict__ sabs_c,
                                                   const int32_t *__restrict__ emin_c, __int128 *__restrict__ csum,
                                                   __int128 *__restrict__ total, const double *__restrict__ base) {
    const int cl = blockIdx.x;
    if (cl >= k || seq_flag[cl] != 1u) return;  // uniform per workgroup
    __syncthreads();  // every thread has read the flag before thread 0 may change it
    if (!(rp_bound(sabs_c, base, cl) * (1.0 + 1.0e-6) < __builtin_ldexp(1.0, emin_c[cl] + 118))) {  // int128 range
        if (threadIdx.x == 0) seq_flag[cl] = 2u;
        return;
    }
    __int128 run = 0;
    for (uint32_t c0 = first[cl]; c0 < first[cl + 1]; c0 += SC_T) {
        const uint32_t c = c0 + threadIdx.x;
        const __int128 v = c < first[cl + 1] ? csum[c] : (__int128)0;
        __int128 tot;
        const __int128 ex = sc_exscan_i128(v, &tot);
        if (c < first[cl + 1]) csum[c] = run + ex;  // in place: exclusive prefix of the chunk
        run += tot;
    }
    if (threadIdx.x == 0) total[cl] = run;
}
__global__ __launch_bounds__(SC_T) void k_rp_cprefix(const uint32_t *__restrict__ first, int k,
                                                    uint32_t *__restrict__ seq_flag, const uint32_t *__restrict__ ccnt,
                                                    uint32_t *__restrict__ cof, uint32_t *__restrict__ ctot,
                                                    uint32_t cap) {
    const int cl = blockIdx.x;
    if (cl >= k || seq_flag[cl] != 1u) return;  // uniform per workgroup
    uint32_t run = 0;
    for (uint32_t c0 = first[cl]; c0 < first[cl + 1]; c0 += SC_T) {
        const uint32_t c = c0 + threadIdx.x;
        const uint32_t v = c < first[cl + 1] ? ccnt[c] : 0u;
        uint32_t tot;
        const uint32_t ex = sc_exscan_u32(v, &tot);
        if (c < first[cl + 1]) cof[c] = run + ex;
        run += tot;
    }
    if (threadIdx.x == 0) {
        ctot[cl] = run;
        if (run > cap) seq_flag[cl] = 2u;  // the sequential chain
    }
}

// C (WRITE = false): candidates per chunk; E (WRITE = true): write them in member order
template <bool WRITE>
__global__ __launch_bounds__(SC_T) void k_rp_cands(const uint32_t *__restrict__ vals, const Chunk *__restrict__ chunks,
                                                  const uint32_t *__restrict__ nchunks,
                                                  const uint32_t *__restrict__ seq_flag,
                                                  const int32_t *__restrict__ emin_c,
                                                  const double *__restrict__ sabs_c,
                                                  const __int128 *__restrict__ coff, uint32_t *__restrict__ ccnt,
                                                  __int128 *__restrict__ cand_all, const double *__restrict__ base) {
    const uint32_t nch = *nchunks;
    for (uint32_t bi = blockIdx.x; bi < nch; bi += gridDim.x) {
        const Chunk ch = chunks[bi];
        if (seq_flag[ch.cl] != 1u) continue;  // uniform per workgroup
        const int e_lo = emin_c[ch.cl];
        const __int128 margin = rp_margin(rp_bound(sabs_c, base, ch.cl), e_lo);
        // this thread's contiguous slice of the chunk
        const uint32_t per = (ch.end - ch.begin + SC_T - 1) / SC_T;
        const uint32_t a = min(ch.end, ch.begin + threadIdx.x * per), b = min(ch.end, a + per);
        __int128 local = 0;
        for (uint32_t j = a; j < b; ++j) local += f32_units(vals[j], e_lo);
        __int128 tot;
        const __int128 off = rp_base(base, ch.cl, e_lo) + coff[bi] + sc_exscan_i128(local, &tot);
        uint32_t mine = 0;
        __int128 P = off;
        for (uint32_t j = a; j < b; ++j) {
            const uint32_t xb = vals[j];
            const __int128 Pn = P + f32_units(xb, e_lo);
            mine += replay_candidate(P, Pn, xb, e_lo, margin) ? 1u : 0u;
            P = Pn;
        }
        uint32_t ctot;
        const uint32_t cof = sc_exscan_u32(mine, &ctot);
        if (!WRITE) {
            if (threadIdx.x == 0) ccnt[bi] = ctot;
            continue;
        }
        uint32_t o = ccnt[bi] + cof;
        __int128 *cand = cand_all + (uint64_t)ch.cl * CAND_MAX;
        P = off;
        for (uint32_t j = a; j < b; ++j) {
            const uint32_t xb = vals[j];
            const __int128 Pn = P + f32_units(xb, e_lo);
            if (replay_candidate(P, Pn, xb, e_lo, margin)) cand[o++] = Pn;
            P = Pn;
        }
    }
}

// F: one lane per flagged cluster replays its candidates; the centroid (cen) or, with a
// running start (base), the f64 sum itself (sum_out)
__global__ __launch_bounds__(64) void k_rp_finish(const uint32_t *__restrict__ start, const uint32_t *__restrict__ ctot_c,
                                                  int k, uint32_t *__restrict__ seq_flag,
                                                  const int32_t *__restrict__ emin_c, const double *__restrict__ sabs_c,
                                                  const __int128 *__restrict__ total, const __int128 *__restrict__ cand_all,
                                                  float *__restrict__ cen, const double *__restrict__ base,
                                                  double *__restrict__ sum_out, const uint32_t *__restrict__ seq_vals) {
    // one workgroup per cluster: the wave stages the candidates in LDS 256 at a time, lane 0
    // replays them (the chain is sequential; its loads need not be).  seq_vals (non-null): the
    // clusters left to the sequential chain (flag 2) take it here too
    const int cl = blockIdx.x;
    if (cl >= k) return;
    const uint32_t flag0 = seq_flag[cl];
    if (flag0 == 2u && seq_vals) {
        if (threadIdx.x == 0) {
            const uint32_t s0 = start[cl], s1 = start[cl + 1];
            cen[cl] = (float)(seq_sum1d(seq_vals, s0, s1) / (double)(s1 - s0));
        }
        return;
    }
    if (flag0 != 1u) return;  // uniform per workgroup
    __shared__ __int128 buf[256];
    const int e_lo = emin_c[cl];
    const __int128 margin = rp_margin(rp_bound(sabs_c, base, cl), e_lo);
    const uint32_t ctot = ctot_c[cl];
    const __int128 *cand = cand_all + (uint64_t)cl * CAND_MAX;
    const __int128 b0 = rp_base(base, cl, e_lo);
    __int128 sv = b0, Pprev = b0;
    bool ok = true;
    for (uint32_t b = 0; b < ctot; b += 256) {
        const uint32_t m = min(256u, ctot - b);
        for (uint32_t i = threadIdx.x; i < m; i += 64) buf[i] = cand[b + i];
        __syncthreads();
        if (threadIdx.x == 0) {
            for (uint32_t i = 0; i < m; ++i) {
                const __int128 Pc = buf[i];
                const __int128 V = sv + (Pc - Pprev);
                sv = f64_representable(V) ? V : f64_units(f64_round(V, e_lo), e_lo);
                Pprev = Pc;
                const __int128 dev = sv - Pc;
                ok = ok && (dev < 0 ? -dev : dev) < margin;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    const __int128 fin = sv + (b0 + total[cl] - Pprev);
    if (!ok || !f64_representable(fin)) {
        seq_flag[cl] = 2u;
        if (seq_vals) {
            const uint32_t s0 = start[cl], s1 = start[cl + 1];
            cen[cl] = (float)(seq_sum1d(seq_vals, s0, s1) / (double)(s1 - s0));
        }
        return;
    }
    if (sum_out)
        sum_out[cl] = f64_round(fin, e_lo);
    else
        cen[cl] = (float)(f64_round(fin, e_lo) / (double)(start[cl + 1] - start[cl]));
    seq_flag[cl] = 0u;
}

// candidates one replay takes (CAND_MAX); ST_REPLAY_CAP lowers it so that tests can drive
// the sequential chain with small inputs
// (read per call: a test sets it around one call)
uint32_t replay_cap() {
    const char *e = getenv("ST_REPLAY_CAP");
    return e ? std::min<uint32_t>((uint32_t)strtoul(e, nullptr, 10), (uint32_t)CAND_MAX) : (uint32_t)CAND_MAX;
}

// stages A-F of the chunked replay for the clusters flagged 1 (left 0 when replayed, 2 when
// the sequential chain must take them)
void chunked_replay(st_ctx *c, const uint32_t *vals, const uint32_t *start, int k, uint64_t maxch, const Chunk *chunks,
                    const uint32_t *ch_first, uint32_t *seq_flag, const int32_t *emin_c, const double *sabs_c,
                    __int128 *csum, __int128 *total, uint32_t *ccnt, uint32_t *cof, uint32_t *ctot, __int128 *cands,
                    float *cen, const double *base, double *sum_out, bool seq_inline = false) {
    const unsigned gch = (unsigned)std::min<uint64_t>(maxch, 2048);  // grid-stride over the chunks
    hipLaunchKernelGGL(k_rp_sums, dim3(gch), dim3(SC_T), 0, c->stream, vals, chunks, ch_first + k, seq_flag, emin_c,
                       csum);
    hipLaunchKernelGGL(k_rp_prefix, dim3(k), dim3(SC_T), 0, c->stream, ch_first, k, seq_flag, sabs_c, emin_c, csum,
                       total, base);
    hipLaunchKernelGGL(k_rp_cands<false>, dim3(gch), dim3(SC_T), 0, c->stream, vals, chunks, ch_first + k, seq_flag,
                       emin_c, sabs_c, csum, ccnt, cands, base);
    hipLaunchKernelGGL(k_rp_cprefix, dim3(k), dim3(SC_T), 0, c->stream, ch_first, k, seq_flag, ccnt, cof, ctot,
                       replay_cap());
    hipLaunchKernelGGL(k_rp_cands<true>, dim3(gch), dim3(SC_T), 0, c->stream, vals, chunks, ch_first + k, seq_flag,
                       emin_c, sabs_c, csum, cof, cands, base);
    hipLaunchKernelGGL(k_rp_finish, dim3(k), dim3(64), 0, c->stream, start, ctot, k, seq_flag, emin_c, sabs_c, total,
                       cands, cen, base, sum_out, seq_inline ? vals : (const uint32_t *)nullptr);
    ST_LAUNCH_CHECK();
}

// counts, their exclusive scan, the chunk list and (acc != null) the accumulators in one
// workgroup for k <= CL_MAX (the 1-D codebooks): one launch instead of four
constexpr int CL_T = 1024, CL_MAX = 4096;
__global__ __launch_bounds__(CL_T) void k_chunk_list_small(const uint32_t *__restrict__ start, int k,
                                                           uint32_t *__restrict__ first, Chunk *__restrict__ chunks,
                                                           SumAcc *acc, uint32_t chsz) {
    constexpr int PER = CL_MAX / CL_T;
    __shared__ uint32_t wsum[CL_T / 64];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t cnt[PER], mine = 0;
#pragma unroll
    for (int u = 0; u < PER; ++u) {  // thread t owns clusters t*PER .. t*PER+PER-1
        const int cl = t * PER + u;
        cnt[u] = cl < k ? (start[cl + 1] - start[cl] + chsz - 1) / chsz : 0u;
        mine += cnt[u];
        if (acc && cl < k) acc[cl] = SumAcc{0.0, 0.0, 1 << 20, 0};
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
    for (int i = 0; i < CL_T / 64; ++i) {
        if (i < w) off += wsum[i];
        total += wsum[i];
    }
    uint32_t o = off + incl - mine;
    // chunk offsets and member starts in LDS; then every thread writes chunks (a cluster of
    // 100k+ members no longer leaves one thread writing all of its chunks)
    __shared__ uint32_t soff[CL_MAX + 1], sst[CL_MAX + 1];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int cl = t * PER + u;
        if (cl < k) {
            first[cl] = o;
            soff[cl] = o;
            sst[cl] = start[cl];
            o += cnt[u];
        }
    }
    if (t == 0) {
        first[k] = total;
        soff[k] = total;
        sst[k] = start[k];
    }
    __syncthreads();
    for (uint32_t q = t; q < total; q += CL_T) {
        uint32_t lo = 0, hi = (uint32_t)k;  // the cluster whose chunk range holds q
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (soff[mid] <= q) lo = mid;
            else hi = mid;
        }
        const uint32_t b = sst[lo] + (q - soff[lo]) * chsz;
        chunks[q] = Chunk{lo, b, min(sst[lo + 1], b + chsz), 0u};
    }
}

// the chunk list of every cluster's member range (k clusters, start[k + 1]); acc (nullable):
// the per-cluster accumulators to reset
void chunk_list(st_ctx *c, const uint32_t *start, int k, uint32_t *ch_cnt, uint32_t *ch_first, Chunk *chunks,
                SumAcc *acc = nullptr, uint32_t chsz = SC_CH) {
    if (k <= CL_MAX) {
        hipLaunchKernelGGL(k_chunk_list_small, dim3(1), dim3(CL_T), 0, c->stream, start, k, ch_first, chunks, acc,
                           chsz);
        ST_LAUNCH_CHECK();
        return;
    }
    const unsigned gk = grid_for((uint64_t)k, 256, 1024);
    hipLaunchKernelGGL(k_chunk_counts, dim3(gk), dim3(256), 0, c->stream, start, k, ch_cnt);
    scan_u32(c, ch_cnt, ch_first, (uint64_t)k, ch_first + k);
    hipLaunchKernelGGL(k_chunk_list, dim3(gk), dim3(256), 0, c->stream, start, k, ch_first, chunks);
    if (acc) hipLaunchKernelGGL(k_sumacc_init, dim3(gk), dim3(256), 0, c->stream, acc, k);
    ST_LAUNCH_CHECK();
}

// ---- the multi-GPU update's 1-D pieces (st_dist.hip) --------------------------------
__global__ __launch_bounds__(256) void k_partials_out(const SumAcc *__restrict__ acc, const uint32_t *__restrict__ start,
                                                      int nk, double *__restrict__ sums, double *__restrict__ sabs,
                                                      int32_t *__restrict__ emin, uint32_t *__restrict__ counts) {
    for (int sc = blockIdx.x * blockDim.x + threadIdx.x; sc < nk; sc += gridDim.x * blockDim.x) {
        const SumAcc a = acc[sc];
        sums[sc] = a.sum;  // only used when certified (then exact in any order)
        sabs[sc] = a.sabs;
        emin[sc] = a.emin;
        counts[sc] = start[sc + 1] - start[sc];
    }
}

// pending pairs (clusters) -> per-cluster flag 1 and running start
__global__ __launch_bounds__(256) void k_pend_in(const uint32_t *__restrict__ pairs, uint32_t npairs,
                                                 const double *__restrict__ running, uint32_t *__restrict__ flag_cl,
                                                 double *__restrict__ base_cl) {
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < npairs; p += gridDim.x * blockDim.x) {
        flag_cl[pairs[p]] = 1u;
        base_cl[pairs[p]] = running[p];
    }
}
__global__ __launch_bounds__(256) void k_pend_out(const uint32_t *__restrict__ pairs, uint32_t npairs,
                                                  const uint32_t *__restrict__ flag_cl, const double *__restrict__ sum_cl,
                                                  double *__restrict__ running, uint32_t *__restrict__ pflag) {
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < npairs; p += gridDim.x * blockDim.x) {
        const uint32_t f = flag_cl[pairs[p]];
        if (f == 0u) running[p] = sum_cl[pairs[p]];
        pflag[p] = f == 2u ? 1u : 0u;
    }
}

// ---- sort-free iteration for k <= 256 (cluster1d's codebooks) --------------------------
// Under the certificate every partial sum of a cluster is exact, so the members' order only
// matters for the clusters that fail it.  The assign therefore accumulates each cluster's
// count, sum, sum|x| and smallest ulp exponent in LDS while it labels the points (one partial
// per workgroup), and one launch reduces the partials, certifies, scans the cluster starts
// and re-seeds the empty clusters.  Only when a cluster fails the certificate are its members
// laid out in point order -- from the byte labels, moving that cluster's values only -- for
// the chunked replay above.  Two launches and one 8-byte read-back per iteration instead of
// the member sort's ~20 launches.
struct Part1 {
    double sum, sabs;
    int32_t emin;
    uint32_t cnt;
};
// a cluster's member-magnitude bounds from the centroid order (k_kd1_assign_acc<true>): used
// by k_kd1_final instead of the accumulated sum|x| / e_min unless acc
struct Bnd1 {
    float maxabs, minabs;
    uint32_t acc;
};
constexpr uint32_t A1_G = 1024;  // most workgroups (partials) of the accumulating assign
constexpr int A1_CELLS = 4096;   // bracket cells of the accumulating assign
constexpr int FF_MAX = 8;         // flagged clusters the wave kernels take (more: the tile kernels)

// workgroups for ntiles tiles: at most A1_G, every workgroup the same number of tiles
uint32_t a1_grid(uint32_t ntiles) {
    const uint32_t per = (ntiles + A1_G - 1) / A1_G;
    return (ntiles + per - 1) / per;
}

// k_kd1_assign_hist's bracket assign with the centroid order built in the workgroup (the
// stable sort of KdTree's build is a rank by (sort key, index)), over the tiles
// blockIdx.x, blockIdx.x + gridDim.x, ...; part[blockIdx.x * 256 + c] = cluster c's partial
template <bool BOUNDS>
__global__ __launch_bounds__(F1_T) void k_kd1_assign_acc(const float *__restrict__ pts, uint64_t n,
                                                        const float *__restrict__ cen, int k,
                                                        uint32_t *__restrict__ labels, uint8_t *__restrict__ lab8,
                                                        uint32_t ntiles, Part1 *__restrict__ part,
                                                        const uint32_t *__restrict__ mm, Bnd1 *__restrict__ bnd) {
    __shared__ float sv[256];
    __shared__ uint32_t si[256], skey[256];
    __shared__ uint16_t cc[256];
    __shared__ uint8_t chk_l[256], chk_r[256];
    __shared__ uint32_t first[A1_CELLS + 1];
    __shared__ double hs[256], ha[256];
    __shared__ uint8_t acc_abs[256];  // cluster: accumulate sum|x| and e_min (no bounds known)
    __shared__ int32_t he[256];
    __shared__ uint32_t hc[256];
    const int t = threadIdx.x;
    const float mine = t < k ? cen[t] : 0.f;
    const uint32_t key = t < k ? sortkey_(mine) : 0u;
    skey[t] = key;
    hs[t] = 0.0;
    ha[t] = 0.0;
    he[t] = 1 << 20;
    hc[t] = 0u;
    __syncthreads();
    if (t < k) {
        uint32_t r = 0;
        for (int j = 0; j < k; ++j) {
            const uint32_t kj = skey[j];
            r += (kj < key || (kj == key && j < t)) ? 1u : 0u;
        }
        sv[r] = mine;
        si[r] = (uint32_t)t;
    }
    __syncthreads();
    const float lo = sv[0], hi = sv[k - 1];
    const float span = hi - lo;
    const float inv = (span > 0.f && span < __builtin_inff()) ? (float)A1_CELLS / span : 0.f;
    auto cell = [&](float x) -> int {
        const float u = (x - lo) * inv;
        return (int)__builtin_fminf(__builtin_fmaxf(u, 0.f), (float)(A1_CELLS - 1));
    };
    if (t < k) {
        cc[t] = (uint16_t)cell(sv[t]);
        // can the outer neighbour of bracket end t share the minimum's rounded distance?  With
        // L = t, a = p - sv[t] < the gap to sv[t + 1], and RN((a + gl)^2) = RN(a^2) needs
        // a > 2^52 gl: only for equal values, a missing right neighbour or a gap ratio past
        // 2^48 (likewise for R = t).  Elsewhere the outer distance is strictly larger.
        const double gl = t >= 1 ? (double)sv[t] - (double)sv[t - 1] : -1.0;
        const double gr = t + 1 < k ? (double)sv[t + 1] - (double)sv[t] : -1.0;
        constexpr double R48 = 281474976710656.0;  // 2^48
        chk_l[t] = (t >= 1 && (gl == 0.0 || gr < 0.0 || gr >= gl * R48)) ? 1 : 0;
        chk_r[t] = (t + 1 < k && (gr == 0.0 || gl < 0.0 || gl >= gr * R48)) ? 1 : 0;
        // BOUNDS: the members of the cluster at sorted position t lie in [sv[t - 1], sv[t + 1]]
        // when both gaps are positive and no point lies 2^48 gaps beyond a neighbour (a point
        // outside is strictly nearer, in rounded f64, to that neighbour); if that interval
        // excludes 0, count x max|end| bounds sum|x| and the inner end's ulp bounds e_min, so
        // the certificate needs no per-point sum|x| / e_min
        bool bounded = false;
        float mx = 0.f, mn = 0.f;
        if (BOUNDS && mm && t >= 1 && t + 1 < k && gl > 0.0 && gr > 0.0) {
            const double xmin = (double)fkey_inv_(mm[0]), xmax = (double)fkey_inv_(mm[1]);
            const float l = sv[t - 1], h = sv[t + 1];
            bounded = ((double)l - xmin) <= gl * R48 && (xmax - (double)h) <= gr * R48 && (l > 0.f || h < 0.f);
            mx = __builtin_fmaxf(__builtin_fabsf(l), __builtin_fabsf(h));
            mn = __builtin_fminf(__builtin_fabsf(l), __builtin_fabsf(h));
        }
        acc_abs[si[t]] = bounded ? 0 : 1;
        if (BOUNDS && blockIdx.x == 0) bnd[si[t]] = Bnd1{mx, mn, bounded ? 0u : 1u};
    }
    __syncthreads();
    for (int g = t; g <= A1_CELLS; g += F1_T) {
        int a = 0, b = k;
        while (a < b) {
            const int m = (a + b) >> 1;
            if ((int)cc[m] < g) a = m + 1;
            else b = m;
        }
        first[g] = (uint32_t)a;
    }
    __syncthreads();
    auto dist = [&](int pos, double p) {
        const double v = (double)sv[pos] - p;
        return 0.0 + v * v;
    };
    auto val = [&](uint32_t pos) -> float { return sv[pos]; };
    auto idx = [&](uint32_t pos) -> uint32_t { return si[pos]; };
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t base = (uint64_t)tile * F1_TILE;
        float pv[F1_ROWS];
#pragma unroll
        for (int r = 0; r < F1_ROWS; ++r) {
            const uint64_t i = base + (uint64_t)r * F1_T + t;
            pv[r] = i < n ? pts[i] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < F1_ROWS; ++r) {
            const uint64_t i = base + (uint64_t)r * F1_T + t;
            if (i >= n) break;
            const float pf = pv[r];
            const double p = pf;
            const int g = cell(pf);
            int u = (int)first[g];
            const int ue = (int)first[g + 1];
            while (u < ue && sv[u] <= pf) ++u;
            const int L = u - 1, R = u;
            // f32 screen: a, b are p - sv[L], sv[R] - p up to 2^-24 relative; a clear winner with
            // unflagged outer neighbours has a strictly smaller rounded f64 distance than any
            // other centroid, so no f64 work (chk_l / chk_r: see above)
            int win = -1;
            if (L >= 0 && R < k && !chk_l[L] && !chk_r[R]) {
                const float a = pf - sv[L], b = sv[R] - pf;
                if (a < b * 0.99999f) win = L;
                else if (b < a * 0.99999f) win = R;
            }
            uint32_t lab;
            if (win >= 0) {
                lab = si[win];
            } else {
                const double dl = L >= 0 ? dist(L, p) : __builtin_inf();
                const double dr = R < k ? dist(R, p) : __builtin_inf();
                const double m = __builtin_fmin(dl, dr);
                const bool tie = dl == dr || (L >= 1 && chk_l[L] && dist(L - 1, p) == m) ||
                                 (R + 1 < k && chk_r[R] && dist(R + 1, p) == m);
                lab = !tie ? si[dl < dr ? L : R] : kd1_walk(p, k, val, idx);
            }
            if (lab8) lab8[i] = (uint8_t)lab;
            if (labels) labels[i] = lab;
            atomicAdd(&hc[lab], 1u);
            atomicAdd(&hs[lab], p);
            if (!BOUNDS || acc_abs[lab]) {
                atomicAdd(&ha[lab], __builtin_fabs(p));
                if (pf != 0.0f) atomicMin(&he[lab], ulp_exp(pf));
            }
        }
    }
    __syncthreads();
    part[(uint64_t)t * gridDim.x + blockIdx.x] = Part1{hs[t], ha[t], he[t], hc[t]};  // cluster-major
}

// one workgroup per cluster reduces its G partials: the count, and the centroid when the
// certificate holds (seq_flag 0) or flag 1 for the replay.  The last workgroup to finish then
// scans the cluster starts (start: every member, fstart: the flagged clusters' members only,
// the replay's compact layout), re-seeds the empty clusters as k_reseed_small does, and
// leaves {flagged clusters, their members} in info.
__global__ __launch_bounds__(256) void k_kd1_final(const Part1 *__restrict__ part, uint32_t G, int k, uint64_t n,
                                                   float *cen, uint32_t *seq_flag, int32_t *__restrict__ emin_c,
                                                   double *__restrict__ sabs_c, uint32_t *cnt_c,
                                                   uint32_t *__restrict__ start, uint32_t *__restrict__ fstart,
                                                   uint32_t *ticket, uint32_t *__restrict__ info,
                                                   const float *const *cols, const double *__restrict__ draws,
                                                   uint64_t ndraws, State *st, uint32_t many_above,
                                                   const Bnd1 *__restrict__ bnd, uint32_t *__restrict__ ffz) {
    const int cl = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    double s = 0, a = 0;
    int e = 1 << 20;
    uint32_t c = 0;
    for (uint32_t g = t; g < G; g += 256) {
        const Part1 p = part[(uint64_t)cl * G + g];
        s += p.sum;
        a += p.sabs;
        e = min(e, p.emin);
        c += p.cnt;
    }
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o, 64);
        a += __shfl_xor(a, o, 64);
        e = min(e, __shfl_xor(e, o, 64));
        c += __shfl_xor(c, o, 64);
    }
    __shared__ double rs[4], ra[4];
    __shared__ int re[4];
    __shared__ uint32_t rc[4];
    __shared__ bool last;
    if (lane == 0) {
        rs[w] = s;
        ra[w] = a;
        re[w] = e;
        rc[w] = c;
    }
    __syncthreads();
    if (t == 0) {
        s = (rs[0] + rs[1]) + (rs[2] + rs[3]);  // exact whenever it is used (the certificate)
        a = (ra[0] + ra[1]) + (ra[2] + ra[3]);
        e = min(min(re[0], re[1]), min(re[2], re[3]));
        c = (rc[0] + rc[1]) + (rc[2] + rc[3]);
        uint32_t f = 0;
        if (c && bnd && !bnd[cl].acc) {  // bounds in place of the accumulated sum|x| / e_min
            a = (double)c * (double)bnd[cl].maxabs * (1.0 + 0x1p-50);
            e = ulp_exp(bnd[cl].minabs);
        }
        if (c) {
            const bool exact = sum_is_exact(a, e);
            f = exact ? 0u : 1u;
            emin_c[cl] = e;
            sabs_c[cl] = a;
            if (exact) cen[cl] = (float)(s / (double)c);
        }
        __hip_atomic_store(&cnt_c[cl], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&seq_flag[cl], f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __threadfence();
        last = atomicAdd(ticket, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    const uint32_t cnt = t < k ? __hip_atomic_load(&cnt_c[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    const uint32_t fl = t < k ? __hip_atomic_load(&seq_flag[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    uint32_t tot, ftot, nempty, nflag;
    const uint32_t off = sc_exscan_u32(cnt, &tot);
    const uint32_t foff = sc_exscan_u32(fl ? cnt : 0u, &ftot);
    const bool empty = t < k && cnt == 0;
    const uint32_t rank = sc_exscan_u32(empty ? 1u : 0u, &nempty);
    sc_exscan_u32(fl, &nflag);
    if (t < k) {
        start[t] = off;
        fstart[t] = foff;
    }
    const uint64_t cursor = st->cursor;
    if (empty) {  // k-means.ts:174-178, as k_reseed_small
        const uint64_t di = cursor + rank;
        if (di >= ndraws) {
            atomicOr(&st->err, ERR_DRAWS);
        } else {
            const double dr = draws[di];
            if (!(dr >= 0.0 && dr < 1.0))
                atomicOr(&st->err, ERR_DRAW_RANGE);
            else
                cen[t] = cols[0][(uint64_t)__builtin_floor(dr * (double)n)];
        }
    }
    __syncthreads();  // every thread has read st->cursor
    if (t == 0) {
        start[k] = (uint32_t)n;
        fstart[k] = ftot;
        st->cursor = cursor + nempty;
        info[0] = nflag;
        info[1] = ftot;
        if (nflag > many_above) atomicOr(&st->err, ERR_K1_MANY);
        if (tot != (uint32_t)n) atomicOr(&st->err, ERR_INTERNAL);
        *ticket = 0u;
        if (ffz)  // k_ff_place's candidate-pool cursors
            for (int i = 0; i < FF_MAX; ++i) ffz[i] = 0u;
    }
}

// the multi-GPU update's partials: segment s's G workgroup partials -> (s, cluster) entries
// of partials1d's layout (sums / sabs / emin / counts[s * k + c])
__global__ __launch_bounds__(256) void k_part_fold(const Part1 *__restrict__ part, uint32_t G, int k,
                                                   double *__restrict__ sums, double *__restrict__ sabs,
                                                   int32_t *__restrict__ emin, uint32_t *__restrict__ counts) {
    const uint32_t sc = blockIdx.x, seg = sc / (uint32_t)k, cl = sc % (uint32_t)k;
    const Part1 *p = part + (uint64_t)seg * G * 256;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    double s = 0, a = 0;
    int e = 1 << 20;
    uint32_t c = 0;
    for (uint32_t g = t; g < G; g += 256) {
        const Part1 q = p[(uint64_t)cl * G + g];
        s += q.sum;
        a += q.sabs;
        e = min(e, q.emin);
        c += q.cnt;
    }
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o, 64);
        a += __shfl_xor(a, o, 64);
        e = min(e, __shfl_xor(e, o, 64));
        c += __shfl_xor(c, o, 64);
    }
    __shared__ double rs[4], ra[4];
    __shared__ int re[4];
    __shared__ uint32_t rc[4];
    if (lane == 0) {
        rs[w] = s;
        ra[w] = a;
        re[w] = e;
        rc[w] = c;
    }
    __syncthreads();
    if (t != 0) return;
    sums[sc] = (rs[0] + rs[1]) + (rs[2] + rs[3]);  // only used under the certificate
    sabs[sc] = (ra[0] + ra[1]) + (ra[2] + ra[3]);
    emin[sc] = min(min(re[0], re[1]), min(re[2], re[3]));
    counts[sc] = (rc[0] + rc[1]) + (rc[2] + rc[3]);
}

// ---- the flagged clusters' members when there are few of them (the usual case: the one or
// two clusters whose range holds values near zero).  A wave takes 1,024 consecutive points
// (16 byte labels per lane, one 16-byte load); per flagged cluster it counts (k_ff_count) or
// places (k_ff_scatter) that cluster's members with a wave prefix sum: no tile histogram.
constexpr uint32_t FF_CH = 1024;  // points per wave chunk

// the flagged clusters in ascending order into list (LDS), their count into *nl
__device__ inline void ff_list(const uint32_t *__restrict__ seq_flag, int k, uint32_t *list, uint32_t *nl) {
    __shared__ uint32_t wcnt[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const bool f = t < k && seq_flag[t] == 1u;
    const uint64_t b = __ballot(f);
    if (lane == 0) wcnt[w] = (uint32_t)__popcll(b);
    __syncthreads();
    uint32_t o = 0;
    for (int i = 0; i < w; ++i) o += wcnt[i];
    o += (uint32_t)__popcll(b & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
    if (f && o < (uint32_t)FF_MAX) list[o] = (uint32_t)t;
    if (t == 0) *nl = min(wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3], (uint32_t)FF_MAX);
    __syncthreads();
}

// the lane's 16 byte labels of chunk ch (bytes past n read as `none`)
__device__ inline uint4 ff_labels(const uint8_t *__restrict__ lab8, uint64_t n, uint32_t ch, int lane) {
    const uint64_t p = (uint64_t)ch * FF_CH + (uint64_t)lane * 16;
    if (p + 16 <= n) return *reinterpret_cast<const uint4 *>(lab8 + p);
    uint32_t w[4] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
    for (int i = 0; i < 16; ++i)
        if (p + i < n) w[i >> 2] = (w[i >> 2] & ~(0xffu << (8 * (i & 3)))) | ((uint32_t)lab8[p + i] << (8 * (i & 3)));
    return make_uint4(w[0], w[1], w[2], w[3]);
}
// 0x80 in each byte of x equal to v (callers mask the bytes past n: ff_valid_mask)
__device__ inline uint32_t ff_match(uint32_t x, uint32_t v) {
    const uint32_t y = x ^ (v * 0x01010101u);
    return ~(((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y | 0x7f7f7f7fu);  // exact zero-byte test
}
__device__ inline uint32_t ff_valid_mask(uint64_t n, uint32_t ch, int lane, int word) {
    const uint64_t p = (uint64_t)ch * FF_CH + (uint64_t)lane * 16 + 4 * word;
    if (p + 4 <= n) return 0x80808080u;
    uint32_t m = 0;
    for (int i = 0; i < 4; ++i)
        if (p + i < n) m |= 0x80u << (8 * i);
    return m;
}

__global__ __launch_bounds__(256) void k_ff_count(const uint8_t *__restrict__ lab8, uint64_t n, uint32_t nch, int k,
                                                  const uint32_t *__restrict__ seq_flag, uint32_t *__restrict__ cnt) {
    __shared__ uint32_t list[FF_MAX], nl;
    ff_list(seq_flag, k, list, &nl);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t nf = nl;
    if (nf == 0) return;
    for (uint32_t ch = blockIdx.x * 4 + w; ch < nch; ch += gridDim.x * 4) {
        const uint4 L = ff_labels(lab8, n, ch, lane);
        const uint32_t v[4] = {L.x, L.y, L.z, L.w};
        for (uint32_t f = 0; f < nf; ++f) {
            uint32_t c = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) c += __popc(ff_match(v[q], list[f]) & ff_valid_mask(n, ch, lane, q));
            for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
            if (lane == 0) cnt[(uint64_t)f * nch + ch] = c;
        }
    }
}

// slot f's chunk counts -> the chunks' first positions in the compact layout (exclusive scan
// from fstart of its cluster); one 1,024-thread workgroup per flagged slot, each thread a
// contiguous run of the counts
constexpr int FS_T = 1024;
__global__ __launch_bounds__(FS_T) void k_ff_scan(uint32_t *__restrict__ cnt, uint32_t nch, int k,
                                                  const uint32_t *__restrict__ seq_flag,
                                                  const uint32_t *__restrict__ fstart) {
    __shared__ uint32_t list[FF_MAX], nl;
    __shared__ uint32_t wsum[FS_T / 64];
    {  // the flagged clusters in ascending order (ff_list over 1,024 threads)
        __shared__ uint32_t wcnt[4];
        const int t = threadIdx.x, lane = t & 63, w = t >> 6;
        const bool f = t < k && t < 256 && seq_flag[t] == 1u;
        const uint64_t b = __ballot(f);
        if (lane == 0 && w < 4) wcnt[w] = (uint32_t)__popcll(b);
        __syncthreads();
        uint32_t o = 0;
        for (int i = 0; i < w && i < 4; ++i) o += wcnt[i];
        o += (uint32_t)__popcll(b & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
        if (f && o < (uint32_t)FF_MAX) list[o] = (uint32_t)t;
        if (t == 0) nl = min(wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3], (uint32_t)FF_MAX);
        __syncthreads();
    }
    const uint32_t f = blockIdx.x;
    if (f >= nl) return;  // uniform
    // pieces of FS_T * FS_PER counts staged in LDS by coalesced loads; each thread scans
    // FS_PER consecutive ones, then one block scan
    constexpr int FS_PER = 16;
    __shared__ uint32_t piece[FS_T * (FS_PER + 1)];  // element e at e + e / FS_PER: no bank conflicts
    auto at = [](uint32_t e) { return e + e / FS_PER; };
    uint32_t *row = cnt + (uint64_t)f * nch;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t carry = fstart[list[f]];
    for (uint32_t b0 = 0; b0 < nch; b0 += FS_T * FS_PER) {
#pragma unroll
        for (int u = 0; u < FS_PER; ++u) {
            const uint32_t i = b0 + u * FS_T + threadIdx.x;
            piece[at(u * FS_T + threadIdx.x)] = i < nch ? row[i] : 0u;
        }
        __syncthreads();
        uint32_t mine = 0;
#pragma unroll
        for (int u = 0; u < FS_PER; ++u) mine += piece[at(threadIdx.x * FS_PER + u)];
        uint32_t incl = mine;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = __shfl_up(incl, o, 64);
            if (lane >= o) incl += v;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        uint32_t o = carry, tot = 0;
        for (int i = 0; i < FS_T / 64; ++i) {
            if (i < w) o += wsum[i];
            tot += wsum[i];
        }
        o += incl - mine;
#pragma unroll
        for (int u = 0; u < FS_PER; ++u) {
            const uint32_t v = piece[at(threadIdx.x * FS_PER + u)];
            piece[at(threadIdx.x * FS_PER + u)] = o;
            o += v;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < FS_PER; ++u) {
            const uint32_t i = b0 + u * FS_T + threadIdx.x;
            if (i < nch) row[i] = piece[at(u * FS_T + threadIdx.x)];
        }
        carry += tot;
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_ff_scatter(const uint8_t *__restrict__ lab8, const float *__restrict__ pts,
                                                    uint64_t n, uint32_t nch, int k,
                                                    const uint32_t *__restrict__ seq_flag,
                                                    const uint32_t *__restrict__ off, uint32_t *__restrict__ fvals) {
    __shared__ uint32_t list[FF_MAX], nl;
    ff_list(seq_flag, k, list, &nl);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t nf = nl;
    if (nf == 0) return;
    for (uint32_t ch = blockIdx.x * 4 + w; ch < nch; ch += gridDim.x * 4) {
        const uint4 L = ff_labels(lab8, n, ch, lane);
        const uint32_t v[4] = {L.x, L.y, L.z, L.w};
        const uint64_t p0 = (uint64_t)ch * FF_CH + (uint64_t)lane * 16;
        for (uint32_t f = 0; f < nf; ++f) {
            uint32_t m[4], c = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                m[q] = ff_match(v[q], list[f]) & ff_valid_mask(n, ch, lane, q);
                c += __popc(m[q]);
            }
            uint32_t incl = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t u = __shfl_up(incl, o, 64);
                if (lane >= o) incl += u;
            }
            uint32_t pos = off[(uint64_t)f * nch + ch] + incl - c;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t mm = m[q];
                while (mm) {
                    const int byte = __builtin_ctz(mm) >> 3;
                    fvals[pos++] = __builtin_bit_cast(uint32_t, pts[p0 + 4 * q + byte]);
                    mm &= mm - 1;
                }
            }
        }
    }
}

// ---- the flagged clusters' update in three passes (the queued path) -------------------
// What count / scan / scatter, the chunk list and the replay's five passes do above, in three
// launches and a finish.  k_ff_batch: each wave takes a batch of FB_B chunks of FF_CH points
// (each lane 16 points of a chunk: one 16-byte label load, four 16-byte value loads), and per
// flagged cluster (slot f) writes the batch's members in point order into its own region of
// scr and the batch's count and exact sum (int128 units of 2^e_lo) into agg.  k_ff_bscan: one
// workgroup per slot scans the batches' (count, sum) into exclusive prefixes.  k_ff_place: one
// wave per (slot, batch) places the batch's members in vals (the sequential chain's input)
// from its prefix and lists the replay candidates P_j of st_replay.h into the slot's pool
// (ccnt / cpos: the batch's candidates and their pool position).  k_ff_finish gathers the
// candidates in batch order and replays them as k_rp_finish does.
constexpr int FB_B = 4;
constexpr uint32_t FB_PTS = FB_B * FF_CH;
struct FAgg {
    __int128 sum;   // exact, units of 2^e_lo (0 when the cluster is past the int128 range)
    uint32_t cnt;   // members
    uint32_t base;  // the slot's first member in the batch's scr region
    uint32_t pad[2];
};

__device__ inline __int128 wave_sum_i128(__int128 v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t lo = __shfl_xor((uint64_t)v, o, 64), hi = __shfl_xor((uint64_t)(v >> 64), o, 64);
        v += (__int128)(((unsigned __int128)hi << 64) | lo);
    }
    return v;
}
// the slot table the three passes share: fl[0] = slots, fl[1 + f] = cluster
__device__ inline bool ff_live(double sabs, int e_lo) {  // the int128 range of the replay
    return sabs * (1.0 + 1.0e-6) < __builtin_ldexp(1.0, e_lo + 118);
}

// v[e] for a run-time e in [0, 16) by a tree of selects (no scratch indexing)
__device__ inline float pick16(const float (&v)[16], int e) {
    float a[8], b[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = (e & 1) ? v[2 * i + 1] : v[2 * i];
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] = (e & 2) ? a[2 * i + 1] : a[2 * i];
    const float c0 = (e & 4) ? b[1] : b[0], c1 = (e & 4) ? b[3] : b[2];
    return (e & 8) ? c1 : c0;
}

__global__ __launch_bounds__(256) void k_ff_batch(const uint8_t *__restrict__ lab8, const float *__restrict__ pts,
                                                  uint64_t n, uint32_t nbt, int k,
                                                  const uint32_t *__restrict__ seq_flag,
                                                  const int32_t *__restrict__ emin_c,
                                                  const double *__restrict__ sabs_c, float *__restrict__ scr,
                                                  FAgg *__restrict__ agg, uint32_t *__restrict__ fl) {
    __shared__ uint32_t list[FF_MAX], nl;
    ff_list(seq_flag, k, list, &nl);
    __shared__ int32_t s_elo[FF_MAX];
    __shared__ uint32_t s_live[FF_MAX];
    const uint32_t nf = nl;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (blockIdx.x == 0 && t <= (int)nf) fl[t] = t == 0 ? nf : list[t - 1];
    if (nf == 0) return;  // uniform
    if (t < (int)nf) {
        const uint32_t cl = list[t];
        s_elo[t] = emin_c[cl];
        s_live[t] = ff_live(sabs_c[cl], emin_c[cl]) ? 1u : 0u;
    }
    __syncthreads();
    for (uint32_t b = blockIdx.x * 4 + (uint32_t)w; b < nbt; b += gridDim.x * 4) {
        // the lane's 16 labels of each chunk; per slot and chunk it loads its 16 values only
        // where it holds members of that slot (L2 serves a second slot's reload), then picks
        // each member's value with a select tree: no LDS staging, no register arrays indexed at
        // run time
        const uint64_t p0 = (uint64_t)b * FB_PTS + (uint64_t)lane * 16;
        uint4 L[FB_B];
#pragma unroll
        for (int j = 0; j < FB_B; ++j) L[j] = ff_labels(lab8, n, b * FB_B + j, lane);
        uint32_t base = 0;  // the slot's first member in the batch's region
        float *out = scr + (uint64_t)b * FB_PTS;
        for (uint32_t f = 0; f < nf; ++f) {
            const uint32_t cl = list[f];
            const int e_lo = s_elo[f];
            const bool live = s_live[f] != 0u;
            uint32_t o = base;
            __int128 s = 0;
#pragma unroll 1
            for (int j = 0; j < FB_B; ++j) {
                static_assert(FB_B == 4, "the label select below");
                const uint4 Lj = j == 0 ? L[0] : j == 1 ? L[1] : j == 2 ? L[2] : L[3];
                const uint32_t x[4] = {Lj.x, Lj.y, Lj.z, Lj.w};
                uint32_t msk = 0;  // bit e: point e of the lane's 16 is a member
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t m = ff_match(x[q], cl) & ff_valid_mask(n, b * FB_B + j, lane, q);
#pragma unroll
                    for (int e = 0; e < 4; ++e) msk |= ((m >> (8 * e + 7)) & 1u) << (4 * q + e);
                }
                const uint32_t c = __popc(msk);
                uint32_t ci = c;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t u = __shfl_up(ci, d, 64);
                    if (lane >= d) ci += u;
                }
                uint32_t at = o + ci - c;
                if (msk) {
                    const uint64_t pj = p0 + (uint64_t)j * FF_CH;
                    float v[16];
                    if (pj + 16 <= n) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const float4 u = *reinterpret_cast<const float4 *>(pts + pj + 4 * q);
                            v[4 * q] = u.x;
                            v[4 * q + 1] = u.y;
                            v[4 * q + 2] = u.z;
                            v[4 * q + 3] = u.w;
                        }
                    } else {
#pragma unroll
                        for (int e = 0; e < 16; ++e) v[e] = pj + e < n ? pts[pj + e] : 0.f;
                    }
                    for (uint32_t mm = msk; mm; mm &= mm - 1) {
                        const float x = pick16(v, __builtin_ctz(mm));
                        out[at++] = x;
                        if (live) s += f32_units(__builtin_bit_cast(uint32_t, x), e_lo);
                    }
                }
                o += __shfl(ci, 63, 64);
            }
            const __int128 S = live ? wave_sum_i128(s) : (__int128)0;
            if (lane == 0) agg[(uint64_t)f * nbt + b] = FAgg{S, o - base, base, {0u, 0u}};
            base = o;
        }
    }
}

// one 1,024-thread workgroup per slot: the batches' exclusive prefixes (in place: agg[.].sum and
// .cnt become the prefix before the batch; .base stays) and the slot's totals.  Each thread
// takes a contiguous run of batches (its sums in registers), so the workgroup scans once.
constexpr int FN_T = 1024;
// block-wide exclusive scan of (int128, u32) pairs over FN_T threads
__device__ inline void fn_exscan(__int128 v, uint32_t c, __int128 &ex, uint32_t &exc, __int128 &all,
                                 uint32_t &allc) {
    __shared__ __int128 ws[FN_T / 64];
    __shared__ uint32_t wc[FN_T / 64];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    __int128 incl = v;
    uint32_t ic = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const __int128 u = shfl_up_i128(incl, d);
        const uint32_t uc = __shfl_up(ic, d, 64);
        if (lane >= d) {
            incl += u;
            ic += uc;
        }
    }
    if (lane == 63) {
        ws[w] = incl;
        wc[w] = ic;
    }
    __syncthreads();
    __int128 off = 0, tot = 0;
    uint32_t offc = 0, totc = 0;
    for (int i = 0; i < FN_T / 64; ++i) {
        if (i < w) {
            off += ws[i];
            offc += wc[i];
        }
        tot += ws[i];
        totc += wc[i];
    }
    __syncthreads();
    ex = off + incl - v;
    exc = offc + ic - c;
    all = tot;
    allc = totc;
}

__global__ __launch_bounds__(FN_T) void k_ff_bscan(uint32_t nbt, const uint32_t *__restrict__ fl,
                                                   FAgg *__restrict__ agg, FAgg *__restrict__ tot) {
    const uint32_t f = blockIdx.x;
    if (f >= fl[0]) return;  // uniform
    const uint32_t t = threadIdx.x, per = (nbt + FN_T - 1) / FN_T;
    const uint32_t b0 = min(nbt, t * per), b1 = min(nbt, b0 + per);
    FAgg *a = agg + (uint64_t)f * nbt;
    __int128 ls = 0;
    uint32_t lc = 0;
    for (uint32_t b = b0; b < b1; ++b) {
        ls += a[b].sum;
        lc += a[b].cnt;
    }
    __int128 ex, all;
    uint32_t exc, allc;
    fn_exscan(ls, lc, ex, exc, all, allc);
    for (uint32_t b = b0; b < b1; ++b) {
        const FAgg v = a[b];
        a[b] = FAgg{ex, exc, v.base, {0u, 0u}};
        ex += v.sum;
        exc += v.cnt;
    }
    if (t == 0) tot[f] = FAgg{all, allc, 0u, {0u, 0u}};
}

// one wave per (slot, batch) with members: each lane a contiguous run of the batch's members;
// their exact running sums give the candidates
__global__ __launch_bounds__(256) void k_ff_place(uint32_t nbt, const uint32_t *__restrict__ fl,
                                                  const uint32_t *__restrict__ fstart,
                                                  const int32_t *__restrict__ emin_c,
                                                  const double *__restrict__ sabs_c, const float *__restrict__ scr,
                                                  const FAgg *__restrict__ agg, uint32_t *__restrict__ ffz,
                                                  uint32_t *__restrict__ vals, __int128 *__restrict__ pool,
                                                  uint32_t *__restrict__ ccnt, uint32_t *__restrict__ cpos,
                                                  const FAgg *__restrict__ tot) {
    const uint32_t nf = fl[0];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (uint64_t q = (uint64_t)blockIdx.x * 4 + w; q < (uint64_t)nf * nbt; q += (uint64_t)gridDim.x * 4) {
        const uint32_t f = (uint32_t)(q / nbt), b = (uint32_t)(q % nbt);
        const FAgg a = agg[q];
        const uint32_t C = (b + 1 < nbt ? agg[q + 1].cnt : tot[f].cnt) - a.cnt;  // the batch's members
        if (C == 0) {
            if (lane == 0) ccnt[q] = 0u;
            continue;
        }
        const uint32_t cl = fl[1 + f];
        const int e_lo = emin_c[cl];
        const double sabs = sabs_c[cl];
        const bool live = ff_live(sabs, e_lo);
        const __int128 margin = rp_margin(sabs, e_lo);
        const float *in = scr + (uint64_t)b * FB_PTS + a.base;
        const uint32_t per = (C + 63) / 64, i0 = min(C, (uint32_t)lane * per), i1 = min(C, i0 + per);
        uint32_t *dst = vals + fstart[cl] + a.cnt;
        __int128 s = 0;
        for (uint32_t i = i0; i < i1; ++i) {
            const uint32_t xb = __builtin_bit_cast(uint32_t, in[i]);
            dst[i] = xb;
            if (live) s += f32_units(xb, e_lo);
        }
        if (!live) {
            if (lane == 0) ccnt[q] = 0u;
            continue;
        }
        __int128 si = s;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const __int128 u = shfl_up_i128(si, d);
            if (lane >= d) si += u;
        }
        const __int128 P0 = a.sum + (si - s);
        uint32_t nc = 0;
        {
            __int128 P = P0;
            for (uint32_t i = i0; i < i1; ++i) {
                const uint32_t xb = __builtin_bit_cast(uint32_t, in[i]);
                const __int128 Pn = P + f32_units(xb, e_lo);
                nc += replay_candidate(P, Pn, xb, e_lo, margin) ? 1u : 0u;
                P = Pn;
            }
        }
        uint32_t nci = nc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t u = __shfl_up(nci, d, 64);
            if (lane >= d) nci += u;
        }
        const uint32_t CT = __shfl(nci, 63, 64);
        uint32_t pos = 0;
        if (lane == 0) {
            if (CT) pos = atomicAdd(&ffz[f], CT);
            ccnt[q] = CT;
            cpos[q] = pos;
        }
        pos = __shfl(pos, 0, 64);
        if (nc) {  // past CAND_MAX: dropped (k_ff_finish then takes the sequential chain)
            uint32_t o = pos + (nci - nc);
            __int128 *pl = pool + (uint64_t)f * CAND_MAX;
            __int128 P = P0;
            for (uint32_t i = i0; i < i1; ++i) {
                const uint32_t xb = __builtin_bit_cast(uint32_t, in[i]);
                const __int128 Pn = P + f32_units(xb, e_lo);
                if (replay_candidate(P, Pn, xb, e_lo, margin)) {
                    if (o < (uint32_t)CAND_MAX) pl[o] = Pn;
                    ++o;
                }
                P = Pn;
            }
        }
    }
}

// one 1,024-thread workgroup per slot: the batches' candidates in batch order into the
// cluster's cand_all row, then the replay of k_rp_finish (the sequential chain for a cluster
// past the int128 range, with more than cap candidates, or whose replay gives up)
__global__ __launch_bounds__(FN_T) void k_ff_finish(uint32_t nbt, const uint32_t *__restrict__ fl,
                                                    uint32_t *__restrict__ seq_flag,
                                                    const uint32_t *__restrict__ fstart,
                                                    const int32_t *__restrict__ emin_c,
                                                    const double *__restrict__ sabs_c, const FAgg *__restrict__ tot,
                                                    const uint32_t *__restrict__ vals,
                                                    const __int128 *__restrict__ pool,
                                                    const uint32_t *__restrict__ ccnt, const uint32_t *__restrict__ cpos,
                                                    __int128 *__restrict__ cand_all, uint32_t cap,
                                                    float *__restrict__ cen, State *st) {
    const uint32_t f = blockIdx.x;
    if (f >= fl[0]) return;  // uniform
    const uint32_t cl = fl[1 + f];
    const int t = threadIdx.x;
    const uint32_t s0 = fstart[cl], s1 = fstart[cl + 1];
    const int e_lo = emin_c[cl];
    const double sabs = sabs_c[cl];
    const FAgg tf = tot[f];
    if (t == 0 && tf.cnt != s1 - s0) atomicOr(&st->err, ERR_INTERNAL);
    bool seq = !ff_live(sabs, e_lo);  // uniform: fn_exscan's barriers below
    __shared__ __int128 buf[FN_T];
    uint32_t ctot = 0;
    __int128 *cand = cand_all + (uint64_t)cl * CAND_MAX;
    if (!seq) {
        // each thread a contiguous run of batches: their candidate counts scanned once, then
        // the run's candidates copied in batch order
        const __int128 *pl = pool + (uint64_t)f * CAND_MAX;
        const uint32_t per = (nbt + FN_T - 1) / FN_T;
        const uint32_t b0 = min(nbt, (uint32_t)t * per), b1 = min(nbt, b0 + per);
        const uint32_t *cc = ccnt + (uint64_t)f * nbt, *cp = cpos + (uint64_t)f * nbt;
        uint32_t lc = 0;
        for (uint32_t b = b0; b < b1; ++b) lc += cc[b];
        __int128 ex_unused, all_unused;
        uint32_t off, all;
        fn_exscan(0, lc, ex_unused, off, all_unused, all);
        for (uint32_t b = b0; b < b1 && lc; ++b) {
            const uint32_t c = cc[b];
            if (c) {
                const uint32_t ps = cp[b];
                for (uint32_t j = 0; j < c; ++j)
                    if (off + j < cap && ps + j < (uint32_t)CAND_MAX) cand[off + j] = pl[ps + j];
            }
            off += c;
        }
        ctot = all;
        seq = ctot > cap;
    }
    __syncthreads();  // the candidates written above, read below by other threads
    bool ok = !seq;
    __int128 sv = 0, Pprev = 0;
    const __int128 margin = rp_margin(sabs, e_lo);
    for (uint32_t b = 0; !seq && b < ctot; b += FN_T) {  // seq, ctot uniform; thread 0 keeps ok
        const uint32_t m = min((uint32_t)FN_T, ctot - b);
        if ((uint32_t)t < m) buf[t] = cand[b + t];
        __syncthreads();
        if (t == 0) {
            for (uint32_t i = 0; i < m; ++i) {
                const __int128 Pc = buf[i];
                const __int128 V = sv + (Pc - Pprev);
                sv = f64_representable(V) ? V : f64_units(f64_round(V, e_lo), e_lo);
                Pprev = Pc;
                const __int128 dev = sv - Pc;
                ok = ok && (dev < 0 ? -dev : dev) < margin;
            }
        }
        __syncthreads();
    }
    if (t != 0) return;
    const __int128 fin = sv + (tf.sum - Pprev);
    if (!ok || !f64_representable(fin)) {
        seq_flag[cl] = 2u;
        cen[cl] = (float)(seq_sum1d(vals, s0, s1) / (double)(s1 - s0));
        return;
    }
    cen[cl] = (float)(f64_round(fin, e_lo) / (double)(s1 - s0));
    seq_flag[cl] = 0u;
}

// per-tile member counts of the flagged clusters: tcnt[c * ntiles + tile] for flagged c
__global__ __launch_bounds__(F1_T) void k_flag_tiles(const uint8_t *__restrict__ lab8, uint64_t n, uint32_t ntiles,
                                                    int k, const uint32_t *__restrict__ seq_flag,
                                                    uint32_t *__restrict__ tcnt) {
    __shared__ uint32_t h[256];
    __shared__ uint8_t fl[256];
    const int t = threadIdx.x;
    fl[t] = (t < k && seq_flag[t] == 1u) ? 1 : 0;
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        h[t] = 0u;
        __syncthreads();
        const uint64_t base = (uint64_t)tile * F1_TILE;
#pragma unroll 4
        for (int r = 0; r < F1_ROWS; ++r) {
            const uint64_t i = base + (uint64_t)r * F1_T + t;
            if (i < n) {
                const uint32_t d = lab8[i];
                if (fl[d]) atomicAdd(&h[d], 1u);
            }
        }
        __syncthreads();
        if (fl[t]) tcnt[(uint64_t)t * ntiles + tile] = h[t];
        __syncthreads();
    }
}

// a flagged cluster's tile counts -> its members' first positions per tile in the compact
// layout (exclusive scan from fstart[c]); one workgroup per cluster
__global__ __launch_bounds__(SC_T) void k_flag_scan(uint32_t *__restrict__ tcnt, uint32_t ntiles,
                                                    const uint32_t *__restrict__ seq_flag,
                                                    const uint32_t *__restrict__ fstart) {
    const int cl = blockIdx.x;
    if (seq_flag[cl] != 1u) return;  // uniform per workgroup
    uint32_t *row = tcnt + (uint64_t)cl * ntiles;
    uint32_t carry = fstart[cl];
    constexpr int PER = 4;
    for (uint32_t b = 0; b < ntiles; b += SC_T * PER) {
        uint32_t v[PER], mine = 0;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const uint32_t i = b + threadIdx.x * PER + u;
            v[u] = i < ntiles ? row[i] : 0u;
            mine += v[u];
        }
        uint32_t tot;
        uint32_t o = carry + sc_exscan_u32(mine, &tot);
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const uint32_t i = b + threadIdx.x * PER + u;
            if (i < ntiles) row[i] = o;
            o += v[u];
        }
        carry += tot;
    }
}

// the flagged clusters' values in point order at their compact positions: each wave ranks
// its 1,024 points of the tile by ballots over the label bits (as k_lab_scatter), the waves
// of a tile take consecutive runs
__global__ __launch_bounds__(F1_T) void k_flag_scatter(const uint8_t *__restrict__ lab8, const float *__restrict__ pts,
                                                      uint64_t n, uint32_t ntiles, int k, int bits,
                                                      const uint32_t *__restrict__ seq_flag,
                                                      const uint32_t *__restrict__ toff, uint32_t *__restrict__ fvals) {
    __shared__ uint32_t wcount[F1_WAVES][256];
    __shared__ uint32_t wpos[F1_WAVES][256];
    __shared__ uint8_t fl[256];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    fl[t] = (t < k && seq_flag[t] == 1u) ? 1 : 0;
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        for (int i = t; i < F1_WAVES * 256; i += F1_T) (&wcount[0][0])[i] = 0u;
        __syncthreads();
        const uint64_t wb = (uint64_t)tile * F1_TILE + (uint64_t)w * 64 * F1_ROWS;
        uint32_t dg[F1_ROWS];
#pragma unroll
        for (int r = 0; r < F1_ROWS; ++r) {
            const uint64_t e = wb + (uint64_t)r * 64 + lane;
            dg[r] = e < n ? (uint32_t)lab8[e] : 0u;
            if (e < n && fl[dg[r]]) atomicAdd(&wcount[w][dg[r]], 1u);
        }
        __syncthreads();
        if (fl[t]) {
            uint32_t s = toff[(uint64_t)t * ntiles + tile];
#pragma unroll
            for (int i = 0; i < F1_WAVES; ++i) {
                wpos[i][t] = s;
                s += wcount[i][t];
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < F1_ROWS; ++r) {
            const uint64_t e = wb + (uint64_t)r * 64 + lane;
            const uint32_t d = dg[r];
            const bool valid = e < n && fl[d];
            uint64_t peers = __ballot(valid);
            if (peers == 0) continue;  // uniform
            for (int b = 0; b < bits; ++b) {
                const bool bit = (d >> b) & 1u;
                const uint64_t bb = __ballot(bit);
                peers &= bit ? bb : ~bb;
            }
            const uint32_t before = valid ? wpos[w][d] : 0u;
            if (valid) fvals[before + __popcll(peers & lt)] = __builtin_bit_cast(uint32_t, pts[e]);
            if (valid && (peers & lt) == 0) wpos[w][d] = before + (uint32_t)__popcll(peers);
            __builtin_amdgcn_wave_barrier();
        }
        __syncthreads();
    }
}

}  // namespace

// one exact 1-D assign: KdTree build == stable sort of the centroid values
// (kd-tree.ts:73-99), then the walk simulation
bool assign1d(st_ctx *c, const float *pts, uint64_t n, int k, const float *cen, uint32_t *labels, uint32_t *keys,
              uint32_t *vals, bool need_labels) {
    auto *ckeys = wsT<uint32_t>(c, "k1.ckeys", (size_t)k);
    auto *corder = wsT<uint32_t>(c, "k1.corder", (size_t)k);
    hipLaunchKernelGGL(k_sortkeys, dim3(grid_for(k, 256, 256)), dim3(256), 0, c->stream, cen, k, ckeys, corder);
    ST_LAUNCH_CHECK();
    radix_sort_u32(c, ckeys, corder, (uint64_t)k, 0, 32, "k1.csort");
    const unsigned g = grid_for(n, 256, 256 * 16);
    KTimer kt(c, "k1.assign");
    if (k <= KD1_LDS) {
        hipLaunchKernelGGL(k_kd1_assign_fast, dim3(g), dim3(256), 0, c->stream, pts, n, cen, corder, k,
                           (keys && !need_labels) ? (uint32_t *)nullptr : labels, keys, vals);
        ST_LAUNCH_CHECK();
        return keys != nullptr;
    }
    hipLaunchKernelGGL(k_kd1_assign<false>, dim3(g), dim3(256), 0, c->stream, pts, n, cen, corder, k, labels);
    ST_LAUNCH_CHECK();
    return false;
}

void kmeans1d_loop(st_ctx *c, const float *pts, const float *const *dcols, uint64_t n, int k, int iters,
                   const double *ddraws, uint64_t ndraws, State *dstate, float *cen, uint32_t *labels) {
    auto *keys = wsT<uint32_t>(c, "k1.keys", n);
    auto *vals = wsT<uint32_t>(c, "k1.vals", n);
    auto *start = wsT<uint32_t>(c, "k1.start", (size_t)k + 1);
    auto *seq_flag = wsT<uint32_t>(c, "k1.seqflag", (size_t)k);
    auto *emin_c = wsT<int32_t>(c, "k1.emin", (size_t)k);
    auto *sabs_c = wsT<double>(c, "k1.sabs", (size_t)k);
    auto *cand_buf = wsT<__int128>(c, "k1.cands", (size_t)k * CAND_MAX);
    const uint64_t maxch = n / SC_CH + (uint64_t)k + 1;
    const uint64_t chcap = n / FL_CH + (uint64_t)k + 1;  // the flagged replay's shorter chunks
    auto *ch_cnt = wsT<uint32_t>(c, "k1.chcnt", (size_t)k);
    auto *ch_first = wsT<uint32_t>(c, "k1.chfirst", (size_t)k + 1);
    auto *chunks = wsT<Chunk>(c, "k1.chunks", chcap);
    auto *acc = wsT<SumAcc>(c, "k1.acc", (size_t)k);
    auto *rp_csum = wsT<__int128>(c, "k1.rpcsum", chcap);
    auto *rp_ccnt = wsT<uint32_t>(c, "k1.rpccnt", chcap);
    auto *rp_cof = wsT<uint32_t>(c, "k1.rpcof", chcap);
    auto *rp_ctot = wsT<uint32_t>(c, "k1.rpctot", (size_t)k);
    auto *rp_total = wsT<__int128>(c, "k1.rptotal", (size_t)k);
    int kbits = 1;
    while ((1ull << kbits) < (uint64_t)k) ++kbits;
    // the fused iteration (k <= 256; ST_K1_PAIRS forces the general one, test hook): byte labels
    // + tile counts, scan, value-only scatter
    const bool fused = k <= 256 && n > 0 && n < (1ull << 32) && !getenv("ST_K1_PAIRS");
    const uint32_t ntiles = (uint32_t)((n + F1_TILE - 1) / F1_TILE);
    uint8_t *lab8 = fused ? wsT<uint8_t>(c, "k1.lab8", n) : nullptr;
    // the sort-free iteration (k_kd1_assign_acc; ST_K1_SORT=1 keeps the member sort)
    const bool accum = fused && !getenv("ST_K1_SORT");
    uint32_t *fhist = fused ? wsT<uint32_t>(c, "k1.fhist", (size_t)256 * ntiles) : nullptr;
    if (accum) {
        const uint32_t G = a1_grid(ntiles);
        auto *part = wsT<Part1>(c, "k1.part", (size_t)G * 256);
        auto *cnt_c = wsT<uint32_t>(c, "k1.cnt", (size_t)k);
        auto *fstart = wsT<uint32_t>(c, "k1.fstart", (size_t)k + 1);
        auto *ticket = wsT<uint32_t>(c, "k1.ticket", 1);
        auto *dinfo = wsT<uint32_t>(c, "k1.info", 2);
        auto *bnd = wsT<Bnd1>(c, "k1.bnd", 256);
        // the points' min / max keys (kmeans_dev's 1-D init)
        const uint32_t *mm = wsT<uint32_t>(c, "km.mm", 2);
        auto *hinfo = static_cast<uint32_t *>(pinned_slot(c, "k1.info", 8));
        ST_HIP(hipMemsetAsync(ticket, 0, sizeof(uint32_t), c->stream));
        // the three-pass flagged update (k_ff_batch / k_ff_bscan / k_ff_place + k_ff_finish)
        const uint32_t nbt = (uint32_t)((n + FB_PTS - 1) / FB_PTS);
        auto *ffz = wsT<uint32_t>(c, "k1.ffz", FF_MAX);
        auto *ffcnt = wsT<uint32_t>(c, "k1.ffcnt", (size_t)FF_MAX * nbt);
        auto *ffpos = wsT<uint32_t>(c, "k1.ffpos", (size_t)FF_MAX * nbt);
        auto *fflist = wsT<uint32_t>(c, "k1.fflist", FF_MAX + 1);
        auto *ffpool = wsT<__int128>(c, "k1.ffpool", (size_t)FF_MAX * CAND_MAX);
        auto *ffagg = wsT<FAgg>(c, "k1.ffagg", (size_t)FF_MAX * nbt);
        auto *fftot = wsT<FAgg>(c, "k1.fftot", FF_MAX);
        auto *ffscr = wsT<float>(c, "k1.ffscr", (size_t)nbt * FB_PTS);
        // queued: no read-back per iteration (more than FF_MAX flagged clusters -> ERR_K1_MANY,
        // and kmeans_dev reruns with k1_sync); otherwise the count decides the flagged path
        const bool queued = !c->k1_sync && !getenv("ST_K1_TILES") && !getenv("ST_K1_SYNC");
        // flagged clusters the wave kernels take (ST_K1_FF_MAX lowers it: tests of the rerun)
        const uint32_t ff_max = getenv("ST_K1_FF_MAX") ? std::min<uint32_t>((uint32_t)atoi(getenv("ST_K1_FF_MAX")),
                                                                            (uint32_t)FF_MAX)
                                                       : (uint32_t)FF_MAX;
        for (int it = 0; it < iters; ++it) {
            {
                KTimer kt(c, "k1.assign");
                hipLaunchKernelGGL(k_kd1_assign_acc<true>, dim3(G), dim3(F1_T), 0, c->stream, pts, n, cen, k,
                                   it == iters - 1 ? labels : (uint32_t *)nullptr, lab8, ntiles, part, mm, bnd);
                ST_LAUNCH_CHECK();
            }
            mark(c, "k1.assign");
            KTimer kt(c, "k1.sum");
            hipLaunchKernelGGL(k_kd1_final, dim3(k), dim3(256), 0, c->stream, part, G, k, n, cen, seq_flag, emin_c,
                               sabs_c, cnt_c, start, fstart, ticket, dinfo, dcols, ddraws, ndraws, dstate,
                               queued ? ff_max : 0xffffffffu, bnd, ffz);
            ST_LAUNCH_CHECK();
            if (queued) {
                // the flagged path queued behind the final with no read-back: its kernels find
                // the flagged clusters on the device and return at once when there are none
                const unsigned gb = (unsigned)std::min<uint64_t>((nbt + 3) / 4, 2048);
                hipLaunchKernelGGL(k_ff_batch, dim3(gb), dim3(256), 0, c->stream, lab8, pts, n, nbt, k, seq_flag,
                                   emin_c, sabs_c, ffscr, ffagg, fflist);
                hipLaunchKernelGGL(k_ff_bscan, dim3(FF_MAX), dim3(FN_T), 0, c->stream, nbt, fflist, ffagg, fftot);
                const unsigned gp = (unsigned)std::min<uint64_t>(((uint64_t)FF_MAX * nbt + 3) / 4, 4096);
                hipLaunchKernelGGL(k_ff_place, dim3(gp), dim3(256), 0, c->stream, nbt, fflist, fstart, emin_c,
                                   sabs_c, ffscr, ffagg, ffz, vals, ffpool, ffcnt, ffpos, fftot);
                hipLaunchKernelGGL(k_ff_finish, dim3(FF_MAX), dim3(FN_T), 0, c->stream, nbt, fflist, seq_flag,
                                   fstart, emin_c, sabs_c, fftot, vals, ffpool, ffcnt, ffpos, cand_buf,
                                   replay_cap(), cen, dstate);
                ST_LAUNCH_CHECK();
                if (getenv("ST_DEBUG")) {  // flagged clusters, their members and replay candidates
                    uint32_t hfl[FF_MAX + 1], hz[FF_MAX];
                    std::vector<uint32_t> f2(k), fs(k + 1);
                    ST_HIP(hipMemcpyAsync(hfl, fflist, sizeof hfl, hipMemcpyDeviceToHost, c->stream));
                    ST_HIP(hipMemcpyAsync(hz, ffz, sizeof hz, hipMemcpyDeviceToHost, c->stream));
                    ST_HIP(hipMemcpyAsync(f2.data(), seq_flag, 4 * k, hipMemcpyDeviceToHost, c->stream));
                    ST_HIP(hipMemcpyAsync(fs.data(), fstart, 4 * (k + 1), hipMemcpyDeviceToHost, c->stream));
                    ST_HIP(hipStreamSynchronize(c->stream));
                    fprintf(stderr, "[st k1] n=%llu flagged=%u", (unsigned long long)n, hfl[0]);
                    for (uint32_t f = 0; f < hfl[0] && f < (uint32_t)FF_MAX; ++f)
                        fprintf(stderr, " c%u:members=%u,cands=%u,seq=%u", hfl[1 + f],
                                fs[hfl[1 + f] + 1] - fs[hfl[1 + f]], hz[f], f2[hfl[1 + f]] == 2u ? 1u : 0u);
                    fprintf(stderr, "\n");
                }
                mark(c, "k1.update");
                continue;
            }
            ST_HIP(hipMemcpyAsync(hinfo, dinfo, 8, hipMemcpyDeviceToHost, c->stream));
            ST_HIP(hipStreamSynchronize(c->stream));
            const uint32_t nflag = hinfo[0], ftotal = hinfo[1];
            uint32_t nseq = 0;
            if (nflag) {
                // the flagged clusters' members in point order (fvals, starts fstart), then
                // the chunked replay and, where it gives up, the sequential chain
                if (nflag <= ff_max && !getenv("ST_K1_TILES")) {
                    const uint32_t nch = (uint32_t)((n + FF_CH - 1) / FF_CH);
                    hipLaunchKernelGGL(k_ff_count, dim3(G), dim3(256), 0, c->stream, lab8, n, nch, k, seq_flag, fhist);
                    hipLaunchKernelGGL(k_ff_scan, dim3(nflag), dim3(FS_T), 0, c->stream, fhist, nch, k, seq_flag,
                                       fstart);
                    hipLaunchKernelGGL(k_ff_scatter, dim3(G), dim3(256), 0, c->stream, lab8, pts, n, nch, k, seq_flag,
                                       fhist, vals);
                } else {
                    hipLaunchKernelGGL(k_flag_tiles, dim3(G), dim3(F1_T), 0, c->stream, lab8, n, ntiles, k, seq_flag,
                                       fhist);
                    hipLaunchKernelGGL(k_flag_scan, dim3(k), dim3(SC_T), 0, c->stream, fhist, ntiles, seq_flag, fstart);
                    hipLaunchKernelGGL(k_flag_scatter, dim3(G), dim3(F1_T), 0, c->stream, lab8, pts, n, ntiles, k,
                                       kbits, seq_flag, fhist, vals);
                }
                ST_LAUNCH_CHECK();
                // short chunks: the flagged clusters are few, their replay passes run over many
                // workgroups at once
                const uint64_t fch = ftotal / FL_CH + nflag + 1;
                chunk_list(c, fstart, k, ch_cnt, ch_first, chunks, nullptr, FL_CH);
                chunked_replay(c, vals, fstart, k, fch, chunks, ch_first, seq_flag, emin_c, sabs_c, rp_csum, rp_total,
                               rp_ccnt, rp_cof, rp_ctot, cand_buf, cen, nullptr, nullptr);
                if (getenv("ST_DEBUG")) {
                    std::vector<uint32_t> f2(k);
                    ST_HIP(hipMemcpyAsync(f2.data(), seq_flag, 4 * k, hipMemcpyDeviceToHost, c->stream));
                    ST_HIP(hipStreamSynchronize(c->stream));
                    for (int i = 0; i < k; ++i) nseq += f2[i] == 2;
                }
                hipLaunchKernelGGL(k_sum1d_seq, dim3(k), dim3(64), 0, c->stream, vals, fstart, seq_flag, cen);
                ST_LAUNCH_CHECK();
            }
            if (getenv("ST_DEBUG"))
                fprintf(stderr, "[st k1] n=%llu uncertified=%u sequential-fallback=%u\n", (unsigned long long)n, nflag,
                        nseq);
            mark(c, "k1.update");
        }
        return;
    }
    for (int it = 0; it < iters; ++it) {
        const uint32_t *vals_s = nullptr;
        if (fused) {
            auto *ckeys = wsT<uint32_t>(c, "k1.ckeys", (size_t)k);
            auto *corder = wsT<uint32_t>(c, "k1.corder", (size_t)k);
            hipLaunchKernelGGL(k_sortkeys, dim3(grid_for(k, 256, 256)), dim3(256), 0, c->stream, cen, k, ckeys, corder);
            ST_LAUNCH_CHECK();
            radix_sort_u32(c, ckeys, corder, (uint64_t)k, 0, 32, "k1.csort");
            {
                KTimer kt(c, "k1.assign");
                hipLaunchKernelGGL(k_kd1_assign_hist, dim3(ntiles), dim3(F1_T), 0, c->stream, pts, n, cen, corder, k,
                                   it == iters - 1 ? labels : (uint32_t *)nullptr, lab8, fhist, ntiles);
                ST_LAUNCH_CHECK();
            }
            mark(c, "k1.assign");
            scan_u32(c, fhist, fhist, (uint64_t)256 * ntiles, nullptr);
            hipLaunchKernelGGL(k_lab_scatter<uint8_t>, dim3(ntiles), dim3(F1_T), 0, c->stream, lab8, pts, n, kbits,
                               fhist, ntiles, vals);
            hipLaunchKernelGGL(k_f1_starts, dim3(grid_for((uint64_t)k + 1, 256, 256)), dim3(256), 0, c->stream,
                               fhist, ntiles, k, n, start);
            ST_LAUNCH_CHECK();
            vals_s = vals;
        } else {
            const bool paired = assign1d(c, pts, n, k, cen, labels, keys, vals, it == iters - 1);
            mark(c, "k1.assign");
            // update
            if (!paired) {
                hipLaunchKernelGGL(k_pairs1d, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c->stream, pts, labels, n,
                                   keys, vals);
                ST_LAUNCH_CHECK();
            }
            uint32_t *skeys = keys, *svals = vals;  // where the sort leaves its result (no copy back)
            radix_sort_u32_inplace_or_swap(c, keys, vals, n, 0, kbits, "k1.msort", &skeys, &svals);
            bounds_from_sorted(c, skeys, n, k, start);
            vals_s = svals;
        }
        {
            KTimer kt(c, "k1.sum");
            {
                const unsigned gk = grid_for((uint64_t)k, 256, 1024);
                chunk_list(c, start, k, ch_cnt, ch_first, chunks, acc);
                hipLaunchKernelGGL(k_sum1d_chunks, dim3(maxch), dim3(SC_T), 0, c->stream, vals_s, chunks, ch_first + k,
                                   acc);
                hipLaunchKernelGGL(k_sum1d_final, dim3(gk), dim3(256), 0, c->stream, acc, start, k, cen, seq_flag,
                                   emin_c, sabs_c);
                ST_LAUNCH_CHECK();
            }
            std::vector<uint32_t> f1;
            if (getenv("ST_DEBUG")) {
                ST_HIP(hipStreamSynchronize(c->stream));
                f1.resize(k);
                ST_HIP(hipMemcpy(f1.data(), seq_flag, 4 * k, hipMemcpyDeviceToHost));
            }
            chunked_replay(c, vals_s, start, k, maxch, chunks, ch_first, seq_flag, emin_c, sabs_c, rp_csum, rp_total,
                           rp_ccnt, rp_cof, rp_ctot, cand_buf, cen, nullptr, nullptr);
            if (getenv("ST_DEBUG")) {
                ST_HIP(hipStreamSynchronize(c->stream));
                std::vector<uint32_t> f2(k);
                ST_HIP(hipMemcpy(f2.data(), seq_flag, 4 * k, hipMemcpyDeviceToHost));
                int a = 0, b = 0;
                for (int i = 0; i < k; ++i) {
                    a += f1[i] == 1;
                    b += f2[i] == 2;
                }
                fprintf(stderr, "[st k1] n=%llu uncertified=%d sequential-fallback=%d\n", (unsigned long long)n, a, b);
            }
            hipLaunchKernelGGL(k_sum1d_seq, dim3(k), dim3(64), 0, c->stream, vals_s, start, seq_flag, cen);
            ST_LAUNCH_CHECK();
        }
        reseed_empty(c, dcols, 1, n, k, start, ddraws, ndraws, dstate, cen);
        mark(c, "k1.update");
    }
}

// the sharded 1-D member order: a stable sort by (segment, label) is a stable sort by label inside
// each segment (segments are contiguous point ranges), done as one counting-sort pass per segment
// that moves value bits only; start[s * k + c] = first position of (s, c), start[nseg * k] = n
void seg_label_sort1d(st_ctx *c, const float *pts, const uint32_t *labels, uint64_t n, int nseg, int k,
                      uint32_t *vals, uint32_t *start) {
    const uint64_t ns = n / (uint64_t)nseg;
    int kbits = 1;
    while ((1 << kbits) < k) ++kbits;
    const uint32_t ntiles = (uint32_t)((ns + F1_TILE - 1) / F1_TILE);
    auto *hist = wsT<uint32_t>(c, "k1.shist", (size_t)256 * (ntiles ? ntiles : 1));
    for (int sg = 0; sg < nseg; ++sg) {
        const uint64_t o = (uint64_t)sg * ns;
        if (ns) {
            hipLaunchKernelGGL(k_lab_hist, dim3(ntiles), dim3(F1_T), 0, c->stream, labels + o, ns, hist, ntiles);
            scan_u32(c, hist, hist, (uint64_t)256 * ntiles, nullptr);
            hipLaunchKernelGGL(k_lab_scatter<uint32_t>, dim3(ntiles), dim3(F1_T), 0, c->stream, labels + o, pts + o, ns,
                               kbits, hist, ntiles, vals + o);
            hipLaunchKernelGGL(k_f1_starts, dim3(grid_for((uint64_t)k + 1, 256, 256)), dim3(256), 0, c->stream, hist,
                               ntiles, k, ns, start + (uint64_t)sg * k, (uint32_t)o);
        } else {
            ST_HIP(hipMemsetD32Async(start + (uint64_t)sg * k, (uint32_t)o, (size_t)k + 1, c->stream));
        }
        ST_LAUNCH_CHECK();
    }
}

__global__ __launch_bounds__(256) void k_part_neutral(Part1 *part) {
    part[(uint64_t)blockIdx.x * 256 + threadIdx.x] = Part1{0.0, 0.0, 1 << 20, 0u};
}

void assign_partials1d(st_ctx *c, const float *pts, uint64_t n, int nseg, int k, const float *cen, uint32_t *labels,
                       double *sums, double *sabs, int32_t *emin, uint32_t *counts) {
    ST_REQUIRE(k >= 1 && k <= 256 && nseg >= 1 && n % (uint64_t)nseg == 0, ST_ERR_ARG,
               "1-D partials: k <= 256 and n in equal segments");
    const uint64_t ns = n / (uint64_t)nseg;
    const uint32_t ntiles = (uint32_t)((ns + F1_TILE - 1) / F1_TILE);
    const uint32_t G = ntiles ? a1_grid(ntiles) : 1;
    auto *part = wsT<Part1>(c, "d1.part", (size_t)nseg * G * 256);
    for (int sg = 0; sg < nseg; ++sg) {
        const uint64_t o = (uint64_t)sg * ns;
        if (ns)
            hipLaunchKernelGGL(k_kd1_assign_acc<false>, dim3(G), dim3(F1_T), 0, c->stream, pts + o, ns, cen, k,
                               labels + o, (uint8_t *)nullptr, ntiles, part + (uint64_t)sg * G * 256,
                               (const uint32_t *)nullptr, (Bnd1 *)nullptr);
        else  // an empty segment: neutral partials (no members, e_min above any real exponent)
            hipLaunchKernelGGL(k_part_neutral, dim3(G), dim3(256), 0, c->stream, part + (uint64_t)sg * G * 256);
    }
    hipLaunchKernelGGL(k_part_fold, dim3((unsigned)nseg * k), dim3(256), 0, c->stream, part, G, k, sums, sabs, emin,
                       counts);
    ST_LAUNCH_CHECK();
}

void partials1d(st_ctx *c, const uint32_t *vals, uint64_t n, const uint32_t *start, int nk, double *sums, double *sabs,
                int32_t *emin, uint32_t *counts) {
    const uint64_t maxch = n / SC_CH + (uint64_t)nk + 1;
    auto *ch_cnt = wsT<uint32_t>(c, "d1.chcnt", (size_t)nk);
    auto *ch_first = wsT<uint32_t>(c, "d1.chfirst", (size_t)nk + 1);
    auto *chunks = wsT<Chunk>(c, "d1.chunks", maxch);
    auto *acc = wsT<SumAcc>(c, "d1.acc", (size_t)nk);
    chunk_list(c, start, nk, ch_cnt, ch_first, chunks, acc);
    const unsigned gk = grid_for((uint64_t)nk, 256, 1024);
    hipLaunchKernelGGL(k_sum1d_chunks, dim3(maxch), dim3(SC_T), 0, c->stream, vals, chunks, ch_first + nk, acc);
    hipLaunchKernelGGL(k_partials_out, dim3(gk), dim3(256), 0, c->stream, acc, start, nk, sums, sabs, emin, counts);
    ST_LAUNCH_CHECK();
}

void seqsum1d(st_ctx *c, const uint32_t *vals, uint64_t n, const uint32_t *start, int k, const uint32_t *pairs,
              uint32_t npairs, double *running, const int32_t *emin, const double *sabs, uint32_t *pflag) {
    const uint64_t maxch = n / SC_CH + (uint64_t)k + 1;
    auto *ch_cnt = wsT<uint32_t>(c, "d1.chcnt", (size_t)k);
    auto *ch_first = wsT<uint32_t>(c, "d1.chfirst", (size_t)k + 1);
    auto *chunks = wsT<Chunk>(c, "d1.chunks", maxch);
    auto *flag_cl = wsT<uint32_t>(c, "d1.flag", (size_t)k);
    auto *base_cl = wsT<double>(c, "d1.base", (size_t)k);
    auto *sum_cl = wsT<double>(c, "d1.sum", (size_t)k);
    auto *csum = wsT<__int128>(c, "d1.csum", maxch);
    auto *ccnt = wsT<uint32_t>(c, "d1.ccnt", maxch);
    auto *cof = wsT<uint32_t>(c, "d1.cof", maxch);
    auto *ctot = wsT<uint32_t>(c, "d1.ctot", (size_t)k);
    auto *total = wsT<__int128>(c, "d1.total", (size_t)k);
    auto *cands = wsT<__int128>(c, "d1.cands", (size_t)k * CAND_MAX);
    ST_HIP(hipMemsetAsync(flag_cl, 0, sizeof(uint32_t) * k, c->stream));
    const unsigned gp = grid_for(npairs, 256, 1024);
    hipLaunchKernelGGL(k_pend_in, dim3(gp), dim3(256), 0, c->stream, pairs, npairs, running, flag_cl, base_cl);
    ST_LAUNCH_CHECK();
    chunk_list(c, start, k, ch_cnt, ch_first, chunks);
    chunked_replay(c, vals, start, k, maxch, chunks, ch_first, flag_cl, emin, sabs, csum, total, ccnt, cof, ctot, cands,
                   nullptr, base_cl, sum_cl);
    hipLaunchKernelGGL(k_pend_out, dim3(gp), dim3(256), 0, c->stream, pairs, npairs, flag_cl, sum_cl, running, pflag);
    ST_LAUNCH_CHECK();
    if (getenv("ST_DEBUG")) {
        std::vector<uint32_t> f(npairs);
        ST_HIP(hipMemcpyAsync(f.data(), pflag, 4ull * npairs, hipMemcpyDeviceToHost, c->stream));
        ST_HIP(hipStreamSynchronize(c->stream));
        uint32_t seq = 0;
        for (uint32_t v : f) seq += v;
        fprintf(stderr, "[st d1] pending=%u replayed=%u sequential=%u\n", npairs, npairs - seq, seq);
    }
}

}  // namespace st
