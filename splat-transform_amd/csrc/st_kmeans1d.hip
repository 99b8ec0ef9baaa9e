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
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const double p = pts[i];
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
        labels[i] = mini;
    }
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


// calcAverage (k-means.ts:41-63) for one cluster: the reference adds the members' values
// in ascending point order into one f64.  When every partial sum is exactly representable
// (certificate: sum|x| < 2^(emin+53), emin = the smallest ulp exponent among the values)
// the order is immaterial and the block sums in parallel; otherwise the cluster is
// flagged (1) for k_sum1d_replay, which replays the sequential sum exactly from one
// rounding event to the next.
__global__ __launch_bounds__(256) void k_sum1d(const uint32_t *__restrict__ vals, const uint32_t *__restrict__ start,
                                               int k, float *__restrict__ cen, uint32_t *__restrict__ seq_flag,
                                               int32_t *__restrict__ emin_c, double *__restrict__ sabs_c) {
    const int cl = blockIdx.x;
    const uint32_t s0 = start[cl], s1 = start[cl + 1];
    if (s1 == s0) {  // empty: re-seeded separately
        if (threadIdx.x == 0) seq_flag[cl] = 0;
        return;
    }
    __shared__ double red_s[4], red_a[4];
    __shared__ int red_e[4];
    double sum = 0, sabs = 0;
    int emin = 1 << 20;
    for (uint32_t j = s0 + threadIdx.x; j < s1; j += blockDim.x) {
        const float x = __builtin_bit_cast(float, vals[j]);
        sum += (double)x;
        sabs += (double)__builtin_fabsf(x);
        if (x != 0.0f) emin = min(emin, ulp_exp(x));
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int o = 32; o > 0; o >>= 1) {
        sum += __shfl_xor(sum, o, 64);
        sabs += __shfl_xor(sabs, o, 64);
        emin = min(emin, __shfl_xor(emin, o, 64));
    }
    if (lane == 0) {
        red_s[w] = sum;
        red_a[w] = sabs;
        red_e[w] = emin;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    sum = (red_s[0] + red_s[1]) + (red_s[2] + red_s[3]);
    sabs = (red_a[0] + red_a[1]) + (red_a[2] + red_a[3]);
    emin = min(min(red_e[0], red_e[1]), min(red_e[2], red_e[3]));
    // sum|x| bounded above with slack for its own rounding
    const bool exact = sum_is_exact(sabs, emin);
    seq_flag[cl] = exact ? 0u : 1u;
    emin_c[cl] = emin;
    sabs_c[cl] = sabs;
    if (exact) cen[cl] = (float)(sum / (double)(s1 - s0));
}

// ---- exact replay of a sequential f64 sum ----------------------------------------------
// Every member is a multiple of 2^e_lo (e_lo = the smallest ulp exponent), so the exact
// prefix sums P_j are integers in units of 2^e_lo; with |P_j| <= sum|x| < 2^(e_lo+120)
// they fit an int128.  Let B be the binade of |P_j|.  If x_j is a multiple of ulp(B) and
// P_{j-1}, P_j lie in B at least M away from its ends (M bounds the accumulated rounding
// drift |s - P|), the sequential step j cannot round: s_{j-1} and x_j are multiples of
// ulp(B) and s_j stays in B.  Every other position is a "candidate" (tiny members, binade
// changes, near-boundary prefixes).  One parallel pass computes P_j and lists the
// candidates in order; one lane then replays the candidates only,
//     V_c = s_prev + (P_c - P_prev),   s_c = RN(V_c),
// and the final sum is s_last + (P_end - P_last).  The drift is checked against M; a
// cluster with too many candidates or too much drift falls back to k_sum1d_seq.
constexpr int RT = 1024;          // threads per cluster
constexpr int CAND_MAX = 16384;   // candidates per cluster

__device__ inline int bitlen128(unsigned __int128 m) {
    const uint64_t hi = (uint64_t)(m >> 64), lo = (uint64_t)m;
    return hi ? 128 - __builtin_clzll(hi) : (lo ? 64 - __builtin_clzll(lo) : 0);
}
__device__ inline int ctz128(unsigned __int128 m) {
    const uint64_t hi = (uint64_t)(m >> 64), lo = (uint64_t)m;
    return lo ? __builtin_ctzll(lo) : 64 + __builtin_ctzll(hi);
}
// exact value of an f32 in units of 2^e_lo (e_lo <= its ulp exponent)
__device__ inline __int128 f32_units(uint32_t bits, int e_lo) {
    const uint32_t ex = (bits >> 23) & 0xffu, man = bits & 0x7fffffu;
    if (ex == 0 && man == 0) return 0;
    const uint32_t m = ex ? (man | 0x800000u) : man;
    const int e = ex ? (int)ex - 150 : -149;
    const __int128 v = (__int128)m << (e - e_lo);
    return (bits >> 31) ? -v : v;
}
__device__ inline bool f64_representable(__int128 v) {
    const unsigned __int128 m = v < 0 ? (unsigned __int128)(-v) : (unsigned __int128)v;
    return m == 0 || bitlen128(m) - ctz128(m) <= 53;
}
// round-to-nearest-even of v * 2^e_lo to f64
__device__ inline double f64_round(__int128 v, int e_lo) {
    const bool neg = v < 0;
    unsigned __int128 m = neg ? (unsigned __int128)(-v) : (unsigned __int128)v;
    const int bl = bitlen128(m);
    int sh = 0;
    if (bl > 53) {
        sh = bl - 53;
        const unsigned __int128 rem = m & ((((unsigned __int128)1) << sh) - 1);
        const unsigned __int128 half = ((unsigned __int128)1) << (sh - 1);
        m >>= sh;
        if (rem > half || (rem == half && (m & 1))) {
            m += 1;
            if (m == (((unsigned __int128)1) << 53)) {
                m >>= 1;
                ++sh;
            }
        }
    }
    const double r = __builtin_ldexp((double)(uint64_t)m, e_lo + sh);
    return neg ? -r : r;
}
// s (a multiple of 2^e_lo) in units of 2^e_lo
__device__ inline __int128 f64_units(double s, int e_lo) {
    if (s == 0) return 0;
    int e;
    const double fr = __builtin_frexp(s, &e);  // s = fr * 2^e, 0.5 <= |fr| < 1
    const int64_t M = (int64_t)__builtin_ldexp(fr, 53);
    const int sh = e - 53 - e_lo;
    return sh >= 0 ? ((__int128)M << sh) : (__int128)(M >> (-sh));
}

// block-wide exclusive scan of one int128 per thread (RT threads)
__device__ inline __int128 block_exscan_i128(__int128 v, __int128 *wsum, __int128 *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __int128 incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t lo = __shfl_up((uint64_t)incl, o, 64), hi = __shfl_up((uint64_t)(incl >> 64), o, 64);
        const __int128 u = (__int128)(((unsigned __int128)hi << 64) | lo);
        if (lane >= o) incl += u;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    __int128 off = 0, tot = 0;
    for (int i = 0; i < RT / 64; ++i) {
        if (i < w) off += wsum[i];
        tot += wsum[i];
    }
    __syncthreads();
    *total = tot;
    return off + incl - v;
}

__device__ inline int binade_of(__int128 P, int e_lo) {  // floor(log2 |P * 2^e_lo|), -1000 for 0
    const unsigned __int128 m = P < 0 ? (unsigned __int128)(-P) : (unsigned __int128)P;
    return m ? bitlen128(m) - 1 + e_lo : -1000;
}

// position j can round (see above): tiny member, binade change, or near a binade end
__device__ inline bool replay_candidate(__int128 Pprev, __int128 P, uint32_t xbits, int e_lo, __int128 margin) {
    const int b = binade_of(P, e_lo);
    if (b == -1000 || b != binade_of(Pprev, e_lo)) return true;
    const uint32_t ex = (xbits >> 23) & 0xffu;
    const int xulp = ex ? (int)ex - 150 : -149;
    if ((xbits & 0x7fffffffu) != 0 && xulp < b - 52) return true;
    const unsigned __int128 m = P < 0 ? (unsigned __int128)(-P) : (unsigned __int128)P;
    const int bl = bitlen128(m);
    const unsigned __int128 lo_end = ((unsigned __int128)1) << (bl - 1), hi_end = ((unsigned __int128)1) << bl;
    return (m - lo_end) < (unsigned __int128)margin || (hi_end - m) <= (unsigned __int128)margin;
}

__global__ __launch_bounds__(RT) void k_sum1d_replay(const uint32_t *__restrict__ vals,
                                                     const uint32_t *__restrict__ start,
                                                     uint32_t *__restrict__ seq_flag,
                                                     const int32_t *__restrict__ emin_c,
                                                     const double *__restrict__ sabs_c, float *__restrict__ cen,
                                                     __int128 *__restrict__ cand_all) {
    const int cl = blockIdx.x;
    if (seq_flag[cl] != 1u) return;
    const uint32_t s0 = start[cl], s1 = start[cl + 1];
    const int e_lo = emin_c[cl];
    const double sabs = sabs_c[cl];
    if (!(sabs * (1.0 + 1.0e-6) < __builtin_ldexp(1.0, e_lo + 118))) {  // int128 range
        if (threadIdx.x == 0) seq_flag[cl] = 2u;
        return;
    }
    // drift bound M = 2^(e_top - 33): far above any accumulated rounding (checked below)
    int e_top;
    __builtin_frexp(sabs, &e_top);
    const int msh = max(e_top - 33 - e_lo, 0);
    const __int128 margin = ((__int128)1) << msh;
    __shared__ __int128 wsum[RT / 64];
    __shared__ uint32_t csum[RT / 64];
    __shared__ uint32_t ncand_sh;
    __int128 *cand = cand_all + (uint64_t)cl * CAND_MAX;
    const uint32_t n = s1 - s0, per = (n + RT - 1) / RT;
    const uint32_t a = s0 + min(n, threadIdx.x * per), b = s0 + min(n, (threadIdx.x + 1) * per);
    __int128 local = 0;
    for (uint32_t j = a; j < b; ++j) local += f32_units(vals[j], e_lo);
    __int128 total;
    const __int128 off = block_exscan_i128(local, wsum, &total);
    // count, then write in order, the candidates of this chunk
    uint32_t mine = 0;
    {
        __int128 P = off;
        for (uint32_t j = a; j < b; ++j) {
            const uint32_t xb = vals[j];
            const __int128 Pn = P + f32_units(xb, e_lo);
            mine += replay_candidate(P, Pn, xb, e_lo, margin) ? 1u : 0u;
            P = Pn;
        }
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
    }
    if (lane == 63) csum[w] = incl;
    __syncthreads();
    uint32_t coff = 0, ctot = 0;
    for (int i = 0; i < RT / 64; ++i) {
        if (i < w) coff += csum[i];
        ctot += csum[i];
    }
    coff += incl - mine;
    if (ctot > CAND_MAX) {
        if (threadIdx.x == 0) seq_flag[cl] = 2u;
        return;
    }
    {
        __int128 P = off;
        uint32_t o = coff;
        for (uint32_t j = a; j < b; ++j) {
            const uint32_t xb = vals[j];
            const __int128 Pn = P + f32_units(xb, e_lo);
            if (replay_candidate(P, Pn, xb, e_lo, margin)) cand[o++] = Pn;
            P = Pn;
        }
    }
    if (threadIdx.x == 0) ncand_sh = ctot;
    __syncthreads();
    if (threadIdx.x != 0) return;
    // replay the candidates on one lane
    __int128 sv = 0, Pprev = 0;
    bool ok = true;
    for (uint32_t i = 0; i < ncand_sh; ++i) {
        const __int128 Pc = cand[i];
        const __int128 V = sv + (Pc - Pprev);
        sv = f64_representable(V) ? V : f64_units(f64_round(V, e_lo), e_lo);
        Pprev = Pc;
        const __int128 dev = sv - Pc;
        ok = ok && (dev < 0 ? -dev : dev) < margin;
    }
    const __int128 fin = sv + (total - Pprev);
    if (!ok || !f64_representable(fin)) {
        seq_flag[cl] = 2u;  // drift beyond the margin: sequential chain
        return;
    }
    cen[cl] = (float)(f64_round(fin, e_lo) / (double)(s1 - s0));
    seq_flag[cl] = 0u;
}

// the sequential f64 sum of a flagged cluster: one lane walks the members in order, the
// loads run PF x 16 bytes ahead of the dependent add chain
__global__ __launch_bounds__(64) void k_sum1d_seq(const uint32_t *__restrict__ vals, const uint32_t *__restrict__ start,
                                                  const uint32_t *__restrict__ seq_flag, float *__restrict__ cen) {
    const int cl = blockIdx.x;
    if (seq_flag[cl] != 2u || threadIdx.x != 0) return;
    const uint32_t s0 = start[cl], s1 = start[cl + 1];
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
    cen[cl] = (float)(s / (double)(s1 - s0));
}

}  // namespace

// one exact 1-D assign: KdTree build == stable sort of the centroid values
// (kd-tree.ts:73-99), then the walk simulation
void assign1d(st_ctx *c, const float *pts, uint64_t n, int k, const float *cen, uint32_t *labels) {
    auto *ckeys = wsT<uint32_t>(c, "k1.ckeys", (size_t)k);
    auto *corder = wsT<uint32_t>(c, "k1.corder", (size_t)k);
    hipLaunchKernelGGL(k_sortkeys, dim3(grid_for(k, 256, 256)), dim3(256), 0, c->stream, cen, k, ckeys, corder);
    ST_LAUNCH_CHECK();
    radix_sort_u32(c, ckeys, corder, (uint64_t)k, 0, 32, "k1.csort");
    const unsigned g = grid_for(n, 256, 256 * 16);
    KTimer kt(c, "k1.assign");
    if (k <= KD1_LDS)
        hipLaunchKernelGGL(k_kd1_assign<true>, dim3(g), dim3(256), 0, c->stream, pts, n, cen, corder, k, labels);
    else
        hipLaunchKernelGGL(k_kd1_assign<false>, dim3(g), dim3(256), 0, c->stream, pts, n, cen, corder, k, labels);
    ST_LAUNCH_CHECK();
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
    int kbits = 1;
    while ((1ull << kbits) < (uint64_t)k) ++kbits;
    for (int it = 0; it < iters; ++it) {
        assign1d(c, pts, n, k, cen, labels);
        mark(c, "k1.assign");
        // update
        hipLaunchKernelGGL(k_pairs1d, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c->stream, pts, labels, n, keys,
                           vals);
        ST_LAUNCH_CHECK();
        radix_sort_u32(c, keys, vals, n, 0, kbits, "k1.msort");
        bounds_from_sorted(c, keys, n, k, start);
        {
            KTimer kt(c, "k1.sum");
            hipLaunchKernelGGL(k_sum1d, dim3(k), dim3(256), 0, c->stream, vals, start, k, cen, seq_flag, emin_c,
                               sabs_c);
            ST_LAUNCH_CHECK();
            std::vector<uint32_t> f1;
            if (getenv("ST_DEBUG")) {
                ST_HIP(hipStreamSynchronize(c->stream));
                f1.resize(k);
                ST_HIP(hipMemcpy(f1.data(), seq_flag, 4 * k, hipMemcpyDeviceToHost));
            }
            hipLaunchKernelGGL(k_sum1d_replay, dim3(k), dim3(RT), 0, c->stream, vals, start, seq_flag, emin_c, sabs_c,
                               cen, cand_buf);
            ST_LAUNCH_CHECK();
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
            hipLaunchKernelGGL(k_sum1d_seq, dim3(k), dim3(64), 0, c->stream, vals, start, seq_flag, cen);
            ST_LAUNCH_CHECK();
        }
        reseed_empty(c, dcols, 1, n, k, start, ddraws, ndraws, dstate, cen);
        mark(c, "k1.update");
    }
}

}  // namespace st
