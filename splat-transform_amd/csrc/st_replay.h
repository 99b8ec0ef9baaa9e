// st_replay.h -- exact replay of a sequential f64 sum (the reference's calcAverage,
// k-means.ts:41-63) in parallel; shared by the 1-D k-means update (st_kmeans1d.hip) and
// the multi-GPU segment chain (st_dist.hip).
#pragma once

#include "st_kmeans.h"

namespace st {
namespace km {

// ---- exact replay of a sequential f64 sum ----------------------------------------------
// Every member is a multiple of 2^e_lo (e_lo = the smallest ulp exponent), so the exact
// prefix sums P_j are integers in units of 2^e_lo; with |P_j| <= sum|x| < 2^(e_lo+120)
// they fit an int128.  M bounds the accumulated rounding drift |s - P|; replay_candidate
// lists the positions where the sequential step may round (tiny members, moves up a
// binade, prefixes within M of a binade's bottom); every other step is exact.  One parallel pass computes P_j and lists the
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

// Position j can round unless all of: P_{j-1} is nonzero and at least M above the bottom of
// its binade bp (so |s_{j-1}| >= 2^bp and s_{j-1} is a multiple of 2^(bp-52)); x_j is a
// multiple of 2^(bp-52); |P_j| + M < 2^(bp+1).  Then s_{j-1} + x_j is a multiple of
// 2^(bp-52) below 2^(bp+1) in magnitude: exactly representable.  Moves down a binade (and
// through zero) are exact steps by this rule, moves up past 2^(bp+1) are candidates.
__device__ inline bool replay_candidate(__int128 Pprev, __int128 P, uint32_t xbits, int e_lo, __int128 margin) {
    const unsigned __int128 mp = Pprev < 0 ? (unsigned __int128)(-Pprev) : (unsigned __int128)Pprev;
    if (mp == 0) return true;
    const int blp = bitlen128(mp);  // |P_{j-1}| in [2^(blp-1), 2^blp) units
    const unsigned __int128 lo_end = ((unsigned __int128)1) << (blp - 1), hi_end = ((unsigned __int128)1) << blp;
    if (mp - lo_end < (unsigned __int128)margin) return true;
    const int bp = blp - 1 + e_lo;
    const uint32_t ex = (xbits >> 23) & 0xffu;
    const int xulp = ex ? (int)ex - 150 : -149;
    if ((xbits & 0x7fffffffu) != 0 && xulp < bp - 52) return true;
    const unsigned __int128 m = P < 0 ? (unsigned __int128)(-P) : (unsigned __int128)P;
    return m + (unsigned __int128)margin >= hi_end;
}

// The replay of one member range [s0, s1) starting from the f64 value s_in (a multiple of
// 2^e_lo, as every sequential partial sum of such members is).  Called by all RT threads
// of a block; thread 0 gets the result.  Returns false (on thread 0) when the range needs
// the plain sequential chain (int128 range, candidate capacity or drift margin exceeded).
__device__ inline bool replay_sum(const uint32_t *__restrict__ vals, uint32_t s0, uint32_t s1, int e_lo, double sabs,
                                  double s_in, __int128 *__restrict__ cand, double *out) {
    __shared__ __int128 wsum[RT / 64];
    __shared__ uint32_t csum[RT / 64];
    const double bound = sabs + __builtin_fabs(s_in);
    if (!(bound * (1.0 + 1.0e-6) < __builtin_ldexp(1.0, e_lo + 118))) return false;  // int128 range
    // drift bound M = 2^(e_top - 33): far above any accumulated rounding (checked below)
    int e_top;
    __builtin_frexp(bound, &e_top);
    const int msh = max(e_top - 33 - e_lo, 0);
    const __int128 margin = ((__int128)1) << msh;
    const __int128 base = f64_units(s_in, e_lo);
    const uint32_t n = s1 - s0, per = (n + RT - 1) / RT;
    const uint32_t a = s0 + min(n, threadIdx.x * per), b = s0 + min(n, (threadIdx.x + 1) * per);
    __int128 local = 0;
    for (uint32_t j = a; j < b; ++j) local += f32_units(vals[j], e_lo);
    __int128 total;
    const __int128 off = base + block_exscan_i128(local, wsum, &total);
    total += base;
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
    if (ctot > CAND_MAX) return false;
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
    __syncthreads();
    if (threadIdx.x != 0) return true;
    // replay the candidates on one lane
    __int128 sv = base, Pprev = base;
    bool ok = true;
    for (uint32_t i = 0; i < ctot; ++i) {
        const __int128 Pc = cand[i];
        const __int128 V = sv + (Pc - Pprev);
        sv = f64_representable(V) ? V : f64_units(f64_round(V, e_lo), e_lo);
        Pprev = Pc;
        const __int128 dev = sv - Pc;
        ok = ok && (dev < 0 ? -dev : dev) < margin;
    }
    const __int128 fin = sv + (total - Pprev);
    if (!ok || !f64_representable(fin)) return false;
    *out = f64_round(fin, e_lo);
    return true;
}

}  // namespace km
}  // namespace st
