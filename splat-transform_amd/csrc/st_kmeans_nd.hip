// st_kmeans_nd.hip -- N-D k-means assign on the matrix cores + exact update.
//
// The SH palette step (write-sog.ts:313): points = the 3C f_rest columns
// (D = 45 at SH3), K = paletteSize (65,536 from 64k splats up).
//
// Score on MFMA.  score(c) = |c|^2 - 2 p.c orders the centroids of a fixed
// point exactly like the reference's distance.  Coordinates are scaled by a
// power of two sigma (max|x|*sigma in [1,2), exact) and rounded to fp16; one
// v_mfma_f32_32x32x16_f16 chain over a K-dim of KP = roundup(D+3, 16) computes
//     A[c] = [ c~ | n1 n2 n3 ]   (centroid rows; n = |sigma c|^2 split in fp16)
//     B[p] = [ -2 p~ | 1 1 1 ]   (point columns)
// Products are exact in f32, so (|x - x~| <= 2^-11 |x| + e_abs)
//     |score_mfma - score| <= E = A |p| cmax + B cmax^2 + e_abs-terms
// with e_abs = 2^-25 when the matrix cores keep fp16 denormals (probed once per
// context) and 2^-14 otherwise.  The epilogue keeps, per point and lane-half, the
// running top-3 of the 16-row tile minima (a v_min3 tree per tile, then two v_med3 +
// one v_min) and the tiles of the best two.  m2 > m1 + W_p (W_p = 2E + 2 delta_p,
// delta_p = the reference's own f64 rounding) decides the point: k_fixrow finds the
// row inside the best tile-half with the exact f64 distance.  m3 > m1 + W_p puts
// every candidate in the best two tile-halves: k_fixpair settles those 32 rows.
// Otherwise the point is ambiguous (~2% at SH3): a second sweep collects every centroid with
// score <= m1 + W_p (a superset of the exact argmin set) and the exact f64
// distance of kd-tree.ts:26-35 decides; exact ties go to the KdTree walk.
//
// Tiling (gfx950, wave64): workgroup = 4 waves, each wave owns PT = 4 tiles of
// 32 points whose B fragments stay in VGPRs for the whole sweep; 32-row
// centroid tiles (pre-laid-out in fragment order, KS x 1 KiB each) stream
// through a double-buffered LDS ring, CT_STAGE tiles per barrier, filled by
// global_load_lds DMA (no VGPRs held for the prefetch).  The C/D
// layout puts the point on the lane (col = lane & 31) and 16 centroid rows per
// lane-half in registers, so the top-3 update is lane-local.
#include <cmath>
#include <utility>

#include "st_kmeans.h"

namespace st {
namespace {

using namespace km;

// compile-time loop: f(std::integral_constant<int, 0>{}) ... f(integral_constant<N - 1>{})
template <typename F, int... I>
__device__ inline void static_for_(F &f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ inline void static_for(F &&f) {
    static_for_(f, std::make_integer_sequence<int, N>{});
}

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int PT = 4;          // point tiles per wave
constexpr int NW = 4;          // waves per workgroup (they share the LDS centroid stages)
constexpr int WG = 64 * NW;    // threads per workgroup
constexpr int CT_STAGE = 8;    // centroid tiles per LDS stage
constexpr int CAND_CAP = 64;   // candidate slots per ambiguous point
constexpr int CAND_CAP2 = 2048;  // ... per point whose list overflowed (a second collect)
constexpr int OVF_BATCH = 4096;  // overflowed points per second collect (32 MiB of lists, kept by the workspace)
// members above which a cluster's sum is split over many workgroups (k_big_*); ST_SUMND_BIG
// lowers it so that tests drive that path with small inputs
uint32_t sumnd_big() {
    const char *e = getenv("ST_SUMND_BIG");  // read per call (tests set it around one call)
    return e ? (uint32_t)std::max(1ul, strtoul(e, nullptr, 10)) : 16384u;
}

__host__ __device__ inline int kp_of(int d) { return ((d + 3) + 15) / 16 * 16; }

// fp16 RNE of a finite float (scaled values are < 2^16)
__device__ inline uint16_t h_bits(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
__device__ inline float h_val(uint16_t b) { return (float)__builtin_bit_cast(_Float16, b); }

// |score_mfma - score| <= E(p, c) = r (|p| |dc| + |dp| |c~|) + a |p~| |c~| + b |c~|^2 + ec (|p~| + |c~|) + ep
// with dp = p - p~, dc = c - c~ the fp16 rounding residuals (p.c - p~.c~ = p.dc + dp.c~, x2 for
// the -2 factor), a / b the f32 accumulation, ec / ep the fp16 underflow; delta = rel (|p| + |c|)^2
struct Bound {
    float r, a, b, ec, ep, rel;
};

// error-bound constants for a given dimension and fp16-denormal behaviour
Bound make_bound(int d, bool denorm) {
    const double u = std::ldexp(1.0, -11);          // fp16 RNE relative half-ulp
    const double e_abs = denorm ? std::ldexp(1.0, -25) : std::ldexp(1.0, -14);
    const double gam = (d + 3 + 3) * std::ldexp(1.0, -23);  // f32 accumulation, truncation-safe
    Bound B{};
    // rounding residuals of p and c (x2 for the -2 factor), accumulation; 5% slack
    B.r = (float)(2 * 1.05);
    B.a = (float)(2.01 * gam * (1 + u) * (1 + u) * 1.05);
    B.b = (float)((1.01 * gam + std::ldexp(1.0, -22)) * 1.05);
    B.ec = (float)(2 * std::sqrt((double)d) * e_abs * (1 + u) * 1.05);
    B.ep = (float)((2 * d * e_abs * e_abs + 3 * e_abs) * 1.05 + 1e-30);
    B.rel = 1.0e-13f;
    return B;
}

// E for point norm pn, residual norm dp and centroid norm cn, residual norm dc (all rounded up;
// |p~| <= pn + dp, |c~| <= cn + dc)
__device__ inline float err_bound(const Bound &B, float pn, float dp, float cn, float dc) {
    const float pt = pn + dp, ct = cn + dc;
    return B.r * (pn * dc + dp * ct) + B.a * pt * ct + B.b * ct * ct + B.ec * (pt + ct) + B.ep;
}

// Norm table: tab[b] = the largest rounding-residual norm among the rows whose norm falls in
// buckets 0..b of [0, cm] (prefix maxima; bucket(x) = min(NB - 1, floor(x NB / cm)), monotone in x)
constexpr int NTAB = 1024;
__device__ inline uint32_t norm_bucket(float x, float scale) {
    return (uint32_t)fminf(x * scale, (float)(NTAB - 1));
}
__global__ __launch_bounds__(NTAB) void k_norm_table(const float *__restrict__ cnorm, const float *__restrict__ cdn,
                                                     uint32_t rows, const uint32_t *__restrict__ cmax_bits,
                                                     float *__restrict__ tab) {
    __shared__ uint32_t m[NTAB];
    const uint32_t t = threadIdx.x;
    m[t] = 0u;
    __syncthreads();
    const float cm = __builtin_bit_cast(float, cmax_bits[0]);
    const float scale = cm > 0.f ? (float)NTAB / cm : 0.f;
    for (uint32_t r = t; r < rows; r += NTAB) {
        // non-negative floats: bit order; the read skips the atomics that cannot raise the slot
        // (the norms crowd into few buckets)
        const uint32_t b = norm_bucket(cnorm[r], scale), v = __builtin_bit_cast(uint32_t, cdn[r]);
        if (v > __hip_atomic_load(&m[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) atomicMax(&m[b], v);
    }
    __syncthreads();
    for (uint32_t o = 1; o < (uint32_t)NTAB; o <<= 1) {
        const uint32_t v = t >= o ? m[t - o] : 0u;
        __syncthreads();
        m[t] = max(m[t], v);
        __syncthreads();
    }
    tab[t] = __builtin_bit_cast(float, m[t]);
}

// The largest norm a row c can have when its score |c|^2 - 2 p.c is at most t: the score is at
// least |c|^2 - 2 pn |c| (pn >= |p|), so |c| <= pn + sqrt(pn^2 + t).  Rounded up past the f32
// arithmetic (q's rounding covered by the 2^-19 term, sqrt and the sum by the factor) and the
// 1e-6 the stored norms carry.
__device__ inline float norm_reach(float pn, float t) {
    const float q = pn * pn + t;
    const float qe = q + 0x1p-19f * (pn * pn + __builtin_fabsf(t));
    return (pn + __builtin_sqrtf(fmaxf(0.f, qe))) * (1.0f + 0x1p-18f);
}

// The decision window with the errors bounded by the norms that can matter (kd-tree.ts:22-70
// finds the exact f64 argmin; a row matters only if it might beat the best):
//   * the best row c1 of the best tile-half scores at most m1u + E(cb, dcb) (cb, dcb: the
//     half's largest norm and residual), so |c1| <= R1 = norm_reach(m1u + E(cb)); its own error
//     takes min(R1, cb) and the largest residual among rows of norm <= R1 (the norm table) --
//     an outlying row in the same tile-half no longer widens it;
//   * a competitor c can reach the best's score (m1u + that error, plus both rows' f64
//     roundings: t) only if |c| <= R = norm_reach(t); its error takes min(R, cm) and the norm
//     table's residual at R instead of the palette's cm / dcm -- one outlying centroid no longer
//     widens every point's window.
// With R1 >= cb and R >= cm this is the palette-wide window of round 3.
__device__ inline float wbound_r(const Bound &B, float pn, float dp, float cb, float dcb, float cm, float ntab_scale,
                                 const float *__restrict__ ntab, float m1u) {
    const float e0 = err_bound(B, pn, dp, cb, dcb);
    const float c1 = fminf(norm_reach(pn, m1u + e0 * 1.0001f), cb);
    const float eb = err_bound(B, pn, dp, c1, fminf(dcb, ntab[norm_bucket(c1, ntab_scale)]));
    const float sb = pn + c1, sm = pn + cm;
    const float t = m1u + eb * 1.0001f + B.rel * (sb * sb + sm * sm);
    const float cr = fminf(norm_reach(pn, t), cm);
    const float dcr = ntab[norm_bucket(cr, ntab_scale)];
    const float sr = pn + cr;
    return (eb + err_bound(B, pn, dp, cr, dcr) + B.rel * (sb * sb + sr * sr)) * 1.0001f;
}

// the window between two given tile-halves (largest norms ca, cb and residuals dca, dcb)
__device__ inline float wbound_pair(const Bound &B, float pn, float dp, float ca, float dca, float cb, float dcb) {
    const float s = pn + fmaxf(ca, cb);
    return (err_bound(B, pn, dp, ca, dca) + err_bound(B, pn, dp, cb, dcb) + 2.0f * B.rel * s * s) * 1.0001f;
}

// largest norm and largest rounding-residual norm (rounded up) among the 16 rows of each tile-half
__global__ __launch_bounds__(256) void k_half_max(const float *__restrict__ cnorm, const float *__restrict__ cdn,
                                                  uint32_t nhalves, float *__restrict__ chalf,
                                                  float *__restrict__ chalf_d) {
    for (uint32_t h = blockIdx.x * blockDim.x + threadIdx.x; h < nhalves; h += gridDim.x * blockDim.x) {
        float m = 0.f, md = 0.f;
        for (int rr = 0; rr < 16; ++rr) {
            const uint32_t r = (h >> 1) * 32 + 4 * (h & 1) + (rr & 3) + 8 * (rr >> 2);
            m = fmaxf(m, cnorm[r]);
            md = fmaxf(md, cdn[r]);
        }
        chalf[h] = m;
        chalf_d[h] = md;
    }
}

// does v_mfma_f32_32x32x16_f16 keep fp16 denormal inputs?
__global__ void k_probe_denorm(float *out) {
    const int lane = threadIdx.x;
    f16x8 a = {}, b = {};
    if (lane == 0) {
        a[0] = __builtin_bit_cast(_Float16, (uint16_t)0x0010u);  // 2^-20
        b[0] = (_Float16)1.0f;
    }
    f32x16 acc = {};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    if (lane == 0) out[0] = acc[0];
}

// ---- preparation kernels ------------------------------------------------------
__global__ __launch_bounds__(256) void k_absmax(const float *const *cols, int d, uint64_t n, uint32_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    float m = 0.f;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        for (int c = 0; c < d; ++c) m = fmaxf(m, __builtin_fabsf(cols[c][i]));
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(out, __builtin_bit_cast(uint32_t, m));
}

// point B fragments: pfrag[t][s][lane] = 8 fp16 of B[k = 16s + 8h + j][p = 32t + (lane&31)];
// also |sigma p| (rounded up) and the AoS f32 copy (row stride aos_ld(d), zero padded).
// One workgroup per PF_PTS points: the d column slices land in LDS (coalesced reads), then
// the AoS rows and the point tiles' fragments leave as contiguous runs (coalesced writes).
constexpr int PF_PTS = 128;            // points (= threads) per workgroup (4 tiles): 31.5 KiB of LDS,
                                       // five workgroups per CU
constexpr int PF_LDS_LD = PF_PTS + 1;  // LDS column stride: row-wise reads hit distinct banks
// DT > 0: the dimension count known at compile time (the SH palettes: 45, 24, 9) -- every column
// load in flight at once and the row / fragment index arithmetic by constants; DT = 0: any d <= 61
template <int DT>
__global__ __launch_bounds__(PF_PTS) void k_point_frags(const float *const *cols, int d_rt, uint64_t n, uint32_t ntiles,
                                                     int ks_rt, float sigma, uint4 *pfrag, float *pnorm, float *pdn,
                                                     float *aos) {
    __shared__ float x[(DT ? DT : 61) * PF_LDS_LD];  // d <= 61
    const int d = DT ? DT : d_rt;
    const int ks = DT ? kp_of(DT) / 16 : ks_rt;
    const uint64_t p0 = (uint64_t)blockIdx.x * PF_PTS;
    const int j = threadIdx.x;
    const bool valid = p0 + j < n;
    const uint64_t pj = valid ? p0 + j : n - 1;  // loads stay in bounds without a branch
    if constexpr (DT > 0) {
        float v[DT];
#pragma unroll
        for (int u = 0; u < DT; ++u) v[u] = cols[u][pj];
#pragma unroll
        for (int u = 0; u < DT; ++u) x[u * PF_LDS_LD + j] = valid ? v[u] : 0.0f;
    } else {
        // batches of 8 columns: the loads of a batch are in flight together
        int k0 = 0;
        for (; k0 + 8 <= d; k0 += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = cols[k0 + u][pj];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[(k0 + u) * PF_LDS_LD + j] = valid ? v[u] : 0.0f;
        }
        for (; k0 < d; ++k0) x[k0 * PF_LDS_LD + j] = valid ? cols[k0][pj] : 0.0f;
    }
    __syncthreads();
    if (valid) {
        // |sigma p| and the norm of its fp16 rounding residual p - p~ (exact in f64), rounded up
        double nn = 0, dd = 0;
        for (int k = 0; k < d; ++k) {
            const float f = x[k * PF_LDS_LD + j] * sigma;
            const double v = (double)f, r = v - (double)h_val(h_bits(f));
            nn += v * v;
            dd += r * r;
        }
        pnorm[p0 + j] = (float)(__builtin_sqrt(nn) * (1.0 + 1e-6));
        pdn[p0 + j] = (float)(__builtin_sqrt(dd) * (1.0 + 1e-6));
    }
    // AoS rows: one float4 per thread-step over the workgroup's contiguous row block
    const int ld = aos_ld(d), q4 = ld / 4;
    const uint32_t rows = (uint32_t)min((uint64_t)PF_PTS, n - min(n, p0));
    float4 *dst = reinterpret_cast<float4 *>(aos + p0 * ld);
    for (uint32_t f = j; f < rows * q4; f += PF_PTS) {
        const uint32_t r = f / q4, c = (f % q4) * 4;
        float4 v;
        v.x = c + 0 < (uint32_t)d ? x[(c + 0) * PF_LDS_LD + r] : 0.0f;
        v.y = c + 1 < (uint32_t)d ? x[(c + 1) * PF_LDS_LD + r] : 0.0f;
        v.z = c + 2 < (uint32_t)d ? x[(c + 2) * PF_LDS_LD + r] : 0.0f;
        v.w = c + 3 < (uint32_t)d ? x[(c + 3) * PF_LDS_LD + r] : 0.0f;
        dst[f] = v;
    }
    // fragments of the workgroup's tiles (contiguous: tile-major, then k-step, then lane)
    const uint32_t t0 = blockIdx.x * (PF_PTS / 32);
    const uint32_t tiles = min((uint32_t)(PF_PTS / 32), ntiles - t0);
    for (uint32_t f = j; f < tiles * ks * 64; f += PF_PTS) {
        const uint32_t t = f / (ks * 64), rem = f % (ks * 64);
        const int st = (int)(rem / 64), h = (int)((rem % 64) / 32), l = (int)(rem % 32);
        const uint32_t r = t * 32 + l;
        const bool pv = p0 + r < n;
        uint16_t e[8];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
            const int k = 16 * st + 8 * h + jj;
            uint16_t bits = 0;
            if (k < d) {
                if (pv) bits = h_bits(-2.0f * h_val(h_bits(x[k * PF_LDS_LD + r] * sigma)));  // -2 p~ exactly
            } else if (k < d + 3) {
                bits = pv ? (uint16_t)0x3c00u : (uint16_t)0;  // 1.0
            }
            e[jj] = bits;
        }
        uint4 v;
        v.x = e[0] | ((uint32_t)e[1] << 16);
        v.y = e[2] | ((uint32_t)e[3] << 16);
        v.z = e[4] | ((uint32_t)e[5] << 16);
        v.w = e[6] | ((uint32_t)e[7] << 16);
        pfrag[(uint64_t)(t0 + t) * ks * 64 + rem] = v;
    }
}

// centroid A fragments + cmax + the AoS f32 copy of the centroids (exact distances);
// one thread per centroid row; rows >= k can never win
// 64 centroid rows per workgroup, one per lane; wave w of the four owns dimensions
// [per w, per (w + 1)) of those rows' caos / cfix entries and its share of their squared norms
// (f64, summed over the waves through LDS in a fixed order), and waves 0..ks-1 their fp16
// fragments (fragment s: dimensions 16s .. 16s + 15; the norm columns d, d + 1, d + 2 in the
// last).  Every column read is 64 consecutive rows; one row per lane over all dimensions left a
// single wave per SIMD to hide those reads' latency.
constexpr int CF_W = 4;
__global__ __launch_bounds__(64 * CF_W) void k_centroid_frags(const float *cen, int d, int k, uint32_t ctiles, int ks,
                                                              float sigma, uint4 *cfrag, uint32_t *cmax_bits,
                                                              float *caos, float2 *cfix, float *cnorm, float *cdn) {
    __shared__ double pn[CF_W][64], pd[CF_W][64];
    const uint32_t total = ctiles * 32;
    const int ld = aos_ld(d);
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int per = (ld / 2 + CF_W - 1) / CF_W * 2;  // dimensions per wave: whole cfix pairs
    const int c0 = w * per, c1 = min(ld, c0 + per);
    float mymax = 0.f, mydmax = 0.f;
    for (uint32_t rb = blockIdx.x; rb * 64 < total; rb += gridDim.x) {
        const uint32_t r = rb * 64 + lane;
        const bool live = r < total;
        const bool valid = live && r < (uint32_t)k;
        double nn = 0, dd = 0;
        if (valid) {
            // k_fixrow layout: [tile][lane-half][dim pair][16 rows] float2, so the 16 lanes of a
            // point read one whole 128-byte line per dimension pair
            const uint32_t row = r & 31, hh = (row >> 2) & 1, r16 = (row & 3) | ((row >> 3) << 2);
            for (int c = c0; c < c1; c += 2) {
                const float a = c < d ? cen[(uint64_t)c * k + r] : 0.0f;
                const float b = c + 1 < d ? cen[(uint64_t)(c + 1) * k + r] : 0.0f;
                caos[(uint64_t)r * ld + c] = a;
                caos[(uint64_t)r * ld + c + 1] = b;
                cfix[(((uint64_t)(r >> 5) * 2 + hh) * (ld / 2) + c / 2) * 16 + r16] = make_float2(a, b);
            }
            for (int c = c0; c < min(c1, d); ++c) {
                const float f = cen[(uint64_t)c * k + r] * sigma;
                const double x = (double)f, e = x - (double)h_val(h_bits(f));
                nn += x * x;
                dd += e * e;
            }
        }
        pn[w][lane] = nn;
        pd[w][lane] = dd;
        __syncthreads();
        nn = ((pn[0][lane] + pn[1][lane]) + pn[2][lane]) + pn[3][lane];
        dd = ((pd[0][lane] + pd[1][lane]) + pd[2][lane]) + pd[3][lane];
        __syncthreads();  // the next row block's partials overwrite these
        static_assert(CF_W == 4, "the fixed-order sum above");
        if (!live || w >= ks) continue;
        uint16_t n1, n2, n3;
        if (valid) {
            n1 = h_bits((float)nn);
            const double r1 = nn - (double)h_val(n1);
            n2 = h_bits((float)r1);
            const double r2 = r1 - (double)h_val(n2);
            n3 = h_bits((float)r2);
            if (w == 0) {
                const float nr = (float)(__builtin_sqrt(nn) * (1.0 + 1e-6));
                const float dr = (float)(__builtin_sqrt(dd) * (1.0 + 1e-6));
                mymax = fmaxf(mymax, nr);
                mydmax = fmaxf(mydmax, dr);
                cnorm[r] = nr;
                cdn[r] = dr;
            }
        } else {
            if (w == 0) {
                cnorm[r] = 0.0f;  // padding row: never the best
                cdn[r] = 0.0f;
            }
            n1 = h_bits(60000.0f);  // padding: score ~6e4 >> any real score (< 200)
            n2 = n3 = 0;
        }
        const int s = w;
        const uint32_t t = r >> 5, row = r & 31;
        for (int h = 0; h < 2; ++h) {
            uint16_t e[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int kk = 16 * s + 8 * h + j;
                uint16_t bits = 0;
                if (kk < d) bits = valid ? h_bits(cen[(uint64_t)kk * k + r] * sigma) : (uint16_t)0;
                else if (kk == d) bits = n1;
                else if (kk == d + 1) bits = n2;
                else if (kk == d + 2) bits = n3;
                e[j] = bits;
            }
            uint4 v;
            v.x = e[0] | ((uint32_t)e[1] << 16);
            v.y = e[2] | ((uint32_t)e[3] << 16);
            v.z = e[4] | ((uint32_t)e[5] << 16);
            v.w = e[6] | ((uint32_t)e[7] << 16);
            cfrag[((uint64_t)t * ks + s) * 64 + h * 32 + row] = v;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        mymax = fmaxf(mymax, __shfl_xor(mymax, o, 64));
        mydmax = fmaxf(mydmax, __shfl_xor(mydmax, o, 64));
    }
    if (lane == 0 && w == 0) {
        atomicMax(cmax_bits, __builtin_bit_cast(uint32_t, mymax));  // non-negative floats: bit order
        atomicMax(cmax_bits + 1, __builtin_bit_cast(uint32_t, mydmax));
    }
}

// ---- the MFMA sweep -------------------------------------------------------------
// MODE 0: main assign (top-3 of tile minima; decided / pair / ambiguous)
// MODE 1: collect candidates of ambiguous points (score <= thr)
//
// Software pipeline over "slots" (one centroid tile x one point tile = KS MFMAs): the
// epilogue of the previous slot is cut into KS slices, slice s issued right behind
// MFMA s of this slot and fenced with sched_barrier, so each MFMA's 32 cycles on the
// matrix pipe cover ~10 VALU ops of the same wave.  Occupancy is 3 waves per SIMD (160 VGPRs:
// B fragments 48, score buffers 64, A ping-pong 24, top-3 state; 48 KiB of LDS per workgroup).
template <int KS, int MODE>
__global__ __launch_bounds__(WG) void k_sweep(const uint4 *__restrict__ pfrag, uint32_t ntiles, uint32_t npts,
                                               const uint4 *__restrict__ cfrag, uint32_t ctiles,
                                               const float *__restrict__ pnorm, const float *__restrict__ pdn,
                                               const uint32_t *__restrict__ cmax_bits, const float *__restrict__ chalf,
                                               const float *__restrict__ chalf_d, const float *__restrict__ ntab,
                                               const Bound bnd, uint32_t *__restrict__ labels,
                                               float *__restrict__ thr, uint32_t *__restrict__ amb, State *st,
                                               uint32_t *__restrict__ cand_cnt, uint32_t *__restrict__ cand,
                                               uint32_t cand_cap,
                                               uint32_t *__restrict__ pair_pts, uint2 *__restrict__ pair_codes,
                                               uint32_t *__restrict__ code_hist) {
    constexpr int STAGE_U4 = CT_STAGE * KS * 64;  // uint4 per stage
    constexpr int PER_THREAD = (STAGE_U4 + WG - 1) / WG;
    static_assert(STAGE_U4 % 64 == 0, "a stage is whole wave-instructions");
    __shared__ uint4 lds[2][STAGE_U4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
    const uint32_t tile0 = (blockIdx.x * NW + w) * PT;

    f16x8 b[PT][KS];
#pragma unroll
    for (int t = 0; t < PT; ++t) {
        const uint32_t tt = tile0 + t;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            uint4 q = (tt < ntiles) ? pfrag[((uint64_t)tt * KS + s) * 64 + lane] : make_uint4(0, 0, 0, 0);
            b[t][s] = __builtin_bit_cast(f16x8, q);
        }
    }
    // -inf the compiler cannot see: med3(x, s, ninf) = min(x, s) stays one v_med3 instead of
    // being folded into v_min plus two NaN canonicalisations
    float ninf;
    asm volatile("v_mov_b32 %0, 0xff800000" : "=v"(ninf));
    // per point tile: top-3 of the keyed tile minima seen by this lane-half (key = the tile
    // minimum with the tile index in its low kbits mantissa bits)
    float m1[PT], m2[PT], m3[PT], th[PT];
    bool full[PT];  // MODE 1: this lane saw its point's candidate list overflow
    const uint32_t kbits = ctiles > 1 ? 32u - (uint32_t)__builtin_clz(ctiles - 1) : 0u;
    const uint32_t kmask = (1u << kbits) - 1u;
    uint32_t kmask_v;  // in a VGPR: v_bfi_b32 takes one scalar operand (the tile index)
    asm volatile("v_mov_b32 %0, %1" : "=v"(kmask_v) : "s"(kmask));
#pragma unroll
    for (int t = 0; t < PT; ++t) {
        m1[t] = __builtin_inff();
        m2[t] = __builtin_inff();
        m3[t] = __builtin_inff();
        th[t] = -__builtin_inff();
        full[t] = false;
        if (MODE == 1) {
            const uint32_t slot = (tile0 + t) * 32 + (lane & 31);
            if (slot < npts) th[t] = thr[slot];
        }
    }

    // slice q of the epilogue of scores sc (point tile t, centroid tile ctile): the minimum
    // of the lane-half's 16 rows (v_min3 tree), then, in the last slice, the running top-3
    // of tile minima.  Two rows of one tile never compete here: k_fixrow / k_fixpair settle
    // the winning tile-halves' rows with the exact distance.
    float mn = 0.f;
    auto slice = [&](const f32x16 &sc, int t, uint32_t ctile, auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr int r0 = q * 16 / KS, r1 = (q + 1) * 16 / KS;
        if (q == 0) mn = sc[0];
#pragma unroll
        for (int r = (q == 0 ? 1 : r0); r < r1; ++r) mn = fminf(mn, sc[r]);
        if (q == KS - 1) {
            if (MODE == 0) {
                // branch-free top-3: the tile index rides in the key's low kbits bits (v_bfi;
                // |key - mn| < 2^kbits ulp, added to the decision window), two v_med3 + one v_min
                uint32_t kb;
                asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(kb) : "v"(kmask_v), "s"(ctile), "v"(mn));
                const float key = __builtin_bit_cast(float, kb);
                m3[t] = __builtin_amdgcn_fmed3f(m2[t], m3[t], key);
                m2[t] = __builtin_amdgcn_fmed3f(m1[t], m2[t], key);
                m1[t] = fminf(m1[t], key);
            } else if (mn <= th[t] && !full[t]) {
                // candidates are rare (a handful of the K centroids per point); once the point's
                // list has overflowed (coinciding centroids: thousands of candidates) this lane
                // stops counting -- k_exact sends an overflowed point to the KdTree walk
                const uint32_t slot = (tile0 + t) * 32 + (lane & 31);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    if (sc[r] <= th[t] && !full[t]) {
                        const uint32_t ci = ctile * 32 + 4 * h + (r & 3) + 8 * (r >> 2);
                        const uint32_t pos = atomicAdd(&cand_cnt[slot], 1u);
                        if (pos < cand_cap) cand[(uint64_t)slot * cand_cap + pos] = ci;
                        else full[t] = true;
                    }
                }
            }
        }
    };

    // ctiles is a multiple of CT_STAGE (the tail is padded with never-winning rows)
    const uint32_t nstages = ctiles / CT_STAGE;
    // MODE 1 splits the centroid stages over gridDim.y workgroups (few ambiguous points:
    // each split sweeps part of the palette, the candidate lists are filled atomically)
    const uint32_t sg_begin = MODE == 1 ? (uint32_t)((uint64_t)blockIdx.y * nstages / gridDim.y) : 0u;
    const uint32_t sg_end = MODE == 1 ? (uint32_t)((uint64_t)(blockIdx.y + 1) * nstages / gridDim.y) : nstages;
    // centroid stages move global -> LDS by DMA (global_load_lds_dwordx4: no VGPR staging,
    // one wave-instruction fills 1 KiB at a wave-uniform base + 16 B per lane)
    const uint32_t wbase = __builtin_amdgcn_readfirstlane(w) * 64;
    auto stage_in = [&](int buf, uint32_t sg_) {
        const uint4 *src = cfrag + (uint64_t)sg_ * STAGE_U4 + threadIdx.x;
#pragma unroll
        for (int q = 0; q < PER_THREAD; ++q)
            if (STAGE_U4 % WG == 0 || wbase + q * WG < (uint32_t)STAGE_U4)
                __builtin_amdgcn_global_load_lds(src + q * WG,
                                                 (__attribute__((address_space(3))) void *)&lds[buf][wbase + q * WG],
                                                 16, 0, 0);
    };
    stage_in(0, sg_begin);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // one score buffer per point tile: slot t of a centroid tile writes buf[t] while the
    // epilogue drains buf[(t + 1) % PT], written PT - 1 slots earlier -- long enough for
    // the MFMA results to have landed, so the VALU never waits on the matrix pipe
    static_assert(PT == 4, "the score-buffer rotation assumes 4 point tiles per wave");
    f32x16 buf[PT];
#pragma unroll
    for (int t = 0; t < PT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) buf[t][r] = 0x1p+120f;  // slots before the first: finite keys, never kept
    uint32_t tile_prev = 0;  // centroid tile of the previous ct iteration
    for (uint32_t sg = sg_begin; sg < sg_end; ++sg) {
        const int cur = (sg - sg_begin) & 1;
        // the other buffer was last read in stage sg - 1, which ended with a barrier
        if (sg + 1 < sg_end) stage_in(cur ^ 1, sg + 1);
        // A fragments ping-pong between two register sets: tile ct + 1 is read from LDS while
        // tile ct's MFMAs run (the read at the stage's last tile re-reads it, unused)
        f16x8 a0[KS], a1[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) a0[s] = __builtin_bit_cast(f16x8, lds[cur][s * 64 + lane]);
        auto tile_step = [&](uint32_t ct, f16x8 (&a)[KS], f16x8 (&an)[KS]) {
            const uint32_t tile_cur = sg * CT_STAGE + ct;
            const uint32_t ctn = (ct + 1 < (uint32_t)CT_STAGE) ? ct + 1 : ct;
#pragma unroll
            for (int s = 0; s < KS; ++s) an[s] = __builtin_bit_cast(f16x8, lds[cur][(ctn * KS + s) * 64 + lane]);
            static_for<PT>([&](auto tc_) {
                constexpr int t = decltype(tc_)::value;
                constexpr int td = (t + 1) % PT;  // point tile whose scores drain in this slot
                const uint32_t tile_d = (td > t) ? tile_prev : tile_cur;
                f32x16 acc = {};
                static_for<KS>([&](auto sc_) {
                    constexpr int s = decltype(sc_)::value;
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[s], b[t][s], acc, 0, 0, 0);
                    slice(buf[td], td, tile_d, sc_);
                    __builtin_amdgcn_sched_barrier(0);
                });
                buf[t] = acc;
            });
            tile_prev = tile_cur;
        };
        static_assert(CT_STAGE % 2 == 0, "ping-pong over pairs of centroid tiles");
#pragma unroll 1
        for (uint32_t ct = 0; ct < (uint32_t)CT_STAGE; ct += 2) {
            tile_step(ct, a0, a1);
            tile_step(ct + 1, a1, a0);
        }
        if (sg + 1 < sg_end) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
    }
    // drain the last centroid tile's slots 1..PT-1 (slot 0 drained in slot PT-1)
    static_for<PT - 1>([&](auto tc_) {
        constexpr int td = decltype(tc_)::value + 1;
        static_for<KS>([&](auto sc_) { slice(buf[td], td, tile_prev, sc_); });
    });
    if (MODE == 1) return;

    const float cm = __builtin_bit_cast(float, cmax_bits[0]);
    const float ntab_scale = cm > 0.f ? (float)NTAB / cm : 0.f;
#pragma unroll
    for (int t = 0; t < PT; ++t) {
        // merge the two lane-halves' top-3 (sorted) into the point's top-3; codes =
        // (tile, lane-half) of the best two
        const float a1 = m1[t], a2 = m2[t], a3 = m3[t];
        const float b1 = __shfl_xor(a1, 32, 64), b2 = __shfl_xor(a2, 32, 64), b3 = __shfl_xor(a3, 32, 64);
        const uint32_t ca1 = (__builtin_bit_cast(uint32_t, a1) & kmask) * 2u + (uint32_t)h;
        const uint32_t ca2 = (__builtin_bit_cast(uint32_t, a2) & kmask) * 2u + (uint32_t)h;
        const uint32_t cb1 = __shfl_xor(ca1, 32, 64), cb2 = __shfl_xor(ca2, 32, 64);
        const float nm1 = fminf(a1, b1);
        const float nm2 = fminf(fmaxf(a1, b1), fminf(a2, b2));
        const float nm3 = fminf(fminf(a3, b3), fminf(fmaxf(a2, b1), fmaxf(a1, b2)));
        const uint32_t code1 = (a1 <= b1) ? ca1 : cb1;
        const uint32_t code2 = (a1 <= b1) ? ((a2 <= b1) ? ca2 : cb1) : ((b2 < a1) ? cb2 : ca1);
        const uint32_t p = (tile0 + t) * 32 + (lane & 31);
        bool is_amb = false, is_pair = false;
        if (h == 0 && p < npts) {
            // keys differ from the tile minima by < 2^kbits ulp <= |key| 2^(kbits - 23) (+ one
            // denormal ulp); 2^-20 |key| on top covers the f32 roundings of the window sums
            const float kr = __builtin_ldexpf(1.0f, (int)kbits - 23) * 1.01f + 0x1p-20f, ka = 0x1p-126f;
            const float e1 = __builtin_fabsf(nm1) * kr + ka;
            const float pn = pnorm[p], dp = pdn[p];
            const float W = wbound_r(bnd, pn, dp, chalf[code1], chalf_d[code1], cm, ntab_scale, ntab, nm1 + e1);
            if (nm2 > nm1 + W + e1 + (__builtin_fabsf(nm2) * kr + ka)) {
                labels[p] = code1;  // k_fixrow turns the code into the centroid index
                if (code_hist) atomicAdd(&code_hist[code1], 1u);  // the decided points' grouping counts
            } else if (nm3 > nm1 + W + e1 + (__builtin_fabsf(nm3) * kr + ka)) {
                // every candidate lies in the two best tile-halves.  Only the second one competes
                // with the first, so its own largest norm bounds its rows' error instead of the
                // palette's (chalf[code2] <= cm): often that already decides the point
                const float W2 = wbound_pair(bnd, pn, dp, chalf[code1], chalf_d[code1], chalf[code2], chalf_d[code2]);
                if (nm2 > nm1 + W2 + e1 + (__builtin_fabsf(nm2) * kr + ka)) {
                    labels[p] = code1;
                    if (code_hist) atomicAdd(&code_hist[code1], 1u);
                } else {
                    is_pair = true;
                    labels[p] = 0xfffffffeu;
                }
            } else {
                is_amb = true;
                labels[p] = 0xffffffffu;
                thr[p] = nm1 + e1 + W;
            }
        }
        const uint64_t pmask = __ballot(is_pair);
        if (pmask) {
            uint32_t base = 0;
            const int leader = __builtin_ctzll(pmask);
            if (lane == leader) base = atomicAdd(&st->pairs, (uint32_t)__popcll(pmask));
            base = __shfl(base, leader, 64);
            if (is_pair) {
                const uint32_t i = base + __popcll(pmask & ((1ull << lane) - 1));
                pair_pts[i] = p;
                pair_codes[i] = make_uint2(code1, code2);
            }
        }
        const uint64_t mask = __ballot(is_amb);
        if (mask) {
            uint32_t base = 0;
            const int leader = __builtin_ctzll(mask);
            if (lane == leader) base = atomicAdd(&st->amb, (uint32_t)__popcll(mask));
            base = __shfl(base, leader, 64);
            if (is_amb) amb[base + __popcll(mask & ((1ull << lane) - 1))] = p;
        }
    }
}

// gather the fragments / thresholds of ambiguous points into compact tiles
__global__ __launch_bounds__(256) void k_gather_amb(const uint4 *__restrict__ pfrag, const uint32_t *__restrict__ amb,
                                                    const float *__restrict__ thr_p, uint32_t namb, int ks,
                                                    uint4 *__restrict__ afrag, float *__restrict__ thr_slot,
                                                    uint32_t *__restrict__ cand_cnt) {
    const uint32_t total = (namb + 31) / 32 * 32;
    for (uint32_t a = blockIdx.x * blockDim.x + threadIdx.x; a < total; a += gridDim.x * blockDim.x) {
        const bool valid = a < namb;
        const uint32_t p = valid ? amb[a] : 0u;
        const uint32_t pt = p >> 5, pc = p & 31, at = a >> 5, ac = a & 31;
        for (int s = 0; s < ks; ++s)
            for (int h = 0; h < 2; ++h)
                afrag[((uint64_t)at * ks + s) * 64 + h * 32 + ac] =
                    valid ? pfrag[((uint64_t)pt * ks + s) * 64 + h * 32 + pc] : make_uint4(0, 0, 0, 0);
        thr_slot[a] = valid ? thr_p[p] : -__builtin_inff();
        cand_cnt[a] = 0;
    }
}

// kd-tree.ts:26-35 distance (c - p per dimension, sequential f64 sum) of two
// zero-padded AoS rows; the padding adds +0 to a non-negative sum, so the result is
// the reference's for the first d dimensions
__device__ inline double ref_dist(const float *__restrict__ crow, const float *__restrict__ prow, int ld) {
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

// decided points: the sweep left (tile, lane-half) of the minimum in labels[p]; every
// other tile's rows score above m1 + W_p, so their reference distances exceed that of
// the best row, and the argmin lies among this lane-half's 16 rows.  16 lanes per point
// (one row each) screen with an f32 distance and a rigorous bound that covers both the
// f32 evaluation and the reference's f64 one: when exactly one row's interval reaches
// the lowest upper end, it is the reference's answer.  Otherwise the candidate rows take
// the exact f64 distance of kd-tree.ts:26-35; a unique minimum decides, an exact tie
// goes to the KdTree walk (kd_resolve_ties).
// G lanes per point (16 rows of one tile-half, or 32 rows of two), lane r scoring row
// r % 16 of tile-half code(r / 16)
// centroid index of row rr (0..15) of tile-half `code` (the MFMA C/D row layout)
__device__ inline uint32_t code_row(uint32_t code, int rr) {
    return (code >> 1) * 32 + 4 * (code & 1) + (rr & 3) + 8 * (rr >> 2);
}

// the group's decision (every lane of the group holds it): the label, and whether it is an
// exact tie left to the KdTree walk (the label then provisional)
struct FixOut {
    uint32_t label;
    bool tie;
};
template <int G>
__device__ inline FixOut fix_decide(float s, bool valid, uint32_t c, int d, const float *__restrict__ caos,
                                    const float *__restrict__ prow, uint64_t p, int r, uint32_t *__restrict__ labels,
                                    uint32_t *__restrict__ ties, State *st);

// all-reduce over a 16-lane DPP row (every lane of the row active): quad_perm xor 1, xor 2,
// then row_ror 4 and 8 -- DPP moves folded into the VALU op, no LDS round trips
template <int CTRL>
__device__ inline uint32_t dpp_u(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ inline float dpp_f(float x) {
    return __builtin_bit_cast(float, dpp_u<CTRL>(__builtin_bit_cast(uint32_t, x)));
}
__device__ inline float row16_min(float v) {
    v = fminf(v, dpp_f<0xB1>(v));
    v = fminf(v, dpp_f<0x4E>(v));
    v = fminf(v, dpp_f<0x124>(v));
    return fminf(v, dpp_f<0x128>(v));
}
__device__ inline uint32_t row16_umin(uint32_t v) {
    v = min(v, dpp_u<0xB1>(v));
    v = min(v, dpp_u<0x4E>(v));
    v = min(v, dpp_u<0x124>(v));
    return min(v, dpp_u<0x128>(v));
}
__device__ inline uint32_t row16_sum(uint32_t v) {
    v += dpp_u<0xB1>(v);
    v += dpp_u<0x4E>(v);
    v += dpp_u<0x124>(v);
    return v + dpp_u<0x128>(v);
}

template <int G>
__device__ inline void fix_group(const float *__restrict__ aos, int d, const float2 *__restrict__ cfix,
                                 const float *__restrict__ caos, int k, uint64_t p, int r, uint32_t code,
                                 uint32_t *__restrict__ labels, uint32_t *__restrict__ ties, State *st) {
    const int ld = aos_ld(d);
    const int rr = r & 15;
    const uint32_t c = code_row(code, rr);
    const bool valid = c < (uint32_t)k;
    const float *prow = aos + p * ld;
    // f32 screen: |s - T| <= (d + 2) u T for fma accumulation of fl(c - p)^2 (u = 2^-24), plus
    // underflow; the reference's f64 error is far below the (d + 4) u margin used
    float s = 0.f;
    if (valid) {
        // padded dimensions hold 0 in both rows: they add +0
        const float4 *p4 = reinterpret_cast<const float4 *>(prow);
        const float2 *crow = cfix + (uint64_t)(code >> 1) * 2 * (ld / 2) * 16 + (uint64_t)(code & 1) * (ld / 2) * 16 + rr;
        for (int q = 0; q < ld / 4; ++q) {
            const float4 pv = p4[q];
            const float2 c0 = crow[(2 * q) * 16], c1 = crow[(2 * q + 1) * 16];
            float v = c0.x - pv.x;
            s = __builtin_fmaf(v, v, s);
            v = c0.y - pv.y;
            s = __builtin_fmaf(v, v, s);
            v = c1.x - pv.z;
            s = __builtin_fmaf(v, v, s);
            v = c1.y - pv.w;
            s = __builtin_fmaf(v, v, s);
        }
    }
    fix_decide<G>(s, valid, c, d, caos, prow, p, r, labels, ties, st);
}

// the decision of a G-lane group from each lane's f32 screen s of row c: a unique interval
// minimum decides; otherwise the exact f64 distances of the surviving rows
template <int G>
__device__ inline FixOut fix_decide(float s, bool valid, uint32_t c, int d, const float *__restrict__ caos,
                                    const float *__restrict__ prow, uint64_t p, int r, uint32_t *__restrict__ labels,
                                    uint32_t *__restrict__ ties, State *st) {
    const int ld = aos_ld(d);
    // the screen's error: (d + 2) u T for any summation order of the d non-negative terms
    const float rel = (float)(d + 4) * 0x1p-24f, ab = (float)(d + 2) * 0x1p-126f;
    const float lo = valid ? s - (s * rel + ab) : __builtin_inff();
    const float hi = valid ? s + (s * rel + ab) : __builtin_inff();
    float mh = hi;
    if (G == 16) {
        mh = row16_min(mh);
    } else if (G == 32) {
        mh = row16_min(mh);
        mh = fminf(mh, __shfl_xor(mh, 16, 64));
    } else {
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) mh = fminf(mh, __shfl_xor(mh, o, 64));
    }
    bool cand = valid && lo <= mh;  // NaN/inf screens fall through to the exact path
    uint32_t ncand = cand ? 1u : 0u;
    if (G == 16) {
        ncand = row16_sum(ncand);
    } else if (G == 32) {
        ncand = row16_sum(ncand);
        ncand += __shfl_xor(ncand, 16, 64);
    } else {
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) ncand += __shfl_xor(ncand, o, 64);
    }
    if (ncand == 1) {
        uint32_t w = cand ? c : 0xffffffffu;
        if (G == 16) {
            w = row16_umin(w);
        } else if (G == 32) {
            w = row16_umin(w);
            w = min(w, __shfl_xor(w, 16, 64));
        } else {
#pragma unroll
            for (int o = G / 2; o > 0; o >>= 1) w = min(w, __shfl_xor(w, o, 64));
        }
        if (r == 0) labels[p] = w;
        return FixOut{w, false};
    }
    if (ncand == 0) cand = valid;
    const double mine = cand ? ref_dist(caos + (uint64_t)c * ld, prow, ld) : __builtin_inf();
    double best = mine;
    uint32_t bidx = c;
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) {
        const double ob = __shfl_xor(best, o, 64);
        const uint32_t oi = __shfl_xor(bidx, o, 64);
        if (ob < best || (ob == best && oi < bidx)) {
            best = ob;
            bidx = oi;
        }
    }
    const uint32_t eq = (cand && mine == best) ? 1u : 0u;
    uint32_t cnt = eq;
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if (r == 0) {
        labels[p] = bidx;  // provisional on a tie; the KdTree pass decides
        if (cnt > 1) ties[atomicAdd(&st->ties, 1u)] = (uint32_t)p;
    }
    return FixOut{bidx, cnt > 1};
}

// decided points (one tile-half): 16 lanes per point
__global__ __launch_bounds__(256) void k_fixrow(const float *__restrict__ aos, int d, const float2 *__restrict__ cfix,
                                                const float *__restrict__ caos, int k, uint32_t n,
                                                uint32_t *__restrict__ labels, uint32_t *__restrict__ ties,
                                                State *st) {
    const uint64_t p = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
    if (p >= n) return;  // uniform per 16-lane group
    const uint32_t code = labels[p];
    if (code >= 0xfffffffeu) return;  // pair (k_fixpair) or ambiguous (k_exact)
    fix_group<16>(aos, d, cfix, caos, k, p, threadIdx.x & 15, code, labels, ties, st);
}

// pair points (two tile-halves): 32 lanes per point
__global__ __launch_bounds__(256) void k_fixpair(const float *__restrict__ aos, int d, const float2 *__restrict__ cfix,
                                                 const float *__restrict__ caos, int k,
                                                 const uint32_t *__restrict__ pair_pts,
                                                 const uint2 *__restrict__ pair_codes, uint32_t npairs,
                                                 uint32_t *__restrict__ labels, uint32_t *__restrict__ ties,
                                                 State *st) {
    const uint32_t i = (blockIdx.x * 256 + threadIdx.x) >> 5;
    if (i >= npairs) return;  // uniform per 32-lane group
    const int r = threadIdx.x & 31;
    const uint2 cc = pair_codes[i];
    fix_group<32>(aos, d, cfix, caos, k, pair_pts[i], r, r < 16 ? cc.x : cc.y, labels, ties, st);
}

// ---- decided points grouped by tile-half ------------------------------------------
// At K = 65,536 there are 4,096 tile-halves and ~2,000 decided points per half.  A
// counting sort groups the points by their half (counts from the sweep, scan, k_code_scatter; the
// order inside a group is immaterial), then k_fixrow_b keeps each lane's centroid row in
// VGPRs across a run of points of one half: centroid rows are read once per run instead of
// 3 KiB per point from L2.
constexpr int FB_MAX_CODES = 8192;  // LDS histogram limit (2 x 4,096 tiles = K <= 131,072)
constexpr int FB_TILE = 4096;        // points per k_code_scatter round (16 per thread)
constexpr int FB_RUN = 32;           // consecutive grouped points per 16-lane group

// cursor = exclusive scan of the histogram; each round ranks its points per code in LDS,
// reserves one range per code with a global atomic, and writes the point indices
// G = uint2: (point, code) pairs (k_fixrow_b); G = uint32_t: the point alone (the fused fix-up's
// slices know their code): half the scattered bytes
template <typename G>
__global__ __launch_bounds__(256) void k_code_scatter(const uint32_t *__restrict__ labels, uint32_t n, uint32_t ncodes,
                                                      uint32_t *__restrict__ cursor, G *__restrict__ grouped) {
    __shared__ uint32_t h[FB_MAX_CODES];
    constexpr int PER = FB_TILE / 256;
    for (uint32_t base = blockIdx.x * FB_TILE; base < n; base += gridDim.x * FB_TILE) {
        for (uint32_t i = threadIdx.x; i < ncodes; i += 256) h[i] = 0;
        __syncthreads();
        uint32_t code[PER], rank[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const uint32_t p = base + j * 256 + threadIdx.x;
            code[j] = p < n ? labels[p] : 0xffffffffu;
            rank[j] = code[j] < ncodes ? atomicAdd(&h[code[j]], 1u) : 0u;
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < ncodes; i += 256)
            if (h[i]) h[i] = atomicAdd(&cursor[i], h[i]);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PER; ++j)
            if (code[j] < ncodes) {
                if constexpr (sizeof(G) == 8)
                    grouped[h[code[j]] + rank[j]] = make_uint2(base + j * 256 + threadIdx.x, code[j]);
                else
                    grouped[h[code[j]] + rank[j]] = base + j * 256 + threadIdx.x;
            }
        __syncthreads();
    }
}

// the same grouping with one reservation per code per workgroup: each workgroup takes a
// contiguous run of ~n / gridDim.x points, counts it per code in LDS, reserves each code's range
// with one global atomic (device-scope atomics cross the XCDs: their number, workgroups x codes
// met, is what k_code_scatter pays per 4,096-point round), then reads the run's codes again and
// places each point at the LDS cursor of its code
template <typename G>
__global__ __launch_bounds__(256) void k_code_scatter_run(const uint32_t *__restrict__ labels, uint32_t n,
                                                          uint32_t ncodes, uint32_t *__restrict__ cursor,
                                                          G *__restrict__ grouped) {
    __shared__ uint32_t h[FB_MAX_CODES];
    // runs of a multiple of 4 points: 16-byte label loads, 4 x U per thread in flight
    const uint32_t per = ((n + gridDim.x - 1) / gridDim.x + 3) & ~3u;
    const uint32_t lo = min(n, blockIdx.x * per), hi = min(n, lo + per);
    for (uint32_t i = threadIdx.x; i < ncodes; i += 256) h[i] = 0;
    __syncthreads();
    constexpr int U = 4;
    const uint4 *l4 = reinterpret_cast<const uint4 *>(labels);
    uint32_t p = lo + 4 * threadIdx.x;
    for (; p + (U - 1) * 1024 + 3 < hi; p += U * 1024) {
        uint4 c[U];
#pragma unroll
        for (int u = 0; u < U; ++u) c[u] = l4[(p >> 2) + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u)
            for (uint32_t v : {c[u].x, c[u].y, c[u].z, c[u].w})
                if (v < ncodes) atomicAdd(&h[v], 1u);
    }
    for (; p < hi; p += 1024)
        for (uint32_t q = p; q < min(hi, p + 4); ++q) {
            const uint32_t v = labels[q];
            if (v < ncodes) atomicAdd(&h[v], 1u);
        }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < ncodes; i += 256)
        if (h[i]) h[i] = atomicAdd(&cursor[i], h[i]);
    __syncthreads();
    auto put = [&](uint32_t q, uint32_t c) {
        if (c >= ncodes) return;
        const uint32_t at = atomicAdd(&h[c], 1u);
        if constexpr (sizeof(G) == 8) grouped[at] = make_uint2(q, c);
        else grouped[at] = q;
    };
    p = lo + 4 * threadIdx.x;
    for (; p + (U - 1) * 1024 + 3 < hi; p += U * 1024) {
        uint4 c[U];
#pragma unroll
        for (int u = 0; u < U; ++u) c[u] = l4[(p >> 2) + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t q = p + u * 1024;
            put(q, c[u].x);
            put(q + 1, c[u].y);
            put(q + 2, c[u].z);
            put(q + 3, c[u].w);
        }
    }
    for (; p < hi; p += 1024)
        for (uint32_t q = p; q < min(hi, p + 4); ++q) put(q, labels[q]);
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
// a 16-byte load issued where it stands (the compiler would sink it to its use), at an immediate offset
template <int OFF>
__device__ inline void load16_at(f32x4 &dst, const void *src) {
    asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(dst) : "v"(src), "i"(OFF) : "memory");
}
// lane q of a 16-lane DPP row reads x from lane Q of its row (row_newbcast); folded into
// the consuming VALU op (v_sub_f32_dpp)
template <int Q>
__device__ inline float row_bcast(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x150 + Q, 0xf, 0xf, true));
}

// 16 lanes (one DPP row) per point over runs of FB_RUN grouped points; lane rr holds row rr
// of the current tile-half in VGPRs (LD floats, zero padded) and reloads it when the half
// changes.  The run's point indices and codes are loaded up front (lane rr holds points rr
// and 16 + rr) and handed out by shuffles.  A point row is loaded once per group -- lane q
// holds its float4 q -- and broadcast inside the row by DPP, so the vector-memory path
// moves 192 B per point instead of 16 x 192 B; the next point's row is in flight while
// this one is scored.  (c - p)^2 is taken as (p - c)^2: the same rounded square.
template <int LD>
__global__ __launch_bounds__(256) void k_fixrow_b(const float *__restrict__ aos, int d, const float *__restrict__ caos,
                                                  int k, const uint2 *__restrict__ grouped,
                                                  const uint32_t *__restrict__ ndecided,
                                                  uint32_t *__restrict__ labels, uint32_t *__restrict__ ties,
                                                  State *st) {
    static_assert(FB_RUN == 32, "two run slots per lane");
    static_assert(LD / 4 <= 16, "one float4 of the point row per lane");
    const uint32_t nd = *ndecided;
    const uint32_t grp = (blockIdx.x * 256 + threadIdx.x) >> 4;
    const uint32_t j0 = grp * FB_RUN;
    if (j0 >= nd) return;  // uniform per 16-lane group
    const int cnt = (int)min(nd - j0, (uint32_t)FB_RUN);
    const int rr = threadIdx.x & 15;
    const int gl = (threadIdx.x & 63) & ~15;  // first lane of this group in the wave
    // (point, tile-half code) pairs: the codes come with the points, not from labels[] at random
    const uint2 ga = rr < cnt ? grouped[j0 + rr] : make_uint2(0u, 0u);
    const uint2 gb = 16 + rr < cnt ? grouped[j0 + 16 + rr] : make_uint2(0u, 0u);
    const uint32_t pa = ga.x, pb = gb.x, ca = ga.y, cb = gb.y;
    auto point_of = [&](int i) { return (uint32_t)__shfl(i < 16 ? pa : pb, gl + (i & 15), 64); };
    auto code_of = [&](int i) { return (uint32_t)__shfl(i < 16 ? ca : cb, gl + (i & 15), 64); };
    // every lane loads (lanes past LD / 4 repeat a slice nobody broadcasts): no branch around
    // the load, so the wait before the scoring covers only the older loads
    const int sq = rr % (LD / 4);
    auto slice = [&](uint32_t pt) { return reinterpret_cast<const f32x4 *>(aos + (uint64_t)pt * LD)[sq]; };
    float4 row[LD / 4];
    uint32_t have = 0xffffffffu, c = 0;
    bool valid = false;
    uint32_t p = point_of(0);
    f32x4 cur = slice(p);  // native vectors: the wait below ties the next row in place
    for (int i = 0; i < cnt; ++i) {
        const uint32_t code = code_of(i);
        const uint32_t pn = point_of(i + 1 < cnt ? i + 1 : i);
        if (code != have) {  // uniform per group
            have = code;
            c = code_row(code, rr);
            valid = c < (uint32_t)k;
            const float4 *src = reinterpret_cast<const float4 *>(caos + (uint64_t)(valid ? c : 0) * LD);
#pragma unroll
            for (int q = 0; q < LD / 4; ++q) row[q] = src[q];
        }
        // the next point's slice is loaded by hand so the compiler cannot sink the load below
        // the scoring (it would wait for it at the top of the next iteration); the wait
        // before `cur = nxt` covers it
        f32x4 nxt;
        load16_at<0>(nxt, reinterpret_cast<const f32x4 *>(aos + (uint64_t)pn * LD) + sq);
        // differences by DPP-broadcast subtracts (v_sub_f32_dpp), squares accumulated in pairs
        // (v_pk_fma_f32): four chains, the screen bound holds for any summation order
        f32x2 a01 = {0.f, 0.f}, a23 = {0.f, 0.f};
        static_for<LD / 4>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            const f32x2 t01 = {row_bcast<q>(cur.x) - row[q].x, row_bcast<q>(cur.y) - row[q].y};
            const f32x2 t23 = {row_bcast<q>(cur.z) - row[q].z, row_bcast<q>(cur.w) - row[q].w};
            a01 = __builtin_elementwise_fma(t01, t01, a01);
            a23 = __builtin_elementwise_fma(t23, t23, a23);
        });
        fix_decide<16>((a01.x + a01.y) + (a23.x + a23.y), valid, c, d, caos, aos + (uint64_t)p * LD, p, rr, labels,
                       ties, st);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("" : "+v"(nxt));  // tied to the wait: nothing reads the row before it landed
        cur = nxt;
        p = pn;
    }
}

// ---- k_fixrow_b with the update folded in ---------------------------------------------
// calcAverage (k-means.ts:41-63) adds a cluster's members in ascending point order in f64.
// Where every member of a (cluster, dimension) is a multiple of 2^e_min and sum|x| <
// 2^(e_min+53), every partial sum is exact, so the order is immaterial: the fix-up pass, which
// already holds each decided point's row and label, accumulates (sum, sum|x|, e_min, count) per
// cluster and dimension in LDS.  One workgroup takes a slice of one tile-half's decided points
// (that tile-half's 16 clusters: no atomics outside LDS).  The other points (pairs, ambiguous,
// exact ties) are summed by k_nd_combine from a short label sort; clusters failing the
// certificate take the sequential sum over their members in point order (k_nd_seq).
constexpr uint32_t FA_SL = 4096;  // decided points per slice (a workgroup's unit of work)
// a cluster's other members above which k_heavy sums them, and others per k_heavy record
// record (ST_OTHERS_SPLIT / ST_OTHERS_CHUNK: test hooks that send small clusters this way)
uint32_t others_split() {
    const char *e = getenv("ST_OTHERS_SPLIT");  // read per call (tests set it around one call)
    return e ? (uint32_t)std::max(1L, atol(e)) : 8192u;
}
uint32_t others_chunk() {
    const char *e = getenv("ST_OTHERS_CHUNK");
    return e ? (uint32_t)std::max(1L, atol(e)) : 4096u;
}
// accumulator slot of dimension j inside a cluster's LD slots (the layout k_nd_combine reads)
template <int LD>
__host__ __device__ inline int fa_slot(int j) { return (j & 3) * (LD / 4) + (j >> 2); }
constexpr uint32_t OTHER_TIE = 0x80000000u;  // others' value bit: a fix-up tie (also in the slices' range)

// local index (0..15) of centroid c inside its tile-half (code_row's inverse)
__device__ inline uint32_t code_local(uint32_t c) { return (c & 3u) | (((c & 31u) >> 3) << 2); }
__device__ inline uint32_t code_of(uint32_t c) { return (c >> 5) * 2 + ((c >> 2) & 1u); }

// slice offsets of the codes' decided points: soff[c] = sum over codes < c of ceil(hist / FA_SL)
constexpr int FS_T = 1024, FS_CODES = FB_MAX_CODES / FS_T;
// ... and the codes' first positions in the grouped order (cursor: exclusive scan of hist,
// k_code_scatter's start) with their total in *ndec: one workgroup (ncodes <= FB_MAX_CODES)
__global__ __launch_bounds__(FS_T) void k_fa_slices(const uint32_t *__restrict__ hist, uint32_t ncodes,
                                                    uint32_t *__restrict__ soff, uint32_t *__restrict__ cursor,
                                                    uint32_t *__restrict__ ndec) {
    __shared__ uint32_t wsum[FS_T / 64], wsum2[FS_T / 64];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t v[FS_CODES], h[FS_CODES], mine = 0, mine2 = 0;
#pragma unroll
    for (int u = 0; u < FS_CODES; ++u) {
        const uint32_t cd = t * FS_CODES + u;
        h[u] = cd < ncodes ? hist[cd] : 0u;
        v[u] = (h[u] + FA_SL - 1) / FA_SL;
        mine += v[u];
        mine2 += h[u];
    }
    uint32_t incl = mine, incl2 = mine2;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t x = __shfl_up(incl, o, 64), x2 = __shfl_up(incl2, o, 64);
        if (lane >= o) {
            incl += x;
            incl2 += x2;
        }
    }
    if (lane == 63) {
        wsum[w] = incl;
        wsum2[w] = incl2;
    }
    __syncthreads();
    uint32_t o = 0, tot = 0, o2 = 0, tot2 = 0;
    for (int i = 0; i < FS_T / 64; ++i) {
        if (i < w) {
            o += wsum[i];
            o2 += wsum2[i];
        }
        tot += wsum[i];
        tot2 += wsum2[i];
    }
    o += incl - mine;
    o2 += incl2 - mine2;
#pragma unroll
    for (int u = 0; u < FS_CODES; ++u) {
        const uint32_t cd = t * FS_CODES + u;
        if (cd < ncodes) {
            soff[cd] = o;
            cursor[cd] = o2;
        }
        o += v[u];
        o2 += h[u];
    }
    if (t == 0) {
        soff[ncodes] = tot;
        *ndec = tot2;
    }
}

typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
// lane R's value of v, into an SGPR (volatile: read where it stands, not hoisted out of the loop)
template <int R>
__device__ inline float readlane_f(float v) {
    float x;
    asm volatile("v_readlane_b32 %0, %1, %2" : "=s"(x) : "v"(v), "i"(R));
    return x;
}
// one centroid row of LD floats at base + OFF bytes into SGPRs: scalar loads issued and waited for
// where they stand (the compiler would hoist all 16 rows' loads and spill them)
template <int LD, int OFF>
__device__ inline void srow(float (&v)[LD], const float *base) {
    if constexpr (LD == 48) {
        f32x16 t0, t1, t2;
        asm volatile("s_load_dwordx16 %0, %3, %4\n\ts_load_dwordx16 %1, %3, %5\n\ts_load_dwordx16 %2, %3, %6\n\t"
                     "s_waitcnt lgkmcnt(0)"
                     : "=s"(t0), "=s"(t1), "=s"(t2) : "s"(base), "i"(OFF), "i"(OFF + 64), "i"(OFF + 128));
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            v[i] = t0[i];
            v[16 + i] = t1[i];
            v[32 + i] = t2[i];
        }
    } else if constexpr (LD == 24) {
        f32x16 t0;
        f32x8 t1;
        asm volatile("s_load_dwordx16 %0, %2, %3\n\ts_load_dwordx8 %1, %2, %4\n\ts_waitcnt lgkmcnt(0)"
                     : "=s"(t0), "=s"(t1) : "s"(base), "i"(OFF), "i"(OFF + 64));
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = t0[i];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[16 + i] = t1[i];
    } else {
        static_assert(LD == 12, "rows of 12, 24 or 48 floats");
        f32x8 t0;
        f32x4 t1;
        asm volatile("s_load_dwordx8 %0, %2, %3\n\ts_load_dwordx4 %1, %2, %4\n\ts_waitcnt lgkmcnt(0)"
                     : "=s"(t0), "=s"(t1) : "s"(base), "i"(OFF), "i"(OFF + 32));
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = t0[i];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[8 + i] = t1[i];
    }
}
constexpr int FL_WAVES = 4;     // waves per workgroup (one slice's batches shared out)
constexpr int FL_TS = 33;       // LDS transpose stride (floats) of a half batch: conflict-free both ways
template <int LD>
__global__ __launch_bounds__(64 * FL_WAVES) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_fixrow_lp(
    const float *__restrict__ aos, int d, const float *__restrict__ caos, int k, const uint32_t *__restrict__ grouped,
    const uint32_t *__restrict__ hist, const uint32_t *__restrict__ cend, const uint32_t *__restrict__ soff,
    uint32_t ncodes, uint32_t *__restrict__ labels, uint32_t *__restrict__ ties, State *st,
    double *__restrict__ psum, double *__restrict__ pabs, int *__restrict__ pemin, uint32_t *__restrict__ pcnt) {
    constexpr int NQ = LD / 4;
    constexpr int DT = LD == 48 ? 45 : LD == 24 ? 24 : 9;  // dimensions that can be non-zero (3C, C = 15 / 8 / 3)
    __shared__ double S[16 * LD], A[16 * LD];
    __shared__ int E[16 * LD];
    __shared__ uint32_t C[16];
    __shared__ float tr[FL_WAVES][DT * FL_TS];  // a half batch (32 points) in the lane = dimension layout
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: the batch loop is a wave loop
    const uint32_t nsl = soff[ncodes];
    // f32 screen error constants (u = 2^-24): 4 FMA chains of NQ terms + 3 adds for p.c
    // (gamma_{NQ+2} per side, x2 for the factor 2), the subtraction's and |c|^2's roundings; rel:
    // the reference's f64 distance (kd-tree.ts:26-35) against the exact one
    constexpr float u = 0x1p-24f;
    constexpr float e1 = (2.0f * (NQ + 2) + 3.0f) * u * 1.01f, e2 = 2.01f * u, rel = 1.0e-13f;
    const float ab = 64.0f * 0x1p-126f;
    for (uint32_t sl = blockIdx.x; sl < nsl; sl += gridDim.x) {
        uint32_t lo = 0, hi = ncodes;  // the code whose slices hold sl
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (soff[mid] <= sl) lo = mid;
            else hi = mid;
        }
        const uint32_t code = __builtin_amdgcn_readfirstlane(lo);
        const uint32_t b0 = cend[code] - hist[code] + (sl - soff[code]) * FA_SL;
        const uint32_t b1 = min(cend[code], b0 + FA_SL);
        for (int e = threadIdx.x; e < 16 * LD; e += 64 * FL_WAVES) {
            S[e] = 0.0;
            A[e] = 0.0;
            E[e] = 1 << 20;
        }
        if (threadIdx.x < 16) C[threadIdx.x] = 0u;
        // per row: |c|^2 (f32, nearest) and the bound's coefficients, from the f64 norm (lanes 0..15);
        // a row past k (padding of the last tile) reads the tile's first row and scores 3e38 (finite:
        // no inf - inf in the bound), never a candidate
        float rnc = 3.0e38f, rbeta = 0.f, rgam = 0.f;
        {
            const uint32_t c = code_row(code, lane & 15);
            if (lane < 16 && c < (uint32_t)k) {
                const float *cr = caos + (uint64_t)c * LD;
                double nn = 0;
                for (int q = 0; q < LD; ++q) nn += (double)cr[q] * cr[q];
                const float cn = (float)(__builtin_sqrt(nn) * (1.0 + 1e-6));
                rnc = (float)nn;
                rbeta = (e1 + 2.0f * rel) * cn;
                rgam = (e2 + rel) * cn * cn + ab;
            }
        }
        __syncthreads();
        const float *cbase = caos + (uint64_t)code_row(code, 0) * LD;
        const bool allvalid = (code >> 1) * 32 + 32 <= (uint32_t)k;  // every row of the tile below k
        // batches of 64 grouped points per wave: wave wv takes batches wv, wv + FL_WAVES, ...  No
        // software pipeline: four workgroups per CU (16 waves) hide each other's gathers
        const uint32_t nb = (b1 - b0 + 63) / 64;
        uint32_t bi = wv;
        uint32_t pnx = bi < nb ? grouped[min(b0 + bi * 64 + lane, b1 - 1)] : 0u;
        for (; bi < nb; bi += FL_WAVES) {  // uniform per wave
            const bool have = b0 + bi * 64 + lane < b1;
            const uint32_t pcur = pnx;
            f32x4 cur[NQ];
            {
                const f32x4 *src = reinterpret_cast<const f32x4 *>(aos + (uint64_t)pcur * LD);
#pragma unroll
                for (int q = 0; q < NQ; ++q) cur[q] = src[q];
            }
            if (bi + FL_WAVES < nb) pnx = grouped[min(b0 + (bi + FL_WAVES) * 64 + lane, b1 - 1)];  // the next index
            // |p|^2 and the 16 screens
            f32x2 pa = {0.f, 0.f}, pb = {0.f, 0.f};
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const f32x2 x01 = {cur[q].x, cur[q].y}, x23 = {cur[q].z, cur[q].w};
                pa = __builtin_elementwise_fma(x01, x01, pa);
                pb = __builtin_elementwise_fma(x23, x23, pb);
            }
            const float pn = __builtin_sqrtf(((pa.x + pa.y) + (pb.x + pb.y)) * (1.0f + 16.0f * u)) * (1.0f + 4.0f * u);
            const float apn = rel * pn * pn;
            float s[16];
            float mh = __builtin_inff();
            // the tile-half's rows: row r at tile row (r & 3) + 8 (r >> 2) (code_row), constant offsets
            // from one base, loaded into SGPRs one row at a time (srow) right before its 2 x NQ packed
            // FMAs; the per-row constants are read from lanes 0..15 at their use
            static_for<16>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                const float nc = readlane_f<r>(rnc), be = readlane_f<r>(rbeta), ga = readlane_f<r>(rgam);
                float lo_r = 3.0e38f;
                if (allvalid || code_row(code, r) < (uint32_t)k) {  // uniform
                    float cv[LD];
                    srow<LD, ((r & 3) + 8 * (r >> 2)) * LD * 4>(cv, cbase);
                    f32x2 a = {0.f, 0.f}, b = {0.f, 0.f};
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        a = __builtin_elementwise_fma((f32x2){cur[q].x, cur[q].y}, (f32x2){cv[4 * q], cv[4 * q + 1]}, a);
                        b = __builtin_elementwise_fma((f32x2){cur[q].z, cur[q].w}, (f32x2){cv[4 * q + 2], cv[4 * q + 3]}, b);
                    }
                    const float sr = nc - 2.0f * ((a.x + a.y) + (b.x + b.y));
                    const float err = __builtin_fmaf(pn, be, ga + apn) * 1.001f + __builtin_fabsf(sr) * 0x1p-22f;
                    mh = fminf(mh, sr + err);
                    lo_r = sr - err;  // the interval's lower end is all the decision needs from here on
                }
                s[r] = lo_r;
                __builtin_amdgcn_sched_barrier(0);  // one row's SGPRs at a time
            });
            uint32_t cand = 0;
#pragma unroll
            for (int r = 0; r < 16; ++r) cand |= (s[r] <= mh ? 1u : 0u) << r;
            uint32_t wl = 16;  // local winner (16: none -- not this lane's point, or an exact tie)
            if (have) {
                uint32_t wc;
                bool tie = false;
                if (__builtin_popcount(cand) == 1 && allvalid) {
                    wl = __builtin_ctz(cand);
                    wc = code_row(code, (int)wl);
                } else {
                    // the exact reference distances of the candidates (every valid row if none)
                    uint32_t valid = 0;
                    for (int r = 0; r < 16; ++r) valid |= (code_row(code, r) < (uint32_t)k ? 1u : 0u) << r;
                    uint32_t cm = cand & valid;
                    if (!cm) cm = valid;
                    const float *prow = aos + (uint64_t)pcur * LD;  // re-read: nothing hoisted into registers
                    double best = __builtin_inf();
                    uint32_t bl = 16, cnt = 0;
                    for (uint32_t m = cm; m; m &= m - 1) {  // ascending rows = ascending centroid index
                        asm volatile("" ::: "memory");
                        const int r = __builtin_ctz(m);
                        const float *cr = caos + (uint64_t)code_row(code, r) * LD;
                        double l = 0;
                        for (int jd = 0; jd < LD; ++jd) {  // kd-tree.ts:26-35: sequential f64 sum of (c - p)^2
                            const double v = (double)cr[jd] - (double)prow[jd];
                            l += v * v;
                        }
                        if (l < best) {
                            best = l;
                            bl = (uint32_t)r;
                            cnt = 1;
                        } else if (l == best) {
                            ++cnt;
                        }
                    }
                    wc = code_row(code, (int)bl);
                    tie = cnt > 1;
                    wl = tie ? 16u : bl;
                }
                labels[pcur] = wc;  // provisional on a tie; the KdTree pass decides
                if (tie) ties[atomicAdd(&st->ties, 1u)] = pcur;
            }
            // the sums: each half batch's rows through LDS into the lane = dimension layout; per
            // cluster, its members' values in this lane's dimension summed in registers (their lanes
            // from one ballot), then added to the slice's LDS sums once
            float *t = tr[wv];
            const int jd = lane < DT ? lane : DT - 1;
            static_for<2>([&](auto hc) {
                constexpr int hf = decltype(hc)::value;
                if ((lane >> 5) == hf) {
                    const int i = lane & 31;
                    static_for<NQ>([&](auto qc) {
                        constexpr int q = decltype(qc)::value;
                        if (4 * q + 0 < DT) t[(4 * q + 0) * FL_TS + i] = cur[q].x;
                        if (4 * q + 1 < DT) t[(4 * q + 1) * FL_TS + i] = cur[q].y;
                        if (4 * q + 2 < DT) t[(4 * q + 2) * FL_TS + i] = cur[q].z;
                        if (4 * q + 3 < DT) t[(4 * q + 3) * FL_TS + i] = cur[q].w;
                    });
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                static_for<16>([&](auto cc) {
                    constexpr int c = decltype(cc)::value;
                    uint64_t m = __ballot(wl == (uint32_t)c);
                    m = hf ? (m >> 32) : (m & 0xffffffffull);
                    if (m) {  // uniform
                        const uint32_t cnt = (uint32_t)__popcll(m);
                        double sm = 0.0, sa = 0.0;
                        float mn = __builtin_inff();
                        while (m) {
                            const int i = __builtin_ctzll(m);
                            m &= m - 1;
                            const float x = t[jd * FL_TS + i];
                            sm += (double)x;
                            sa += (double)__builtin_fabsf(x);
                            mn = fminf(mn, x != 0.0f ? __builtin_fabsf(x) : __builtin_inff());
                        }
                        if (lane < DT) {  // the padding dimensions add 0 (and no exponent)
                            const int e = c * LD + fa_slot<LD>(lane);
                            atomicAdd(&S[e], sm);
                            atomicAdd(&A[e], sa);
                            if (mn != __builtin_inff()) atomicMin(&E[e], ulp_exp(mn));
                        }
                        if (lane == 0) atomicAdd(&C[c], cnt);
                    }
                });
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            });
        }
        __syncthreads();
        for (int e = threadIdx.x; e < 16 * LD; e += 64 * FL_WAVES) {
            psum[(uint64_t)sl * 16 * LD + e] = S[e];
            pabs[(uint64_t)sl * 16 * LD + e] = A[e];
            pemin[(uint64_t)sl * 16 * LD + e] = E[e];
        }
        if (threadIdx.x < 16) pcnt[(uint64_t)sl * 16 + threadIdx.x] = C[threadIdx.x];
        __syncthreads();
    }
}

// the points the fused fix-up did not sum (pairs, ambiguous, its own exact ties), keyed by
// their final label
__global__ __launch_bounds__(256) void k_others_keys(const uint32_t *__restrict__ pair_pts, uint32_t npair,
                                                     const uint32_t *__restrict__ amb, uint32_t namb,
                                                     const uint32_t *__restrict__ ties, uint32_t nties,
                                                     const uint32_t *__restrict__ labels, uint32_t *__restrict__ keys,
                                                     uint32_t *__restrict__ vals) {
    const uint32_t m = npair + namb + nties;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const uint32_t p = i < npair ? pair_pts[i] : i < npair + namb ? amb[i - npair] : ties[i - npair - namb];
        keys[i] = labels[p];
        vals[i] = i < npair + namb ? p : p | OTHER_TIE;
    }
}

// a cluster's other members (ovals[o0 .. o1), label-sorted; lane = dimension) added in list
// order: the wave loads 64 list entries at once (one per lane) and then up to U member rows in
// flight, each row's index broadcast from its lane -- a cluster holds a handful of others, and
// loading them one list entry, then one row, at a time made each a chain of dependent reads
template <int LD>
__device__ inline void others_sum(const float *__restrict__ aos, const uint32_t *__restrict__ ovals, uint32_t o0,
                                  uint32_t o1, int lane, double &sum, double &sabs, int &emin) {
    constexpr int U = 8;  // member rows in flight
    for (uint32_t b = o0; b < o1; b += 64) {
        const uint32_t m = min(64u, o1 - b);
        const uint32_t mine = (uint32_t)lane < m ? (ovals[b + lane] & ~OTHER_TIE) : 0u;
        for (uint32_t u0 = 0; u0 < m; u0 += U) {
            float v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t row = __shfl(mine, (int)(u0 + u) & 63, 64);
                v[u] = (u0 + u < m && lane < LD) ? aos[(uint64_t)row * LD + lane] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (u0 + u < m) {  // uniform
                    sum += (double)v[u];
                    sabs += (double)__builtin_fabsf(v[u]);
                    if (v[u] != 0.0f) emin = min(emin, ulp_exp(v[u]));
                }
            }
        }
    }
}

// one wave per cluster, lane = dimension: the slices' partials of its tile-half plus its other
// members (ostart / ovals: the label-sorted others); the centroid where every dimension is
// certified, otherwise the cluster is listed for k_nd_seq.  counts[cl] = its members.
template <int LD>
__global__ __launch_bounds__(256) void k_nd_combine(const float *__restrict__ aos, int d, int k,
                                                    const uint32_t *__restrict__ soff,
                                                    const double *__restrict__ psum, const double *__restrict__ pabs,
                                                    const int *__restrict__ pemin, const uint32_t *__restrict__ pcnt,
                                                    const uint32_t *__restrict__ ostart,
                                                    const uint32_t *__restrict__ ovals, float *__restrict__ cen,
                                                    uint32_t *__restrict__ counts, uint32_t *__restrict__ flagged,
                                                    uint32_t *__restrict__ nflagged, uint32_t *__restrict__ heavy,
                                                    uint32_t *__restrict__ nheavy, uint32_t os_split) {
    const int lane = threadIdx.x & 63;
    const uint32_t cl = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (cl >= (uint32_t)k) return;  // uniform per wave
    const uint32_t o0 = ostart[cl], o1 = ostart[cl + 1];
    if (o1 - o0 > os_split) {  // many others: summed over the chip (k_heavy)
        if (lane == 0) heavy[atomicAdd(nheavy, 1u)] = cl;
        return;
    }
    const uint32_t code = code_of(cl), loc = code_local(cl);
    double sum = 0, sabs = 0;
    int emin = 1 << 20;
    uint32_t cnt = 0;
    for (uint32_t sl = soff[code]; sl < soff[code + 1]; ++sl) {
        if (lane < LD) {
            const uint64_t e = (uint64_t)sl * 16 * LD + loc * LD + fa_slot<LD>(lane);
            sum += psum[e];
            sabs += pabs[e];
            emin = min(emin, pemin[e]);
        }
        cnt += pcnt[(uint64_t)sl * 16 + loc];
    }
    others_sum<LD>(aos, ovals, o0, o1, lane, sum, sabs, emin);
    cnt += o1 - o0;
    if (lane == 0) counts[cl] = cnt;
    if (cnt == 0) return;  // empty: re-seeded
    const bool exact = lane >= d || sum_is_exact(sabs, emin);
    if (__ballot(!exact) == 0) {
        if (lane < d) cen[(uint64_t)lane * k + cl] = (float)(sum / (double)cnt);
    } else if (lane == 0) {
        flagged[atomicAdd(nflagged, 1u)] = cl;
    }
}

// the sharded writer's form of k_nd_combine (one segment: the whole shard): the same sums over
// the slices' partials and the other members, written as the (dimension, cluster) partials the
// all-reduce takes (dist_partials' layout [dim][k]) instead of certified centroids
template <int LD>
__global__ __launch_bounds__(256) void k_nd_partials(const float *__restrict__ aos, int d, int k,
                                                     const uint32_t *__restrict__ soff,
                                                     const double *__restrict__ psum, const double *__restrict__ pabs,
                                                     const int *__restrict__ pemin, const uint32_t *__restrict__ pcnt,
                                                     const uint32_t *__restrict__ ostart,
                                                     const uint32_t *__restrict__ ovals, double *__restrict__ sums,
                                                     double *__restrict__ sabs_out, int32_t *__restrict__ emin_out,
                                                     uint32_t *__restrict__ counts, uint32_t *__restrict__ heavy,
                                                     uint32_t *__restrict__ nheavy, uint32_t os_split) {
    const int lane = threadIdx.x & 63;
    const uint32_t cl = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (cl >= (uint32_t)k) return;  // uniform per wave
    if (ostart[cl + 1] - ostart[cl] > os_split) {  // many others: k_heavy
        if (lane == 0) heavy[atomicAdd(nheavy, 1u)] = cl;
        return;
    }
    const uint32_t code = code_of(cl), loc = code_local(cl);
    double sum = 0, sabs = 0;
    int emin = 1 << 20;
    uint32_t cnt = 0;
    for (uint32_t sl = soff[code]; sl < soff[code + 1]; ++sl) {
        if (lane < LD) {
            const uint64_t e = (uint64_t)sl * 16 * LD + loc * LD + fa_slot<LD>(lane);
            sum += psum[e];
            sabs += pabs[e];
            emin = min(emin, pemin[e]);
        }
        cnt += pcnt[(uint64_t)sl * 16 + loc];
    }
    const uint32_t o0 = ostart[cl], o1 = ostart[cl + 1];
    others_sum<LD>(aos, ovals, o0, o1, lane, sum, sabs, emin);
    cnt += o1 - o0;
    if (lane == 0) counts[cl] = cnt;
    if (lane < d) {
        const uint64_t o = (uint64_t)lane * k + cl;
        sums[o] = sum;
        sabs_out[o] = sabs;
        emin_out[o] = emin;
    }
}

// ---- clusters with many other members (others_split()): a cluster of the table's all-zero rows sits
// on a near-tie with another centroid every other iteration, and its millions of pair points were
// one wave's sequential loop inside k_nd_combine (100 ms per update at 10M).  Their others are
// cut into others_chunk()-row chunks summed by the whole chip (sum, sum|x|, smallest ulp exponent per
// dimension), then one wave per such cluster adds its slices' and its chunks' partials.  Under
// the certificate every partial sum is exact, so the order of these additions does not matter;
// a cluster the certificate fails is flagged as in k_nd_combine (the sequential sum over its
// members in point order decides it).
// chunk j of the heavy clusters' others -> (cluster index i in the heavy list, its first chunk);
// the list is short (none, usually; at most m / others_split()): a linear scan
__device__ inline uint32_t heavy_of_chunk(const uint32_t *__restrict__ ostart, const uint32_t *__restrict__ heavy,
                                          uint32_t nh, uint32_t os_chunk, uint32_t j, uint32_t *first) {
    uint32_t o = 0;
    for (uint32_t i = 0; i < nh; ++i) {
        const uint32_t c = (ostart[heavy[i] + 1] - ostart[heavy[i]] + os_chunk - 1) / os_chunk;
        if (j < o + c) {
            *first = o;
            return i;
        }
        o += c;
    }
    *first = o;
    return nh;
}

// One launch: every workgroup sums chunks of the heavy clusters' others (4 waves, lane =
// dimension; record j = (sum, sum|x|, smallest ulp exponent)); the workgroup that finishes last
// then adds, one wave per heavy cluster, its tile-half's slice partials and its chunk records:
// SHARD, the sharded writer's partials (k_nd_partials' outputs), else the certified centroid or
// the flag.  done: zeroed before the launch.  No heavy cluster: every workgroup returns at once.
template <int LD, bool SHARD>
__global__ __launch_bounds__(256) void k_heavy(const float *__restrict__ aos, int d, int k,
                                               const uint32_t *__restrict__ soff, const double *__restrict__ psum,
                                               const double *__restrict__ pabs, const int *__restrict__ pemin,
                                               const uint32_t *__restrict__ pcnt, const uint32_t *__restrict__ ostart,
                                               const uint32_t *__restrict__ ovals, const uint32_t *__restrict__ heavy,
                                               const uint32_t *__restrict__ nheavy, uint32_t *__restrict__ done,
                                               uint32_t os_chunk, double *__restrict__ rsum, double *__restrict__ rabs,
                                               int *__restrict__ remin, float *__restrict__ cen,
                                               uint32_t *__restrict__ counts, uint32_t *__restrict__ flagged,
                                               uint32_t *__restrict__ nflagged, double *__restrict__ sums,
                                               double *__restrict__ sabs_out, int32_t *__restrict__ emin_out) {
    __shared__ double ls[4][64], la[4][64];
    __shared__ int le[4][64];
    __shared__ bool last;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t nh = *nheavy;
    if (nh == 0) return;
    uint32_t total;
    heavy_of_chunk(ostart, heavy, nh, os_chunk, 0xffffffffu, &total);
    for (uint32_t j = blockIdx.x; j < total; j += gridDim.x) {
        uint32_t first;
        const uint32_t cl = heavy[heavy_of_chunk(ostart, heavy, nh, os_chunk, j, &first)];
        const uint32_t c0 = ostart[cl] + (j - first) * os_chunk, c1 = min(ostart[cl + 1], c0 + os_chunk);
        const uint32_t per = (c1 - c0 + 3) / 4;
        const uint32_t a = c0 + min(c1 - c0, w * per), b = c0 + min(c1 - c0, (w + 1) * per);
        double sum = 0, sabs = 0;
        int emin = 1 << 20;
        others_sum<LD>(aos, ovals, a, b, lane, sum, sabs, emin);
        ls[w][lane] = sum;
        la[w][lane] = sabs;
        le[w][lane] = emin;
        __syncthreads();
        if (w == 0) {
            rsum[(uint64_t)j * 64 + lane] = ((ls[0][lane] + ls[1][lane]) + ls[2][lane]) + ls[3][lane];
            rabs[(uint64_t)j * 64 + lane] = ((la[0][lane] + la[1][lane]) + la[2][lane]) + la[3][lane];
            remin[(uint64_t)j * 64 + lane] = min(min(le[0][lane], le[1][lane]), min(le[2][lane], le[3][lane]));
        }
        __syncthreads();
    }
    __threadfence();  // this workgroup's records, before its ticket
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(done, 1u) == gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    __threadfence();  // every other workgroup's records, after the last ticket
    for (uint32_t i = w; i < nh; i += 4) {
        const uint32_t cl = heavy[i], code = code_of(cl), loc = code_local(cl);
        uint32_t j0 = 0;
        for (uint32_t t = 0; t < i; ++t) j0 += (ostart[heavy[t] + 1] - ostart[heavy[t]] + os_chunk - 1) / os_chunk;
        const uint32_t j1 = j0 + (ostart[cl + 1] - ostart[cl] + os_chunk - 1) / os_chunk;
        double sum = 0, sabs = 0;
        int emin = 1 << 20;
        uint32_t cnt = 0;
        for (uint32_t sl = soff[code]; sl < soff[code + 1]; ++sl) {
            if (lane < LD) {
                const uint64_t e = (uint64_t)sl * 16 * LD + loc * LD + fa_slot<LD>(lane);
                sum += psum[e];
                sabs += pabs[e];
                emin = min(emin, pemin[e]);
            }
            cnt += pcnt[(uint64_t)sl * 16 + loc];
        }
        for (uint32_t j = j0; j < j1; ++j) {
            sum += __builtin_nontemporal_load(&rsum[(uint64_t)j * 64 + lane]);
            sabs += __builtin_nontemporal_load(&rabs[(uint64_t)j * 64 + lane]);
            emin = min(emin, __builtin_nontemporal_load(&remin[(uint64_t)j * 64 + lane]));
        }
        cnt += ostart[cl + 1] - ostart[cl];
        if (lane == 0) counts[cl] = cnt;
        if constexpr (SHARD) {
            if (lane < d) {
                const uint64_t o = (uint64_t)lane * k + cl;
                sums[o] = sum;
                sabs_out[o] = sabs;
                emin_out[o] = emin;
            }
        } else {
            const bool exact = lane >= d || sum_is_exact(sabs, emin);
            if (__ballot(!exact) == 0) {
                if (lane < d) cen[(uint64_t)lane * k + cl] = (float)(sum / (double)cnt);
            } else if (lane == 0) {
                flagged[atomicAdd(nflagged, 1u)] = cl;
            }
        }
    }
}

// one workgroup per cluster the certificate fails: its members are the decided points of its
// tile-half's grouped range that carry its label (fix-up ties included, with their final
// label) and its pair / ambiguous points among the label-sorted others; sorted into point
// order (bitonic, LDS), then lane = dimension runs calcAverage's sequential f64 sum.  More
// than NS_CAP members: listed in big (the caller sums those over the member sort).
constexpr uint32_t NS_CAP = 4096;
__global__ __launch_bounds__(256) void k_nd_seq(const float *__restrict__ aos, int d, int k,
                                                const uint32_t *__restrict__ flagged, const uint32_t *__restrict__ nflagged,
                                                const uint32_t *__restrict__ grouped, const uint32_t *__restrict__ hist,
                                                const uint32_t *__restrict__ cend, const uint32_t *__restrict__ labels,
                                                const uint32_t *__restrict__ ostart,
                                                const uint32_t *__restrict__ ovals, float *__restrict__ cen,
                                                uint32_t *__restrict__ big, uint32_t *__restrict__ nbig) {
    __shared__ uint32_t m[NS_CAP];
    __shared__ uint32_t cnt_s;
    const uint32_t nf = *nflagged;
    for (uint32_t f = blockIdx.x; f < nf; f += gridDim.x) {
    const uint32_t cl = flagged[f], code = code_of(cl);
    if (threadIdx.x == 0) cnt_s = 0u;
    __syncthreads();
    auto put = [&](uint32_t p) {
        const uint32_t i = atomicAdd(&cnt_s, 1u);
        if (i < NS_CAP) m[i] = p;
    };
    for (uint32_t i = cend[code] - hist[code] + threadIdx.x; i < cend[code]; i += 256) {
        const uint32_t p = grouped[i];
        if (labels[p] == cl) put(p);
    }
    for (uint32_t j = ostart[cl] + threadIdx.x; j < ostart[cl + 1]; j += 256) {
        const uint32_t v = ovals[j];
        if (!(v & OTHER_TIE)) put(v);
    }
    __syncthreads();
    const uint32_t cnt = cnt_s;
    if (cnt > NS_CAP) {  // summed over the member sort (nd_fused_update)
        if (threadIdx.x == 0) big[atomicAdd(nbig, 1u)] = cl;
        __syncthreads();
        continue;
    }
    uint32_t np2 = 1;
    while (np2 < cnt) np2 <<= 1;
    for (uint32_t i = cnt + threadIdx.x; i < np2; i += 256) m[i] = 0xffffffffu;
    __syncthreads();
    for (uint32_t sz = 2; sz <= np2; sz <<= 1)
        for (uint32_t st = sz >> 1; st > 0; st >>= 1) {
            for (uint32_t i = threadIdx.x; i < np2; i += 256) {
                const uint32_t j = i ^ st;
                if (j > i) {
                    const bool up = (i & sz) == 0;
                    const uint32_t a = m[i], b = m[j];
                    if ((a > b) == up) {
                        m[i] = b;
                        m[j] = a;
                    }
                }
            }
            __syncthreads();
        }
    const int lane = threadIdx.x;
    if (lane < d && cnt) {
        const int ld = aos_ld(d);
        double sum = 0;
        // the member values move 8 at a time (independent loads in flight), the adds stay in
        // point order
        constexpr uint32_t U = 8;
        uint32_t i = 0;
        for (; i + U <= cnt; i += U) {
            float v[U];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) v[u] = aos[(uint64_t)m[i + u] * ld + lane];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) sum += (double)v[u];
        }
        for (; i < cnt; ++i) sum += (double)aos[(uint64_t)m[i] * ld + lane];
        cen[(uint64_t)lane * k + cl] = (float)(sum / (double)cnt);
    }
    __syncthreads();  // m and cnt_s are reused by the next flagged cluster
    }
}

// pair points with the point row broadcast by DPP: lanes 0-15 score the rows of the first
// tile-half, lanes 16-31 the second (two DPP rows); each lane loads one float4 slice of the
// point, rows come from the coalesced cfix layout
template <int LD>
__global__ __launch_bounds__(256) void k_fixpair_b(const float *__restrict__ aos, int d,
                                                   const float2 *__restrict__ cfix, const float *__restrict__ caos,
                                                   int k, const uint32_t *__restrict__ pair_pts,
                                                   const uint2 *__restrict__ pair_codes, uint32_t npairs,
                                                   uint32_t *__restrict__ labels, uint32_t *__restrict__ ties,
                                                   State *st) {
    const uint32_t i = (blockIdx.x * 256 + threadIdx.x) >> 5;
    if (i >= npairs) return;  // uniform per 32-lane group
    const int r = threadIdx.x & 31, rr = r & 15;
    const uint2 cc = pair_codes[i];
    const uint32_t p = pair_pts[i];
    const uint32_t code = r < 16 ? cc.x : cc.y;
    const uint32_t c = code_row(code, rr);
    const bool valid = c < (uint32_t)k;
    const float4 pv = reinterpret_cast<const float4 *>(aos + (uint64_t)p * LD)[rr % (LD / 4)];
    const float2 *crow = cfix + (uint64_t)(code >> 1) * 2 * (LD / 2) * 16 + (uint64_t)(code & 1) * (LD / 2) * 16 + rr;
    f32x2 a01 = {0.f, 0.f}, a23 = {0.f, 0.f};  // DPP subtracts, packed FMAs (as k_fixrow_b)
    static_for<LD / 4>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        const float2 c0 = crow[(2 * q) * 16], c1 = crow[(2 * q + 1) * 16];
        const f32x2 t01 = {row_bcast<q>(pv.x) - c0.x, row_bcast<q>(pv.y) - c0.y};
        const f32x2 t23 = {row_bcast<q>(pv.z) - c1.x, row_bcast<q>(pv.w) - c1.y};
        a01 = __builtin_elementwise_fma(t01, t01, a01);
        a23 = __builtin_elementwise_fma(t23, t23, a23);
    });
    const float s = (a01.x + a01.y) + (a23.x + a23.y);
    fix_decide<32>(valid ? s : 0.f, valid, c, d, caos, aos + (uint64_t)p * LD, p, r, labels, ties, st);
}

// one wave per ambiguous point: exact distances over its candidates.  A point with more than
// CAND_CAP candidates (many centroids within its window -- duplicated centroids, e.g. from
// duplicated points) goes straight to the KdTree walk, the reference's own search, instead of
// an exact scan of all K (0.9 s per iteration at 2M points with 5% duplicated rows)
__global__ __launch_bounds__(256) void k_exact(const float *__restrict__ aos, int d, const float *__restrict__ caos,
                                               int k, const uint32_t *__restrict__ amb, uint32_t namb,
                                               const uint32_t *__restrict__ cand_cnt,
                                               const uint32_t *__restrict__ cand, uint32_t cap,
                                               uint32_t *__restrict__ labels, uint32_t *__restrict__ ties,
                                               uint32_t *__restrict__ ovf, State *st) {
    const int lane = threadIdx.x & 63;
    const uint32_t a = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (a >= namb) return;
    const uint32_t p = amb[a];
    const int ld = aos_ld(d);
    const float *prow = aos + (uint64_t)p * ld;
    const uint32_t cnt = cand_cnt[a];
    if (cnt > cap) {  // uniform per wave
        if (lane == 0) {
            const uint32_t o = atomicAdd(&st->overflow, 1u);
            if (ovf) {
                ovf[o] = p;  // collected again with a larger list
            } else {
                labels[p] = 0;  // the walk decides
                ties[atomicAdd(&st->ties, 1u)] = p;
            }
        }
        return;
    }
    double best = __builtin_inf();
    uint32_t bidx = 0xffffffffu;
    const uint32_t limit = cnt;
    for (uint32_t j = lane; j < limit; j += 64) {
        const uint32_t c = cand[(uint64_t)a * cap + j];
        const double dd = ref_dist(caos + (uint64_t)c * ld, prow, ld);
        if (dd < best || (dd == best && c < bidx)) {
            best = dd;
            bidx = c;
        }
    }
    double m = best;
    for (int o = 32; o > 0; o >>= 1) m = fmin(m, __shfl_xor(m, o, 64));
    // how many distinct centroids reach the minimum?  (any lane may hold several)
    uint32_t mine = 0;
    uint32_t lowest = 0xffffffffu;
    for (uint32_t j = lane; j < limit; j += 64) {
        const uint32_t c = cand[(uint64_t)a * cap + j];
        if (ref_dist(caos + (uint64_t)c * ld, prow, ld) == m) {
            ++mine;
            lowest = min(lowest, c);
        }
    }
    uint32_t total = mine;
    for (int o = 32; o > 0; o >>= 1) {
        total += __shfl_xor(total, o, 64);
        lowest = min(lowest, __shfl_xor(lowest, o, 64));
    }
    if (lane == 0) {
        if (total == 1) {
            labels[p] = lowest;
        } else if (total == 0) {
            atomicOr(&st->err, ERR_INTERNAL);
        } else {
            labels[p] = lowest;  // provisional; the KdTree pass decides
            ties[atomicAdd(&st->ties, 1u)] = p;
        }
    }
}

// calcAverage (k-means.ts:41-63): one wave per cluster, lane = dimension,
// f64 running sum over the members in ascending point order
// (T = double: the members' JS numbers when the SH columns are not float32 -- calcAverage sums
// the row's numbers, k-means.ts:49-55, while the assign sees Float32Array points)
template <typename T>
__global__ __launch_bounds__(256) void k_sumnd(const T *__restrict__ aos, int d,
                                               const uint32_t *__restrict__ members,
                                               const uint32_t *__restrict__ start, int k, float *__restrict__ cen,
                                               uint32_t big, uint32_t cap, uint32_t *__restrict__ big_list,
                                               uint32_t *__restrict__ nbig, const uint32_t *__restrict__ only,
                                               const uint32_t *__restrict__ nonly) {
    const int lane = threadIdx.x & 63;
    const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (only ? w >= *nonly : w >= (uint32_t)k) return;
    const uint32_t cl = only ? only[w] : w;  // only: the listed clusters (one wave each)
    const uint32_t s0 = start[cl], s1 = start[cl + 1];
    if (s1 - s0 > big) {  // huge clusters: listed for k_big_* (at most cap of them exist)
        if (lane == 0) {
            const uint32_t i = atomicAdd(nbig, 1u);
            if (i < cap) big_list[i] = cl;
        }
        return;
    }
    if (s0 == s1 || lane >= d) return;
    const int ld = aos_ld(d);
    double sum = 0;
    uint32_t j = s0;
    // 32 member rows in flight per wave (the adds stay in ascending point order)
    constexpr int U = 32;
    for (; j + U <= s1; j += U) {
        T v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = aos[(uint64_t)members[j + u] * ld + lane];
#pragma unroll
        for (int u = 0; u < U; ++u) sum += (double)v[u];
    }
    for (; j < s1; ++j) sum += (double)aos[(uint64_t)members[j] * ld + lane];
    cen[(uint64_t)lane * k + cl] = (float)(sum / (double)(s1 - s0));
}

// clusters of more than `big` members (duplicated points pile into one, e.g. every all-zero
// row of a table in one cluster) are cut into slices of SB_SLICE members summed by many
// workgroups at once, each slice with sum|x| and the smallest ulp exponent; when the
// certificate holds for a dimension every partial sum is exact, so the slices' sums add to the
// sequential result, otherwise one lane runs the sequential chain over the whole cluster.
constexpr uint32_t SB_SLICE = 4096;

// the listed clusters' running slice counts (one thread: the list is short, usually empty)
__global__ void k_big_prefix(const uint32_t *__restrict__ start, uint32_t cap, const uint32_t *__restrict__ list,
                             uint32_t *__restrict__ soff, uint32_t *__restrict__ nlist) {
    if (threadIdx.x != 0) return;
    const uint32_t m = min(*nlist, cap);  // cap = n / (big + 1) + 1 clusters can exceed big
    uint32_t o = 0;
    for (uint32_t i = 0; i < m; ++i) {
        soff[i] = o;
        o += (start[list[i] + 1] - start[list[i]] + SB_SLICE - 1) / SB_SLICE;
    }
    soff[m] = o;
    *nlist = m;
}

// slice s of the listed clusters: 4 waves, lane = dimension; (sum, sum|x|, min ulp exponent),
// and each wave's members whose row is not all zero, in order (nzl: SB_SLICE / 4 per wave, nzc
// their count): the sequential fallback of k_big_final walks only those.  Adding +-0 leaves an
// f64 running sum unchanged (it starts at +0 and never becomes -0 under round-to-nearest), so
// the walk over the nonzero rows IS the chain over all members -- a cluster of the table's
// all-zero rows (30% of a scene's rows can be untrained SH) costs its nonzero members only.
constexpr uint32_t SB_WAVE = 1024;  // SB_SLICE / 4
template <typename T>
__global__ __launch_bounds__(256) void k_big_partial(const T *__restrict__ aos, int d,
                                                     const uint32_t *__restrict__ members,
                                                     const uint32_t *__restrict__ start,
                                                     const uint32_t *__restrict__ list,
                                                     const uint32_t *__restrict__ soff,
                                                     const uint32_t *__restrict__ nlist, double *__restrict__ psum,
                                                     double *__restrict__ pabs, int *__restrict__ pemin,
                                                     uint32_t *__restrict__ nzl, uint32_t *__restrict__ nzc) {
    __shared__ double ls[4][64], la[4][64];
    __shared__ int le[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ld = aos_ld(d);
    const uint32_t nl = *nlist, total = soff[nl];
    for (uint32_t sl = blockIdx.x; sl < total; sl += gridDim.x) {
        uint32_t lo = 0, hi = nl;  // the listed cluster whose slices hold sl
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (soff[mid] <= sl) lo = mid;
            else hi = mid;
        }
        const uint32_t cl = list[lo];
        const uint32_t s0 = start[cl] + (sl - soff[lo]) * SB_SLICE;
        const uint32_t s1 = min(start[cl + 1], s0 + SB_SLICE);
        const uint32_t per = (s1 - s0 + 3) / 4;
        const uint32_t a = s0 + min(s1 - s0, w * per), b = s0 + min(s1 - s0, (w + 1) * per);
        double sum = 0, sabs = 0;
        int emin = 0x7fffffff;
        uint32_t *nz = nzl + ((uint64_t)sl * 4 + w) * SB_WAVE;
        uint32_t cnt = 0;  // the same on every active lane
        auto take = [&](T x, uint32_t mem) {
            sum += (double)x;
            sabs += __builtin_fabs((double)x);
            if (x != 0) emin = min(emin, ulp_exp(x));
            if (__ballot(x != 0)) {  // the row is not all zero (the active lanes are lane < d)
                if (lane == 0) nz[cnt] = mem;
                ++cnt;
            }
        };
        if (lane < d) {
            constexpr int U = 32;  // member rows in flight, as k_sumnd
            uint32_t j = a;
            for (; j + U <= b; j += U) {
                T v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) v[u] = aos[(uint64_t)members[j + u] * ld + lane];
#pragma unroll
                for (int u = 0; u < U; ++u) take(v[u], members[j + u]);
            }
            for (; j < b; ++j) take(aos[(uint64_t)members[j] * ld + lane], members[j]);
            if (lane == 0) nzc[(uint64_t)sl * 4 + w] = cnt;
        }
        ls[w][lane] = sum;
        la[w][lane] = sabs;
        le[w][lane] = emin;
        __syncthreads();
        if (w == 0 && lane < d) {
            psum[(uint64_t)sl * 64 + lane] = ((ls[0][lane] + ls[1][lane]) + ls[2][lane]) + ls[3][lane];
            pabs[(uint64_t)sl * 64 + lane] = ((la[0][lane] + la[1][lane]) + la[2][lane]) + la[3][lane];
            pemin[(uint64_t)sl * 64 + lane] = min(min(le[0][lane], le[1][lane]), min(le[2][lane], le[3][lane]));
        }
        __syncthreads();
    }
}

// one wave per listed cluster, lane = dimension: the slices' sums under the certificate, else
// the sequential chain (k-means.ts:41-63)
template <typename T>
__global__ __launch_bounds__(64) void k_big_final(const T *__restrict__ aos, int d,
                                                  const uint32_t *__restrict__ members,
                                                  const uint32_t *__restrict__ start, int k,
                                                  const uint32_t *__restrict__ list, const uint32_t *__restrict__ soff,
                                                  const uint32_t *__restrict__ nlist, const double *__restrict__ psum,
                                                  const double *__restrict__ pabs, const int *__restrict__ pemin,
                                                  const uint32_t *__restrict__ nzl, const uint32_t *__restrict__ nzc,
                                                  float *__restrict__ cen) {
    const int lane = threadIdx.x;
    const int ld = aos_ld(d);
    const uint32_t nl = *nlist;
    for (uint32_t i = blockIdx.x; i < nl; i += gridDim.x) {
        if (lane >= d) continue;
        const uint32_t cl = list[i], s0 = start[cl], s1 = start[cl + 1], m = s1 - s0;
        double S = 0, A = 0;
        int E = 0x7fffffff;
        for (uint32_t sl = soff[i]; sl < soff[i + 1]; ++sl) {
            S += psum[(uint64_t)sl * 64 + lane];
            A += pabs[(uint64_t)sl * 64 + lane];
            E = min(E, pemin[(uint64_t)sl * 64 + lane]);
        }
        if (!sum_is_exact(A, E)) {
            // the sequential chain (k-means.ts:41-63) over the members' nonzero rows, slice by
            // slice, wave part by wave part: the members' order
            S = 0;
            constexpr int U = 32;
            for (uint64_t part = (uint64_t)soff[i] * 4; part < (uint64_t)soff[i + 1] * 4; ++part) {
                const uint32_t *mem = nzl + part * SB_WAVE;
                const uint32_t c = nzc[part];
                uint32_t j = 0;
                for (; j + U <= c; j += U) {
                    T v[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) v[u] = aos[(uint64_t)mem[j + u] * ld + lane];
#pragma unroll
                    for (int u = 0; u < U; ++u) S += (double)v[u];
                }
                for (; j < c; ++j) S += (double)aos[(uint64_t)mem[j] * ld + lane];
            }
        }
        (void)members;
        (void)s0;
        cen[(uint64_t)lane * k + cl] = (float)(S / (double)m);
    }
}

// the float64 member rows (row stride aos_ld(d), zero padded) for the sums of k_sumnd<double>
__global__ __launch_bounds__(256) void k_aos64(const double *const *cols, int d, uint64_t n, double *__restrict__ aos) {
    const int ld = aos_ld(d);
    for (uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; f < n * ld; f += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = f / ld;
        const int a = (int)(f % ld);
        aos[f] = a < d ? cols[a][r] : 0.0;
    }
}

// the clusters k_sumnd listed as huge (list / nlist, at most cap): sliced partials, then the
// certified sums or the sequential chain over their nonzero rows
template <typename T>
void big_sums(st_ctx *c, const T *aos, int d, uint64_t n, int k, const uint32_t *members, const uint32_t *start,
              float *cen, uint32_t cap, uint32_t *list, uint32_t *nlist) {
    const uint64_t slices = n / SB_SLICE + cap;  // bound on the listed clusters' slices
    auto *soff = wsT<uint32_t>(c, "kn.bsoff", (size_t)cap + 1);
    auto *psum = wsT<double>(c, "kn.bsum", slices * 64);
    auto *pabs = wsT<double>(c, "kn.babs", slices * 64);
    auto *pemin = wsT<int>(c, "kn.bemin", slices * 64);
    auto *nzl = wsT<uint32_t>(c, "kn.bnzl", slices * 4 * SB_WAVE);
    auto *nzc = wsT<uint32_t>(c, "kn.bnzc", slices * 4);
    hipLaunchKernelGGL(k_big_prefix, dim3(1), dim3(64), 0, c->stream, start, cap, list, soff, nlist);
    hipLaunchKernelGGL(k_big_partial<T>, dim3(grid_for(slices, 1, 2048)), dim3(256), 0, c->stream, aos, d, members,
                       start, list, soff, nlist, psum, pabs, pemin, nzl, nzc);
    hipLaunchKernelGGL(k_big_final<T>, dim3(std::min<unsigned>(cap, 1024u)), dim3(64), 0, c->stream, aos, d, members,
                       start, k, list, soff, nlist, psum, pabs, pemin, nzl, nzc, cen);
    ST_LAUNCH_CHECK();
}

template <typename T>
void launch_sums(st_ctx *c, const T *aos, int d, uint64_t n, int k, const uint32_t *members, const uint32_t *start,
                 float *cen) {
    const uint32_t big = sumnd_big();
    const uint32_t cap = (uint32_t)(n / ((uint64_t)big + 1) + 1);
    auto *list = wsT<uint32_t>(c, "kn.blist", cap);
    auto *nlist = wsT<uint32_t>(c, "kn.bn", 1);
    ST_HIP(hipMemsetAsync(nlist, 0, 4, c->stream));
    hipLaunchKernelGGL(k_sumnd<T>, dim3((k + 3) / 4), dim3(256), 0, c->stream, aos, d, members, start, k, cen, big,
                       cap, list, nlist, (const uint32_t *)nullptr, (const uint32_t *)nullptr);
    if (n > big) big_sums(c, aos, d, n, k, members, start, cen, cap, list, nlist);
    ST_LAUNCH_CHECK();
}

template <int KS>
struct Sweep {
    static void main(st_ctx *c, const uint4 *pfrag, uint32_t ntiles, uint32_t n, const uint4 *cfrag, uint32_t ctiles,
                     const float *pnorm, const float *pdn, const uint32_t *cmax, const float *chalf,
                     const float *chalf_d, const float *ntab, const Bound &bnd,
                     uint32_t *labels, float *thr, uint32_t *amb, State *st, uint32_t *pair_pts, uint2 *pair_codes,
                     uint32_t *code_hist) {
        const uint32_t per_block = NW * PT;
        const dim3 grid((ntiles + per_block - 1) / per_block);
        KTimer kt(c, "kn.sweep");
        hipLaunchKernelGGL((k_sweep<KS, 0>), grid, dim3(WG), 0, c->stream, pfrag, ntiles, n, cfrag, ctiles, pnorm,
                           pdn, cmax, chalf, chalf_d, ntab, bnd, labels, thr, amb, st, (uint32_t *)nullptr, (uint32_t *)nullptr, 0u,
                           pair_pts,
                           pair_codes, code_hist);
        ST_LAUNCH_CHECK();
    }
    static void collect(st_ctx *c, const uint4 *afrag, uint32_t atiles, uint32_t namb, const uint4 *cfrag,
                        uint32_t ctiles, const Bound &bnd, float *thr_slot, uint32_t *cand_cnt, uint32_t *cand,
                        uint32_t cap, hipStream_t s) {
        const uint32_t per_block = NW * PT;
        const uint32_t blocks = (atiles + per_block - 1) / per_block;
        // enough workgroups to cover the chip twice over
        const uint32_t split = std::max(1u, std::min(ctiles / CT_STAGE, (2048u + blocks - 1) / blocks));
        const dim3 grid(blocks, split);
        KTimer kt(c, "kn.collect", s);
        hipLaunchKernelGGL((k_sweep<KS, 1>), grid, dim3(WG), 0, s, afrag, atiles, namb, cfrag, ctiles,
                           (const float *)nullptr, (const float *)nullptr, (const uint32_t *)nullptr,
                           (const float *)nullptr, (const float *)nullptr, (const float *)nullptr, bnd,
                           (uint32_t *)nullptr, thr_slot,
                           (uint32_t *)nullptr, (State *)nullptr, cand_cnt, cand, cap, (uint32_t *)nullptr,
                           (uint2 *)nullptr, (uint32_t *)nullptr);
        ST_LAUNCH_CHECK();
    }
};

bool probe_denorm(st_ctx *c) {
    static thread_local std::map<int, bool> cache;
    auto it = cache.find(c->device);
    if (it != cache.end()) return it->second;
    auto *d = wsT<float>(c, "kn.probe", 1);
    hipLaunchKernelGGL(k_probe_denorm, dim3(1), dim3(64), 0, c->stream, d);
    ST_LAUNCH_CHECK();
    float v = 0;
    ST_HIP(hipMemcpyAsync(&v, d, 4, hipMemcpyDeviceToHost, c->stream));
    ST_HIP(hipStreamSynchronize(c->stream));
    const bool keep = (v == std::ldexp(1.0f, -20));
    cache[c->device] = keep;
    return keep;
}

}  // namespace

#define ST_KS_DISPATCH(KSV, CALL) \
    switch (KSV) {                \
        case 1: { constexpr int KS = 1; CALL; } break; \
        case 2: { constexpr int KS = 2; CALL; } break; \
        case 3: { constexpr int KS = 3; CALL; } break; \
        case 4: { constexpr int KS = 4; CALL; } break; \
        default: throw Error(ST_ERR_UNSUPPORTED, "kmeans: dimension too large for the MFMA assign (D <= 61)"); \
    }

// ---- steps: prepare the point set once, then one exact assign per iteration -------
void nd_prepare(st_ctx *c, const float *const *dcols, int d, uint64_t n) {
    ST_REQUIRE(d <= 61, ST_ERR_UNSUPPORTED, "kmeans: D > 61 not supported by the MFMA assign");
    const int ks = kp_of(d) / 16;
    const uint32_t ntiles = (uint32_t)((n + 31) / 32);
    auto *pfrag = wsT<uint4>(c, "kn.pfrag", (size_t)ntiles * ks * 64);
    auto *pnorm = wsT<float>(c, "kn.pnorm", n);
    auto *pdn = wsT<float>(c, "kn.pdn", n);
    auto *aos = wsT<float>(c, "kn.aos", n * (size_t)aos_ld(d));
    auto *scal = wsT<uint32_t>(c, "kn.scal", 4);  // [0]=absmax bits [1]=cmax bits [2]=max residual norm bits
    // scale: max|x| * sigma in [1, 2); check_finite found max|x| in its pass over the points
    ST_HIP(hipMemsetAsync(scal, 0, 16, c->stream));
    float amax = c->km_absmax;
    c->km_absmax = -1.0f;
    if (amax < 0.0f) {
        hipLaunchKernelGGL(k_absmax, dim3(grid_for(n, 256, 2048)), dim3(256), 0, c->stream, dcols, d, n, scal);
        ST_LAUNCH_CHECK();
        uint32_t amax_bits = 0;
        ST_HIP(hipMemcpyAsync(&amax_bits, scal, 4, hipMemcpyDeviceToHost, c->stream));
        ST_HIP(hipStreamSynchronize(c->stream));
        amax = __builtin_bit_cast(float, amax_bits);
    }
    float sigma = 1.0f;
    if (amax > 0) sigma = std::ldexp(1.0f, -std::ilogb(amax));
    const dim3 gpf((unsigned)(((uint64_t)ntiles * 32 + PF_PTS - 1) / PF_PTS));
    if (d == 45)
        hipLaunchKernelGGL(k_point_frags<45>, gpf, dim3(PF_PTS), 0, c->stream, dcols, d, n, ntiles, ks, sigma, pfrag,
                           pnorm, pdn, aos);
    else if (d == 24)
        hipLaunchKernelGGL(k_point_frags<24>, gpf, dim3(PF_PTS), 0, c->stream, dcols, d, n, ntiles, ks, sigma, pfrag,
                           pnorm, pdn, aos);
    else if (d == 9)
        hipLaunchKernelGGL(k_point_frags<9>, gpf, dim3(PF_PTS), 0, c->stream, dcols, d, n, ntiles, ks, sigma, pfrag,
                           pnorm, pdn, aos);
    else
        hipLaunchKernelGGL(k_point_frags<0>, gpf, dim3(PF_PTS), 0, c->stream, dcols, d, n, ntiles, ks, sigma, pfrag,
                           pnorm, pdn, aos);
    ST_LAUNCH_CHECK();
    c->kn_sigma = sigma;
    c->kn_n = n;
    c->kn_d = d;
    mark(c, "kn.prep");
}

namespace {
__global__ __launch_bounds__(256) void k_rows_aos(const float *__restrict__ cen, int d, int k, float *__restrict__ caos) {
    const int ld = aos_ld(d);
    for (uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; f < (uint64_t)k * ld;
         f += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t r = (uint32_t)(f / ld), a = (uint32_t)(f % ld);
        caos[f] = a < (uint32_t)d ? cen[(uint64_t)a * k + r] : 0.0f;
    }
}

uint32_t nd_assign_core(st_ctx *c, const float *const *dcols, int d, uint64_t n, int k, const float *cen,
                        uint32_t *labels, km::State *dstate, bool walk_ties, NdFused *fz = nullptr);
}  // namespace

// The assign over the distinct centroid rows: when several centroids share a row (duplicated
// input rows drawn by the init or a re-seed), the sweep and its fix-ups see one representative
// per row and a point that lands on a shared row takes the member the reference's KdTree walk
// meets first (kd_group_labels, a descent of the tree); exact ties between distinct rows go to
// the walk over the whole tree.  Without shared rows this is the plain assign.
void nd_assign(st_ctx *c, const float *const *dcols, int d, uint64_t n, int k, const float *cen, uint32_t *labels,
               km::State *dstate, NdFused *fz, const std::function<bool()> &settle) {
    if (fz) fz->valid = false;
    CenGroups g;
    const bool try_groups = k > 1 && !getenv("ST_NO_CEN_GROUPS");
    bool grouped = try_groups && cen_groups(c, d, k, cen, &g);
    if (settle && settle()) grouped = try_groups && cen_groups(c, d, k, cen, &g);
    if (grouped) {
        const uint32_t nties = nd_assign_core(c, dcols, d, n, (int)g.kr, g.cen_r, labels, dstate, false);
        const int ld = aos_ld(d);
        auto *aos = wsT<float>(c, "kn.aos", n * (size_t)ld);
        {
            KTimer kt(c, "kn.groups");
            kd_group_labels(c, d, k, cen, g, aos, ld, n, labels, &dstate->err);
        }
        if (nties) {
            KTimer kt(c, "kn.ties");
            auto *caos = wsT<float>(c, "kn.caosfull", (size_t)k * ld);
            hipLaunchKernelGGL(k_rows_aos, dim3(grid_for((uint64_t)k * ld, 256, 2048)), dim3(256), 0, c->stream, cen, d,
                               k, caos);
            ST_LAUNCH_CHECK();
            kd_resolve_ties(c, d, k, cen, aos, caos, ld, wsT<uint32_t>(c, "kn.ties", n), nties, labels, true);
        }
        mark(c, "kn.exact");
        return;
    }
    nd_assign_core(c, dcols, d, n, k, cen, labels, dstate, true, fz);
}

namespace {
// the exact assign against the k centroids cen; exact ties go to the KdTree walk over these
// centroids (walk_ties) or are left listed in kn.ties for the caller: returns their count
uint32_t nd_assign_core(st_ctx *c, const float *const *dcols, int d, uint64_t n, int k, const float *cen,
                        uint32_t *labels, km::State *dstate, bool walk_ties, NdFused *fz) {
    ST_REQUIRE(c->kn_n == n && c->kn_d == d, ST_ERR_ARG, "kmeans assign: point set not prepared");
    ST_REQUIRE(k <= (1 << 24), ST_ERR_UNSUPPORTED, "kmeans: K too large");
    const int ks = kp_of(d) / 16;
    const uint32_t ntiles = (uint32_t)((n + 31) / 32);
    // centroid tiles, padded to whole LDS stages with rows that can never win (k_centroid_frags)
    const uint32_t ctiles = (uint32_t)(((k + 31) / 32 + CT_STAGE - 1) / CT_STAGE * CT_STAGE);
    auto *pfrag = wsT<uint4>(c, "kn.pfrag", (size_t)ntiles * ks * 64);
    auto *pnorm = wsT<float>(c, "kn.pnorm", n);
    auto *pdn = wsT<float>(c, "kn.pdn", n);
    auto *aos = wsT<float>(c, "kn.aos", n * (size_t)aos_ld(d));
    auto *scal = wsT<uint32_t>(c, "kn.scal", 4);
    auto *cfrag = wsT<uint4>(c, "kn.cfrag", (size_t)ctiles * ks * 64);
    auto *thr = wsT<float>(c, "kn.thr", n);
    auto *amb = wsT<uint32_t>(c, "kn.amb", n);
    auto *ties = wsT<uint32_t>(c, "kn.ties", n);
    auto *h = static_cast<State *>(pinned(c, sizeof(State)));
    const Bound bnd = make_bound(d, probe_denorm(c));
    const float sigma = c->kn_sigma;

    ST_HIP(hipMemsetAsync(scal + 1, 0, 8, c->stream));
    auto *caos = wsT<float>(c, "kn.caos", (size_t)k * aos_ld(d));
    auto *cfix = wsT<float2>(c, "kn.cfix", (size_t)ctiles * 32 * (aos_ld(d) / 2));
    auto *cnorm = wsT<float>(c, "kn.cnorm", (size_t)ctiles * 32);
    auto *chalf = wsT<float>(c, "kn.chalf", (size_t)ctiles * 2);
    auto *cdn = wsT<float>(c, "kn.cdn", (size_t)ctiles * 32);
    auto *chalf_d = wsT<float>(c, "kn.chalfd", (size_t)ctiles * 2);
    ST_REQUIRE(ks <= CF_W, ST_ERR_INTERNAL, "kmeans: more fragments per row than centroid waves");
    hipLaunchKernelGGL(k_centroid_frags, dim3(grid_for((uint64_t)ctiles * 32, 64, 4096)), dim3(64 * CF_W), 0, c->stream,
                       cen, d, k, ctiles, ks, sigma, cfrag, scal + 1, caos, cfix, cnorm, cdn);
    hipLaunchKernelGGL(k_half_max, dim3(grid_for((uint64_t)ctiles * 2, 256, 1024)), dim3(256), 0, c->stream, cnorm,
                       cdn, ctiles * 2, chalf, chalf_d);
    auto *ntab = wsT<float>(c, "kn.ntab", NTAB);
    hipLaunchKernelGGL(k_norm_table, dim3(1), dim3(NTAB), 0, c->stream, cnorm, cdn, ctiles * 32, scal + 1, ntab);
    ST_LAUNCH_CHECK();
    auto *pair_pts = wsT<uint32_t>(c, "kn.pairpts", n);
    auto *pair_codes = wsT<uint2>(c, "kn.paircodes", n);
    ST_HIP(hipMemsetAsync(&dstate->amb, 0, 16, c->stream));  // amb + ties + overflow + pairs
    const uint32_t ncodes = ctiles * 2;
    const int ld = aos_ld(d);
    // decided points grouped by tile-half for k_fixrow_b: the sweep counts them per code
    const bool grouped_fix =
        ncodes <= (uint32_t)FB_MAX_CODES && (ld == 48 || ld == 24 || ld == 12) && !getenv("ST_FIXROW_L2");
    auto *hist = grouped_fix ? wsT<uint32_t>(c, "kn.fbhist", ncodes) : nullptr;
    if (hist) ST_HIP(hipMemsetAsync(hist, 0, ncodes * sizeof(uint32_t), c->stream));
    ST_KS_DISPATCH(ks, (Sweep<KS>::main(c, pfrag, ntiles, (uint32_t)n, cfrag, ctiles, pnorm, pdn, scal + 1, chalf,
                                        chalf_d, ntab, bnd,
                                        labels, thr, amb, dstate, pair_pts, pair_codes, hist)));
    // the sweep's pair / ambiguous counts are final here (the fix-up only adds ties): read back
    // behind the sweep, waited for while the fix-up runs, so that the pairs' and the ambiguous
    // points' kernels queue up behind it with no idle gap; the fix-up's own tie count (h_fix)
    // is read behind it and waited for only where it is needed
    auto *h_fix = static_cast<State *>(pinned_slot(c, "kn.hfix", sizeof(State)));
    ST_HIP(hipMemcpyAsync(h, dstate, sizeof(State), hipMemcpyDeviceToHost, c->stream));
    for (auto &e : c->kn_ev)
        if (!e) ST_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    hipEvent_t ev_sw = c->kn_ev[0], ev_fix = c->kn_ev[1], ev_grp = c->kn_ev[2], ev_side = c->kn_ev[3];
    bool grouped_ev = false;
    ST_HIP(hipEventRecord(ev_sw, c->stream));
    if (grouped_fix) {
        // group the decided points by tile-half, then settle them with register-resident rows
        KTimer kt(c, "kn.fixrow");
        auto *cursor = wsT<uint32_t>(c, "kn.fbcur", ncodes);
        auto *ndec = wsT<uint32_t>(c, "kn.fbnd", 1);
        // k_fixrow_lp sums DT = 45 / 24 / 9 dimensions of its LD-wide rows (the SH palettes' d):
        // any other d in the same row width (10-12, 21-23, 46-48) takes the member-sort update
        const bool fused = fz && fz->want && walk_ties && d == (ld == 48 ? 45 : ld == 24 ? 24 : 9);
        // fused: the grouped points alone (a slice knows its code); otherwise (point, code) pairs
        auto *grouped = fused ? nullptr : wsT<uint2>(c, "kn.fbpts2", n);
        auto *grouped1 = fused ? wsT<uint32_t>(c, "kn.fbpts1", n) : nullptr;
        auto *soff = fused ? wsT<uint32_t>(c, "kn.fasoff", (size_t)ncodes + 1) : nullptr;
        // workgroups of the one-reservation grouping (0: k_code_scatter's 4,096-point rounds)
        // (k_code_scatter_run reads the labels 16 bytes at a time: a caller's unaligned labels take
        // the rounds)
        static const int cs_env = getenv("ST_CS_WG") ? atoi(getenv("ST_CS_WG")) : 256;
        const int cs_wg = ((uintptr_t)labels & 15u) ? 0 : cs_env;
        const unsigned gcs = cs_wg > 0 ? grid_for(n, 256, (unsigned)cs_wg) : grid_for(n, FB_TILE, 2048);
        if (fused) {  // slice offsets and the codes' starts in one workgroup
            hipLaunchKernelGGL(k_fa_slices, dim3(1), dim3(FS_T), 0, c->stream, hist, ncodes, soff, cursor, ndec);
            if (cs_wg > 0)
                hipLaunchKernelGGL(k_code_scatter_run<uint32_t>, dim3(gcs), dim3(256), 0, c->stream, labels, (uint32_t)n,
                                   ncodes, cursor, grouped1);
            else
                hipLaunchKernelGGL(k_code_scatter<uint32_t>, dim3(gcs), dim3(256), 0, c->stream, labels, (uint32_t)n,
                                   ncodes, cursor, grouped1);
        } else {
            scan_u32(c, hist, cursor, ncodes, ndec);
            if (cs_wg > 0)
                hipLaunchKernelGGL(k_code_scatter_run<uint2>, dim3(gcs), dim3(256), 0, c->stream, labels, (uint32_t)n,
                                   ncodes, cursor, grouped);
            else
                hipLaunchKernelGGL(k_code_scatter<uint2>, dim3(gcs), dim3(256), 0, c->stream, labels, (uint32_t)n,
                                   ncodes, cursor, grouped);
        }
        ST_LAUNCH_CHECK();
        // the grouping has read every label: the pair / ambiguous fix-ups may write theirs from here
        ST_HIP(hipEventRecord(ev_grp, c->stream));
        grouped_ev = true;
        const dim3 g((unsigned)(((n + FB_RUN - 1) / FB_RUN * 16 + 255) / 256));
        if (fused) {
            // the fix-up with the decided points' sums (k_fixrow_lp), slices shared out over the workgroups
            const uint64_t slices = ncodes + n / FA_SL + 1;
            auto *psum = wsT<double>(c, "kn.fasum", slices * 16 * ld);
            auto *pabs = wsT<double>(c, "kn.faabs", slices * 16 * ld);
            auto *pemin = wsT<int>(c, "kn.faemin", slices * 16 * ld);
            auto *pcnt = wsT<uint32_t>(c, "kn.facnt", slices * 16);
            // the slices (their count is on the device) shared out over up to 4,096 workgroups: about
            // one slice each at the palette shapes (1,024 stay resident; at 2,048 -- two slices per
            // workgroup in two rounds -- the launch took 5% longer, 850 against 812 us at 10M x 45)
            const dim3 gl((unsigned)std::min<uint64_t>(slices, 4096));
            if (ld == 48)
                hipLaunchKernelGGL(k_fixrow_lp<48>, gl, dim3(64 * FL_WAVES), 0, c->stream, aos, d, caos, k, grouped1, hist,
                                   cursor, soff, ncodes, labels, ties, dstate, psum, pabs, pemin, pcnt);
            else if (ld == 24)
                hipLaunchKernelGGL(k_fixrow_lp<24>, gl, dim3(64 * FL_WAVES), 0, c->stream, aos, d, caos, k, grouped1, hist,
                                   cursor, soff, ncodes, labels, ties, dstate, psum, pabs, pemin, pcnt);
            else
                hipLaunchKernelGGL(k_fixrow_lp<12>, gl, dim3(64 * FL_WAVES), 0, c->stream, aos, d, caos, k, grouped1, hist,
                                   cursor, soff, ncodes, labels, ties, dstate, psum, pabs, pemin, pcnt);
            fz->valid = true;
            fz->ncodes = ncodes;
        } else if (ld == 48)
            hipLaunchKernelGGL(k_fixrow_b<48>, g, dim3(256), 0, c->stream, aos, d, caos, k, grouped, ndec, labels,
                               ties, dstate);
        else if (ld == 24)
            hipLaunchKernelGGL(k_fixrow_b<24>, g, dim3(256), 0, c->stream, aos, d, caos, k, grouped, ndec, labels,
                               ties, dstate);
        else
            hipLaunchKernelGGL(k_fixrow_b<12>, g, dim3(256), 0, c->stream, aos, d, caos, k, grouped, ndec, labels,
                               ties, dstate);
        ST_LAUNCH_CHECK();
    } else {
        KTimer kt(c, "kn.fixrow");
        hipLaunchKernelGGL(k_fixrow, dim3((unsigned)((n * 16 + 255) / 256)), dim3(256), 0, c->stream, aos, d, cfix,
                           caos, k, (uint32_t)n, labels, ties, dstate);
        ST_LAUNCH_CHECK();
    }
    ST_HIP(hipMemcpyAsync(h_fix, dstate, sizeof(State), hipMemcpyDeviceToHost, c->stream));
    ST_HIP(hipEventRecord(ev_fix, c->stream));
    ST_HIP(hipEventSynchronize(ev_sw));
    const uint32_t npair = h->pairs;
    const uint32_t namb = h->amb;
    // The pair and ambiguous points' fix-ups, on the side stream beside the decided points' one
    // when the one-device loop asks for it (c->fix_overlap) and the grouping has read the labels
    // (ev_grp): their ties go to a list and counters of their own (kn.ties2, kn.state2), appended to
    // the fix-up's list afterwards -- the same list, in the same order, as one stream gives.
    const bool overlap = c->fix_overlap && grouped_ev && (npair || namb) && !getenv("ST_FIX_SERIAL");
    const hipStream_t fs = overlap ? side_stream(c) : c->stream;
    State *ds = overlap ? static_cast<State *>(ws(c, "kn.state2", sizeof(State))) : dstate;
    uint32_t *tl = overlap ? wsT<uint32_t>(c, "kn.ties2", n) : ties;
    auto *hs = overlap ? static_cast<State *>(pinned_slot(c, "kn.hside", sizeof(State))) : h;
    if (overlap) {
        ST_HIP(hipStreamWaitEvent(fs, ev_grp, 0));
        ST_HIP(hipMemsetAsync(ds, 0, sizeof(State), fs));
    }
    if (npair) {
        KTimer kt(c, "kn.fixpair", fs);
        const dim3 g((npair * 32 + 255) / 256);
        if (ld == 48)
            hipLaunchKernelGGL(k_fixpair_b<48>, g, dim3(256), 0, fs, aos, d, cfix, caos, k, pair_pts,
                               pair_codes, npair, labels, tl, ds);
        else if (ld == 24)
            hipLaunchKernelGGL(k_fixpair_b<24>, g, dim3(256), 0, fs, aos, d, cfix, caos, k, pair_pts,
                               pair_codes, npair, labels, tl, ds);
        else if (ld == 12)
            hipLaunchKernelGGL(k_fixpair_b<12>, g, dim3(256), 0, fs, aos, d, cfix, caos, k, pair_pts,
                               pair_codes, npair, labels, tl, ds);
        else
            hipLaunchKernelGGL(k_fixpair, g, dim3(256), 0, fs, aos, d, cfix, caos, k, pair_pts, pair_codes,
                               npair, labels, tl, ds);
        ST_LAUNCH_CHECK();
    }
    mark(c, "kn.assign");
    uint32_t ovf1 = 0;  // first lists that overflowed (collected again with CAND_CAP2)
    if (namb) {
        const uint32_t atiles = (namb + 31) / 32;
        auto *afrag = wsT<uint4>(c, "kn.afrag", (size_t)atiles * ks * 64);
        auto *thr_slot = wsT<float>(c, "kn.thrslot", (size_t)atiles * 32);
        auto *cand_cnt = wsT<uint32_t>(c, "kn.ccnt", (size_t)atiles * 32);
        auto *cand = wsT<uint32_t>(c, "kn.cand", (size_t)namb * CAND_CAP);
        hipLaunchKernelGGL(k_gather_amb, dim3(grid_for((uint64_t)atiles * 32, 256, 4096)), dim3(256), 0, fs,
                           pfrag, amb, thr, namb, ks, afrag, thr_slot, cand_cnt);
        ST_LAUNCH_CHECK();
        auto *ovf = wsT<uint32_t>(c, "kn.ovf", namb);
        ST_KS_DISPATCH(ks, (Sweep<KS>::collect(c, afrag, atiles, namb, cfrag, ctiles, bnd, thr_slot, cand_cnt, cand,
                                               (uint32_t)CAND_CAP, fs)));
        {
            KTimer kt(c, "kn.exact", fs);
            hipLaunchKernelGGL(k_exact, dim3((namb + 3) / 4), dim3(256), 0, fs, aos, d, caos, k, amb, namb,
                               cand_cnt, cand, (uint32_t)CAND_CAP, labels, tl, ovf, ds);
            ST_LAUNCH_CHECK();
        }
        ST_HIP(hipMemcpyAsync(hs, ds, sizeof(State), hipMemcpyDeviceToHost, fs));
        ST_HIP(hipStreamSynchronize(fs));
        ovf1 = hs->overflow;
        if (hs->overflow) {
            // points whose window holds more than CAND_CAP rows (wide windows: outlying points of
            // heavy-tailed data): collected again with lists of CAND_CAP2, in batches; only those
            // that overflow these too take the KdTree walk
            const uint32_t nov = hs->overflow, batch = std::min(nov, (uint32_t)OVF_BATCH);
            const uint32_t btiles = (batch + 31) / 32;
            auto *afrag2 = wsT<uint4>(c, "kn.afrag2", (size_t)btiles * ks * 64);
            auto *thr2 = wsT<float>(c, "kn.thrslot2", (size_t)btiles * 32);
            auto *cnt2 = wsT<uint32_t>(c, "kn.ccnt2", (size_t)btiles * 32);
            auto *cand2 = wsT<uint32_t>(c, "kn.cand2", (size_t)batch * CAND_CAP2);
            for (uint32_t b0 = 0; b0 < nov; b0 += batch) {
                const uint32_t m = std::min(batch, nov - b0), mt = (m + 31) / 32;
                hipLaunchKernelGGL(k_gather_amb, dim3(grid_for((uint64_t)mt * 32, 256, 4096)), dim3(256), 0, fs,
                                   pfrag, ovf + b0, thr, m, ks, afrag2, thr2, cnt2);
                ST_LAUNCH_CHECK();
                ST_KS_DISPATCH(ks, (Sweep<KS>::collect(c, afrag2, mt, m, cfrag, ctiles, bnd, thr2, cnt2, cand2,
                                                       (uint32_t)CAND_CAP2, fs)));
                KTimer kt(c, "kn.exact", fs);
                hipLaunchKernelGGL(k_exact, dim3((m + 3) / 4), dim3(256), 0, fs, aos, d, caos, k, ovf + b0, m,
                                   cnt2, cand2, (uint32_t)CAND_CAP2, labels, tl, (uint32_t *)nullptr, ds);
                ST_LAUNCH_CHECK();
            }
            ST_HIP(hipMemcpyAsync(hs, ds, sizeof(State), hipMemcpyDeviceToHost, fs));
            ST_HIP(hipStreamSynchronize(fs));
        }
        if (getenv("ST_DEBUG")) {  // candidate-count histogram of the ambiguous points
            std::vector<uint32_t> cc(namb);
            ST_HIP(hipMemcpy(cc.data(), cand_cnt, namb * 4, hipMemcpyDeviceToHost));
            uint64_t hist[6] = {0, 0, 0, 0, 0, 0};
            for (uint32_t v : cc) ++hist[v < 5 ? v : 5];
            fprintf(stderr, "[st kmeans] candidates per ambiguous point: 0:%llu 1:%llu 2:%llu 3:%llu 4:%llu 5+:%llu\n",
                    (unsigned long long)hist[0], (unsigned long long)hist[1], (unsigned long long)hist[2],
                    (unsigned long long)hist[3], (unsigned long long)hist[4], (unsigned long long)hist[5]);
        }
    } else if (npair) {  // the pairs' ties and counters
        ST_HIP(hipMemcpyAsync(hs, ds, sizeof(State), hipMemcpyDeviceToHost, fs));
        ST_HIP(hipStreamSynchronize(fs));
    }
    // the decided points' fix-up (its read-back was queued behind it)
    ST_HIP(hipEventSynchronize(ev_fix));
    const uint32_t nties_fix = h_fix->ties;
    if (overlap) {
        // join: the side stream's ties follow the fix-up's in one list (kn.ties), as one stream
        // would have listed them; its overflow count is the assign's
        ST_HIP(hipEventRecord(ev_side, fs));
        ST_HIP(hipStreamWaitEvent(c->stream, ev_side, 0));
        if (hs->ties)
            ST_HIP(hipMemcpyAsync(ties + nties_fix, tl, (size_t)hs->ties * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                                  c->stream));
        *h = *h_fix;
        h->ties = nties_fix + hs->ties;
        h->overflow = hs->overflow;
    } else if (!npair && !namb) {
        *h = *h_fix;
    }
    if (fz && fz->valid) {  // the fix-up's own ties are listed first; pairs and ambiguous come next
        fz->nties_fix = nties_fix;
        fz->npair = npair;
        fz->namb = namb;
    }
    if (getenv("ST_DEBUG"))
        fprintf(stderr, "[st kmeans] n=%llu k=%d pairs=%u ambiguous=%u ties=%u overflow=%u sigma=%g\n",
                (unsigned long long)n, k, npair, namb, h->ties, h->overflow, sigma);
    {
        auto &ks_ = c->kn_stats;
        ++ks_.assigns;
        ks_.points += n;
        ks_.pairs += npair;
        ks_.ambiguous += namb;
        ks_.overflow += ovf1;
        ks_.walked_overflow += h->overflow - ovf1;  // the second lists' overflows go to the walk
        ks_.ties += h->ties;
    }
    // exact ties from k_fixrow, k_fixpair and k_exact (and candidate overflows): the KdTree walk
    if (!walk_ties) return h->ties;
    if (h->ties) {
        KTimer kt(c, "kn.ties");
        kd_resolve_ties(c, d, k, cen, aos, caos, ld, ties, h->ties, labels);
    }
    mark(c, "kn.exact");
    return h->ties;
}
}  // namespace

namespace {
// the points the fused fix-up did not sum (pairs, ambiguous, its own exact ties), sorted by final
// label: kn.ovals in label order, kn.ostart their cluster ranges; returns their count
uint32_t others_sort(st_ctx *c, uint64_t n, int k, const NdFused &fz, const uint32_t *labels) {
    const uint32_t m = fz.npair + fz.namb + fz.nties_fix;
    auto *okeys = wsT<uint32_t>(c, "kn.okeys", (size_t)m + 1);
    auto *ovals = wsT<uint32_t>(c, "kn.ovals", (size_t)m + 1);
    auto *ostart = wsT<uint32_t>(c, "kn.ostart", (size_t)k + 1);
    if (m) {
        hipLaunchKernelGGL(k_others_keys, dim3(grid_for(m, 256, 4096)), dim3(256), 0, c->stream,
                           wsT<uint32_t>(c, "kn.pairpts", n), fz.npair, wsT<uint32_t>(c, "kn.amb", n), fz.namb,
                           wsT<uint32_t>(c, "kn.ties", n), fz.nties_fix, labels, okeys, ovals);
        ST_LAUNCH_CHECK();
        int bits = 1;
        while ((1ull << bits) < (uint64_t)k) ++bits;
        radix_sort_u32(c, okeys, ovals, m, 0, bits, "kn.osort");
    }
    bounds_from_sorted(c, okeys, m, k, ostart);
    return m;
}
}  // namespace

namespace {
// the update after a fused fix-up: the other points' sums by label, the certified centroids,
// the sequential sums of the clusters the certificate fails.  Returns false when a flagged
// cluster has more members than k_nd_seq takes: those are summed over the member sort.
// the clusters k_nd_combine / k_nd_partials listed as heavy (heavy / nheavy on the device): their
// others' chunk records, then one wave each (no host sync)
template <int LD, bool SHARD>
void heavy_pass_t(st_ctx *c, int d, uint64_t n, int k, uint32_t m, const float *aos, const uint32_t *soff,
                  const double *psum, const double *pabs, const int *pemin, const uint32_t *pcnt,
                  const uint32_t *ostart, const uint32_t *ovals, const uint32_t *heavy, const uint32_t *nheavy,
                  float *cen, uint32_t *counts, uint32_t *flagged, uint32_t *nflagged, double *sums, double *sabs,
                  int32_t *emin) {
    (void)n;
    const uint32_t split = others_split(), chunk = others_chunk();
    const uint64_t chunks = m / chunk + m / split + 2;  // bound: every heavy cluster holds > split others
    auto *rsum = wsT<double>(c, "kn.hrsum", chunks * 64);
    auto *rabs = wsT<double>(c, "kn.hrabs", chunks * 64);
    auto *remin = wsT<int>(c, "kn.hremin", chunks * 64);
    hipLaunchKernelGGL((k_heavy<LD, SHARD>), dim3(grid_for(chunks, 1, 2048)), dim3(256), 0, c->stream, aos, d, k, soff,
                       psum, pabs, pemin, pcnt, ostart, ovals, heavy, nheavy, const_cast<uint32_t *>(nheavy) + 1, chunk, rsum, rabs, remin,
                       cen, counts, flagged, nflagged, sums, sabs, emin);
    ST_LAUNCH_CHECK();
}

template <bool SHARD>
void heavy_pass(st_ctx *c, int ld, int d, uint64_t n, int k, uint32_t m, const float *aos, const uint32_t *soff,
                const double *psum, const double *pabs, const int *pemin, const uint32_t *pcnt, const uint32_t *ostart,
                const uint32_t *ovals, const uint32_t *heavy, const uint32_t *nheavy, float *cen, uint32_t *counts,
                uint32_t *flagged, uint32_t *nflagged, double *sums, double *sabs, int32_t *emin) {
    if (m <= others_split()) return;  // no cluster can hold more others than there are
    if (ld == 48)
        heavy_pass_t<48, SHARD>(c, d, n, k, m, aos, soff, psum, pabs, pemin, pcnt, ostart, ovals, heavy, nheavy, cen,
                                counts, flagged, nflagged, sums, sabs, emin);
    else if (ld == 24)
        heavy_pass_t<24, SHARD>(c, d, n, k, m, aos, soff, psum, pabs, pemin, pcnt, ostart, ovals, heavy, nheavy, cen,
                                counts, flagged, nflagged, sums, sabs, emin);
    else
        heavy_pass_t<12, SHARD>(c, d, n, k, m, aos, soff, psum, pabs, pemin, pcnt, ostart, ovals, heavy, nheavy, cen,
                                counts, flagged, nflagged, sums, sabs, emin);
}

bool nd_fused_update(st_ctx *c, int d, uint64_t n, int k, const NdFused &fz, const uint32_t *labels, float *cen,
                     uint32_t *counts, State *dstate) {
    KTimer kt(c, "kn.sumnd");
    const int ld = aos_ld(d);
    auto *aos = wsT<float>(c, "kn.aos", n * (size_t)ld);
    const uint64_t slices = fz.ncodes + n / FA_SL + 1;
    auto *soff = wsT<uint32_t>(c, "kn.fasoff", (size_t)fz.ncodes + 1);
    auto *psum = wsT<double>(c, "kn.fasum", slices * 16 * ld);
    auto *pabs = wsT<double>(c, "kn.faabs", slices * 16 * ld);
    auto *pemin = wsT<int>(c, "kn.faemin", slices * 16 * ld);
    auto *pcnt = wsT<uint32_t>(c, "kn.facnt", slices * 16);
    const uint32_t m = others_sort(c, n, k, fz, labels);
    auto *ovals = wsT<uint32_t>(c, "kn.ovals", (size_t)m + 1);
    auto *ostart = wsT<uint32_t>(c, "kn.ostart", (size_t)k + 1);
    auto *flagged = wsT<uint32_t>(c, "kn.flagged", (size_t)k);
    // [0] flagged clusters, [1] collect overflow, [2] heavy clusters, [3] k_heavy's finished workgroups
    auto *nflag = wsT<uint32_t>(c, "kn.nflag", 4);
    const uint32_t split = others_split();
    auto *heavy = wsT<uint32_t>(c, "kn.heavy", (size_t)m / split + 2);
    ST_HIP(hipMemsetAsync(nflag, 0, 16, c->stream));
    const dim3 g((k + 3) / 4);
    if (ld == 48)
        hipLaunchKernelGGL(k_nd_combine<48>, g, dim3(256), 0, c->stream, aos, d, k, soff, psum, pabs, pemin, pcnt,
                           ostart, ovals, cen, counts, flagged, nflag, heavy, nflag + 2, split);
    else if (ld == 24)
        hipLaunchKernelGGL(k_nd_combine<24>, g, dim3(256), 0, c->stream, aos, d, k, soff, psum, pabs, pemin, pcnt,
                           ostart, ovals, cen, counts, flagged, nflag, heavy, nflag + 2, split);
    else
        hipLaunchKernelGGL(k_nd_combine<12>, g, dim3(256), 0, c->stream, aos, d, k, soff, psum, pabs, pemin, pcnt,
                           ostart, ovals, cen, counts, flagged, nflag, heavy, nflag + 2, split);
    ST_LAUNCH_CHECK();
    heavy_pass<false>(c, ld, d, n, k, m, aos, soff, psum, pabs, pemin, pcnt, ostart, ovals, heavy, nflag + 2, cen,
                      counts, flagged, nflag, nullptr, nullptr, nullptr);
    // the clusters the certificate fails: their members in point order, the sequential sums
    // (grid-stride over the flagged list; none: every workgroup returns at once)
    auto *big = wsT<uint32_t>(c, "kn.big", (size_t)k);
    hipLaunchKernelGGL(k_nd_seq, dim3(256), dim3(256), 0, c->stream, aos, d, k, flagged, nflag,
                       wsT<uint32_t>(c, "kn.fbpts1", n), wsT<uint32_t>(c, "kn.fbhist", fz.ncodes),
                       wsT<uint32_t>(c, "kn.fbcur", fz.ncodes), labels, ostart, ovals, cen, big, nflag + 1);
    ST_LAUNCH_CHECK();
    // the count of uncertified clusters too large for k_nd_seq is read at the next host sync
    // (nd_big_sums, before anything reads these centroids): no sync of its own
    auto *h = static_cast<uint32_t *>(pinned_slot(c, "kn.hflag", 8));
    ST_HIP(hipMemcpyAsync(h, nflag, 8, hipMemcpyDeviceToHost, c->stream));
    if (getenv("ST_DEBUG")) {
        ST_HIP(hipStreamSynchronize(c->stream));
        fprintf(stderr, "[st kmeans] fused update: others=%u uncertified clusters=%u over %u members=%u\n", m, h[0],
                NS_CAP, h[1]);
    }
    return true;
}

// the fused update's pending count (kn.hflag, copied behind its kernels): the clusters k_nd_seq
// left to the member sort get their sequential sums now.  Their rows are disjoint from the
// re-seeded (empty) ones queued in between.  Returns true when centroids changed.
bool nd_big_sums(st_ctx *c, int d, uint64_t n, int k, const uint32_t *labels, float *cen) {
    ST_HIP(hipStreamSynchronize(c->stream));
    const uint32_t nbig = static_cast<uint32_t *>(pinned_slot(c, "kn.hflag", 8))[1];
    if (!nbig) return false;
    auto *aos = wsT<float>(c, "kn.aos", n * (size_t)aos_ld(d));
    auto *sorted_labels = wsT<uint32_t>(c, "kn.slab", n);
    auto *members = wsT<uint32_t>(c, "kn.members", n);
    auto *start = wsT<uint32_t>(c, "kn.start", (size_t)k + 1);
    member_sort(c, labels, n, k, sorted_labels, members, start);
    // the listed clusters: one wave each up to sumnd_big() members, the huge ones (a cluster of
    // the table's all-zero rows) sliced over the chip (big_sums)
    const uint32_t big = sumnd_big();
    const uint32_t cap = (uint32_t)(n / ((uint64_t)big + 1) + 1);
    auto *list = wsT<uint32_t>(c, "kn.blist", cap);
    auto *nlist = wsT<uint32_t>(c, "kn.bn", 1);
    ST_HIP(hipMemsetAsync(nlist, 0, 4, c->stream));
    hipLaunchKernelGGL(k_sumnd<float>, dim3((nbig + 3) / 4), dim3(256), 0, c->stream, aos, d, members, start, k, cen,
                       big, cap, list, nlist, wsT<uint32_t>(c, "kn.big", (size_t)k), wsT<uint32_t>(c, "kn.nflag", 2) + 1);
    ST_LAUNCH_CHECK();
    if (n > big) big_sums(c, aos, d, n, k, members, start, cen, cap, list, nlist);
    return true;
}
}  // namespace

void nd_fused_partials(st_ctx *c, int d, uint64_t n, int k, const NdFused &fz, const uint32_t *labels, double *sums,
                       double *sabs, int32_t *emin, uint32_t *counts) {
    KTimer kt(c, "kn.partials");
    const int ld = aos_ld(d);
    auto *aos = wsT<float>(c, "kn.aos", n * (size_t)ld);
    const uint64_t slices = fz.ncodes + n / FA_SL + 1;
    auto *soff = wsT<uint32_t>(c, "kn.fasoff", (size_t)fz.ncodes + 1);
    auto *psum = wsT<double>(c, "kn.fasum", slices * 16 * ld);
    auto *pabs = wsT<double>(c, "kn.faabs", slices * 16 * ld);
    auto *pemin = wsT<int>(c, "kn.faemin", slices * 16 * ld);
    auto *pcnt = wsT<uint32_t>(c, "kn.facnt", slices * 16);
    const uint32_t m = others_sort(c, n, k, fz, labels);
    auto *ovals = wsT<uint32_t>(c, "kn.ovals", (size_t)m + 1);
    auto *ostart = wsT<uint32_t>(c, "kn.ostart", (size_t)k + 1);
    auto *nheavy = wsT<uint32_t>(c, "kn.pnheavy", 2);  // [0] heavy clusters, [1] k_heavy's finished workgroups
    const uint32_t split = others_split();
    auto *heavy = wsT<uint32_t>(c, "kn.heavy", (size_t)m / split + 2);
    ST_HIP(hipMemsetAsync(nheavy, 0, 8, c->stream));
    const dim3 g((k + 3) / 4);
    if (ld == 48)
        hipLaunchKernelGGL(k_nd_partials<48>, g, dim3(256), 0, c->stream, aos, d, k, soff, psum, pabs, pemin, pcnt,
                           ostart, ovals, sums, sabs, emin, counts, heavy, nheavy, split);
    else if (ld == 24)
        hipLaunchKernelGGL(k_nd_partials<24>, g, dim3(256), 0, c->stream, aos, d, k, soff, psum, pabs, pemin, pcnt,
                           ostart, ovals, sums, sabs, emin, counts, heavy, nheavy, split);
    else
        hipLaunchKernelGGL(k_nd_partials<12>, g, dim3(256), 0, c->stream, aos, d, k, soff, psum, pabs, pemin, pcnt,
                           ostart, ovals, sums, sabs, emin, counts, heavy, nheavy, split);
    ST_LAUNCH_CHECK();
    heavy_pass<true>(c, ld, d, n, k, m, aos, soff, psum, pabs, pemin, pcnt, ostart, ovals, heavy, nheavy, nullptr,
                     counts, nullptr, nullptr, sums, sabs, emin);
}

void kmeansnd_loop(st_ctx *c, const float *const *cols, const float *const *dcols, int d, uint64_t n, int k,
                   int iters, const double *ddraws, uint64_t ndraws, km::State *dstate, float *cen, uint32_t *labels,
                   const double *const *sum64) {
    (void)cols;
    // one device: the assign's pair / ambiguous fix-ups overlap the decided points' (nd_assign_core)
    struct Overlap {
        st_ctx *c;
        bool was;
        ~Overlap() { c->fix_overlap = was; }
    } overlap{c, c->fix_overlap};
    c->fix_overlap = true;
    auto *aos = wsT<float>(c, "kn.aos", n * (size_t)aos_ld(d));
    double *aos64 = nullptr;
    if (sum64) {  // the members' float64 numbers for the sums
        aos64 = wsT<double>(c, "kn.aos64", n * (size_t)aos_ld(d));
        auto **d64 = wsT<const double *>(c, "kn.cols64", (size_t)d);
        ST_HIP(hipMemcpyAsync(d64, sum64, sizeof(double *) * d, hipMemcpyHostToDevice, c->stream));
        hipLaunchKernelGGL(k_aos64, dim3(grid_for(n * aos_ld(d), 256, 8192)), dim3(256), 0, c->stream, d64, d, n,
                           aos64);
        ST_LAUNCH_CHECK();
    }
    auto *sorted_labels = wsT<uint32_t>(c, "kn.slab", n);
    auto *members = wsT<uint32_t>(c, "kn.members", n);
    auto *start = wsT<uint32_t>(c, "kn.start", (size_t)k + 1);
    auto *counts = wsT<uint32_t>(c, "kn.counts", (size_t)k);
    nd_prepare(c, dcols, d, n);
    const size_t cbytes = (size_t)k * d * sizeof(float);
    // a fused update's large uncertified clusters are summed at the next assign's first sync
    bool pending = false;
    const std::function<bool()> settle = [&]() {
        pending = false;
        return nd_big_sums(c, d, n, k, labels, cen);
    };
    for (int it = 0; it < iters; ++it) {
        // a speculative host form whose compare found the host columns changed stops here
        if (c->spec_abort && c->spec_abort->load(std::memory_order_relaxed)) throw SpecAbort();
        if (pending && c->verify && it == iters - 1) settle();
        if (c->verify && it == iters - 1)
            ST_HIP(hipMemcpyAsync(ws(c, "verify.prev", cbytes), cen, cbytes, hipMemcpyDeviceToDevice, c->stream));
        NdFused fz;
        fz.want = !aos64 && !getenv("ST_ND_SORT");
        nd_assign(c, dcols, d, n, k, cen, labels, dstate, &fz, pending ? settle : std::function<bool()>());
        // update
        if (fz.valid && nd_fused_update(c, d, n, k, fz, labels, cen, counts, dstate)) {
            reseed_empty_counts(c, dcols, d, n, k, counts, ddraws, ndraws, dstate, cen);
            pending = true;
        } else {
            member_sort(c, labels, n, k, sorted_labels, members, start);
            {
                KTimer kt(c, "kn.sumnd");
                if (aos64) launch_sums<double>(c, aos64, d, n, k, members, start, cen);
                else launch_sums<float>(c, aos, d, n, k, members, start, cen);
            }
            reseed_empty(c, dcols, d, n, k, start, ddraws, ndraws, dstate, cen);
        }
        mark(c, "kn.update");
    }
    if (pending) settle();
    if (c->verify && iters > 0) {
        ST_HIP(hipMemcpyAsync(ws(c, "verify.cen", cbytes), cen, cbytes, hipMemcpyDeviceToDevice, c->stream));
        ST_HIP(hipMemcpyAsync(ws(c, "verify.labels", n * 4), labels, n * 4, hipMemcpyDeviceToDevice, c->stream));
        c->vf_d = d;
        c->vf_k = k;
        c->vf_n = n;
    }
}

}  // namespace st

