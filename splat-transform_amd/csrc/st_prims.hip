// st_prims.hip -- device-wide primitives: exclusive scan and stable LSD radix sort.
//
// Radix sort: 8-bit digits, reduce-then-scan per pass.  A block owns a tile of
// 4096 keys; each of its four waves owns a contiguous quarter, visited in 16
// rows of 64 lanes, so (wave, row, lane) order == input order.  Within a row a
// key's stable rank among equal digits comes from 8 ballots (wave64 match),
// per-wave digit counters live in LDS, and a per-digit prefix over the waves
// plus the global (digit, block) offset gives the output slot.  Stability is
// what ordering.ts:82-83 (V8's stable TypedArray.sort) and the in-cluster
// member order of k-means.ts:123-135 require.
#include "st_internal.h"

namespace st {

namespace {

constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;

__device__ inline uint32_t wave_inclusive_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    return v;
}

// exclusive scan of the 256 per-thread values of a block; returns block total via *total
__device__ inline uint32_t block_exclusive_scan(uint32_t v, uint32_t *total) {
    __shared__ uint32_t wsum[SCAN_THREADS / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = wave_inclusive_scan(v);
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < SCAN_THREADS / 64; ++i) {
        if (i < w) before += wsum[i];
        tot += wsum[i];
    }
    __syncthreads();
    *total = tot;
    return before + inc - v;
}

__global__ __launch_bounds__(SCAN_THREADS) void k_scan_reduce(const uint32_t *__restrict__ in, uint64_t n,
                                                              uint32_t *__restrict__ partial) {
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i)
        if (base + i < n) s += in[base + i];
    uint32_t tot;
    block_exclusive_scan(s, &tot);
    if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SCAN_THREADS) void k_scan_down(const uint32_t *in, uint64_t n, uint32_t *out,
                                                            const uint32_t *__restrict__ partial_ex,
                                                            uint32_t *d_total, int write_total) {
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS];
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        v[i] = (base + i < n) ? in[base + i] : 0u;
        s += v[i];
    }
    uint32_t tot;
    uint32_t ex = block_exclusive_scan(s, &tot) + (partial_ex ? partial_ex[blockIdx.x] : 0u);
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        if (base + i < n) out[base + i] = ex;
        ex += v[i];
    }
    if (write_total && d_total && blockIdx.x == gridDim.x - 1 && threadIdx.x == SCAN_THREADS - 1) *d_total = ex;
}

__global__ void k_iota(uint32_t *out, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = (uint32_t)i;
}

// ---------------------------------------------------------------------------
constexpr int RS_THREADS = 256;
constexpr int RS_ROWS = 16;
constexpr int RS_WAVES = RS_THREADS / 64;
constexpr int RS_TILE = RS_THREADS * RS_ROWS;  // 4096
static_assert(RS_TILE == RADIX_TILE, "st_internal.h's tile size");
constexpr int RS_WAVE_SPAN = 64 * RS_ROWS;     // 1024

// per-tile digit counts: one LDS histogram per wave (less same-bin contention), 32-bit keys
// read as four 16-byte quads per thread on whole aligned tiles
template <typename K>
__global__ __launch_bounds__(RS_THREADS) void k_rs_hist(const K *__restrict__ keys, uint64_t n, int shift, int bits,
                                                        uint32_t *__restrict__ hist, uint32_t nblocks) {
    __shared__ uint32_t h[RS_WAVES][256];
    for (int i = threadIdx.x; i < RS_WAVES * 256; i += RS_THREADS) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
    const uint32_t mask = (1u << bits) - 1u;
    uint32_t *hw = h[threadIdx.x >> 6];
    bool quads = false;
    if constexpr (sizeof(K) == 4) quads = base + RS_TILE <= n && (((uintptr_t)(keys + base)) & 15u) == 0;
    if (quads) {
        const uint4 *k4 = reinterpret_cast<const uint4 *>(keys + base);
        uint4 q[RS_ROWS / 4];
#pragma unroll
        for (int r = 0; r < RS_ROWS / 4; ++r) q[r] = k4[r * RS_THREADS + threadIdx.x];
#pragma unroll
        for (int r = 0; r < RS_ROWS / 4; ++r) {
            atomicAdd(&hw[(q[r].x >> shift) & mask], 1u);
            atomicAdd(&hw[(q[r].y >> shift) & mask], 1u);
            atomicAdd(&hw[(q[r].z >> shift) & mask], 1u);
            atomicAdd(&hw[(q[r].w >> shift) & mask], 1u);
        }
    } else {
#pragma unroll 4
        for (int r = 0; r < RS_ROWS; ++r) {
            const uint64_t e = base + (uint64_t)r * RS_THREADS + threadIdx.x;
            if (e < n) atomicAdd(&hw[(uint32_t)(keys[e] >> shift) & mask], 1u);
        }
    }
    __syncthreads();
    uint32_t t = 0;
#pragma unroll
    for (int i = 0; i < RS_WAVES; ++i) t += h[i][threadIdx.x];
    hist[(uint64_t)threadIdx.x * nblocks + blockIdx.x] = t;
}

// One tile of RS_TILE elements: wave-level ranks by ballot (stable), then the tile is
// reordered by digit in LDS so each digit's run leaves as consecutive addresses
// (coalesced stores) at its global offset.
template <typename K>
__global__ __launch_bounds__(RS_THREADS) void k_rs_scatter(const K *__restrict__ keys, const uint32_t *__restrict__ vals,
                                                           uint64_t n, int shift, int bits,
                                                           const uint32_t *__restrict__ offs, uint32_t nblocks,
                                                           K *__restrict__ okeys, uint32_t *__restrict__ ovals) {
    __shared__ uint32_t wcount[RS_WAVES][256];
    __shared__ uint32_t wbase[RS_WAVES][256];
    __shared__ uint32_t goff[256];
    __shared__ uint32_t dstart[256];  // first local position of each digit
    __shared__ uint32_t wtot[RS_WAVES];
    __shared__ K sk[RS_TILE];
    __shared__ uint32_t sv[RS_TILE];
    for (int i = threadIdx.x; i < RS_WAVES * 256; i += RS_THREADS) (&wcount[0][0])[i] = 0;
    goff[threadIdx.x] = offs[(uint64_t)threadIdx.x * nblocks + blockIdx.x];
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const uint32_t mask = (1u << bits) - 1u;
    const uint64_t tbase = (uint64_t)blockIdx.x * RS_TILE;
    const uint64_t wbase_e = tbase + (uint64_t)w * RS_WAVE_SPAN;
    K k[RS_ROWS];
    uint32_t v[RS_ROWS];
    uint32_t off[RS_ROWS];
    uint32_t dg[RS_ROWS];
#pragma unroll
    for (int r = 0; r < RS_ROWS; ++r) {
        const uint64_t e = wbase_e + (uint64_t)r * 64 + lane;
        const bool valid = e < n;
        k[r] = valid ? keys[e] : (K)0;
        v[r] = valid ? (vals ? vals[e] : (uint32_t)e) : 0u;  // no vals: the identity permutation
    }
#pragma unroll
    for (int r = 0; r < RS_ROWS; ++r) {
        const uint64_t e = wbase_e + (uint64_t)r * 64 + lane;
        const bool valid = e < n;
        const uint32_t d = (uint32_t)(k[r] >> shift) & mask;
        dg[r] = d;
        uint64_t peers = __ballot(valid);
        for (int b = 0; b < bits; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint32_t rank = __popcll(peers & lt);
        const uint32_t before = valid ? wcount[w][d] : 0u;
        off[r] = before + rank;
        const bool leader = valid && ((peers & lt) == 0);
        if (leader) wcount[w][d] = before + (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    {
        // per digit: offsets of the waves, and the digit's total for the tile
        const int d = threadIdx.x;
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < RS_WAVES; ++i) {
            wbase[i][d] = s;
            s += wcount[i][d];
        }
        // exclusive scan of the digit totals across the block (256 threads)
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
    for (int r = 0; r < RS_ROWS; ++r) {
        const uint64_t e = wbase_e + (uint64_t)r * 64 + lane;
        if (e < n) {
            const uint32_t lp = dstart[dg[r]] + wbase[w][dg[r]] + off[r];
            sk[lp] = k[r];
            sv[lp] = v[r];
        }
    }
    __syncthreads();
    const uint32_t cnt = (uint32_t)((n - tbase) < (uint64_t)RS_TILE ? (n - tbase) : (uint64_t)RS_TILE);
    for (uint32_t i = threadIdx.x; i < cnt; i += RS_THREADS) {
        const K kk = sk[i];
        const uint32_t d = (uint32_t)(kk >> shift) & mask;
        const uint32_t pos = goff[d] + (i - dstart[d]);
        okeys[pos] = kk;
        ovals[pos] = sv[i];
    }
}

// ---- min/max of columns as order-preserving keys (NaN skipped), two stages ----------
// Stage 1: gridDim.y = column, each workgroup reduces a contiguous slice (float4 loads
// when the column is 16-byte aligned, 4 quads in flight per thread) to one partial;
// stage 2: one workgroup per column.  No same-address atomics (a few thousand workgroups
// hammering six words cost more than the reads).
constexpr int MM_BLOCKS = 512;
__device__ inline uint32_t mm_key(float v) {
    const uint32_t u = __builtin_bit_cast(uint32_t, v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline void mm_take(float v, uint32_t &lo, uint32_t &hi) {
    if (v == v) {
        const uint32_t k = mm_key(v);
        lo = k < lo ? k : lo;
        hi = k > hi ? k : hi;
    }
}
__device__ inline void mm_block(uint32_t &lo, uint32_t &hi) {
    __shared__ uint32_t slo[4], shi[4];
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t t0 = __shfl_xor(lo, o, 64), t1 = __shfl_xor(hi, o, 64);
        lo = t0 < lo ? t0 : lo;
        hi = t1 > hi ? t1 : hi;
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        slo[w] = lo;
        shi[w] = hi;
    }
    __syncthreads();
    lo = min(min(slo[0], slo[1]), min(slo[2], slo[3]));
    hi = max(max(shi[0], shi[1]), max(shi[2], shi[3]));
}
struct MMCols {
    const float *p[64];
};
__global__ __launch_bounds__(256) void k_mm_partial(const MMCols cols, uint64_t n, uint32_t *__restrict__ part) {
    const float *v = cols.p[blockIdx.y];
    const uint64_t per = ((n + gridDim.x - 1) / gridDim.x + 3) & ~(uint64_t)3;  // slices keep 16-B alignment
    const uint64_t a = min(n, (uint64_t)blockIdx.x * per), b = min(n, a + per);
    uint32_t lo = 0xffffffffu, hi = 0;
    if ((((uintptr_t)(v + a)) & 15u) == 0) {
        const uint64_t nq = (b - a) / 4;
        const float4 *v4 = reinterpret_cast<const float4 *>(v + a);
        uint64_t q = threadIdx.x;
        for (; q + 3 * 256 < nq; q += 4 * 256) {
            float4 t[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) t[u] = v4[q + u * 256];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                mm_take(t[u].x, lo, hi);
                mm_take(t[u].y, lo, hi);
                mm_take(t[u].z, lo, hi);
                mm_take(t[u].w, lo, hi);
            }
        }
        for (; q < nq; q += 256) {
            const float4 t = v4[q];
            mm_take(t.x, lo, hi);
            mm_take(t.y, lo, hi);
            mm_take(t.z, lo, hi);
            mm_take(t.w, lo, hi);
        }
        for (uint64_t i = a + nq * 4 + threadIdx.x; i < b; i += 256) mm_take(v[i], lo, hi);
    } else {
        for (uint64_t i = a + threadIdx.x; i < b; i += 256) mm_take(v[i], lo, hi);
    }
    mm_block(lo, hi);
    if (threadIdx.x == 0) {
        part[(uint64_t)blockIdx.y * 2 * gridDim.x + blockIdx.x] = lo;
        part[(uint64_t)blockIdx.y * 2 * gridDim.x + gridDim.x + blockIdx.x] = hi;
    }
}
__global__ __launch_bounds__(256) void k_mm_final(const uint32_t *__restrict__ part, int nb, uint32_t *__restrict__ out) {
    const uint32_t *p = part + (uint64_t)blockIdx.x * 2 * nb;
    uint32_t lo = 0xffffffffu, hi = 0;
    for (int i = threadIdx.x; i < nb; i += 256) {
        lo = min(lo, p[i]);
        hi = max(hi, p[nb + i]);
    }
    mm_block(lo, hi);
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = lo;
        out[2 * blockIdx.x + 1] = hi;
    }
}

// stable sort of at most SS_MAX pairs in one workgroup: every element's rank is the count
// of smaller keys plus equal keys before it (the LDS reads of key j are broadcasts).  Short
// sorts -- the 256 centroids of every 1-D k-means iteration -- were 4 passes x 3 launches
constexpr uint32_t SS_MAX = 2048;
constexpr int SS_T = 1024;
template <typename K>
__global__ __launch_bounds__(SS_T) void k_small_sort(K *__restrict__ keys, uint32_t *__restrict__ vals, uint32_t n,
                                                     int shift, int bits) {
    __shared__ K sk[SS_MAX];
    __shared__ uint32_t sv[SS_MAX];
    for (uint32_t i = threadIdx.x; i < n; i += SS_T) {
        sk[i] = keys[i];
        sv[i] = vals[i];
    }
    __syncthreads();
    const K mask = bits >= (int)(8 * sizeof(K)) ? ~(K)0 : (((K)1 << bits) - 1);
    K mine[SS_MAX / SS_T];
    uint32_t rank[SS_MAX / SS_T];
#pragma unroll
    for (int u = 0; u < (int)(SS_MAX / SS_T); ++u) {
        const uint32_t e = threadIdx.x + u * SS_T;
        mine[u] = e < n ? (sk[e] >> shift) & mask : (K)0;
        rank[u] = 0;
    }
    // eight broadcast LDS reads in flight per step: the loop was bound by one read's latency
    constexpr uint32_t SU = 8;
    uint32_t j = 0;
    for (; j + SU <= n; j += SU) {
        K kj[SU];
#pragma unroll
        for (uint32_t q = 0; q < SU; ++q) kj[q] = (sk[j + q] >> shift) & mask;
#pragma unroll
        for (uint32_t q = 0; q < SU; ++q)
#pragma unroll
            for (int u = 0; u < (int)(SS_MAX / SS_T); ++u) {
                const uint32_t e = threadIdx.x + u * SS_T;
                rank[u] += (kj[q] < mine[u] || (kj[q] == mine[u] && j + q < e)) ? 1u : 0u;
            }
    }
    for (; j < n; ++j) {
        const K kj = (sk[j] >> shift) & mask;
#pragma unroll
        for (int u = 0; u < (int)(SS_MAX / SS_T); ++u) {
            const uint32_t e = threadIdx.x + u * SS_T;
            rank[u] += (kj < mine[u] || (kj == mine[u] && j < e)) ? 1u : 0u;
        }
    }
#pragma unroll
    for (int u = 0; u < (int)(SS_MAX / SS_T); ++u) {
        const uint32_t e = threadIdx.x + u * SS_T;
        if (e < n) {
            keys[rank[u]] = sk[e];
            vals[rank[u]] = sv[e];
        }
    }
}

// stable sort of at most 256 u32-keyed pairs in one wave: a bitonic network over the
// composite (digit bits << 32 | input position), unique keys, so the network's order is the
// stable one; element i = r * 64 + lane, partners at distance < 64 by shuffles, larger ones
// inside the lane's four registers.  (The rank sort above spent 23 us on the 256 centroids of
// every 1-D k-means iteration: sixteen waves of one CU re-reading LDS.)
__global__ __launch_bounds__(64) void k_sort256(uint32_t *__restrict__ keys, uint32_t *__restrict__ vals, uint32_t n,
                                                int shift, int bits) {
    const int lane = threadIdx.x;
    const uint32_t mask = bits >= 32 ? 0xffffffffu : ((1u << bits) - 1u);
    uint64_t v[4];
    uint32_t kin[4], vin[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t i = r * 64 + lane;
        kin[r] = i < n ? keys[i] : 0u;
        vin[r] = i < n ? vals[i] : 0u;
        v[r] = i < n ? (((uint64_t)((kin[r] >> shift) & mask) << 32) | i) : ~0ull;
    }
#pragma unroll
    for (uint32_t k = 2; k <= 256; k <<= 1) {
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            uint64_t nv[4];  // every partner value is read before any is replaced
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t i = r * 64 + lane;
                const uint64_t o = j < 64 ? __shfl_xor(v[r], (int)j, 64) : v[r ^ (int)(j >> 6)];
                const bool up = (i & k) == 0, lower = (i & j) == 0;
                const uint64_t lo = v[r] < o ? v[r] : o, hi = v[r] < o ? o : v[r];
                nv[r] = (up == lower) ? lo : hi;
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = nv[r];
        }
    }
    // inputs to LDS, then the sorted order reads them by position
    __shared__ uint32_t sk[256], sv[256];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        sk[r * 64 + lane] = kin[r];
        sv[r * 64 + lane] = vin[r];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t i = r * 64 + lane;
        if (i < n) {
            const uint32_t src = (uint32_t)v[r];
            keys[i] = sk[src];
            vals[i] = sv[src];
        }
    }
}

template <typename K>
void radix_sort_impl(st_ctx *c, K *keys, uint32_t *vals, uint64_t n, int begin_bit, int end_bit,
                     const std::string &tag, K **out_keys = nullptr, uint32_t **out_vals = nullptr) {
    if (out_keys) *out_keys = keys;
    if (out_vals) *out_vals = vals;
    if (n <= 1 || end_bit <= begin_bit) return;
    ST_REQUIRE(n < (1ull << 32), ST_ERR_ARG, "radix sort: n must be < 2^32");
    if (sizeof(K) == 4 && n <= 256) {  // in place, one wave
        hipLaunchKernelGGL(k_sort256, dim3(1), dim3(64), 0, c->stream, reinterpret_cast<uint32_t *>(keys), vals,
                           (uint32_t)n, begin_bit, end_bit - begin_bit);
        ST_LAUNCH_CHECK();
        return;
    }
    if (n <= SS_MAX) {  // in place, one launch
        hipLaunchKernelGGL(k_small_sort<K>, dim3(1), dim3(SS_T), 0, c->stream, keys, vals, (uint32_t)n, begin_bit,
                           end_bit - begin_bit);
        ST_LAUNCH_CHECK();
        return;
    }
    const uint32_t nblocks = (uint32_t)((n + RS_TILE - 1) / RS_TILE);
    K *k2 = wsT<K>(c, tag + ".k2", n);
    uint32_t *v2 = wsT<uint32_t>(c, tag + ".v2", n);
    uint32_t *hist = wsT<uint32_t>(c, tag + ".hist", (uint64_t)256 * nblocks);
    K *ka = keys, *kb = k2;
    uint32_t *va = vals, *vb = v2;
    int passes = 0;
    for (int shift = begin_bit; shift < end_bit; shift += 8) {
        const int bits = (end_bit - shift) < 8 ? (end_bit - shift) : 8;
        hipLaunchKernelGGL(k_rs_hist<K>, dim3(nblocks), dim3(RS_THREADS), 0, c->stream, ka, n, shift, bits, hist,
                           nblocks);
        ST_LAUNCH_CHECK();
        scan_u32(c, hist, hist, (uint64_t)256 * nblocks, nullptr);
        hipLaunchKernelGGL(k_rs_scatter<K>, dim3(nblocks), dim3(RS_THREADS), 0, c->stream, ka, va, n, shift, bits,
                           hist, nblocks, kb, vb);
        ST_LAUNCH_CHECK();
        std::swap(ka, kb);
        std::swap(va, vb);
        ++passes;
    }
    if (out_keys) {  // the caller takes the result where the last pass left it
        *out_keys = ka;
        *out_vals = va;
        return;
    }
    if (passes & 1) {
        ST_HIP(hipMemcpyAsync(keys, ka, n * sizeof(K), hipMemcpyDeviceToDevice, c->stream));
        ST_HIP(hipMemcpyAsync(vals, va, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, c->stream));
    }
}

}  // namespace

void scan_u32(st_ctx *c, const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *d_total) {
    if (n == 0) {
        if (d_total) ST_HIP(hipMemsetAsync(d_total, 0, sizeof(uint32_t), c->stream));
        return;
    }
    const uint64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    if (nb == 1) {
        hipLaunchKernelGGL(k_scan_down, dim3(1), dim3(SCAN_THREADS), 0, c->stream, in, n, out, nullptr, d_total, 1);
        ST_LAUNCH_CHECK();
        return;
    }
    // per-level partial buffers keyed by size class so nested scans do not collide
    std::string tag = "scan.p" + std::to_string(nb);
    uint32_t *partial = wsT<uint32_t>(c, tag, nb + 1);
    hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)nb), dim3(SCAN_THREADS), 0, c->stream, in, n, partial);
    ST_LAUNCH_CHECK();
    scan_u32(c, partial, partial, nb, partial + nb);
    hipLaunchKernelGGL(k_scan_down, dim3((unsigned)nb), dim3(SCAN_THREADS), 0, c->stream, in, n, out, partial,
                       nullptr, 0);
    ST_LAUNCH_CHECK();
    if (d_total) ST_HIP(hipMemcpyAsync(d_total, partial + nb, sizeof(uint32_t), hipMemcpyDeviceToDevice, c->stream));
}

// stable sort of in_keys (left unchanged) with in_vals (null: the identity permutation) as
// values: the first pass reads the inputs, the passes alternate so the last writes out_*
void radix_sort_u32_from(st_ctx *c, const uint32_t *in_keys, const uint32_t *in_vals, uint64_t n, int b0, int b1,
                         uint32_t *out_keys, uint32_t *out_vals, uint32_t *hist0, const std::string &tag) {
    if (n == 0) return;
    const int passes = (b1 - b0 + 7) / 8;
    ST_REQUIRE(!(((in_vals && in_vals == out_vals) || in_keys == out_keys) && (passes & 1)), ST_ERR_INTERNAL,
               "radix sort: in-place outputs need an even pass count");
    if (n <= SS_MAX || passes == 0) {
        if (out_keys != in_keys)
            ST_HIP(hipMemcpyAsync(out_keys, in_keys, n * 4, hipMemcpyDeviceToDevice, c->stream));
        if (!in_vals) iota_u32(c, out_vals, n);
        else if (out_vals != in_vals)
            ST_HIP(hipMemcpyAsync(out_vals, in_vals, n * 4, hipMemcpyDeviceToDevice, c->stream));
        radix_sort_impl<uint32_t>(c, out_keys, out_vals, n, b0, b1, tag);
        return;
    }
    ST_REQUIRE(n < (1ull << 32), ST_ERR_ARG, "radix sort: n must be < 2^32");
    const uint32_t nblocks = (uint32_t)((n + RS_TILE - 1) / RS_TILE);
    uint32_t *k2 = wsT<uint32_t>(c, tag + ".k2", n);
    uint32_t *v2 = wsT<uint32_t>(c, tag + ".v2", n);
    uint32_t *hist = hist0 ? hist0 : wsT<uint32_t>(c, tag + ".hist", (uint64_t)256 * nblocks);
    // an even number of passes starts into the scratch pair, an odd one into out_*
    uint32_t *dk = (passes & 1) ? out_keys : k2, *dv = (passes & 1) ? out_vals : v2;
    const uint32_t *ka = in_keys, *va = in_vals;
    for (int shift = b0, p = 0; shift < b1; shift += 8, ++p) {
        const int bits = (b1 - shift) < 8 ? (b1 - shift) : 8;
        if (p > 0 || !hist0) {
            hipLaunchKernelGGL(k_rs_hist<uint32_t>, dim3(nblocks), dim3(RS_THREADS), 0, c->stream, ka, n, shift, bits,
                               hist, nblocks);
            ST_LAUNCH_CHECK();
        }
        scan_u32(c, hist, hist, (uint64_t)256 * nblocks, nullptr);
        hipLaunchKernelGGL(k_rs_scatter<uint32_t>, dim3(nblocks), dim3(RS_THREADS), 0, c->stream, ka, va, n, shift,
                           bits, hist, nblocks, dk, dv);
        ST_LAUNCH_CHECK();
        ka = dk;
        va = dv;
        const bool to_out = dk == out_keys;
        dk = to_out ? k2 : out_keys;
        dv = to_out ? v2 : out_vals;
    }
}

void radix_sort_u32_iota(st_ctx *c, const uint32_t *in_keys, uint64_t n, int b0, int b1, uint32_t *out_keys,
                         uint32_t *out_vals, const std::string &tag) {
    radix_sort_u32_from(c, in_keys, nullptr, n, b0, b1, out_keys, out_vals, nullptr, tag);
}

void radix_sort_u32(st_ctx *c, uint32_t *keys, uint32_t *vals, uint64_t n, int b0, int b1, const std::string &tag) {
    radix_sort_impl<uint32_t>(c, keys, vals, n, b0, b1, tag);
}

void radix_sort_u32_inplace_or_swap(st_ctx *c, uint32_t *keys, uint32_t *vals, uint64_t n, int b0, int b1,
                                    const std::string &tag, uint32_t **out_keys, uint32_t **out_vals) {
    radix_sort_impl<uint32_t>(c, keys, vals, n, b0, b1, tag, out_keys, out_vals);
}

void radix_sort_u64(st_ctx *c, uint64_t *keys, uint32_t *vals, uint64_t n, int b0, int b1, const std::string &tag) {
    radix_sort_impl<uint64_t>(c, keys, vals, n, b0, b1, tag);
}

void minmax_keys_dev(st_ctx *c, const float *const *cols, int ncols, uint64_t n, uint32_t *out) {
    ST_REQUIRE(ncols >= 1 && ncols <= 64, ST_ERR_ARG, "minmax: 1..64 columns");
    MMCols mc{};
    for (int i = 0; i < ncols; ++i) mc.p[i] = cols[i];
    const unsigned nb = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(MM_BLOCKS, (n + 4095) / 4096));
    auto *part = wsT<uint32_t>(c, "mm.part", (size_t)ncols * 2 * nb);
    hipLaunchKernelGGL(k_mm_partial, dim3(nb, ncols), dim3(256), 0, c->stream, mc, n, part);
    hipLaunchKernelGGL(k_mm_final, dim3(ncols), dim3(256), 0, c->stream, part, (int)nb, out);
    ST_LAUNCH_CHECK();
}

void iota_u32(st_ctx *c, uint32_t *out, uint64_t n) {
    if (!n) return;
    hipLaunchKernelGGL(k_iota, dim3(grid_for(n, 256, 4096)), dim3(256), 0, c->stream, out, n);
    ST_LAUNCH_CHECK();
}

}  // namespace st
