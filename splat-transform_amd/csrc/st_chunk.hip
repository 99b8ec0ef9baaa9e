// st_chunk.hip -- compressed-PLY chunk packing (write-compressed-ply.ts:56-109,
// CompressedChunk.pack compressed-chunk.ts:44-180).
//
// One 256-thread workgroup per 256-splat chunk, one lane per splat of the
// Morton order.  Per-chunk min/max use Math.min/Math.max semantics (NaN
// propagates, -0 < +0) through wave64 shuffles + LDS; the quantisers run in
// f64 exactly as the JS; the final partial chunk is padded with its last
// splat (write-compressed-ply.ts:90-93).  HBM traffic per splat: the column
// transpose (14 + 3C floats read, the padded row written), one gathered row,
// 16 B vertex + 3C bytes SH out.
#include <cstdlib>

#include "st_internal.h"
#include "st_jsmath.h"

namespace st {
namespace {

constexpr double SH_C0 = 0.28209479177387814;

// Math.min / Math.max with a NaN operand return V8's NaN, the x86-64 default NaN (sign bit
// set): stored to the Float32Array chunk it is 0xffc00000 (reference fixture process_chain)
__device__ inline float js_nan() { return __builtin_bit_cast(float, 0xffc00000u); }

__device__ inline float jmin(float a, float b) {
    if (a != a || b != b) return js_nan();
    if (a == b) return __builtin_signbit(a) ? a : b;
    return a < b ? a : b;
}
__device__ inline float jmax(float a, float b) {
    if (a != a || b != b) return js_nan();
    if (a == b) return __builtin_signbit(a) ? b : a;
    return a > b ? a : b;
}

// JS min and max over the 256 lanes of the block for NV values each
template <int NV>
__device__ inline void block_minmax(float (&mn)[NV], float (&mx)[NV]) {
    __shared__ float smn[NV][4], smx[NV][4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            mn[v] = jmin(mn[v], __shfl_xor(mn[v], o, 64));
            mx[v] = jmax(mx[v], __shfl_xor(mx[v], o, 64));
        }
        if (lane == 0) {
            smn[v][w] = mn[v];
            smx[v][w] = mx[v];
        }
    }
    __syncthreads();
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        mn[v] = jmin(jmin(smn[v][0], smn[v][1]), jmin(smn[v][2], smn[v][3]));
        mx[v] = jmax(jmax(smx[v][0], smx[v][1]), jmax(smx[v][2], smx[v][3]));
    }
    __syncthreads();
}

__device__ inline double normalize01(double x, double mn, double mx) {
    if (x <= mn) return 0;
    if (x >= mx) return 1;
    return (mx - mn < 0.00001) ? 0 : (x - mn) / (mx - mn);
}

__device__ inline uint32_t pack_unorm(double value, int bits) {
    const double t = (double)((1 << bits) - 1);
    return (uint32_t)js::to_int32(js::max_(0, js::min_(t, __builtin_floor(value * t + 0.5))));
}

__device__ inline uint32_t pack111011(double x, double y, double z) {
    return (pack_unorm(x, 11) << 21) | (pack_unorm(y, 10) << 11) | pack_unorm(z, 11);
}

__device__ inline uint32_t pack8888(double x, double y, double z, double w) {
    return (pack_unorm(x, 8) << 24) | (pack_unorm(y, 8) << 16) | (pack_unorm(z, 8) << 8) | pack_unorm(w, 8);
}

// packRot: Quat(x=rot_0, y=rot_1, z=rot_2, w=rot_3).normalize(), smallest-three 2+10+10+10
__device__ inline uint32_t pack_rot(double x, double y, double z, double w) {
    double len = __builtin_sqrt(x * x + y * y + z * z + w * w);
    double a[4];
    if (len == 0) {
        a[0] = a[1] = a[2] = 0;
        a[3] = 1;
    } else {
        len = 1 / len;
        a[0] = x * len;
        a[1] = y * len;
        a[2] = z * len;
        a[3] = w * len;
    }
    int largest = 0;
#pragma unroll
    for (int i = 1; i < 4; ++i)
        if (__builtin_fabs(a[i]) > __builtin_fabs(a[largest])) largest = i;
    if (a[largest] < 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = -a[i];
    }
    const double norm = __builtin_sqrt(2.0) * 0.5;
    uint32_t result = (uint32_t)largest;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (i != largest) result = (result << 10) | pack_unorm(a[i] * norm + 0.5, 10);
    return result;
}

// Rows are gathered through the Morton order, i.e. at random.  Gathering 59 SoA
// columns would touch one cache line per (splat, column); the columns are first
// transposed (streaming, coalesced) into 16-byte-aligned AoS rows of RL floats
// ([14 members][3C SH][pad]) so a gathered row is RL*4 contiguous bytes.
struct TransposeArgs {
    const float *src[64];
    int ncol, rl;
    uint64_t n;
    float *rows;
};

// RA_ROWS rows per block through LDS: coalesced column reads (all of a thread's loads issued
// before the first LDS store), coalesced row writes
constexpr int RA_ROWS = 256;
__global__ __launch_bounds__(256) void k_rows_aos(const TransposeArgs a) {
    __shared__ float tile[RA_ROWS * 16];  // rl <= 16
    const uint64_t r0 = (uint64_t)blockIdx.x * RA_ROWS;
    const int t = threadIdx.x;
    const uint64_t row = r0 + t;
    const uint64_t rsafe = row < a.n ? row : a.n - 1;  // every load in bounds, no branch around it
    float v[16];
#pragma unroll
    for (int col = 0; col < 16; ++col) v[col] = (col < a.ncol) ? a.src[col][rsafe] : 0.0f;
#pragma unroll
    for (int col = 0; col < 16; ++col)
        if (col < a.rl) tile[t * a.rl + col] = (col < a.ncol && row < a.n) ? v[col] : 0.0f;
    __syncthreads();
    const uint64_t nrows = (a.n - r0 < RA_ROWS) ? (a.n - r0) : RA_ROWS;
    float4 *dst = reinterpret_cast<float4 *>(a.rows + r0 * a.rl);
    const float4 *s4 = reinterpret_cast<const float4 *>(tile);
    for (uint64_t e = t; e < nrows * a.rl / 4; e += 256) dst[e] = s4[e];
}

// SH bytes (write-compressed-ply.ts:83-87) in the input's row order: a value depends on its
// own splat only, so it is computed while the columns stream in (coalesced), then gathered
// with the row as SHB contiguous bytes (3C bytes, padded to 16-byte rows)
constexpr int SHB = 48;  // byte row stride of the SH rows (3C <= 45)
__device__ inline uint8_t sh_byte(float v) {
    const double nv = (double)v / 8 + 0.5;
    return js::to_uint8(js::max_(0, js::min_(255, __builtin_trunc(nv * 256))));
}
__global__ __launch_bounds__(256) void k_sh_rows(const TransposeArgs a, int nsh, uint8_t *__restrict__ shrows) {
    __shared__ uint32_t stage[256 * SHB / 4];
    const uint64_t r0 = (uint64_t)blockIdx.x * 256;
    const uint32_t t = threadIdx.x;
    uint8_t *st8 = reinterpret_cast<uint8_t *>(stage);
    const bool real = r0 + t < a.n;
    const uint64_t rsafe = real ? r0 + t : a.n - 1;  // loads stay in bounds without a branch
    // batches of 12 columns: the loads of a batch are in flight together
    for (int k0 = 0; k0 < SHB; k0 += 12) {
        float v[12];
#pragma unroll
        for (int u = 0; u < 12; ++u) v[u] = a.src[14 + min(k0 + u, nsh - 1)][rsafe];
#pragma unroll
        for (int u = 0; u < 12; ++u) st8[t * SHB + k0 + u] = (k0 + u < nsh && real) ? sh_byte(v[u]) : 0u;
    }
    __syncthreads();
    const uint64_t nrows = (a.n - r0 < 256) ? (a.n - r0) : 256;
    uint4 *dst = reinterpret_cast<uint4 *>(shrows + r0 * SHB);
    const uint4 *s4 = reinterpret_cast<const uint4 *>(stage);
    for (uint64_t e = t; e < nrows * SHB / 16; e += 256) dst[e] = s4[e];
}

// the same from float64 values (the JS numbers of SH columns of another type than float32:
// write-compressed-ply.ts:85 divides the row's number itself)
struct ShRowsD {
    const double *src[45];
    uint64_t n;
};
__global__ __launch_bounds__(256) void k_sh_rows_d(const ShRowsD a, int nsh, uint8_t *__restrict__ shrows) {
    __shared__ uint32_t stage[256 * SHB / 4];
    const uint64_t r0 = (uint64_t)blockIdx.x * 256;
    const uint32_t t = threadIdx.x;
    uint8_t *st8 = reinterpret_cast<uint8_t *>(stage);
    const bool real = r0 + t < a.n;
    const uint64_t rsafe = real ? r0 + t : a.n - 1;
    for (int k = 0; k < SHB; ++k) {
        uint8_t b = 0;
        if (k < nsh && real) {
            const double nv = a.src[k][rsafe] / 8 + 0.5;
            b = js::to_uint8(js::max_(0, js::min_(255, __builtin_trunc(nv * 256))));
        }
        st8[t * SHB + k] = b;
    }
    __syncthreads();
    const uint64_t nrows = (a.n - r0 < 256) ? (a.n - r0) : 256;
    uint4 *dst = reinterpret_cast<uint4 *>(shrows + r0 * SHB);
    const uint4 *s4 = reinterpret_cast<const uint4 *>(stage);
    for (uint64_t e = t; e < nrows * SHB / 16; e += 256) dst[e] = s4[e];
}

struct ChunkArgs {
    const float *rows;  // AoS rows of RL = 16 floats: x y z scale_0..2 f_dc_0..2 opacity rot_0..3
    const uint8_t *shrows;  // SH bytes, SHB per row (k_sh_rows)
    int rl, nsh;
    uint64_t n;
    const uint32_t *order;
    float *chunk;
    uint4 *vertex;
    uint8_t *sh_out;
};

__global__ __launch_bounds__(256) void k_pack_chunk(const ChunkArgs a) {
    enum { X, Y, Z, S0, S1, S2, R, G, B, OP, Q0, Q1, Q2, Q3 };
    __shared__ uint32_t sh_stage[256 * 45 / 4];
    const uint64_t c = blockIdx.x;
    const uint64_t base = c * 256;
    const uint32_t num = (uint32_t)((a.n < base + 256 ? a.n : base + 256) - base);
    const uint32_t j = threadIdx.x;
    const bool real = j < num;
    const uint32_t row = a.order[base + (real ? j : num - 1)];
    const float4 *r4 = reinterpret_cast<const float4 *>(a.rows + (uint64_t)row * a.rl);
    // both gathered rows are requested before anything waits on them (the padded lanes
    // read the chunk's last row, always in bounds)
    float4 mv[4];
    uint4 sv[SHB / 16];
#pragma unroll
    for (int q = 0; q < 4; ++q) mv[q] = r4[q];
    if (a.nsh) {
        const uint4 *src = reinterpret_cast<const uint4 *>(a.shrows + (uint64_t)row * SHB);
#pragma unroll
        for (int q = 0; q < SHB / 16; ++q) sv[q] = src[q];
    }
    float d[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        d[4 * q] = mv[q].x;
        d[4 * q + 1] = mv[q].y;
        d[4 * q + 2] = mv[q].z;
        d[4 * q + 3] = mv[q].w;
    }
    // 8-bit SH (write-compressed-ply.ts:83-87), staged in LDS for coalesced stores
    if (a.nsh) {
        uint8_t *stage = reinterpret_cast<uint8_t *>(sh_stage);
        if (real) {
            uint32_t w[SHB / 4];
#pragma unroll
            for (int q = 0; q < SHB / 16; ++q) {
                w[4 * q] = sv[q].x;
                w[4 * q + 1] = sv[q].y;
                w[4 * q + 2] = sv[q].z;
                w[4 * q + 3] = sv[q].w;
            }
            for (int k = 0; k < a.nsh; ++k) stage[j * a.nsh + k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
        }
        __syncthreads();
        uint8_t *o = a.sh_out + base * (uint64_t)a.nsh;
        const uint32_t bytes = num * (uint32_t)a.nsh;
        // chunk bases are multiples of 256 * nsh bytes, so o is 4-byte aligned
        for (uint32_t e = j; e < bytes / 4; e += 256) reinterpret_cast<uint32_t *>(o)[e] = sh_stage[e];
        for (uint32_t e = (bytes / 4) * 4 + j; e < bytes; e += 256) o[e] = stage[e];
    }
    float mn[6] = {d[X], d[Y], d[Z], d[S0], d[S1], d[S2]};
    float mx[6] = {d[X], d[Y], d[Z], d[S0], d[S1], d[S2]};
    block_minmax<6>(mn, mx);
    double smn[3], smx[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {  // clamp(v, -20, 20) = Math.max(-20, Math.min(20, v))
        smn[i] = js::max_(-20, js::min_(20, (double)mn[3 + i]));
        smx[i] = js::max_(-20, js::min_(20, (double)mx[3 + i]));
    }
    const float col[3] = {(float)((double)d[R] * SH_C0 + 0.5), (float)((double)d[G] * SH_C0 + 0.5),
                          (float)((double)d[B] * SH_C0 + 0.5)};
    float cmn[3] = {col[0], col[1], col[2]}, cmx[3] = {col[0], col[1], col[2]};
    block_minmax<3>(cmn, cmx);
    if (real) {
        uint4 v;
        v.x = pack111011(normalize01(d[X], mn[0], mx[0]), normalize01(d[Y], mn[1], mx[1]),
                         normalize01(d[Z], mn[2], mx[2]));
        v.y = pack_rot(d[Q0], d[Q1], d[Q2], d[Q3]);
        v.z = pack111011(normalize01(d[S0], smn[0], smx[0]), normalize01(d[S1], smn[1], smx[1]),
                         normalize01(d[S2], smn[2], smx[2]));
        v.w = pack8888(normalize01(col[0], cmn[0], cmx[0]), normalize01(col[1], cmn[1], cmx[1]),
                       normalize01(col[2], cmn[2], cmx[2]), js::sigmoid(d[OP]));
        a.vertex[base + j] = v;
    }
    if (j < 18) {
        const double cd[18] = {mn[0], mn[1], mn[2], mx[0], mx[1], mx[2], smn[0], smn[1], smn[2],
                               smx[0], smx[1], smx[2], cmn[0], cmn[1], cmn[2], cmx[0], cmx[1], cmx[2]};
        a.chunk[c * 18 + j] = (float)cd[j];
    }
}

// ---- packed rows, one wave per chunk --------------------------------------------------
// Everything of a splat that does not depend on its chunk is computed once, in input order,
// while its columns stream in: the colour (f_dc * SH_C0 + 0.5 stored to f32, compressed-
// chunk.ts:98-103), the rotation word (packRot, :128-149), the opacity byte (packUnorm(sigmoid),
// :120-125) and the SH bytes (write-compressed-ply.ts:83-87).  With the positions and scales
// they make one row of RS dwords (96 B at SH3, 64 B below): floats x y z s0 s1 s2 c0 c1 c2,
// the rotation word, then byte 40 = opacity byte, bytes 41.. = the SH bytes.  The chunk pass
// gathers one row per splat (two 64-B sectors at most) instead of a 64-B member row and a
// 48-B SH row, and only the chunk-dependent quantisation remains there.
template <int NSH>
struct PR {
    static constexpr int RS = NSH > 23 ? 24 : 16;  // row dwords
};

struct PackRowsArgs {
    const float *m[14];      // x y z scale_0..2 f_dc_0..2 opacity rot_0..3
    const float *sh[45];
    const double *sh64[45];  // set instead of sh: the SH columns' numbers (other column types)
    uint64_t n;
    uint32_t *rows;
};

template <int NSH, bool SH64>
__global__ __launch_bounds__(256) void k_pack_rows(const PackRowsArgs a) {
    constexpr int RS = PR<NSH>::RS, LDSS = RS + 1;  // odd LDS stride: row-wise stores spread over banks
    __shared__ uint32_t stage[256 * LDSS];
    enum { X, Y, Z, S0, S1, S2, R, G, B, OP, Q0, Q1, Q2, Q3 };
    const uint64_t r0 = (uint64_t)blockIdx.x * 256;
    const uint32_t t = threadIdx.x;
    const bool real = r0 + t < a.n;
    const uint64_t r = real ? r0 + t : a.n - 1;  // loads stay in bounds without a branch
    float m[14];
#pragma unroll
    for (int i = 0; i < 14; ++i) m[i] = a.m[i][r];
    uint32_t w[RS];
#pragma unroll
    for (int i = 0; i < RS; ++i) w[i] = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) w[i] = __builtin_bit_cast(uint32_t, m[i]);
#pragma unroll
    for (int k = 0; k < 3; ++k) w[6 + k] = __builtin_bit_cast(uint32_t, (float)((double)m[R + k] * SH_C0 + 0.5));
    w[9] = pack_rot(m[Q0], m[Q1], m[Q2], m[Q3]);
    w[10] = pack_unorm(js::sigmoid(m[OP]), 8);  // byte 40
    // SH bytes at byte 41 + k, in batches of 12 columns (their loads in flight together)
#pragma unroll
    for (int k0 = 0; k0 < NSH; k0 += 12) {
        double v[12];
#pragma unroll
        for (int u = 0; u < 12; ++u)
            if (k0 + u < NSH) v[u] = SH64 ? a.sh64[k0 + u][r] : (double)a.sh[k0 + u][r];
#pragma unroll
        for (int u = 0; u < 12; ++u) {
            const int k = k0 + u;
            if (k < NSH) {
                const double nv = v[u] / 8 + 0.5;
                const uint32_t b = js::to_uint8(js::max_(0, js::min_(255, __builtin_trunc(nv * 256))));
                w[(41 + k) >> 2] |= b << (8 * ((41 + k) & 3));
            }
        }
    }
#pragma unroll
    for (int i = 0; i < RS; ++i) stage[t * LDSS + i] = real ? w[i] : 0u;
    __syncthreads();
    const uint32_t nrows = (uint32_t)((a.n - r0 < 256) ? (a.n - r0) : 256);
    uint32_t *dst = a.rows + r0 * RS;
    for (uint32_t e = t; e < nrows * RS; e += 256) dst[e] = stage[(e / RS) * LDSS + e % RS];
}

template <int NV>
__device__ inline void wave_minmax(float (&mn)[NV], float (&mx)[NV]) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            mn[v] = jmin(mn[v], __shfl_xor(mn[v], o, 64));
            mx[v] = jmax(mx[v], __shfl_xor(mx[v], o, 64));
        }
    }
}

// Lane l packs splats 4l .. 4l+3 of the chunk: its four rows are in flight before the first use,
// the chunk's min / max reduce in registers (4 values per lane) and across the wave by shuffles
// -- no LDS, no barriers -- and the outputs leave as 64 contiguous bytes of vertex data and
// 4 * NSH bytes of SH per lane.  Four chunks per 256-thread workgroup, each wave on its own.
template <int NSH>
__global__ __launch_bounds__(256) void k_pack_rows_chunk(const uint32_t *__restrict__ rows,
                                                         const uint32_t *__restrict__ order, uint64_t n,
                                                         float *__restrict__ chunk, uint4 *__restrict__ vertex,
                                                         uint8_t *__restrict__ sh_out) {
    constexpr int RS = PR<NSH>::RS;
    enum { X, Y, Z, S0, S1, S2, C0, C1, C2 };
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t c = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t nch = (n + 255) / 256;
    if (c >= nch) return;  // uniform per wave
    const uint64_t base = c * 256;
    const uint32_t num = (uint32_t)((n < base + 256 ? n : base + 256) - base);
    uint32_t row[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const uint32_t j = 4 * lane + s;
        row[s] = order[base + (j < num ? j : num - 1)];  // padding repeats the last splat
    }
    uint32_t w[4][RS];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const uint4 *r4 = reinterpret_cast<const uint4 *>(rows + (uint64_t)row[s] * RS);
#pragma unroll
        for (int q = 0; q < (NSH > 0 ? RS / 4 : 3); ++q) {  // SH0: bytes 0..43 are all there is
            const uint4 v = r4[q];
            w[s][4 * q] = v.x, w[s][4 * q + 1] = v.y, w[s][4 * q + 2] = v.z, w[s][4 * q + 3] = v.w;
        }
    }
    auto f = [&](int s, int i) { return __builtin_bit_cast(float, w[s][i]); };
    if (NSH > 0) {  // output byte t of this lane: coefficient t % NSH of splat t / NSH
        constexpr int NS = NSH > 0 ? NSH : 1;
        auto byte_at = [&](int t) -> uint32_t {
            const int s = t / NS, b = 41 + t % NS;
            return (w[s][b >> 2] >> (8 * (b & 3))) & 0xffu;
        };
        uint8_t *o = sh_out + (base + 4 * lane) * (uint64_t)NSH;
        if (num == 256) {  // whole chunk: 4 * NSH bytes per lane, dword aligned
            uint32_t *o4 = reinterpret_cast<uint32_t *>(o);
#pragma unroll
            for (int q = 0; q < NSH; ++q)
                o4[q] = byte_at(4 * q) | (byte_at(4 * q + 1) << 8) | (byte_at(4 * q + 2) << 16) | (byte_at(4 * q + 3) << 24);
        } else {
#pragma unroll
            for (int t = 0; t < 4 * NSH; ++t)
                if (4 * lane + t / NS < num) o[t] = (uint8_t)byte_at(t);
        }
    }
    float mn[9], mx[9];
#pragma unroll
    for (int v = 0; v < 9; ++v) {
        mn[v] = jmin(jmin(f(0, v), f(1, v)), jmin(f(2, v), f(3, v)));
        mx[v] = jmax(jmax(f(0, v), f(1, v)), jmax(f(2, v), f(3, v)));
    }
    wave_minmax<9>(mn, mx);
    double smn[3], smx[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {  // clamp(v, -20, 20) = Math.max(-20, Math.min(20, v))
        smn[i] = js::max_(-20, js::min_(20, (double)mn[S0 + i]));
        smx[i] = js::max_(-20, js::min_(20, (double)mx[S0 + i]));
    }
    uint4 v[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        v[s].x = pack111011(normalize01(f(s, X), mn[X], mx[X]), normalize01(f(s, Y), mn[Y], mx[Y]),
                            normalize01(f(s, Z), mn[Z], mx[Z]));
        v[s].y = w[s][9];
        v[s].z = pack111011(normalize01(f(s, S0), smn[0], smx[0]), normalize01(f(s, S1), smn[1], smx[1]),
                            normalize01(f(s, S2), smn[2], smx[2]));
        v[s].w = (pack_unorm(normalize01(f(s, C0), mn[C0], mx[C0]), 8) << 24) |
                 (pack_unorm(normalize01(f(s, C1), mn[C1], mx[C1]), 8) << 16) |
                 (pack_unorm(normalize01(f(s, C2), mn[C2], mx[C2]), 8) << 8) | (w[s][10] & 0xffu);
    }
    uint4 *vo = vertex + base + 4 * lane;
    if (num == 256) {
#pragma unroll
        for (int s = 0; s < 4; ++s) vo[s] = v[s];
    } else {
#pragma unroll
        for (int s = 0; s < 4; ++s)
            if (4 * lane + s < num) vo[s] = v[s];
    }
    if (lane < 18) {
        const double cd[18] = {mn[X], mn[Y], mn[Z], mx[X], mx[Y], mx[Z], smn[0], smn[1], smn[2],
                               smx[0], smx[1], smx[2], mn[C0], mn[C1], mn[C2], mx[C0], mx[C1], mx[C2]};
        chunk[c * 18 + lane] = (float)cd[lane];
    }
}

template <int NSH>
void launch_pack_rows(st_ctx *c, const PackRowsArgs &pa, const uint32_t *order, float *chunk, uint32_t *vertex,
                      uint8_t *sh) {
    const uint64_t n = pa.n, nchunks = (n + 255) / 256;
    if (pa.sh64[0])
        hipLaunchKernelGGL((k_pack_rows<NSH, true>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, pa);
    else
        hipLaunchKernelGGL((k_pack_rows<NSH, false>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, pa);
    hipLaunchKernelGGL(k_pack_rows_chunk<NSH>, dim3((unsigned)((nchunks + 3) / 4)), dim3(256), 0, c->stream, pa.rows,
                       order, n, chunk, reinterpret_cast<uint4 *>(vertex), sh);
}

}  // namespace

void pack_compressed_dev(st_ctx *c, const st_table *t, const uint32_t *order, float *chunk, uint32_t *vertex,
                         uint8_t *sh, const double *const *sh64, int sh_coeffs) {
    const uint64_t n = t->n;
    if (n == 0) return;
    static const char *members[14] = {"x", "y", "z", "scale_0", "scale_1", "scale_2", "f_dc_0",
                                      "f_dc_1", "f_dc_2", "opacity", "rot_0", "rot_1", "rot_2", "rot_3"};
    TransposeArgs ta{};
    for (int i = 0; i < 14; ++i) {
        ta.src[i] = col_or_null(t, members[i]);
        ST_REQUIRE(ta.src[i], ST_ERR_ARG, std::string("pack_compressed: missing column ") + members[i]);
    }
    const int C = sh64 ? sh_coeffs : sh_coeffs_of(t);
    const int nsh = 3 * C;
    if (nsh) ST_REQUIRE(sh, ST_ERR_ARG, "pack_compressed: sh output is NULL");
    char nm[32];
    for (int i = 0; i < nsh; ++i) {
        snprintf(nm, sizeof nm, "f_rest_%d", i);
        ta.src[14 + i] = sh64 ? nullptr : col_or_null(t, nm);
    }
    KTimer kt(c, "chunk.pack");
    if (!getenv("ST_PACK_WG")) {
        // packed rows (k_pack_rows), one wave per chunk (k_pack_rows_chunk)
        PackRowsArgs pa{};
        for (int i = 0; i < 14; ++i) pa.m[i] = ta.src[i];
        for (int i = 0; i < nsh; ++i) {
            if (sh64) pa.sh64[i] = sh64[i];
            else pa.sh[i] = ta.src[14 + i];
        }
        pa.n = n;
        pa.rows = wsT<uint32_t>(c, "chunk.prows", n * (uint64_t)(nsh > 23 ? 24 : 16));
        switch (nsh) {
            case 0: launch_pack_rows<0>(c, pa, order, chunk, vertex, sh); break;
            case 9: launch_pack_rows<9>(c, pa, order, chunk, vertex, sh); break;
            case 24: launch_pack_rows<24>(c, pa, order, chunk, vertex, sh); break;
            default: launch_pack_rows<45>(c, pa, order, chunk, vertex, sh); break;
        }
        ST_LAUNCH_CHECK();
        return;
    }
    // one workgroup per chunk over a 64-B member row and a 48-B SH row (the round-2 kernels;
    // ST_PACK_WG=1, experiments)
    ta.ncol = 14;
    ta.rl = 16;
    ta.n = n;
    ta.rows = wsT<float>(c, "chunk.rows", n * (uint64_t)ta.rl);
    uint8_t *shrows = nsh ? wsT<uint8_t>(c, "chunk.shrows", n * (uint64_t)SHB) : nullptr;
    ChunkArgs a{};
    a.rows = ta.rows;
    a.shrows = shrows;
    a.rl = ta.rl;
    a.nsh = nsh;
    a.n = n;
    a.order = order;
    a.chunk = chunk;
    a.vertex = reinterpret_cast<uint4 *>(vertex);
    a.sh_out = sh;
    const uint64_t nchunks = (n + 255) / 256;
    hipLaunchKernelGGL(k_rows_aos, dim3((unsigned)((n + RA_ROWS - 1) / RA_ROWS)), dim3(256), 0, c->stream, ta);
    if (nsh && sh64) {
        ShRowsD sd{};
        for (int i = 0; i < nsh; ++i) sd.src[i] = sh64[i];
        sd.n = n;
        hipLaunchKernelGGL(k_sh_rows_d, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, sd, nsh, shrows);
    } else if (nsh) {
        hipLaunchKernelGGL(k_sh_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, ta, nsh, shrows);
    }
    hipLaunchKernelGGL(k_pack_chunk, dim3((unsigned)nchunks), dim3(256), 0, c->stream, a);
    ST_LAUNCH_CHECK();
}

}  // namespace st
