// st_chunk.hip -- compressed-PLY chunk packing (write-compressed-ply.ts:56-109,
// CompressedChunk.pack compressed-chunk.ts:44-180).
//
// Two passes.  k_pack_rows reads the 14 member columns and the 3C SH columns in input order
// (coalesced) and writes one packed row per splat with everything that does not depend on the
// chunk (positions, scales, the colour and opacity bytes' inputs, the rotation word, the SH
// bytes).  k_pack_rows_chunk takes one 256-splat chunk of the Morton order per wave: each lane
// gathers four rows, the chunk's min / max reduce with Math.min / Math.max semantics (NaN
// propagates, -0 < +0) in registers and wave64 shuffles, the quantisers run in f64 exactly as
// the JS, and the final partial chunk is padded with its last splat
// (write-compressed-ply.ts:90-93).  HBM traffic per splat: 59 columns read and a 96-B row
// written, then the row gathered and 16 B vertex + 3C bytes SH written.
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
}

}  // namespace st
