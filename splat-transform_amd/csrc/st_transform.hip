// st_transform.hip -- per-splat TRS + SH-band rotation, filterNaN compaction,
// row gather and row concatenation on SoA float32 columns.
//
// transform(): transform.ts:12-65.  One thread per splat, f64 arithmetic in the
// reference's order (no FMA contraction), f32 stores:
//   position  p' = Mat4.transformPoint(p)            (f32 matrix entries)
//   rotation  q' = r (x) q,  q = (rot_1, rot_2, rot_3, rot_0)   (Quat.mul2)
//   scale     log(exp(s_i) * s)                      (V8 fdlibm exp/log)
//   SH        per colour channel: RotateSH.apply      (rotate-sh.ts:152-187)
// HBM-bound: it reads and writes 10 + 3C columns once (440 B/splat at SH3).
#include "st_internal.h"
#include "st_jsmath.h"

namespace st {
namespace {

struct TransformArgs {
    float *x, *y, *z;
    float *rot[4];
    float *scale[3];
    float *sh[45];
    uint64_t n;
    float m[16];
    double r[4];
    double s;
    double sh1[9], sh2[25], sh3[49];
};

template <int N>
__device__ inline double dp(const float *src, const double *row) {
    double sum = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) sum += (double)src[i] * row[i];
    return sum;
}

template <int C, bool POS, bool ROT, bool SCL>
__global__ __launch_bounds__(256) void k_transform(const TransformArgs a) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
        if (POS) {
            const double vx = a.x[i], vy = a.y[i], vz = a.z[i];
            a.x[i] = (float)(vx * a.m[0] + vy * a.m[4] + vz * a.m[8] + a.m[12]);
            a.y[i] = (float)(vx * a.m[1] + vy * a.m[5] + vz * a.m[9] + a.m[13]);
            a.z[i] = (float)(vx * a.m[2] + vy * a.m[6] + vz * a.m[10] + a.m[14]);
        }
        if (ROT) {
            const double q2w = a.rot[0][i], q2x = a.rot[1][i], q2y = a.rot[2][i], q2z = a.rot[3][i];
            const double q1x = a.r[0], q1y = a.r[1], q1z = a.r[2], q1w = a.r[3];
            const double nx = q1w * q2x + q1x * q2w + q1y * q2z - q1z * q2y;
            const double ny = q1w * q2y + q1y * q2w + q1z * q2x - q1x * q2z;
            const double nz = q1w * q2z + q1z * q2w + q1x * q2y - q1y * q2x;
            const double nw = q1w * q2w - q1x * q2x - q1y * q2y - q1z * q2z;
            a.rot[0][i] = (float)nw;
            a.rot[1][i] = (float)nx;
            a.rot[2][i] = (float)ny;
            a.rot[3][i] = (float)nz;
        }
        if (SCL) {
#pragma unroll
            for (int c = 0; c < 3; ++c) a.scale[c][i] = (float)js::log(js::exp((double)a.scale[c][i]) * a.s);
        }
        if (C > 0) {
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) {
                float src[C > 0 ? C : 1];
#pragma unroll
                for (int k = 0; k < C; ++k) src[k] = a.sh[k + ch * C][i];
                float out[C > 0 ? C : 1];
#pragma unroll
                for (int r = 0; r < 3; ++r) out[r] = (float)dp<3>(src, a.sh1 + r * 3);
                if (C >= 8) {
#pragma unroll
                    for (int r = 0; r < 5; ++r) out[3 + r] = (float)dp<5>(src + 3, a.sh2 + r * 5);
                }
                if (C >= 15) {
#pragma unroll
                    for (int r = 0; r < 7; ++r) out[8 + r] = (float)dp<7>(src + 8, a.sh3 + r * 7);
                }
#pragma unroll
                for (int k = 0; k < C; ++k) a.sh[k + ch * C][i] = out[k];
            }
        }
    }
}

template <int C>
void launch_transform(st_ctx *c, const TransformArgs &a, bool pos, bool rot, bool scl) {
    const dim3 grid(grid_for(a.n, 256, 256 * 32)), block(256);
#define ST_T(P, R, S) \
    if (pos == P && rot == R && scl == S) { hipLaunchKernelGGL((k_transform<C, P, R, S>), grid, block, 0, c->stream, a); return; }
    ST_T(true, true, true) ST_T(true, true, false) ST_T(true, false, true) ST_T(true, false, false)
    ST_T(false, true, true) ST_T(false, true, false) ST_T(false, false, true) ST_T(false, false, false)
#undef ST_T
}

// ---------------------------------------------------------------------------
// filterNaN: keep row iff every column value is finite (process.ts:84-95)
__global__ __launch_bounds__(256) void k_finite_flags(float *const *cols, int ncol, uint64_t n, uint32_t *flags) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint32_t ok = 1;
        for (int c = 0; c < ncol; ++c) ok &= js::isfinitef_(cols[c][i]) ? 1u : 0u;
        flags[i] = ok;
    }
}

__global__ __launch_bounds__(256) void k_compact(const uint32_t *flags, const uint32_t *pos, uint64_t n,
                                                 uint32_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        if (flags[i]) out[pos[i]] = (uint32_t)i;
}

// permuteRows (data-table.ts:135-149): dst[c][j] = src[c][idx[j]]
__global__ __launch_bounds__(256) void k_gather_cols(float *const *src, float *const *dst, int ncol,
                                                     const uint32_t *__restrict__ idx, uint64_t m) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
        const uint32_t s = idx[j];
        for (int c = 0; c < ncol; ++c) dst[c][j] = src[c][s];
    }
}

// ---- wide streaming forms: 4 consecutive rows per thread, column pointers in kernel
// arguments, 8 columns' loads in flight before any test (the loops above wait on every
// column's load in turn)
constexpr int WIDE_COLS = 64;
struct ColPtrs {
    const float *p[WIDE_COLS];
};

__device__ inline uint32_t nonfinite_bit(float x) {
    return ((__builtin_bit_cast(uint32_t, x) & 0x7f800000u) == 0x7f800000u) ? 1u : 0u;
}

__global__ __launch_bounds__(256) void k_finite_flags4(const ColPtrs cp, int ncol, uint64_t n,
                                                       uint32_t *__restrict__ flags) {
    const uint64_t nq = n / 4;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += stride) {
        uint32_t bad = 0;  // bit r: row 4q + r holds a non-finite value
        int c = 0;
        for (; c + 8 <= ncol; c += 8) {
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = reinterpret_cast<const float4 *>(cp.p[c + u])[q];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                bad |= nonfinite_bit(v[u].x) | (nonfinite_bit(v[u].y) << 1) | (nonfinite_bit(v[u].z) << 2) |
                       (nonfinite_bit(v[u].w) << 3);
        }
        for (; c < ncol; ++c) {
            const float4 v = reinterpret_cast<const float4 *>(cp.p[c])[q];
            bad |= nonfinite_bit(v.x) | (nonfinite_bit(v.y) << 1) | (nonfinite_bit(v.z) << 2) | (nonfinite_bit(v.w) << 3);
        }
        reinterpret_cast<uint4 *>(flags)[q] =
            make_uint4((bad & 1u) ^ 1u, ((bad >> 1) & 1u) ^ 1u, ((bad >> 2) & 1u) ^ 1u, ((bad >> 3) & 1u) ^ 1u);
    }
    if (blockIdx.x == 0 && threadIdx.x < n % 4) {  // the last n % 4 rows
        const uint64_t i = nq * 4 + threadIdx.x;
        uint32_t bad = 0;
        for (int c = 0; c < ncol; ++c) bad |= nonfinite_bit(cp.p[c][i]);
        flags[i] = bad ^ 1u;
    }
}

// permuteRows with 4 destination rows per thread: 4 x 8 gathered loads in flight, float4
// stores (dst columns and idx 16-byte aligned)
__global__ __launch_bounds__(256) void k_gather_cols4(const ColPtrs src, const ColPtrs dst, int ncol,
                                                      const uint32_t *__restrict__ idx, uint64_t m) {
    const uint64_t mq = m / 4;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < mq; q += stride) {
        const uint4 ii = reinterpret_cast<const uint4 *>(idx)[q];
        int c = 0;
        for (; c + 8 <= ncol; c += 8) {
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const float *sp = src.p[c + u];
                v[u] = make_float4(sp[ii.x], sp[ii.y], sp[ii.z], sp[ii.w]);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) reinterpret_cast<float4 *>(const_cast<float *>(dst.p[c + u]))[q] = v[u];
        }
        for (; c < ncol; ++c) {
            const float *sp = src.p[c];
            reinterpret_cast<float4 *>(const_cast<float *>(dst.p[c]))[q] =
                make_float4(sp[ii.x], sp[ii.y], sp[ii.z], sp[ii.w]);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < m % 4) {
        const uint64_t j = mq * 4 + threadIdx.x;
        const uint32_t sj = idx[j];
        for (int c = 0; c < ncol; ++c) const_cast<float *>(dst.p[c])[j] = src.p[c][sj];
    }
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace

void transform_dev(st_ctx *c, const st_table *t, const st_transform_params *p) {
    TransformArgs a{};
    a.n = t->n;
    if (a.n == 0) return;
    a.x = col_or_null(t, "x");
    a.y = col_or_null(t, "y");
    a.z = col_or_null(t, "z");
    const bool pos = a.x && a.y && a.z;
    bool rot = true, scl = true;
    char nm[32];
    for (int i = 0; i < 4; ++i) {
        snprintf(nm, sizeof nm, "rot_%d", i);
        a.rot[i] = col_or_null(t, nm);
        rot = rot && a.rot[i];
    }
    for (int i = 0; i < 3; ++i) {
        snprintf(nm, sizeof nm, "scale_%d", i);
        a.scale[i] = col_or_null(t, nm);
        scl = scl && a.scale[i];
    }
    const int C = sh_coeffs_of(t);
    for (int i = 0; i < 3 * C; ++i) {
        snprintf(nm, sizeof nm, "f_rest_%d", i);
        a.sh[i] = col_or_null(t, nm);
    }
    for (int i = 0; i < 16; ++i) a.m[i] = p->m4[i];
    for (int i = 0; i < 4; ++i) a.r[i] = p->r[i];
    a.s = p->s;
    for (int i = 0; i < 9; ++i) a.sh1[i] = p->sh1[i];
    for (int i = 0; i < 25; ++i) a.sh2[i] = p->sh2[i];
    for (int i = 0; i < 49; ++i) a.sh3[i] = p->sh3[i];
    KTimer kt(c, "transform");
    switch (C) {
        case 0: launch_transform<0>(c, a, pos, rot, scl); break;
        case 3: launch_transform<3>(c, a, pos, rot, scl); break;
        case 8: launch_transform<8>(c, a, pos, rot, scl); break;
        default: launch_transform<15>(c, a, pos, rot, scl); break;
    }
    ST_LAUNCH_CHECK();
}

static float *const *upload_ptrs(st_ctx *c, const std::string &slot, float *const *ptrs, int n) {
    auto **d = wsT<float *>(c, slot, (size_t)(n > 0 ? n : 1));
    if (n > 0) ST_HIP(hipMemcpyAsync(d, ptrs, sizeof(float *) * n, hipMemcpyHostToDevice, c->stream));
    return d;
}

uint64_t filter_finite_dev(st_ctx *c, const st_table *t, uint32_t *out_idx) {
    const uint64_t n = t->n;
    if (n == 0) return 0;
    auto *flags = wsT<uint32_t>(c, "filter.flags", n);
    auto *pos = wsT<uint32_t>(c, "filter.pos", n + 1);
    bool wide = t->ncol <= WIDE_COLS;
    ColPtrs cp{};
    for (int i = 0; wide && i < t->ncol; ++i) {
        cp.p[i] = t->cols[i];
        wide = aligned16(t->cols[i]);
    }
    if (wide) {
        hipLaunchKernelGGL(k_finite_flags4, dim3(grid_for((n + 3) / 4, 256, 8192)), dim3(256), 0, c->stream, cp,
                           t->ncol, n, flags);
    } else {
        float *const *dcols = upload_ptrs(c, "filter.cols", t->cols, t->ncol);
        hipLaunchKernelGGL(k_finite_flags, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c->stream, dcols, t->ncol, n,
                           flags);
    }
    ST_LAUNCH_CHECK();
    scan_u32(c, flags, pos, n, pos + n);
    hipLaunchKernelGGL(k_compact, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c->stream, flags, pos, n, out_idx);
    ST_LAUNCH_CHECK();
    auto *h = static_cast<uint32_t *>(pinned(c, 16));
    ST_HIP(hipMemcpyAsync(h, pos + n, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    ST_HIP(hipStreamSynchronize(c->stream));
    return h[0];
}

void permute_rows_dev(st_ctx *c, const st_table *src, const uint32_t *idx, uint64_t m, const st_table *dst) {
    if (m == 0 || src->ncol == 0) return;
    bool wide = src->ncol <= WIDE_COLS && aligned16(idx);
    ColPtrs sp{}, dp{};
    for (int i = 0; wide && i < src->ncol; ++i) {
        sp.p[i] = src->cols[i];
        dp.p[i] = dst->cols[i];
        wide = aligned16(dst->cols[i]);
    }
    if (wide) {
        hipLaunchKernelGGL(k_gather_cols4, dim3(grid_for((m + 3) / 4, 256, 8192)), dim3(256), 0, c->stream, sp, dp,
                           src->ncol, idx, m);
    } else {
        float *const *s = upload_ptrs(c, "permute.src", src->cols, src->ncol);
        float *const *d = upload_ptrs(c, "permute.dst", dst->cols, dst->ncol);
        hipLaunchKernelGGL(k_gather_cols, dim3(grid_for(m, 256, 8192)), dim3(256), 0, c->stream, s, d, src->ncol, idx,
                           m);
    }
    ST_LAUNCH_CHECK();
}

// combine() (index.ts:158-210): dst columns are the union by name (f32 only);
// rows are appended in source order, absent columns zero-filled.
void concat_rows_dev(st_ctx *c, const st_table *const *srcs, int nsrc, const st_table *dst) {
    uint64_t total = 0;
    for (int i = 0; i < nsrc; ++i) total += srcs[i]->n;
    ST_REQUIRE(total == dst->n, ST_ERR_ARG, "concat_rows: dst rows != sum of src rows");
    for (int col = 0; col < dst->ncol; ++col) {
        uint64_t off = 0;
        for (int i = 0; i < nsrc; ++i) {
            const uint64_t n = srcs[i]->n;
            float *s = col_or_null(srcs[i], dst->names[col]);
            if (n) {
                if (s)
                    ST_HIP(hipMemcpyAsync(dst->cols[col] + off, s, n * sizeof(float), hipMemcpyDeviceToDevice,
                                          c->stream));
                else
                    ST_HIP(hipMemsetAsync(dst->cols[col] + off, 0, n * sizeof(float), c->stream));
            }
            off += n;
        }
    }
}

}  // namespace st
