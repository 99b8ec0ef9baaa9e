// st_transform.hip -- per-splat TRS + SH-band rotation on SoA float32 columns
// (filterNaN / permuteRows / combine: st_table.hip).
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
#include "st_typed.h"

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
        // (NaN results follow V8 on x86-64: js::x86_nan)
        if (POS) {
            const double vx = a.x[i], vy = a.y[i], vz = a.z[i];
            const bool nn = vx != vx || vy != vy || vz != vz;
            a.x[i] = (float)js::x86_nan(vx * a.m[0] + vy * a.m[4] + vz * a.m[8] + a.m[12], nn);
            a.y[i] = (float)js::x86_nan(vx * a.m[1] + vy * a.m[5] + vz * a.m[9] + a.m[13], nn);
            a.z[i] = (float)js::x86_nan(vx * a.m[2] + vy * a.m[6] + vz * a.m[10] + a.m[14], nn);
        }
        if (ROT) {
            const double q2w = a.rot[0][i], q2x = a.rot[1][i], q2y = a.rot[2][i], q2z = a.rot[3][i];
            const double q1x = a.r[0], q1y = a.r[1], q1z = a.r[2], q1w = a.r[3];
            const bool nn = q2w != q2w || q2x != q2x || q2y != q2y || q2z != q2z;
            const double nx = q1w * q2x + q1x * q2w + q1y * q2z - q1z * q2y;
            const double ny = q1w * q2y + q1y * q2w + q1z * q2x - q1x * q2z;
            const double nz = q1w * q2z + q1z * q2w + q1x * q2y - q1y * q2x;
            const double nw = q1w * q2w - q1x * q2x - q1y * q2y - q1z * q2z;
            a.rot[0][i] = (float)js::x86_nan(nw, nn);
            a.rot[1][i] = (float)js::x86_nan(nx, nn);
            a.rot[2][i] = (float)js::x86_nan(ny, nn);
            a.rot[3][i] = (float)js::x86_nan(nz, nn);
        }
        if (SCL) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const double v = a.scale[c][i];
                a.scale[c][i] = (float)js::x86_nan(js::log(js::exp(v) * a.s), v != v);
            }
        }
        if (C > 0) {
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) {
                float src[C > 0 ? C : 1];
#pragma unroll
                for (int k = 0; k < C; ++k) src[k] = a.sh[k + ch * C][i];
                float out[C > 0 ? C : 1];
                bool n1 = false, n2 = false, n3 = false;  // a NaN coefficient in the band
#pragma unroll
                for (int k = 0; k < C; ++k) (k < 3 ? n1 : k < 8 ? n2 : n3) |= src[k] != src[k];
#pragma unroll
                for (int r = 0; r < 3; ++r) out[r] = js::x86_nanf((float)dp<3>(src, a.sh1 + r * 3), n1);
                if (C >= 8) {
#pragma unroll
                    for (int r = 0; r < 5; ++r) out[3 + r] = js::x86_nanf((float)dp<5>(src + 3, a.sh2 + r * 5), n2);
                }
                if (C >= 15) {
#pragma unroll
                    for (int r = 0; r < 7; ++r) out[8 + r] = js::x86_nanf((float)dp<7>(src + 8, a.sh3 + r * 7), n3);
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

// any column type (the reference reads through getRow and writes through setRow): the same
// f64 arithmetic on the columns' JS numbers, stores with the TypedArray conversions; the SH
// coefficients pass through the Float32Array shCoeffs (transform.ts:21,52,55) both ways
struct TransformArgsT {
    TCol x, y, z;
    TCol rot[4];
    TCol scale[3];
    TCol sh[45];
    uint64_t n;
    float m[16];
    double r[4];
    double s;
    double sh1[9], sh2[25], sh3[49];
};

template <int C, bool POS, bool ROT, bool SCL>
__global__ __launch_bounds__(256) void k_transform_t(const TransformArgsT a) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
        if (POS) {
            const double vx = ta_load(a.x.p, a.x.t, i), vy = ta_load(a.y.p, a.y.t, i), vz = ta_load(a.z.p, a.z.t, i);
            const bool nn = vx != vx || vy != vy || vz != vz;
            ta_store(a.x.p, a.x.t, i, js::x86_nan(vx * a.m[0] + vy * a.m[4] + vz * a.m[8] + a.m[12], nn));
            ta_store(a.y.p, a.y.t, i, js::x86_nan(vx * a.m[1] + vy * a.m[5] + vz * a.m[9] + a.m[13], nn));
            ta_store(a.z.p, a.z.t, i, js::x86_nan(vx * a.m[2] + vy * a.m[6] + vz * a.m[10] + a.m[14], nn));
        }
        if (ROT) {
            const double q2w = ta_load(a.rot[0].p, a.rot[0].t, i), q2x = ta_load(a.rot[1].p, a.rot[1].t, i);
            const double q2y = ta_load(a.rot[2].p, a.rot[2].t, i), q2z = ta_load(a.rot[3].p, a.rot[3].t, i);
            const double q1x = a.r[0], q1y = a.r[1], q1z = a.r[2], q1w = a.r[3];
            const bool nn = q2w != q2w || q2x != q2x || q2y != q2y || q2z != q2z;
            const double nx = q1w * q2x + q1x * q2w + q1y * q2z - q1z * q2y;
            const double ny = q1w * q2y + q1y * q2w + q1z * q2x - q1x * q2z;
            const double nz = q1w * q2z + q1z * q2w + q1x * q2y - q1y * q2x;
            const double nw = q1w * q2w - q1x * q2x - q1y * q2y - q1z * q2z;
            ta_store(a.rot[0].p, a.rot[0].t, i, js::x86_nan(nw, nn));
            ta_store(a.rot[1].p, a.rot[1].t, i, js::x86_nan(nx, nn));
            ta_store(a.rot[2].p, a.rot[2].t, i, js::x86_nan(ny, nn));
            ta_store(a.rot[3].p, a.rot[3].t, i, js::x86_nan(nz, nn));
        }
        if (SCL) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const double v = ta_load(a.scale[c].p, a.scale[c].t, i);
                ta_store(a.scale[c].p, a.scale[c].t, i, js::x86_nan(js::log(js::exp(v) * a.s), v != v));
            }
        }
        if (C > 0) {
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) {
                float src[C > 0 ? C : 1];
#pragma unroll
                for (int k = 0; k < C; ++k) src[k] = (float)ta_load(a.sh[k + ch * C].p, a.sh[k + ch * C].t, i);
                float out[C > 0 ? C : 1];
                bool n1 = false, n2 = false, n3 = false;  // a NaN coefficient in the band
#pragma unroll
                for (int k = 0; k < C; ++k) (k < 3 ? n1 : k < 8 ? n2 : n3) |= src[k] != src[k];
#pragma unroll
                for (int r = 0; r < 3; ++r) out[r] = js::x86_nanf((float)dp<3>(src, a.sh1 + r * 3), n1);
                if (C >= 8) {
#pragma unroll
                    for (int r = 0; r < 5; ++r) out[3 + r] = js::x86_nanf((float)dp<5>(src + 3, a.sh2 + r * 5), n2);
                }
                if (C >= 15) {
#pragma unroll
                    for (int r = 0; r < 7; ++r) out[8 + r] = js::x86_nanf((float)dp<7>(src + 8, a.sh3 + r * 7), n3);
                }
#pragma unroll
                for (int k = 0; k < C; ++k) ta_store(a.sh[k + ch * C].p, a.sh[k + ch * C].t, i, (double)out[k]);
            }
        }
    }
}

template <int C>
void launch_transform_t(st_ctx *c, const TransformArgsT &a, bool pos, bool rot, bool scl) {
    const dim3 grid(grid_for(a.n, 256, 256 * 32)), block(256);
#define ST_T(P, R, S) \
    if (pos == P && rot == R && scl == S) { hipLaunchKernelGGL((k_transform_t<C, P, R, S>), grid, block, 0, c->stream, a); return; }
    ST_T(true, true, true) ST_T(true, true, false) ST_T(true, false, true) ST_T(true, false, false)
    ST_T(false, true, true) ST_T(false, true, false) ST_T(false, false, true) ST_T(false, false, false)
#undef ST_T
}

int sh_coeffs_t(const st_ttable *t) {
    int first_missing = -1;
    char nm[32];
    for (int i = 0; i < 45 && first_missing < 0; ++i) {
        snprintf(nm, sizeof nm, "f_rest_%d", i);
        if (!tcol_or_null(t, nm).p) first_missing = i;
    }
    return first_missing == 9 ? 3 : first_missing == 24 ? 8 : first_missing == -1 ? 15 : 0;
}

}  // namespace

// transform() over a typed device table, in place (transform.ts:12-65).  Float32 tables take
// the float32 kernel; any other type of a transformed column takes the typed one.
void transform_tdev(st_ctx *c, const st_ttable *t, const st_transform_params *p) {
    if (t->n == 0) return;
    static const char *tcols[10] = {"x", "y", "z", "rot_0", "rot_1", "rot_2", "rot_3", "scale_0", "scale_1", "scale_2"};
    std::vector<const char *> names(tcols, tcols + 10);
    std::vector<std::string> shn;
    const int C = sh_coeffs_t(t);
    for (int i = 0; i < 3 * C; ++i) shn.push_back("f_rest_" + std::to_string(i));
    for (auto &s : shn) names.push_back(s.c_str());
    if (all_f32(t, names.data(), (int)names.size())) {
        std::vector<const char *> fn;
        std::vector<float *> fp;
        for (int i = 0; i < t->ncol; ++i)
            if (t->types[i] == ST_PLY_FLOAT) fn.push_back(t->names[i]), fp.push_back(static_cast<float *>(t->cols[i]));
        const st_table ft{t->n, (int32_t)fp.size(), fn.data(), fp.data()};
        transform_dev(c, &ft, p);
        return;
    }
    TransformArgsT a{};
    a.n = t->n;
    a.x = tcol_or_null(t, "x");
    a.y = tcol_or_null(t, "y");
    a.z = tcol_or_null(t, "z");
    const bool pos = a.x.p && a.y.p && a.z.p;
    bool rot = true, scl = true;
    for (int i = 0; i < 4; ++i) rot = (a.rot[i] = tcol_or_null(t, tcols[3 + i])).p && rot;
    for (int i = 0; i < 3; ++i) scl = (a.scale[i] = tcol_or_null(t, tcols[7 + i])).p && scl;
    for (int i = 0; i < 3 * C; ++i) a.sh[i] = tcol_or_null(t, shn[i].c_str());
    for (int i = 0; i < 16; ++i) a.m[i] = p->m4[i];
    for (int i = 0; i < 4; ++i) a.r[i] = p->r[i];
    a.s = p->s;
    for (int i = 0; i < 9; ++i) a.sh1[i] = p->sh1[i];
    for (int i = 0; i < 25; ++i) a.sh2[i] = p->sh2[i];
    for (int i = 0; i < 49; ++i) a.sh3[i] = p->sh3[i];
    KTimer kt(c, "transform");
    switch (C) {
        case 0: launch_transform_t<0>(c, a, pos, rot, scl); break;
        case 3: launch_transform_t<3>(c, a, pos, rot, scl); break;
        case 8: launch_transform_t<8>(c, a, pos, rot, scl); break;
        default: launch_transform_t<15>(c, a, pos, rot, scl); break;
    }
    ST_LAUNCH_CHECK();
}

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

}  // namespace st
