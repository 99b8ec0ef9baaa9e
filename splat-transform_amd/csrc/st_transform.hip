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

}  // namespace st
