// st_params.cpp -- host-side constants of one transform() call.
//
// The reference builds these per action on the host with PlayCanvas math
// (process.ts:75-79 Quat.setFromEulerAngles; transform.ts:13-15
// Mat4.setTRS / Mat3.setFromQuat / new RotateSH(mat3)).  playcanvas@2.11.8 is
// not in the image, so its published algorithms are restated with the
// engine's evaluation order and Float32Array matrix storage.  Compiled with
// -ffp-contract=off.  Pinned by tests/golden/transform (p*_quat/mat4/mat3/shrot).
#include <cmath>
#include <cstring>

#include "../../include/st_abi.h"

namespace {

struct QuatTerms {
    double xx, xy, xz, yy, yz, zz, wx, wy, wz;
};

QuatTerms quat_terms(const double q[4]) {
    const double x2 = q[0] + q[0], y2 = q[1] + q[1], z2 = q[2] + q[2];
    return {q[0] * x2, q[0] * y2, q[0] * z2, q[1] * y2, q[1] * z2, q[2] * z2, q[3] * x2, q[3] * y2, q[3] * z2};
}

// RotateSH constructor (rotate-sh.ts:49-149): band-1 from the f32 Mat3 data,
// bands 2 and 3 by the sh-lib recurrences, all in f64, evaluated exactly as written there.
void rotate_sh(const float m[9], double o1[9], double o2[25], double o3[49]) {
    const double s32 = std::sqrt(3.0 / 2.0), s13 = std::sqrt(1.0 / 3.0), s23 = std::sqrt(2.0 / 3.0),
                 s43 = std::sqrt(4.0 / 3.0), s14 = std::sqrt(1.0 / 4.0), s34 = std::sqrt(3.0 / 4.0),
                 s15 = std::sqrt(1.0 / 5.0), s35 = std::sqrt(3.0 / 5.0), s65 = std::sqrt(6.0 / 5.0),
                 s85 = std::sqrt(8.0 / 5.0), s95 = std::sqrt(9.0 / 5.0), s16 = std::sqrt(1.0 / 6.0),
                 s56 = std::sqrt(5.0 / 6.0), s38 = std::sqrt(3.0 / 8.0), s58 = std::sqrt(5.0 / 8.0),
                 s98 = std::sqrt(9.0 / 8.0), s59 = std::sqrt(5.0 / 9.0), s89 = std::sqrt(8.0 / 9.0),
                 s110 = std::sqrt(1.0 / 10.0), s310 = std::sqrt(3.0 / 10.0), s112 = std::sqrt(1.0 / 12.0),
                 s415 = std::sqrt(4.0 / 15.0), s116 = std::sqrt(1.0 / 16.0), s1516 = std::sqrt(15.0 / 16.0),
                 s118 = std::sqrt(1.0 / 18.0), s160 = std::sqrt(1.0 / 60.0);
    double a[3][3] = {{m[4], -(double)m[7], m[1]}, {-(double)m[5], m[8], -(double)m[2]}, {m[3], -(double)m[6], m[0]}};
    double b[5][5];
    // rows 0,1,3,4 share one shape: (p,q) = rows of a combined with row 0 / row 2
    auto row_a = [&](double *o, int i, int j, double sgn_outer) {
        // generic form used by rows 0 (i=2,j=0), 1 (i=1,j=0), 3 (i=1,j=2)
        o[0] = s14 * ((a[i][2] * a[j][0] + a[i][0] * a[j][2]) + (a[j][2] * a[i][0] + a[j][0] * a[i][2]));
        o[1] = (a[i][1] * a[j][0] + a[j][1] * a[i][0]);
        o[2] = s34 * (a[i][1] * a[j][1] + a[j][1] * a[i][1]);
        o[3] = (a[i][1] * a[j][2] + a[j][1] * a[i][2]);
        o[4] = s14 * ((a[i][2] * a[j][2] - a[i][0] * a[j][0]) + (a[j][2] * a[i][2] - a[j][0] * a[i][0]));
        (void)sgn_outer;
    };
    row_a(b[0], 2, 0, 1);
    row_a(b[1], 1, 0, 1);
    b[2][0] = s13 * (a[1][2] * a[1][0] + a[1][0] * a[1][2]) -
              s112 * ((a[2][2] * a[2][0] + a[2][0] * a[2][2]) + (a[0][2] * a[0][0] + a[0][0] * a[0][2]));
    b[2][1] = s43 * a[1][1] * a[1][0] - s13 * (a[2][1] * a[2][0] + a[0][1] * a[0][0]);
    b[2][2] = a[1][1] * a[1][1] - s14 * (a[2][1] * a[2][1] + a[0][1] * a[0][1]);
    b[2][3] = s43 * a[1][1] * a[1][2] - s13 * (a[2][1] * a[2][2] + a[0][1] * a[0][2]);
    b[2][4] = s13 * (a[1][2] * a[1][2] - a[1][0] * a[1][0]) -
              s112 * ((a[2][2] * a[2][2] - a[2][0] * a[2][0]) + (a[0][2] * a[0][2] - a[0][0] * a[0][0]));
    row_a(b[3], 1, 2, 1);
    b[4][0] = s14 * ((a[2][2] * a[2][0] + a[2][0] * a[2][2]) - (a[0][2] * a[0][0] + a[0][0] * a[0][2]));
    b[4][1] = (a[2][1] * a[2][0] - a[0][1] * a[0][0]);
    b[4][2] = s34 * (a[2][1] * a[2][1] - a[0][1] * a[0][1]);
    b[4][3] = (a[2][1] * a[2][2] - a[0][1] * a[0][2]);
    b[4][4] = s14 * ((a[2][2] * a[2][2] - a[2][0] * a[2][0]) - (a[0][2] * a[0][2] - a[0][0] * a[0][0]));

    double c[7][7];
    // band 3 rows 0 and 6: P(i) = a[2][*] with b[0|4][*] +/- a[0][*] with b[4|0][*]
    c[0][0] = s14 * ((a[2][2] * b[0][0] + a[2][0] * b[0][4]) + (a[0][2] * b[4][0] + a[0][0] * b[4][4]));
    c[0][1] = s32 * (a[2][1] * b[0][0] + a[0][1] * b[4][0]);
    c[0][2] = s1516 * (a[2][1] * b[0][1] + a[0][1] * b[4][1]);
    c[0][3] = s56 * (a[2][1] * b[0][2] + a[0][1] * b[4][2]);
    c[0][4] = s1516 * (a[2][1] * b[0][3] + a[0][1] * b[4][3]);
    c[0][5] = s32 * (a[2][1] * b[0][4] + a[0][1] * b[4][4]);
    c[0][6] = s14 * ((a[2][2] * b[0][4] - a[2][0] * b[0][0]) + (a[0][2] * b[4][4] - a[0][0] * b[4][0]));
    c[1][0] = s16 * (a[1][2] * b[0][0] + a[1][0] * b[0][4]) +
              s16 * ((a[2][2] * b[1][0] + a[2][0] * b[1][4]) + (a[0][2] * b[3][0] + a[0][0] * b[3][4]));
    c[1][1] = a[1][1] * b[0][0] + (a[2][1] * b[1][0] + a[0][1] * b[3][0]);
    c[1][2] = s58 * a[1][1] * b[0][1] + s58 * (a[2][1] * b[1][1] + a[0][1] * b[3][1]);
    c[1][3] = s59 * a[1][1] * b[0][2] + s59 * (a[2][1] * b[1][2] + a[0][1] * b[3][2]);
    c[1][4] = s58 * a[1][1] * b[0][3] + s58 * (a[2][1] * b[1][3] + a[0][1] * b[3][3]);
    c[1][5] = a[1][1] * b[0][4] + (a[2][1] * b[1][4] + a[0][1] * b[3][4]);
    c[1][6] = s16 * (a[1][2] * b[0][4] - a[1][0] * b[0][0]) +
              s16 * ((a[2][2] * b[1][4] - a[2][0] * b[1][0]) + (a[0][2] * b[3][4] - a[0][0] * b[3][0]));
    c[2][0] = s415 * (a[1][2] * b[1][0] + a[1][0] * b[1][4]) + s15 * (a[0][2] * b[2][0] + a[0][0] * b[2][4]) -
              s160 * ((a[2][2] * b[0][0] + a[2][0] * b[0][4]) - (a[0][2] * b[4][0] + a[0][0] * b[4][4]));
    c[2][1] = s85 * a[1][1] * b[1][0] + s65 * a[0][1] * b[2][0] - s110 * (a[2][1] * b[0][0] - a[0][1] * b[4][0]);
    c[2][2] = a[1][1] * b[1][1] + s34 * a[0][1] * b[2][1] - s116 * (a[2][1] * b[0][1] - a[0][1] * b[4][1]);
    c[2][3] = s89 * a[1][1] * b[1][2] + s23 * a[0][1] * b[2][2] - s118 * (a[2][1] * b[0][2] - a[0][1] * b[4][2]);
    c[2][4] = a[1][1] * b[1][3] + s34 * a[0][1] * b[2][3] - s116 * (a[2][1] * b[0][3] - a[0][1] * b[4][3]);
    c[2][5] = s85 * a[1][1] * b[1][4] + s65 * a[0][1] * b[2][4] - s110 * (a[2][1] * b[0][4] - a[0][1] * b[4][4]);
    c[2][6] = s415 * (a[1][2] * b[1][4] - a[1][0] * b[1][0]) + s15 * (a[0][2] * b[2][4] - a[0][0] * b[2][0]) -
              s160 * ((a[2][2] * b[0][4] - a[2][0] * b[0][0]) - (a[0][2] * b[4][4] - a[0][0] * b[4][0]));
    c[3][0] = s310 * (a[1][2] * b[2][0] + a[1][0] * b[2][4]) -
              s110 * ((a[2][2] * b[3][0] + a[2][0] * b[3][4]) + (a[0][2] * b[1][0] + a[0][0] * b[1][4]));
    c[3][1] = s95 * a[1][1] * b[2][0] - s35 * (a[2][1] * b[3][0] + a[0][1] * b[1][0]);
    c[3][2] = s98 * a[1][1] * b[2][1] - s38 * (a[2][1] * b[3][1] + a[0][1] * b[1][1]);
    c[3][3] = a[1][1] * b[2][2] - s13 * (a[2][1] * b[3][2] + a[0][1] * b[1][2]);
    c[3][4] = s98 * a[1][1] * b[2][3] - s38 * (a[2][1] * b[3][3] + a[0][1] * b[1][3]);
    c[3][5] = s95 * a[1][1] * b[2][4] - s35 * (a[2][1] * b[3][4] + a[0][1] * b[1][4]);
    c[3][6] = s310 * (a[1][2] * b[2][4] - a[1][0] * b[2][0]) -
              s110 * ((a[2][2] * b[3][4] - a[2][0] * b[3][0]) + (a[0][2] * b[1][4] - a[0][0] * b[1][0]));
    c[4][0] = s415 * (a[1][2] * b[3][0] + a[1][0] * b[3][4]) + s15 * (a[2][2] * b[2][0] + a[2][0] * b[2][4]) -
              s160 * ((a[2][2] * b[4][0] + a[2][0] * b[4][4]) + (a[0][2] * b[0][0] + a[0][0] * b[0][4]));
    c[4][1] = s85 * a[1][1] * b[3][0] + s65 * a[2][1] * b[2][0] - s110 * (a[2][1] * b[4][0] + a[0][1] * b[0][0]);
    c[4][2] = a[1][1] * b[3][1] + s34 * a[2][1] * b[2][1] - s116 * (a[2][1] * b[4][1] + a[0][1] * b[0][1]);
    c[4][3] = s89 * a[1][1] * b[3][2] + s23 * a[2][1] * b[2][2] - s118 * (a[2][1] * b[4][2] + a[0][1] * b[0][2]);
    c[4][4] = a[1][1] * b[3][3] + s34 * a[2][1] * b[2][3] - s116 * (a[2][1] * b[4][3] + a[0][1] * b[0][3]);
    c[4][5] = s85 * a[1][1] * b[3][4] + s65 * a[2][1] * b[2][4] - s110 * (a[2][1] * b[4][4] + a[0][1] * b[0][4]);
    c[4][6] = s415 * (a[1][2] * b[3][4] - a[1][0] * b[3][0]) + s15 * (a[2][2] * b[2][4] - a[2][0] * b[2][0]) -
              s160 * ((a[2][2] * b[4][4] - a[2][0] * b[4][0]) + (a[0][2] * b[0][4] - a[0][0] * b[0][0]));
    c[5][0] = s16 * (a[1][2] * b[4][0] + a[1][0] * b[4][4]) +
              s16 * ((a[2][2] * b[3][0] + a[2][0] * b[3][4]) - (a[0][2] * b[1][0] + a[0][0] * b[1][4]));
    c[5][1] = a[1][1] * b[4][0] + (a[2][1] * b[3][0] - a[0][1] * b[1][0]);
    c[5][2] = s58 * a[1][1] * b[4][1] + s58 * (a[2][1] * b[3][1] - a[0][1] * b[1][1]);
    c[5][3] = s59 * a[1][1] * b[4][2] + s59 * (a[2][1] * b[3][2] - a[0][1] * b[1][2]);
    c[5][4] = s58 * a[1][1] * b[4][3] + s58 * (a[2][1] * b[3][3] - a[0][1] * b[1][3]);
    c[5][5] = a[1][1] * b[4][4] + (a[2][1] * b[3][4] - a[0][1] * b[1][4]);
    c[5][6] = s16 * (a[1][2] * b[4][4] - a[1][0] * b[4][0]) +
              s16 * ((a[2][2] * b[3][4] - a[2][0] * b[3][0]) - (a[0][2] * b[1][4] - a[0][0] * b[1][0]));
    c[6][0] = s14 * ((a[2][2] * b[4][0] + a[2][0] * b[4][4]) - (a[0][2] * b[0][0] + a[0][0] * b[0][4]));
    c[6][1] = s32 * (a[2][1] * b[4][0] - a[0][1] * b[0][0]);
    c[6][2] = s1516 * (a[2][1] * b[4][1] - a[0][1] * b[0][1]);
    c[6][3] = s56 * (a[2][1] * b[4][2] - a[0][1] * b[0][2]);
    c[6][4] = s1516 * (a[2][1] * b[4][3] - a[0][1] * b[0][3]);
    c[6][5] = s32 * (a[2][1] * b[4][4] - a[0][1] * b[0][4]);
    c[6][6] = s14 * ((a[2][2] * b[4][4] - a[2][0] * b[4][0]) - (a[0][2] * b[0][4] - a[0][0] * b[0][0]));
    std::memcpy(o1, a, sizeof a);
    std::memcpy(o2, b, sizeof b);
    std::memcpy(o3, c, sizeof c);
}

}  // namespace

extern "C" {

int st_quat_from_euler(double ex, double ey, double ez, double q[4]) {
    if (!q) return ST_ERR_ARG;
    const double h = 0.5 * (M_PI / 180);  // 0.5 * math.DEG_TO_RAD
    ex *= h;
    ey *= h;
    ez *= h;
    const double sx = std::sin(ex), cx = std::cos(ex), sy = std::sin(ey), cy = std::cos(ey), sz = std::sin(ez),
                 cz = std::cos(ez);
    q[0] = sx * cy * cz - cx * sy * sz;
    q[1] = cx * sy * cz + sx * cy * sz;
    q[2] = cx * cy * sz - sx * sy * cz;
    q[3] = cx * cy * cz + sx * sy * sz;
    return ST_OK;
}

int st_transform_params_make(const double t[3], const double r[4], double s, st_transform_params *out) {
    if (!t || !r || !out) return ST_ERR_ARG;
    const QuatTerms p = quat_terms(r);
    float *m = out->m4;
    // Mat4.setTRS(t, r, Vec3(s, s, s))
    m[0] = (float)((1 - (p.yy + p.zz)) * s);
    m[1] = (float)((p.xy + p.wz) * s);
    m[2] = (float)((p.xz - p.wy) * s);
    m[3] = 0;
    m[4] = (float)((p.xy - p.wz) * s);
    m[5] = (float)((1 - (p.xx + p.zz)) * s);
    m[6] = (float)((p.yz + p.wx) * s);
    m[7] = 0;
    m[8] = (float)((p.xz + p.wy) * s);
    m[9] = (float)((p.yz - p.wx) * s);
    m[10] = (float)((1 - (p.xx + p.yy)) * s);
    m[11] = 0;
    m[12] = (float)t[0];
    m[13] = (float)t[1];
    m[14] = (float)t[2];
    m[15] = 1;
    // Mat3.setFromQuat(r)
    const float m3[9] = {(float)(1 - (p.yy + p.zz)), (float)(p.xy + p.wz),       (float)(p.xz - p.wy),
                         (float)(p.xy - p.wz),       (float)(1 - (p.xx + p.zz)), (float)(p.yz + p.wx),
                         (float)(p.xz + p.wy),       (float)(p.yz - p.wx),       (float)(1 - (p.xx + p.yy))};
    for (int i = 0; i < 4; ++i) out->r[i] = r[i];
    out->s = s;
    rotate_sh(m3, out->sh1, out->sh2, out->sh3);
    return ST_OK;
}

}  // extern "C"
