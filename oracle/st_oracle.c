/*
 * st_oracle.c -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE).
 *
 * Parity checker only: loaded by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py.  Never linked into the product.
 *
 * JS-number semantics throughout: every arithmetic expression is evaluated in
 * IEEE binary64 in the reference's source order; Float32Array stores round to
 * nearest-even; typed-array integer stores use ToInt32/ToUint32/ToUint8.
 * Build with -ffp-contract=off (no FMA contraction) -- see oracle/Makefile.
 */
#include "st_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* JS primitive semantics                                                      */

static inline int32_t js_to_int32(double v)
{
    if (!isfinite(v)) return 0;
    double t = trunc(v);
    double m = fmod(t, 4294967296.0);
    if (m < 0) m += 4294967296.0;
    uint32_t u = (uint32_t)m;
    return (int32_t)u;
}

static inline uint32_t js_to_uint32(double v) { return (uint32_t)js_to_int32(v); }

static inline uint8_t js_to_uint8(double v) { return (uint8_t)(js_to_uint32(v) & 0xff); }

/* Math.min / Math.max: NaN-propagating, -0 < +0.  A NaN result is V8's NaN on x86-64, the
 * default NaN with the sign bit set (0xfff8000000000000; 0xffc00000 once stored to a
 * Float32Array: tests/golden/process_chain, make_golden.js) */
static inline double js_nan(void)
{
    const uint64_t bits = 0xfff8000000000000ull;
    double v;
    memcpy(&v, &bits, sizeof v);
    return v;
}

static inline double js_min(double a, double b)
{
    if (isnan(a) || isnan(b)) return js_nan();
    if (a == 0 && b == 0) return signbit(a) ? a : b;
    return a < b ? a : b;
}

static inline double js_max(double a, double b)
{
    if (isnan(a) || isnan(b)) return js_nan();
    if (a == 0 && b == 0) return signbit(a) ? b : a;
    return a > b ? a : b;
}

static inline double js_sign(double v)
{
    if (isnan(v)) return NAN;
    if (v > 0) return 1;
    if (v < 0) return -1;
    return v; /* +-0 */
}

/* ------------------------------------------------------------------------- */
/* fdlibm e_exp.c / e_log.c as used by V8 (src/base/ieee754.cc)               */

typedef union { double d; uint64_t u; } dbits;
static inline uint32_t hi_word(double x) { dbits b; b.d = x; return (uint32_t)(b.u >> 32); }
static inline uint32_t lo_word(double x) { dbits b; b.d = x; return (uint32_t)b.u; }
static inline double from_words(uint32_t hi, uint32_t lo) { dbits b; b.u = ((uint64_t)hi << 32) | lo; return b.d; }

double st_o_exp(double x)
{
    static const double one = 1.0, halF[2] = {0.5, -0.5}, huge = 1.0e+300,
        o_threshold = 7.09782712893383973096e+02, u_threshold = -7.45133219101941108420e+02,
        ln2HI[2] = {6.93147180369123816490e-01, -6.93147180369123816490e-01},
        ln2LO[2] = {1.90821492927058770002e-10, -1.90821492927058770002e-10},
        invln2 = 1.44269504088896338700e+00,
        P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
        P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
        P5 = 4.13813679705723846039e-08,
        twom1000 = 9.33263618503218878990e-302;
    double y, hi = 0.0, lo = 0.0, c, t, twopk;
    int32_t k = 0, xsb;
    uint32_t hx = hi_word(x);
    xsb = (hx >> 31) & 1;
    hx &= 0x7fffffff;
    if (hx >= 0x40862E42) {
        if (hx >= 0x7ff00000) {
            if (((hx & 0xfffff) | lo_word(x)) != 0) return x + x;
            return (xsb == 0) ? x : 0.0;
        }
        if (x > o_threshold) return huge * huge;
        if (x < u_threshold) return twom1000 * twom1000;
    }
    if (hx > 0x3fd62e42) {
        if (hx < 0x3FF0A2B2) {
            /* V8 special-cases exp(1) so that Math.exp(1) === Math.E */
            if (x == 1.0) return 2.718281828459045;
            hi = x - ln2HI[xsb];
            lo = ln2LO[xsb];
            k = 1 - xsb - xsb;
        } else {
            k = (int32_t)(invln2 * x + halF[xsb]);
            t = k;
            hi = x - t * ln2HI[0];
            lo = t * ln2LO[0];
        }
        x = hi - lo;
    } else if (hx < 0x3e300000) {
        if (huge + x > one) return one + x;
    } else {
        k = 0;
    }
    t = x * x;
    if (k >= -1021)
        twopk = from_words(0x3ff00000u + ((uint32_t)k << 20), 0);
    else
        twopk = from_words(0x3ff00000u + ((uint32_t)(k + 1000) << 20), 0);
    c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    if (k == 0) return one - ((x * c) / (c - 2.0) - x);
    y = one - ((lo - (x * c) / (2.0 - c)) - hi);
    if (k >= -1021) {
        if (k == 1024) return y * 2.0 * 8.98846567431157953865e+307; /* 0x1p1023 */
        return y * twopk;
    }
    return y * twopk * twom1000;
}

double st_o_log(double x)
{
    static const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
        two54 = 1.80143985094819840000e+16,
        Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
        Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
        Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
        Lg7 = 1.479819860511658591e-01;
    static volatile double vzero = 0.0;
    double hfsq, f, s, z, R, w, t1, t2, dk;
    int32_t k, hx, i, j;
    uint32_t lx;
    hx = (int32_t)hi_word(x);
    lx = lo_word(x);
    k = 0;
    if (hx < 0x00100000) {
        if (((hx & 0x7fffffff) | lx) == 0) return -two54 / vzero;
        if (hx < 0) return (x - x) / vzero;
        k -= 54;
        x *= two54;
        hx = (int32_t)hi_word(x);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    i = (hx + 0x95f64) & 0x100000;
    x = from_words((uint32_t)(hx | (i ^ 0x3ff00000)), lo_word(x));
    k += (i >> 20);
    f = x - 1.0;
    if ((0x000fffff & (2 + hx)) < 3) {
        if (f == 0.0) {
            if (k == 0) return 0.0;
            dk = (double)k;
            return dk * ln2_hi + dk * ln2_lo;
        }
        R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        dk = (double)k;
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    s = f / (2.0 + f);
    dk = (double)k;
    z = s * s;
    i = hx - 0x6147a;
    w = z * z;
    j = 0x6b851 - hx;
    t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    R = t2 + t1;
    if (i > 0) {
        hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

static inline double sigmoid(double v) { return 1 / (1 + st_o_exp(-v)); } /* utils/math.ts:1 */

/* ------------------------------------------------------------------------- */
/* PlayCanvas math (restated, playcanvas@2.11.8)                               */

void st_o_quat_from_euler(double ex, double ey, double ez, double q[4])
{
    const double halfToRad = 0.5 * (M_PI / 180);
    ex *= halfToRad;
    ey *= halfToRad;
    ez *= halfToRad;
    const double sx = sin(ex), cx = cos(ex), sy = sin(ey), cy = cos(ey), sz = sin(ez), cz = cos(ez);
    q[0] = sx * cy * cz - cx * sy * sz;
    q[1] = cx * sy * cz + sx * cy * sz;
    q[2] = cx * cy * sz - sx * sy * cz;
    q[3] = cx * cy * cz + sx * sy * sz;
}

typedef struct { double xx, xy, xz, yy, yz, zz, wx, wy, wz; } qprod;

static qprod quat_products(const double q[4])
{
    const double qx = q[0], qy = q[1], qz = q[2], qw = q[3];
    const double x2 = qx + qx, y2 = qy + qy, z2 = qz + qz;
    qprod p = {qx * x2, qx * y2, qx * z2, qy * y2, qy * z2, qz * z2, qw * x2, qw * y2, qw * z2};
    return p;
}

void st_o_mat4_trs(const double t[3], const double q[4], double s, float m[16])
{
    qprod p = quat_products(q);
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
}

void st_o_mat3_from_quat(const double q[4], float m[9])
{
    qprod p = quat_products(q);
    m[0] = (float)(1 - (p.yy + p.zz));
    m[1] = (float)(p.xy + p.wz);
    m[2] = (float)(p.xz - p.wy);
    m[3] = (float)(p.xy - p.wz);
    m[4] = (float)(1 - (p.xx + p.zz));
    m[5] = (float)(p.yz + p.wx);
    m[6] = (float)(p.xz + p.wy);
    m[7] = (float)(p.yz - p.wx);
    m[8] = (float)(1 - (p.xx + p.yy));
}

/* ------------------------------------------------------------------------- */
/* RotateSH (rotate-sh.ts:49-149)                                              */

void st_o_rotate_sh(const float m3[9], double o1[9], double o2[25], double o3[49])
{
    const double k03_02 = sqrt(3.0 / 2.0), k01_03 = sqrt(1.0 / 3.0), k02_03 = sqrt(2.0 / 3.0),
        k04_03 = sqrt(4.0 / 3.0), k01_04 = sqrt(1.0 / 4.0), k03_04 = sqrt(3.0 / 4.0),
        k01_05 = sqrt(1.0 / 5.0), k03_05 = sqrt(3.0 / 5.0), k06_05 = sqrt(6.0 / 5.0),
        k08_05 = sqrt(8.0 / 5.0), k09_05 = sqrt(9.0 / 5.0), k01_06 = sqrt(1.0 / 6.0),
        k05_06 = sqrt(5.0 / 6.0), k03_08 = sqrt(3.0 / 8.0), k05_08 = sqrt(5.0 / 8.0),
        k09_08 = sqrt(9.0 / 8.0), k05_09 = sqrt(5.0 / 9.0), k08_09 = sqrt(8.0 / 9.0),
        k01_10 = sqrt(1.0 / 10.0), k03_10 = sqrt(3.0 / 10.0), k01_12 = sqrt(1.0 / 12.0),
        k04_15 = sqrt(4.0 / 15.0), k01_16 = sqrt(1.0 / 16.0), k15_16 = sqrt(15.0 / 16.0),
        k01_18 = sqrt(1.0 / 18.0), k01_60 = sqrt(1.0 / 60.0);
    const double r[9] = {m3[0], m3[1], m3[2], m3[3], m3[4], m3[5], m3[6], m3[7], m3[8]};
    double a[3][3]; /* sh1 */
    a[0][0] = r[4]; a[0][1] = -r[7]; a[0][2] = r[1];
    a[1][0] = -r[5]; a[1][1] = r[8]; a[1][2] = -r[2];
    a[2][0] = r[3]; a[2][1] = -r[6]; a[2][2] = r[0];
    double b[5][5]; /* sh2 */
    b[0][0] = k01_04 * ((a[2][2] * a[0][0] + a[2][0] * a[0][2]) + (a[0][2] * a[2][0] + a[0][0] * a[2][2]));
    b[0][1] = (a[2][1] * a[0][0] + a[0][1] * a[2][0]);
    b[0][2] = k03_04 * (a[2][1] * a[0][1] + a[0][1] * a[2][1]);
    b[0][3] = (a[2][1] * a[0][2] + a[0][1] * a[2][2]);
    b[0][4] = k01_04 * ((a[2][2] * a[0][2] - a[2][0] * a[0][0]) + (a[0][2] * a[2][2] - a[0][0] * a[2][0]));
    b[1][0] = k01_04 * ((a[1][2] * a[0][0] + a[1][0] * a[0][2]) + (a[0][2] * a[1][0] + a[0][0] * a[1][2]));
    b[1][1] = a[1][1] * a[0][0] + a[0][1] * a[1][0];
    b[1][2] = k03_04 * (a[1][1] * a[0][1] + a[0][1] * a[1][1]);
    b[1][3] = a[1][1] * a[0][2] + a[0][1] * a[1][2];
    b[1][4] = k01_04 * ((a[1][2] * a[0][2] - a[1][0] * a[0][0]) + (a[0][2] * a[1][2] - a[0][0] * a[1][0]));
    b[2][0] = k01_03 * (a[1][2] * a[1][0] + a[1][0] * a[1][2]) - k01_12 * ((a[2][2] * a[2][0] + a[2][0] * a[2][2]) + (a[0][2] * a[0][0] + a[0][0] * a[0][2]));
    b[2][1] = k04_03 * a[1][1] * a[1][0] - k01_03 * (a[2][1] * a[2][0] + a[0][1] * a[0][0]);
    b[2][2] = a[1][1] * a[1][1] - k01_04 * (a[2][1] * a[2][1] + a[0][1] * a[0][1]);
    b[2][3] = k04_03 * a[1][1] * a[1][2] - k01_03 * (a[2][1] * a[2][2] + a[0][1] * a[0][2]);
    b[2][4] = k01_03 * (a[1][2] * a[1][2] - a[1][0] * a[1][0]) - k01_12 * ((a[2][2] * a[2][2] - a[2][0] * a[2][0]) + (a[0][2] * a[0][2] - a[0][0] * a[0][0]));
    b[3][0] = k01_04 * ((a[1][2] * a[2][0] + a[1][0] * a[2][2]) + (a[2][2] * a[1][0] + a[2][0] * a[1][2]));
    b[3][1] = a[1][1] * a[2][0] + a[2][1] * a[1][0];
    b[3][2] = k03_04 * (a[1][1] * a[2][1] + a[2][1] * a[1][1]);
    b[3][3] = a[1][1] * a[2][2] + a[2][1] * a[1][2];
    b[3][4] = k01_04 * ((a[1][2] * a[2][2] - a[1][0] * a[2][0]) + (a[2][2] * a[1][2] - a[2][0] * a[1][0]));
    b[4][0] = k01_04 * ((a[2][2] * a[2][0] + a[2][0] * a[2][2]) - (a[0][2] * a[0][0] + a[0][0] * a[0][2]));
    b[4][1] = (a[2][1] * a[2][0] - a[0][1] * a[0][0]);
    b[4][2] = k03_04 * (a[2][1] * a[2][1] - a[0][1] * a[0][1]);
    b[4][3] = (a[2][1] * a[2][2] - a[0][1] * a[0][2]);
    b[4][4] = k01_04 * ((a[2][2] * a[2][2] - a[2][0] * a[2][0]) - (a[0][2] * a[0][2] - a[0][0] * a[0][0]));
    double c[7][7]; /* sh3 */
    c[0][0] = k01_04 * ((a[2][2] * b[0][0] + a[2][0] * b[0][4]) + (a[0][2] * b[4][0] + a[0][0] * b[4][4]));
    c[0][1] = k03_02 * (a[2][1] * b[0][0] + a[0][1] * b[4][0]);
    c[0][2] = k15_16 * (a[2][1] * b[0][1] + a[0][1] * b[4][1]);
    c[0][3] = k05_06 * (a[2][1] * b[0][2] + a[0][1] * b[4][2]);
    c[0][4] = k15_16 * (a[2][1] * b[0][3] + a[0][1] * b[4][3]);
    c[0][5] = k03_02 * (a[2][1] * b[0][4] + a[0][1] * b[4][4]);
    c[0][6] = k01_04 * ((a[2][2] * b[0][4] - a[2][0] * b[0][0]) + (a[0][2] * b[4][4] - a[0][0] * b[4][0]));
    c[1][0] = k01_06 * (a[1][2] * b[0][0] + a[1][0] * b[0][4]) + k01_06 * ((a[2][2] * b[1][0] + a[2][0] * b[1][4]) + (a[0][2] * b[3][0] + a[0][0] * b[3][4]));
    c[1][1] = a[1][1] * b[0][0] + (a[2][1] * b[1][0] + a[0][1] * b[3][0]);
    c[1][2] = k05_08 * a[1][1] * b[0][1] + k05_08 * (a[2][1] * b[1][1] + a[0][1] * b[3][1]);
    c[1][3] = k05_09 * a[1][1] * b[0][2] + k05_09 * (a[2][1] * b[1][2] + a[0][1] * b[3][2]);
    c[1][4] = k05_08 * a[1][1] * b[0][3] + k05_08 * (a[2][1] * b[1][3] + a[0][1] * b[3][3]);
    c[1][5] = a[1][1] * b[0][4] + (a[2][1] * b[1][4] + a[0][1] * b[3][4]);
    c[1][6] = k01_06 * (a[1][2] * b[0][4] - a[1][0] * b[0][0]) + k01_06 * ((a[2][2] * b[1][4] - a[2][0] * b[1][0]) + (a[0][2] * b[3][4] - a[0][0] * b[3][0]));
    c[2][0] = k04_15 * (a[1][2] * b[1][0] + a[1][0] * b[1][4]) + k01_05 * (a[0][2] * b[2][0] + a[0][0] * b[2][4]) - k01_60 * ((a[2][2] * b[0][0] + a[2][0] * b[0][4]) - (a[0][2] * b[4][0] + a[0][0] * b[4][4]));
    c[2][1] = k08_05 * a[1][1] * b[1][0] + k06_05 * a[0][1] * b[2][0] - k01_10 * (a[2][1] * b[0][0] - a[0][1] * b[4][0]);
    c[2][2] = a[1][1] * b[1][1] + k03_04 * a[0][1] * b[2][1] - k01_16 * (a[2][1] * b[0][1] - a[0][1] * b[4][1]);
    c[2][3] = k08_09 * a[1][1] * b[1][2] + k02_03 * a[0][1] * b[2][2] - k01_18 * (a[2][1] * b[0][2] - a[0][1] * b[4][2]);
    c[2][4] = a[1][1] * b[1][3] + k03_04 * a[0][1] * b[2][3] - k01_16 * (a[2][1] * b[0][3] - a[0][1] * b[4][3]);
    c[2][5] = k08_05 * a[1][1] * b[1][4] + k06_05 * a[0][1] * b[2][4] - k01_10 * (a[2][1] * b[0][4] - a[0][1] * b[4][4]);
    c[2][6] = k04_15 * (a[1][2] * b[1][4] - a[1][0] * b[1][0]) + k01_05 * (a[0][2] * b[2][4] - a[0][0] * b[2][0]) - k01_60 * ((a[2][2] * b[0][4] - a[2][0] * b[0][0]) - (a[0][2] * b[4][4] - a[0][0] * b[4][0]));
    c[3][0] = k03_10 * (a[1][2] * b[2][0] + a[1][0] * b[2][4]) - k01_10 * ((a[2][2] * b[3][0] + a[2][0] * b[3][4]) + (a[0][2] * b[1][0] + a[0][0] * b[1][4]));
    c[3][1] = k09_05 * a[1][1] * b[2][0] - k03_05 * (a[2][1] * b[3][0] + a[0][1] * b[1][0]);
    c[3][2] = k09_08 * a[1][1] * b[2][1] - k03_08 * (a[2][1] * b[3][1] + a[0][1] * b[1][1]);
    c[3][3] = a[1][1] * b[2][2] - k01_03 * (a[2][1] * b[3][2] + a[0][1] * b[1][2]);
    c[3][4] = k09_08 * a[1][1] * b[2][3] - k03_08 * (a[2][1] * b[3][3] + a[0][1] * b[1][3]);
    c[3][5] = k09_05 * a[1][1] * b[2][4] - k03_05 * (a[2][1] * b[3][4] + a[0][1] * b[1][4]);
    c[3][6] = k03_10 * (a[1][2] * b[2][4] - a[1][0] * b[2][0]) - k01_10 * ((a[2][2] * b[3][4] - a[2][0] * b[3][0]) + (a[0][2] * b[1][4] - a[0][0] * b[1][0]));
    c[4][0] = k04_15 * (a[1][2] * b[3][0] + a[1][0] * b[3][4]) + k01_05 * (a[2][2] * b[2][0] + a[2][0] * b[2][4]) - k01_60 * ((a[2][2] * b[4][0] + a[2][0] * b[4][4]) + (a[0][2] * b[0][0] + a[0][0] * b[0][4]));
    c[4][1] = k08_05 * a[1][1] * b[3][0] + k06_05 * a[2][1] * b[2][0] - k01_10 * (a[2][1] * b[4][0] + a[0][1] * b[0][0]);
    c[4][2] = a[1][1] * b[3][1] + k03_04 * a[2][1] * b[2][1] - k01_16 * (a[2][1] * b[4][1] + a[0][1] * b[0][1]);
    c[4][3] = k08_09 * a[1][1] * b[3][2] + k02_03 * a[2][1] * b[2][2] - k01_18 * (a[2][1] * b[4][2] + a[0][1] * b[0][2]);
    c[4][4] = a[1][1] * b[3][3] + k03_04 * a[2][1] * b[2][3] - k01_16 * (a[2][1] * b[4][3] + a[0][1] * b[0][3]);
    c[4][5] = k08_05 * a[1][1] * b[3][4] + k06_05 * a[2][1] * b[2][4] - k01_10 * (a[2][1] * b[4][4] + a[0][1] * b[0][4]);
    c[4][6] = k04_15 * (a[1][2] * b[3][4] - a[1][0] * b[3][0]) + k01_05 * (a[2][2] * b[2][4] - a[2][0] * b[2][0]) - k01_60 * ((a[2][2] * b[4][4] - a[2][0] * b[4][0]) + (a[0][2] * b[0][4] - a[0][0] * b[0][0]));
    c[5][0] = k01_06 * (a[1][2] * b[4][0] + a[1][0] * b[4][4]) + k01_06 * ((a[2][2] * b[3][0] + a[2][0] * b[3][4]) - (a[0][2] * b[1][0] + a[0][0] * b[1][4]));
    c[5][1] = a[1][1] * b[4][0] + (a[2][1] * b[3][0] - a[0][1] * b[1][0]);
    c[5][2] = k05_08 * a[1][1] * b[4][1] + k05_08 * (a[2][1] * b[3][1] - a[0][1] * b[1][1]);
    c[5][3] = k05_09 * a[1][1] * b[4][2] + k05_09 * (a[2][1] * b[3][2] - a[0][1] * b[1][2]);
    c[5][4] = k05_08 * a[1][1] * b[4][3] + k05_08 * (a[2][1] * b[3][3] - a[0][1] * b[1][3]);
    c[5][5] = a[1][1] * b[4][4] + (a[2][1] * b[3][4] - a[0][1] * b[1][4]);
    c[5][6] = k01_06 * (a[1][2] * b[4][4] - a[1][0] * b[4][0]) + k01_06 * ((a[2][2] * b[3][4] - a[2][0] * b[3][0]) - (a[0][2] * b[1][4] - a[0][0] * b[1][0]));
    c[6][0] = k01_04 * ((a[2][2] * b[4][0] + a[2][0] * b[4][4]) - (a[0][2] * b[0][0] + a[0][0] * b[0][4]));
    c[6][1] = k03_02 * (a[2][1] * b[4][0] - a[0][1] * b[0][0]);
    c[6][2] = k15_16 * (a[2][1] * b[4][1] - a[0][1] * b[0][1]);
    c[6][3] = k05_06 * (a[2][1] * b[4][2] - a[0][1] * b[0][2]);
    c[6][4] = k15_16 * (a[2][1] * b[4][3] - a[0][1] * b[0][3]);
    c[6][5] = k03_02 * (a[2][1] * b[4][4] - a[0][1] * b[0][4]);
    c[6][6] = k01_04 * ((a[2][2] * b[4][4] - a[2][0] * b[4][0]) - (a[0][2] * b[0][4] - a[0][0] * b[0][0]));
    memcpy(o1, a, sizeof(a));
    memcpy(o2, b, sizeof(b));
    memcpy(o3, c, sizeof(c));
}

/* dp (rotate-sh.ts:32-38): sequential f64 sum starting from 0 */
static inline double dp(int n, const float *src, const double *row)
{
    double sum = 0;
    for (int i = 0; i < n; i++) sum += (double)src[i] * row[i];
    return sum;
}

/* ------------------------------------------------------------------------- */
/* transform (transform.ts:12-65)                                              */

void st_o_transform(uint64_t n, float *x, float *y, float *z, float *const rot[4],
                    float *const scale[3], float *const *sh, int C,
                    const float m[16], const double r[4], double s,
                    const double sh1[9], const double sh2[25], const double sh3[49])
{
    float coeffs[15], src[15];
    for (uint64_t i = 0; i < n; ++i) {
        if (x && y && z) {
            const double vx = x[i], vy = y[i], vz = z[i];
            x[i] = (float)(vx * m[0] + vy * m[4] + vz * m[8] + m[12]);
            y[i] = (float)(vx * m[1] + vy * m[5] + vz * m[9] + m[13]);
            z[i] = (float)(vx * m[2] + vy * m[6] + vz * m[10] + m[14]);
        }
        if (rot) {
            /* q = (x=rot_1, y=rot_2, z=rot_3, w=rot_0); q.mul2(r, q) */
            const double q2x = rot[1][i], q2y = rot[2][i], q2z = rot[3][i], q2w = rot[0][i];
            const double q1x = r[0], q1y = r[1], q1z = r[2], q1w = r[3];
            const double nx = q1w * q2x + q1x * q2w + q1y * q2z - q1z * q2y;
            const double ny = q1w * q2y + q1y * q2w + q1z * q2x - q1x * q2z;
            const double nz = q1w * q2z + q1z * q2w + q1x * q2y - q1y * q2x;
            const double nw = q1w * q2w - q1x * q2x - q1y * q2y - q1z * q2z;
            rot[0][i] = (float)nw;
            rot[1][i] = (float)nx;
            rot[2][i] = (float)ny;
            rot[3][i] = (float)nz;
        }
        if (scale) {
            for (int c = 0; c < 3; ++c) scale[c][i] = (float)st_o_log(st_o_exp((double)scale[c][i]) * s);
        }
        if (C > 0) {
            for (int ch = 0; ch < 3; ++ch) {
                for (int k = 0; k < C; ++k) coeffs[k] = sh[k + ch * C][i];
                memcpy(src, coeffs, sizeof(float) * C);
                for (int r1 = 0; r1 < 3; ++r1) coeffs[r1] = (float)dp(3, src, sh1 + r1 * 3);
                if (C >= 8)
                    for (int r2 = 0; r2 < 5; ++r2) coeffs[3 + r2] = (float)dp(5, src + 3, sh2 + r2 * 5);
                if (C >= 15)
                    for (int r3 = 0; r3 < 7; ++r3) coeffs[8 + r3] = (float)dp(7, src + 8, sh3 + r3 * 7);
                for (int k = 0; k < C; ++k) sh[k + ch * C][i] = coeffs[k];
            }
        }
    }
}

/* ------------------------------------------------------------------------- */
/* filterNaN (process.ts:84-95 -> filter :47-61)                               */

uint64_t st_o_filter_finite(uint64_t n, int ncol, const float *const *cols, uint32_t *out_idx)
{
    uint64_t m = 0;
    for (uint64_t i = 0; i < n; ++i) {
        int keep = 1;
        for (int c = 0; c < ncol && keep; ++c)
            if (!isfinite(cols[c][i])) keep = 0;
        if (keep) out_idx[m++] = (uint32_t)i;
    }
    return m;
}

/* ------------------------------------------------------------------------- */
/* stable merge sort of uint32 indices by a comparator returning a double whose
 * sign orders (V8 TypedArray.prototype.sort is stable; NaN compares as 0). */

typedef double (*cmp_fn)(const void *ctx, uint32_t a, uint32_t b);

static void merge_sort(uint32_t *a, uint32_t *tmp, uint64_t n, cmp_fn cmp, const void *ctx)
{
    if (n < 2) return;
    for (uint64_t w = 1; w < n; w *= 2) {
        for (uint64_t lo = 0; lo < n; lo += 2 * w) {
            uint64_t mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
            uint64_t i = lo, j = mid, k = lo;
            while (i < mid && j < hi) {
                double c = cmp(ctx, a[i], a[j]);
                if (c > 0) tmp[k++] = a[j++]; /* NaN / <=0 keeps the left element first */
                else tmp[k++] = a[i++];
            }
            while (i < mid) tmp[k++] = a[i++];
            while (j < hi) tmp[k++] = a[j++];
        }
        memcpy(a, tmp, n * sizeof(uint32_t));
    }
}

static double cmp_u32_key(const void *ctx, uint32_t a, uint32_t b)
{
    const uint32_t *key = (const uint32_t *)ctx;
    return (double)key[a] - (double)key[b];
}

static double cmp_f32_key(const void *ctx, uint32_t a, uint32_t b)
{
    const float *key = (const float *)ctx;
    return (double)key[a] - (double)key[b];
}

/* ------------------------------------------------------------------------- */
/* generateOrdering (ordering.ts:4-110)                                        */

static uint32_t part1by2(uint32_t x)
{
    x &= 0x000003ff;
    x = (x ^ (x << 16)) & 0xff0000ff;
    x = (x ^ (x << 8)) & 0x0300f00f;
    x = (x ^ (x << 4)) & 0x030c30c3;
    x = (x ^ (x << 2)) & 0x09249249;
    return x;
}

static uint32_t morton_axis(double v, double mn, double mul)
{
    return js_to_uint32(js_min(1023, (v - mn) * mul));
}

static void morton_generate(const float *cx, const float *cy, const float *cz, uint32_t *indices, uint64_t len)
{
    if (len == 0) return; /* extents undefined -> 'invalid extents' */
    double mx, my, mz, Mx, My, Mz;
    mx = Mx = cx[indices[0]];
    my = My = cy[indices[0]];
    mz = Mz = cz[indices[0]];
    for (uint64_t i = 1; i < len; ++i) {
        const double x = cx[indices[i]], y = cy[indices[i]], z = cz[indices[i]];
        if (x < mx) mx = x; else if (x > Mx) Mx = x;
        if (y < my) my = y; else if (y > My) My = y;
        if (z < mz) mz = z; else if (z > Mz) Mz = z;
    }
    const double xlen = Mx - mx, ylen = My - my, zlen = Mz - mz;
    if (!isfinite(xlen) || !isfinite(ylen) || !isfinite(zlen)) return;
    if (xlen == 0 && ylen == 0 && zlen == 0) return;
    const double xmul = (xlen == 0) ? 0 : 1024 / xlen;
    const double ymul = (ylen == 0) ? 0 : 1024 / ylen;
    const double zmul = (zlen == 0) ? 0 : 1024 / zlen;
    uint32_t *morton = (uint32_t *)malloc(len * sizeof(uint32_t));
    uint32_t *order = (uint32_t *)malloc(len * sizeof(uint32_t));
    uint32_t *tmp = (uint32_t *)malloc(len * sizeof(uint32_t));
    for (uint64_t i = 0; i < len; ++i) {
        const uint32_t ri = indices[i];
        const uint32_t ix = morton_axis(cx[ri], mx, xmul);
        const uint32_t iy = morton_axis(cy[ri], my, ymul);
        const uint32_t iz = morton_axis(cz[ri], mz, zmul);
        morton[i] = (part1by2(iz) << 2) + (part1by2(iy) << 1) + part1by2(ix);
        order[i] = (uint32_t)i;
    }
    merge_sort(order, tmp, len, cmp_u32_key, morton);
    memcpy(tmp, indices, len * sizeof(uint32_t));
    for (uint64_t i = 0; i < len; ++i) indices[i] = tmp[order[i]];
    uint64_t start = 0, end = 1;
    while (start < len) {
        while (end < len && morton[order[end]] == morton[order[start]]) ++end;
        if (end - start > 256) morton_generate(cx, cy, cz, indices + start, end - start);
        start = end;
    }
    free(morton);
    free(order);
    free(tmp);
}

void st_o_morton_order(const float *x, const float *y, const float *z, uint32_t *indices, uint64_t n)
{
    morton_generate(x, y, z, indices, n);
}

/* ------------------------------------------------------------------------- */
/* CompressedChunk.pack (compressed-chunk.ts:44-180)                           */

static inline double normalize01(double x, double mn, double mx)
{
    if (x <= mn) return 0;
    if (x >= mx) return 1;
    return (mx - mn < 0.00001) ? 0 : (x - mn) / (mx - mn);
}

static inline int32_t pack_unorm(double value, int bits)
{
    const double t = (double)((1 << bits) - 1);
    return js_to_int32(js_max(0, js_min(t, floor(value * t + 0.5))));
}

static inline uint32_t pack111011(double x, double y, double z)
{
    return ((uint32_t)pack_unorm(x, 11) << 21) | ((uint32_t)pack_unorm(y, 10) << 11) | (uint32_t)pack_unorm(z, 11);
}

static inline uint32_t pack8888(double x, double y, double z, double w)
{
    return ((uint32_t)pack_unorm(x, 8) << 24) | ((uint32_t)pack_unorm(y, 8) << 16) |
           ((uint32_t)pack_unorm(z, 8) << 8) | (uint32_t)pack_unorm(w, 8);
}

static uint32_t pack_rot(double x, double y, double z, double w)
{
    double len = sqrt(x * x + y * y + z * z + w * w);
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
    for (int i = 0; i < 4; ++i)
        if (fabs(a[i]) > fabs(a[largest])) largest = i;
    if (a[largest] < 0) {
        a[0] = -a[0];
        a[1] = -a[1];
        a[2] = -a[2];
        a[3] = -a[3];
    }
    const double norm = sqrt(2) * 0.5;
    uint32_t result = (uint32_t)largest;
    for (int i = 0; i < 4; ++i)
        if (i != largest) result = (result << 10) | (uint32_t)pack_unorm(a[i] * norm + 0.5, 10);
    return result;
}

static void minmax_js(const float *d, int n, double *mn, double *mx)
{
    double a = d[0], b = d[0];
    for (int i = 1; i < n; ++i) {
        a = js_min(a, d[i]);
        b = js_max(b, d[i]);
    }
    *mn = a;
    *mx = b;
}

static inline double clamp_js(double v, double lo, double hi) { return js_max(lo, js_min(hi, v)); }

void st_o_pack_compressed(uint64_t n, const float *const m14[14], const float *const *sh, int nsh,
                          const uint32_t *order, float *chunk_out, uint32_t *vertex, uint8_t *sh_out)
{
    enum { X, Y, Z, S0, S1, S2, R, G, B, OP, Q0, Q1, Q2, Q3 };
    const double SH_C0 = 0.28209479177387814;
    float d[14][256];
    const uint64_t nchunks = (n + 255) / 256;
    for (uint64_t c = 0; c < nchunks; ++c) {
        const uint64_t num = (n < (c + 1) * 256 ? n : (c + 1) * 256) - c * 256;
        uint32_t last = 0;
        for (uint64_t j = 0; j < num; ++j) {
            const uint32_t idx = order[c * 256 + j];
            last = idx;
            for (int m = 0; m < 14; ++m) d[m][j] = m14[m][idx];
            uint8_t *o = sh_out + (c * 256 + j) * (uint64_t)nsh;
            for (int k = 0; k < nsh; ++k) {
                const double nv = (double)sh[k][idx] / 8 + 0.5;
                o[k] = js_to_uint8(js_max(0, js_min(255, trunc(nv * 256))));
            }
        }
        for (uint64_t j = num; j < 256; ++j)
            for (int m = 0; m < 14; ++m) d[m][j] = m14[m][last];
        double pxn, pxx, pyn, pyx, pzn, pzx, sxn, sxx, syn, syx, szn, szx;
        minmax_js(d[X], 256, &pxn, &pxx);
        minmax_js(d[Y], 256, &pyn, &pyx);
        minmax_js(d[Z], 256, &pzn, &pzx);
        minmax_js(d[S0], 256, &sxn, &sxx);
        minmax_js(d[S1], 256, &syn, &syx);
        minmax_js(d[S2], 256, &szn, &szx);
        sxn = clamp_js(sxn, -20, 20); sxx = clamp_js(sxx, -20, 20);
        syn = clamp_js(syn, -20, 20); syx = clamp_js(syx, -20, 20);
        szn = clamp_js(szn, -20, 20); szx = clamp_js(szx, -20, 20);
        for (int i = 0; i < 256; ++i) {
            d[R][i] = (float)((double)d[R][i] * SH_C0 + 0.5);
            d[G][i] = (float)((double)d[G][i] * SH_C0 + 0.5);
            d[B][i] = (float)((double)d[B][i] * SH_C0 + 0.5);
        }
        double crn, crx, cgn, cgx, cbn, cbx;
        minmax_js(d[R], 256, &crn, &crx);
        minmax_js(d[G], 256, &cgn, &cgx);
        minmax_js(d[B], 256, &cbn, &cbx);
        for (uint64_t j = 0; j < num; ++j) {
            uint32_t *v = vertex + (c * 256 + j) * 4;
            v[0] = pack111011(normalize01(d[X][j], pxn, pxx), normalize01(d[Y][j], pyn, pyx), normalize01(d[Z][j], pzn, pzx));
            v[1] = pack_rot(d[Q0][j], d[Q1][j], d[Q2][j], d[Q3][j]);
            v[2] = pack111011(normalize01(d[S0][j], sxn, sxx), normalize01(d[S1][j], syn, syx), normalize01(d[S2][j], szn, szx));
            v[3] = pack8888(normalize01(d[R][j], crn, crx), normalize01(d[G][j], cgn, cgx), normalize01(d[B][j], cbn, cbx),
                            sigmoid(d[OP][j]));
        }
        const double cd[18] = {pxn, pyn, pzn, pxx, pyx, pzx, sxn, syn, szn, sxx, syx, szx, crn, cgn, cbn, crx, cgx, cbx};
        for (int q = 0; q < 18; ++q) chunk_out[c * 18 + q] = (float)cd[q];
    }
}

/* ------------------------------------------------------------------------- */
/* KdTree (kd-tree.ts:9-100)                                                   */

typedef struct { int32_t index, left, right; } kdnode;

typedef struct {
    const float *const *cols; /* d columns of k centroids */
    int d;
    kdnode *nodes;
    int nnodes;
    uint32_t *tmp;
} kdtree;

static int kd_build(kdtree *t, uint32_t *idx, uint64_t len, int depth)
{
    const float *values = t->cols[depth % t->d];
    merge_sort(idx, t->tmp, len, cmp_f32_key, values);
    const int me = t->nnodes++;
    if (len == 1) {
        t->nodes[me] = (kdnode){(int32_t)idx[0], -1, -1};
        return me;
    }
    if (len == 2) {
        const int r = t->nnodes++;
        t->nodes[r] = (kdnode){(int32_t)idx[1], -1, -1};
        t->nodes[me] = (kdnode){(int32_t)idx[0], -1, r};
        return me;
    }
    const uint64_t mid = len >> 1;
    const int l = kd_build(t, idx, mid, depth + 1);
    const int r = kd_build(t, idx + mid + 1, len - mid - 1, depth + 1);
    t->nodes[me] = (kdnode){(int32_t)idx[mid], l, r};
    return me;
}

typedef struct { const kdtree *t; const float *point; double mind; int32_t mini; } kdsearch;

static double kd_distance(const kdtree *t, uint32_t index, const float *point)
{
    double l = 0;
    for (int i = 0; i < t->d; ++i) {
        const double v = (double)t->cols[i][index] - (double)point[i];
        l += v * v;
    }
    return l;
}

static void kd_recurse(kdsearch *s, int node, int depth)
{
    const kdtree *t = s->t;
    const kdnode *nd = &t->nodes[node];
    const int axis = depth % t->d;
    const double distance = (double)s->point[axis] - (double)t->cols[axis][nd->index];
    const int next = (distance > 0) ? nd->right : nd->left;
    if (next >= 0) kd_recurse(s, next, depth + 1);
    const double thisd = kd_distance(t, (uint32_t)nd->index, s->point);
    if (thisd < s->mind) {
        s->mind = thisd;
        s->mini = nd->index;
    }
    if (distance * distance < s->mind) {
        const int other = (next == nd->right) ? nd->left : nd->right;
        if (other >= 0) kd_recurse(s, other, depth + 1);
    }
}

/* ------------------------------------------------------------------------- */
/* kmeans (k-means.ts:137-201)                                                 */

typedef struct { const double *draws; uint64_t n, used; } rng;

/* threads for st_o_kmeans's assign loop (1 = the reference's sequential loop) */
static int o_threads = 1;
void st_o_set_threads(int threads) { o_threads = threads > 1 ? threads : 1; }

static int rng_next(rng *r, double *out)
{
    if (r->used >= r->n) return -2;
    *out = r->draws[r->used++];
    return 0;
}

int st_o_kmeans(const float *const *cols, int d, uint64_t n, int k, int iters,
                const double *draws, uint64_t ndraws, uint64_t *used,
                float *centroids, uint32_t *labels)
{
    rng R = {draws, ndraws, 0};
    if (n < (uint64_t)k) {
        for (int c = 0; c < d; ++c) memcpy(centroids + (uint64_t)c * n, cols[c], n * sizeof(float));
        for (uint64_t i = 0; i < n; ++i) labels[i] = (uint32_t)i;
        *used = 0;
        return 0;
    }
    float **ccols = (float **)malloc(sizeof(float *) * d);
    for (int c = 0; c < d; ++c) ccols[c] = centroids + (uint64_t)c * k;
    if (d == 1) {
        double m = INFINITY, M = -INFINITY;
        for (uint64_t i = 0; i < n; ++i) {
            const double v = cols[0][i];
            if (v < m) m = v;
            if (v > M) M = v;
        }
        for (int i = 0; i < k; ++i) ccols[0][i] = (float)(m + (M - m) * i / (k - 1));
    } else {
        uint8_t *chosen = (uint8_t *)calloc(n, 1);
        for (int i = 0; i < k; ++i) {
            uint64_t cand;
            do {
                double u;
                if (rng_next(&R, &u)) { free(chosen); free(ccols); return -2; }
                cand = (uint64_t)floor(u * (double)n);
            } while (chosen[cand]);
            chosen[cand] = 1;
            for (int c = 0; c < d; ++c) ccols[c][i] = cols[c][cand];
        }
        free(chosen);
    }
    kdtree t;
    t.cols = (const float *const *)ccols;
    t.d = d;
    t.nodes = (kdnode *)malloc(sizeof(kdnode) * k);
    t.tmp = (uint32_t *)malloc(sizeof(uint32_t) * k);
    uint32_t *kidx = (uint32_t *)malloc(sizeof(uint32_t) * k);
    float *point = (float *)malloc(sizeof(float) * d);
    uint64_t *count = (uint64_t *)malloc(sizeof(uint64_t) * k);
    double *sums = (double *)malloc(sizeof(double) * (uint64_t)k * d);
    int rc = 0;
    for (int step = 0; step < iters && rc == 0; ++step) {
        for (int i = 0; i < k; ++i) kidx[i] = (uint32_t)i;
        t.nnodes = 0;
        const int root = kd_build(&t, kidx, (uint64_t)k, 0);
        if (o_threads > 1) {
            /* the point loop over OpenMP threads: each search only reads the tree, so the
             * labels are those of the sequential loop (fixture generation at N = 100k) */
#pragma omp parallel num_threads(o_threads) reduction(|: rc)
            {
                float *pt = (float *)malloc(sizeof(float) * d);
#pragma omp for schedule(dynamic, 16)
                for (uint64_t i = 0; i < n; ++i) {
                    for (int c = 0; c < d; ++c) pt[c] = cols[c][i];
                    kdsearch s = {&t, pt, INFINITY, -1};
                    kd_recurse(&s, root, 0);
                    if (s.mini < 0) rc = -1;
                    else labels[i] = (uint32_t)s.mini;
                }
                free(pt);
            }
        } else {
            for (uint64_t i = 0; i < n; ++i) {
                for (int c = 0; c < d; ++c) point[c] = cols[c][i];
                kdsearch s = {&t, point, INFINITY, -1};
                kd_recurse(&s, root, 0);
                if (s.mini < 0) { rc = -1; break; } /* reference crashes (labels[i] = -1) */
                labels[i] = (uint32_t)s.mini;
            }
        }
        if (rc) break;
        /* groupLabels + calcAverage: f64 running sum in ascending point order */
        memset(count, 0, sizeof(uint64_t) * k);
        memset(sums, 0, sizeof(double) * (uint64_t)k * d);
        for (uint64_t i = 0; i < n; ++i) {
            const uint32_t l = labels[i];
            count[l]++;
            for (int c = 0; c < d; ++c) sums[(uint64_t)l * d + c] += (double)cols[c][i];
        }
        for (int i = 0; i < k; ++i) {
            if (count[i] == 0) {
                double u;
                if (rng_next(&R, &u)) { rc = -2; break; }
                const uint64_t idx = (uint64_t)floor(u * (double)n);
                for (int c = 0; c < d; ++c) ccols[c][i] = cols[c][idx];
            } else {
                for (int c = 0; c < d; ++c) ccols[c][i] = (float)(sums[(uint64_t)i * d + c] / (double)count[i]);
            }
        }
    }
    *used = R.used;
    free(ccols); free(t.nodes); free(t.tmp); free(kidx); free(point); free(count); free(sums);
    return rc;
}

int st_o_kmeans_assign(const float *const *cols, int d, uint64_t n, const float *centroids, int k, uint32_t *labels)
{
    const float **ccols = (const float **)malloc(sizeof(float *) * d);
    for (int c = 0; c < d; ++c) ccols[c] = centroids + (uint64_t)c * k;
    kdtree t;
    t.cols = ccols;
    t.d = d;
    t.nodes = (kdnode *)malloc(sizeof(kdnode) * k);
    t.tmp = (uint32_t *)malloc(sizeof(uint32_t) * k);
    t.nnodes = 0;
    uint32_t *kidx = (uint32_t *)malloc(sizeof(uint32_t) * k);
    for (int i = 0; i < k; ++i) kidx[i] = (uint32_t)i;
    const int root = kd_build(&t, kidx, (uint64_t)k, 0);
    float *point = (float *)malloc(sizeof(float) * d);
    int rc = 0;
    for (uint64_t i = 0; i < n; ++i) {
        for (int c = 0; c < d; ++c) point[c] = cols[c][i];
        kdsearch s = {&t, point, INFINITY, -1};
        kd_recurse(&s, root, 0);
        if (s.mini < 0) { rc = -1; break; }
        labels[i] = (uint32_t)s.mini;
    }
    free(ccols); free(t.nodes); free(t.tmp); free(kidx); free(point);
    return rc;
}

/* The same assign with the point loop split over `threads` OpenMP threads (one tree, built
 * once; each search reads it only).  Used to time the reference algorithm on every host core
 * for the bench's CPU baseline; the labels are those of st_o_kmeans_assign. */
int st_o_kmeans_assign_mt(const float *const *cols, int d, uint64_t n, const float *centroids, int k,
                          uint32_t *labels, int threads)
{
    const float **ccols = (const float **)malloc(sizeof(float *) * d);
    for (int c = 0; c < d; ++c) ccols[c] = centroids + (uint64_t)c * k;
    kdtree t;
    t.cols = ccols;
    t.d = d;
    t.nodes = (kdnode *)malloc(sizeof(kdnode) * k);
    t.tmp = (uint32_t *)malloc(sizeof(uint32_t) * k);
    t.nnodes = 0;
    uint32_t *kidx = (uint32_t *)malloc(sizeof(uint32_t) * k);
    for (int i = 0; i < k; ++i) kidx[i] = (uint32_t)i;
    const int root = kd_build(&t, kidx, (uint64_t)k, 0);
    int rc = 0;
#pragma omp parallel num_threads(threads) reduction(|: rc)
    {
        float *point = (float *)malloc(sizeof(float) * d);
#pragma omp for schedule(dynamic, 16)
        for (uint64_t i = 0; i < n; ++i) {
            for (int c = 0; c < d; ++c) point[c] = cols[c][i];
            kdsearch s = {&t, point, INFINITY, -1};
            kd_recurse(&s, root, 0);
            if (s.mini < 0) rc = -1;
            else labels[i] = (uint32_t)s.mini;
        }
        free(point);
    }
    free(ccols); free(t.nodes); free(t.tmp); free(kidx);
    return rc;
}

/* cluster1d (write-sog.ts:56-99) */
int st_o_cluster1d(const float *const *cols, int ncols, uint64_t n, int iters,
                   const double *draws, uint64_t ndraws, uint64_t *used,
                   float *centroids, uint8_t *labels_out)
{
    const uint64_t total = n * (uint64_t)ncols;
    if (total < 256) return -3; /* reference: kmeans returns a plain Array; .subarray throws */
    float *data = (float *)malloc(sizeof(float) * total);
    for (int c = 0; c < ncols; ++c) memcpy(data + c * n, cols[c], n * sizeof(float));
    uint32_t *labels = (uint32_t *)malloc(sizeof(uint32_t) * total);
    const float *pcols[1] = {data};
    float cent[256];
    int rc = st_o_kmeans(pcols, 1, total, 256, iters, draws, ndraws, used, cent, labels);
    if (rc == 0) {
        uint32_t order[256], tmp[256], inv[256];
        for (int i = 0; i < 256; ++i) order[i] = (uint32_t)i;
        merge_sort(order, tmp, 256, cmp_f32_key, cent);
        for (int i = 0; i < 256; ++i) centroids[i] = cent[order[i]];
        for (int i = 0; i < 256; ++i) inv[order[i]] = (uint32_t)i;
        for (uint64_t i = 0; i < total; ++i) labels_out[i] = (uint8_t)inv[labels[i]];
    }
    free(data);
    free(labels);
    return rc;
}

/* ------------------------------------------------------------------------- */
/* writeSog (write-sog.ts:110-370)                                             */

static inline double log_transform(double v) { return js_sign(v) * st_o_log(fabs(v) + 1); }

int st_o_sog(uint64_t n, const float *const m14[14], const float *const *sh, int C, int iters,
             const double *draws, uint64_t ndraws, uint64_t *used, st_o_sog_meta *meta,
             uint8_t *means_l, uint8_t *means_u, uint8_t *quats, uint8_t *scales, uint8_t *sh0,
             uint8_t *shn_centroids, uint8_t *shn_labels)
{
    enum { X, Y, Z, S0, S1, S2, R, G, B, OP, Q0, Q1, Q2, Q3 };
    uint64_t cursor = 0, u = 0;
    int rc;
    uint32_t *indices = (uint32_t *)malloc(sizeof(uint32_t) * n);
    for (uint64_t i = 0; i < n; ++i) indices[i] = (uint32_t)i;
    st_o_morton_order(m14[X], m14[Y], m14[Z], indices, n);
    const int width = (int)(ceil(sqrt((double)n) / 4) * 4);
    const int height = (int)(ceil((double)n / width / 4) * 4);
    meta->width = width;
    meta->height = height;
    const uint64_t texels = (uint64_t)width * height * 4;
    memset(means_l, 0, texels); memset(means_u, 0, texels); memset(quats, 0, texels);
    memset(scales, 0, texels); memset(sh0, 0, texels);
    /* means */
    double mm[3][2];
    for (int a = 0; a < 3; ++a) {
        double lo = INFINITY, hi = -INFINITY;
        for (uint64_t i = 0; i < n; ++i) {
            const double v = m14[a][indices[i]];
            if (v < lo) lo = v;
            if (v > hi) hi = v;
        }
        mm[a][0] = log_transform(lo);
        mm[a][1] = log_transform(hi);
        meta->means_min[a] = mm[a][0];
        meta->means_max[a] = mm[a][1];
    }
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t r = indices[i];
        for (int a = 0; a < 3; ++a) {
            const double v = 65535 * (log_transform(m14[a][r]) - mm[a][0]) / (mm[a][1] - mm[a][0]);
            const int32_t iv = js_to_int32(v);
            means_l[i * 4 + a] = (uint8_t)(iv & 0xff);
            means_u[i * 4 + a] = (uint8_t)((iv >> 8) & 0xff);
        }
        means_l[i * 4 + 3] = 0xff;
        means_u[i * 4 + 3] = 0xff;
    }
    /* quats */
    static const int qidx[4][3] = {{1, 2, 3}, {0, 2, 3}, {0, 1, 3}, {0, 1, 2}};
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t r = indices[i];
        double q[4] = {m14[Q0][r], m14[Q1][r], m14[Q2][r], m14[Q3][r]};
        const double l = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        for (int j = 0; j < 4; ++j) q[j] = q[j] / l;
        int maxc = 0;
        for (int j = 0; j < 4; ++j)
            if (fabs(q[j]) > fabs(q[maxc])) maxc = j;
        if (q[maxc] < 0)
            for (int j = 0; j < 4; ++j) q[j] *= -1;
        const double sqrt2 = sqrt(2);
        for (int j = 0; j < 4; ++j) q[j] *= sqrt2;
        for (int k = 0; k < 3; ++k) quats[i * 4 + k] = js_to_uint8(255 * (q[qidx[maxc][k]] * 0.5 + 0.5));
        quats[i * 4 + 3] = (uint8_t)(252 + maxc);
    }
    /* scales */
    uint8_t *lab = (uint8_t *)malloc(n * 3);
    const float *scols[3] = {m14[S0], m14[S1], m14[S2]};
    rc = st_o_cluster1d(scols, 3, n, iters, draws + cursor, ndraws - cursor, &u, meta->scales_codebook, lab);
    cursor += u;
    if (rc) goto done;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t r = indices[i];
        scales[i * 4 + 0] = lab[r];
        scales[i * 4 + 1] = lab[n + r];
        scales[i * 4 + 2] = lab[2 * n + r];
        scales[i * 4 + 3] = 255;
    }
    /* colour + opacity */
    const float *ccols[3] = {m14[R], m14[G], m14[B]};
    rc = st_o_cluster1d(ccols, 3, n, iters, draws + cursor, ndraws - cursor, &u, meta->sh0_codebook, lab);
    cursor += u;
    if (rc) goto done;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t r = indices[i];
        sh0[i * 4 + 0] = lab[r];
        sh0[i * 4 + 1] = lab[n + r];
        sh0[i * 4 + 2] = lab[2 * n + r];
        sh0[i * 4 + 3] = js_to_uint8(js_max(0, js_min(255, sigmoid(m14[OP][r]) * 255)));
    }
    /* spherical harmonics */
    meta->sh_bands = C == 15 ? 3 : C == 8 ? 2 : C == 3 ? 1 : 0;
    meta->palette_size = 0;
    if (C > 0) {
        int lg = 0;
        while ((2ull << lg) <= n) ++lg; /* floor(log2(n)) */
        const int p = lg - 10;
        const int pal = (p >= 6 ? 64 * 1024 : (p >= 0 ? (1 << p) * 1024 : 1024 >> (-p)));
        meta->palette_size = pal;
        const int D = 3 * C;
        float *cent = (float *)malloc(sizeof(float) * (uint64_t)pal * D);
        uint32_t *labels = (uint32_t *)malloc(sizeof(uint32_t) * n);
        rc = st_o_kmeans(sh, D, n, pal, iters, draws + cursor, ndraws - cursor, &u, cent, labels);
        cursor += u;
        if (rc == 0) {
            uint8_t *cl = (uint8_t *)malloc((uint64_t)pal * D);
            const float **cc = (const float **)malloc(sizeof(float *) * D);
            for (int c = 0; c < D; ++c) cc[c] = cent + (uint64_t)c * pal;
            rc = st_o_cluster1d(cc, D, (uint64_t)pal, iters, draws + cursor, ndraws - cursor, &u, meta->shn_codebook, cl);
            cursor += u;
            if (rc == 0) {
                const int cw = 64 * C, chh = (pal + 63) / 64;
                meta->shn_width = cw;
                meta->shn_height = chh;
                memset(shn_centroids, 0, (uint64_t)cw * chh * 4);
                for (int i = 0; i < pal; ++i)
                    for (int j = 0; j < C; ++j) {
                        uint8_t *o = shn_centroids + ((uint64_t)i * C * 4 + j * 4);
                        o[0] = cl[(uint64_t)j * pal + i];
                        o[1] = cl[(uint64_t)(C + j) * pal + i];
                        o[2] = cl[(uint64_t)(2 * C + j) * pal + i];
                        o[3] = 0xff;
                    }
                memset(shn_labels, 0, texels);
                for (uint64_t i = 0; i < n; ++i) {
                    const uint32_t label = labels[indices[i]];
                    shn_labels[i * 4 + 0] = (uint8_t)(label & 0xff);
                    shn_labels[i * 4 + 1] = (uint8_t)((label >> 8) & 0xff);
                    shn_labels[i * 4 + 2] = 0;
                    shn_labels[i * 4 + 3] = 0xff;
                }
            }
            free(cl);
            free(cc);
        }
        free(cent);
        free(labels);
    }
done:
    *used = cursor;
    free(lab);
    free(indices);
    return rc;
}

/* ---- compressed-PLY reader (readers/decompress-ply.ts:82-232) ------------------
 * chunk: the 18 chunk columns in the order of decompress-ply.ts:14-33 (min_x .. max_b);
 * vertex: packed_position, packed_rotation, packed_scale, packed_color;
 * out: 14 columns x, y, z, f_dc_0..2, opacity, rot_0..3, scale_0..2 (decompress-ply.ts:112-128),
 * then nsh f_rest columns. */
static inline double dp_unorm(uint32_t v, int bits) {
    const uint32_t t = (1u << bits) - 1;  /* decompress-ply.ts:132-135 */
    return (double)(v & t) / (double)t;
}
static inline double dp_lerp(double a, double b, double t) { return a * (1 - t) + b * t; }

void st_o_decompress_ply(uint64_t n, const float *const chunk[18], const uint32_t *const vertex[4],
                         const uint8_t *const *sh, int nsh, float *const *out) {
    const double SH_C0 = 0.28209479177387814;
    const double norm = 1.0 / (sqrt(2) * 0.5);
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t ci = i / 256;
        const uint32_t pp = vertex[0][i], pr = vertex[1][i], ps = vertex[2][i], pc = vertex[3][i];
        /* unpack111011 (:136-140) */
        const double px = dp_unorm(pp >> 21, 11), py = dp_unorm(pp >> 11, 10), pz = dp_unorm(pp, 11);
        const double sx = dp_unorm(ps >> 21, 11), sy = dp_unorm(ps >> 11, 10), sz = dp_unorm(ps, 11);
        /* unpack8888 (:141-146) */
        const double cx = dp_unorm(pc >> 24, 8), cy = dp_unorm(pc >> 16, 8), cz = dp_unorm(pc >> 8, 8),
                     cw = dp_unorm(pc, 8);
        /* unpackRot (:147-163) */
        const double a = (dp_unorm(pr >> 20, 10) - 0.5) * norm;
        const double b = (dp_unorm(pr >> 10, 10) - 0.5) * norm;
        const double c = (dp_unorm(pr, 10) - 0.5) * norm;
        const double m = sqrt(fmax(0, 1.0 - (a * a + b * b + c * c)));
        double r[4];
        switch (pr >> 30) {
            case 0: r[0] = m; r[1] = a; r[2] = b; r[3] = c; break;
            case 1: r[0] = a; r[1] = m; r[2] = b; r[3] = c; break;
            case 2: r[0] = a; r[1] = b; r[2] = m; r[3] = c; break;
            default: r[0] = a; r[1] = b; r[2] = c; r[3] = m; break;
        }
        /* :183-216 */
        out[0][i] = (float)dp_lerp(chunk[0][ci], chunk[3][ci], px);
        out[1][i] = (float)dp_lerp(chunk[1][ci], chunk[4][ci], py);
        out[2][i] = (float)dp_lerp(chunk[2][ci], chunk[5][ci], pz);
        const double cr = dp_lerp(chunk[12][ci], chunk[15][ci], cx);
        const double cg = dp_lerp(chunk[13][ci], chunk[16][ci], cy);
        const double cb = dp_lerp(chunk[14][ci], chunk[17][ci], cz);
        out[3][i] = (float)((cr - 0.5) / SH_C0);
        out[4][i] = (float)((cg - 0.5) / SH_C0);
        out[5][i] = (float)((cb - 0.5) / SH_C0);
        out[6][i] = (float)(-st_o_log(1 / cw - 1));
        for (int k = 0; k < 4; ++k) out[7 + k][i] = (float)r[k];
        out[11][i] = (float)dp_lerp(chunk[6][ci], chunk[9][ci], sx);
        out[12][i] = (float)dp_lerp(chunk[7][ci], chunk[10][ci], sy);
        out[13][i] = (float)dp_lerp(chunk[8][ci], chunk[11][ci], sz);
    }
    /* :219-229 */
    for (int k = 0; k < nsh; ++k)
        for (uint64_t i = 0; i < n; ++i) {
            const uint8_t v = sh[k][i];
            const double t = (v == 0) ? 0 : (v == 255) ? 1 : (v + 0.5) / 256;
            out[14 + k][i] = (float)((t - 0.5) * 8);
        }
}
