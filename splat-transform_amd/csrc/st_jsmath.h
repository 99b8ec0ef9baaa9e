// st_jsmath.h -- JS-number (IEEE binary64) semantics on the device.
//
// The reference computes in JS numbers and stores into typed arrays, so the
// kernels reproduce: f64 arithmetic in source order (the library is built with
// -ffp-contract=off: no FMA contraction), Float32Array stores (RNE), the
// ToInt32/ToUint32/ToUint8 conversions of `<<`, `>>>` and Uint8Array stores,
// NaN-propagating Math.min/Math.max with -0 < +0, and V8's Math.exp/Math.log,
// which are fdlibm (src/base/ieee754.cc).  The fdlibm routines below follow the
// published e_exp.c / e_log.c algorithms, including V8's exp(1) === Math.E.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace st {
namespace js {

__host__ __device__ inline uint32_t hiw(double x) { return (uint32_t)(__builtin_bit_cast(uint64_t, x) >> 32); }
__host__ __device__ inline uint32_t low(double x) { return (uint32_t)__builtin_bit_cast(uint64_t, x); }
__host__ __device__ inline double mkd(uint32_t h, uint32_t l) {
    return __builtin_bit_cast(double, ((uint64_t)h << 32) | l);
}

__host__ __device__ inline bool isnan_(double v) { return v != v; }
__host__ __device__ inline bool isfinite_(double v) { return (hiw(v) & 0x7ff00000u) != 0x7ff00000u; }
__host__ __device__ inline bool isfinitef_(float v) {
    return (__builtin_bit_cast(uint32_t, v) & 0x7f800000u) != 0x7f800000u;
}
__host__ __device__ inline bool signbit_(double v) { return (hiw(v) >> 31) != 0; }

// ToInt32 (ECMA-262 7.1.6)
__host__ __device__ inline int32_t to_int32(double v) {
    if (!isfinite_(v)) return 0;
    double t = __builtin_trunc(v);
    // |t| < 2^63 is exact in int64; beyond that ToInt32 is t mod 2^32 of an even multiple -> use fmod
    if (t > -9.2e18 && t < 9.2e18) return (int32_t)(uint32_t)(uint64_t)(int64_t)t;
    double m = __builtin_fmod(t, 4294967296.0);
    if (m < 0) m += 4294967296.0;
    return (int32_t)(uint32_t)m;
}
__host__ __device__ inline uint32_t to_uint32(double v) { return (uint32_t)to_int32(v); }
__host__ __device__ inline uint8_t to_uint8(double v) { return (uint8_t)(to_uint32(v) & 0xffu); }

// Math.min / Math.max with a NaN operand return V8's NaN: the x86-64 default NaN, sign bit set
// (0xffc00000 once stored to a Float32Array; reference fixture process_chain)
__host__ __device__ inline double nan_() { return mkd(0xfff80000u, 0u); }
// V8 on x86-64: an invalid operation (Inf - Inf, 0 * Inf, 0 / 0, log of a negative) on operands
// that are not NaN yields the default NaN with the sign bit set (0xFFF8000000000000, 0xFFC00000
// once stored to a Float32Array); the GPU's default NaN is positive.  A NaN operand propagates on
// both.  r: an expression's result, nan_in: whether any of its operands was NaN.
__host__ __device__ inline double x86_nan(double r, bool nan_in) { return (r != r && !nan_in) ? nan_() : r; }
__host__ __device__ inline float x86_nanf(float r, bool nan_in) {
    return (r != r && !nan_in) ? __builtin_bit_cast(float, 0xffc00000u) : r;
}

__host__ __device__ inline double min_(double a, double b) {
    if (isnan_(a) || isnan_(b)) return nan_();
    if (a == 0 && b == 0) return signbit_(a) ? a : b;
    return a < b ? a : b;
}
__host__ __device__ inline double max_(double a, double b) {
    if (isnan_(a) || isnan_(b)) return nan_();
    if (a == 0 && b == 0) return signbit_(a) ? b : a;
    return a > b ? a : b;
}
__host__ __device__ inline double sign_(double v) {
    if (isnan_(v)) return v;
    if (v > 0) return 1;
    if (v < 0) return -1;
    return v;
}

// fdlibm e_exp.c (FreeBSD form used by V8)
__host__ __device__ inline double exp(double x) {
    const double one = 1.0, huge = 1.0e+300, o_threshold = 7.09782712893383973096e+02,
                 u_threshold = -7.45133219101941108420e+02, invln2 = 1.44269504088896338700e+00,
                 P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
                 P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                 P5 = 4.13813679705723846039e-08, twom1000 = 9.33263618503218878990e-302,
                 ln2HI0 = 6.93147180369123816490e-01, ln2LO0 = 1.90821492927058770002e-10;
    double y, hi = 0.0, lo = 0.0, c, t, twopk;
    int32_t k = 0;
    uint32_t hx = hiw(x);
    const int32_t xsb = (int32_t)((hx >> 31) & 1);
    hx &= 0x7fffffffu;
    if (hx >= 0x40862E42u) {
        if (hx >= 0x7ff00000u) {
            if (((hx & 0xfffffu) | low(x)) != 0) return x + x;
            return (xsb == 0) ? x : 0.0;
        }
        if (x > o_threshold) return huge * huge;
        if (x < u_threshold) return twom1000 * twom1000;
    }
    if (hx > 0x3fd62e42u) {
        if (hx < 0x3FF0A2B2u) {
            if (x == 1.0) return 2.718281828459045;  // V8: Math.exp(1) === Math.E
            hi = xsb ? x + ln2HI0 : x - ln2HI0;
            lo = xsb ? -ln2LO0 : ln2LO0;
            k = 1 - xsb - xsb;
        } else {
            k = (int32_t)(invln2 * x + (xsb ? -0.5 : 0.5));
            t = k;
            hi = x - t * ln2HI0;
            lo = t * ln2LO0;
        }
        x = hi - lo;
    } else if (hx < 0x3e300000u) {
        if (huge + x > one) return one + x;
    } else {
        k = 0;
    }
    t = x * x;
    if (k >= -1021)
        twopk = mkd(0x3ff00000u + ((uint32_t)k << 20), 0);
    else
        twopk = mkd(0x3ff00000u + ((uint32_t)(k + 1000) << 20), 0);
    c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    if (k == 0) return one - ((x * c) / (c - 2.0) - x);
    y = one - ((lo - (x * c) / (2.0 - c)) - hi);
    if (k >= -1021) {
        if (k == 1024) return y * 2.0 * 8.98846567431157953865e+307;
        return y * twopk;
    }
    return y * twopk * twom1000;
}

// fdlibm e_log.c (FreeBSD form used by V8)
__host__ __device__ inline double log(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                 two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
                 Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                 Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01,
                 Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
    double hfsq, f, s, z, R, w, t1, t2, dk;
    int32_t k = 0, hx = (int32_t)hiw(x), i, j;
    const uint32_t lx = low(x);
    if (hx < 0x00100000) {
        if (((hx & 0x7fffffff) | lx) == 0) return -__builtin_inf();
        if (hx < 0) return __builtin_nan("");
        k -= 54;
        x *= two54;
        hx = (int32_t)hiw(x);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    i = (hx + 0x95f64) & 0x100000;
    x = mkd((uint32_t)(hx | (i ^ 0x3ff00000)), low(x));
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

__host__ __device__ inline double sigmoid(double v) { return 1 / (1 + exp(-v)); }  // utils/math.ts:1

// write-sog.ts:33-35
__host__ __device__ inline double log_transform(double v) { return sign_(v) * log(__builtin_fabs(v) + 1); }

}  // namespace js
}  // namespace st
