/* pbrt_fmath.h -- the transcendental functions of the parity definition.
 *
 * The reference calls glibc's float sinf/cosf/powf/acosf/atan2f/tanf/atanf.  The GPU core
 * and the CPU oracle both evaluate   f_float(x) = (float) pbrt_fm_f((double) x)   with the
 * double-precision algorithms below.  This one header is compiled into libpbrtgpu.so (HIP) and
 * oracle/liboracle.so (C), so the two agree bit for bit by construction: every step is an
 * IEEE-754 double add/sub/mul/div/sqrt in a fixed order (both builds use -ffp-contract=off),
 * plus exact bit manipulation.  Accuracy is ~1e-16 relative (pow: ~1e-16 * |y ln x|), so the
 * float result equals the correctly rounded float of the true value except when the true
 * value lies within that distance of a float rounding boundary (a few in 1e7 calls).
 *
 * Algorithms: Cody-Waite reduction by pi/2 with a three-part constant; Taylor polynomials on
 * |r| <= pi/4 (sin to r^17, cos to r^18); atan by a table of atan(k/8) and a Taylor
 * polynomial on |t| <= 1/16; log by atanh series on [sqrt(.5), sqrt(2)); exp by reduction
 * modulo ln 2 and a Taylor polynomial.  Arguments beyond |x| = 2^20 reduce less accurately
 * (deterministic either way; never reached by the renderer).
 */
#ifndef PBRT_FMATH_H
#define PBRT_FMATH_H
#include <stdint.h>

#if defined(__HIPCC__)
#define PBRT_FM_FN __host__ __device__ __forceinline__
#else
#define PBRT_FM_FN static inline
#endif

PBRT_FM_FN uint64_t pbrt_fm_bits(double x) { union { double d; uint64_t u; } v; v.d = x; return v.u; }
PBRT_FM_FN double pbrt_fm_from_bits(uint64_t u) { union { double d; uint64_t u; } v; v.u = u; return v.d; }
PBRT_FM_FN double pbrt_fm_fabs(double x) { return pbrt_fm_from_bits(pbrt_fm_bits(x) & 0x7fffffffffffffffull); }
PBRT_FM_FN int pbrt_fm_isnan(double x) { return (pbrt_fm_bits(x) & 0x7fffffffffffffffull) > 0x7ff0000000000000ull; }
PBRT_FM_FN int pbrt_fm_isinf(double x) { return (pbrt_fm_bits(x) & 0x7fffffffffffffffull) == 0x7ff0000000000000ull; }
/* round to nearest integer (ties to even) for |x| < 2^51 */
PBRT_FM_FN double pbrt_fm_rint(double x) {
    const double big = 0x1.8p52;
    return (x + big) - big;
}
/* x * 2^k for -2000 < k < 2000 (two steps keep subnormal results exact to one rounding) */
PBRT_FM_FN double pbrt_fm_ldexp(double x, int k) {
    if (k > 1000) { x *= 0x1p1000; k -= 1000; if (k > 1000) { x *= 0x1p1000; k -= 1000; } }
    else if (k < -1000) { x *= 0x1p-1000; k += 1000; if (k < -1000) { x *= 0x1p-1000; k += 1000; } }
    return x * pbrt_fm_from_bits((uint64_t)(k + 1023) << 52);
}

/* ---- sin / cos / tan ------------------------------------------------------------- */
#define PBRT_FM_PIO2_1 0x1.921fb544p+0            /* pi/2 in three parts: 33 + 33 + 53 bits */
#define PBRT_FM_PIO2_2 0x1.0b4611a6p-34
#define PBRT_FM_PIO2_3 0x1.3198a2e037073p-69
#define PBRT_FM_2OPI 0x1.45f306dc9c883p-1

/* r = x - k pi/2, returns k mod 4 */
PBRT_FM_FN int pbrt_fm_reduce(double x, double *r) {
    double k = pbrt_fm_rint(x * PBRT_FM_2OPI);
    *r = ((x - k * PBRT_FM_PIO2_1) - k * PBRT_FM_PIO2_2) - k * PBRT_FM_PIO2_3;
    int64_t ki = (int64_t)k;
    return (int)(ki & 3);
}
PBRT_FM_FN double pbrt_fm_ksin(double r) {   /* |r| <= pi/4: Taylor to r^17 */
    double z = r * r;
    double p = -1.0 / 355687428096000.0;            /* -1/17! */
    p = p * z + 1.0 / 1307674368000.0;              /*  1/15! */
    p = p * z - 1.0 / 6227020800.0;                 /* -1/13! */
    p = p * z + 1.0 / 39916800.0;                   /*  1/11! */
    p = p * z - 1.0 / 362880.0;                     /* -1/9!  */
    p = p * z + 1.0 / 5040.0;                       /*  1/7!  */
    p = p * z - 1.0 / 120.0;                        /* -1/5!  */
    p = p * z + 1.0 / 6.0;                          /*  1/3!  */
    return r - (r * z) * p;
}
PBRT_FM_FN double pbrt_fm_kcos(double r) {   /* |r| <= pi/4: Taylor to r^18 */
    double z = r * r;
    double p = -1.0 / 6402373705728000.0;           /* -1/18! */
    p = p * z + 1.0 / 20922789888000.0;             /*  1/16! */
    p = p * z - 1.0 / 87178291200.0;                /* -1/14! */
    p = p * z + 1.0 / 479001600.0;                  /*  1/12! */
    p = p * z - 1.0 / 3628800.0;                    /* -1/10! */
    p = p * z + 1.0 / 40320.0;                      /*  1/8!  */
    p = p * z - 1.0 / 720.0;                        /* -1/6!  */
    p = p * z + 1.0 / 24.0;                         /*  1/4!  */
    double hz = 0.5 * z;
    return (1.0 - hz) + (z * z) * p;
}
PBRT_FM_FN double pbrt_fm_sin(double x) {
    if (pbrt_fm_isnan(x) || pbrt_fm_isinf(x)) return x - x;
    if (pbrt_fm_fabs(x) < 0x1p-27) return x;
    double r;
    int q = pbrt_fm_reduce(x, &r);
    switch (q) {
        case 0: return pbrt_fm_ksin(r);
        case 1: return pbrt_fm_kcos(r);
        case 2: return -pbrt_fm_ksin(r);
        default: return -pbrt_fm_kcos(r);
    }
}
PBRT_FM_FN double pbrt_fm_cos(double x) {
    if (pbrt_fm_isnan(x) || pbrt_fm_isinf(x)) return x - x;
    double r;
    int q = pbrt_fm_reduce(x, &r);
    switch (q) {
        case 0: return pbrt_fm_kcos(r);
        case 1: return -pbrt_fm_ksin(r);
        case 2: return -pbrt_fm_kcos(r);
        default: return pbrt_fm_ksin(r);
    }
}
/* sin and cos of one argument: exactly pbrt_fm_sin(x) and pbrt_fm_cos(x) */
PBRT_FM_FN void pbrt_fm_sincos(double x, double *s, double *c) {
    if (pbrt_fm_isnan(x) || pbrt_fm_isinf(x)) { *s = x - x; *c = x - x; return; }
    double r;
    int q = pbrt_fm_reduce(x, &r);
    double ks = pbrt_fm_ksin(r), kc = pbrt_fm_kcos(r);
    switch (q) {
        case 0: *s = ks; *c = kc; break;
        case 1: *s = kc; *c = -ks; break;
        case 2: *s = -ks; *c = -kc; break;
        default: *s = -kc; *c = ks; break;
    }
    if (pbrt_fm_fabs(x) < 0x1p-27) *s = x;
}
PBRT_FM_FN double pbrt_fm_tan(double x) {
    if (pbrt_fm_isnan(x) || pbrt_fm_isinf(x)) return x - x;
    if (pbrt_fm_fabs(x) < 0x1p-27) return x;
    double r;
    int q = pbrt_fm_reduce(x, &r);
    double s = pbrt_fm_ksin(r), c = pbrt_fm_kcos(r);
    return (q & 1) ? -c / s : s / c;
}

/* ---- atan / atan2 / acos --------------------------------------------------------- */
PBRT_FM_FN double pbrt_fm_katan(double t) {   /* |t| <= 1/16: Taylor to t^17 */
    double z = t * t;
    double p = 1.0 / 17.0;
    p = -p * z + 1.0 / 15.0;
    p = -p * z + 1.0 / 13.0;
    p = -p * z + 1.0 / 11.0;
    p = -p * z + 1.0 / 9.0;
    p = -p * z + 1.0 / 7.0;
    p = -p * z + 1.0 / 5.0;
    p = -p * z + 1.0 / 3.0;
    return t - (t * z) * p;
}
/* atan(k/8), k = 0..8 */
#define PBRT_FM_ATAN_TAB(k) ( \
    (k) == 0 ? 0.0 : (k) == 1 ? 0x1.fd5ba9aac2f6ep-4 : (k) == 2 ? 0x1.f5b75f92c80ddp-3 : \
    (k) == 3 ? 0x1.6f61941e4def1p-2 : (k) == 4 ? 0x1.dac670561bb4fp-2 : (k) == 5 ? 0x1.1e00babdefeb4p-1 : \
    (k) == 6 ? 0x1.4978fa3269ee1p-1 : (k) == 7 ? 0x1.700a7c5784634p-1 : 0x1.921fb54442d18p-1)
#define PBRT_FM_PIO2 0x1.921fb54442d18p+0
#define PBRT_FM_PIO2_LO 0x1.1a62633145c07p-54
#define PBRT_FM_PI 0x1.921fb54442d18p+1
#define PBRT_FM_PI_LO 0x1.1a62633145c07p-53
/* atan for 0 <= a <= 1 */
PBRT_FM_FN double pbrt_fm_atan01(double a) {
    double kd = pbrt_fm_rint(a * 8.0);
    int k = (int)kd;
    double c = kd * 0.125;
    double t = (a - c) / (1.0 + a * c);
    return PBRT_FM_ATAN_TAB(k) + pbrt_fm_katan(t);
}
PBRT_FM_FN double pbrt_fm_atan(double x) {
    if (pbrt_fm_isnan(x)) return x;
    double a = pbrt_fm_fabs(x), r;
    if (a <= 1.0) r = pbrt_fm_atan01(a);
    else if (pbrt_fm_isinf(a)) r = PBRT_FM_PIO2;
    else r = (PBRT_FM_PIO2 - pbrt_fm_atan01(1.0 / a)) + PBRT_FM_PIO2_LO;
    return x < 0 ? -r : r;
}
PBRT_FM_FN double pbrt_fm_atan2(double y, double x) {
    if (pbrt_fm_isnan(x) || pbrt_fm_isnan(y)) return x + y;
    int ysgn = (pbrt_fm_bits(y) >> 63) != 0, xsgn = (pbrt_fm_bits(x) >> 63) != 0;
    double ay = pbrt_fm_fabs(y), ax = pbrt_fm_fabs(x), r;
    if (ay == 0.0) r = xsgn ? PBRT_FM_PI : 0.0;
    else if (ax == 0.0) r = PBRT_FM_PIO2;
    else if (pbrt_fm_isinf(ax) && pbrt_fm_isinf(ay)) r = xsgn ? 3.0 * (PBRT_FM_PI / 4.0) : PBRT_FM_PI / 4.0;
    else if (pbrt_fm_isinf(ax)) r = xsgn ? PBRT_FM_PI : 0.0;
    else if (pbrt_fm_isinf(ay)) r = PBRT_FM_PIO2;
    else {
        double a = ay <= ax ? pbrt_fm_atan01(ay / ax) : (PBRT_FM_PIO2 - pbrt_fm_atan01(ax / ay)) + PBRT_FM_PIO2_LO;
        r = xsgn ? (PBRT_FM_PI - a) + PBRT_FM_PI_LO : a;
    }
    return ysgn ? -r : r;
}
PBRT_FM_FN double pbrt_fm_acos(double x) {
    if (pbrt_fm_isnan(x)) return x;
    if (x > 1.0 || x < -1.0) return (x - x) / (x - x);
    double s = (1.0 - x) * (1.0 + x);
    double sq = __builtin_sqrt(s);   /* correctly rounded on both targets */
    return pbrt_fm_atan2(sq, x);
}

/* ---- pow ---------------------------------------------------------------------------- */
#define PBRT_FM_LN2_HI 0x1.62e42fefa3800p-1     /* ln 2, 43 + 53 bits */
#define PBRT_FM_LN2_LO 0x1.ef35793c76730p-45
/* ln(x) for finite x > 0 */
PBRT_FM_FN double pbrt_fm_log(double x) {
    uint64_t b = pbrt_fm_bits(x);
    int e = (int)((b >> 52) & 0x7ff);
    if (e == 0) { x *= 0x1p54; b = pbrt_fm_bits(x); e = (int)((b >> 52) & 0x7ff) - 54; }
    e -= 1023;
    double m = pbrt_fm_from_bits((b & 0x000fffffffffffffull) | 0x3ff0000000000000ull);   /* [1, 2) */
    if (m > 0x1.6a09e667f3bcdp+0) { m *= 0.5; e += 1; }                                    /* [sqrt.5, sqrt2) */
    double s = (m - 1.0) / (m + 1.0), z = s * s;
    double p = 1.0 / 23.0;
    p = p * z + 1.0 / 21.0;
    p = p * z + 1.0 / 19.0;
    p = p * z + 1.0 / 17.0;
    p = p * z + 1.0 / 15.0;
    p = p * z + 1.0 / 13.0;
    p = p * z + 1.0 / 11.0;
    p = p * z + 1.0 / 9.0;
    p = p * z + 1.0 / 7.0;
    p = p * z + 1.0 / 5.0;
    p = p * z + 1.0 / 3.0;
    double lm = 2.0 * s + (2.0 * s) * (z * p);
    double de = (double)e;
    return (de * PBRT_FM_LN2_HI + lm) + de * PBRT_FM_LN2_LO;
}
/* ln(x) for every x (NaN / negative -> NaN, 0 -> -inf, +inf -> +inf) */
PBRT_FM_FN double pbrt_fm_log_any(double x) {
    if (pbrt_fm_isnan(x) || x < 0.0) return pbrt_fm_from_bits(0x7ff8000000000000ull);
    if (x == 0.0) return pbrt_fm_from_bits(0xfff0000000000000ull);
    if (pbrt_fm_isinf(x)) return x;
    return pbrt_fm_log(x);
}
PBRT_FM_FN double pbrt_fm_exp(double z) {
    if (pbrt_fm_isnan(z)) return z;
    if (z > 709.8) return pbrt_fm_from_bits(0x7ff0000000000000ull);
    if (z < -745.2) return 0.0;
    double k = pbrt_fm_rint(z * 0x1.71547652b82fep+0);
    double r = (z - k * PBRT_FM_LN2_HI) - k * PBRT_FM_LN2_LO;   /* |r| <= ln2/2 */
    double p = 1.0 / 6227020800.0;                             /* 1/13! */
    p = p * r + 1.0 / 479001600.0;
    p = p * r + 1.0 / 39916800.0;
    p = p * r + 1.0 / 3628800.0;
    p = p * r + 1.0 / 362880.0;
    p = p * r + 1.0 / 40320.0;
    p = p * r + 1.0 / 5040.0;
    p = p * r + 1.0 / 720.0;
    p = p * r + 1.0 / 120.0;
    p = p * r + 1.0 / 24.0;
    p = p * r + 1.0 / 6.0;
    p = p * r + 0.5;
    double er = 1.0 + (r + (r * r) * p);
    return pbrt_fm_ldexp(er, (int)k);
}
PBRT_FM_FN double pbrt_fm_pow(double x, double y) {
    if (y == 0.0 || x == 1.0) return 1.0;
    if (pbrt_fm_isnan(x) || pbrt_fm_isnan(y)) return x + y;
    double ax = pbrt_fm_fabs(x);
    int neg = 0;
    if (x < 0.0) {
        double yi = pbrt_fm_rint(y);
        if (yi != y && !pbrt_fm_isinf(y)) return (x - x) / (x - x);
        neg = !pbrt_fm_isinf(y) && pbrt_fm_fabs(y) < 0x1p53 && (((int64_t)yi) & 1);
    }
    double r;
    if (ax == 0.0) r = y > 0.0 ? 0.0 : pbrt_fm_from_bits(0x7ff0000000000000ull);
    else if (pbrt_fm_isinf(y)) r = (ax < 1.0) == (y > 0.0) ? 0.0 : pbrt_fm_from_bits(0x7ff0000000000000ull);
    else if (pbrt_fm_isinf(ax)) r = y > 0.0 ? ax : 0.0;
    else r = pbrt_fm_exp(y * pbrt_fm_log(ax));
    return neg ? -r : r;
}

#endif /* PBRT_FMATH_H */
