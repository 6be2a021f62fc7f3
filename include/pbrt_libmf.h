/* pbrt_libmf.h -- the reference's float transcendentals, bit for bit.
 *
 * The reference calls the C library's float functions (sinf, cosf, powf, expf, logf, acosf,
 * atan2f, atanf, tanf).  Its goldens were produced, and the reference runs, on x86-64 glibc 2.35
 * (this image and the GPU box).  This header restates those glibc routines' algorithms --
 * operation for operation, with their tables and polynomial coefficients -- so that the GPU core
 * and the CPU oracle return exactly what the reference's libm returns:
 *
 *   sinf / cosf / sincosf   sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, s_sincosf.c, sincosf.h,
 *                           sincosf_data.c (double-precision polynomials, |x| < 120 reduced by
 *                           one multiply-subtract with pi/2, larger |x| by the 4/pi bit table)
 *   expf                    e_expf.c, e_exp2f_data.c (2^(k/32) table, cubic polynomial)
 *   logf                    e_logf.c, e_logf_data.c (16-entry 1/c, log c table, cubic)
 *   powf                    e_powf.c, e_powf_log2_data.c (log2 in double with a 16-entry table,
 *                           then the exp2f table)
 *   acosf, atan2f, atanf    e_acosf.c, e_atan2f.c, s_atanf.c (fdlibm single precision)
 *   tanf                    s_tanf.c, k_tanf.c (fdlibm single-precision kernel after sincosf.h's
 *                           double reductions)
 *
 * x86-64 glibc selects FMA builds of sinf/cosf/sincosf/expf/logf/powf at run time (IFUNC) on
 * every CPU with FMA; GCC contracts their `a * b + c` expressions into fused multiply-adds.
 * The restatement writes those contractions as explicit fma() and everything else with
 * -ffp-contract=off, which both builds (hipcc for gfx950, gcc for the oracle) use.  The
 * fdlibm float routines have no FMA build and are plain single-precision arithmetic.
 *
 * Pinned by tools/libmf_check.c against the system libm: every float input (2^32) for the
 * unary functions, and dense random and structured samples for
 * powf and atan2f (tests/test_libmf.py).  NaN results compare as NaN (x86 and the GPU produce
 * different default NaN bits; the renderer's guard zeroes NaN radiance either way).
 *
 * The table values below are the glibc sources' hexadecimal constants; tools/libmf_check.c
 * verifies each one against the data of the system libm.
 *
 * ATTRIBUTION AND LICENSE.  This file is a derivative of the GNU C Library, version 2.35, and is
 * distributed under the GNU Lesser General Public License, version 2.1 or (at your option) any
 * later version (https://www.gnu.org/licenses/old-licenses/lgpl-2.1.html), as those sources are:
 *   - sinf, cosf, sincosf, expf, logf, powf and their data tables (sysdeps/ieee754/flt-32,
 *     sincosf.h, e_exp2f_data.c, e_logf_data.c, e_powf_log2_data.c, math_config.h):
 *     Copyright (C) 2017-2022 Free Software Foundation, Inc.; contributed by ARM Ltd
 *     (Szabolcs Nagy, Wilco Dijkstra).
 *   - acosf, atanf, atan2f, tanf (e_acosf.c, s_atanf.c, e_atan2f.c, s_tanf.c, k_tanf.c): from
 *     fdlibm, Copyright (C) 1993 by Sun Microsystems, Inc.  All rights reserved.  Developed at
 *     SunPro, a Sun Microsystems, Inc. business.  Permission to use, copy, modify, and distribute
 *     this software is freely granted, provided that this notice is preserved.  Float versions by
 *     Ian Lance Taylor, Cygnus Support.
 * This library is distributed in the hope that it will be useful, but WITHOUT ANY WARRANTY;
 * without even the implied warranty of MERCHANTABILITY or FITNESS FOR A PARTICULAR PURPOSE.  See
 * the GNU Lesser General Public License for more details.  The rest of this repository is not
 * derived from glibc; the LGPL terms apply to this file and the object code compiled from it.
 */
#ifndef PBRT_LIBMF_H
#define PBRT_LIBMF_H
#include <stdint.h>

#if defined(__HIPCC__)
#define PBRT_LIBMF_FN static __device__ __forceinline__
#define PBRT_LIBMF_DATA static __constant__ const
#else
#define PBRT_LIBMF_FN static inline
#define PBRT_LIBMF_DATA static const
#endif

PBRT_LIBMF_FN uint32_t libmf_asuint(float x) { uint32_t u; __builtin_memcpy(&u, &x, 4); return u; }
PBRT_LIBMF_FN float libmf_asfloat(uint32_t u) { float x; __builtin_memcpy(&x, &u, 4); return x; }
PBRT_LIBMF_FN uint64_t libmf_asuint64(double x) { uint64_t u; __builtin_memcpy(&u, &x, 8); return u; }
PBRT_LIBMF_FN double libmf_asdouble(uint64_t u) { double x; __builtin_memcpy(&x, &u, 8); return x; }
PBRT_LIBMF_FN double libmf_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
PBRT_LIBMF_FN float libmf_fabsf(float x) { return libmf_asfloat(libmf_asuint(x) & 0x7fffffffu); }
#if defined(__HIPCC__)
PBRT_LIBMF_FN float libmf_sqrtf(float x) { return sqrtf(x); }   /* correctly rounded (the device code's sqrtf) */
#else
PBRT_LIBMF_FN float libmf_sqrtf(float x) { return __builtin_sqrtf(x); }
#endif

/* ================================================================ sinf / cosf / sincosf */
/* sincosf_data.c: sign[4], 2/pi * 2^24 (no rounding intrinsics on x86-64), pi/2, then the cosine
 * (c0..c4) and sine (s1..s3) coefficients; table 1 is table 0 with the cosine negated */
typedef struct { double sign[4], hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3; } libmf_sincos_t;
PBRT_LIBMF_DATA libmf_sincos_t libmf_sincosf_table[2] = {
    { { 1.0, -1.0, -1.0, 1.0 }, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0, -0x1.ffffffd0c621cp-2,
      0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
      0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13 },
    { { 1.0, -1.0, -1.0, 1.0 }, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0, 0x1.ffffffd0c621cp-2,
      -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
      0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13 } };
/* 4/pi in 32-bit windows at byte steps (sincosf_data.c __inv_pio4) */
PBRT_LIBMF_DATA uint32_t libmf_inv_pio4[24] = {
    0xa2u, 0xa2f9u, 0xa2f983u, 0xa2f9836eu, 0xf9836e4eu, 0x836e4e44u, 0x6e4e4415u, 0x4e441529u,
    0x441529fcu, 0x1529fc27u, 0x29fc2757u, 0xfc2757d1u, 0x2757d1f5u, 0x57d1f534u, 0xd1f534ddu, 0xf534ddc0u,
    0x34ddc0dbu, 0xddc0db62u, 0xc0db6295u, 0xdb629599u, 0x6295993cu, 0x95993c43u, 0x993c4390u, 0x3c439041u };

PBRT_LIBMF_FN uint32_t libmf_abstop12(float x) { return (libmf_asuint(x) >> 20) & 0x7ff; }

/* sincosf.h sinf_poly: n even -> sine polynomial, odd -> cosine polynomial (FMA build) */
PBRT_LIBMF_FN double libmf_sinf_poly(double x, double x2, const libmf_sincos_t *p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = libmf_fma(x2, p->s3, p->s2);
        double x7 = x3 * x2;
        double s = libmf_fma(x3, p->s1, x);
        return libmf_fma(x7, s1, s);
    }
    double x4 = x2 * x2;
    double c2 = libmf_fma(x2, p->c4, p->c3);
    double c1 = libmf_fma(x2, p->c1, p->c0);
    double x6 = x4 * x2;
    double c = libmf_fma(x4, p->c2, c1);
    return libmf_fma(x6, c2, c);
}
/* sincosf.h reduce_fast: |x| < 120, quadrant in *np, result in [-pi/4, pi/4] */
PBRT_LIBMF_FN double libmf_reduce_fast(double x, const libmf_sincos_t *p, int *np) {
    double r = x * p->hpi_inv;
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return libmf_fma(-(double)n, p->hpi, x);    /* x - n * hpi, contracted */
}
/* sincosf.h reduce_large: 4/pi to 192 bits, 32x96 -> 128-bit fixed-point product */
PBRT_LIBMF_FN double libmf_reduce_large(uint32_t xi, int *np) {
    const uint32_t *arr = &libmf_inv_pio4[(xi >> 26) & 15];
    int shift = (xi >> 23) & 7;
    uint64_t n, res0, res1, res2;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    res0 = (uint32_t)(xi * arr[0]);
    res1 = (uint64_t)xi * arr[4];
    res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    double x = (double)(int64_t)res0;
    *np = (int)n;
    return x * 0x1.921FB54442D18p-62;            /* pi63 = 2 pi 2^-64 */
}
PBRT_LIBMF_FN float libmf_sinf(float y) {
    double x = y, s;
    int n;
    const libmf_sincos_t *p = &libmf_sincosf_table[0];
    if (libmf_abstop12(y) < libmf_abstop12(0x1.921FB6p-1f)) {       /* |y| < pi/4 */
        s = x * x;
        if (libmf_abstop12(y) < libmf_abstop12(0x1p-12f)) return y;
        return (float)libmf_sinf_poly(x, s, p, 0);
    } else if (libmf_abstop12(y) < libmf_abstop12(120.0f)) {
        x = libmf_reduce_fast(x, p, &n);
        s = p->sign[n & 3];
        if (n & 2) p = &libmf_sincosf_table[1];
        return (float)libmf_sinf_poly(x * s, x * x, p, n);
    } else if (libmf_abstop12(y) < libmf_abstop12(__builtin_inff())) {
        uint32_t xi = libmf_asuint(y);
        int sign = xi >> 31;
        x = libmf_reduce_large(xi, &n);
        s = p->sign[(n + sign) & 3];
        if ((n + sign) & 2) p = &libmf_sincosf_table[1];
        return (float)libmf_sinf_poly(x * s, x * x, p, n);
    }
    return (y - y) / (y - y);
}
PBRT_LIBMF_FN float libmf_cosf(float y) {
    double x = y, s;
    int n;
    const libmf_sincos_t *p = &libmf_sincosf_table[0];
    if (libmf_abstop12(y) < libmf_abstop12(0x1.921FB6p-1f)) {
        double x2 = x * x;
        if (libmf_abstop12(y) < libmf_abstop12(0x1p-12f)) return 1.0f;
        return (float)libmf_sinf_poly(x, x2, p, 1);
    } else if (libmf_abstop12(y) < libmf_abstop12(120.0f)) {
        x = libmf_reduce_fast(x, p, &n);
        s = p->sign[n & 3];
        if (n & 2) p = &libmf_sincosf_table[1];
        return (float)libmf_sinf_poly(x * s, x * x, p, n ^ 1);
    } else if (libmf_abstop12(y) < libmf_abstop12(__builtin_inff())) {
        uint32_t xi = libmf_asuint(y);
        int sign = xi >> 31;
        x = libmf_reduce_large(xi, &n);
        s = p->sign[(n + sign) & 3];
        if ((n + sign) & 2) p = &libmf_sincosf_table[1];
        return (float)libmf_sinf_poly(x * s, x * x, p, n ^ 1);
    }
    return (y - y) / (y - y);
}
/* s_sincosf.c: the same two polynomials from one reduction (sincosf_poly evaluates each with
 * sinf_poly's operation order), so (sinf(y), cosf(y)) */
PBRT_LIBMF_FN void libmf_sincosf(float y, float *sinp, float *cosp) {
    double x = y, s;
    int n;
    const libmf_sincos_t *p = &libmf_sincosf_table[0];
    if (libmf_abstop12(y) < libmf_abstop12(0x1.921FB6p-1f)) {
        double x2 = x * x;
        if (libmf_abstop12(y) < libmf_abstop12(0x1p-12f)) { *sinp = y; *cosp = 1.0f; return; }
        *sinp = (float)libmf_sinf_poly(x, x2, p, 0);
        *cosp = (float)libmf_sinf_poly(x, x2, p, 1);
        return;
    } else if (libmf_abstop12(y) < libmf_abstop12(120.0f)) {
        x = libmf_reduce_fast(x, p, &n);
        s = p->sign[n & 3];
        if (n & 2) p = &libmf_sincosf_table[1];
    } else if (libmf_abstop12(y) < libmf_abstop12(__builtin_inff())) {
        uint32_t xi = libmf_asuint(y);
        int sign = xi >> 31;
        x = libmf_reduce_large(xi, &n);
        s = p->sign[(n + sign) & 3];
        if ((n + sign) & 2) p = &libmf_sincosf_table[1];
    } else {
        *sinp = *cosp = (y - y) / (y - y);
        return;
    }
    double xs = x * s, x2 = x * x;
    float a = (float)libmf_sinf_poly(xs, x2, p, 0), b = (float)libmf_sinf_poly(xs, x2, p, 1);
    *sinp = (n & 1) ? b : a;
    *cosp = (n & 1) ? a : b;
}

/* ================================================================ expf, and exp2 for powf */
/* e_exp2f_data.c: tab[i] = asuint64(2^(i/32)) - (i << 47) */
PBRT_LIBMF_DATA uint64_t libmf_exp2f_tab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull };
#define LIBMF_EXP2F_C0 0x1.c6af84b912394p-5
#define LIBMF_EXP2F_C1 0x1.ebfce50fac4f3p-3
#define LIBMF_EXP2F_C2 0x1.62e42ff0c52d6p-1
#define LIBMF_EXPF_INVLN2N 0x1.71547652b82fep+5               /* 32 / ln 2 */

PBRT_LIBMF_FN float libmf_expf(float x) {
    uint32_t abstop = (libmf_asuint(x) >> 20) & 0x7ff;
    double xd = (double)x;
    if (abstop >= (libmf_asuint(88.0f) >> 20)) {
        if (libmf_asuint(x) == libmf_asuint(-__builtin_inff())) return 0.0f;
        if (abstop >= (libmf_asuint(__builtin_inff()) >> 20)) return x + x;
        if (x > 0x1.62e42ep6f) return 0x1p97f * 0x1p97f;        /* __math_oflowf: +inf */
        if (x < -0x1.9fe368p6f) return 0x1p-95f * 0x1p-95f;     /* __math_uflowf: +0 */
        if (x < -0x1.9d1d9ep6f) return 0x1.4p-75f * 0x1.4p-75f; /* __math_may_uflowf */
    }
    /* z = InvLn2N * xd feeds both the shift and the remainder, so GCC fuses the product into
     * each of them (and drops z) */
    double kd = libmf_fma(LIBMF_EXPF_INVLN2N, xd, 0x1.8p+52);
    uint64_t ki = libmf_asuint64(kd);
    kd -= 0x1.8p+52;
    double r = libmf_fma(LIBMF_EXPF_INVLN2N, xd, -kd);
    uint64_t t = libmf_exp2f_tab[ki % 32];
    t += ki << 47;
    double s = libmf_asdouble(t);
    /* poly_scaled = poly / 32^3, / 32^2, / 32 (exact power-of-two scalings) */
    double zz = libmf_fma(LIBMF_EXP2F_C0 / 32768.0, r, LIBMF_EXP2F_C1 / 1024.0);
    double r2 = r * r;
    double y = libmf_fma(LIBMF_EXP2F_C2 / 32.0, r, 1.0);
    y = libmf_fma(zz, r2, y);
    y = y * s;
    return (float)y;
}

/* ================================================================ logf */
/* e_logf_data.c: {1/c, log c} per subinterval of [0x3f330000, 2 * 0x3f330000) */
PBRT_LIBMF_DATA double libmf_logf_tab[16][2] = {
    { 0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2 }, { 0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2 },
    { 0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2 },  { 0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3 },
    { 0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3 }, { 0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3 },
    { 0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4 }, { 0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4 },
    { 0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5 }, { 0x1p+0, 0x0p+0 },
    { 0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5 },  { 0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4 },
    { 0x1.b2036576afce6p-1, 0x1.526e57720db08p-3 },  { 0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3 },
    { 0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2 },  { 0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2 } };
#define LIBMF_LOGF_LN2 0x1.62e42fefa39efp-1
#define LIBMF_LOGF_A0 -0x1.00ea348b88334p-2
#define LIBMF_LOGF_A1 0x1.5575b0be00b6ap-2
#define LIBMF_LOGF_A2 -0x1.ffffef20a4123p-2

PBRT_LIBMF_FN float libmf_logf(float x) {
    uint32_t ix = libmf_asuint(x);
    if (ix == 0x3f800000) return 0;
    if (ix - 0x00800000 >= 0x7f800000 - 0x00800000) {
        if (ix * 2 == 0) return -1.0f / 0.0f;                   /* __math_divzerof(1) */
        if (ix == 0x7f800000) return x;
        if ((ix & 0x80000000) || ix * 2 >= 0xff000000) return (x - x) / (x - x);
        ix = libmf_asuint(x * 0x1p23f);                          /* subnormal: normalize */
        ix -= 23 << 23;
    }
    uint32_t tmp = ix - 0x3f330000;
    int i = (tmp >> (23 - 4)) % 16;
    int k = (int32_t)tmp >> 23;
    uint32_t iz = ix - (tmp & 0x1ffu << 23);
    double invc = libmf_logf_tab[i][0], logc = libmf_logf_tab[i][1];
    double z = (double)libmf_asfloat(iz);
    double r = libmf_fma(z, invc, -1.0);
    double y0 = libmf_fma((double)k, LIBMF_LOGF_LN2, logc);
    double r2 = r * r;
    double y = libmf_fma(LIBMF_LOGF_A1, r, LIBMF_LOGF_A2);
    y = libmf_fma(LIBMF_LOGF_A0, r2, y);
    y = libmf_fma(y, r2, y0 + r);
    return (float)y;
}

/* ================================================================ powf */
/* e_powf_log2_data.c: {1/c, log2 c}; poly approximates log1p(r) / ln 2 */
PBRT_LIBMF_DATA double libmf_powf_log2_tab[16][2] = {
    { 0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2 }, { 0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2 },
    { 0x1.49539f0f010bp+0, -0x1.7418b0a1fb77bp-2 },  { 0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2 },
    { 0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2 }, { 0x1.25e227b0b8eap+0, -0x1.97c1d1b3b7afp-3 },
    { 0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3 }, { 0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4 },
    { 0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5 }, { 0x1p+0, 0x0p+0 },
    { 0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4 },  { 0x1.ca4b31f026aap-1, 0x1.476a9543891bap-3 },
    { 0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3 },  { 0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2 },
    { 0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2 },  { 0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2 } };
#define LIBMF_POWF_A0 0x1.27616c9496e0bp-2
#define LIBMF_POWF_A1 -0x1.71969a075c67ap-2
#define LIBMF_POWF_A2 0x1.ec70a6ca7baddp-2
#define LIBMF_POWF_A3 -0x1.7154748bef6c8p-1
#define LIBMF_POWF_A4 0x1.71547652ab82bp0

PBRT_LIBMF_FN double libmf_powf_log2(uint32_t ix) {
    uint32_t tmp = ix - 0x3f330000;
    int i = (tmp >> (23 - 4)) % 16;
    uint32_t top = tmp & 0xff800000;
    uint32_t iz = ix - top;
    int k = (int32_t)top >> 23;
    double invc = libmf_powf_log2_tab[i][0], logc = libmf_powf_log2_tab[i][1];
    double z = (double)libmf_asfloat(iz);
    double r = libmf_fma(z, invc, -1.0);
    double y0 = logc + (double)k;
    double r2 = r * r;
    double y = libmf_fma(LIBMF_POWF_A0, r, LIBMF_POWF_A1);
    double p = libmf_fma(LIBMF_POWF_A2, r, LIBMF_POWF_A3);
    double r4 = r2 * r2;
    double q = libmf_fma(LIBMF_POWF_A4, r, y0);
    q = libmf_fma(p, r2, q);
    y = libmf_fma(y, r4, q);
    return y;
}
PBRT_LIBMF_FN float libmf_powf_exp2(double xd, uint32_t sign_bias) {
    double kd = xd + 0x1.8p+47;                          /* shift_scaled = 0x1.8p+52 / 32 */
    uint64_t ki = libmf_asuint64(kd);
    kd -= 0x1.8p+47;
    double r = xd - kd;
    uint64_t t = libmf_exp2f_tab[ki % 32];
    uint64_t ski = ki + sign_bias;
    t += ski << 47;
    double s = libmf_asdouble(t);
    double z = libmf_fma(LIBMF_EXP2F_C0, r, LIBMF_EXP2F_C1);
    double r2 = r * r;
    double y = libmf_fma(LIBMF_EXP2F_C2, r, 1.0);
    y = libmf_fma(z, r2, y);
    y = y * s;
    return (float)y;
}
/* 0: not an integer, 1: odd, 2: even (iy: a non-zero finite float's bits) */
PBRT_LIBMF_FN int libmf_checkint(uint32_t iy) {
    int e = iy >> 23 & 0xff;
    if (e < 0x7f) return 0;
    if (e > 0x7f + 23) return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1)) return 0;
    if (iy & (1u << (0x7f + 23 - e))) return 1;
    return 2;
}
PBRT_LIBMF_FN int libmf_zeroinfnan(uint32_t ix) { return 2 * ix - 1 >= 2u * 0x7f800000 - 1; }
PBRT_LIBMF_FN float libmf_powf(float x, float y) {
    uint32_t sign_bias = 0;
    uint32_t ix = libmf_asuint(x), iy = libmf_asuint(y);
    if (ix - 0x00800000 >= 0x7f800000 - 0x00800000 || libmf_zeroinfnan(iy)) {
        if (libmf_zeroinfnan(iy)) {
            if (2 * iy == 0) return 1.0f;                     /* (signaling NaN x: not reached) */
            if (ix == 0x3f800000) return 1.0f;
            if (2 * ix > 2u * 0x7f800000 || 2 * iy > 2u * 0x7f800000) return x + y;
            if (2 * ix == 2 * 0x3f800000) return 1.0f;
            if ((2 * ix < 2 * 0x3f800000) == !(iy & 0x80000000)) return 0.0f;
            return y * y;
        }
        if (libmf_zeroinfnan(ix)) {
            float x2 = x * x;
            if (ix & 0x80000000 && libmf_checkint(iy) == 1) x2 = -x2;
            return iy & 0x80000000 ? 1 / x2 : x2;
        }
        if (ix & 0x80000000) {
            int yint = libmf_checkint(iy);
            if (yint == 0) return (x - x) / (x - x);
            if (yint == 1) sign_bias = 1u << (5 + 11);
            ix &= 0x7fffffff;
        }
        if (ix < 0x00800000) {
            ix = libmf_asuint(x * 0x1p23f);
            ix &= 0x7fffffff;
            ix -= 23 << 23;
        }
    }
    double logx = libmf_powf_log2(ix);
    double ylogx = (double)y * logx;
    if (((libmf_asuint64(ylogx) >> 47) & 0xffff) >= (libmf_asuint64(126.0) >> 47)) {
        if (ylogx > 0x1.fffffffd1d571p+6) return (sign_bias ? -0x1p97f : 0x1p97f) * 0x1p97f;
        if (ylogx <= -150.0) return (sign_bias ? -0x1p-95f : 0x1p-95f) * 0x1p-95f;
    }
    return libmf_powf_exp2(ylogx, sign_bias);
}

/* ================================================================ atanf, atan2f (fdlibm) */
PBRT_LIBMF_DATA float libmf_atanhi[4] = { 4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f };
PBRT_LIBMF_DATA float libmf_atanlo[4] = { 5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f };
PBRT_LIBMF_DATA float libmf_aT[11] = { 3.3333334327e-01f, -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f,
                                       9.0908870101e-02f, -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f,
                                       4.9768779427e-02f, -3.6531571299e-02f, 1.6285819933e-02f };
PBRT_LIBMF_FN float libmf_atanf(float x) {
    float w, s1, s2, z;
    int32_t ix, hx, id;
    hx = (int32_t)libmf_asuint(x);
    ix = hx & 0x7fffffff;
    if (ix >= 0x4c000000) {                     /* |x| >= 2^25 */
        if (ix > 0x7f800000) return x + x;
        if (hx > 0) return libmf_atanhi[3] + libmf_atanlo[3];
        return -libmf_atanhi[3] - libmf_atanlo[3];
    }
    if (ix < 0x3ee00000) {                      /* |x| < 0.4375 */
        if (ix < 0x31000000) return x;          /* |x| < 2^-29 */
        id = -1;
    } else {
        x = libmf_fabsf(x);
        if (ix < 0x3f980000) {                  /* |x| < 1.1875 */
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
            else { id = 1; x = (x - 1.0f) / (x + 1.0f); }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
            else { id = 3; x = -1.0f / x; }
        }
    }
    z = x * x;
    w = z * z;
    s1 = z * (libmf_aT[0] + w * (libmf_aT[2] + w * (libmf_aT[4] + w * (libmf_aT[6] + w * (libmf_aT[8] + w * libmf_aT[10])))));
    s2 = w * (libmf_aT[1] + w * (libmf_aT[3] + w * (libmf_aT[5] + w * (libmf_aT[7] + w * libmf_aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    z = libmf_atanhi[id] - ((x * (s1 + s2) - libmf_atanlo[id]) - x);
    return (hx < 0) ? -z : z;
}
PBRT_LIBMF_FN float libmf_atan2f(float y, float x) {
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f,
                pi_lo = -8.7422776573e-08f;
    float z;
    int32_t k, m, hx, hy, ix, iy;
    hx = (int32_t)libmf_asuint(x);
    ix = hx & 0x7fffffff;
    hy = (int32_t)libmf_asuint(y);
    iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return libmf_atanf(y);
    m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        switch (m) {
        case 0:
        case 1: return y;
        case 2: return pi + tiny;
        default: return -pi - tiny;
        }
    }
    if (ix == 0) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
            case 0: return pi_o_4 + tiny;
            case 1: return -pi_o_4 - tiny;
            case 2: return 3.0f * pi_o_4 + tiny;
            default: return -3.0f * pi_o_4 - tiny;
            }
        } else {
            switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return pi + tiny;
            default: return -pi - tiny;
            }
        }
    }
    if (iy == 0x7f800000) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    k = (iy - ix) >> 23;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0f;
    else z = libmf_atanf(libmf_fabsf(y / x));
    switch (m) {
    case 0: return z;
    case 1: return libmf_asfloat(libmf_asuint(z) ^ 0x80000000u);
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
    }
}

/* ================================================================ acosf (fdlibm) */
PBRT_LIBMF_FN float libmf_acosf(float x) {
    const float pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f,
                pS0 = 1.6666667163e-01f, pS1 = -3.2556581497e-01f, pS2 = 2.0121252537e-01f, pS3 = -4.0055535734e-02f,
                pS4 = 7.9153501429e-04f, pS5 = 3.4793309169e-05f, qS1 = -2.4033949375e+00f, qS2 = 2.0209457874e+00f,
                qS3 = -6.8828397989e-01f, qS4 = 7.7038154006e-02f;
    float z, p, q, r, w, s, c, df;
    int32_t hx = (int32_t)libmf_asuint(x), ix = hx & 0x7fffffff;
    if (ix == 0x3f800000) {
        if (hx > 0) return 0.0f;
        return pi + 2.0f * pio2_lo;
    } else if (ix > 0x3f800000) {
        return (x - x) / (x - x);
    }
    if (ix < 0x3f000000) {                      /* |x| < 0.5 */
        if (ix <= 0x32800000) return pio2_hi + pio2_lo;
        z = x * x;
        p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        r = p / q;
        return pio2_hi - (x - (pio2_lo - x * r));
    } else if (hx < 0) {                        /* x < -0.5 */
        z = (1.0f + x) * 0.5f;
        p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        s = libmf_sqrtf(z);
        r = p / q;
        w = r * s - pio2_lo;
        return pi - 2.0f * (s + w);
    }
    z = (1.0f - x) * 0.5f;                      /* x > 0.5 */
    s = libmf_sqrtf(z);
    df = libmf_asfloat(libmf_asuint(s) & 0xfffff000u);
    c = (z - df * df) / (s + df);
    p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    r = p / q;
    w = r * s + c;
    return 2.0f * (df + w);
}

/* ================================================================ tanf (fdlibm) */
PBRT_LIBMF_DATA float libmf_tanT[13] = { 3.3333334327e-01f, 1.3333334029e-01f, 5.3968254477e-02f, 2.1869488060e-02f,
                                         8.8632395491e-03f, 3.5920790397e-03f, 1.4562094584e-03f, 5.8804126456e-04f,
                                         2.4646313977e-04f, 7.8179444245e-05f, 7.1407252108e-05f, -1.8558637748e-05f,
                                         2.5907305826e-05f };
PBRT_LIBMF_FN float libmf_kernel_tanf(float x, float y, int iy) {
    const float pio4 = 7.8539812565e-01f, pio4lo = 3.7748947079e-08f;
    const float *T = libmf_tanT;
    float z, r, v, w, s;
    int32_t ix, hx;
    hx = (int32_t)libmf_asuint(x);
    ix = hx & 0x7fffffff;
    if (ix < 0x39000000) {                      /* |x| < 2^-13 */
        if ((int)x == 0) {
            if ((ix | (iy + 1)) == 0) return 1.0f / libmf_fabsf(x);
            else if (iy == 1) return x;
            else return -1.0f / x;
        }
    }
    if (ix >= 0x3f2ca140) {                     /* |x| >= 0.6744 */
        if (hx < 0) { x = -x; y = -y; }
        z = pio4 - x;
        w = pio4lo - y;
        x = z + w;
        y = 0.0f;
        if (libmf_fabsf(x) < 0x1p-13f) return (float)(1 - ((hx >> 30) & 2)) * iy * (1.0f - 2 * iy * x);
    }
    z = x * x;
    w = z * z;
    r = T[1] + w * (T[3] + w * (T[5] + w * (T[7] + w * (T[9] + w * T[11]))));
    v = z * (T[2] + w * (T[4] + w * (T[6] + w * (T[8] + w * (T[10] + w * T[12])))));
    s = z * x;
    r = y + z * (s * (r + v) + y);
    r += T[0] * s;
    w = x + r;
    if (ix >= 0x3f2ca140) {
        v = (float)iy;
        return (float)(1 - ((hx >> 30) & 2)) * (v - 2.0f * (x - (w * w / (w + v) - r)));
    }
    if (iy == 1) return w;
    {
        float a, t;
        z = libmf_asfloat(libmf_asuint(w) & 0xfffff000u);
        v = r - (z - x);
        t = a = -1.0f / w;
        t = libmf_asfloat(libmf_asuint(t) & 0xfffff000u);
        s = 1.0f + t * z;
        return t + a * (s + t * v);
    }
}
/* s_tanf.c rem_pio2f: sincosf.h's reductions (reduce_fast without FMA: tanf has no FMA build),
 * the double remainder split into two floats */
PBRT_LIBMF_FN int libmf_rem_pio2f(float x, float *y) {
    double dx = x;
    int n;
    const libmf_sincos_t *p = &libmf_sincosf_table[0];
    if (libmf_abstop12(x) < libmf_abstop12(120.0f)) {
        double r = dx * p->hpi_inv;
        n = ((int32_t)r + 0x800000) >> 24;
        dx = dx - (double)n * p->hpi;
    } else {
        uint32_t xi = libmf_asuint(x);
        int sign = xi >> 31;
        dx = libmf_reduce_large(xi, &n);
        dx = sign ? -dx : dx;
    }
    y[0] = (float)dx;
    y[1] = (float)(dx - (double)y[0]);
    return n;
}
PBRT_LIBMF_FN float libmf_tanf(float x) {
    float y[2];
    int32_t ix = (int32_t)(libmf_asuint(x) & 0x7fffffffu);
    if (ix <= 0x3f490fda) return libmf_kernel_tanf(x, 0.0f, 1);
    if (ix >= 0x7f800000) return x - x;
    int32_t n = libmf_rem_pio2f(x, y);
    return libmf_kernel_tanf(y[0], y[1], 1 - ((n & 1) << 1));
}

#endif
