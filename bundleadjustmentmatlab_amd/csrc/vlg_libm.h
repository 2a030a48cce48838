/*
 * vlg_libm.h -- sin / cos bit-identical to the host glibc (2.35, x86-64 FMA
 * variant __sin_fma / __cos_fma), for the device rotations of the GPU path.
 *
 * Why: the reference builds every Jacobian by forward differences with
 * h = 1e-10 (toolbox/bundle/mex_bundle_1_XABeUVWeAeB.c:23,39-40,52,68-69), so a
 * one-ulp difference in a rotation entry shows up at ~1e-6 in a Jacobian.  The
 * reference's rotations are VLFeat's vl_rodrigues linked against the host libm
 * (SURVEY.md App. B); the CPU oracle calls the host libm
 * sin / cos directly.  The device therefore evaluates glibc's own algorithm:
 *
 *   glibc sysdeps/ieee754/dbl-64/s_sin.c (__sin, __cos, do_sin, do_cos,
 *   reduce_sincos, do_sincos), usncs.h constants, sincostab.c table
 *   (vlg_sincostab.h, extracted by tools/gen_sincostab.py).
 *   IBM Accurate Mathematical Library, Copyright (C) 2001-2022 Free Software
 *   Foundation, Inc.; LGPL-2.1-or-later.  Restated here in a different form.
 *
 * On x86-64 with FMA + AVX2 (this image's hosts, and the GPU box's) glibc
 * dispatches to s_sin-fma.c, i.e. the same C compiled with -mfma -mavx2 and
 * GCC's default floating-point contraction.  The products GCC fused there are
 * written below as explicit fma() calls (identified by compiling the plain
 * restatement with gcc -O2 -mfma -mavx2 and reading its code), and everything
 * else is a plain IEEE operation under -ffp-contract=off.  Bit equality with
 * the host libm is checked by tests/test_device_math.py on >10^7 arguments
 * spanning every branch (and every table row), and on the device by the
 * stage-1 parity tests against the libm-linked oracle.
 *
 * Domain: |x| < 105414350 (glibc's reduce_sincos range; rotation angles are
 * far inside it); larger or non-finite arguments return NaN here (glibc uses a
 * multi-precision reduction there).
 */
#ifndef VLG_LIBM_H
#define VLG_LIBM_H

#if defined(__HIPCC__)
#define VLG_LHD __host__ __device__ static inline
#else
#define VLG_LHD static inline
#endif

#include <math.h>
#include <stdint.h>
#include <string.h>

#include "vlg_sincostab.h"

/* usncs.h / s_sin.c constants (bit patterns as in glibc 2.35) */
#define VLG_LM_S1 (-0x1.5555555555555p-3)
#define VLG_LM_S2 (0x1.1111111110ecep-7)
#define VLG_LM_S3 (-0x1.a01a019db08b8p-13)
#define VLG_LM_S4 (0x1.71de27b9a7ed9p-19)
#define VLG_LM_S5 (-0x1.addffc2fcdf59p-26)
#define VLG_LM_SN3 (-0x1.5555555555515p-3)
#define VLG_LM_SN5 (0x1.11110e829872fp-7)
#define VLG_LM_CS2 (0x1.0000000000000p-1)
#define VLG_LM_CS4 (-0x1.5555555555535p-5)
#define VLG_LM_CS6 (0x1.6c16bedd9e239p-10)
#define VLG_LM_BIG (0x1.8p+45)
#define VLG_LM_HP0 (0x1.921fb54442d18p+0)
#define VLG_LM_HP1 (0x1.1a62633145c07p-54)
#define VLG_LM_MP1 (0x1.921fb58000000p+0)
#define VLG_LM_MP2 (-0x1.dde973c000000p-27)
#define VLG_LM_PP3 (-0x1.cb3b398000000p-55)
#define VLG_LM_PP4 (-0x1.d747f23e32ed7p-83)
#define VLG_LM_HPINV (0x1.45f306dc9c883p-1)
#define VLG_LM_TOINT (0x1.8p+52)

VLG_LHD uint32_t vlg_lm_hi(double x)
{
    uint64_t u;
    memcpy(&u, &x, sizeof u);
    return (uint32_t)(u >> 32);
}

VLG_LHD uint32_t vlg_lm_lo(double x)
{
    uint64_t u;
    memcpy(&u, &x, sizeof u);
    return (uint32_t)u;
}

#ifndef VLG_LM_FMA
#define VLG_LM_FMA(a, b, c) fma((a), (b), (c))
#endif

/* TAYLOR_SIN (s_sin.c): a + ((poly(xx) a - 0.5 da) xx + da) */
VLG_LHD double vlg_lm_taylor_sin(double xx, double a, double da)
{
    double p = VLG_LM_FMA(VLG_LM_S5, xx, VLG_LM_S4);
    p = VLG_LM_FMA(p, xx, VLG_LM_S3);
    p = VLG_LM_FMA(p, xx, VLG_LM_S2);
    p = VLG_LM_FMA(p, xx, VLG_LM_S1);
    double t = VLG_LM_FMA(p, a, -0.5 * da);
    t = VLG_LM_FMA(t, xx, da);
    return a + t;
}

/* do_sin (s_sin.c) */
VLG_LHD double vlg_lm_do_sin(double x, double dx)
{
    const double xold = x;
    double u, xx, s, c, sn, ssn, cs, ccs, cor;
    int k;
    if (fabs(x) < 0.126)
        return vlg_lm_taylor_sin(x * x, x, dx);
    if (x <= 0)
        dx = -dx;
    u = VLG_LM_BIG + fabs(x);
    x = fabs(x) - (u - VLG_LM_BIG);
    xx = x * x;
    s = x + VLG_LM_FMA(x * xx, VLG_LM_FMA(xx, VLG_LM_SN5, VLG_LM_SN3), dx);
    c = VLG_LM_FMA(x, dx, xx * VLG_LM_FMA(xx, VLG_LM_FMA(xx, VLG_LM_CS6, VLG_LM_CS4), VLG_LM_CS2));
    k = (int)(vlg_lm_lo(u) << 2);
    sn = vlg_sincostab[k];
    ssn = vlg_sincostab[k + 1];
    cs = vlg_sincostab[k + 2];
    ccs = vlg_sincostab[k + 3];
    cor = VLG_LM_FMA(cs, s, VLG_LM_FMA(-sn, c, VLG_LM_FMA(s, ccs, ssn)));
    return copysign(sn + cor, xold);
}

/* do_cos (s_sin.c) */
VLG_LHD double vlg_lm_do_cos(double x, double dx)
{
    double u, xx, s, c, sn, ssn, cs, ccs, cor;
    int k;
    if (x < 0)
        dx = -dx;
    u = VLG_LM_BIG + fabs(x);
    x = fabs(x) - (u - VLG_LM_BIG) + dx;
    xx = x * x;
    s = VLG_LM_FMA(x * xx, VLG_LM_FMA(xx, VLG_LM_SN5, VLG_LM_SN3), x);
    c = xx * VLG_LM_FMA(xx, VLG_LM_FMA(xx, VLG_LM_CS6, VLG_LM_CS4), VLG_LM_CS2);
    k = (int)(vlg_lm_lo(u) << 2);
    sn = vlg_sincostab[k];
    ssn = vlg_sincostab[k + 1];
    cs = vlg_sincostab[k + 2];
    ccs = vlg_sincostab[k + 3];
    cor = VLG_LM_FMA(-sn, s, VLG_LM_FMA(-cs, c, VLG_LM_FMA(-s, ssn, ccs)));
    return cs + cor;
}

/* reduce_sincos (s_sin.c): x = n pi/2 + (a + da) */
VLG_LHD int vlg_lm_reduce(double x, double *a, double *da)
{
    const double t = VLG_LM_FMA(x, VLG_LM_HPINV, VLG_LM_TOINT);
    const double xn = t - VLG_LM_TOINT;
    const double y = VLG_LM_FMA(-xn, VLG_LM_MP2, VLG_LM_FMA(-xn, VLG_LM_MP1, x));
    const int n = (int)(vlg_lm_lo(t) & 3);
    /* t1 = xn pp3; t2 = y - t1; db = (y - t2) - t1; t1 = xn pp4; b = t2 - t1;
     * db += (t2 - b) - t1 -- every "- t1" fused with its product */
    const double t2 = VLG_LM_FMA(-xn, VLG_LM_PP3, y);
    double db = VLG_LM_FMA(-xn, VLG_LM_PP3, y - t2);
    const double b = VLG_LM_FMA(-xn, VLG_LM_PP4, t2);
    db = db + VLG_LM_FMA(-xn, VLG_LM_PP4, t2 - b);
    *a = b;
    *da = db;
    return n;
}

VLG_LHD double vlg_lm_do_sincos(double a, double da, int n)
{
    const double r = (n & 1) ? vlg_lm_do_cos(a, da) : vlg_lm_do_sin(a, da);
    return (n & 2) ? -r : r;
}

/* __sin (s_sin.c) */
VLG_LHD double vlg_lm_sin(double x)
{
    const uint32_t k = vlg_lm_hi(x) & 0x7fffffffu;
    double a, da;
    if (k < 0x3e500000u) /* |x| < 2^-26 */
        return x;
    if (k < 0x3feb6000u) /* |x| < 0.855469 */
        return vlg_lm_do_sin(x, 0);
    if (k < 0x400368fdu) { /* |x| < 2.426265 */
        const double t = VLG_LM_HP0 - fabs(x);
        return copysign(vlg_lm_do_cos(t, VLG_LM_HP1), x);
    }
    if (k < 0x419921fbu) { /* |x| < 105414350 */
        const int n = vlg_lm_reduce(x, &a, &da);
        return vlg_lm_do_sincos(a, da, n);
    }
    return x - x + NAN;
}

/* __cos (s_sin.c) */
VLG_LHD double vlg_lm_cos(double x)
{
    const uint32_t k = vlg_lm_hi(x) & 0x7fffffffu;
    double a, da;
    if (k < 0x3e400000u) /* |x| < 2^-27 */
        return 1.0;
    if (k < 0x3feb6000u)
        return vlg_lm_do_cos(x, 0);
    if (k < 0x400368fdu) {
        const double y = VLG_LM_HP0 - fabs(x);
        a = y + VLG_LM_HP1;
        da = (y - a) + VLG_LM_HP1;
        return vlg_lm_do_sin(a, da);
    }
    if (k < 0x419921fbu) {
        const int n = vlg_lm_reduce(x, &a, &da);
        return vlg_lm_do_sincos(a, da, n + 1);
    }
    return x - x + NAN;
}

#endif /* VLG_LIBM_H */
