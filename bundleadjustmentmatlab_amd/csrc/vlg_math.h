/*
 * vlg_math.h -- deterministic fp64 math shared by the gfx950 kernels and the CPU oracle.
 *
 * Why this file exists
 * --------------------
 * The reference builds every Jacobian by forward differences with h = 1e-10
 * (toolbox/bundle/mex_bundle_1_XABeUVWeAeB.c:23,39-40,52,68-69).  A one-ulp
 * difference in a projection is amplified by 1/h, so the device projection has
 * to be bit-identical to the CPU oracle.  Device OCML sin/cos and host glibc
 * sin/cos may disagree by an ulp, so both sides use the SAME sin/cos defined
 * here (fdlibm-style: Cody-Waite reduction by pi/2 plus the published minimax
 * kernels), compiled with -ffp-contract=off on both sides and IEEE division
 * and sqrt (HIP f64 '/' and sqrt are correctly rounded).
 *
 * Contents
 *   vlg_sin / vlg_cos       deterministic sin / cos (< 1 ulp, see tests)
 *   vlg_rodrigues           VLFeat vl_rodrigues (R only), SURVEY.md App. B,
 *                           called from toolbox/bundle/reproject_point.h:44
 *   vlg_project             toolbox/bundle/reproject_point.h:16-57 with the
 *                           rotation supplied by the caller (so a kernel can
 *                           hoist the per-camera Rodrigues out of the
 *                           per-observation loop without changing a bit)
 *   vlg_project_proj        reproject_projective_point of
 *                           toolbox/bundle/mex_bundle_proj_1_XABeUVWeAeB.c:13-32
 *
 * Every expression keeps the reference's evaluation order.
 * Include from C99, C++ or HIP.  Define VLG_ORACLE_LIBM to make the oracle use
 * the host libm sin/cos instead (used only to quantify the libm gap in tests).
 */
#ifndef VLG_MATH_H
#define VLG_MATH_H

#if defined(__HIPCC__)
#define VLG_HD __host__ __device__ static inline
#else
#define VLG_HD static inline
#endif

#include <stdint.h>
#include <string.h>
#include <math.h>

/* ---- bit helpers ------------------------------------------------------- */
VLG_HD uint32_t vlg_high_word(double x)
{
    uint64_t u;
    memcpy(&u, &x, sizeof u);
    return (uint32_t)(u >> 32);
}

/* ---- minimax kernels on [-pi/4, pi/4] (fdlibm k_sin.c / k_cos.c constants) */
VLG_HD double vlg_ksin(double x, double y, int iy)
{
    const double S1 = -1.66666666666666324348e-01;
    const double S2 = 8.33333333332248946124e-03;
    const double S3 = -1.98412698298579493134e-04;
    const double S4 = 2.75573137070700676789e-06;
    const double S5 = -2.50507602534068634195e-08;
    const double S6 = 1.58969099521155010221e-10;
    double z = x * x;
    double w = z * z;
    double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
    double v = z * x;
    if (iy == 0)
        return x + v * (S1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

VLG_HD double vlg_kcos(double x, double y)
{
    const double C1 = 4.16666666666666019037e-02;
    const double C2 = -1.38888888888741095749e-03;
    const double C3 = 2.48015872894767294178e-05;
    const double C4 = -2.75573143513906633035e-07;
    const double C5 = 2.08757232129817482790e-09;
    const double C6 = -1.13596475577881948265e-11;
    double z = x * x;
    double w = z * z;
    double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
    double hz = 0.5 * z;
    double t = 1.0 - hz;
    return t + (((1.0 - t) - hz) + (z * r - x * y));
}

/* Cody-Waite reduction x = n*pi/2 + (y0 + y1), three rounds (fdlibm e_rem_pio2.c
 * "medium" path).  Exact enough for |x| < 2^20*pi/2; rotation angles are tiny
 * compared with that.  Returns n. */
VLG_HD int vlg_rem_pio2(double x, double *y0, double *y1)
{
    const double invpio2 = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;
    const double pio2_1t = 6.07710050650619224932e-11;
    const double pio2_2 = 6.07710050630396597660e-11;
    const double pio2_2t = 2.02226624879595063154e-21;
    const double pio2_3 = 2.02226624871116645580e-21;
    const double pio2_3t = 8.47842766036889956997e-32;
    const double toint = 6755399441055744.0; /* 1.5 * 2^52 : round to nearest */
    double fn = (x * invpio2 + toint) - toint;
    int n = (int)fn;
    double r = x - fn * pio2_1;
    double w = fn * pio2_1t;
    int j = (int)((vlg_high_word(x) >> 20) & 0x7ff);
    double t;
    *y0 = r - w;
    if (j - (int)((vlg_high_word(*y0) >> 20) & 0x7ff) > 16) {
        t = r;
        w = fn * pio2_2;
        r = t - w;
        w = fn * pio2_2t - ((t - r) - w);
        *y0 = r - w;
        if (j - (int)((vlg_high_word(*y0) >> 20) & 0x7ff) > 49) {
            t = r;
            w = fn * pio2_3;
            r = t - w;
            w = fn * pio2_3t - ((t - r) - w);
            *y0 = r - w;
        }
    }
    *y1 = (r - *y0) - w;
    return n;
}

VLG_HD double vlg_sin(double x)
{
    double y0, y1;
    int n;
    if ((vlg_high_word(x) & 0x7fffffffu) <= 0x3fe921fbu)
        return vlg_ksin(x, 0.0, 0);
    n = vlg_rem_pio2(x, &y0, &y1);
    switch (n & 3) {
    case 0: return vlg_ksin(y0, y1, 1);
    case 1: return vlg_kcos(y0, y1);
    case 2: return -vlg_ksin(y0, y1, 1);
    default: return -vlg_kcos(y0, y1);
    }
}

VLG_HD double vlg_cos(double x)
{
    double y0, y1;
    int n;
    if ((vlg_high_word(x) & 0x7fffffffu) <= 0x3fe921fbu)
        return vlg_kcos(x, 0.0);
    n = vlg_rem_pio2(x, &y0, &y1);
    switch (n & 3) {
    case 0: return vlg_kcos(y0, y1);
    case 1: return -vlg_ksin(y0, y1, 1);
    case 2: return -vlg_kcos(y0, y1);
    default: return vlg_ksin(y0, y1, 1);
    }
}

#if defined(VLG_ORACLE_LIBM) && !defined(__HIPCC__)
#define VLG_SIN sin
#define VLG_COS cos
#else
#define VLG_SIN vlg_sin
#define VLG_COS vlg_cos
#endif

/* ---- Rodrigues: rotation vector -> R (3x3, column major R[i + 3*j]) --------
 * VLFeat vl_rodrigues (not vendored; spec recovered in SURVEY.md App. B):
 * theta < 1e-6 gives exactly I, which makes the finite-difference rotation
 * Jacobian exactly zero for cameras with |w| < ~1e-6 (App. A Q2).            */
VLG_HD void vlg_rodrigues(double R[9], const double om[3])
{
    const double small = 1e-6;
    double th = sqrt(om[0] * om[0] + om[1] * om[1] + om[2] * om[2]);
    double x, y, z, xx, xy, xz, yy, yz, zz, sth, cth, mcth;
    if (th < small) {
        R[0] = 1.0; R[3] = 0.0; R[6] = 0.0;
        R[1] = 0.0; R[4] = 1.0; R[7] = 0.0;
        R[2] = 0.0; R[5] = 0.0; R[8] = 1.0;
        return;
    }
    x = om[0] / th;
    y = om[1] / th;
    z = om[2] / th;
    xx = x * x; xy = x * y; xz = x * z;
    yy = y * y; yz = y * z; zz = z * z;
    sth = VLG_SIN(th);
    cth = VLG_COS(th);
    mcth = 1.0 - cth;
    R[0] = 1 - mcth * (yy + zz);
    R[1] = sth * z + mcth * xy;
    R[2] = -sth * y + mcth * xz;
    R[3] = -sth * z + mcth * xy;
    R[4] = 1 - mcth * (zz + xx);
    R[5] = sth * x + mcth * yz;
    R[6] = sth * y + mcth * xz;
    R[7] = -sth * x + mcth * yz;
    R[8] = 1 - mcth * (xx + yy);
}

/* ---- calibration override: reproject_point.h:29-41 ----------------------
 * Kc[9] starts as the 3x3 built from the 4-vector [fx fy cx cy]
 * (mex_bundle_1_XABeUVWeAeB.c:186-188); num_variableK 1 uses a[6] for both
 * focal lengths (App. A Q13), num_variableK 4 uses a[6..9].                 */
VLG_HD void vlg_calib(double Kc[9], const double K4[4], const double *a, int nvk)
{
    Kc[0] = K4[0]; Kc[3] = 0.0;   Kc[6] = K4[2];
    Kc[1] = 0.0;   Kc[4] = K4[1]; Kc[7] = K4[3];
    Kc[2] = 0.0;   Kc[5] = 0.0;   Kc[8] = 1.0;
    if (nvk == 1) {
        Kc[0] = a[6];
        Kc[4] = a[6];
    } else if (nvk == 4) {
        Kc[0] = a[6];
        Kc[4] = a[7];
        Kc[6] = a[8];
        Kc[7] = a[9];
    }
}

/* ---- projection: reproject_point.h:46-56, rotation given -----------------
 * x = dehom(Kc * (R*b + t)), every sum left-to-right as written there.      */
/* The same expression in two steps, so a kernel can share the rotated point
 * between projections that differ only in t: S = R*b without t (the first
 * three terms of each left-to-right row sum), then x = dehom(Kc * (S + t)).
 * vlg_project(Kc, R, t, b) == vlg_project_s(Kc, S, t) for S = vlg_rot_b(R, b)
 * bit for bit: C evaluates ((R0 b0 + R3 b1) + R6 b2) + t0 in that order. */
VLG_HD void vlg_rot_b(const double R[9], const double b[3], double S[3])
{
    S[0] = R[0] * b[0] + R[3] * b[1] + R[6] * b[2];
    S[1] = R[1] * b[0] + R[4] * b[1] + R[7] * b[2];
    S[2] = R[2] * b[0] + R[5] * b[1] + R[8] * b[2];
}

VLG_HD void vlg_project_s(const double Kc[9], const double S[3], const double t[3], double x[2])
{
    double Rb0 = S[0] + t[0];
    double Rb1 = S[1] + t[1];
    double Rb2 = S[2] + t[2];
    double x0 = Kc[0] * Rb0 + Kc[3] * Rb1 + Kc[6] * Rb2;
    double x1 = Kc[1] * Rb0 + Kc[4] * Rb1 + Kc[7] * Rb2;
    double x2 = Kc[2] * Rb0 + Kc[5] * Rb1 + Kc[8] * Rb2;
    x[0] = x0 / x2;
    x[1] = x1 / x2;
}

VLG_HD void vlg_project(const double Kc[9], const double R[9], const double t[3],
                        const double b[3], double x[2])
{
    double S[3];
    vlg_rot_b(R, b, S);
    vlg_project_s(Kc, S, t, x);
}

/* Projective camera (a = P(:), 3 x 4 column major, num_a = 12):
 * x_ = P [b; 1], x = x_(1:2) / x_(3), each row summed left to right
 * (mex_bundle_proj_1_XABeUVWeAeB.c:13-32, identical in
 * mex_bundle_proj_3_db_new.c:13-31). */
VLG_HD void vlg_project_proj(const double P[12], const double b[3], double x[2])
{
    double x0 = P[0] * b[0] + P[3] * b[1] + P[6] * b[2] + P[9];
    double x1 = P[1] * b[0] + P[4] * b[1] + P[7] * b[2] + P[10];
    double x2 = P[2] * b[0] + P[5] * b[1] + P[8] * b[2] + P[11];
    x[0] = x0 / x2;
    x[1] = x1 / x2;
}

/* Finite-difference step of the reference (mex_bundle_1_XABeUVWeAeB.c:23,52). */
#define VLG_FD_H 1e-10

/* (x1 - x0) / h of the forward differences (mex_bundle_1 :39-40, 68-69),
 * correctly rounded without a division.  Markstein's theorem (IBM J. R&D 34,
 * 1990; Cornea-Hasegan, Golliver, Markstein, ARITH-14 1999): if y is within
 * half an ulp of 1/h and q is within one ulp of d/h, the remainder
 * r = d - q h is exact (one FMA) and RN(q + r y) = RN(d/h).  Here
 * y = RN(1/h) and y h = 1 + e1 with |e1| <= 2^-54 (checked exactly in
 * tests/test_oracle.py::test_fd_quotient), so q = RN(d y) is within one ulp
 * of d/h.  Both theorems need d and q h away from the subnormal range; tiny
 * |d| (including 0, whose sign the remainder step would lose) and non-finite
 * d take the plain division.  The device uses this (3 fp64 ops instead of
 * ~10 + a quarter-rate reciprocal); the oracle keeps '/' as the reference
 * writes it, and the stage-1 parity tests compare the two bit for bit. */
#define VLG_FD_RH (1.0 / VLG_FD_H)
VLG_HD double vlg_fd_quot(double d)
{
    const double ad = fabs(d);
    if (!(ad >= 0x1p-900 && ad <= 0x1p900)) return d / VLG_FD_H;
    const double q = d * VLG_FD_RH;
    const double r = fma(-q, VLG_FD_H, d);
    return fma(r, VLG_FD_RH, q);
}

/* ---- 3x3 symmetric pseudo-inverse ------------------------------------------
 * The reference inverts every damped point block with MATLAB pinv
 * (bundle_euclid.m:180).  Here: adjugate / determinant for a well-conditioned
 * block, an all-zero block maps to zero (pinv(0) = 0, App. A Q8), and a
 * numerically singular block goes through a cyclic-Jacobi eigen pseudo-inverse
 * with MATLAB's tolerance max(size)*eps(sigma_max).  The same function runs on
 * the device and in the oracle's "device-formula" mode; the oracle's "pinv"
 * mode uses an SVD instead, and the tests bound the gap between the two.     */
VLG_HD double vlg_eps_of(double x)
{
    int e;
    if (!(x > 0.0))
        return 4.9406564584124654e-324;
    (void)frexp(x, &e); /* x = f * 2^e, f in [0.5,1) */
    return ldexp(1.0, e - 53);
}

VLG_HD void vlg_pinv3_jacobi(const double M[9], double P[9])
{
    double a[3][3], q[3][3], d[3], smax, tol;
    int i, j, k, sweep;
    for (i = 0; i < 3; i++)
        for (j = 0; j < 3; j++) {
            a[i][j] = 0.5 * (M[i + 3 * j] + M[j + 3 * i]);
            q[i][j] = (i == j) ? 1.0 : 0.0;
        }
    for (sweep = 0; sweep < 32; sweep++) {
        double off = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
        if (off == 0.0)
            break;
        for (i = 0; i < 2; i++)
            for (j = i + 1; j < 3; j++) {
                double apq = a[i][j], theta, t, c, s;
                if (apq == 0.0)
                    continue;
                theta = (a[j][j] - a[i][i]) / (2.0 * apq);
                t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                c = 1.0 / sqrt(t * t + 1.0);
                s = t * c;
                for (k = 0; k < 3; k++) { /* A <- A J */
                    double akp = a[k][i], akq = a[k][j];
                    a[k][i] = c * akp - s * akq;
                    a[k][j] = s * akp + c * akq;
                }
                for (k = 0; k < 3; k++) { /* A <- J^T A */
                    double apk = a[i][k], aqk = a[j][k];
                    a[i][k] = c * apk - s * aqk;
                    a[j][k] = s * apk + c * aqk;
                }
                for (k = 0; k < 3; k++) { /* Q <- Q J */
                    double qkp = q[k][i], qkq = q[k][j];
                    q[k][i] = c * qkp - s * qkq;
                    q[k][j] = s * qkp + c * qkq;
                }
            }
    }
    smax = 0.0;
    for (i = 0; i < 3; i++) {
        d[i] = a[i][i];
        if (fabs(d[i]) > smax)
            smax = fabs(d[i]);
    }
    tol = 3.0 * vlg_eps_of(smax);
    for (i = 0; i < 9; i++)
        P[i] = 0.0;
    for (k = 0; k < 3; k++) {
        double inv;
        if (!(fabs(d[k]) > tol))
            continue;
        inv = 1.0 / d[k];
        for (i = 0; i < 3; i++)
            for (j = 0; j < 3; j++)
                P[i + 3 * j] += q[i][k] * q[j][k] * inv;
    }
}

VLG_HD void vlg_pinv3(const double M[9], double P[9])
{
    double m00 = M[0], m10 = M[1], m20 = M[2];
    double m01 = M[3], m11 = M[4], m21 = M[5];
    double m02 = M[6], m12 = M[7], m22 = M[8];
    double c00 = m11 * m22 - m12 * m21;
    double c01 = m12 * m20 - m10 * m22;
    double c02 = m10 * m21 - m11 * m20;
    double c10 = m02 * m21 - m01 * m22;
    double c11 = m00 * m22 - m02 * m20;
    double c12 = m01 * m20 - m00 * m21;
    double c20 = m01 * m12 - m02 * m11;
    double c21 = m02 * m10 - m00 * m12;
    double c22 = m00 * m11 - m01 * m10;
    double det = m00 * c00 + m01 * c01 + m02 * c02;
    double s = 0.0, r;
    int i;
    for (i = 0; i < 9; i++)
        if (fabs(M[i]) > s)
            s = fabs(M[i]);
    if (s == 0.0) {
        for (i = 0; i < 9; i++)
            P[i] = 0.0;
        return;
    }
    if (!(fabs(det) > 1e-12 * s * s * s)) {
        vlg_pinv3_jacobi(M, P);
        return;
    }
    r = 1.0 / det;
    P[0] = c00 * r; P[3] = c10 * r; P[6] = c20 * r;
    P[1] = c01 * r; P[4] = c11 * r; P[7] = c21 * r;
    P[2] = c02 * r; P[5] = c12 * r; P[8] = c22 * r;
}

#endif /* VLG_MATH_H */
