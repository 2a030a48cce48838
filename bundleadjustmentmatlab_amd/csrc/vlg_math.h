/*
 * vlg_math.h -- deterministic fp64 math of the gfx950 kernels (product code;
 * the CPU oracle restates the same reference formulas independently with the
 * host libm and never includes this file).
 *
 * Why this file exists
 * --------------------
 * The reference builds every Jacobian by forward differences with h = 1e-10
 * (toolbox/bundle/mex_bundle_1_XABeUVWeAeB.c:23,39-40,52,68-69).  A one-ulp
 * difference in a projection is amplified by 1/h, so the device projection has
 * to be bit-identical to the reference arithmetic: the rotations use glibc's
 * own sin / cos algorithm (vlg_libm.h, equal to the host libm bit for bit),
 * every expression keeps the reference's evaluation order, the kernels are
 * compiled with -ffp-contract=off, and '/' and sqrt are IEEE (HIP f64 '/' and
 * sqrt are correctly rounded).
 *
 * Contents
 *   vlg_rodrigues           VLFeat vl_rodrigues (R only), SURVEY.md App. B,
 *                           called from toolbox/bundle/reproject_point.h:44
 *   vlg_calib, vlg_project  toolbox/bundle/reproject_point.h:16-57 with the
 *                           rotation supplied by the caller (so a kernel can
 *                           hoist the per-camera Rodrigues out of the
 *                           per-observation loop without changing a bit)
 *   vlg_project_proj        reproject_projective_point of
 *                           toolbox/bundle/mex_bundle_proj_1_XABeUVWeAeB.c:13-32
 *   vlg_fd_quot             (x1 - x0) / h without a division, bit-identical
 *   vlg_pinv3               3x3 pseudo-inverse of the damped point blocks
 *
 * Every expression keeps the reference's evaluation order.
 * Include from C99, C++ or HIP.
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

#include "vlg_libm.h"

/* sin / cos of the rotations: glibc's algorithm (vlg_libm.h), bit-identical to
 * the host libm that VLFeat's vl_rodrigues -- and the oracle -- call */
#define VLG_SIN vlg_lm_sin
#define VLG_COS vlg_lm_cos

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

/* the homogeneous image point Kc * (S + t) before the division */
VLG_HD void vlg_project_h(const double Kc[9], const double S[3], const double t[3], double xn[3])
{
    double Rb0 = S[0] + t[0];
    double Rb1 = S[1] + t[1];
    double Rb2 = S[2] + t[2];
    xn[0] = Kc[0] * Rb0 + Kc[3] * Rb1 + Kc[6] * Rb2;
    xn[1] = Kc[1] * Rb0 + Kc[4] * Rb1 + Kc[7] * Rb2;
    xn[2] = Kc[2] * Rb0 + Kc[5] * Rb1 + Kc[8] * Rb2;
}

VLG_HD void vlg_project_s(const double Kc[9], const double S[3], const double t[3], double x[2])
{
    double xn[3];
    vlg_project_h(Kc, S, t, xn);
    x[0] = xn[0] / xn[2];
    x[1] = xn[1] / xn[2];
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
