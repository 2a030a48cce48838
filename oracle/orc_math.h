/*
 * orc_math.h -- the oracle's own restatement of the per-observation math of
 * the reference (TEST INFRASTRUCTURE ONLY; shared by ba_oracle.c and
 * ba_cpu_mt.c, never by the product).  It does not include any product
 * header: projection, calibration override and Rodrigues are restated here
 * from the reference sources, with the host libm sin / cos / sqrt that
 * VLFeat's vl_rodrigues links against.
 *
 *   orc_rodrigues   VLFeat vl_rodrigues, R only (called at
 *                   toolbox/bundle/reproject_point.h:44), libm sin / cos
 *   orc_reproject   toolbox/bundle/reproject_point.h:16-57 (K override
 *                   :29-41, Rb :47-49, x_ = K_ Rb :50-52, dehom :55-56), every
 *                   sum left to right exactly as written there
 *   orc_reproject_proj  reproject_projective_point,
 *                   toolbox/bundle/mex_bundle_proj_1_XABeUVWeAeB.c:13-32
 *   orc_pinv3_formula   the 3x3 pseudo-inverse the GPU uses for the damped
 *                   point blocks.  The reference uses MATLAB pinv (LAPACK SVD,
 *                   bundle_euclid.m:180), whose bits are not reproducible
 *                   outside MATLAB; bundle_euclid_ref.py's default vinv="pinv"
 *                   is that SVD pinv, and this formula mode exists so that
 *                   the downstream stages can be compared bit for bit.  The
 *                   tests bound formula vs SVD pinv (tests/test_oracle.py).
 *
 * Compile with -ffp-contract=off (the x86-64 SSE2 rendering of the reference
 * C).
 */
#ifndef ORC_MATH_H
#define ORC_MATH_H

#include <math.h>
#include <string.h>

#define ORC_FD_H 1e-10 /* mex_bundle_1_XABeUVWeAeB.c:23,52 */

/* vl_rodrigues (R only): theta < 1e-6 gives exactly I (App. A Q2) */
static inline void orc_rodrigues(double R[9], const double om[3])
{
    const double small = 1e-6;
    const double th = sqrt(om[0] * om[0] + om[1] * om[1] + om[2] * om[2]);
    double x, y, z, xx, xy, xz, yy, yz, zz, sth, cth, mcth;
    if (th < small) {
        memset(R, 0, 9 * sizeof(double));
        R[0] = R[4] = R[8] = 1.0;
        return;
    }
    x = om[0] / th;
    y = om[1] / th;
    z = om[2] / th;
    xx = x * x;
    xy = x * y;
    xz = x * z;
    yy = y * y;
    yz = y * z;
    zz = z * z;
    sth = sin(th);
    cth = cos(th);
    mcth = 1.0 - cth;
    /* column major R[i + 3 j] */
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

/* reproject_point(K, a, b, num_variableK, x); K4 = [fx fy cx cy] forms the
 * 3x3 K of mex_bundle_1_XABeUVWeAeB.c:181-189 (K(1,2) = K(3,1) = K(3,2) = 0,
 * K(3,3) = 1) */
static inline void orc_reproject(const double K4[4], const double *a, const double b[3], int nvk,
                          double x[2])
{
    double K_[9], R[9], Rb[3], x_[3];
    K_[0] = K4[0];
    K_[1] = 0.0;
    K_[2] = 0.0;
    K_[3] = 0.0;
    K_[4] = K4[1];
    K_[5] = 0.0;
    K_[6] = K4[2];
    K_[7] = K4[3];
    K_[8] = 1.0;
    if (nvk == 1) {
        K_[0] = a[6];
        K_[4] = a[6];
    } else if (nvk == 4) {
        K_[0] = a[6];
        K_[4] = a[7];
        K_[6] = a[8];
        K_[7] = a[9];
    }
    orc_rodrigues(R, a);
    Rb[0] = R[0] * b[0] + R[3] * b[1] + R[6] * b[2] + a[3];
    Rb[1] = R[1] * b[0] + R[4] * b[1] + R[7] * b[2] + a[4];
    Rb[2] = R[2] * b[0] + R[5] * b[1] + R[8] * b[2] + a[5];
    x_[0] = K_[0] * Rb[0] + K_[3] * Rb[1] + K_[6] * Rb[2];
    x_[1] = K_[1] * Rb[0] + K_[4] * Rb[1] + K_[7] * Rb[2];
    x_[2] = K_[2] * Rb[0] + K_[5] * Rb[1] + K_[8] * Rb[2];
    x[0] = x_[0] / x_[2];
    x[1] = x_[1] / x_[2];
}

/* projective camera P(:) (3 x 4 column major) */
static inline void orc_reproject_proj(const double P[12], const double b[3], double x[2])
{
    double x_[3];
    x_[0] = P[0] * b[0] + P[3] * b[1] + P[6] * b[2] + P[9];
    x_[1] = P[1] * b[0] + P[4] * b[1] + P[7] * b[2] + P[10];
    x_[2] = P[2] * b[0] + P[5] * b[1] + P[8] * b[2] + P[11];
    x[0] = x_[0] / x_[2];
    x[1] = x_[1] / x_[2];
}

/* ---- 3x3 pseudo-inverse, formula mode (see the header) -------------------
 * Adjugate / determinant when |det| > 1e-12 * max|M|^3; the zero block maps to
 * zero (pinv(0) = 0, App. A Q8); otherwise a cyclic-Jacobi eigen-decomposition
 * of the symmetrised block with MATLAB's tolerance 3 * eps(max |eigenvalue|). */
static inline double orc_eps_of(double x)
{
    int e;
    if (!(x > 0.0))
        return 4.9406564584124654e-324;
    (void)frexp(x, &e);
    return ldexp(1.0, e - 53);
}

static inline void orc_pinv3_eig(const double M[9], double P[9])
{
    double A[3][3], Q[3][3], ev[3], emax = 0.0, tol;
    int p, q, k, sweep;
    for (p = 0; p < 3; p++)
        for (q = 0; q < 3; q++) {
            A[p][q] = 0.5 * (M[p + 3 * q] + M[q + 3 * p]);
            Q[p][q] = p == q ? 1.0 : 0.0;
        }
    for (sweep = 0; sweep < 32; sweep++) {
        if (A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[1][2] * A[1][2] == 0.0)
            break;
        for (p = 0; p < 2; p++)
            for (q = p + 1; q < 3; q++) {
                double th, t, c, s;
                if (A[p][q] == 0.0)
                    continue;
                th = (A[q][q] - A[p][p]) / (2.0 * A[p][q]);
                t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
                c = 1.0 / sqrt(t * t + 1.0);
                s = t * c;
                for (k = 0; k < 3; k++) { /* columns p, q of A J */
                    const double u = A[k][p], v = A[k][q];
                    A[k][p] = c * u - s * v;
                    A[k][q] = s * u + c * v;
                }
                for (k = 0; k < 3; k++) { /* rows p, q of J^T A */
                    const double u = A[p][k], v = A[q][k];
                    A[p][k] = c * u - s * v;
                    A[q][k] = s * u + c * v;
                }
                for (k = 0; k < 3; k++) { /* Q J */
                    const double u = Q[k][p], v = Q[k][q];
                    Q[k][p] = c * u - s * v;
                    Q[k][q] = s * u + c * v;
                }
            }
    }
    for (k = 0; k < 3; k++) {
        ev[k] = A[k][k];
        if (fabs(ev[k]) > emax)
            emax = fabs(ev[k]);
    }
    tol = 3.0 * orc_eps_of(emax);
    memset(P, 0, 9 * sizeof(double));
    for (k = 0; k < 3; k++) {
        double r;
        if (!(fabs(ev[k]) > tol))
            continue;
        r = 1.0 / ev[k];
        for (p = 0; p < 3; p++)
            for (q = 0; q < 3; q++)
                P[p + 3 * q] += Q[p][k] * Q[q][k] * r;
    }
}

static inline void orc_pinv3_formula(const double M[9], double P[9])
{
    /* cofactors C(r,c) of M (column major M[r + 3 c]) */
    const double c00 = M[4] * M[8] - M[7] * M[5];
    const double c01 = M[7] * M[2] - M[1] * M[8];
    const double c02 = M[1] * M[5] - M[4] * M[2];
    const double c10 = M[6] * M[5] - M[3] * M[8];
    const double c11 = M[0] * M[8] - M[6] * M[2];
    const double c12 = M[3] * M[2] - M[0] * M[5];
    const double c20 = M[3] * M[7] - M[6] * M[4];
    const double c21 = M[6] * M[1] - M[0] * M[7];
    const double c22 = M[0] * M[4] - M[3] * M[1];
    const double det = M[0] * c00 + M[3] * c01 + M[6] * c02;
    double mx = 0.0, r;
    int q;
    for (q = 0; q < 9; q++)
        if (fabs(M[q]) > mx)
            mx = fabs(M[q]);
    if (mx == 0.0) {
        memset(P, 0, 9 * sizeof(double));
        return;
    }
    if (!(fabs(det) > 1e-12 * mx * mx * mx)) {
        orc_pinv3_eig(M, P);
        return;
    }
    r = 1.0 / det;
    P[0] = c00 * r;
    P[1] = c01 * r;
    P[2] = c02 * r;
    P[3] = c10 * r;
    P[4] = c11 * r;
    P[5] = c12 * r;
    P[6] = c20 * r;
    P[7] = c21 * r;
    P[8] = c22 * r;
}

#endif /* ORC_MATH_H */
