/*
 * ba_oracle.c -- CPU restatement of the reference's LM stages: Euclidean
 * (toolbox/bundle/mex_bundle_{1,2,3}*.c, num_a = 6 / 7 / 10) and projective
 * (mex_bundle_proj_{1,2,3}*.c, num_a = 12: same loops, camera P(:) instead of
 * [w; T; (K)]; mex_bundle_proj_2_Se_.c differs from mex_bundle_2_Se_.c only
 * in fixing num_a = 12, and mex_bundle_proj_3_db_new.c keeps the 6-term
 * back substitution of App. A Q3).
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in bundleadjustmentmatlab_amd/ links,
 * loads or calls this library; only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may use it, and only as the checker / baseline.
 *
 * PARITY STATUS: "parity unpinned".  The reference stages are MATLAB MEX
 * files (toolbox/bundle/mex_bundle_{1,2,3}*.c) that include MATLAB's mex API
 * through VLFeat's <mexutils.h> and VLFeat's "vl/rodrigues.h"; neither
 * library is in the image, so the reference C is unbuildable here, and the
 * reference's own tests hold no golden vectors.  This file
 * restates each stage from the reference source (file:line cited per
 * function); tests/ cross-check it against an independent numpy restatement
 * of bundle_euclid_nomex.m, an analytic Jacobian and scipy's rotation.
 *
 * Two storage forms:
 *  - dense  (oracle_mex1/2/3): exactly the MEX argument layouts, column major,
 *    every (point i, camera j) pair visited (SURVEY.md sec. 8.b "Argument
 *    layouts").  Feasible for configs 1-2.
 *  - sparse (oracle_sp_*): a point-major observation list (points ascending,
 *    each point's observations with cameras ascending) with the same
 *    per-element arithmetic and the same ascending summation order, so every
 *    output equals the dense form (exact zeros added by the dense loops for
 *    invisible pairs do not change a sum).
 *
 * Compiled with -O2 -ffp-contract=off (no FMA contraction; App. A Q15).
 */
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include "orc_math.h"

#define ORC_MAX_NUM_A 12
#define ORC_PROJ_NUM_A 12  /* num_a of the projective model (bundle_projective.m:70) */

/* reproject_point.h:16-57 (calibration override + Rodrigues + projection). */
void oracle_reproject(const double K4[4], const double *a, const double b[3],
                      int nvk, double x[2])
{
    orc_reproject(K4, a, b, nvk, x);
}

/* reproject_projective_point, mex_bundle_proj_1_XABeUVWeAeB.c:13-32 */
void oracle_reproject_proj(const double *a, const double b[3], double x[2])
{
    orc_reproject_proj(a, b, x);
}

/* The camera model follows num_a: 12 is the projective camera P(:) of
 * bundle_projective.m:70-73 (K4 unused, may be NULL); 6 / 7 / 10 the
 * Euclidean [w; T; (K)] of bundle_euclid.m:88-96. */
static void orc_project(const double *K4, const double *a, const double b[3], int num_a,
                        double x[2])
{
    if (num_a == ORC_PROJ_NUM_A)
        orc_reproject_proj(a, b, x);
    else
        orc_reproject(K4, a, b, num_a - 6, x);
}

static const double *orc_k4(const double *K4, int j)
{
    return K4 ? K4 + 4 * (size_t)j : NULL;
}

void oracle_rodrigues(const double om[3], double R[9]) { orc_rodrigues(R, om); }
/* the host libm sin / cos the oracle's rotations use (vl_rodrigues links libm) */
void oracle_libm_sincos(const double *x, double *s, double *c, long long n)
{
    long long k;
    for (k = 0; k < n; k++) {
        s[k] = sin(x[k]);
        c[k] = cos(x[k]);
    }
}
void oracle_pinv3(const double M[9], double P[9]) { orc_pinv3_formula(M, P); }

/* Camera-parameter derivative, forward difference:
 * mex_bundle_1_XABeUVWeAeB.c:14-41 (a1 = a0 + h*e_k for every component,
 * divide by h); projective: mex_bundle_proj_1_XABeUVWeAeB.c:34-59. */
static void orc_dcam(const double K4[4], const double *a0, const double b[3], int num_a,
                     int k, const double x0[2], double out[2])
{
    double a1[ORC_MAX_NUM_A], x1[2];
    const double h = ORC_FD_H;
    int c;
    for (c = 0; c < num_a; c++)
        a1[c] = a0[c] + h * (c == k ? 1.0 : 0.0);
    orc_project(K4, a1, b, num_a, x1);
    out[0] = (x1[0] - x0[0]) / h;
    out[1] = (x1[1] - x0[1]) / h;
}

/* Point derivative: mex_bundle_1_XABeUVWeAeB.c:43-70
 * (mex_bundle_proj_1_XABeUVWeAeB.c:61-86). */
static void orc_dpt(const double K4[4], const double *a, const double b0[3], int num_a,
                    int k, const double x0[2], double out[2])
{
    double b1[3], x1[2];
    const double h = ORC_FD_H;
    int c;
    for (c = 0; c < 3; c++)
        b1[c] = b0[c] + h * (c == k ? 1.0 : 0.0);
    orc_project(K4, a, b1, num_a, x1);
    out[0] = (x1[0] - x0[0]) / h;
    out[1] = (x1[1] - x0[1]) / h;
}

/* One visible observation: X_hat, A (2 x num_a col-major), B (2x3), e.
 * mex_bundle_1_XABeUVWeAeB.c:196-225. */
static void orc_linearize_obs(const double K4[4], const double *a, const double *b,
                              const double X[2], int num_a, double xh[2],
                              double *A, double *B, double e[2])
{
    int k;
    orc_project(K4, a, b, num_a, xh);
    for (k = 0; k < num_a; k++)
        orc_dcam(K4, a, b, num_a, k, xh, A + 2 * k);
    for (k = 0; k < 3; k++)
        orc_dpt(K4, a, b, num_a, k, xh, B + 2 * k);
    e[0] = X[0] - xh[0];
    e[1] = X[1] - xh[1];
}

/* Block products of one observation accumulated in place, each entry as the
 * reference writes it: acc += (p0r*p0c + p1r*p1c)
 * (mex_bundle_1_XABeUVWeAeB.c:280-332). */
static void orc_accum_obs(const double *A, const double *B, const double *e, int num_a,
                          double *U, double *V, double *W, double *eA, double *eB)
{
    int r, c;
    for (c = 0; c < num_a; c++)
        for (r = 0; r < num_a; r++)
            U[r + num_a * c] += A[2 * r] * A[2 * c] + A[2 * r + 1] * A[2 * c + 1];
    for (c = 0; c < 3; c++)
        for (r = 0; r < 3; r++)
            V[r + 3 * c] += B[2 * r] * B[2 * c] + B[2 * r + 1] * B[2 * c + 1];
    for (c = 0; c < 3; c++)
        for (r = 0; r < num_a; r++)
            W[r + num_a * c] += A[2 * r] * B[2 * c] + A[2 * r + 1] * B[2 * c + 1];
    for (r = 0; r < num_a; r++)
        eA[r] += A[2 * r] * e[0] + A[2 * r + 1] * e[1];
    for (r = 0; r < 3; r++)
        eB[r] += B[2 * r] * e[0] + B[2 * r + 1] * e[1];
}

/* ===================================================================== *
 *  Dense forms (MEX layouts)                                            *
 * ===================================================================== */

/* mex_bundle_1_XABeUVWeAeB (mex_bundle_1_XABeUVWeAeB.c:72-337).
 * Inputs K 4xm, a num_a x m, b 3xn, X 2xnxm, vis nxm.  All outputs are
 * written in full (they are zeroed first, like mxCreate*). */
void oracle_mex1(int m, int n, int num_a, const double *K4, const double *a,
                 const double *b, const double *X, const double *vis,
                 double *X_hat, double *A, double *B, double *e, double *U,
                 double *V, double *W, double *eA, double *eB)
{
    size_t nm = (size_t)n * m, p;
    int i, j;
    memset(U, 0, sizeof(double) * num_a * num_a * m);
    memset(V, 0, sizeof(double) * 9 * n);
    memset(W, 0, sizeof(double) * num_a * 3 * nm);
    memset(eA, 0, sizeof(double) * num_a * m);
    memset(eB, 0, sizeof(double) * 3 * n);
    /* pass 1: projections / Jacobians / residuals, j outer, i inner (:192-256) */
    for (j = 0; j < m; j++)
        for (i = 0; i < n; i++) {
            p = (size_t)i + (size_t)n * j;
            if (vis[p] != 0.0) {
                orc_linearize_obs(orc_k4(K4, j), a + (size_t)num_a * j, b + 3 * (size_t)i,
                                  X + 2 * p, num_a, X_hat + 2 * p, A + 2 * num_a * p,
                                  B + 6 * p, e + 2 * p);
            } else {
                X_hat[2 * p] = X[2 * p];
                X_hat[2 * p + 1] = X[2 * p + 1];
                memset(A + 2 * num_a * p, 0, sizeof(double) * 2 * num_a);
                memset(B + 6 * p, 0, sizeof(double) * 6);
                e[2 * p] = 0.0;
                e[2 * p + 1] = 0.0;
            }
        }
    /* pass 2: U, V, W, eA, eB over every pair (:266-334) */
    for (j = 0; j < m; j++)
        for (i = 0; i < n; i++) {
            p = (size_t)i + (size_t)n * j;
            orc_accum_obs(A + 2 * num_a * p, B + 6 * p, e + 2 * p, num_a,
                          U + (size_t)num_a * num_a * j, V + 9 * (size_t)i,
                          W + (size_t)num_a * 3 * p, eA + (size_t)num_a * j,
                          eB + 3 * (size_t)i);
        }
}

/* mex_bundle_2_Se_ (mex_bundle_2_Se_.c:15-158).
 * S (num_a*m)^2 column major: S_jk = delta_jk U*_j - sum_i Y_ij W_ik^T,
 * e_j = eA_j - sum_i Y_ij eB_i.  Dense O(m^2 n) loop, i ascending. */
void oracle_mex2(int m, int n, int num_a, const double *Y, const double *W,
                 const double *Us, const double *eA, const double *eB, double *S,
                 double *e_)
{
    size_t ld = (size_t)num_a * m;
    double blk[ORC_MAX_NUM_A * ORC_MAX_NUM_A], acc[ORC_MAX_NUM_A];
    int i, j, k, r, c;
    for (k = 0; k < m; k++)
        for (j = 0; j < m; j++) {
            for (c = 0; c < num_a; c++)
                for (r = 0; r < num_a; r++)
                    blk[r + num_a * c] =
                        (j == k) ? Us[r + num_a * c + (size_t)num_a * num_a * j] : 0.0;
            for (i = 0; i < n; i++) {
                const double *y = Y + (size_t)num_a * 3 * ((size_t)i + (size_t)n * j);
                const double *w = W + (size_t)num_a * 3 * ((size_t)i + (size_t)n * k);
                for (c = 0; c < num_a; c++)
                    for (r = 0; r < num_a; r++)
                        blk[r + num_a * c] -= y[r] * w[c] + y[r + num_a] * w[c + num_a] +
                                              y[r + 2 * num_a] * w[c + 2 * num_a];
            }
            for (c = 0; c < num_a; c++)
                for (r = 0; r < num_a; r++)
                    S[(size_t)num_a * j + r + ld * ((size_t)num_a * k + c)] = blk[r + num_a * c];
        }
    for (j = 0; j < m; j++) {
        for (r = 0; r < num_a; r++)
            acc[r] = 0.0;
        for (i = 0; i < n; i++) {
            const double *y = Y + (size_t)num_a * 3 * ((size_t)i + (size_t)n * j);
            const double *eb = eB + 3 * (size_t)i;
            for (r = 0; r < num_a; r++)
                acc[r] += y[r] * eb[0] + y[r + num_a] * eb[1] + y[r + 2 * num_a] * eb[2];
        }
        for (r = 0; r < num_a; r++)
            e_[(size_t)num_a * j + r] = eA[(size_t)num_a * j + r] - acc[r];
    }
}

/* mex_bundle_3_db_new (mex_bundle_3_db_new.c:20-170).  Back substitution
 * (:99-134, sum :113-120) uses only the first SIX camera components of da
 * (App. A Q3); a_new :137-140, b_new :143-146, X_hat :149-166. */
void oracle_mex3(int m, int n, int num_a, const double *W, const double *da,
                 const double *eB, const double *Vinv, const double *K4, const double *a,
                 const double *b, const double *X, const double *vis, double *db,
                 double *a_new, double *b_new, double *X_hat)
{
    int i, j, r, k;
    size_t p;
    for (i = 0; i < n; i++) {
        double rhs[3];
        for (r = 0; r < 3; r++)
            rhs[r] = eB[3 * (size_t)i + r];
        for (j = 0; j < m; j++) {
            const double *w = W + (size_t)num_a * 3 * ((size_t)i + (size_t)n * j);
            const double *d = da + (size_t)num_a * j;
            for (r = 0; r < 3; r++) {
                const double *wr = w + num_a * r;
                rhs[r] -= wr[0] * d[0] + wr[1] * d[1] + wr[2] * d[2] + wr[3] * d[3] +
                          wr[4] * d[4] + wr[5] * d[5];
            }
        }
        for (r = 0; r < 3; r++) {
            const double *vi = Vinv + 9 * (size_t)i;
            db[3 * (size_t)i + r] = vi[r] * rhs[0] + vi[r + 3] * rhs[1] + vi[r + 6] * rhs[2];
        }
    }
    for (k = 0; k < num_a * m; k++)
        a_new[k] = a[k] + da[k];
    for (k = 0; k < 3 * n; k++)
        b_new[k] = b[k] + db[k];
    for (j = 0; j < m; j++)
        for (i = 0; i < n; i++) {
            p = (size_t)i + (size_t)n * j;
            if (vis[p] != 0.0) {
                orc_project(orc_k4(K4, j), a_new + (size_t)num_a * j, b_new + 3 * (size_t)i,
                            num_a, X_hat + 2 * p);
            } else {
                X_hat[2 * p] = X[2 * p];
                X_hat[2 * p + 1] = X[2 * p + 1];
            }
        }
}

/* ===================================================================== *
 *  Sparse forms (point-major observation list)                          *
 *                                                                       *
 *  pt_ptr[n+1]   : observations of point i are pt_ptr[i] .. pt_ptr[i+1]-1 *
 *  obs_cam[N]    : camera of each observation (ascending within a point) *
 *  obs_x[2N]     : measured (u,v) of each observation                    *
 *  per-observation blocks: A [N][2*num_a], B [N][6], e [N][2],          *
 *  W, Y [N][num_a*3] (num_a x 3, column major, as the MEX W_ij / Y_ij)  *
 * ===================================================================== */

/* mex_1 on the observation list.  U_j receives its terms in ascending point
 * order and V_i / eB_i in ascending camera order, as in the dense loops. */
void oracle_sp_linearize(int m, int n, int num_a, const int *pt_ptr, const int *obs_cam,
                         const double *obs_x, const double *K4, const double *a,
                         const double *b, double *obs_xhat, double *A, double *B,
                         double *e, double *U, double *V, double *W, double *eA,
                         double *eB)
{
    int i, o;
    memset(U, 0, sizeof(double) * num_a * num_a * m);
    memset(V, 0, sizeof(double) * 9 * n);
    memset(eA, 0, sizeof(double) * num_a * m);
    memset(eB, 0, sizeof(double) * 3 * n);
    for (i = 0; i < n; i++)
        for (o = pt_ptr[i]; o < pt_ptr[i + 1]; o++) {
            int j = obs_cam[o];
            double *w = W + (size_t)num_a * 3 * o;
            memset(w, 0, sizeof(double) * num_a * 3);
            orc_linearize_obs(orc_k4(K4, j), a + (size_t)num_a * j, b + 3 * (size_t)i,
                              obs_x + 2 * (size_t)o, num_a, obs_xhat + 2 * (size_t)o,
                              A + 2 * (size_t)num_a * o, B + 6 * (size_t)o, e + 2 * (size_t)o);
            orc_accum_obs(A + 2 * (size_t)num_a * o, B + 6 * (size_t)o, e + 2 * (size_t)o,
                          num_a, U + (size_t)num_a * num_a * j, V + 9 * (size_t)i, w,
                          eA + (size_t)num_a * j, eB + 3 * (size_t)i);
        }
}

/* Y_o = W_o * Vinv_i (bundle_euclid.m:182), each entry summed left to right. */
void oracle_sp_y(int n, int num_a, const int *pt_ptr, const double *W, const double *Vinv,
                 double *Y)
{
    int i, o, r, c;
    for (i = 0; i < n; i++) {
        const double *vi = Vinv + 9 * (size_t)i;
        for (o = pt_ptr[i]; o < pt_ptr[i + 1]; o++) {
            const double *w = W + (size_t)num_a * 3 * o;
            double *y = Y + (size_t)num_a * 3 * o;
            for (c = 0; c < 3; c++)
                for (r = 0; r < num_a; r++)
                    y[r + num_a * c] = w[r] * vi[3 * c] + w[r + num_a] * vi[1 + 3 * c] +
                                       w[r + 2 * num_a] * vi[2 + 3 * c];
        }
    }
}

/* Damped per-point blocks and their pseudo-inverse with the device formula
 * (bundle_euclid.m:168-180 with the formula pinv of orc_math.h in place of MATLAB pinv). */
void oracle_sp_vinv(int n, double lambda, const double *V, double *Vinv)
{
    int i, k;
    double vs[9];
    for (i = 0; i < n; i++) {
        memcpy(vs, V + 9 * (size_t)i, sizeof vs);
        for (k = 0; k < 3; k++)
            vs[4 * k] = (1 + lambda) * V[9 * (size_t)i + 4 * k];
        orc_pinv3_formula(vs, Vinv + 9 * (size_t)i);
    }
}

/* mex_2 on the observation list.  Both triangles are computed, like
 * mex_bundle_2_Se_.c:72-129; each S_jk entry receives its terms in
 * ascending point order. */
void oracle_sp_schur(int m, int n, int num_a, const int *pt_ptr, const int *obs_cam,
                     const double *Y, const double *W, const double *Us, const double *eA,
                     const double *eB, double *S, double *e_)
{
    size_t ld = (size_t)num_a * m;
    int i, j, oa, ob, r, c;
    double *acc = (double *)calloc(ld, sizeof(double));
    memset(S, 0, sizeof(double) * ld * ld);
    for (j = 0; j < m; j++)
        for (c = 0; c < num_a; c++)
            for (r = 0; r < num_a; r++)
                S[(size_t)num_a * j + r + ld * ((size_t)num_a * j + c)] =
                    Us[r + num_a * c + (size_t)num_a * num_a * j];
    for (i = 0; i < n; i++)
        for (oa = pt_ptr[i]; oa < pt_ptr[i + 1]; oa++) {
            const double *y = Y + (size_t)num_a * 3 * oa;
            const double *eb = eB + 3 * (size_t)i;
            size_t rj = (size_t)num_a * obs_cam[oa];
            for (ob = pt_ptr[i]; ob < pt_ptr[i + 1]; ob++) {
                const double *w = W + (size_t)num_a * 3 * ob;
                size_t ck = (size_t)num_a * obs_cam[ob];
                for (c = 0; c < num_a; c++)
                    for (r = 0; r < num_a; r++)
                        S[rj + r + ld * (ck + c)] -= y[r] * w[c] + y[r + num_a] * w[c + num_a] +
                                                    y[r + 2 * num_a] * w[c + 2 * num_a];
            }
            for (r = 0; r < num_a; r++)
                acc[rj + r] += y[r] * eb[0] + y[r + num_a] * eb[1] + y[r + 2 * num_a] * eb[2];
        }
    for (j = 0; j < (int)ld; j++)
        e_[j] = eA[j] - acc[j];
    free(acc);
}

/* mex_3 on the observation list: db, a_new, b_new and the new projections of
 * the (visible) observations.  Returns sum of squared new residuals. */
/* ndb: camera parameters used in the back substitution -- 6 as
 * mex_bundle_3_db_new.c:113-120 (App. A Q3), or num_a for the pure-MATLAB twin
 * bundle_euclid_nomex.m:268-277 (W(:,:,i,j)' * da(k:k+num_a-1), summed here
 * left to right after the first six terms). */
double oracle_sp_update_nd(int m, int n, int num_a, int ndb, const int *pt_ptr,
                           const int *obs_cam, const double *obs_x, const double *W,
                           const double *da, const double *eB, const double *Vinv,
                           const double *K4, const double *a, const double *b, double *db,
                           double *a_new, double *b_new, double *obs_xhat)
{
    int i, o, r, k;
    double sse = 0.0;
    for (i = 0; i < n; i++) {
        double rhs[3];
        const double *vi = Vinv + 9 * (size_t)i;
        for (r = 0; r < 3; r++)
            rhs[r] = eB[3 * (size_t)i + r];
        for (o = pt_ptr[i]; o < pt_ptr[i + 1]; o++) {
            const double *w = W + (size_t)num_a * 3 * o;
            const double *d = da + (size_t)num_a * obs_cam[o];
            for (r = 0; r < 3; r++) {
                const double *wr = w + num_a * r;
                double t = wr[0] * d[0] + wr[1] * d[1] + wr[2] * d[2] + wr[3] * d[3] +
                           wr[4] * d[4] + wr[5] * d[5];
                for (k = 6; k < ndb; k++)
                    t = t + wr[k] * d[k];
                rhs[r] -= t;
            }
        }
        for (r = 0; r < 3; r++)
            db[3 * (size_t)i + r] = vi[r] * rhs[0] + vi[r + 3] * rhs[1] + vi[r + 6] * rhs[2];
    }
    for (k = 0; k < num_a * m; k++)
        a_new[k] = a[k] + da[k];
    for (k = 0; k < 3 * n; k++)
        b_new[k] = b[k] + db[k];
    for (i = 0; i < n; i++)
        for (o = pt_ptr[i]; o < pt_ptr[i + 1]; o++) {
            int j = obs_cam[o];
            double *xh = obs_xhat + 2 * (size_t)o, d0, d1;
            orc_project(orc_k4(K4, j), a_new + (size_t)num_a * j, b_new + 3 * (size_t)i,
                        num_a, xh);
            d0 = obs_x[2 * (size_t)o] - xh[0];
            d1 = obs_x[2 * (size_t)o + 1] - xh[1];
            sse += d0 * d0 + d1 * d1;
        }
    return sse;
}

/* mex_bundle_3_db_new.c:99-166 on the observation list (6-term db, App. A Q3) */
double oracle_sp_update(int m, int n, int num_a, const int *pt_ptr, const int *obs_cam,
                        const double *obs_x, const double *W, const double *da,
                        const double *eB, const double *Vinv, const double *K4,
                        const double *a, const double *b, double *db, double *a_new,
                        double *b_new, double *obs_xhat)
{
    return oracle_sp_update_nd(m, n, num_a, 6, pt_ptr, obs_cam, obs_x, W, da, eB, Vinv, K4, a,
                               b, db, a_new, b_new, obs_xhat);
}

/* ===================================================================== *
 *  Parity-mode pieces (the GPU's vlgba_options.ordered = 2)             *
 * ===================================================================== */

/* sum_k x[k] * y[k], sequentially in index order (a naive dot: the order of
 * MATLAB's e_stack' * e_stack, bundle_euclid.m:207-210, is BLAS's and not
 * reproducible; this fixes one) */
double oracle_seq_dot(const double *x, const double *y, long long n)
{
    long long k;
    double s = 0.0;
    for (k = 0; k < n; k++)
        s = s + x[k] * y[k];
    return s;
}

/* sum_k dp[k] * (lambda * dp[k] + g[k]) sequentially (bundle_euclid.m:217) */
double oracle_seq_dpg(const double *dp, const double *g, double lambda, long long n)
{
    long long k;
    double s = 0.0;
    for (k = 0; k < n; k++)
        s = s + dp[k] * (lambda * dp[k] + g[k]);
    return s;
}

/* da = S \ e_ by a left-looking Cholesky of the lower triangle of S (column
 * major, ld x ld, overwritten by L), every sum in ascending index order, and
 * the two triangular solves.  Rows whose diagonal is exactly zero (fixed
 * parameters, App. A Q2/Q8) get a unit diagonal and a zero right-hand side:
 * pinv(S) e_ is zero there.  Returns 0, or j + 1 for a non-positive pivot at
 * column j (the caller then uses pinv, as bundle_euclid.m:193 always does). */
int oracle_chol_seq(int n, double *S, const double *e_, double *da)
{
    const size_t ld = (size_t)n;
    int i, j, k;
    for (j = 0; j < n; j++)
        da[j] = e_[j];
    for (j = 0; j < n; j++)
        if (S[j + ld * j] == 0.0) {
            S[j + ld * j] = 1.0;
            da[j] = 0.0;
        }
    for (j = 0; j < n; j++) {
        double s = S[j + ld * j], p;
        for (k = 0; k < j; k++)
            s = s - S[j + ld * k] * S[j + ld * k];
        if (!(s > 0.0))
            return j + 1;
        p = sqrt(s);
        S[j + ld * j] = p;
        for (i = j + 1; i < n; i++) {
            double t = S[i + ld * j];
            for (k = 0; k < j; k++)
                t = t - S[i + ld * k] * S[j + ld * k];
            S[i + ld * j] = t / p;
        }
    }
    for (i = 0; i < n; i++) {
        double t = da[i];
        for (k = 0; k < i; k++)
            t = t - S[i + ld * k] * da[k];
        da[i] = t / S[i + ld * i];
    }
    for (i = n - 1; i >= 0; i--) {
        double t = da[i];
        for (k = i + 1; k < n; k++)
            t = t - S[k + ld * i] * da[k];
        da[i] = t / S[i + ld * i];
    }
    return 0;
}
