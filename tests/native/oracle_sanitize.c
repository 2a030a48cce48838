/* Host AddressSanitizer / UndefinedBehaviorSanitizer driver for the CPU
 * restatement ("Race detection / sanitizers").  TEST
 * INFRASTRUCTURE ONLY: built by tests/test_sanitize.py together with
 * oracle/ba_oracle.c and oracle/ba_cpu_mt.c under
 * -fsanitize=address,undefined -fno-sanitize-recover=all, then run.
 *
 * It drives every exported stage on a small seeded scene with ragged tracks,
 * a point seen by one camera only, an invisible (point, camera) pair and a
 * zero-rotation first camera (App. A Q2), and cross-checks the dense MEX-layout
 * stages against the sparse and the OpenMP forms: a sanitizer report or a
 * mismatch exits non-zero. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void oracle_mex1(int m, int n, int num_a, const double *K4, const double *a, const double *b,
                 const double *X, const double *vis, double *X_hat, double *A, double *B,
                 double *e, double *U, double *V, double *W, double *eA, double *eB);
void oracle_mex2(int m, int n, int num_a, const double *Y, const double *W, const double *Us,
                 const double *eA, const double *eB, double *S, double *e_);
void oracle_mex3(int m, int n, int num_a, const double *W, const double *da, const double *eB,
                 const double *Vinv, const double *K4, const double *a, const double *b,
                 const double *X, const double *vis, double *db, double *a_new,
                 double *b_new, double *X_hat);
void oracle_sp_linearize(int m, int n, int num_a, const int *pt_ptr, const int *obs_cam,
                         const double *obs_x, const double *K4, const double *a,
                         const double *b, double *obs_xhat, double *A, double *B, double *e,
                         double *U, double *V, double *W, double *eA, double *eB);
void oracle_sp_vinv(int n, double lambda, const double *V, double *Vinv);
void oracle_sp_y(int n, int num_a, const int *pt_ptr, const double *W, const double *Vinv,
                 double *Y);
void oracle_sp_schur(int m, int n, int num_a, const int *pt_ptr, const int *obs_cam,
                     const double *Y, const double *W, const double *Us, const double *eA,
                     const double *eB, double *S, double *e_);
double oracle_sp_update(int m, int n, int num_a, const int *pt_ptr, const int *obs_cam,
                        const double *obs_x, const double *W, const double *da,
                        const double *eB, const double *Vinv, const double *K4,
                        const double *a, const double *b, double *db, double *a_new,
                        double *b_new, double *obs_xhat);
int oracle_chol_seq(int n, double *S, const double *e_, double *da);
double oracle_seq_dot(const double *x, const double *y, long long n);
void oracle_pinv3(const double M[9], double P[9]);

double mt_linearize(int n, const int *pt_ptr, const int *obs_cam, const double *obs_x,
                    const double *K4, const double *a, const double *b, double *jrec,
                    double *W, double *V, double *eB);
void mt_camera_reduce(int m, const int *cam_ptr, const int *cam_obs, const double *jrec,
                      double *U, double *eA);
void mt_damp_y(int n, const int *pt_ptr, double lambda, const double *V, const double *W,
               double *Vinv, double *Y);
void mt_schur(int m, const int *cam_ptr, const int *cam_obs, const int *obs_pt,
              const int *pt_ptr, const int *obs_cam, const double *Y, const double *W,
              const double *U, double lambda, const double *eA, const double *eB, double *S,
              double *e_);
double mt_update(int m, int n, const int *pt_ptr, const int *obs_cam, const double *obs_x,
                 const double *K4, const double *W, const double *da, const double *eB,
                 const double *Vinv, const double *a, const double *b, double *db,
                 double *a_new, double *b_new);

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static double urand(void)   /* xorshift64*, [0, 1) */
{
    rs ^= rs >> 12;
    rs ^= rs << 25;
    rs ^= rs >> 27;
    return (double)((rs * 0x2545F4914F6CDD1Dull) >> 11) * 0x1.0p-53;
}

static void *xcalloc(size_t n, size_t sz)
{
    void *p = calloc(n ? n : 1, sz);
    if (!p) {
        fprintf(stderr, "out of memory\n");
        exit(2);
    }
    return p;
}

static int fails = 0;
static void check(const char *what, const double *x, const double *y, size_t n, double tol)
{
    double scale = 0.0, err = 0.0;
    size_t k;
    for (k = 0; k < n; k++) {
        scale = fmax(scale, fabs(y[k]));
        err = fmax(err, fabs(x[k] - y[k]));
    }
    if (!(err <= tol * fmax(scale, 1e-300))) {
        fprintf(stderr, "MISMATCH %s: max err %.3g (scale %.3g)\n", what, err, scale);
        fails++;
    }
}

int main(void)
{
    enum { m = 7, n = 60, NA = 6 };
    const double lam = 1e-3;
    double K4[4 * m], a[NA * m], b[3 * n];
    int i, j, k;
    for (j = 0; j < m; j++) {
        K4[4 * j] = 500.0;
        K4[4 * j + 1] = 500.0;
        K4[4 * j + 2] = 250.0;
        K4[4 * j + 3] = 250.0;
        for (k = 0; k < 3; k++)   /* camera 0 keeps w = 0 (App. A Q2) */
            a[NA * j + k] = j ? 0.01 * (urand() - 0.5) : 0.0;
        a[NA * j + 3] = 0.3 * j + 0.05 * urand();
        a[NA * j + 4] = 0.02 * (urand() - 0.5);
        a[NA * j + 5] = 0.01 * (urand() - 0.5);
    }
    for (i = 0; i < n; i++) {
        b[3 * i] = 2.0 * (urand() - 0.5) * 40.0 + 0.3 * m / 2;
        b[3 * i + 1] = 2.0 * (urand() - 0.5) * 40.0;
        b[3 * i + 2] = 80.0 + 40.0 * urand();
    }
    /* visibility: ragged consecutive tracks (1..m cameras), plus one hole */
    double *vis = xcalloc((size_t)n * m, sizeof(double));
    int *pt_ptr = xcalloc(n + 1, sizeof(int));
    for (i = 0; i < n; i++) {
        int s = (int)(urand() * m), len = 1 + (int)(urand() * (m - s));
        if (i == 0) { s = 0; len = 1; }   /* seen once */
        for (j = s; j < s + len; j++)
            vis[i + (size_t)n * j] = 1.0;
        if (i == 1 && len > 2)
            vis[i + (size_t)n * (s + 1)] = 0.0;   /* a hole in the track */
    }
    int N = 0;
    for (i = 0; i < n; i++) {
        pt_ptr[i] = N;
        for (j = 0; j < m; j++)
            N += vis[i + (size_t)n * j] != 0.0;
    }
    pt_ptr[n] = N;
    int *obs_cam = xcalloc(N, sizeof(int)), *obs_pt = xcalloc(N, sizeof(int));
    double *X = xcalloc(2 * (size_t)n * m, sizeof(double)), *obs_x = xcalloc(2 * (size_t)N, sizeof(double));
    for (i = 0, k = 0; i < n; i++)
        for (j = 0; j < m; j++)
            if (vis[i + (size_t)n * j] != 0.0) {
                const double *aj = a + NA * j, *bi = b + 3 * i;
                /* a rough pinhole measurement (the exact model is not needed) */
                double z = bi[2] + aj[5], u = 500.0 * (bi[0] + aj[3]) / z + 250.0 + urand() - 0.5,
                       v = 500.0 * (bi[1] + aj[4]) / z + 250.0 + urand() - 0.5;
                X[2 * (i + (size_t)n * j)] = u;
                X[2 * (i + (size_t)n * j) + 1] = v;
                obs_x[2 * k] = u;
                obs_x[2 * k + 1] = v;
                obs_cam[k] = j;
                obs_pt[k] = i;
                k++;
            }
    /* camera-major view for the OpenMP port */
    int *cam_ptr = xcalloc(m + 1, sizeof(int)), *cam_obs = xcalloc(N, sizeof(int));
    for (k = 0; k < N; k++)
        cam_ptr[obs_cam[k] + 1]++;
    for (j = 0; j < m; j++)
        cam_ptr[j + 1] += cam_ptr[j];
    {
        int *pos = xcalloc(m, sizeof(int));
        for (j = 0; j < m; j++)
            pos[j] = cam_ptr[j];
        for (k = 0; k < N; k++)
            cam_obs[pos[obs_cam[k]]++] = k;
        free(pos);
    }

    /* ---- dense MEX-layout stages ---- */
    const size_t nm = (size_t)n * m, ld = (size_t)NA * m;
    double *Xh = xcalloc(2 * nm, 8), *A = xcalloc(2 * NA * nm, 8), *B = xcalloc(6 * nm, 8),
           *e = xcalloc(2 * nm, 8), *U = xcalloc(NA * NA * m, 8), *V = xcalloc(9 * n, 8),
           *W = xcalloc(NA * 3 * nm, 8), *eA = xcalloc(NA * m, 8), *eB = xcalloc(3 * n, 8);
    oracle_mex1(m, n, NA, K4, a, b, X, vis, Xh, A, B, e, U, V, W, eA, eB);
    double *Us = xcalloc(NA * NA * m, 8), *Vinv = xcalloc(9 * n, 8), *Y = xcalloc(NA * 3 * nm, 8);
    memcpy(Us, U, sizeof(double) * NA * NA * m);
    for (j = 0; j < m; j++)
        for (k = 0; k < NA; k++)
            Us[NA * NA * j + k * (NA + 1)] *= 1 + lam;
    oracle_sp_vinv(n, lam, V, Vinv);
    for (j = 0; j < m; j++)   /* Y_ij = W_ij Vinv_i over every pair */
        for (i = 0; i < n; i++) {
            const double *w = W + NA * 3 * (i + (size_t)n * j), *vi = Vinv + 9 * i;
            double *y = Y + NA * 3 * (i + (size_t)n * j);
            int r, c;
            for (c = 0; c < 3; c++)
                for (r = 0; r < NA; r++)
                    y[r + NA * c] = w[r] * vi[3 * c] + w[r + NA] * vi[1 + 3 * c] +
                                    w[r + 2 * NA] * vi[2 + 3 * c];
        }
    double *S = xcalloc(ld * ld, 8), *e_ = xcalloc(ld, 8), *da = xcalloc(ld, 8);
    oracle_mex2(m, n, NA, Y, W, Us, eA, eB, S, e_);
    double *L = xcalloc(ld * ld, 8);
    memcpy(L, S, sizeof(double) * ld * ld);
    if (oracle_chol_seq((int)ld, L, e_, da) != 0) {
        fprintf(stderr, "reduced system not positive definite\n");
        fails++;
    }
    double *db = xcalloc(3 * n, 8), *a_new = xcalloc(ld, 8), *b_new = xcalloc(3 * n, 8),
           *Xh2 = xcalloc(2 * nm, 8);
    oracle_mex3(m, n, NA, W, da, eB, Vinv, K4, a, b, X, vis, db, a_new, b_new, Xh2);

    /* ---- sparse forms: same numbers ---- */
    double *sxh = xcalloc(2 * (size_t)N, 8), *sA = xcalloc(2 * NA * (size_t)N, 8),
           *sB = xcalloc(6 * (size_t)N, 8), *se = xcalloc(2 * (size_t)N, 8),
           *sU = xcalloc(NA * NA * m, 8), *sV = xcalloc(9 * n, 8),
           *sW = xcalloc(NA * 3 * (size_t)N, 8), *seA = xcalloc(NA * m, 8), *seB = xcalloc(3 * n, 8),
           *sY = xcalloc(NA * 3 * (size_t)N, 8), *sS = xcalloc(ld * ld, 8), *se_ = xcalloc(ld, 8);
    oracle_sp_linearize(m, n, NA, pt_ptr, obs_cam, obs_x, K4, a, b, sxh, sA, sB, se, sU, sV, sW,
                        seA, seB);
    check("U", sU, U, NA * NA * m, 0.0);
    check("V", sV, V, 9 * n, 0.0);
    check("eB", seB, eB, 3 * n, 0.0);
    oracle_sp_y(n, NA, pt_ptr, sW, Vinv, sY);
    oracle_sp_schur(m, n, NA, pt_ptr, obs_cam, sY, sW, Us, seA, seB, sS, se_);
    check("S", sS, S, ld * ld, 0.0);
    check("e_", se_, e_, ld, 0.0);
    double *sdb = xcalloc(3 * n, 8), *sa = xcalloc(ld, 8), *sb = xcalloc(3 * n, 8),
           *sxh2 = xcalloc(2 * (size_t)N, 8);
    double sse = oracle_sp_update(m, n, NA, pt_ptr, obs_cam, obs_x, sW, da, seB, Vinv, K4, a, b,
                                  sdb, sa, sb, sxh2);
    check("db", sdb, db, 3 * n, 0.0);
    check("b_new", sb, b_new, 3 * n, 0.0);
    (void)oracle_seq_dot(se, se, 2 * (long long)N);

    /* ---- OpenMP port ---- */
    double *jrec = xcalloc(20 * (size_t)N, 8), *mW = xcalloc(18 * (size_t)N, 8),
           *mV = xcalloc(9 * n, 8), *meB = xcalloc(3 * n, 8), *mU = xcalloc(36 * m, 8),
           *meA = xcalloc(6 * m, 8), *mVinv = xcalloc(9 * n, 8), *mY = xcalloc(18 * (size_t)N, 8),
           *mS = xcalloc(ld * ld, 8), *me_ = xcalloc(ld, 8), *mdb = xcalloc(3 * n, 8),
           *ma = xcalloc(ld, 8), *mb = xcalloc(3 * n, 8);
    (void)mt_linearize(n, pt_ptr, obs_cam, obs_x, K4, a, b, jrec, mW, mV, meB);
    mt_camera_reduce(m, cam_ptr, cam_obs, jrec, mU, meA);
    check("mt U", mU, U, 36 * m, 1e-13);
    mt_damp_y(n, pt_ptr, lam, mV, mW, mVinv, mY);
    mt_schur(m, cam_ptr, cam_obs, obs_pt, pt_ptr, obs_cam, mY, mW, mU, lam, meA, meB, mS, me_);
    {   /* the port fills the lower triangle: compare that */
        size_t r, c;
        double *lo = xcalloc(ld * ld, 8), *lm = xcalloc(ld * ld, 8);
        for (c = 0; c < ld; c++)
            for (r = c; r < ld; r++) {
                lo[r + ld * c] = S[r + ld * c];
                lm[r + ld * c] = mS[r + ld * c];
            }
        check("mt S", lm, lo, ld * ld, 1e-12);
        free(lo);
        free(lm);
    }
    check("mt e_", me_, e_, ld, 1e-12);
    double msse = mt_update(m, n, pt_ptr, obs_cam, obs_x, K4, mW, da, meB, mVinv, a, b, mdb, ma, mb);
    if (!(fabs(msse - sse) <= 1e-12 * sse)) {
        fprintf(stderr, "MISMATCH new sse %.17g vs %.17g\n", msse, sse);
        fails++;
    }
    {
        double P[9], M3[9] = {0};   /* zero block: pinv 0 (bundle_euclid.m:180) */
        oracle_pinv3(M3, P);
        for (k = 0; k < 9; k++)
            if (P[k] != 0.0)
                fails++;
    }
    printf("oracle sanitize: N=%d sse=%.6g fails=%d\n", N, sse, fails);
    free(vis); free(pt_ptr); free(obs_cam); free(obs_pt); free(X); free(obs_x);
    free(cam_ptr); free(cam_obs);
    free(Xh); free(A); free(B); free(e); free(U); free(V); free(W); free(eA); free(eB);
    free(Us); free(Vinv); free(Y); free(S); free(e_); free(da); free(L);
    free(db); free(a_new); free(b_new); free(Xh2);
    free(sxh); free(sA); free(sB); free(se); free(sU); free(sV); free(sW); free(seA); free(seB);
    free(sY); free(sS); free(se_); free(sdb); free(sa); free(sb); free(sxh2);
    free(jrec); free(mW); free(mV); free(meB); free(mU); free(meA); free(mVinv); free(mY);
    free(mS); free(me_); free(mdb); free(ma); free(mb);
    return fails ? 1 : 0;
}
