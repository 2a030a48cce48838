/*
 * vlgba.h -- C ABI of libvlgba, the MI355X (gfx950) bundle adjuster.
 *
 * Drop-in for the Levenberg-Marquardt paths of caomw/BundleAdjustmentMatlab
 * (VLG toolbox/bundle): Euclidean (bundle_euclid.m + mex_bundle_{1,2,3}) and
 * projective (bundle_projective.m + mex_bundle_proj_{1,2,3}).  Plain C:
 * pointers and sizes only, no C++ / torch / HIP types.  All arrays are fp64 column major in the reference's MATLAB
 * layouts unless stated otherwise; indices are 0-based int32.
 *
 * Return codes: 0 on success; VLGBA_E_* (< 0) for argument errors; a
 * negative hipError_t (-1 .. -999) for device failures.
 *
 * Threading: a vlgba_ctx is single-threaded (one HIP stream per context);
 * distinct contexts may be used from distinct threads.
 */
#ifndef VLGBA_H
#define VLGBA_H

#ifdef __cplusplus
extern "C" {
#endif

#define VLGBA_E_ARG (-1001)      /* bad size / option                        */
#define VLGBA_E_NUMA (-1002)     /* num_a not in {6, 7, 10} (Euclidean) / 12 (projective) */
#define VLGBA_E_ORDER (-1003)    /* observation list not point-major / dups  */
#define VLGBA_E_NOMEM (-1004)    /* host allocation failed                    */
#define VLGBA_E_COMM (-1005)     /* RCCL failure                              */
#define VLGBA_E_ABI (-1006)      /* caller built against another vlgba.h      */

/* ABI of this header.  Bumped whenever a public struct, constant or entry
 * point changes: 1 = the round-1/2 layouts; 2 = vlgba_stats.pinv_passes /
 * spin_retries, vlgba_step_info.spin_retry, VLGBA_NPLAN 28; 3 =
 * vlgba_stats.nd_retries, vlgba_step_info.nd_retry, vlgba_comm_release,
 * VLGBA_NKERNELS 18 (k_update_linearize), vlgba_kernel_flops; 4 =
 * vlgba_debug_dehom; 5 = vlgba_debug_dehom removed, VLGBA_NPLAN 29 (the
 * envelope runner's launch count), vlgba_debug_force_status word 6.  Callers
 * check it once at load time with VLGBA_ABI_CHECK() (the MEX gateways and the Python
 * loader do): the library compares the version and the struct sizes the
 * caller was compiled with against its own and returns 0 or VLGBA_E_ABI. */
#define VLGBA_ABI_VERSION 5

/* camera models (vlgba_problem.model) */
#define VLGBA_MODEL_EUCLIDEAN 0   /* bundle_euclid.m: a = [w; T; (K)], num_a 6/7/10     */
#define VLGBA_MODEL_PROJECTIVE 1  /* bundle_projective.m: a = P(:) (3x4), num_a = 12   */

/* ------------------------------------------------------------------------
 * Problem: the reference's packed parameters and a COO observation list.
 *   a      num_a x m   [w; T; (K)] per camera  (bundle_euclid.m:88-96), or
 *                      P(:) per camera          (bundle_projective.m:70-73)
 *   b      3 x n       Xe(1:3,:)               (bundle_euclid.m:99;
 *                      Xp(1:3,:), bundle_projective.m:76)
 *   obs    visible (point, camera) pairs of x(1:2,:,:) / 'visibility'
 *          (bundle_euclid.m:50,71,102); any order, duplicates rejected.
 * ------------------------------------------------------------------------ */
typedef struct {
    int m;                 /* cameras                                            */
    int n;                 /* points                                             */
    int num_a;             /* 6 fix_calibration, 7 fix_principal, 10 variable K;
                              12 projective                                      */
    long long num_obs;     /* visible observations                               */
    const int *obs_pt;     /* [num_obs] point index                              */
    const int *obs_cam;    /* [num_obs] camera index                             */
    const double *obs_x;   /* [2*num_obs] measured (u, v)                        */
    const double *K;       /* [4*m] fx fy cx cy (mex_bundle_1_XABeUVWeAeB.c:186);
                              unused (may be NULL) for the projective model      */
    double num_vis;        /* sum of the visibility values (bundle_euclid.m:82);
                              <= 0 means num_obs                                 */
    int model;             /* VLGBA_MODEL_*; 0 (zero-initialised) = Euclidean.
                              Projective: LM rule of bundle_projective.m:182-207
                              (errors / num_vis compared, lambda / 10 on accept,
                              * 10 on reject); fix_pivot is not an option there */
} vlgba_problem;

struct vlgba_step_info;

typedef struct {
    int fix_structure;           /* bundle_euclid.m:58-59                      */
    int fix_motion;              /* :60-61                                     */
    const unsigned char *pivot;  /* [m] or NULL: 'fix_pivot', pivot (:62-65)   */
    int verbose;                 /* 'verbose' (:73-74, printed to stdout)     */
    int max_iter;                /* 0 -> 20  (:117)                            */
    int max_iter2;               /* 0 -> 10  (:118)                            */
    double lambda0;              /* 0 -> 1e-3 (:111)                           */
    int device;                  /* HIP device ordinal                         */
    /* point sharding over ranks (one process per GPU); world_size <= 1: none  */
    int rank;
    int world_size;
    const void *comm_id;         /* 128-byte ncclUniqueId from rank 0, or NULL */
    /* reduced-camera solve (replaces pinv(S)*e_, bundle_euclid.m:193):
     * 0 (default) automatic -- block cyclic reduction (odd-even nested
     *   dissection, log2 depth) when S is tile-tridiagonal (co-visibility
     *   band narrower than 64 rows), else the envelope tile Cholesky;
     * 1: tile Cholesky over every lower tile (measurement);
     * 2: envelope tile Cholesky (tiles outside the envelope are exactly zero,
     *   so 1 and 2 give identical results);
     * 3: one-workgroup sequential Cholesky (parity mode, small problems);
 * 4: the envelope Cholesky on a nested-dissection camera order whenever the
 *   cameras split into independent arcs + a separator (0 takes that order
 *   when it shortens the chain of factor steps by a quarter or more).
     * Any of them meeting a non-positive pivot falls back to pinv(S) e_ from
     * a symmetric eigen-decomposition on the GPU (vlgba_step_info.pinv)      */
    int dense_solve;
    /* 1: "ordered" mode -- every sum over points runs sequentially in
     * ascending point order exactly as the reference loops do, making the
     * reduced system bit-identical to the reference arithmetic; 2: "parity"
     * mode -- ordered, plus the sequential Cholesky (dense_solve 3) and the LM
     * scalars e'e, dp'(lambda dp + g) summed in the reference's flat order,
     * so the whole LM trajectory (error_, a, b) is bit-identical to the CPU
     * oracle's (single rank, small problems); 0 (default): the fused chunked
     * Schur path (same terms, sums grouped per chunk of points, deterministic
     * run to run)                                                            */
    int ordered;
    /* world_size > 1 without comm_id: a host collective instead of RCCL.  The
     * library copies the buffer to host memory, calls allreduce(buf, count,
     * user), which must leave the element-wise sum over ranks in buf and
     * return 0, and copies it back (e.g. gloo via torch.distributed). */
    int (*allreduce)(double *buf, long long count, void *user);
    void *allreduce_user;
    /* fast-path Schur complement kernel (ordered = 0): 0 (default) automatic --
     * dense per-chunk Y W^T products on fp64 MFMA when every point has at most
     * 16 * (num_a == 6 ? 3 : 4) / num_a observations, else per-term sums;
     * 1: per-term sums (measurement / cross-check).  Same terms either way. */
    int schur_kernel;
    /* driver semantics: 0 (default) bundle_euclid.m (MEX-backed: the back
     * substitution uses da(1:6,j) only, mex_bundle_3_db_new.c:113-120, App. A
     * Q3; 'fix_pivot' honoured); 1 bundle_euclid_nomex.m (the pure-MATLAB
     * twin: db uses all num_a rows of da, bundle_euclid_nomex.m:268-277; no
     * fix_pivot -- pivot is ignored) */
    int semantics;
    /* stop rule of bundle_euclid.m:123: stop once the accepted step lowers
     * error_ by no more than stop_rel * error_(previous); 0 -> 1e-3          */
    double stop_rel;
    /* per-pass log hook (NULL: none): vlgba_run calls on_pass(pass, iter, info,
     * user) after every LM pass (1-based pass counter, iter = the reference's
     * iteration counter after the pass, bundle_euclid.m:221), on the calling
     * thread, rank 0 only; bundle.py writes it as one JSON line per pass */
    void (*on_pass)(int pass, int iter, const struct vlgba_step_info *info, void *user);
    void *on_pass_user;
} vlgba_options;

typedef struct {
    int iterations;        /* LM passes (accepted + rejected)                 */
    int accepted;          /* accepted steps                                  */
    int num_error;         /* entries written to error_out                    */
    double lambda;         /* final damping                                   */
    double seconds;        /* wall time of the solve (setup excluded)         */
    int pinv_passes;       /* passes whose step came from the pinv fallback   */
    int spin_retries;      /* passes re-solved after a hand-off spin timeout  */
    int nd_retries;        /* passes whose nested-dissection Cholesky met a
                              non-positive pivot and the natural-order Cholesky
                              (rocSOLVER dpotrf) took the step instead        */
} vlgba_stats;

/* One LM pass, for benchmarking / custom drivers. */
typedef struct vlgba_step_info {
    double old_sse;        /* e'e before the step (bundle_euclid.m:209)       */
    double new_sse;        /* e_new'e_new (:210)                              */
    double dpg;            /* dp'(lambda dp + g) (:217)                       */
    double rho;
    double lambda;         /* lambda used by this pass                        */
    int accepted;
    int chol_failed;       /* non-positive pivot in the reduced solve: the
                              step came from the pinv fallback (= pinv)       */
    int pinv;              /* da = pinv(S) e_ by eigen-decomposition: a dense
                              (num_a m)^2 copy of S + rocSOLVER dsyevd, i.e.
                              8 (num_a m)^2 bytes of device memory and
                              O((num_a m)^3) flops (cfg3: 288 MB); the library
                              notes each such pass on stderr (ld, seconds)    */
    int spin_retry;        /* the one-launch solve gave up waiting on a
                              hand-off (a bounded spin): the pass was solved
                              again with the per-level launches (every rank
                              takes the same decision: the status words are
                              all-reduced with the pass scalars)              */
    int nd_retry;          /* the nested-dissection order met a non-positive
                              pivot; the natural-order dpotrf solved the pass
                              (pinv = 0) or failed too (pinv = 1)             */
} vlgba_step_info;

typedef struct vlgba_ctx vlgba_ctx;

/* ---- fused solver: the whole bundle_euclid.m LM loop on the GPU -----------
 * Replaces bundle_euclid.m:111-249 (and its three MEX calls :139,192,204).
 * a (num_a*m) and b (3*n) are read as the start point and overwritten with
 * the result.  error_out (may be NULL) receives error_ (SSE / num_vis per
 * accepted step, :219-231): at most error_cap entries are written (error_ has
 * at most max_iter entries; stats->num_error is its full length). */
int vlgba_solve(const vlgba_problem *prob, const vlgba_options *opt, double *a, double *b,
                double *error_out, int error_cap, vlgba_stats *stats);

/* ---- handle API -------------------------------------------------------- */
int vlgba_create(const vlgba_problem *prob, const vlgba_options *opt, vlgba_ctx **out);
int vlgba_set_params(vlgba_ctx *ctx, const double *a, const double *b);
int vlgba_get_params(vlgba_ctx *ctx, double *a, double *b);
/* one LM pass at the context's lambda; relinearize != 0 forces stage 1 even
 * when the previous pass was rejected (bench: every pass does full work).
 * update_lm != 0 applies the accept/reject rule (:218-241) to the context. */
int vlgba_step(vlgba_ctx *ctx, int relinearize, int update_lm, vlgba_step_info *info);
/* stage 1 at the current parameters (mex_bundle_1_XABeUVWeAeB.c outputs, the
 * reduced forms of bundle_euclid.m:139-154) -- the one the context holds when
 * it is current (after a rejected step, or the fast path's fused update after
 * an accepted one), else computed: U (num_a x num_a x m), eA
 * (num_a x m) summed over all ranks; V (3 x 3 x n_local), eB (3 x n_local) and
 * W (num_a x 3 per observation, observations point-major: points ascending,
 * cameras ascending within a point) for this rank's points.  Any pointer may
 * be NULL.  Also marks the linearisation valid for the next vlgba_step. */
int vlgba_get_linearization(vlgba_ctx *ctx, double *U, double *eA, double *V, double *eB,
                            double *W);
/* the LM loop from the context's parameters; error_out / error_cap as
 * vlgba_solve.  Every handle entry point makes the context's device current.
 * The accept / lambda / stop decisions are the host's (a handful of scalars
 * per pass, as bundle_euclid.m keeps them in MATLAB). */
int vlgba_run(vlgba_ctx *ctx, double *error_out, int error_cap, vlgba_stats *stats);
/* npass full passes at the context's parameters and lambda, each
 * relinearising, none changing the context (vlgba_step(ctx, 1, 0, .) npass
 * times); info: the last pass */
int vlgba_run_passes(vlgba_ctx *ctx, int npass, vlgba_step_info *info);
/* the last pass's step: da (num_a * m, the reduced solve) and db (3 x
 * n_local, this rank's points); either may be NULL */
int vlgba_get_step(vlgba_ctx *ctx, double *da, double *db);
/* the reduced camera system at the context's lambda (mex_bundle_2_Se_ output,
 * bundle_euclid.m:192): the co-visible blocks S_jk, j >= k (num_a x num_a
 * column major each, lower triangle meaningful for j == k; count =
 * vlgba_plan_info [10]) with their camera pairs blk_jk [2 * count], and e_
 * (num_a * m).  Linearises first if the parameters changed.  NULL skips. */
int vlgba_get_reduced_system(vlgba_ctx *ctx, int *blk_jk, double *blocks, double *e_);
int vlgba_sync(vlgba_ctx *ctx);
void vlgba_destroy(vlgba_ctx *ctx);
/* device-kernel timing of the last vlgba_step, milliseconds per phase:
 * [0] linearize [1] camera reduce [2] damp/Y [3] schur [4] assemble
 * [5] cholesky+solve [6] update; requires vlgba_set_timing(ctx, 1) first. */
int vlgba_set_timing(vlgba_ctx *ctx, int on);
int vlgba_phase_ms(vlgba_ctx *ctx, double *ms7);
/* per-kernel device time accumulated over the passes run with timing on
 * (HIP events around every launch): ms[k], calls[k] for k < VLGBA_NKERNELS,
 * named by vlgba_kernel_name(k); reset = 1 clears the accumulators.  ctx NULL:
 * the process-wide sums of the contexts destroyed with timing on (environment
 * VLGBA_KTIME_ALL=1 switches timing on at every vlgba_create: the growing
 * replay's device-busy time). */
#define VLGBA_NKERNELS 18
int vlgba_kernel_ms(vlgba_ctx *ctx, double *ms, long long *calls, int reset);
/* the reduced solve's algorithmic flops (vlgba_plan_info [25..27]) of the timed
 * passes, on the timer that ran them (k_cr_factor / k_factor_step, k_syrk,
 * k_cr_back / k_backward); ctx NULL: process-wide as vlgba_kernel_ms.  Cleared
 * by vlgba_kernel_ms(.., reset = 1). */
int vlgba_kernel_flops(vlgba_ctx *ctx, double *flops);
const char *vlgba_kernel_name(int k);
/* execution-plan sizes of this rank (roofline accounting in bench.py):
 * [0] observations [1] points [2] cameras [3] num_a [4] Schur chunks
 * [5] chunk block slots [6] chunk camera slots [7] Schur groups [8] group
 * block slots [9] group camera slots [10] co-visible blocks (j >= k)
 * [11] 64-row tiles of S [12] cyclic-reduction levels (0: tile Cholesky)
 * [13] eliminated tiles [14] kept-tile updates [15] ordered mode
 * [16] Schur (obs, obs) terms [17] chunk metadata words [18] MFMA Schur
 * chunks in use [19] rows per cyclic-reduction tile (64, or NA * floor(32 /
 * NA) for the camera-aligned tiles; 0 without cyclic reduction) [20] MFMA
 * Schur groups (the leading ones; the rest use per-term sums) [21] points
 * reordered internally (1: short tracks first, input order restored at the
 * API) [22] long tracks (more views than a Schur chunk holds: segment chunks
 * + the long-track kernels) [23] nested-dissection arcs of the envelope
 * Cholesky (0: natural camera order) [24] its separator tiles [25] the
 * reduced solve's algorithmic flops in the launches timed as k_factor_step /
 * k_cr_factor (the one-launch cyclic reduction: all of it) [26] in the
 * separator SYRK (k_syrk) [27] in the backward solve (k_backward / k_cr_back):
 * tile-dense potrf + trtri, GEMMs and GEMVs, each counted once [28] envelope
 * runner launches (k_env_runner, opt-in VLGBA_ENV_RUNNER=1) made by this
 * context so far.  Writes min(len, VLGBA_NPLAN) entries, returns VLGBA_NPLAN. */
#define VLGBA_NPLAN 29
int vlgba_plan_info(vlgba_ctx *ctx, long long *info, int len);

/* ---- stage entries with the reference MEX argument layouts ---------------
 * Host pointers in, host pointers out; every output is fully written (zeros
 * / X for invisible pairs, as the MEX files leave them).  vis is n x m
 * (non-zero = visible, bundle_euclid.m:81). */

/* [X_hat A B e U V W eA eB] = mex_bundle_1_XABeUVWeAeB(K, a, b, X, visible)
 * replaces toolbox/bundle/mex_bundle_1_XABeUVWeAeB.c:72-337. */
int vlgba_mex_bundle_1(int m, int n, int num_a, const double *K, const double *a,
                       const double *b, const double *X, const double *vis,
                       double *X_hat, double *A, double *B, double *e, double *U, double *V,
                       double *W, double *eA, double *eB);

/* [S e_] = mex_bundle_2_Se_(Y, W, U, eA, eB)
 * replaces toolbox/bundle/mex_bundle_2_Se_.c:15-158.  The co-visibility
 * pattern is taken from the non-zero W_ij / Y_ij blocks (exact: the
 * reference adds exact zeros for the others). */
int vlgba_mex_bundle_2(int m, int n, int num_a, const double *Y, const double *W,
                       const double *U, const double *eA, const double *eB, double *S,
                       double *e_);

/* [db a_new b_new X_hat] = mex_bundle_3_db_new(W, da, eB, V_inv, K, a, b, X, visible)
 * replaces toolbox/bundle/mex_bundle_3_db_new.c:12-170 (db :99-134 uses da(1:6,j)
 * only, as the reference does). */
int vlgba_mex_bundle_3(int m, int n, int num_a, const double *W, const double *da,
                       const double *eB, const double *Vinv, const double *K, const double *a,
                       const double *b, const double *X, const double *vis, double *db,
                       double *a_new, double *b_new, double *X_hat);

/* Projective stages (mex_bundle_proj_*.c: the same layouts with num_a = 12
 * and no K):
 * [X_hat A B e U V W eA eB] = mex_bundle_proj_1_XABeUVWeAeB(a, b, X, visible)
 * replaces toolbox/bundle/mex_bundle_proj_1_XABeUVWeAeB.c:88-332. */
int vlgba_mex_bundle_proj_1(int m, int n, const double *a, const double *b, const double *X,
                            const double *vis, double *X_hat, double *A, double *B, double *e,
                            double *U, double *V, double *W, double *eA, double *eB);

/* [S e_] = mex_bundle_proj_2_Se_(Y, W, U, eA, eB)
 * replaces toolbox/bundle/mex_bundle_proj_2_Se_.c:15-158 (num_a = 12). */
int vlgba_mex_bundle_proj_2(int m, int n, const double *Y, const double *W, const double *U,
                            const double *eA, const double *eB, double *S, double *e_);

/* [db a_new b_new X_hat] = mex_bundle_proj_3_db_new(W, da, eB, V_inv, a, b, X, visible)
 * replaces toolbox/bundle/mex_bundle_proj_3_db_new.c:34-178 (db uses
 * da(1:6,j) only, :107-121, as the Euclidean stage does). */
int vlgba_mex_bundle_proj_3(int m, int n, const double *W, const double *da, const double *eB,
                            const double *Vinv, const double *a, const double *b,
                            const double *X, const double *vis, double *db, double *a_new,
                            double *b_new, double *X_hat);

/* ---- batched one-camera refinement with the structure fixed ---------------
 * The bundle_euclid call of estimate_camera.m:247-253,
 *   bundle_euclid(K, T, Omega, X, x0, ['fix_calibration',] 'fix_structure',
 *                 'visibility', inlier')
 * for nprob independent cameras at once (one workgroup per camera and LM
 * pass; the LM rule of bundle_euclid.m:111-241 per camera on the host).  Each
 * camera's trajectory equals the parity-mode solver's (and the CPU oracle's)
 * bit for bit.  Camera q sees observations obs_ptr[q] .. obs_ptr[q+1]-1 of
 * fixed points X (3 per observation) measured at x (2 per observation);
 * num_vis = its observation count. */
typedef struct {
    int nprob;
    int num_a;                 /* 6 fix_calibration, 7 fix_principal, 10 free K */
    const long long *obs_ptr;  /* [nprob + 1], obs_ptr[0] = 0                  */
    const double *X;           /* [3 * N] world point of each observation      */
    const double *x;           /* [2 * N] measured (u, v)                       */
    const double *K;           /* [4 * nprob] fx fy cx cy                       */
} vlgba_resect_problem;

/* a (num_a x nprob, [w; T; (K)] per camera) is the start point and receives the
 * result; error_out (nprob x error_cap, row q = camera q's error_) and
 * num_error (nprob) may be NULL.  opt: max_iter, max_iter2, lambda0,
 * stop_rel, device are honoured (the rest does not apply). */
int vlgba_resect(const vlgba_resect_problem *prob, const vlgba_options *opt, double *a,
                 double *error_out, int error_cap, int *num_error, vlgba_stats *stats);

/* Multi-GPU: rank 0 creates the 128-byte RCCL unique id, the caller
 * broadcasts it (e.g. torch.distributed) and passes it as opt->comm_id.
 * NOTE: reuse one id for every solve of a device set, or release each id
 * with vlgba_comm_release once no context will pass it again -- the library
 * keeps the communicators an id made (below); past 64 idle ones it destroys
 * those of the oldest ids, with a warning. */
int vlgba_get_unique_id(void *id128);
/* The library keeps RCCL communicators for the next context created with the
 * same (id, world size, rank).  A caller that will not pass an id again
 * releases it: the idle communicators made from it are destroyed (ones still
 * held by a context are destroyed with it).  Returns the number destroyed. */
int vlgba_comm_release(const void *id128);

/* Diagnostics: the device sin / cos the rotation tables use (glibc's
 * algorithm, vlg_libm.h) for n host arguments -- the parity tests compare them
 * with the host libm bit for bit.  |x| < 105414350. */
int vlgba_debug_sincos(const double *x, double *s, double *c, long long n);
/* the pinv fallback of the reduced solve (rocSOLVER dsyevd + the pinv kernels)
 * on a host ld x ld symmetric S (lower triangle read) and e_: da = pinv(S) e_
 * with MATLAB's tolerance ld * eps(max |eigenvalue|). */
int vlgba_debug_pinv_solve(int ld, const double *S, const double *e_, double *da);
/* Fault injection (tests / the bench's fallback timing): the next `passes`
 * passes of ctx report word 4 = a non-positive pivot (the pass then takes the
 * pinv step) or word 5 = a hand-off spin timeout of the one-launch solve (the
 * pass is solved again without spins), or word 6 = the envelope runner
 * (k_env_runner, opt-in VLGBA_ENV_RUNNER=1) fails to start (the factorization
 * then runs with the column launches alone).  VLGBA_DEBUG_SPIN_TIMEOUT=
 * "rank:passes" sets word 5 at context creation. */
int vlgba_debug_force_status(vlgba_ctx *ctx, int word, int passes);
/* The envelope solve's nested-dissection planner on the host (no GPU): for
 * m cameras of num_a parameters and the co-visible blocks blk_jk [2 * nb]
 * (j >= k), the chosen arc count K (0: none), the arc boundaries bnd [K + 1]
 * (cameras bnd[t] .. bnd[t+1]-1, minus the separator: the cameras co-visible
 * with an earlier arc) and the predicted chain of factor steps (crit).
 * bnd must hold 9 ints. */
int vlgba_debug_nd_plan(int m, int num_a, const int *blk_jk, int nb, int *bnd, int *crit);

/* Library / device info: writes a NUL-terminated string, returns its length. */
int vlgba_version(char *buf, int len);
/* 0 when abi_version and the sizes of the public structs the caller was
 * compiled with are the library's, else VLGBA_E_ABI (see VLGBA_ABI_VERSION). */
int vlgba_abi_check(int abi_version, long long sz_problem, long long sz_options,
                    long long sz_stats, long long sz_step_info, long long sz_resect_problem);
#define VLGBA_ABI_CHECK()                                                                    \
    vlgba_abi_check(VLGBA_ABI_VERSION, (long long)sizeof(vlgba_problem),                     \
                    (long long)sizeof(vlgba_options), (long long)sizeof(vlgba_stats),        \
                    (long long)sizeof(vlgba_step_info), (long long)sizeof(vlgba_resect_problem))
int vlgba_device_count(void);

/* ---- synthetic scenes on the GPU --------------
 * Configs 2-4's banded model (a restatement of
 * toolbox/test/generate_scene_and_motion.m:36-117: f = width, c = centre,
 * damped random-walk cameras, points at depth U(lo, hi) seen by `track`
 * consecutive cameras, N(0, noise^2) pixel noise) and the perturbation of
 * toolbox/test/demo_bundle_euclid.m:29-31, generated by counter-based
 * (Philox4x32-10) kernels: the same seed gives the same scene on any GPU and
 * launch geometry.  Outputs are host buffers (NULL: not copied); observations
 * are point-major with cameras ascending, N = n * min(track, m).            */
typedef struct {
    int m, n, track;
    double depth_lo, depth_hi;     /* point depth in front of its first camera  */
    double noise;                  /* pixel noise sigma                         */
    unsigned long long seed;
    int keep_first_rotation;       /* w0(:,1) = w(:,1) (the test_mview path)    */
    double width, height;          /* image size; 0 -> 500                      */
} vlgba_scene_spec;

typedef struct {
    double *K, *w, *T, *X;         /* [4m] [3m] [3m] [4n] ground truth (X(4,:) = 1) */
    double *w0, *T0, *X0;          /* [3m] [3m] [4n] perturbed initial values       */
    int *obs_pt, *obs_cam;         /* [N]                                           */
    double *obs_x;                 /* [2N] measured (u, v)                          */
    long long num_obs_cap;         /* capacity of the observation arrays (>= N)     */
    long long num_obs;             /* out: N                                        */
    long long behind;              /* out: observations at depth <= 0.01 depth_lo   */
} vlgba_scene_out;

int vlgba_scene_banded(const vlgba_scene_spec *spec, int device, vlgba_scene_out *out);

#ifdef __cplusplus
}
#endif
#endif /* VLGBA_H */
