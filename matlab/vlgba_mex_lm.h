/*
 * vlgba_mex_lm.h -- the fused LM gateways' common body (mex_bundle_euclid_lm.c,
 * mex_bundle_projective_lm.c): dense MATLAB inputs -> COO problem -> the whole
 * LM loop on the GPU (vlgba_solve) -> a, b, error_.
 *
 * options struct (every field optional; the drop-in bundle_euclid.m /
 * bundle_projective.m fill it from their name / value arguments):
 *   fix_structure, fix_motion, verbose   0 / 1   (bundle_euclid.m:58-61,73-74)
 *   pivot        'fix_pivot' as camera numbers: 1-based indices (any count,
 *                duplicates allowed), as U(:,:,pivot) reads a numeric pivot
 *                (bundle_euclid.m:62-65,150-153)
 *   pivot_mask   'fix_pivot' as a logical mask (sent as double): 1 x k,
 *                non-zero = fixed; entries past m must be zero
 *   (an index outside 1..m or a mask entry past m is an error: MATLAB would
 *   grow U / W / eA there)
 *   semantics    0 bundle_euclid.m, 1 bundle_euclid_nomex.m
 *   max_iter, max_iter2, lambda0        0 = the reference's 20 / 10 / 1e-3
 *   device                              HIP device
 *   ordered        1 ordered sums, 2 parity mode (bit-identical LM trajectory)
 *   stop_rel       relative-decrease stop of bundle_euclid.m:123 (0 = 1e-3)
 */
#ifndef VLGBA_MEX_LM_H
#define VLGBA_MEX_LM_H

#include "vlgba_mex_util.h"

#include <stdlib.h>
#include <string.h>

static double vm_opt(const mxArray *s, const char *name, double dflt)
{
    const mxArray *f = s ? mxGetField(s, 0, name) : NULL;
    if (!f || mxIsEmpty(f))
        return dflt;
    if (!mxIsDouble(f))
        mexErrMsgIdAndTxt("vlgba:args", "option %s must be double", name);
    return mxGetScalar(f);
}

/* a (num_a x m) and b (3 x n) as the start point, X 2 x n x m, visible n x m;
 * returns a_new, b_new, error_ (1 x k) in out[0..2] */
static void vm_lm(const char *who, int model, const double *K, const mxArray *pa,
                  const mxArray *pb, const mxArray *pX, const mxArray *pvis,
                  const mxArray *popt, mxArray *out[3])
{
    const int m = vm_int(mxGetN(pa), who, "m"), n = vm_int(mxGetN(pb), who, "n");
    const int na = vm_int(mxGetM(pa), who, "num_a");
    const double *X = mxGetPr(pX), *vis = mxGetPr(pvis);
    vlgba_problem p;
    vlgba_options o;
    vlgba_stats st;
    unsigned char *pivot = NULL;
    int *opt_pt, *opt_cam, rc, i, j, max_iter;
    double *ox, *err, num_vis = 0.0;
    long long N = 0, q = 0;
    size_t ij;
    if (popt && !mxIsStruct(popt))
        vm_fail(who, "options must be a struct");
    vm_numel(who, pb, 3 * (size_t)n, "b");
    vm_numel(who, pX, 2 * (size_t)n * m, "X");
    vm_numel(who, pvis, (size_t)n * m, "visible");
    for (ij = 0; ij < (size_t)n * m; ij++)
        if (vis[ij] != 0.0) {   /* any non-zero double is visible (App. A Q10) */
            N++;
            num_vis += vis[ij];   /* bundle_euclid.m:82 sums the values */
        }
    memset(&o, 0, sizeof o);
    o.fix_structure = vm_opt(popt, "fix_structure", 0) != 0;
    o.fix_motion = vm_opt(popt, "fix_motion", 0) != 0;
    o.verbose = vm_opt(popt, "verbose", 0) != 0;
    o.semantics = (int)vm_opt(popt, "semantics", 0);
    o.max_iter = (int)vm_opt(popt, "max_iter", 0);
    o.max_iter2 = (int)vm_opt(popt, "max_iter2", 0);
    o.lambda0 = vm_opt(popt, "lambda0", 0);
    o.device = (int)vm_opt(popt, "device", 0);
    o.ordered = (int)vm_opt(popt, "ordered", 0);
    o.stop_rel = vm_opt(popt, "stop_rel", 0);
    max_iter = o.max_iter > 0 ? o.max_iter : 20;
    {
        const mxArray *pv = popt ? mxGetField(popt, 0, "pivot") : NULL;
        const mxArray *pm = popt ? mxGetField(popt, 0, "pivot_mask") : NULL;
        const int has_pv = pv && !mxIsEmpty(pv), has_pm = pm && !mxIsEmpty(pm);
        if (has_pv || has_pm) {
            const char *bad = NULL;
            size_t k, cnt;
            if ((has_pv && !mxIsDouble(pv)) || (has_pm && !mxIsDouble(pm)))
                vm_fail(who, "pivot / pivot_mask must be double");
            pivot = (unsigned char *)calloc((size_t)m, 1);
            if (!pivot)
                mexErrMsgIdAndTxt("vlgba:nomem", "out of memory");
            if (has_pm) {   /* logical mask */
                const double *v = mxGetPr(pm);
                cnt = mxGetNumberOfElements(pm);
                for (k = 0; k < cnt && !bad; k++)
                    if (v[k] != 0.0) {
                        if (k >= (size_t)m)
                            bad = "fix_pivot: logical index past the camera count";
                        else
                            pivot[k] = 1;
                    }
            }
            if (has_pv) {   /* 1-based camera numbers */
                const double *v = mxGetPr(pv);
                cnt = mxGetNumberOfElements(pv);
                for (k = 0; k < cnt && !bad; k++) {
                    const double x = v[k];
                    if (!(x >= 1.0 && x <= (double)m) || x != (double)(long long)x)
                        bad = "fix_pivot: camera indices must be integers in 1..m";
                    else
                        pivot[(long long)x - 1] = 1;
                }
            }
            if (bad) {
                free(pivot);
                vm_fail(who, bad);
            }
            o.pivot = pivot;
        }
    }
    opt_pt = (int *)malloc(sizeof(int) * (size_t)(N ? N : 1));
    opt_cam = (int *)malloc(sizeof(int) * (size_t)(N ? N : 1));
    ox = (double *)malloc(sizeof(double) * 2 * (size_t)(N ? N : 1));
    err = (double *)malloc(sizeof(double) * (size_t)(max_iter + 1));
    if (!opt_pt || !opt_cam || !ox || !err) {
        free(opt_pt);
        free(opt_cam);
        free(ox);
        free(err);
        free(pivot);
        mexErrMsgIdAndTxt("vlgba:nomem", "out of memory");
    }
    /* point-major COO (i ascending, j ascending: the reference's visiting order) */
    for (i = 0; i < n; i++)
        for (j = 0; j < m; j++) {
            ij = (size_t)i + (size_t)n * j;
            if (vis[ij] != 0.0) {
                opt_pt[q] = i;
                opt_cam[q] = j;
                ox[2 * q] = X[2 * ij];
                ox[2 * q + 1] = X[2 * ij + 1];
                q++;
            }
        }
    memset(&p, 0, sizeof p);
    p.m = m;
    p.n = n;
    p.num_a = na;
    p.num_obs = N;
    p.obs_pt = opt_pt;
    p.obs_cam = opt_cam;
    p.obs_x = ox;
    p.K = K;
    p.num_vis = num_vis;
    p.model = model;
    out[0] = vm_array(2, na, m, 1, 1);
    out[1] = vm_array(2, 3, n, 1, 1);
    memcpy(mxGetPr(out[0]), mxGetPr(pa), sizeof(double) * (size_t)na * m);
    memcpy(mxGetPr(out[1]), mxGetPr(pb), sizeof(double) * 3 * (size_t)n);
    memset(&st, 0, sizeof st);
    rc = vlgba_solve(&p, &o, mxGetPr(out[0]), mxGetPr(out[1]), err, max_iter + 1, &st);
    free(opt_pt);
    free(opt_cam);
    free(ox);
    free(pivot);
    if (rc) {
        free(err);
        mxDestroyArray(out[0]);
        mxDestroyArray(out[1]);
        mexErrMsgIdAndTxt("vlgba:lib", "%s: vlgba_solve failed (%d)", who, rc);
    }
    out[2] = vm_array(2, 1, st.num_error < max_iter + 1 ? st.num_error : max_iter + 1, 1, 1);
    memcpy(mxGetPr(out[2]), err, sizeof(double) * mxGetNumberOfElements(out[2]));
    free(err);
}

#endif /* VLGBA_MEX_LM_H */
