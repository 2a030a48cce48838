/*
 * [db a_new b_new X_hat] = mex_bundle_proj_3_db_new(W, da, eB, V_inv, a, b, X, visible)
 *
 * Drop-in for toolbox/bundle/mex_bundle_proj_3_db_new.c:34-178 (called at
 * bundle_projective.m:177): back substitution with da(1:6,j) only
 * (:107-142, App. A Q3), a_new / b_new (:144-154), X_hat (:156-175);
 * m = cols(a), n = cols(b) (:79-80).  GPU: vlgba_mex_bundle_proj_3.
 */
#include "vlgba_mex_util.h"

#define WHO "mex_bundle_proj_3_db_new"

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[])
{
    mxArray *out[4];
    const int na = 12;
    int m, n, rc;
    vm_check(WHO, nrhs, prhs, 8, nlhs, 4);
    m = vm_int(mxGetN(prhs[4]), WHO, "m");
    n = vm_int(mxGetN(prhs[5]), WHO, "n");
    if (mxGetM(prhs[4]) != 12)
        vm_fail(WHO, "a must be 12 x m (P(:))");
    vm_numel(WHO, prhs[0], (size_t)na * 3 * n * m, "W");
    vm_numel(WHO, prhs[1], (size_t)na * m, "da");
    vm_numel(WHO, prhs[2], 3 * (size_t)n, "eB");
    vm_numel(WHO, prhs[3], 9 * (size_t)n, "V_inv");
    vm_numel(WHO, prhs[6], 2 * (size_t)n * m, "X");
    vm_numel(WHO, prhs[7], (size_t)n * m, "visible");
    out[0] = vm_array(2, 3, n, 1, 1);
    out[1] = vm_array(2, na, m, 1, 1);
    out[2] = vm_array(2, 3, n, 1, 1);
    out[3] = vm_array(3, 2, n, m, 1);
    rc = vlgba_mex_bundle_proj_3(m, n, mxGetPr(prhs[0]), mxGetPr(prhs[1]), mxGetPr(prhs[2]),
                                 mxGetPr(prhs[3]), mxGetPr(prhs[4]), mxGetPr(prhs[5]),
                                 mxGetPr(prhs[6]), mxGetPr(prhs[7]), mxGetPr(out[0]),
                                 mxGetPr(out[1]), mxGetPr(out[2]), mxGetPr(out[3]));
    vm_rc(WHO, rc, out, 4);
    vm_publish(nlhs, plhs, out, 4);
}
