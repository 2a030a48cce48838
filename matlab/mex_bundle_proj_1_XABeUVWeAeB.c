/*
 * [X_hat A B e U V W eA eB] = mex_bundle_proj_1_XABeUVWeAeB(a, b, X, visible)
 *
 * Drop-in for toolbox/bundle/mex_bundle_proj_1_XABeUVWeAeB.c:88-332 (called at
 * bundle_projective.m:116): the projective camera a = P(:) (12 x m), no K;
 * m = cols(a), n = cols(b) (:140-141); outputs as mex_bundle_1 with num_a = 12.
 * GPU: vlgba_mex_bundle_proj_1.
 */
#include "vlgba_mex_util.h"

#define WHO "mex_bundle_proj_1_XABeUVWeAeB"

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[])
{
    mxArray *out[9];
    const int na = 12;
    int m, n, rc;
    vm_check(WHO, nrhs, prhs, 4, nlhs, 9);
    m = vm_int(mxGetN(prhs[0]), WHO, "m");
    n = vm_int(mxGetN(prhs[1]), WHO, "n");
    if (mxGetM(prhs[0]) != 12)
        vm_fail(WHO, "a must be 12 x m (P(:))");
    vm_numel(WHO, prhs[1], 3 * (size_t)n, "b");
    vm_numel(WHO, prhs[2], 2 * (size_t)n * m, "X");
    vm_numel(WHO, prhs[3], (size_t)n * m, "visible");
    out[0] = vm_array(3, 2, n, m, 1);
    out[1] = vm_array(4, 2, na, n, m);
    out[2] = vm_array(4, 2, 3, n, m);
    out[3] = vm_array(3, 2, n, m, 1);
    out[4] = vm_array(3, na, na, m, 1);
    out[5] = vm_array(3, 3, 3, n, 1);
    out[6] = vm_array(4, na, 3, n, m);
    out[7] = vm_array(2, na, m, 1, 1);
    out[8] = vm_array(2, 3, n, 1, 1);
    rc = vlgba_mex_bundle_proj_1(m, n, mxGetPr(prhs[0]), mxGetPr(prhs[1]), mxGetPr(prhs[2]),
                                 mxGetPr(prhs[3]), mxGetPr(out[0]), mxGetPr(out[1]),
                                 mxGetPr(out[2]), mxGetPr(out[3]), mxGetPr(out[4]),
                                 mxGetPr(out[5]), mxGetPr(out[6]), mxGetPr(out[7]),
                                 mxGetPr(out[8]));
    vm_rc(WHO, rc, out, 9);
    vm_publish(nlhs, plhs, out, 9);
}
