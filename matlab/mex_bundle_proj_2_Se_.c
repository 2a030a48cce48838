/*
 * [S e_] = mex_bundle_proj_2_Se_(Y, W, U, eA, eB)
 *
 * Drop-in for toolbox/bundle/mex_bundle_proj_2_Se_.c:15-158 (called at
 * bundle_projective.m:164): mex_bundle_2_Se_ with num_a = 12; m = cols(eA),
 * n = cols(eB) (:53-54).  GPU: vlgba_mex_bundle_proj_2 (ordered sums).
 */
#include "vlgba_mex_util.h"

#define WHO "mex_bundle_proj_2_Se_"

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[])
{
    mxArray *out[2];
    const int na = 12;
    int m, n, rc;
    vm_check(WHO, nrhs, prhs, 5, nlhs, 2);
    m = vm_int(mxGetN(prhs[3]), WHO, "m");
    n = vm_int(mxGetN(prhs[4]), WHO, "n");
    vm_numel(WHO, prhs[0], (size_t)na * 3 * n * m, "Y");
    vm_numel(WHO, prhs[1], (size_t)na * 3 * n * m, "W");
    vm_numel(WHO, prhs[2], (size_t)na * na * m, "U");
    vm_numel(WHO, prhs[3], (size_t)na * m, "eA");
    vm_numel(WHO, prhs[4], 3 * (size_t)n, "eB");
    out[0] = vm_array(2, (mwSize)na * m, (mwSize)na * m, 1, 1);
    out[1] = vm_array(2, (mwSize)na * m, 1, 1, 1);
    rc = vlgba_mex_bundle_proj_2(m, n, mxGetPr(prhs[0]), mxGetPr(prhs[1]), mxGetPr(prhs[2]),
                                 mxGetPr(prhs[3]), mxGetPr(prhs[4]), mxGetPr(out[0]),
                                 mxGetPr(out[1]));
    vm_rc(WHO, rc, out, 2);
    vm_publish(nlhs, plhs, out, 2);
}
