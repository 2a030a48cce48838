/*
 * [S e_] = mex_bundle_2_Se_(Y, W, U, eA, eB)
 *
 * Drop-in for toolbox/bundle/mex_bundle_2_Se_.c:15-158 (called at
 * bundle_euclid.m:192 with the damped U_): the reduced camera system
 * S_jk = delta_jk U_j - sum_i Y_ij W_ik', e_j = eA_j - sum_i Y_ij eB_i, on
 * the GPU (vlgba_mex_bundle_2, ordered sums: bit-identical to the reference
 * loops).  m = cols(eA), n = cols(eB), num_a = rows(Y) (:53-57); S is
 * (num_a m) x (num_a m), e_ (num_a m) x 1.
 */
#include "vlgba_mex_util.h"

#define WHO "mex_bundle_2_Se_"

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[])
{
    mxArray *out[2];
    int m, n, na, rc;
    vm_check(WHO, nrhs, prhs, 5, nlhs, 2);
    m = vm_int(mxGetN(prhs[3]), WHO, "m");
    n = vm_int(mxGetN(prhs[4]), WHO, "n");
    na = vm_int(mxGetM(prhs[0]), WHO, "num_a");
    if (na != 6 && na != 7 && na != 10)
        vm_fail(WHO, "rows(Y) must be 6, 7 or 10");
    vm_numel(WHO, prhs[0], (size_t)na * 3 * n * m, "Y");
    vm_numel(WHO, prhs[1], (size_t)na * 3 * n * m, "W");
    vm_numel(WHO, prhs[2], (size_t)na * na * m, "U");
    vm_numel(WHO, prhs[3], (size_t)na * m, "eA");
    vm_numel(WHO, prhs[4], 3 * (size_t)n, "eB");
    out[0] = vm_array(2, (mwSize)na * m, (mwSize)na * m, 1, 1);
    out[1] = vm_array(2, (mwSize)na * m, 1, 1, 1);
    rc = vlgba_mex_bundle_2(m, n, na, mxGetPr(prhs[0]), mxGetPr(prhs[1]), mxGetPr(prhs[2]),
                            mxGetPr(prhs[3]), mxGetPr(prhs[4]), mxGetPr(out[0]), mxGetPr(out[1]));
    vm_rc(WHO, rc, out, 2);
    vm_publish(nlhs, plhs, out, 2);
}
