/*
 * [X_hat A B e U V W eA eB] = mex_bundle_1_XABeUVWeAeB(K, a, b, X, visible)
 *
 * Drop-in for toolbox/bundle/mex_bundle_1_XABeUVWeAeB.c:72-337 (called at
 * bundle_euclid.m:139): projection, forward-difference Jacobians (h = 1e-10)
 * and the JtJ blocks, computed on the GPU by vlgba_mex_bundle_1.  Inputs /
 * outputs exactly as the reference: K 4xm, a num_a x m (num_a = rows(a),
 * :131), b 3xn, X 2xnxm, visible nxm (m = cols(a), n = cols(b),
 * :127-128); outputs X_hat 2xnxm, A 2 x num_a x n x m, B 2x3xnxm, e 2xnxm,
 * U num_a x num_a x m, V 3x3xn, W num_a x 3 x n x m, eA num_a x m, eB 3xn.
 */
#include "vlgba_mex_util.h"

#define WHO "mex_bundle_1_XABeUVWeAeB"

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[])
{
    mxArray *out[9];
    int m, n, na, rc;
    vm_check(WHO, nrhs, prhs, 5, nlhs, 9);
    m = vm_int(mxGetN(prhs[1]), WHO, "m");
    n = vm_int(mxGetN(prhs[2]), WHO, "n");
    na = vm_int(mxGetM(prhs[1]), WHO, "num_a");
    if (na != 6 && na != 7 && na != 10)
        vm_fail(WHO, "rows(a) must be 6, 7 or 10");
    vm_numel(WHO, prhs[0], 4 * (size_t)m, "K");
    vm_numel(WHO, prhs[2], 3 * (size_t)n, "b");
    vm_numel(WHO, prhs[3], 2 * (size_t)n * m, "X");
    vm_numel(WHO, prhs[4], (size_t)n * m, "visible");
    out[0] = vm_array(3, 2, n, m, 1);
    out[1] = vm_array(4, 2, na, n, m);
    out[2] = vm_array(4, 2, 3, n, m);
    out[3] = vm_array(3, 2, n, m, 1);
    out[4] = vm_array(3, na, na, m, 1);
    out[5] = vm_array(3, 3, 3, n, 1);
    out[6] = vm_array(4, na, 3, n, m);
    out[7] = vm_array(2, na, m, 1, 1);
    out[8] = vm_array(2, 3, n, 1, 1);
    rc = vlgba_mex_bundle_1(m, n, na, mxGetPr(prhs[0]), mxGetPr(prhs[1]), mxGetPr(prhs[2]),
                            mxGetPr(prhs[3]), mxGetPr(prhs[4]), mxGetPr(out[0]),
                            mxGetPr(out[1]), mxGetPr(out[2]), mxGetPr(out[3]), mxGetPr(out[4]),
                            mxGetPr(out[5]), mxGetPr(out[6]), mxGetPr(out[7]), mxGetPr(out[8]));
    vm_rc(WHO, rc, out, 9);
    vm_publish(nlhs, plhs, out, 9);
}
