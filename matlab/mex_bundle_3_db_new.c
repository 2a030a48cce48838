/*
 * [db a_new b_new X_hat] = mex_bundle_3_db_new(W, da, eB, V_inv, K, a, b, X, visible)
 *
 * Drop-in for toolbox/bundle/mex_bundle_3_db_new.c:12-170 (called at
 * bundle_euclid.m:204): back substitution db_i = V_inv_i (eB_i - sum_j
 * W_ij(1:6,:)' da_j(1:6)) (:99-134, the six-term sum of :113-120 kept, App. A
 * Q3), a_new = a + da (:137-140), b_new = b + db (:143-146), X_hat of the
 * visible pairs, X elsewhere (:149-166); on the GPU (vlgba_mex_bundle_3).
 * m = cols(a), n = cols(b), num_a = rows(W) (:60-64).
 */
#include "vlgba_mex_util.h"

#define WHO "mex_bundle_3_db_new"

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[])
{
    mxArray *out[4];
    int m, n, na, rc;
    vm_check(WHO, nrhs, prhs, 9, nlhs, 4);
    m = vm_int(mxGetN(prhs[5]), WHO, "m");
    n = vm_int(mxGetN(prhs[6]), WHO, "n");
    na = vm_int(mxGetM(prhs[0]), WHO, "num_a");
    if (na != 6 && na != 7 && na != 10)
        vm_fail(WHO, "rows(W) must be 6, 7 or 10");
    vm_numel(WHO, prhs[0], (size_t)na * 3 * n * m, "W");
    vm_numel(WHO, prhs[1], (size_t)na * m, "da");
    vm_numel(WHO, prhs[2], 3 * (size_t)n, "eB");
    vm_numel(WHO, prhs[3], 9 * (size_t)n, "V_inv");
    vm_numel(WHO, prhs[4], 4 * (size_t)m, "K");
    vm_numel(WHO, prhs[5], (size_t)na * m, "a");
    vm_numel(WHO, prhs[7], 2 * (size_t)n * m, "X");
    vm_numel(WHO, prhs[8], (size_t)n * m, "visible");
    out[0] = vm_array(2, 3, n, 1, 1);
    out[1] = vm_array(2, na, m, 1, 1);
    out[2] = vm_array(2, 3, n, 1, 1);
    out[3] = vm_array(3, 2, n, m, 1);
    rc = vlgba_mex_bundle_3(m, n, na, mxGetPr(prhs[0]), mxGetPr(prhs[1]), mxGetPr(prhs[2]),
                            mxGetPr(prhs[3]), mxGetPr(prhs[4]), mxGetPr(prhs[5]),
                            mxGetPr(prhs[6]), mxGetPr(prhs[7]), mxGetPr(prhs[8]),
                            mxGetPr(out[0]), mxGetPr(out[1]), mxGetPr(out[2]), mxGetPr(out[3]));
    vm_rc(WHO, rc, out, 4);
    vm_publish(nlhs, plhs, out, 4);
}
