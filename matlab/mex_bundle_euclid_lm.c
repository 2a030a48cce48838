/*
 * [a_new b_new error_] = mex_bundle_euclid_lm(K, a, b, X, visible, options)
 *
 * The fused gateway behind the drop-in matlab/bundle_euclid.m: the whole
 * Levenberg-Marquardt loop of toolbox/bundle/bundle_euclid.m:111-249 (its three
 * MEX calls :139,192,204, the MATLAB-side damping / pinv / Y of :162-193 and
 * the accept / reject rule :205-241) on the GPU, one call per solve.  a is the
 * packed [w; T; (K)] (num_a x m, :88-96), b = Xe(1:3,:) (3 x n, :99), X =
 * x(1:2,:,:) (:102), visible n x m (double, :81).  Returns the final a and b
 * and error_ (1 x k, SSE / num_vis per accepted step, :219-231).  options:
 * see vlgba_mex_lm.h.
 */
#include "vlgba_mex_lm.h"

#define WHO "mex_bundle_euclid_lm"

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[])
{
    mxArray *out[3];
    int m, na;
    if (nrhs != 5 && nrhs != 6)
        vm_fail(WHO, "5 or 6 inputs required");
    vm_check(WHO, 5, prhs, 5, nlhs, 3);
    m = vm_int(mxGetN(prhs[1]), WHO, "m");
    na = vm_int(mxGetM(prhs[1]), WHO, "num_a");
    if (na != 6 && na != 7 && na != 10)
        vm_fail(WHO, "rows(a) must be 6, 7 or 10");
    vm_numel(WHO, prhs[0], 4 * (size_t)m, "K");
    vm_lm(WHO, VLGBA_MODEL_EUCLIDEAN, mxGetPr(prhs[0]), prhs[1], prhs[2], prhs[3], prhs[4],
          nrhs == 6 ? prhs[5] : NULL, out);
    vm_publish(nlhs, plhs, out, 3);
}
