/*
 * [a_new b_new error_] = mex_bundle_projective_lm(a, b, X, visible, options)
 *
 * The fused gateway behind the drop-in matlab/bundle_projective.m: the LM loop
 * of toolbox/bundle/bundle_projective.m:86-215 (MEX calls :116,164,177; errors
 * compared after scaling by 1/num_vis, lambda / 10 on accept and * 10 on
 * reject, :182-207) on the GPU.  a = P(:) per camera (12 x m, :70-73), b =
 * Xp(1:3,:) (:76), X 2 x n x m, visible n x m.  options: see vlgba_mex_lm.h
 * (pivot is not an option of bundle_projective.m and is ignored).
 */
#include "vlgba_mex_lm.h"

#define WHO "mex_bundle_projective_lm"

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[])
{
    mxArray *out[3];
    if (nrhs != 4 && nrhs != 5)
        vm_fail(WHO, "4 or 5 inputs required");
    vm_check(WHO, 4, prhs, 4, nlhs, 3);
    if (mxGetM(prhs[0]) != 12)
        vm_fail(WHO, "a must be 12 x m (P(:))");
    vm_lm(WHO, VLGBA_MODEL_PROJECTIVE, NULL, prhs[0], prhs[1], prhs[2], prhs[3],
          nrhs == 5 ? prhs[4] : NULL, out);
    vm_publish(nlhs, plhs, out, 3);
}
