/*
 * mex.h -- the subset of MATLAB's MEX / mx C API the vlgba gateways use.
 *
 * Product code of this repository (not MATLAB's header): it declares the same
 * functions with the same signatures as MATLAB's <mex.h> / <matrix.h> for the
 * calls the gateways make, so the gateway sources compile unchanged either
 *   - with MATLAB's `mex` (MATLAB's own headers and libmx / libmex win), or
 *   - against this header and mx_host.c, the repository's minimal mx runtime
 *     (libvlgmx.so) for hosts without MATLAB and for the tests.
 * The reference gateways reach the same API through VLFeat's <mexutils.h>
 * (toolbox/bundle/mex_bundle_1_XABeUVWeAeB.c:9).
 *
 * Semantics kept from MATLAB: arrays are column major doubles; mxGetN is the
 * product of all dimensions but the first; mxCreate* return ZERO-filled arrays
 * (the reference's mex_bundle_1 accumulates into them); mexErrMsgIdAndTxt does
 * not return (mx_host.c longjmps back to mxhost_call).
 */
#ifndef VLG_MEX_H
#define VLG_MEX_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef size_t mwSize;
typedef size_t mwIndex;
typedef struct mxArray_tag mxArray;

typedef enum { mxREAL = 0, mxCOMPLEX = 1 } mxComplexity;
/* numbering as MATLAB's matrix.h */
typedef enum {
    mxUNKNOWN_CLASS = 0,
    mxCELL_CLASS,
    mxSTRUCT_CLASS,
    mxLOGICAL_CLASS,
    mxCHAR_CLASS,
    mxVOID_CLASS,
    mxDOUBLE_CLASS,
    mxSINGLE_CLASS
} mxClassID;

double *mxGetPr(const mxArray *pa);
size_t mxGetM(const mxArray *pa);
size_t mxGetN(const mxArray *pa);
mwSize mxGetNumberOfDimensions(const mxArray *pa);
const mwSize *mxGetDimensions(const mxArray *pa);
size_t mxGetNumberOfElements(const mxArray *pa);
mxClassID mxGetClassID(const mxArray *pa);
int mxIsDouble(const mxArray *pa);
int mxIsStruct(const mxArray *pa);
int mxIsEmpty(const mxArray *pa);
double mxGetScalar(const mxArray *pa);
mxArray *mxGetField(const mxArray *pa, mwIndex i, const char *fieldname);
mxArray *mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity flag);
mxArray *mxCreateNumericArray(mwSize ndim, const mwSize *dims, mxClassID classid,
                              mxComplexity flag);
void mxDestroyArray(mxArray *pa);

void mexErrMsgIdAndTxt(const char *errorid, const char *errormsg, ...);
int mexPrintf(const char *fmt, ...);

/* the gateway entry point every MEX file exports */
void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]);

#ifdef __cplusplus
}
#endif
#endif /* VLG_MEX_H */
