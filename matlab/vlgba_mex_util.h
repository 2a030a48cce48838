/*
 * vlgba_mex_util.h -- argument handling shared by the vlgba MEX gateways.
 *
 * The reference gateways check nothing (SURVEY.md sec. 8.b "Errors"): a wrong
 * class or shape is silently misread.  These gateways keep the reference's
 * layouts and the reference's way of deriving m / n / num_a from the inputs,
 * and turn every mismatch into a MATLAB error instead of a wild read.
 */
#ifndef VLGBA_MEX_UTIL_H
#define VLGBA_MEX_UTIL_H

#include "mex.h"
#include "../include/vlgba.h"

#include <stddef.h>

static void vm_fail(const char *who, const char *what)
{
    mexErrMsgIdAndTxt("vlgba:args", "%s: %s", who, what);
}

/* nrhs inputs exactly, at most max_out outputs, every input a real double */
static void vm_check(const char *who, int nrhs, const mxArray *prhs[], int want_in, int nlhs,
                     int max_out)
{
    static int abi_ok = 0;   /* libvlgba built from the header this gateway saw */
    int k;
    if (!abi_ok) {
        if (VLGBA_ABI_CHECK() != 0)
            mexErrMsgIdAndTxt("vlgba:abi", "%s: libvlgba does not match vlgba.h (ABI %d)", who,
                              VLGBA_ABI_VERSION);
        abi_ok = 1;
    }
    if (nrhs != want_in)
        mexErrMsgIdAndTxt("vlgba:args", "%s: %d inputs required", who, want_in);
    if (nlhs > max_out)
        mexErrMsgIdAndTxt("vlgba:args", "%s: at most %d outputs", who, max_out);
    for (k = 0; k < nrhs; k++)
        if (!mxIsDouble(prhs[k]))
            mexErrMsgIdAndTxt("vlgba:args", "%s: input %d must be double", who, k + 1);
}

/* numel(a) == want, else an error naming the argument */
static void vm_numel(const char *who, const mxArray *a, size_t want, const char *name)
{
    if (mxGetNumberOfElements(a) != want)
        mexErrMsgIdAndTxt("vlgba:args", "%s: %s has %zu elements, expected %zu", who, name,
                          (size_t)mxGetNumberOfElements(a), want);
}

static mxArray *vm_array(int nd, mwSize d0, mwSize d1, mwSize d2, mwSize d3)
{
    mwSize d[4];
    mxArray *a;
    d[0] = d0;
    d[1] = d1;
    d[2] = d2;
    d[3] = d3;
    a = mxCreateNumericArray((mwSize)nd, d, mxDOUBLE_CLASS, mxREAL);
    if (!a)
        mexErrMsgIdAndTxt("vlgba:nomem", "out of memory");
    return a;
}

/* hand the first max(nlhs, 1) of nout outputs to MATLAB, free the rest (the
 * reference writes all of them into pout[] whatever nout is) */
static void vm_publish(int nlhs, mxArray *plhs[], mxArray **out, int nout)
{
    int k, keep = nlhs > 0 ? nlhs : 1;
    for (k = 0; k < nout; k++) {
        if (k < keep)
            plhs[k] = out[k];
        else
            mxDestroyArray(out[k]);
    }
}

static void vm_rc(const char *who, int rc, mxArray **out, int nout)
{
    int k;
    if (rc == 0)
        return;
    for (k = 0; k < nout; k++)
        mxDestroyArray(out[k]);
    mexErrMsgIdAndTxt("vlgba:lib", "%s: libvlgba error %d", who, rc);
}

static int vm_int(size_t v, const char *who, const char *name)
{
    if (v > 0x7fffffff)
        mexErrMsgIdAndTxt("vlgba:args", "%s: %s too large", who, name);
    return (int)v;
}

#endif /* VLGBA_MEX_UTIL_H */
