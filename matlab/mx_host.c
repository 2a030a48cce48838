/*
 * mx_host.c -- minimal mx / mex runtime (libvlgmx.so) for hosts without MATLAB.
 *
 * Implements the subset of MATLAB's mx API declared in mex.h so that the vlgba
 * MEX gateways (matlab/mex_*.c) can be loaded and called from C or Python:
 * double arrays (any rank, zero-filled on creation like mxCreate*), 1x1
 * structs with named fields (the option struct of the fused gateways), error
 * reporting by longjmp back to mxhost_call (MATLAB's mexErrMsgIdAndTxt does not
 * return either).  Under MATLAB none of this is used: libmx / libmex provide
 * the same symbols.
 */
#define _POSIX_C_SOURCE 200809L   /* strdup */
#include "mex.h"

#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define MX_MAXDIM 8
#define MX_MAXFIELD 32

struct mxArray_tag {
    mxClassID cls;
    mwSize nd;
    mwSize dims[MX_MAXDIM];
    double *pr;
    int nfield;
    char *fname[MX_MAXFIELD];
    mxArray *fval[MX_MAXFIELD];
};

static size_t numel(const mxArray *a)
{
    size_t k, n = 1;
    for (k = 0; k < a->nd; k++)
        n *= a->dims[k];
    return n;
}

double *mxGetPr(const mxArray *pa) { return pa ? pa->pr : NULL; }
size_t mxGetM(const mxArray *pa) { return pa && pa->nd ? pa->dims[0] : 0; }
size_t mxGetN(const mxArray *pa)
{
    size_t k, n = 1;
    if (!pa || pa->nd < 2)
        return pa && pa->nd == 1 ? 1 : 0;
    for (k = 1; k < pa->nd; k++)
        n *= pa->dims[k];
    return n;
}
mwSize mxGetNumberOfDimensions(const mxArray *pa) { return pa ? pa->nd : 0; }
const mwSize *mxGetDimensions(const mxArray *pa) { return pa ? pa->dims : NULL; }
size_t mxGetNumberOfElements(const mxArray *pa) { return pa ? numel(pa) : 0; }
mxClassID mxGetClassID(const mxArray *pa) { return pa ? pa->cls : mxUNKNOWN_CLASS; }
int mxIsDouble(const mxArray *pa) { return pa && pa->cls == mxDOUBLE_CLASS; }
int mxIsStruct(const mxArray *pa) { return pa && pa->cls == mxSTRUCT_CLASS; }
int mxIsEmpty(const mxArray *pa) { return !pa || numel(pa) == 0; }
double mxGetScalar(const mxArray *pa)
{
    return (pa && pa->cls == mxDOUBLE_CLASS && pa->pr && numel(pa) > 0) ? pa->pr[0] : 0.0;
}

mxArray *mxGetField(const mxArray *pa, mwIndex i, const char *fieldname)
{
    int k;
    if (!pa || pa->cls != mxSTRUCT_CLASS || i != 0 || !fieldname)
        return NULL;
    for (k = 0; k < pa->nfield; k++)
        if (strcmp(pa->fname[k], fieldname) == 0)
            return pa->fval[k];
    return NULL;
}

mxArray *mxCreateNumericArray(mwSize ndim, const mwSize *dims, mxClassID classid,
                              mxComplexity flag)
{
    mxArray *a;
    size_t k, n;
    if (classid != mxDOUBLE_CLASS || flag != mxREAL || ndim > MX_MAXDIM)
        return NULL;
    a = (mxArray *)calloc(1, sizeof *a);
    if (!a)
        return NULL;
    a->cls = mxDOUBLE_CLASS;
    a->nd = ndim < 2 ? 2 : ndim;
    a->dims[0] = a->dims[1] = 1;
    for (k = 0; k < ndim; k++)
        a->dims[k] = dims[k];
    if (ndim == 1)
        a->dims[1] = 1;
    n = numel(a);
    a->pr = (double *)calloc(n ? n : 1, sizeof(double));   /* zero-filled, as MATLAB's */
    if (!a->pr) {
        free(a);
        return NULL;
    }
    return a;
}

mxArray *mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity flag)
{
    mwSize d[2];
    d[0] = m;
    d[1] = n;
    return mxCreateNumericArray(2, d, mxDOUBLE_CLASS, flag);
}

void mxDestroyArray(mxArray *pa)
{
    int k;
    if (!pa)
        return;
    for (k = 0; k < pa->nfield; k++) {
        free(pa->fname[k]);
        mxDestroyArray(pa->fval[k]);
    }
    free(pa->pr);
    free(pa);
}

/* ---- errors: mexErrMsgIdAndTxt jumps back to the active mxhost_call -------- */
static __thread jmp_buf *g_jmp;
static __thread char g_err[512];

void mexErrMsgIdAndTxt(const char *errorid, const char *errormsg, ...)
{
    va_list ap;
    int k = snprintf(g_err, sizeof g_err, "%s: ", errorid ? errorid : "");
    if (k < 0 || k >= (int)sizeof g_err)
        k = 0;
    va_start(ap, errormsg);
    vsnprintf(g_err + k, sizeof g_err - (size_t)k, errormsg, ap);
    va_end(ap);
    if (g_jmp)
        longjmp(*g_jmp, 1);
    fprintf(stderr, "%s\n", g_err);
    abort();
}

int mexPrintf(const char *fmt, ...)
{
    va_list ap;
    int r;
    va_start(ap, fmt);
    r = vprintf(fmt, ap);
    va_end(ap);
    fflush(stdout);
    return r;
}

/* ---- host-side helpers (not part of MATLAB's API) -------------------------- */
typedef void (*mxhost_gateway)(int, mxArray **, int, const mxArray **);

/* call a gateway; 0 on success, 1 if it raised (message in errbuf) */
int mxhost_call(mxhost_gateway fn, int nlhs, mxArray **plhs, int nrhs, const mxArray **prhs,
                char *errbuf, int errlen)
{
    jmp_buf jb;
    jmp_buf *prev = g_jmp;
    volatile int rc = 0;
    g_err[0] = 0;
    g_jmp = &jb;
    if (setjmp(jb) == 0)
        fn(nlhs, plhs, nrhs, prhs);
    else
        rc = 1;
    g_jmp = prev;
    if (errbuf && errlen > 0) {
        strncpy(errbuf, g_err, (size_t)errlen - 1);
        errbuf[errlen - 1] = 0;
    }
    return rc;
}

/* a double array with the given dims, copied from data (column major) or zero */
mxArray *mxhost_double(int ndim, const long long *dims, const double *data)
{
    mwSize d[MX_MAXDIM];
    int k;
    mxArray *a;
    if (ndim < 0 || ndim > MX_MAXDIM)
        return NULL;
    for (k = 0; k < ndim; k++)
        d[k] = (mwSize)dims[k];
    a = mxCreateNumericArray((mwSize)ndim, d, mxDOUBLE_CLASS, mxREAL);
    if (a && data)
        memcpy(a->pr, data, sizeof(double) * numel(a));
    return a;
}

/* an empty 1x1 struct; fields added by mxhost_set_field (takes ownership) */
mxArray *mxhost_struct(void)
{
    mxArray *a = (mxArray *)calloc(1, sizeof *a);
    if (!a)
        return NULL;
    a->cls = mxSTRUCT_CLASS;
    a->nd = 2;
    a->dims[0] = a->dims[1] = 1;
    return a;
}

int mxhost_set_field(mxArray *s, const char *name, mxArray *val)
{
    int k;
    if (!s || s->cls != mxSTRUCT_CLASS || !name)
        return -1;
    for (k = 0; k < s->nfield; k++)
        if (strcmp(s->fname[k], name) == 0) {
            mxDestroyArray(s->fval[k]);
            s->fval[k] = val;
            return 0;
        }
    if (s->nfield >= MX_MAXFIELD)
        return -1;
    s->fname[s->nfield] = strdup(name);
    s->fval[s->nfield] = val;
    s->nfield++;
    return 0;
}

/* dims of a (up to 8), returns the rank */
int mxhost_dims(const mxArray *a, long long *dims)
{
    mwSize k;
    if (!a)
        return -1;
    for (k = 0; k < a->nd; k++)
        dims[k] = (long long)a->dims[k];
    return (int)a->nd;
}
