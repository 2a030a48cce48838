/*
 * math_host.c -- host build of the product's device math headers, for the CPU
 * tests only (tests/test_device_math.py compiles it with gcc).  It checks the
 * product code itself: vlg_libm.h sin / cos against the host libm, and
 * vlg_fd_quot against the plain quotient d / h.  The oracle never includes
 * product headers; this file is not part of the oracle.
 */
#include <math.h>
#include "../../bundleadjustmentmatlab_amd/csrc/vlg_math.h"

/* count (and record up to cap) arguments where vlg_lm_sin / vlg_lm_cos differ
 * from the host libm bit for bit */
long long tm_sincos_mismatch(const double *x, long long n, double *bad, long long cap)
{
    long long k, nb = 0;
    for (k = 0; k < n; k++) {
        volatile double xs = x[k];
        const double s0 = sin(xs), c0 = cos(xs);
        const double s1 = vlg_lm_sin(xs), c1 = vlg_lm_cos(xs);
        if (memcmp(&s0, &s1, 8) != 0 || memcmp(&c0, &c1, 8) != 0) {
            if (nb < cap)
                bad[nb] = x[k];
            nb++;
        }
    }
    return nb;
}

/* uniform random arguments in [lo, hi) with random sign, xorshift, n draws */
long long tm_sincos_random(double lo, double hi, long long n, unsigned long long seed)
{
    unsigned long long st = seed * 0x9E3779B97F4A7C15ull + 1;
    long long k, nb = 0;
    for (k = 0; k < n; k++) {
        double x, s0, c0, s1, c1;
        st ^= st << 13;
        st ^= st >> 7;
        st ^= st << 17;
        x = lo + (hi - lo) * ((double)(st >> 11) * 0x1p-53);
        if (st & 1)
            x = -x;
        {
            volatile double xs = x;
            s0 = sin(xs);
            c0 = cos(xs);
            s1 = vlg_lm_sin(xs);
            c1 = vlg_lm_cos(xs);
        }
        nb += memcmp(&s0, &s1, 8) != 0 || memcmp(&c0, &c1, 8) != 0;
    }
    return nb;
}

/* rotations of the product (vlg_rodrigues) vs the oracle formula with libm;
 * returns the number of matrices that differ in any bit */
long long tm_rodrigues_mismatch(const double *om, long long n)
{
    long long k, nb = 0;
    for (k = 0; k < n; k++) {
        double R[9], Q[9];
        const double *w = om + 3 * k;
        const double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
        vlg_rodrigues(R, w);
        if (th < 1e-6) {
            memset(Q, 0, sizeof Q);
            Q[0] = Q[4] = Q[8] = 1.0;
        } else {
            const double x = w[0] / th, y = w[1] / th, z = w[2] / th;
            const double s = sin(th), m = 1.0 - cos(th);
            Q[0] = 1 - m * (y * y + z * z);
            Q[1] = s * z + m * (x * y);
            Q[2] = -s * y + m * (x * z);
            Q[3] = -s * z + m * (x * y);
            Q[4] = 1 - m * (z * z + x * x);
            Q[5] = s * x + m * (y * z);
            Q[6] = s * y + m * (x * z);
            Q[7] = -s * x + m * (y * z);
            Q[8] = 1 - m * (x * x + y * y);
        }
        nb += memcmp(R, Q, sizeof R) != 0;
    }
    return nb;
}

void tm_fd_quot(const double *d, double *out, long long n)
{
    long long k;
    for (k = 0; k < n; k++)
        out[k] = vlg_fd_quot(d[k]);
}
