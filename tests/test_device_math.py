"""Host build of the product's device math (bundleadjustmentmatlab_amd/csrc/
vlg_math.h + vlg_libm.h) checked against the host libm and exact arithmetic.

The reference's rotations are VLFeat's vl_rodrigues linked against the host
libm, and the forward differences with h = 1e-10
(mex_bundle_1_XABeUVWeAeB.c:23) turn a one-ulp rotation difference into a
~1e-6 Jacobian difference, so the GPU must reproduce libm's sin / cos bit for
bit.  vlg_libm.h restates glibc 2.35's s_sin.c (FMA variant); these tests check
it on >10^7 arguments covering every branch and every table row, plus the
rotations themselves.  tests/test_gpu_parity.py checks the device build.
"""
import ctypes
import math
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
_dp = ctypes.POINTER(ctypes.c_double)


@pytest.fixture(scope="module")
def tm(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("tm") / "libtm.so")
    subprocess.run(["gcc", "-std=c99", "-O2", "-ffp-contract=off", "-fno-builtin-sin", "-fno-builtin-cos",
                    "-fPIC", "-shared",
                    "-o", out, os.path.join(HERE, "native", "math_host.c"), "-lm"], check=True)
    L = ctypes.CDLL(out)
    L.tm_sincos_mismatch.restype = ctypes.c_longlong
    L.tm_sincos_random.restype = ctypes.c_longlong
    L.tm_sincos_random.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_longlong,
                                   ctypes.c_ulonglong]
    L.tm_rodrigues_mismatch.restype = ctypes.c_longlong
    return L


def _P(a):
    return a.ctypes.data_as(_dp)


@pytest.mark.parametrize("lo,hi", [(0.0, 2.0 ** -26), (2.0 ** -26, 0.126), (0.126, 0.855469),
                                   (0.855469, 2.426265), (2.426265, 10.0), (10.0, 1e4),
                                   (1e4, 1e8), (0.0, 3.2)])
def test_sincos_random_ranges(tm, lo, hi):
    """Uniform arguments in each branch of glibc's __sin / __cos."""
    n = 1_500_000
    assert tm.tm_sincos_random(lo, hi, n, int(lo * 1000) + 7) == 0


def test_sincos_edges(tm):
    """Branch thresholds, table rows i/128 (+-1..64 ulp), pi/2 multiples."""
    xs = []
    for t in [2.0 ** -27, 2.0 ** -26, 0.126, 0.855469, 2.426265, 105414350.0]:
        xs.append(t + np.arange(-200, 201) * np.spacing(t))
    rows = np.arange(0, 110) / 128.0
    for k in range(-64, 65):
        xs.append(rows + k * np.spacing(np.maximum(rows, 1e-300)))
    for q in range(1, 400):
        c = q * math.pi / 2
        xs.append(c + np.arange(-50, 51) * np.spacing(c))
    x = np.abs(np.concatenate(xs))
    lim = np.array([0x419921FB00000000], dtype=np.uint64).view(np.float64)[0]
    x = x[x < lim]          # glibc's multi-precision reduction range is out of scope
    x = np.ascontiguousarray(np.concatenate([x, -x]))
    bad = np.zeros(16)
    nb = tm.tm_sincos_mismatch(_P(x), ctypes.c_longlong(x.size), _P(bad), ctypes.c_longlong(16))
    assert nb == 0, bad[:nb]


def test_rodrigues_rotations(tm):
    """vlg_rodrigues == the App. B formula with libm, incl. the FD-perturbed
    vectors w + h e_k the linearisation uses (mex_bundle_1 :30-33)."""
    rng = np.random.default_rng(5)
    w = rng.normal(0, 1, (200_000, 3)) * rng.choice([1e-7, 1e-4, 1e-2, 0.3, 1.0, 2.5],
                                                    (200_000, 1))
    ws = [w]
    for k in range(3):
        wk = w.copy()
        wk[:, k] = wk[:, k] + 1e-10 * 1.0
        ws.append(wk)
    om = np.ascontiguousarray(np.concatenate(ws))
    assert tm.tm_rodrigues_mismatch(_P(om), ctypes.c_longlong(len(om))) == 0


def test_fd_quotient(tm):
    """The device's division-free FD quotient vlg_fd_quot(d) (vlg_math.h) equals
    d / h bit for bit.  Markstein's condition is checked exactly: y = RN(1/h)
    satisfies |y h - 1| <= 2^-54, so q = RN(d y) is within one ulp of d / h and
    the FMA remainder correction is correctly rounded; then ~5e6 operands over
    every binade FD differences occupy (and the guarded edges) are compared."""
    from fractions import Fraction
    h = 1e-10
    y = 1.0 / h
    assert abs(Fraction(y) * Fraction(h) - 1) <= Fraction(1, 2 ** 54)
    rng = np.random.default_rng(0)
    parts = []
    for e in range(-80, 40):      # |x1 - x0| from 2^-80 (tiny FD noise) to 2^40
        sig = rng.uniform(1.0, 2.0, 40_000)
        parts.append(np.ldexp(sig, e) * rng.choice([-1.0, 1.0], sig.size))
    parts.append(np.ldexp(1.0 + np.arange(1, 20_001) * 2.0 ** -52, -20))   # near powers of 2
    parts.append(np.ldexp(2.0 - np.arange(1, 20_001) * 2.0 ** -52, -20))
    parts.append(np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -5e-324, 1e-300,
                           2.0 ** -900, -(2.0 ** -900), 2.0 ** 900, 1e300]))
    d = np.ascontiguousarray(np.concatenate(parts))
    out = np.empty_like(d)
    tm.tm_fd_quot(_P(d), _P(out), ctypes.c_longlong(d.size))
    with np.errstate(all="ignore"):
        ref = d / h
    same = (out.view(np.int64) == ref.view(np.int64)) | (np.isnan(out) & np.isnan(ref))
    assert same.all(), d[~same][:5]
