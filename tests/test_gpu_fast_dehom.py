"""The linearisation's division-free quotients (ba_kernels.hip: dehom_fast,
fd_quot_fast, the redo list and k_linearize_redo).

The fast path (NA = 6) forms x0 / x2 and x1 / x2 of every projection with one
shared reciprocal and the FD quotient (x1 - x0) / h without its range branch.
Inside their operand windows both equal IEEE division bit for bit; a chunk
with an operand outside is linearised again with '/'.  Checked here:
  * the quotients against '/' on random and edge operands (zeros of either
    sign, denormals, the window's edges, huge, inf, NaN), and the window flags;
  * whole passes and LM runs with the fast quotients (VLGBA_FAST_DEHOM=1), with
    '/' everywhere (the default) and with every chunk redone
    (VLGBA_DEBUG_REDO=1): the same reduced system, step and trajectory bit for
    bit.
The fast quotients are opt-in: 15 % fewer instructions, but the fused
linearisation ran 6 % slower with them on MI355X (333 vs 314 us at config 3,
profiles/r05g_*), so the default keeps '/' (DESIGN.md sec. 5).
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _dehom(L, xn):
    xn = np.ascontiguousarray(xn, dtype=np.float64)
    n = xn.shape[0]
    fast = np.zeros((n, 4))
    ref = np.zeros((n, 4))
    win = np.zeros(n, dtype=np.int32)
    dp = ctypes.POINTER(ctypes.c_double)
    rc = L.vlgba_debug_dehom(xn.ctypes.data_as(dp), fast.ctypes.data_as(dp),
                             ref.ctypes.data_as(dp),
                             win.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), n)
    assert rc == 0
    return fast, ref, win


def _bits(x):
    return x.view(np.int64)


def test_quotients_match_division(gpu):
    from bundleadjustmentmatlab_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(5)
    n = 1 << 20
    # image-like operands: homogeneous coordinates and depths over many decades
    mag = 10.0 ** rng.uniform(-8, 8, size=(n, 3))
    xn = mag * rng.choice([-1.0, 1.0], size=(n, 3))
    # FD-like differences: a few ulps to 1e-4, and exact zeros
    xn[: n // 4, 0:2] = rng.normal(size=(n // 4, 2)) * 10.0 ** rng.uniform(-14, -4, (n // 4, 2))
    xn[n // 4: n // 4 + 1000, 0] = 0.0
    xn[n // 4 + 1000: n // 4 + 2000, 1] = -0.0
    fast, ref, win = _dehom(L, xn)
    q = (win & 1) == 1
    d = (win & 2) == 2
    assert q.mean() > 0.99 and d.mean() > 0.99, (q.mean(), d.mean())
    assert np.array_equal(_bits(fast[q, 0:2]), _bits(ref[q, 0:2]))
    assert np.array_equal(_bits(fast[d, 2:4]), _bits(ref[d, 2:4]))
    # zeros of either sign are inside the FD window and keep their sign
    z = np.arange(n // 4, n // 4 + 1000)
    assert d[z].all() and np.array_equal(_bits(fast[z, 2]), _bits(ref[z, 2]))
    z = np.arange(n // 4 + 1000, n // 4 + 2000)
    assert d[z].all() and np.array_equal(_bits(fast[z, 3]), _bits(ref[z, 3]))
    assert np.signbit(fast[z, 3]).all()


def test_window_edges(gpu):
    from bundleadjustmentmatlab_amd import _lib
    L = _lib.lib()
    lo, hi = 2.0 ** -300, 2.0 ** 301
    tiny, inside = np.nextafter(lo, 0.0), np.nextafter(hi, 0.0)
    # (x0, x1, x2) -> bit 0: quotients vouched for, bit 1: FD quotients of x0, x1
    cases = [
        ([1.0, 2.0, 3.0], 3),
        ([lo, -lo, lo], 3),                 # the window's lower edge
        ([inside, -inside, inside], 3),     # the largest value inside
        ([tiny, 1.0, 1.0], 0),              # just below: outside both
        ([1.0, 1.0, hi], 2),                # the denominator just above
        ([0.0, 1.0, 2.0], 2),               # zero numerator: redone; FD exact
        ([-0.0, 1.0, 2.0], 2),
        ([1.0, 1.0, 0.0], 2),               # zero denominator
        ([5e-324, 1.0, 1.0], 0),            # denormal
        ([np.inf, 1.0, 1.0], 0),
        ([np.nan, 1.0, 1.0], 0),
        ([1e300, 1.0, 1.0], 0),
    ]
    xn = np.array([c[0] for c in cases])
    fast, ref, win = _dehom(L, xn)
    expect = [c[1] for c in cases]
    assert list(win) == expect, (list(win), expect)
    for k in range(len(cases)):
        if win[k] & 1:
            assert np.array_equal(_bits(fast[k, 0:2]), _bits(ref[k, 0:2])), k
        if win[k] & 2:
            assert np.array_equal(_bits(fast[k, 2:4]), _bits(ref[k, 2:4])), k


def _scene():
    from bundleadjustmentmatlab_amd.scene import make_config
    return make_config("cfg2", m=24, n=2000, seed=11)


def _one_pass(gpu, sc):
    a = np.zeros((6, sc.m), order="F")
    a[0:3], a[3:6] = sc.w0, sc.T0
    b = np.asfortranarray(sc.X0[:3])
    with gpu.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, 6) as ba:
        ba.set_params(a, b)
        S, e = ba.reduced_system(dense=True)
        info = ba.step(relinearize=False, update_lm=False)
        da, db = ba.last_step()
        return S.copy(), e.copy(), da.copy(), db.copy(), info.old_sse, info.new_sse


def _run(gpu, sc):
    a = np.zeros((6, sc.m), order="F")
    a[0:3], a[3:6] = sc.w0, sc.T0
    b = np.asfortranarray(sc.X0[:3])
    with gpu.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, 6,
                            stop_rel=1e-9, max_iter=12) as ba:
        ba.set_params(a, b)
        err, st = ba.run()
        return err.copy(), [x.copy() for x in ba.get_params()]


@pytest.mark.parametrize("mode", ["fast", "redo_all"])
def test_pass_bit_identical(gpu, monkeypatch, mode):
    sc = _scene()
    base = _one_pass(gpu, sc)
    monkeypatch.setenv("VLGBA_FAST_DEHOM", "1")
    if mode == "redo_all":
        monkeypatch.setenv("VLGBA_DEBUG_REDO", "1")
    other = _one_pass(gpu, sc)
    for x, y in zip(base, other):
        assert np.array_equal(np.asarray(x), np.asarray(y))


@pytest.mark.parametrize("fused", ["1", "0"])
def test_lm_run_bit_identical(gpu, monkeypatch, fused):
    sc = _scene()
    monkeypatch.setenv("VLGBA_FUSED", fused)
    e0, p0 = _run(gpu, sc)
    monkeypatch.setenv("VLGBA_FAST_DEHOM", "1")
    e1, p1 = _run(gpu, sc)
    monkeypatch.setenv("VLGBA_DEBUG_REDO", "1")
    e2, p2 = _run(gpu, sc)
    assert len(e0) >= 3
    assert np.array_equal(e0, e1) and np.array_equal(e0, e2)
    for x, y, z in zip(p0, p1, p2):
        assert np.array_equal(x, y) and np.array_equal(x, z)
