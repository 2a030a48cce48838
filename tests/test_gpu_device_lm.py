"""The LM loop with its decisions on the device (vlgba_run on the fast path).

k_lm_decide takes every pass's accept / lambda / error_ / stop decision
(bundle_euclid.m:205-241, bundle_projective.m:182-207, the stop test of
:111-123) and the pass kernels read lambda, "relinearise or not" and the
current parameter buffers from that device state, so the host enqueues passes
one ahead instead of waiting for each pass's scalars (opt-in:
VLGBA_DEVICE_LM=1, read when the context is created).  Checked against the
host-decided loop (VLGBA_DEVICE_LM=0): the
same passes, accepts, error_ and parameters -- the only arithmetic that may
differ is (2 rho - 1)^3 (a double-double cube on the device, glibc pow on the
host), so the comparison allows the rounding that 1-ulp lambda difference
could propagate.  A non-positive pivot hands the pass to the host (pinv step).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _solve(gpu, sc, num_a, device_lm, run=True, **kw):
    old = os.environ.get("VLGBA_DEVICE_LM")
    os.environ["VLGBA_DEVICE_LM"] = "1" if device_lm else "0"
    try:
        if kw.get("model") == "projective":
            from bundleadjustmentmatlab_amd.scene import projective_from
            Pp, Xp = projective_from(sc)
            a = np.asfortranarray(Pp.reshape(12, sc.m, order="F"))
            b = np.asfortranarray(Xp[0:3])
            K = None
            kw = dict(kw, m=sc.m)
        else:
            a = np.zeros((num_a, sc.m), order="F")
            a[0:3], a[3:6] = sc.w0, sc.T0
            if num_a == 7:
                a[6] = sc.K[0]
            elif num_a == 10:
                a[6:10] = sc.K
            b = np.asfortranarray(sc.X0[:3])
            K = sc.K
        with gpu.BundleAdjuster(K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, num_a, **kw) as ba:
            ba.set_params(a, b)
            if run:
                err, st = ba.run()
                a1, b1 = ba.get_params()
                return (np.array(err, copy=True), st.iterations, st.accepted, st.lambda_,
                        a1.copy(), b1.copy())
            return ba
    finally:
        if old is None:
            del os.environ["VLGBA_DEVICE_LM"]
        else:
            os.environ["VLGBA_DEVICE_LM"] = old


def _close(x, y, rtol):
    return np.abs(x - y).max() <= rtol * max(np.abs(y).max(), 1e-300)


@pytest.mark.parametrize("num_a,kw", [(6, {}), (7, {}), (10, {}), (12, {"model": "projective"}),
                                      (6, {"stop_rel": 1e-9, "max_iter": 40}),
                                      (6, {"pivot_first": 2})])
def test_device_lm_matches_host_loop(gpu, num_a, kw):
    from bundleadjustmentmatlab_amd.scene import make_config
    sc = make_config("cfg2", m=40, n=4000, seed=71 + num_a)
    kw = dict(kw)
    if kw.pop("pivot_first", 0):
        kw["pivot"] = np.arange(sc.m) < 2
    d = _solve(gpu, sc, num_a, True, **kw)
    h = _solve(gpu, sc, num_a, False, **kw)
    (de, dn, dacc, dlam, da, db), (he, hn, hacc, hlam, ha, hb) = d, h
    assert dn == hn and dacc == hacc and len(de) == len(he) and dn > 2
    assert _close(de, he, 1e-12), (de, he)
    assert abs(dlam - hlam) <= 1e-12 * abs(hlam)
    assert _close(da, ha, 1e-9) and _close(db, hb, 1e-9)


def test_device_lm_pinv_handoff(gpu):
    """lambda0 = 1e-10: the first pass's Cholesky meets a non-positive pivot
    (test_gpu_lm_parity.py::test_pinv_fallback_takes_the_step); the device
    loop stops without committing and the host takes that pass's pinv step and
    the rest of the solve: the result is the host loop's, bit for bit."""
    from bundleadjustmentmatlab_amd.scene import make_config
    sc = make_config("cfg1")
    x, vis = sc.dense()
    pt, cam = np.nonzero(vis)
    obs_x = np.stack([x[0, pt, cam], x[1, pt, cam]], 1)
    a = np.vstack([sc.w0, sc.T0])
    b = np.asfortranarray(sc.X0[:3])
    out = []
    for dev in (True, False):
        old = os.environ.get("VLGBA_DEVICE_LM")
        os.environ["VLGBA_DEVICE_LM"] = "1" if dev else "0"
        try:
            with gpu.BundleAdjuster(sc.K, pt, cam, obs_x, sc.n, 6, lambda0=1e-10) as ba:
                ba.set_params(a, b)
                err, st = ba.run()
                a1, b1 = ba.get_params()
                out.append((err.copy(), st.iterations, a1.copy(), b1.copy()))
        finally:
            if old is None:
                del os.environ["VLGBA_DEVICE_LM"]
            else:
                os.environ["VLGBA_DEVICE_LM"] = old
    (de, dn, da, db), (he, hn, ha, hb) = out
    assert dn == hn
    assert np.array_equal(de, he)
    assert np.array_equal(da, ha) and np.array_equal(db, hb)


def test_passes_equal_host_steps(gpu, monkeypatch):
    """vlgba_run_passes (K relinearising passes enqueued back to back, the
    decisions on the device, nothing committed) = K host-decided
    vlgba_step(relinearize=1, update_lm=0): the same last-pass scalars bit for
    bit, and the parameters unchanged."""
    from bundleadjustmentmatlab_amd.scene import make_config
    monkeypatch.setenv("VLGBA_DEVICE_LM", "1")
    sc = make_config("cfg2", m=60, n=6000, seed=5)
    a = np.zeros((6, sc.m), order="F")
    a[0:3], a[3:6] = sc.w0, sc.T0
    b = np.asfortranarray(sc.X0[:3])
    with gpu.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, 6) as ba:
        ba.set_params(a, b)
        for _ in range(3):
            hs = ba.step(relinearize=True, update_lm=False)
        ds = ba.passes(5)
        a1, b1 = ba.get_params()
        hs2 = ba.step(relinearize=True, update_lm=False)
    assert ds.old_sse == hs.old_sse and ds.new_sse == hs.new_sse and ds.dpg == hs.dpg
    assert hs2.old_sse == hs.old_sse and hs2.new_sse == hs.new_sse
    assert np.array_equal(a1, a) and np.array_equal(b1, b)
