"""The reduced solve's two status words (ba_internal.h: scal[4] a non-positive
pivot, scal[5] a one-launch solve that gave up waiting on a hand-off).

* A hand-off timeout says nothing about S: the pass is solved again with the
  launches that never wait on other workgroups (ba_chol_solve nospin) and the
  result is the one-launch solve's, bit for bit -- for the cyclic reduction
  (k_cr32_fused -> per-level k_cr32_factor / k_cr32_level / k_cr32_back) and
  for the envelope Cholesky (k_backward_all -> per-column k_backward).  The
  timeout is forced by the test hook VLGBA_DEBUG_SPIN_TIMEOUT="rank:passes".
* With several ranks the status words travel in the pass scalars' all-reduce:
  a timeout on one rank makes every rank re-solve (the re-solve's all-reduce
  pairs up), and the sharded solve ends as without the timeout.
* A non-positive pivot takes da = pinv(S) e_ (bundle_euclid.m:193), counted in
  vlgba_stats.pinv_passes.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _solve(gpu, sc, **kw):
    a = np.vstack([sc.w0, sc.T0])
    b = np.asfortranarray(sc.X0[:3])
    with gpu.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, 6, **kw) as ba:
        ba.set_params(a, b)
        err, st = ba.run()
        a1, b1 = ba.get_params()
        plan = ba.plan_info()
    return err.copy(), st, a1.copy(), b1.copy(), plan


@pytest.mark.parametrize("kind", ["cr", "envelope"])
def test_spin_timeout_resolves_bit_identically(gpu, monkeypatch, kind):
    from bundleadjustmentmatlab_amd.scene import make_config
    if kind == "cr":     # tile-tridiagonal S: the one-launch cyclic reduction
        sc = make_config("cfg2", m=60, n=6000, seed=5)
    else:                # banded + loop-closure border: envelope Cholesky
        sc = make_config("ladybug", m=120, n=12000, seed=7)
    kw = dict(stop_rel=1e-9, max_iter=30)   # enough passes for three forced timeouts
    e0, s0, a0, b0, plan = _solve(gpu, sc, **kw)
    assert (plan["cr_levels"] > 0) == (kind == "cr"), plan
    monkeypatch.setenv("VLGBA_DEBUG_SPIN_TIMEOUT", "0:3")
    e1, s1, a1, b1, _ = _solve(gpu, sc, **kw)
    assert s0.spin_retries == 0 and s1.spin_retries == 3
    assert s0.iterations == s1.iterations > 3
    assert np.array_equal(e0, e1)
    assert np.array_equal(a0, a1) and np.array_equal(b0, b1)


def test_spin_timeout_on_one_rank_every_rank_resolves(gpu, monkeypatch):
    """Two rank threads on one GPU (host collective): rank 1 alone reports a
    timeout on its first two passes; both ranks re-solve and the sharded
    solve is bit-identical to the same sharded solve without timeouts."""
    from bundleadjustmentmatlab_amd.dist import run_sharded
    from bundleadjustmentmatlab_amd.scene import make_config
    sc = make_config("cfg2", m=40, n=5000, seed=21)
    a = np.vstack([sc.w0, sc.T0])
    b = np.asfortranarray(sc.X0[:3])
    args = (sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, 6, a, b, 2)
    a0, b0, e0, s0 = run_sharded(*args)
    monkeypatch.setenv("VLGBA_DEBUG_SPIN_TIMEOUT", "1:2")
    a1, b1, e1, s1 = run_sharded(*args)
    assert s0.spin_retries == 0 and s1.spin_retries == 2   # rank 0's count: it re-solved too
    assert np.array_equal(e0, e1) and np.array_equal(a0, a1) and np.array_equal(b0, b1)


def test_pinv_passes_counted(gpu):
    """lambda0 = 1e-10: the first pass's Cholesky meets a non-positive pivot
    and takes the pinv step (test_gpu_lm_parity.py::test_pinv_fallback_takes_the_step)."""
    from bundleadjustmentmatlab_amd.scene import make_config
    sc = make_config("cfg1")
    _, st, _, _, _ = _solve(gpu, sc, lambda0=1e-10)
    _, st2, _, _, _ = _solve(gpu, sc)
    assert st.pinv_passes >= 1 and st2.pinv_passes == 0
