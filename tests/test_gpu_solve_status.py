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
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPIN1 = os.path.join(ROOT, "bundleadjustmentmatlab_amd", "libvlgba_spin1.so")


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


_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import bundleadjustmentmatlab_amd as gpu
from bundleadjustmentmatlab_amd.scene import make_config
kind, out = sys.argv[2], sys.argv[3]
sc = (make_config("cfg2", m=60, n=6000, seed=5) if kind == "cr" else
      make_config("ladybug", m=120, n=12000, seed=7))
with gpu.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, 6, stop_rel=1e-9,
                        max_iter=30) as ba:
    ba.set_params(np.vstack([sc.w0, sc.T0]), np.asfortranarray(sc.X0[:3]))
    err, st = ba.run()
    a, b = ba.get_params()
np.savez(out, err=err, a=a, b=b, spin=st.spin_retries, passes=st.iterations)
"""


@pytest.mark.parametrize("kind", ["cr", "envelope"])
def test_genuine_spin_timeout_resolves_bit_identically(gpu, tmp_path, kind):
    """a REAL timeout, not the forced status word.  The test build
    libvlgba_spin1.so (BA_BACK_SPIN_MAX = 1: every hand-off spin of
    k_cr32_fused / k_backward_all gives up after one poll, leaving a partial
    launch behind) runs the solve in a child process; the passes whose solve
    timed out are re-solved without spins, and the whole LM run is the
    product library's bit for bit."""
    assert os.path.exists(SPIN1), "built by __graft_entry__.build()"
    from bundleadjustmentmatlab_amd.scene import make_config
    out = str(tmp_path / "spin1.npz")
    env = dict(os.environ, VLGBA_LIB=SPIN1, VLGBA_QUIET="1")
    subprocess.run([sys.executable, "-c", _CHILD, ROOT, kind, out], check=True, env=env,
                   timeout=300)
    r = np.load(out)
    sc = (make_config("cfg2", m=60, n=6000, seed=5) if kind == "cr" else
          make_config("ladybug", m=120, n=12000, seed=7))
    e0, s0, a0, b0, plan = _solve(gpu, sc, stop_rel=1e-9, max_iter=30)
    assert (plan["cr_levels"] > 0) == (kind == "cr"), plan
    assert s0.spin_retries == 0 and int(r["spin"]) >= 1, int(r["spin"])
    assert int(r["passes"]) == s0.iterations
    assert np.array_equal(r["err"], e0)
    assert np.array_equal(r["a"], a0) and np.array_equal(r["b"], b0)


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
