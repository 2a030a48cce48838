"""Converged cost on the BASELINE scenes (north star: "final cost within 1e-6
relative of reference"), configs 2 and 3 at full size.

* Parity mode on config 2 (50 x 10k x 60k): ordered sums, the sequential
  Cholesky and the LM scalars in the reference's flat order -- the whole LM
  trajectory to convergence under the tightened stop rule is bit-identical to
  the CPU oracle's (oracle/bundle_euclid_ref.py over oracle/ba_oracle.c), so
  the final cost is the oracle's exactly.
* The default fast path (chunked MFMA Schur sums, cyclic-reduction solve):
  its converged cost against the reference's converged-cost band
  (tests/golden/converged_cfg2_cfg3.json, tests/golden/make_converged.py):
  the final costs of 8 (config 3) / 16 (config 2) CPU restatements of
  bundle_euclid.m with MATLAB semantics (pinv of V*_i and of S) and rounding
  variants of them (summation orders, closed-form V*^-1, Cholesky solves).
  With h = 1e-10 forward differences the converged cost is path dependent:
  LM stalls where the FD Jacobians' rounding noise stops it (run past the
  stop rule, the variants keep their values to 1e-10 for 20 iterations), at
  a cost that depends on the summation order -- the reference's own
  variants end 2.7e-6 (config 3) / 4.1e-6 (config 2) apart, a 3-camera
  solve of config 5 up to 1e-5.  A bar of 1e-6 against one variant is
  therefore not met by the reference against itself; the bar here is: the
  GPU's converged cost within max(1e-6, the band's own width) of the band.
  The arithmetic itself is pinned by the parity-mode test above (identical
  converged cost at full config-2 size).
  The scene and the start are checked first: error_(1) equal to the
  fixture's to 1e-12.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
STOP = dict(stop_rel=1e-12, max_iter=200, max_iter2=30)   # = make_converged.STOP


def _fixture(name):
    with open(os.path.join(HERE, "golden", "converged_cfg2_cfg3.json")) as f:
        fx = json.load(f)[name]
    assert fx["stop"] == STOP
    return fx


def _gpu_solve(gpu, sc, **kw):
    a = np.vstack([sc.w0, sc.T0])
    b = np.asfortranarray(sc.X0[:3])
    with gpu.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, 6, **STOP, **kw) as ba:
        ba.set_params(a, b)
        err, st = ba.run()
    return err.copy(), st


@pytest.mark.timeout(600)
def test_cfg2_parity_mode_converged_bit_identical(gpu, oracle):
    from bundleadjustmentmatlab_amd.scene import make_config
    sc = make_config("cfg2")
    x, vis = sc.dense()
    got = gpu.bundle_euclid(sc.K, sc.T0, sc.w0, sc.X0, x, "visibility", vis, "fix_calibration",
                            parity=True, **STOP)
    ref = oracle.bundle_euclid_ref(sc.K, sc.T0, sc.w0, sc.X0, x, "visibility", vis,
                                   "fix_calibration", form="sparse", vinv="formula", solve="seq",
                                   sums="seq", **STOP)
    assert len(got[4]) > 20, got[4]
    assert np.array_equal(got[4], ref[4]), (got[4], ref[4])
    for g, r, nm in zip(got[:4], ref[:4], ("K_", "Te_", "w_", "Xe_")):
        assert np.array_equal(g, r), nm


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", ["cfg2", "cfg3"])
def test_fast_path_converged_cost_in_reference_band(gpu, name):
    from bundleadjustmentmatlab_amd.scene import make_config
    fx = _fixture(name)
    sc = make_config(name, gpu=False)
    assert (sc.m, sc.n, sc.num_obs) == (fx["scene"]["m"], fx["scene"]["n"],
                                        fx["scene"]["num_obs"])
    err, st = _gpu_solve(gpu, sc)
    e0 = next(iter(fx["variants"].values()))["error"][0]
    assert abs(err[0] - e0) <= 1e-12 * e0, (err[0], e0)
    finals = {k: v["error"][-1] for k, v in fx["variants"].items()}
    lo, hi = fx["final_min"], fx["final_max"]
    out = max(lo - err[-1], err[-1] - hi, 0.0) / lo     # distance to the band
    bar = max(1e-6, fx["spread_rel"])
    print(f"{name}: GPU final {err[-1]:.10g} after {st.iterations} passes; reference band "
          f"[{lo:.10g}, {hi:.10g}] over {len(finals)} variants (spread "
          f"{fx['spread_rel']:.2e}); outside the band by {out:.2e} (bar {bar:.2e})")
    assert out <= bar, (err[-1], finals)
    # pinv(S) e_ is the banded solve on these scenes: no eigenvalue of S falls
    # below MATLAB pinv's tolerance (checked when the fixture was made)
    margins = [v["pinv_margin"] for v in fx["variants"].values() if "pinv_margin" in v]
    assert margins and min(margins) > 1.0
