"""Is the default fast path's converged cost biased against the reference's?
(four of four GPU finals had landed above the
MATLAB-semantics oracle.)

Each solve starts from the SAME point on the GPU (default fast path: chunked
MFMA Schur sums, cyclic-reduction solve, fused update) and on the oracle with
the reference's MATLAB semantics (SVD pinv of V*_i and of S,
oracle/bundle_euclid_ref.py), under the tightened stop rule; d = (GPU final -
oracle final) / oracle final.  Beside it the reference's own floor: the
oracle with lambda0 moved by one part in 1e9 against the unmoved oracle, f.
Over 16 seeds of config 1's model and of the 6-camera "small" model:
  * the signs of d are balanced (both present; two-sided sign test p >= 0.01);
  * the median |d| is within the north star's 1e-6 and within 3x the
    reference's own median |f| (a rounding-size change of the reference's
    start moves its final cost as much as the GPU does);
  * every |d| <= 1e-4 (the reference's own |f| reaches 1.2e-4 on these models:
    profiles/r05d_converged_bias.json, 194 solves over six sets incl. the cfg5
    replay and cfg2 / cfg3 seeds: 97 above, 97 below).
tools/converged_bias.py runs the full study.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KW = dict(stop_rel=1e-9, max_iter=100, max_iter2=30)
SEEDS = range(100, 116)


def _scene(kind, seed):
    from bundleadjustmentmatlab_amd.scene import make_config
    if kind == "small":
        return make_config("cfg1", m=6, min_n=30, max_n=60, seed=seed)
    return make_config("cfg1", seed=seed)


def _sign_p(pos, neg):
    n = pos + neg
    k = min(pos, neg)
    return min(1.0, 2 * sum(math.comb(n, i) for i in range(k + 1)) / 2.0 ** n)


@pytest.mark.timeout(600)
def test_converged_cost_unbiased(gpu, oracle):
    d, f = [], []
    for kind in ("small", "cfg1"):
        for seed in SEEDS:
            sc = _scene(kind, seed)
            x, vis = sc.dense()
            opts = ("visibility", vis, "fix_calibration")
            g = gpu.bundle_euclid(sc.K, sc.T0, sc.w0, sc.X0, x, *opts, **KW)[4][-1]
            r = oracle.bundle_euclid_ref(sc.K, sc.T0, sc.w0, sc.X0, x, *opts, form="sparse",
                                         vinv="pinv", solve="pinv", **KW)[4][-1]
            r9 = oracle.bundle_euclid_ref(sc.K, sc.T0, sc.w0, sc.X0, x, *opts, form="sparse",
                                          vinv="pinv", solve="pinv", lambda0=1e-3 * (1 + 1e-9),
                                          **KW)[4][-1]
            d.append((g - r) / r)
            f.append((r9 - r) / r)
    d, f = np.array(d), np.array(f)
    pos, neg = int((d > 0).sum()), int((d < 0).sum())
    p = _sign_p(pos, neg)
    med, floor = float(np.median(np.abs(d))), float(np.median(np.abs(f)))
    print(f"{len(d)} solves: GPU above the reference {pos}, below {neg} (sign test p {p:.3f}); "
          f"median |d| {med:.2e}, max {np.abs(d).max():.2e}; the reference's lambda0 floor "
          f"median {floor:.2e}, max {np.abs(f).max():.2e}")
    assert pos > 0 and neg > 0, d
    assert p >= 0.01, (pos, neg)
    assert med <= 1e-6, med
    assert med <= 3 * floor + 1e-9, (med, floor)
    assert np.abs(d).max() <= 1e-4, d
