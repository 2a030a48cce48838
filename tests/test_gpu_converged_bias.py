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


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name", ["cfg2", "cfg3"])
def test_converged_cost_cfg2_cfg3(gpu, name):
    """the BASELINE scenes at full size, 12 seeds each
    (cfg2 seeds 2-13, cfg3 seeds 3-14), the GPU's converged cost under the
    tightened stop rule against the reference's finals (MATLAB semantics on the
    CPU port, tests/golden/converged_cfg2_cfg3_12seeds.json -- generated on the
    GPU box's host by tools/converged_bias.py; a cfg3 reference solve takes
    ~15 s of 16 CPU threads, so the finals are data here).  The same bars as
    above at the reference's own floor: both signs, sign test p >= 0.01, the
    median |d| within 2x the reference's own median |f| (a 1e-9 move of its
    lambda0: measured 1.50e-6 against 1.43e-6 at cfg3, 1.76e-6 against 2.84e-6
    at cfg2 -- the north star's 1e-6 is below the reference's own floor at
    these sizes), every |d| <= 1e-4."""
    import json
    import os
    from bundleadjustmentmatlab_amd.scene import make_config
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                           "converged_cfg2_cfg3_12seeds.json")) as fh:
        fx = json.load(fh)
    stop = fx["stop"]
    d, f = [], []
    for seed, ref in sorted(fx["finals"][name].items(), key=lambda kv: int(kv[0])):
        sc = make_config(name, seed=int(seed))
        a = np.vstack([sc.w0, sc.T0])
        b = np.asfortranarray(sc.X0[:3])
        with gpu.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, 6, **stop) as ba:
            ba.set_params(a, b)
            err, _ = ba.run()
        d.append((err[-1] - ref["ref"]) / ref["ref"])
        f.append((ref["ref_l0"] - ref["ref"]) / ref["ref"])
    d, f = np.array(d), np.array(f)
    pos, neg = int((d > 0).sum()), int((d < 0).sum())
    p = _sign_p(pos, neg)
    med, floor = float(np.median(np.abs(d))), float(np.median(np.abs(f)))
    print(f"{name}: {len(d)} solves: GPU above the reference {pos}, below {neg} (sign test "
          f"p {p:.3f}); median |d| {med:.2e}, max {np.abs(d).max():.2e}; the reference's "
          f"lambda0 floor median {floor:.2e}, max {np.abs(f).max():.2e}")
    assert len(d) == 12
    assert pos > 0 and neg > 0, d
    assert p >= 0.01, (pos, neg)
    assert med <= 2 * floor, (med, floor)
    assert np.abs(d).max() <= 1e-4, d
