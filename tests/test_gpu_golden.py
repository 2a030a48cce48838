"""GPU vs the committed golden fixtures (tests/golden/*.npz, made by
make_golden.py from the CPU oracle).  Needs no oracle build on the GPU box.

Stage fixtures: bit-exact (np.array_equal) for stages 1 and 2 and for stage 3
given the fixture's da.  LM fixture (reference semantics: MATLAB pinv for V*
and S): same number of accepted steps, final cost within 1e-4 relative.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("name", ["stages_na6", "stages_na7", "stages_na10"])
def test_golden_stages(gpu, name):
    g = np.load(os.path.join(HERE, f"{name}.npz"), allow_pickle=False)
    out = gpu.mex_bundle_1_XABeUVWeAeB(g["K"], g["a"], g["b"], g["X"], g["vis"])
    for k, v in zip("X_hat A B e U V W eA eB".split(), out):
        assert np.array_equal(v, g[k]), k
    S, e_ = gpu.mex_bundle_2_Se_(g["Y"], g["W"], g["Us"], g["eA"], g["eB"])
    assert np.array_equal(S, g["S"]) and np.array_equal(e_, g["e_"])
    db, a_new, b_new, X_hat = gpu.mex_bundle_3_db_new(g["W"], g["da"], g["eB"], g["Vinv"],
                                                      g["K"], g["a"], g["b"], g["X"], g["vis"])
    assert np.array_equal(db, g["db"]) and np.array_equal(a_new, g["a_new"])
    assert np.array_equal(b_new, g["b_new"]) and np.array_equal(X_hat, g["X_hat_new"])


def test_golden_lm_cfg1(gpu):
    g = np.load(os.path.join(HERE, "lm_cfg1.npz"), allow_pickle=False)
    K_, Te_, w_, Xe_, err = gpu.bundle_euclid(g["K"], g["T0"], g["w0"], g["X0"], g["x"],
                                              "visibility", g["vis"], "fix_calibration")
    want = g["error_"]
    assert len(err) == len(want)
    assert abs(err[0] - want[0]) <= 1e-12 * want[0]
    assert abs(err[-1] - want[-1]) <= 1e-4 * want[-1]
    assert np.array_equal(Xe_[3], g["Xe_"][3])       # Xe_(4,:) is the input's (Q5)
