import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvlgba on HIP)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def oracle():
    import bundle_euclid_ref as ref
    ref._lib()
    return ref


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test on a machine without a GPU")
    import bundleadjustmentmatlab_amd as pkg
    pkg.lib()
    return pkg


def random_problem(seed, m=6, n=40, num_a=6, density=0.6, zero_w_cam=True):
    """Small random MEX-layout problem (dense visibility, K 4xm, a num_a x m)."""
    from bundleadjustmentmatlab_amd.scene import make_config
    rng = np.random.default_rng(seed)
    sc = make_config("cfg1", m=m, min_n=n // 2, max_n=n, seed=seed)
    x, vis = sc.dense()
    n = sc.n
    # thin the visibility randomly (keep >= 1 obs per point)
    keep = rng.random(vis.shape) < density
    keep[np.arange(n), rng.integers(0, m, n)] = True
    vis = vis * keep
    K = sc.K.copy()
    K[0] += rng.normal(0, 3, m)
    K[1] += rng.normal(0, 3, m)
    a = np.zeros((num_a, m), order="F")
    a[0:3] = sc.w0
    a[3:6] = sc.T0
    if num_a == 7:
        a[6] = K[0]
    elif num_a == 10:
        a[6:10] = K
    if zero_w_cam:
        a[0:3, 0] = 0.0
    b = np.asfortranarray(sc.X0[0:3])
    X = np.asfortranarray(x[0:2])
    return K, a, b, X, np.asfortranarray(vis), sc


@pytest.fixture(scope="session")
def poracle():
    """Projective oracle (oracle/bundle_projective_ref.py)."""
    import bundle_projective_ref as pref
    import bundle_euclid_ref as ref
    ref._lib()
    return pref


def random_projective_problem(seed, m=6, n=40, density=0.6):
    """Small random mex_bundle_proj_* problem: a = P(:) (12 x m) of a perturbed
    Euclidean scene (scene.projective_from), b 3 x n, X 2 x n x m, vis n x m."""
    from bundleadjustmentmatlab_amd.scene import make_config, projective_from
    rng = np.random.default_rng(seed)
    sc = make_config("cfg1", m=m, min_n=n // 2, max_n=n, seed=seed)
    x, vis = sc.dense()
    n = sc.n
    keep = rng.random(vis.shape) < density
    keep[np.arange(n), rng.integers(0, m, n)] = True
    vis = vis * keep
    Pp, Xp = projective_from(sc)
    a = np.asfortranarray(Pp.reshape(12, m, order="F"))
    b = np.asfortranarray(Xp[0:3])
    X = np.asfortranarray(x[0:2])
    return a, b, X, np.asfortranarray(vis), sc, Pp, Xp
