"""Generate the golden fixtures in tests/golden/ (run: python tests/golden/make_golden.py).

Each fixture holds seeded inputs and the CPU oracle's outputs (oracle/ba_oracle.c
+ oracle/bundle_euclid_ref.py, device-formula mode where stated).  They pin the
oracle against regressions (tests/test_oracle.py::test_golden_fixtures) and
give the GPU tests reference outputs that need no oracle build
(tests/test_gpu_golden.py).  The reference itself cannot run in this image, so
these are NOT reference outputs: see DESIGN.md "Oracle / parity status".
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(HERE))

CASES = ["stages_na6", "stages_na7", "stages_na10", "lm_cfg1"]


def _stages(num_a, seed):
    import bundle_euclid_ref as ref
    from conftest import random_problem
    K, a, b, X, vis, _ = random_problem(seed, num_a=num_a)
    X_hat, A, B, e, U, V, W, eA, eB = ref.mex1(K, a, b, X, vis)
    lam = 1e-3
    Us = U.copy(order="F")
    for k in range(num_a):
        Us[k, k] = (1 + lam) * U[k, k]
    Vs = V.copy(order="F")
    for k in range(3):
        Vs[k, k] = (1 + lam) * V[k, k]
    Vinv = ref.pinv3_formula(Vs)
    Y = ref.y_dense(W, Vinv)
    S, e_ = ref.mex2(Y, W, Us, eA, eB)
    da = ref.chol_solve_fixed(S, e_)
    db, a_new, b_new, X_hat_new = ref.mex3(W, da, eB, Vinv, K, a, b, X, vis)
    return dict(K=K, a=a, b=b, X=X, vis=vis, X_hat=X_hat, A=A, B=B, e=e, U=U, V=V, W=W,
                eA=eA, eB=eB, Us=Us, Vinv=Vinv, Y=Y, S=S, e_=e_, da=da, db=db, a_new=a_new,
                b_new=b_new, X_hat_new=X_hat_new)


def _lm_cfg1():
    import bundle_euclid_ref as ref
    from bundleadjustmentmatlab_amd.scene import make_config
    sc = make_config("cfg1")
    x, vis = sc.dense()
    K_, Te_, w_, Xe_, err = ref.bundle_euclid_ref(sc.K, sc.T0, sc.w0, sc.X0, x, "visibility",
                                                  vis, "fix_calibration", form="sparse")
    return dict(K=sc.K, T0=sc.T0, w0=sc.w0, X0=sc.X0, x=x, vis=vis, K_=K_, Te_=Te_, w_=w_,
                Xe_=Xe_, error_=err)


def compute(name):
    if name == "lm_cfg1":
        return _lm_cfg1()
    num_a = int(name.split("na")[1])
    return _stages(num_a, 100 + num_a)


if __name__ == "__main__":
    for name in CASES:
        d = compute(name)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **d)
        print(name, os.path.getsize(os.path.join(HERE, f"{name}.npz")), "bytes")
