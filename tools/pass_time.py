"""Untimed wall time per relinearising pass (no kernel events) on cfg5x
sub-problems or a named config, per solver: for A/B of two builds
(VLGBA_LIB=...).  usage: python tools/pass_time.py [M | config ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402

import bundleadjustmentmatlab_amd as pkg  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402
from prof_cfg5x_solve import sub_problem  # noqa: E402

Ms = sys.argv[1:] or ["600", "900"]
full = make_config("cfg5x")
for M in Ms:
    if M.isdigit():
        M = int(M)
        used, pt, cam, x = sub_problem(full, M)
        K, n = full.K[:, :M], len(used)
        a0 = np.zeros((6, M), order="F")
        a0[0:3], a0[3:6] = full.w0[:, :M], full.T0[:, :M]
        b0 = np.asfortranarray(full.X0[:3, used])
    else:
        sc = make_config(M)
        K, pt, cam, x, n = sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n
        a0 = np.vstack([sc.w0, sc.T0])
        b0 = np.asfortranarray(sc.X0[:3])
    for solver in ("auto", "dense"):
        with pkg.BundleAdjuster(K, pt, cam, x, n, 6, solver=solver) as ba:
            ba.set_params(a0, b0)
            for _ in range(3):
                ba.step(relinearize=True, update_lm=False)
            ba.sync()
            t0 = time.perf_counter()
            for _ in range(10):
                ba.step(relinearize=True, update_lm=False)
            ba.sync()
            print(f"M={M} {solver}: {1e3 * (time.perf_counter() - t0) / 10:.3f} ms/pass (untimed)",
                  flush=True)
