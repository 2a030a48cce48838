"""Nested-dissection envelope vs the natural order on the scaled growing
replay's sub-problems (first M cameras of cfg5x): the planner's choice, the
pass time, and da of each solver against numpy's dense solve of the same
reduced system (vlgba_get_reduced_system).

usage: python tools/nd_check.py [M ...]        (default 300 600 900 1000)
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bundleadjustmentmatlab_amd as pkg  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_cfg5x_solve import sub_problem  # noqa: E402


def main():
    Ms = [int(a) for a in sys.argv[1:]] or [300, 600, 900, 1000]
    sc = make_config("cfg5x")
    for M in Ms:
        used, pt, cam, x = sub_problem(sc, M)
        a0 = np.zeros((6, M), order="F")
        a0[0:3], a0[3:6] = sc.w0[:, :M], sc.T0[:, :M]
        b0 = np.asfortranarray(sc.X0[:3, used])
        ref = None
        for solver in ("envelope", "nd", "auto"):
            with pkg.BundleAdjuster(sc.K[:, :M], pt, cam, x, len(used), 6, solver=solver) as ba:
                ba.set_params(a0, b0)
                info = ba.step(relinearize=True, update_lm=False)
                da, _ = ba.last_step()
                if ref is None:
                    S, e = ba.reduced_system(dense=True)
                    S = np.tril(S) + np.tril(S, -1).T
                    e = e.reshape(-1).copy()
                    z = np.flatnonzero(np.diag(S) == 0.0)   # exactly-zero rows: da = 0
                    S[z, z] = 1.0
                    e[z] = 0.0
                    ref = np.linalg.solve(S, e)
                    cond = np.linalg.cond(S)
                ba.sync()
                t0 = time.perf_counter()
                for _ in range(5):
                    ba.step(relinearize=True, update_lm=False)
                ba.sync()
                dt = (time.perf_counter() - t0) / 5
                plan = ba.plan_info()
            d = da.reshape(-1, order="F")
            err = np.max(np.abs(d - ref)) / np.max(np.abs(ref))
            print(f"M={M} {solver:8s} tiles={plan['tiles']:4d} arcs={plan['nd_arcs']} "
                  f"sep={plan['nd_sep_tiles']:3d} chol_failed={info.chol_failed} "
                  f"{1e3 * dt:7.3f} ms/pass  da rel err vs numpy {err:.2e} (cond {cond:.1e})",
                  flush=True)


if __name__ == "__main__":
    main()
