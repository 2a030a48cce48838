"""Where one large solve of the scaled growing replay (cfg5x) spends its time
(GPU box): the first M cameras of scene.growing_scene and the points they see,
one relinearising LM pass with per-kernel HIP-event timing, for each solver.

usage: python tools/prof_cfg5x_solve.py [M ...]        (default 300 600 900)
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bundleadjustmentmatlab_amd as pkg  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402


def sub_problem(sc, M):
    keep = sc.obs_cam < M
    pt, cam, x = sc.obs_pt[keep], sc.obs_cam[keep], sc.obs_x[keep]
    used, inv = np.unique(pt, return_inverse=True)
    return used, inv.astype(np.int32), cam.astype(np.int32), x


def main():
    Ms = [int(a) for a in sys.argv[1:]] or [300, 600, 900]
    sc = make_config("cfg5x")
    for M in Ms:
        used, pt, cam, x = sub_problem(sc, M)
        a0 = np.zeros((6, M), order="F")
        a0[0:3], a0[3:6] = sc.w0[:, :M], sc.T0[:, :M]
        b0 = np.asfortranarray(sc.X0[:3, used])
        # co-visibility reach: the widest camera span of a track
        span = np.zeros(len(used), np.int64)
        np.maximum.at(span, pt, cam)
        lo = np.full(len(used), M, np.int64)
        np.minimum.at(lo, pt, cam)
        reach = int((span - lo).max())
        for solver in ("auto", "dense"):
            ba = pkg.BundleAdjuster(sc.K[:, :M], pt, cam, x, len(used), 6, solver=solver)
            ba.set_params(a0, b0)
            for _ in range(2):
                ba.step(relinearize=True, update_lm=False)
            ba.sync()
            ba.set_timing(True)
            ba.kernel_ms(reset=True)
            t0 = time.perf_counter()
            for _ in range(3):
                ba.step(relinearize=True, update_lm=False)
            ba.sync()
            dt = (time.perf_counter() - t0) / 3
            km = ba.kernel_ms(reset=True)
            plan = ba.plan_info()
            ph = ba.phase_ms()
            ba.set_timing(False)
            ba.close()
            top = sorted(km.items(), key=lambda kv: -kv[1][0])[:8]
            print(f"M={M} obs={len(pt)} pts={len(used)} reach={reach} cams solver={solver}: "
                  f"{1e3 * dt:.2f} ms/pass; tiles={plan['tiles']} cr_levels={plan['cr_levels']} "
                  f"blocks={plan['blocks']}", flush=True)
            print("   phases(ms): " + " ".join(f"{k}={v:.3f}" for k, v in ph.items()))
            print("   kernels: " + "  ".join(f"{k}={t / 3:.3f}ms x{c / 3:.0f}" for k, (t, c) in top),
                  flush=True)


if __name__ == "__main__":
    main()
