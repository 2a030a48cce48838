"""One relinearising pass per solver on a scene; da / db / the pass scalars
saved to an .npz (bit-identity checks between two builds: VLGBA_LIB=...).

usage: python tools/da_dump.py OUT.npz [config] [m]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bundleadjustmentmatlab_amd as pkg  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402

out = sys.argv[1]
cfg = sys.argv[2] if len(sys.argv) > 2 else "ladybug"
if cfg == "long":      # tests/test_gpu_parity.py::test_long_tracks_fast_path's scene
    sc = make_config("ladybug", m=300, n=5000, max_track=30, radius=150.0, seed=29,
                     long_frac=0.01, long_len=(100, 220))
    K, pt, cam, x, n = sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n
    a = np.vstack([sc.w0, sc.T0])
    b = np.asfortranarray(sc.X0[:3])
elif cfg == "cfg5x":   # the first M cameras of the scaled growing scene (long tracks)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from prof_cfg5x_solve import sub_problem
    M = int(sys.argv[3]) if len(sys.argv) > 3 else 600
    sc = make_config("cfg5x")
    used, pt, cam, x = sub_problem(sc, M)
    K, n = sc.K[:, :M], len(used)
    a = np.vstack([sc.w0[:, :M], sc.T0[:, :M]])
    b = np.asfortranarray(sc.X0[:3, used])
else:
    kw = {"m": int(sys.argv[3]), "n": 100 * int(sys.argv[3])} if len(sys.argv) > 3 else {}
    sc = make_config(cfg, **kw)
    K, pt, cam, x, n = sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n
    a = np.vstack([sc.w0, sc.T0])
    b = np.asfortranarray(sc.X0[:3])
res = {}
for solver in ("auto", "envelope", "nd", "dense"):
    with pkg.BundleAdjuster(K, pt, cam, x, n, 6, solver=solver) as ba:
        ba.set_params(a, b)
        for _ in range(3):
            info = ba.step(relinearize=True, update_lm=True)
        da, db = ba.last_step()
        res[solver + "_da"], res[solver + "_db"] = da, db
        res[solver + "_sse"] = np.array([info.old_sse, info.new_sse])
np.savez(out, **res)
print("saved", out, {k: v.shape for k, v in res.items()})
