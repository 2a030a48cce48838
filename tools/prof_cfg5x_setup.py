"""Setup vs solve time of one large cfg5x-like solve (GPU box): context
creation (host plan + uploads, VLGBA_SETUP_TRACE=1 prints its phases), then
a whole LM solve (run)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bundleadjustmentmatlab_amd as pkg  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_cfg5x_solve import sub_problem  # noqa: E402

os.environ["VLGBA_SETUP_TRACE"] = "1"
sc = make_config("cfg5x")
for M in [int(a) for a in sys.argv[1:]] or [900]:
    used, pt, cam, x = sub_problem(sc, M)
    a0 = np.zeros((6, M), order="F")
    a0[0:3], a0[3:6] = sc.w0[:, :M], sc.T0[:, :M]
    b0 = np.asfortranarray(sc.X0[:3, used])
    for rep in range(2):
        t0 = time.perf_counter()
        ba = pkg.BundleAdjuster(sc.K[:, :M], pt, cam, x, len(used), 6)
        t1 = time.perf_counter()
        ba.set_params(a0, b0)
        err, st = ba.run()
        ba.sync()
        t2 = time.perf_counter()
        ba.close()
        t3 = time.perf_counter()
        print(f"M={M} obs={len(pt)}: setup {1e3*(t1-t0):.1f} ms, run {1e3*(t2-t1):.1f} ms "
              f"({st.iterations} passes), close {1e3*(t3-t2):.1f} ms", flush=True)
