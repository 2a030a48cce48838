"""Where a growing-replay solve's set_params time goes (GPU box): context
creation, a stream sync right after it, then set_params twice and close, on
cfg5x sub-problems of increasing size (repeated sizes re-use cached blocks).

usage: VLGBA_SETP_TIMING=1 python tools/setp_probe.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402

import bundleadjustmentmatlab_amd as pkg  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402
from prof_cfg5x_solve import sub_problem  # noqa: E402

sc = make_config("cfg5x")
for M in (300, 600, 900, 900, 910, 920, 930):
    used, pt, cam, x = sub_problem(sc, M)
    a0 = np.zeros((6, M), order="F")
    a0[0:3], a0[3:6] = sc.w0[:, :M], sc.T0[:, :M]
    b0 = np.asfortranarray(sc.X0[:3, used])
    t = [time.perf_counter()]
    ba = pkg.BundleAdjuster(sc.K[:, :M], pt, cam, x, len(used), 6)
    t.append(time.perf_counter())
    ba.sync()
    t.append(time.perf_counter())
    ba.set_params(a0, b0)
    t.append(time.perf_counter())
    ba.set_params(a0, b0)
    t.append(time.perf_counter())
    err, st = ba.run()
    t.append(time.perf_counter())
    ba.close()
    t.append(time.perf_counter())
    d = np.diff(t) * 1e3
    print(f"M={M}: create {d[0]:.2f} sync {d[1]:.2f} set {d[2]:.2f} set2 {d[3]:.2f} "
          f"run {d[4]:.2f} ({st.iterations} passes) close {d[5]:.2f} ms", flush=True)
