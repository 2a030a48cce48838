"""Per-context setup time breakdown (VLGBA_SETUP_TRACE=1) on config-5-sized solves."""
import os
import sys
import time
os.environ["VLGBA_SETUP_TRACE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import bundleadjustmentmatlab_amd as pkg
from bundleadjustmentmatlab_amd.scene import make_config

sc = make_config("cfg5")
for kern in ("auto", "terms"):
    for rep in range(4):
        t0 = time.perf_counter()
        ba = pkg.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, 6, schur_kernel=kern)
        t1 = time.perf_counter()
        ba.close()
        print(f"{kern}: create {1e3*(t1-t0):.3f} ms", flush=True)
