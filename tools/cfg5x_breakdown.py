"""Where the scaled growing replay (cfg5x) spends its solve time (GPU box):
context creation (the host plan + uploads), the LM loop, and the rest, per
solve-size bucket (cameras in the solve).

usage: python tools/cfg5x_breakdown.py [config]      (default cfg5x)
"""
import os
import sys
import time
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bundleadjustmentmatlab_amd.bundle as bundle  # noqa: E402
from bundleadjustmentmatlab_amd.incremental import incremental_bundle  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402

acc = defaultdict(float)
cur = {}
init0, run0, close0 = (bundle.BundleAdjuster.__init__, bundle.BundleAdjuster.run,
                       bundle.BundleAdjuster.close)


def init(self, *a, **k):
    t = time.perf_counter()
    init0(self, *a, **k)
    cur["init"] = time.perf_counter() - t


def run(self):
    t = time.perf_counter()
    r = run0(self)
    cur["run"] = time.perf_counter() - t
    return r


def timed(name, fn):
    def w(self, *a, **k):
        t = time.perf_counter()
        r = fn(self, *a, **k)
        cur[name] = cur.get(name, 0.0) + time.perf_counter() - t
        return r
    return w


bundle.BundleAdjuster.__init__, bundle.BundleAdjuster.run = init, run
for nm in ("set_params", "get_params", "close"):
    setattr(bundle.BundleAdjuster, nm, timed(nm, getattr(bundle.BundleAdjuster, nm)))
cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg5x"
sc = make_config(cfg)
rows = []


def progress(solves):
    s = solves[-1]
    rows.append((s["cameras"], s["observations"], s["passes"], s["seconds"], cur.get("init", 0.0),
                 cur.get("run", 0.0), cur.get("set_params", 0.0), cur.get("get_params", 0.0),
                 cur.get("close", 0.0)))
    cur.clear()


t0 = time.perf_counter()
incremental_bundle(sc, devices=[0], progress=progress)
total = time.perf_counter() - t0
R = np.array(rows)
print(f"{cfg}: replay {total:.1f} s, {len(R)} solves, solve time {R[:, 3].sum():.1f} s "
      f"(context creation {R[:, 4].sum():.1f} s, LM loop {R[:, 5].sum():.1f} s), "
      f"{int(R[:, 2].sum())} passes")
edges = [0, 100, 300, 600, 800, 1001]
for lo, hi in zip(edges[:-1], edges[1:]):
    sel = (R[:, 0] >= lo) & (R[:, 0] < hi)
    if not sel.any():
        continue
    r = R[sel]
    print(f"  cams [{lo:4d},{hi:4d}): {sel.sum():5d} solves  {r[:, 3].sum():6.2f} s  "
          f"create {r[:, 4].sum():6.2f} s ({1e3 * r[:, 4].mean():6.2f} ms each)  "
          f"loop {r[:, 5].sum():6.2f} s  passes {int(r[:, 2].sum()):6d} "
          f"({1e3 * r[:, 5].sum() / max(1, r[:, 2].sum()):.2f} ms/pass)  set {r[:, 6].sum():.2f} "
          f"get {r[:, 7].sum():.2f} close {r[:, 8].sum():.2f} s")
