"""Diagnostic (GPU box): where and why the fast path stops on a small scene
under the tightened stop rule.  Prints the last LM passes of the GPU run
(lambda, accept), then the drop of a fresh LM (lambda0 = 1e-3) started at
the GPU's answer: the GPU's own and the oracle's (MATLAB semantics).

usage: python tools/diag_small_stop.py [small|banded]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import bundleadjustmentmatlab_amd as gpu  # noqa: E402
import bundle_euclid_ref as oracle  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "small"
sc = (make_config("cfg1", m=6, min_n=30, max_n=60, seed=7) if kind == "small"
      else make_config("cfg2", m=24, n=1500, seed=9))
x, vis = sc.dense()
kw = dict(stop_rel=1e-12, max_iter=200, max_iter2=30)
for solver in ("auto", "dense"):
    recs = []
    got = gpu.bundle_euclid(sc.K, sc.T0, sc.w0, sc.X0, x, "visibility", vis, "fix_calibration",
                            solver=solver, log=recs.append, **kw)
    print(f"== GPU solver {solver}: final {got[4][-1]:.12f}, {len(recs)} passes, "
          f"{sum(r['accepted'] for r in recs)} accepted")
    for r in recs[-34:]:
        print(f"   pass {r['pass']:3d} lambda {r['lambda']:.3e} accepted {int(r['accepted'])} "
              f"old {r['old_sse']:.15e} new {r['new_sse']:.15e}")
    again = gpu.bundle_euclid(*got[:4], x, "visibility", vis, "fix_calibration", solver=solver, **kw)[4]
    ref_c = oracle.bundle_euclid_ref(*got[:4], x, "visibility", vis, "fix_calibration",
                                     form="sparse", vinv="pinv", solve="pinv", **kw)[4]
    for nm, e in (("GPU", again), ("oracle", ref_c)):
        if len(e):
            print(f"   fresh {nm} LM from the GPU's answer: {e[0]:.12f} -> {e[-1]:.12f} "
                  f"(drop {(e[0] - e[-1]) / e[0]:.2e}, {len(e)} error_ entries)")
        else:
            print(f"   fresh {nm} LM from the GPU's answer: no step accepted")
ref = oracle.bundle_euclid_ref(sc.K, sc.T0, sc.w0, sc.X0, x, "visibility", vis, "fix_calibration",
                               form="sparse", vinv="pinv", solve="pinv", **kw)
print(f"== oracle final {ref[4][-1]:.12f} ({len(ref[4])} error_ entries)")
