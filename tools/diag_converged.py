"""Diagnostic (GPU box): converged cost of the cfg3 fast path and of its
internal variants (Schur kernel, reduced solver, ordered sums) under the
tightened stop rule, beside the reference band of
tests/golden/converged_cfg2_cfg3.json."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bundleadjustmentmatlab_amd as gpu   # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config   # noqa: E402

STOP = dict(stop_rel=1e-12, max_iter=200, max_iter2=30)
name = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
fx = json.load(open(os.path.join(ROOT, "tests", "golden", "converged_cfg2_cfg3.json")))[name]
print("band", fx["final_min"], fx["final_max"])
for k, v in fx["variants"].items():
    e = np.array(v["error"])
    print(f"  {k:28s} n={len(e):3d} final={e[-1]:.10f} e[10]={e[10]:.10f} e[20]={e[20]:.10f}")
sc = make_config(name, gpu=False)
a = np.vstack([sc.w0, sc.T0])
b = np.asfortranarray(sc.X0[:3])
for kw in ({}, {"schur_kernel": "terms"}, {"solver": "envelope"}, {"solver": "dense"},
           {"ordered": True}, {"lambda0": 1.0001e-3}):
    with gpu.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, 6, **STOP, **kw) as ba:
        ba.set_params(a, b)
        err, st = ba.run()
    print(f"GPU {str(kw):28s} n={len(err):3d} final={err[-1]:.10f} e[10]={err[10]:.10f} "
          f"e[20]={err[20]:.10f} passes={st.iterations} acc={st.accepted}", flush=True)
