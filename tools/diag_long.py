import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import numpy as np
import bundleadjustmentmatlab_amd as gpu
from bundleadjustmentmatlab_amd.scene import make_config
kw_scene = dict(m=300, n=5000, max_track=30, radius=150.0, seed=29, long_frac=0.01, long_len=(100, 220))
if len(sys.argv) > 1 and sys.argv[1] == "nolong":
    kw_scene["long_frac"] = 0.0
sc = make_config("ladybug", **kw_scene)
num_a = 6
a = np.zeros((num_a, sc.m), order="F"); a[0:3], a[3:6] = sc.w0, sc.T0
b = np.asfortranarray(sc.X0[:3])
for name, kw in (("ordered", dict(ordered=True)), ("fast", {}), ("terms", dict(schur_kernel="terms"))):
    row = []
    ba = gpu.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, num_a, **kw)
    ba.set_params(a, b)
    for it in range(4):
        info = ba.step(relinearize=True, update_lm=True)
        row.append(f"old {info.old_sse:.12g} new {info.new_sse:.12g} lam {info.lambda_:.4g}")
    ba.close()
    print(name, " | ".join(row))
