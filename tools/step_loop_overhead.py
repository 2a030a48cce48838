import sys, time, numpy as np
sys.path.insert(0, "/root/repo")
import bundleadjustmentmatlab_amd as pkg
from bundleadjustmentmatlab_amd.scene import make_config
sc = make_config("cfg3")
a0 = np.vstack([sc.w0, sc.T0]); b0 = np.asfortranarray(sc.X0[:3])
ba = pkg.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, 6)
ba.set_params(a0, b0)
for _ in range(5): ba.step(relinearize=True, update_lm=False)
ba.sync()
for rep in range(3):
    t0 = time.perf_counter()
    for _ in range(100): ba.step(relinearize=True, update_lm=False)
    ba.sync(); t1 = time.perf_counter()
    ba.passes(100); ba.sync(); t2 = time.perf_counter()
    print(f"python step loop {1e3*(t1-t0)/100:.4f} ms/pass; C++ run_passes {1e3*(t2-t1)/100:.4f} ms/pass", flush=True)
