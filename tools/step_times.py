import sys, time, numpy as np
sys.path.insert(0, "/root/repo")
import torch
import bundleadjustmentmatlab_amd as pkg
from bundleadjustmentmatlab_amd.scene import make_config
torch.cuda.set_device(0)
sc = make_config("cfg3", gpu=True, device=0)
a0 = np.zeros((6, sc.m), order="F"); a0[0:3], a0[3:6] = sc.w0, sc.T0; b0 = np.asfortranarray(sc.X0[:3])
ba = pkg.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, 6)
ba.set_params(a0, b0)
for _ in range(6): ba.step(relinearize=True, update_lm=False)
ba.sync(); torch.cuda.synchronize()
for rep in range(3):
    ts = [time.perf_counter()]
    for _ in range(20):
        ba.step(relinearize=True, update_lm=False); ts.append(time.perf_counter())
    ba.sync(); torch.cuda.synchronize(); te = time.perf_counter()
    d = np.diff(ts) * 1e3
    print("first", np.round(d[:4], 4), "median", round(float(np.median(d)), 4), "tail", round((te - ts[-1]) * 1e3, 4), "total/20", round((te - ts[0]) / 20 * 1e3, 4), flush=True)
