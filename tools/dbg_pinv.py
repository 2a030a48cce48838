"""Debug: the pinv fallback on the oracle's S at lambda = 1e-10 (cfg1)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bundle_euclid_ref as oracle  # noqa: E402
import bundleadjustmentmatlab_amd as gpu  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402

sc = make_config("cfg1")
x, vis = sc.dense()
pt, cam = np.nonzero(vis)
obs_x = np.stack([x[0, pt, cam], x[1, pt, cam]], 1)
a = np.vstack([sc.w0, sc.T0])
b = np.asfortranarray(sc.X0[:3])
pb = oracle.SparseProblem(sc.m, sc.n, pt, cam, obs_x, sc.K)
L = oracle.sp_linearize(pb, a, b, 6)
lam = 1e-10
Us = L["U"].copy(order="F")
for k in range(6):
    Us[k, k] = (1 + lam) * L["U"][k, k]
Vs = L["V"].copy(order="F")
for k in range(3):
    Vs[k, k] = (1 + lam) * L["V"][k, k]
Vi = oracle.pinv3_formula(Vs)
Y = oracle.sp_y(pb, L["W"], Vi, 6)
S, e_ = oracle.sp_schur(pb, Y, L["W"], Us, L["eA"], L["eB"], 6)
n = S.shape[0]
Sl = np.asfortranarray(S)
da_g = np.zeros(n)
e1 = np.ascontiguousarray(e_.reshape(-1))
P = lambda v: v.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
print("rc", gpu.lib().vlgba_debug_pinv_solve(n, P(Sl), P(e1), P(da_g)))
da_m = (oracle.matlab_pinv(S) @ e_).reshape(-1)
Ss = np.tril(S) + np.tril(S, -1).T
w, V = np.linalg.eigh(Ss)
tol = n * np.spacing(np.abs(w).max())
keep = np.abs(w) > tol
da_e = V[:, keep] @ ((V[:, keep].T @ e1) / w[keep])
for nm, d in (("matlab", da_m), ("eigh", da_e), ("gpu", da_g)):
    _, _, _, _, sse = oracle.sp_update(pb, L["W"], d.reshape(-1, 1), L["eB"], Vi, a, b, 6)
    print(nm, sse, np.abs(d - da_m).max() / np.abs(da_m).max())
print("ev", np.sort(np.abs(w))[:6], w.max())
Lold = float(L["e"].reshape(-1) @ L["e"].reshape(-1))
print("oracle old", Lold)
for solver in ("auto", "sequential", "envelope"):
    for ordered in (False, True):
        ba = gpu.BundleAdjuster(sc.K, pt, cam, obs_x, sc.n, 6, lambda0=lam, solver=solver,
                                ordered=ordered)
        ba.set_params(a, b)
        info = ba.step(relinearize=True, update_lm=False)
        da, db = ba.last_step()
        print("step", solver, ordered, info.new_sse, info.pinv, info.old_sse,
              np.abs(da.reshape(-1, order="F") - da_e).max() / np.abs(da_e).max(),
              np.abs(da.reshape(-1, order="F") - da_m).max() / np.abs(da_m).max())
        ba.close()

for ordered in (False, True):
    ba = gpu.BundleAdjuster(sc.K, pt, cam, obs_x, sc.n, 6, lambda0=lam, ordered=ordered)
    ba.set_params(a, b)
    Sg, eg = ba.reduced_system()
    ba.close()
    St = np.tril(S)
    print("S", ordered, np.abs(Sg - St).max(), np.abs(St).max(), np.abs(eg - e1).max(),
          np.abs(e1).max())
    bad = np.argwhere(np.abs(Sg - St) > 1e-6 * np.abs(St).max())
    print(bad[:10])
