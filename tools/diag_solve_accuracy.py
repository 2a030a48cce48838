"""Diagnostic (GPU box): accuracy of the reduced solve per solver on config 3
(one pass at the start point): relative residual ||S da - e_|| / ||e_|| of
the GPU's da for the cyclic reduction ("auto"), the envelope and the dense
tile Cholesky, and of LAPACK's banded Cholesky on the same S (oracle port)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bundleadjustmentmatlab_amd as gpu   # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config   # noqa: E402
import scipy.sparse as sp   # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
sc = make_config(name, gpu=False)
a = np.vstack([sc.w0, sc.T0])
b = np.asfortranarray(sc.X0[:3])
na, m = 6, sc.m
ld = na * m
S = e_ = None
for solver in ("auto", "envelope", "dense"):
    with gpu.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, 6, solver=solver) as ba:
        ba.set_params(a, b)
        jk, blocks, e = ba.reduced_system(dense=False)
        if S is None:
            rows, cols, vals = [], [], []
            for (j, k), B in zip(jk, blocks):
                r0, c0 = na * j, na * k
                for rr in range(na):
                    for cc in range(na):
                        if j == k and cc > rr:
                            continue
                        rows.append(r0 + rr); cols.append(c0 + cc); vals.append(B[rr, cc])
            L = sp.csr_matrix((vals, (rows, cols)), shape=(ld, ld))
            S = (L + L.T - sp.diags(L.diagonal())).tocsr()
            e_ = e.copy()
        ba.step(relinearize=False, update_lm=False)
        da, _ = ba.last_step()
        da = da.reshape(-1, order="F")
        zero = S.diagonal() == 0
        r = S @ da - np.where(zero, 0.0, e_)
        print(f"{solver:9s} rel residual {np.linalg.norm(r) / np.linalg.norm(e_):.3e}  "
              f"max|r|/max|e| {np.abs(r).max() / np.abs(e_).max():.3e}  |da| {np.abs(da).max():.4e}",
              flush=True)
        if solver == "auto":
            da_cr = da
import cpu_port   # noqa: E402
Sd = S.toarray()
db, bw = cpu_port.band_cholesky_solve(Sd, e_)
r = S @ db - np.where(S.diagonal() == 0, 0.0, e_)
print(f"lapack-band rel residual {np.linalg.norm(r) / np.linalg.norm(e_):.3e}  "
      f"max|da_cr - da_band| / max|da| {np.abs(da_cr - db).max() / np.abs(db).max():.3e}")
# one step of iterative refinement on the CR solution (in fp64)
r = np.where(S.diagonal() == 0, 0.0, e_) - S @ da_cr
dd, _ = cpu_port.band_cholesky_solve(Sd, r)
da2 = da_cr + dd
r2 = S @ da2 - np.where(S.diagonal() == 0, 0.0, e_)
print(f"cr + 1 refinement rel residual {np.linalg.norm(r2) / np.linalg.norm(e_):.3e}")
