"""Scene evaluation around the BA path:
``error_reproj`` (toolbox/test/error_reproj.m) and ``align_scene``
(toolbox/geometry/align_scene.m), plus the Rodrigues maps they use.

Host-side numpy (vectorised): these run once per solve on n x m data and are
not on the LM hot path.  Arrays keep the reference's MATLAB shapes.

Reference quirk kept by default (App. A Q16): error_reproj.m:78 tests
``vis(n,m)`` -- the LAST entry of the visibility map -- instead of
``vis(i,j)``, so every pair with X(4,i) == 1 contributes when vis(n,m) != 0,
while the average divides by sum(vis(:)).  ``per_pair_visibility=True`` is the
opt-in fix (only visible pairs contribute).
"""
from __future__ import annotations

import numpy as np

__all__ = ["vl_rodr", "vl_irodr", "calibration_matrix", "error_reproj", "align_scene"]


def vl_rodr(w):
    """Rotation vectors (3,) or (3, k) -> R (3, 3) or (k, 3, 3) (VLFeat
    vl_rodrigues, SURVEY.md App. B: theta < 1e-6 gives I)."""
    w = np.asarray(w, dtype=np.float64)
    single = w.ndim == 1
    w = w.reshape(3, -1)
    th = np.sqrt((w * w).sum(0))
    small = th < 1e-6
    ths = np.where(small, 1.0, th)
    x, y, z = w / ths
    s, c = np.sin(th), np.cos(th)
    mc = 1.0 - c
    R = np.empty((w.shape[1], 3, 3))
    R[:, 0, 0] = 1 - mc * (y * y + z * z)
    R[:, 1, 0] = s * z + mc * x * y
    R[:, 2, 0] = -s * y + mc * x * z
    R[:, 0, 1] = -s * z + mc * x * y
    R[:, 1, 1] = 1 - mc * (z * z + x * x)
    R[:, 2, 1] = s * x + mc * y * z
    R[:, 0, 2] = s * y + mc * x * z
    R[:, 1, 2] = -s * x + mc * y * z
    R[:, 2, 2] = 1 - mc * (x * x + y * y)
    R[small] = np.eye(3)
    return R[0] if single else R


def vl_irodr(R):
    """Inverse Rodrigues map R (3, 3) -> w (3,), or a stack (k, 3, 3) -> (3, k)
    (VLFeat vl_irodr): the rotation angle from the trace, the axis from the
    skew part; the angle-pi case from the symmetric part."""
    R = np.asarray(R, dtype=np.float64)
    if R.ndim == 3:
        c = np.clip((np.trace(R, axis1=1, axis2=2) - 1.0) / 2.0, -1.0, 1.0)
        th = np.arccos(c)
        v = np.stack([R[:, 2, 1] - R[:, 1, 2], R[:, 0, 2] - R[:, 2, 0], R[:, 1, 0] - R[:, 0, 1]])
        s = np.sin(th)
        reg = s > 1e-8
        out = np.where(th < 1e-6, 0.5 * v, th / (2.0 * np.where(reg, s, 1.0)) * v)
        for k in np.nonzero((th >= 1e-6) & ~reg)[0]:   # theta ~ pi (rare): one by one
            out[:, k] = vl_irodr(R[k])
        return out
    c = np.clip((np.trace(R) - 1.0) / 2.0, -1.0, 1.0)
    th = np.arccos(c)
    v = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    s = np.sin(th)
    if th < 1e-6:
        return 0.5 * v
    if s > 1e-8:
        return th / (2.0 * s) * v
    # theta ~ pi: R = 2 a a^T - I
    A = (R + np.eye(3)) / 2.0
    k = int(np.argmax(np.diag(A)))
    a = A[:, k] / np.sqrt(A[k, k])
    return th * a / np.linalg.norm(a)


def calibration_matrix(Kparam):
    """toolbox/geometry/calibration_matrix.m: [fx 0 cx; 0 fy cy; 0 0 1]."""
    fx, fy, cx, cy = np.asarray(Kparam, dtype=np.float64).reshape(4)
    return np.array([[fx, 0.0, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]])


def _k_stack(K, m):
    K = np.asarray(K, dtype=np.float64)
    if K.shape[0] == 4:                                   # error_reproj.m:52-59
        return np.stack([calibration_matrix(K[:, j]) for j in range(m)])
    if K.ndim == 2:                                       # :60-68
        return np.repeat(K[None], m, axis=0)
    return np.moveaxis(K, -1, 0)


def error_reproj(x, K, T, w, X, *varargin, per_pair_visibility=False):
    """[err error] = error_reproj(x, K, T, w, X, 'visibility', vis)
    (toolbox/test/error_reproj.m:1-86).  Returns (err, error (n x m))."""
    x, T, w, X = (np.asarray(v, dtype=np.float64) for v in (x, T, w, X))
    m, n = T.shape[1], X.shape[1]
    vis = np.ones((n, m))
    k = 0
    while k < len(varargin):
        if str(varargin[k]).lower() == "visibility":
            vis = np.asarray(varargin[k + 1], dtype=np.float64).reshape(n, m)
            k += 1
        k += 1
    Ks = _k_stack(K, m)
    R = vl_rodr(w)
    P = np.einsum("jab,jbc->jac", Ks, np.concatenate([R, T.T[:, :, None]], axis=2))  # (m,3,4)
    xr = np.einsum("jab,bi->jai", P, X)                  # (m, 3, n)
    xr = xr / xr[:, 2:3, :]
    d = x[0:2].transpose(2, 0, 1) - xr[:, 0:2, :]         # (m, 2, n)
    err_ij = np.sqrt((d * d).sum(1)).T                    # (n, m)
    if per_pair_visibility:
        mask = (X[3] == 1)[:, None] & (vis != 0)
    else:                                                 # :78 tests vis(n,m) (Q16)
        mask = np.broadcast_to((X[3] == 1)[:, None] & (vis[n - 1, m - 1] != 0), (n, m))
    error = np.where(mask, err_ij, 0.0)
    return float(error.sum() / vis.sum()), error


def align_scene(T, Omega, X, TRef=None, OmegaRef=None, XRef=None, ScaleOption="centroid"):
    """[T_ Omega_ X_] = align_scene(T, Omega, X[, TRef, OmegaRef, XRef[, ScaleOption]])
    (toolbox/geometry/align_scene.m:1-106): the first camera becomes the
    reference frame ([I|0] by default) and the scene is scaled so that the
    centroid of the points (or the first baseline, 'translation') matches."""
    T, Omega, X = (np.asarray(v, dtype=np.float64) for v in (T, Omega, X))
    m, n = T.shape[1], X.shape[1]
    opt = str(ScaleOption).lower()
    opt = opt if opt in ("centroid", "translation") else "centroid"
    iref = 1                                              # iRef = 2 (1-based)
    default_ref = TRef is None
    if default_ref:                                       # :58-62
        TRef, OmegaRef, XRef = np.zeros((3, m)), np.zeros((3, m)), None
    TRef, OmegaRef = (np.asarray(v, dtype=np.float64) for v in (TRef, OmegaRef))
    Tref1 = TRef[:, 0]
    Rref1 = vl_rodr(OmegaRef[:, 0])
    if opt == "centroid":
        if default_ref:   # XRef = ones(4, n) in [I | 0]: every point is (1, 1, 1)
            Sref = 1.0 / np.linalg.norm(np.ones(3))
        else:
            XRef = np.asarray(XRef, dtype=np.float64)
            Xref1 = (Rref1 @ XRef[0:3] + Tref1[:, None]) * XRef[3]
            Sref = 1.0 / np.linalg.norm(Xref1[:, XRef[3] == 1].mean(1))
    else:
        Sref = 1.0 / np.linalg.norm(Rref1.T @ Tref1 - vl_rodr(OmegaRef[:, iref]).T @ TRef[:, iref])
    R1 = vl_rodr(Omega[:, 0])
    T1 = T[:, 0]
    on = X[3] == 1                                        # :98-104
    allon = bool(on.all())
    Xon = X[0:3] if allon else X[0:3, on]
    X1 = R1 @ Xon + T1[:, None]                           # the points in camera 1's frame
    if opt == "centroid":
        S1 = 1.0 / np.linalg.norm(X1.mean(1))
    else:
        S1 = 1.0 / np.linalg.norm(R1.T @ T1 - vl_rodr(Omega[:, iref]).T @ T[:, iref])
    Rj = vl_rodr(Omega).reshape(m, 3, 3)                 # :90-97, all cameras at once
    RjR1_ = Rj @ R1.T
    Omega_ = vl_irodr(RjR1_ @ Rref1)
    T_ = (RjR1_ @ Tref1).T + S1 / Sref * (-(RjR1_ @ T1).T + T)
    X_ = np.zeros((4, n))
    Xn = Rref1.T @ (S1 / Sref * X1 - Tref1[:, None])
    if allon:
        X_[0:3] = Xn
    else:
        X_[0:3, on] = Xn
    X_[3, on] = 1.0
    return T_, Omega_, X_
