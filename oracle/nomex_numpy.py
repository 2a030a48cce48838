"""Independent numpy restatement of toolbox/bundle/bundle_euclid_nomex.m.

TEST INFRASTRUCTURE ONLY (cross-check of the C oracle; never imported by the
product).  Follows the reference's pure-MATLAB twin, vectorised over the
visible observations, with host-libm rotations (math.sin/cos) and numpy's
own reductions, so it shares no arithmetic code path with ba_oracle.c:

  reprojection_point.m:11-22, derivative_camera.m:9-13 / derivative_point.m:9-13
  (forward differences h = 1e-10, dx/||dx|| = e_k), bundle_euclid_nomex.m:123-178
  (A, B, e, U, V, W, eA, eB), :180-189 (fix masks), :197-219 (damping, pinv,
  Y), :227-258 (S, e_, da = pinv(S) e_), :269-278 (db with ALL num_a terms,
  App. A Q3), :284-302 (update), :304-338 (rho / lambda), :353-364 (output with
  Xe_(4,:) = 1, App. A Q5).
"""
from __future__ import annotations

import math

import numpy as np

import bundle_euclid_ref as _ref


def _rodrigues(w):
    """vl_rodr for a batch of rotation vectors (k, 3) -> (k, 3, 3)."""
    th = np.sqrt((w * w).sum(1))
    small = th < 1e-6
    ths = np.where(small, 1.0, th)
    x, y, z = (w / ths[:, None]).T
    # glibc sin / cos one argument at a time (numpy's vectorised sin is not libm)
    s = np.array([math.sin(t) for t in th])
    c = np.array([math.cos(t) for t in th])
    mc = 1.0 - c
    R = np.empty((w.shape[0], 3, 3))
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
    return R


def _project(Kp, a, b, nvk):
    """reprojection_point.m for batches: Kp (k,4), a (k,num_a), b (k,3)."""
    Kp = Kp.copy()
    if nvk == 1:
        Kp[:, 0] = a[:, 6]
        Kp[:, 1] = a[:, 6]
    elif nvk == 4:
        Kp = a[:, 6:10].copy()
    R = _rodrigues(a[:, 0:3])
    Xc = np.einsum("kij,kj->ki", R, b) + a[:, 3:6]
    x0 = Kp[:, 0] * Xc[:, 0] + Kp[:, 2] * Xc[:, 2]
    x1 = Kp[:, 1] * Xc[:, 1] + Kp[:, 3] * Xc[:, 2]
    return np.stack([x0 / Xc[:, 2], x1 / Xc[:, 2]], 1)


def bundle_euclid_nomex(K, Te, w, Xe, x, *varargin, stop_rel=1e-3, max_iter=20, max_iter2=10):
    """stop_rel / max_iter / max_iter2: the stop rule's constants
    (bundle_euclid_nomex.m:106-109: 1e-3, 20, 10), exposed so that a test can
    run both twins to convergence."""
    K, Te, w, Xe, x = map(np.asarray, (K, Te, w, Xe, x))
    m, n = w.shape[1], x.shape[1]
    o = _ref.parse_options(m, n, x, varargin)
    nvk = o["num_variableK"]
    vis = o["visible"]
    num_vis = vis.sum()
    num_a = 6 + nvk
    a = np.array(_ref.pack_a(K, Te, w, nvk))
    b = np.array(Xe[0:3], dtype=np.float64)
    pt, cam = np.nonzero(vis)
    N = len(pt)
    Xo = np.stack([x[0, pt, cam], x[1, pt, cam]], 1)
    h = 1e-10
    lam, nu = 0.001, 2.0
    it, it2 = 1, 0
    err = []
    while it < max_iter and it2 < max_iter2 and (
            it < 3 or (err[it - 1] > 1e-20 and
                       err[it - 2] - err[it - 1] > stop_rel * err[it - 2])):
        ao, bo, Ko = a[:, cam].T, b[:, pt].T, K[:, cam].T
        xh = _project(Ko, ao, bo, nvk)
        A = np.zeros((N, 2, num_a))
        B = np.zeros((N, 2, 3))
        for k in range(num_a):
            d = np.zeros(num_a); d[k] = 1.0
            A[:, :, k] = (_project(Ko, ao + h * d, bo, nvk) - xh) / h
        for k in range(3):
            d = np.zeros(3); d[k] = 1.0
            B[:, :, k] = (_project(Ko, ao, bo + h * d, nvk) - xh) / h
        e = Xo - xh
        U = np.zeros((m, num_a, num_a)); V = np.zeros((n, 3, 3))
        eA = np.zeros((m, num_a)); eB = np.zeros((n, 3))
        np.add.at(U, cam, np.einsum("kri,krj->kij", A, A))
        np.add.at(V, pt, np.einsum("kri,krj->kij", B, B))
        W = np.einsum("kri,krj->kij", A, B)
        np.add.at(eA, cam, np.einsum("kri,kr->ki", A, e))
        np.add.at(eB, pt, np.einsum("kri,kr->ki", B, e))
        if o["fix_structure"]:
            V[:] = 0; W[:] = 0; eB[:] = 0
        if o["fix_motion"]:
            U[:] = 0; W[:] = 0; eA[:] = 0
        Us = U.copy(); Vs = V.copy()
        di = np.arange(num_a)
        Us[:, di, di] *= (1 + lam)
        Vs[:, [0, 1, 2], [0, 1, 2]] *= (1 + lam)
        Vinv = np.stack([np.linalg.pinv(v) if np.any(v) else np.zeros((3, 3)) for v in Vs])
        Y = np.einsum("kij,kjl->kil", W, Vinv[pt])
        S = np.zeros((num_a * m, num_a * m))
        for j in range(m):
            S[num_a * j:num_a * j + num_a, num_a * j:num_a * j + num_a] = Us[j]
        ptr = np.concatenate([[0], np.cumsum(np.bincount(pt, minlength=n))])
        for i in range(n):
            for p in range(ptr[i], ptr[i + 1]):
                for q in range(ptr[i], ptr[i + 1]):
                    j, k = cam[p], cam[q]
                    S[num_a * j:num_a * j + num_a, num_a * k:num_a * k + num_a] -= Y[p] @ W[q].T
        YeB = np.zeros((m, num_a))
        np.add.at(YeB, cam, np.einsum("kij,kj->ki", Y, eB[pt]))
        e_ = (eA - YeB).reshape(-1)
        da = np.linalg.pinv(S) @ e_
        WtDa = np.zeros((n, 3))
        np.add.at(WtDa, pt, np.einsum("kij,ki->kj", W, da.reshape(m, num_a)[cam]))
        db = np.einsum("kij,kj->ki", Vinv, eB - WtDa)
        a_new = a + da.reshape(m, num_a).T
        b_new = b + db.T
        xn = _project(Ko, a_new[:, cam].T, b_new[:, pt].T, nvk)
        en = Xo - xn
        old, new = float((e * e).sum()), float((en * en).sum())
        g = np.concatenate([eA.reshape(-1), eB.reshape(-1)])
        dp = np.concatenate([da, db.reshape(-1)])
        rho = (old - new) / float(dp @ (lam * dp + g))
        if old - new > 0:
            a, b = a_new, b_new
            lam *= max(1 / 3, 1 - (2 * rho - 1) ** 3)
            nu = 2.0
            if len(err) < it:
                err.append(old / num_vis)
            else:
                err[it - 1] = old / num_vis
            it += 1
            err.append(new / num_vis)
            it2 = 0
        else:
            lam *= nu
            nu *= 2
            it2 += 1
    K_, Te_, w_, _ = _ref.unpack(K, a, b, Xe, nvk)
    return K_, Te_, w_, np.vstack([b, np.ones((1, n))]), np.array(err)
