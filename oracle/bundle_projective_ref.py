"""CPU oracle for the projective LM path -- TEST INFRASTRUCTURE ONLY.

Restates ``toolbox/bundle/bundle_projective.m`` (the MATLAB driver) in numpy
on top of the C restatement of its three MEX stages (``oracle/ba_oracle.c``
with num_a = 12: ``mex_bundle_proj_1_XABeUVWeAeB.c``, ``mex_bundle_proj_2_Se_.c``,
``mex_bundle_proj_3_db_new.c``).  Only ``tests/`` and ``bench.py``'s
``cpu_baseline`` leg may import this module; the product never does.

PARITY STATUS: "parity unpinned" (same reasons as bundle_euclid_ref.py: no
MATLAB, the MEX sources need MATLAB's mx API, no golden vectors in the
reference).  ``bundle_projective_nomex`` below is an independent numpy
restatement of the pure-MATLAB twin ``bundle_projective_nomex.m`` used as the
cross-check.

Differences from the Euclidean driver that the restatement keeps
(bundle_projective.m):
  * a(:,j) = Pp(:,:,j)(:) (12 x m, :70-73); b = Xp(1:3,:) (:76) -- the 4th
    homogeneous coordinate is ignored on input and copied to the output (:227)
  * no fix_pivot / fix_calibration options (:46-56)
  * old_error / new_error are normalised by num_vis BEFORE the comparison
    (:182-188): accept iff new_error < old_error
  * lambda / 10 on accept, lambda * 10 on reject (:195, :205) -- no rho, no nu
  * mex_bundle_proj_3_db_new.c:107-121 uses only da(1:6,j) in db (App. A Q3);
    the nomex twin uses all 12 (bundle_projective_nomex.m:247-256)
"""
from __future__ import annotations

import numpy as np

import bundle_euclid_ref as _e
from bundle_euclid_ref import F, P

NUM_A = 12


def mex1(a, b, X, vis, lib=None):
    """mex_bundle_proj_1_XABeUVWeAeB(a, b, X, visible) -> (X_hat A B e U V W eA eB)."""
    lib = lib or _e._lib()
    a, b, X, vis = F(a), F(b), F(X), F(vis)
    num_a, m = a.shape
    assert num_a == NUM_A
    n = b.shape[1]
    z = lambda *s: np.zeros(s, order="F")
    out = [z(2, n, m), z(2, num_a, n, m), z(2, 3, n, m), z(2, n, m), z(num_a, num_a, m),
           z(3, 3, n), z(num_a, 3, n, m), z(num_a, m), z(3, n)]
    lib.oracle_mex1(m, n, num_a, None, P(a), P(b), P(X), P(vis), *[P(o) for o in out])
    return tuple(out)


mex2 = _e.mex2   # mex_bundle_proj_2_Se_.c == mex_bundle_2_Se_.c with num_a = 12


def mex3(W, da, eB, Vinv, a, b, X, vis, lib=None):
    """mex_bundle_proj_3_db_new(W, da, eB, V_inv, a, b, X, visible) -> (db a_new b_new X_hat)."""
    lib = lib or _e._lib()
    W, da, eB, Vinv, a, b, X, vis = map(F, (W, da, eB, Vinv, a, b, X, vis))
    num_a, m = a.shape
    n = b.shape[1]
    db = np.zeros((3, n), order="F")
    a_new = np.zeros((num_a, m), order="F")
    b_new = np.zeros((3, n), order="F")
    X_hat = np.zeros((2, n, m), order="F")
    lib.oracle_mex3(m, n, num_a, P(W), P(da), P(eB), P(Vinv), None, P(a), P(b), P(X), P(vis),
                    P(db), P(a_new), P(b_new), P(X_hat))
    return db, a_new, b_new, X_hat


def parse_options(m, n, x, varargin):
    """bundle_projective.m:36-63."""
    o = dict(fix_structure=False, fix_motion=False, visible=None, verbose=False)
    k = 0
    while k < len(varargin):
        name = str(varargin[k]).lower()
        if name == "fix_structure":
            o["fix_structure"] = True
        elif name == "fix_motion":
            o["fix_motion"] = True
        elif name == "visibility":
            o["visible"] = np.asarray(varargin[k + 1])
            k += 1
        elif name == "verbose":
            o["verbose"] = True
        k += 1
    if o["visible"] is None:
        o["visible"] = (x[0] != 0) | (x[1] != 0)
    o["visible"] = np.asarray(o["visible"], dtype=np.float64).reshape(n, m)
    return o


def pack_a(Pp):
    """bundle_projective.m:70-73: a(1:12,j) = reshape(Pp(:,:,j),12,1)."""
    Pp = F(Pp)
    m = Pp.shape[2]
    return F(Pp.reshape(12, m, order="F"))


def unpack(a, b, Xp):
    """bundle_projective.m:221-227."""
    m = a.shape[1]
    return F(np.asarray(a).reshape(3, 4, m, order="F")), np.vstack([b, np.asarray(Xp)[3:4]])


def bundle_projective_ref(Pp, Xp, x, *varargin, form="dense", vinv="pinv", solve="pinv",
                          lib=None, trace=None, semantics="mex"):
    """[Pp_ Xp_ error_] = bundle_projective(Pp, Xp, x, ...) restated.

    semantics="nomex": the back substitution uses all 12 camera parameters
    (bundle_projective_nomex.m:247-256); requires form="sparse"."""
    nomex = semantics == "nomex"
    assert semantics in ("mex", "nomex") and (form == "sparse" or not nomex)
    lib = lib or _e._lib()
    Pp, Xp, x = F(Pp), F(Xp), F(x)
    m = Pp.shape[2]
    n = x.shape[1]
    o = parse_options(m, n, x, varargin)
    vis = F(o["visible"])
    num_vis = vis.sum()
    a = pack_a(Pp)
    b = F(Xp[0:3])
    X = F(x[0:2])
    if form == "sparse":
        pt, cam, _ = _e.obs_from_visibility(vis)
        obs_x = np.stack([X[0, pt, cam], X[1, pt, cam]], axis=1)
        pb = _e.SparseProblem(m, n, pt, cam, obs_x, np.zeros((4, m)))
        pb.K = None
    lam = 0.001
    it, it2, max_iter, max_iter2 = 1, 0, 20, 10
    err: list = []

    def cont():
        if not (it < max_iter and it2 < max_iter2):
            return False
        if it < 3:
            return True
        return err[it - 1] > 1e-20 and err[it - 2] - err[it - 1] > 1e-3 * err[it - 2]

    while cont():
        if form == "dense":                                          # :116
            X_hat, A, B, e, U, V, W, eA, eB = mex1(a, b, X, vis, lib)
        else:
            L = _sp_linearize(pb, a, b, lib)
            e, U, V, W, eA, eB = L["e"], L["U"], L["V"], L["W"], L["eA"], L["eB"]
        if o["fix_structure"]:                                       # :117-121
            V[:] = 0; W[:] = 0; eB[:] = 0
        if o["fix_motion"]:                                          # :122-126
            U[:] = 0; W[:] = 0; eA[:] = 0
        Us = U.copy(order="F")                                       # :134-145
        for k in range(NUM_A):
            Us[k, k, :] = (1 + lam) * U[k, k, :]
        Vs = V.copy(order="F")
        for k in range(3):
            Vs[k, k, :] = (1 + lam) * V[k, k, :]
        Vinv = _e.matlab_pinv(Vs) if vinv == "pinv" else _e.pinv3_formula(Vs, lib)   # :150-156
        Vinv = F(Vinv)
        if form == "dense":
            Y = _e.y_dense(W, Vinv)
            S, e_ = mex2(Y, W, Us, eA, eB, lib)                      # :164
        else:
            Y = _e.sp_y(pb, W, Vinv, NUM_A, lib)
            S, e_ = _e.sp_schur(pb, Y, W, Us, eA, eB, NUM_A, lib)
        da = _e.matlab_pinv(S) @ e_ if solve == "pinv" else _e.chol_solve_fixed(S, e_)  # :165
        da = F(da)
        if form == "dense":                                          # :177-183
            db, a_new, b_new, X_hat_new = mex3(W, da, eB, Vinv, a, b, X, vis, lib)
            e_new = X - X_hat_new
            es, ens = e.reshape(-1, order="F"), e_new.reshape(-1, order="F")
        else:
            db, a_new, b_new, xh, _ = _e.sp_update(pb, W, da, eB, Vinv, a, b, NUM_A, lib,
                                                   ndb=NUM_A if nomex else 6)
            es, ens = e.reshape(-1), (pb.obs_x - xh).reshape(-1)
        old_error = 1 / num_vis * float(es @ es)
        new_error = 1 / num_vis * float(ens @ ens)
        accepted = new_error < old_error                             # :188
        if trace is not None:
            trace.append(dict(lam=lam, accepted=bool(accepted), old=old_error, new=new_error,
                              da=da.copy(), db=db.copy()))
        if accepted:
            if o["verbose"]:
                print(f"iter {it}: error= {old_error:g} -> {new_error:g}")
            a, b = a_new, b_new
            lam = lam / 10                                           # :195
            if len(err) < it:
                err.append(old_error)
            else:
                err[it - 1] = old_error
            it += 1
            err.append(new_error)
            it2 = 0
        else:
            lam = lam * 10                                           # :205
            it2 += 1
    Pp_, Xp_ = unpack(a, b, Xp)
    return Pp_, Xp_, np.array(err)


def _sp_linearize(pb, a, b, lib):
    N, m, n = pb.N, pb.m, pb.n
    a, b = F(a), F(b)
    xh = np.zeros((N, 2)); A = np.zeros((N, 2 * NUM_A)); B = np.zeros((N, 6))
    e = np.zeros((N, 2)); W = np.zeros((N, 3 * NUM_A))
    U = np.zeros((NUM_A, NUM_A, m), order="F"); V = np.zeros((3, 3, n), order="F")
    eA = np.zeros((NUM_A, m), order="F"); eB = np.zeros((3, n), order="F")
    lib.oracle_sp_linearize(m, n, NUM_A, P(pb.pt_ptr), P(pb.obs_cam), P(pb.obs_x), None,
                            P(a), P(b), P(xh), P(A), P(B), P(e), P(U), P(V), P(W), P(eA),
                            P(eB))
    return dict(xh=xh, A=A, B=B, e=e, W=W, U=U, V=V, eA=eA, eB=eB)


# --------------------------------------------------------------------------
# independent numpy twin of bundle_projective_nomex.m (cross-check only)
# --------------------------------------------------------------------------
def _project(a, b):
    """reprojection_projective_point.m:10-11 for batches a (k,12), b (k,3)."""
    Pm = a.reshape(-1, 4, 3).transpose(0, 2, 1)      # (k, 3, 4): column-major 3x4
    x_ = np.einsum("kij,kj->ki", Pm[:, :, :3], b) + Pm[:, :, 3]
    return x_[:, :2] / x_[:, 2:3]


def bundle_projective_nomex(Pp, Xp, x, *varargin):
    """bundle_projective_nomex.m restated with numpy reductions (libm-free:
    the projective camera has no trigonometry)."""
    Pp, Xp, x = map(np.asarray, (Pp, Xp, x))
    m, n = Pp.shape[2], x.shape[1]
    o = parse_options(m, n, x, varargin)
    vis = o["visible"]
    num_vis = vis.sum()
    a = np.array(pack_a(Pp))
    b = np.array(Xp[0:3], dtype=np.float64)
    pt, cam = np.nonzero(vis)
    N = len(pt)
    Xo = np.stack([x[0, pt, cam], x[1, pt, cam]], 1)
    h = 1e-10
    lam = 0.001
    it, it2 = 1, 0
    err = []
    while it < 20 and it2 < 10 and (it < 3 or (err[it - 1] > 1e-20 and
                                               err[it - 2] - err[it - 1] > 1e-3 * err[it - 2])):
        ao, bo = a[:, cam].T, b[:, pt].T
        xh = _project(ao, bo)
        A = np.zeros((N, 2, NUM_A))
        B = np.zeros((N, 2, 3))
        for k in range(NUM_A):                   # derivative_projective_camera.m:9-14
            d = np.zeros(NUM_A); d[k] = 1.0
            A[:, :, k] = (_project(ao + h * d, bo) - xh) / h
        for k in range(3):
            d = np.zeros(3); d[k] = 1.0
            B[:, :, k] = (_project(ao, bo + h * d) - xh) / h
        e = Xo - xh
        U = np.zeros((m, NUM_A, NUM_A)); V = np.zeros((n, 3, 3))
        eA = np.zeros((m, NUM_A)); eB = np.zeros((n, 3))
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
        di = np.arange(NUM_A)
        Us[:, di, di] *= (1 + lam)
        Vs[:, [0, 1, 2], [0, 1, 2]] *= (1 + lam)
        Vinv = np.stack([np.linalg.pinv(v) if np.any(v) else np.zeros((3, 3)) for v in Vs])
        Y = np.einsum("kij,kjl->kil", W, Vinv[pt])
        S = np.zeros((NUM_A * m, NUM_A * m))
        for j in range(m):
            S[NUM_A * j:NUM_A * (j + 1), NUM_A * j:NUM_A * (j + 1)] = Us[j]
        ptr = np.concatenate([[0], np.cumsum(np.bincount(pt, minlength=n))])
        for i in range(n):
            for p in range(ptr[i], ptr[i + 1]):
                for q in range(ptr[i], ptr[i + 1]):
                    j, k = cam[p], cam[q]
                    S[NUM_A * j:NUM_A * (j + 1), NUM_A * k:NUM_A * (k + 1)] -= Y[p] @ W[q].T
        YeB = np.zeros((m, NUM_A))
        np.add.at(YeB, cam, np.einsum("kij,kj->ki", Y, eB[pt]))
        e_ = (eA - YeB).reshape(-1)
        da = np.linalg.pinv(S) @ e_
        WtDa = np.zeros((n, 3))
        np.add.at(WtDa, pt, np.einsum("kij,ki->kj", W, da.reshape(m, NUM_A)[cam]))
        db = np.einsum("kij,kj->ki", Vinv, eB - WtDa)
        a_new = a + da.reshape(m, NUM_A).T
        b_new = b + db.T
        en = Xo - _project(a_new[:, cam].T, b_new[:, pt].T)
        old, new = float((e * e).sum()) / num_vis, float((en * en).sum()) / num_vis
        if new < old:
            a, b = a_new, b_new
            lam /= 10
            if len(err) < it:
                err.append(old)
            else:
                err[it - 1] = old
            it += 1
            err.append(new)
            it2 = 0
        else:
            lam *= 10
            it2 += 1
    return F(a.reshape(3, 4, m, order="F")), np.vstack([b, Xp[3:4]]), np.array(err)
