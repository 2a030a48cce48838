"""CPU oracle for the Euclidean LM path -- TEST INFRASTRUCTURE ONLY.

Restates ``toolbox/bundle/bundle_euclid.m`` (the MATLAB driver) in numpy on top
of the C restatement of its three MEX stages (``oracle/ba_oracle.c``).  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module; the product (``bundleadjustmentmatlab_amd``) never does.

PARITY STATUS: "parity unpinned" -- the reference (MATLAB + MEX needing
MATLAB's mx API and VLFeat) cannot run in this image and ships no golden
vectors; see DESIGN.md "Oracle".  Cross-checks live in tests/test_oracle.py.

Knobs (all default to the reference's semantics):
  form  = 'dense'  -> oracle_mex1/2/3 on the n x m MEX layouts (configs 1-2)
          'sparse' -> oracle_sp_* on the point-major observation list
  vinv  = 'pinv'   -> MATLAB pinv of each damped 3x3 block (SVD, tol =
                      max(size)*eps(sigma_max)), bundle_euclid.m:180
          'formula'-> the closed-form 3x3 pinv the GPU uses, restated in
                      oracle/orc_math.h (bit-exact chain; bounded vs 'pinv')
  solve = 'pinv'   -> da = pinv(S) * e_ (bundle_euclid.m:193)
          'chol'   -> Cholesky with exact-zero rows fixed (the device's rule)
          'seq'    -> oracle_chol_seq: left-looking Cholesky, sums in index
                      order (the GPU's parity-mode solve, bit for bit); pinv
                      on a non-positive pivot
  sums  = 'blas'   -> e'e and dp'(lambda dp + g) as numpy dots
          'seq'    -> sequential sums in MATLAB's flat (column-major) order
                      (the GPU's parity mode)
  stop_rel / max_iter / max_iter2 / lambda0: the LM constants of
          bundle_euclid.m:111-123 (defaults 1e-3 / 20 / 10 / 1e-3)
"""
from __future__ import annotations

import ctypes
import os
import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIBS: dict = {}

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)


def _lib(variant: str = ""):
    """Load build/libba_oracle{variant}.so (built by oracle/Makefile)."""
    if variant not in _LIBS:
        path = os.path.join(_HERE, "build", f"libba_oracle{variant}.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.run(["make", "-C", _HERE], check=True, capture_output=True)
        lib = ctypes.CDLL(path)
        lib.oracle_sp_update.restype = ctypes.c_double
        lib.oracle_sp_update_nd.restype = ctypes.c_double
        lib.oracle_seq_dot.restype = ctypes.c_double
        lib.oracle_seq_dot.argtypes = [_dp, _dp, ctypes.c_longlong]
        lib.oracle_seq_dpg.restype = ctypes.c_double
        lib.oracle_seq_dpg.argtypes = [_dp, _dp, ctypes.c_double, ctypes.c_longlong]
        lib.oracle_chol_seq.restype = ctypes.c_int
        lib.oracle_chol_seq.argtypes = [ctypes.c_int, _dp, _dp, _dp]
        _LIBS[variant] = lib
    return _LIBS[variant]


def P(a):
    """ctypes pointer to a contiguous float64 / int32 numpy buffer (None -> NULL)."""
    if a is None:
        return None
    if a.dtype == np.float64:
        assert a.flags.c_contiguous or a.flags.f_contiguous
        return a.ctypes.data_as(_dp)
    if a.dtype == np.int32:
        assert a.flags.c_contiguous
        return a.ctypes.data_as(_ip)
    raise TypeError(a.dtype)


def F(a):
    return np.asfortranarray(a, dtype=np.float64)


# --------------------------------------------------------------------------
# Stage wrappers (MEX argument layouts; arrays are MATLAB-shaped, Fortran order)
# --------------------------------------------------------------------------
def mex1(K, a, b, X, vis, lib=None):
    """mex_bundle_1_XABeUVWeAeB(K, a, b, X, visible) -> (X_hat A B e U V W eA eB)."""
    lib = lib or _lib()
    K, a, b, X, vis = F(K), F(a), F(b), F(X), F(vis)
    num_a, m = a.shape
    n = b.shape[1]
    z = lambda *s: np.zeros(s, order="F")
    out = [z(2, n, m), z(2, num_a, n, m), z(2, 3, n, m), z(2, n, m), z(num_a, num_a, m),
           z(3, 3, n), z(num_a, 3, n, m), z(num_a, m), z(3, n)]
    lib.oracle_mex1(m, n, num_a, P(K), P(a), P(b), P(X), P(vis), *[P(o) for o in out])
    return tuple(out)


def mex2(Y, W, Us, eA, eB, lib=None):
    """mex_bundle_2_Se_(Y, W, U*, eA, eB) -> (S, e_)."""
    lib = lib or _lib()
    Y, W, Us, eA, eB = F(Y), F(W), F(Us), F(eA), F(eB)
    num_a, m = eA.shape
    n = eB.shape[1]
    S = np.zeros((num_a * m, num_a * m), order="F")
    e_ = np.zeros((num_a * m, 1), order="F")
    lib.oracle_mex2(m, n, num_a, P(Y), P(W), P(Us), P(eA), P(eB), P(S), P(e_))
    return S, e_


def mex3(W, da, eB, Vinv, K, a, b, X, vis, lib=None):
    """mex_bundle_3_db_new(W, da, eB, V_inv, K, a, b, X, visible) -> (db a_new b_new X_hat)."""
    lib = lib or _lib()
    W, da, eB, Vinv, K, a, b, X, vis = map(F, (W, da, eB, Vinv, K, a, b, X, vis))
    num_a, m = a.shape
    n = b.shape[1]
    db = np.zeros((3, n), order="F")
    a_new = np.zeros((num_a, m), order="F")
    b_new = np.zeros((3, n), order="F")
    X_hat = np.zeros((2, n, m), order="F")
    lib.oracle_mex3(m, n, num_a, P(W), P(da), P(eB), P(Vinv), P(K), P(a), P(b), P(X), P(vis),
                    P(db), P(a_new), P(b_new), P(X_hat))
    return db, a_new, b_new, X_hat


# --------------------------------------------------------------------------
# MATLAB pinv and the solves
# --------------------------------------------------------------------------
def matlab_pinv(A):
    """MATLAB pinv: SVD, tol = max(size(A)) * eps(max singular value)."""
    A = np.asarray(A, dtype=np.float64)
    if A.ndim == 2:
        if not np.any(A):
            return np.zeros(A.T.shape)
        U, s, Vt = np.linalg.svd(A, full_matrices=False)
        tol = max(A.shape) * np.spacing(s.max())
        r = s > tol
        return (Vt[r].T / s[r]) @ U[:, r].T
    # batched over a trailing axis: A is (3, 3, n) MATLAB-shaped
    B = np.moveaxis(A, -1, 0)
    U, s, Vt = np.linalg.svd(B)
    tol = (max(B.shape[1:]) * np.spacing(s.max(axis=1)))[:, None]
    sinv = np.where(s > tol, 1.0 / np.where(s > tol, s, 1.0), 0.0)
    Pi = np.einsum("nji,nj,nkj->nik", Vt, sinv, U)
    return np.moveaxis(Pi, 0, -1)


def chol_solve_fixed(S, e_):
    """Cholesky solve treating exact-zero diagonal rows as fixed (da = 0)."""
    import scipy.linalg as sl
    S = np.array(S, dtype=np.float64)
    d = np.diag(S).copy()
    zero = d == 0.0
    S[zero, :] = 0.0
    S[:, zero] = 0.0
    S[zero, zero] = 1.0
    rhs = np.array(e_, dtype=np.float64).reshape(-1).copy()
    rhs[zero] = 0.0
    c = sl.cho_factor(S, lower=True, check_finite=False)
    return sl.cho_solve(c, rhs, check_finite=False).reshape(-1, 1)


def chol_seq(S, e_, lib=None):
    """oracle_chol_seq on a copy of S: (da (ld, 1), rc); rc != 0 = non-positive pivot."""
    lib = lib or _lib()
    A = np.array(S, dtype=np.float64, order="F")
    rhs = np.ascontiguousarray(np.array(e_, dtype=np.float64).reshape(-1))
    da = np.zeros_like(rhs)
    rc = lib.oracle_chol_seq(A.shape[0], P(A), P(rhs), P(da))
    return da.reshape(-1, 1), rc


def seq_dot(v, lib=None):
    lib = lib or _lib()
    v = np.ascontiguousarray(v, dtype=np.float64).reshape(-1)
    return float(lib.oracle_seq_dot(P(v), P(v), v.size))


def seq_dpg(dp, g, lam, lib=None):
    lib = lib or _lib()
    dp = np.ascontiguousarray(dp, dtype=np.float64).reshape(-1)
    g = np.ascontiguousarray(g, dtype=np.float64).reshape(-1)
    return float(lib.oracle_seq_dpg(P(dp), P(g), float(lam), dp.size))


def pinv3_formula(Vs, lib=None):
    """orc_pinv3_formula (oracle/orc_math.h) applied to each (3,3,i) block."""
    lib = lib or _lib()
    Vs = F(Vs)
    out = np.zeros_like(Vs, order="F")
    for i in range(Vs.shape[2]):
        blk = np.ascontiguousarray(Vs[:, :, i].reshape(-1, order="F"))
        o = np.zeros(9)
        lib.oracle_pinv3(P(blk), P(o))
        out[:, :, i] = o.reshape(3, 3, order="F")
    return out


def y_dense(W, Vinv):
    """Y_ij = W_ij * V_inv_i (bundle_euclid.m:182), each entry summed t = 0,1,2."""
    t = [W[:, k][:, None, :, :] * Vinv[k][None, :, :, None] for k in range(3)]
    return F((t[0] + t[1]) + t[2])


# --------------------------------------------------------------------------
# Observation list helpers
# --------------------------------------------------------------------------
def obs_from_visibility(vis):
    """Point-major observation list of the non-zero entries of vis (n x m)."""
    vis = np.asarray(vis)
    pt, cam = np.nonzero(vis)           # row-major nonzero: point ascending, camera ascending
    n = vis.shape[0]
    pt_ptr = np.zeros(n + 1, dtype=np.int32)
    np.add.at(pt_ptr, pt + 1, 1)
    pt_ptr = np.cumsum(pt_ptr).astype(np.int32)
    return pt.astype(np.int32), cam.astype(np.int32), pt_ptr


class SparseProblem:
    """Observation-list form: obs_pt/obs_cam sorted point-major, obs_x (N,2)."""

    def __init__(self, m, n, obs_pt, obs_cam, obs_x, K):
        self.m, self.n = int(m), int(n)
        self.obs_pt = np.ascontiguousarray(obs_pt, dtype=np.int32)
        self.obs_cam = np.ascontiguousarray(obs_cam, dtype=np.int32)
        self.obs_x = np.ascontiguousarray(obs_x, dtype=np.float64).reshape(-1, 2)
        self.K = F(K)
        cnt = np.bincount(self.obs_pt, minlength=self.n)
        self.pt_ptr = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
        self.N = len(self.obs_pt)


def sp_linearize(pb, a, b, num_a, lib=None):
    lib = lib or _lib()
    N, m, n = pb.N, pb.m, pb.n
    a, b = F(a), F(b)
    xh = np.zeros((N, 2)); A = np.zeros((N, 2 * num_a)); B = np.zeros((N, 6))
    e = np.zeros((N, 2)); W = np.zeros((N, 3 * num_a))
    U = np.zeros((num_a, num_a, m), order="F"); V = np.zeros((3, 3, n), order="F")
    eA = np.zeros((num_a, m), order="F"); eB = np.zeros((3, n), order="F")
    lib.oracle_sp_linearize(m, n, num_a, P(pb.pt_ptr), P(pb.obs_cam), P(pb.obs_x), P(pb.K),
                            P(a), P(b), P(xh), P(A), P(B), P(e), P(U), P(V), P(W), P(eA),
                            P(eB))
    return dict(xh=xh, A=A, B=B, e=e, W=W, U=U, V=V, eA=eA, eB=eB)


def sp_y(pb, W, Vinv, num_a, lib=None):
    lib = lib or _lib()
    Y = np.zeros_like(W)
    lib.oracle_sp_y(pb.n, num_a, P(pb.pt_ptr), P(W), P(F(Vinv)), P(Y))
    return Y


def sp_schur(pb, Y, W, Us, eA, eB, num_a, lib=None):
    lib = lib or _lib()
    ld = num_a * pb.m
    S = np.zeros((ld, ld), order="F")
    e_ = np.zeros((ld, 1), order="F")
    lib.oracle_sp_schur(pb.m, pb.n, num_a, P(pb.pt_ptr), P(pb.obs_cam), P(Y), P(W), P(F(Us)),
                        P(F(eA)), P(F(eB)), P(S), P(e_))
    return S, e_


def sp_update(pb, W, da, eB, Vinv, a, b, num_a, lib=None, ndb=6):
    """mex_bundle_3_db_new.c:99-166 on the observation list; ndb = num_a gives
    the back substitution of bundle_euclid_nomex.m:268-277 instead."""
    lib = lib or _lib()
    db = np.zeros((3, pb.n), order="F")
    a_new = np.zeros((num_a, pb.m), order="F")
    b_new = np.zeros((3, pb.n), order="F")
    xh = np.zeros((pb.N, 2))
    sse = lib.oracle_sp_update_nd(pb.m, pb.n, num_a, ndb, P(pb.pt_ptr), P(pb.obs_cam),
                                  P(pb.obs_x), P(W), P(F(da)), P(F(eB)), P(F(Vinv)),
                                  None if pb.K is None else P(pb.K),
                                  P(F(a)), P(F(b)), P(db), P(a_new), P(b_new), P(xh))
    return db, a_new, b_new, xh, sse


# --------------------------------------------------------------------------
# The driver: bundle_euclid.m restated
# --------------------------------------------------------------------------
def _matlab_index_mask(idx, m):
    """Which pages of an m-page array MATLAB's X(:,:,idx) = 0 addresses
    (bundle_euclid.m:151): logical idx -> its true positions (any length, none
    past m), numeric idx -> the 1-based positions it lists.  Positions past m
    (MATLAB would grow the array) and non-positive / fractional indices
    (MATLAB errors) raise."""
    a = np.asarray(idx)
    pos = np.flatnonzero(a.reshape(-1)) if a.dtype == bool else a.reshape(-1) - 1
    pos = np.asarray(pos, dtype=np.float64)
    if pos.size and (np.any(pos != np.round(pos)) or pos.min() < 0 or pos.max() >= m):
        raise ValueError("pivot index outside 1..m")
    out = np.zeros(m, dtype=bool)
    out[pos.astype(np.int64)] = True
    return out


def parse_options(m, n, x, varargin):
    """bundle_euclid.m:44-82."""
    o = dict(fix_structure=False, fix_motion=False, fix_pivot=False,
             pivot=np.zeros(m, dtype=bool), num_variableK=4, visible=None, verbose=False)
    k = 0
    while k < len(varargin):
        name = str(varargin[k]).lower()
        if name == "fix_structure":
            o["fix_structure"] = True
        elif name == "fix_motion":
            o["fix_motion"] = True
        elif name == "fix_pivot":
            o["fix_pivot"] = True
            o["pivot"] = _matlab_index_mask(varargin[k + 1], m)
            k += 1
        elif name == "fix_calibration":
            o["num_variableK"] = 0
        elif name == "fix_principal":
            o["num_variableK"] = 1
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


def pack_a(K, Te, w, nvk):
    """bundle_euclid.m:89-96."""
    m = w.shape[1]
    a = np.zeros((6 + nvk, m), order="F")
    a[0:3] = w
    a[3:6] = Te
    if nvk == 1:
        a[6] = K[0]
    elif nvk == 4:
        a[6:10] = K
    return a


def unpack(K, a, b, Xe, nvk):
    """bundle_euclid.m:255-267."""
    K_ = np.array(K, dtype=np.float64)
    if nvk == 1:
        K_[0] = a[6]
        K_[1] = a[6]
    elif nvk == 4:
        K_[:] = a[6:10]
    return K_, a[3:6].copy(), a[0:3].copy(), np.vstack([b, Xe[3:4]])


def bundle_euclid_ref(K, Te, w, Xe, x, *varargin, form="dense", vinv="pinv", solve="pinv",
                      lib=None, trace=None, semantics="mex", sums="blas", stop_rel=1e-3,
                      max_iter=20, max_iter2=10, lambda0=1e-3):
    """[K_ Te_ w_ Xe_ error_] = bundle_euclid(K, Te, w, Xe, x, ...) restated.

    trace: optional list; per iteration a dict (lambda, accepted, old, new, rho)
    is appended.  semantics="nomex" restates bundle_euclid_nomex.m instead: the
    back substitution uses every camera parameter (:268-277), 'fix_pivot' is
    not an option (ignored), Xe_(4,:) = 1 (:364); requires form="sparse".
    """
    nomex = semantics == "nomex"
    assert semantics in ("mex", "nomex") and (form == "sparse" or not nomex)
    lib = lib or _lib()
    K, Te, w, Xe, x = F(K), F(Te), F(w), F(Xe), F(x)
    m = w.shape[1]
    n = x.shape[1]
    o = parse_options(m, n, x, varargin)
    if nomex:
        o["fix_pivot"] = False
    nvk = o["num_variableK"]
    vis = F(o["visible"])
    num_vis = vis.sum()
    num_a = 6 + nvk
    a = pack_a(K, Te, w, nvk)
    b = F(Xe[0:3])
    X = F(x[0:2])
    if form == "sparse":
        pt, cam, _ = obs_from_visibility(vis)
        obs_x = np.stack([X[0, pt, cam], X[1, pt, cam]], axis=1)
        pb = SparseProblem(m, n, pt, cam, obs_x, K)
    lam, nu = lambda0, 2.0
    it, it2 = 1, 0
    err: list = []
    if form == "sparse" and sums == "seq":   # camera-major: MATLAB's e(:) order
        cm = np.lexsort((pb.obs_pt, pb.obs_cam))

    def cont():
        if not (it < max_iter and it2 < max_iter2):
            return False
        if it < 3:
            return True
        return err[it - 1] > 1e-20 and err[it - 2] - err[it - 1] > stop_rel * err[it - 2]

    while cont():
        # (ii)-(iii) linearisation, bundle_euclid.m:139
        if form == "dense":
            X_hat, A, B, e, U, V, W, eA, eB = mex1(K, a, b, X, vis, lib)
        else:
            L = sp_linearize(pb, a, b, num_a, lib)
            e, U, V, W, eA, eB = L["e"], L["U"], L["V"], L["W"], L["eA"], L["eB"]
        # fix masks, bundle_euclid.m:140-154
        if o["fix_structure"]:
            V[:] = 0; W[:] = 0; eB[:] = 0
        if o["fix_motion"]:
            U[:] = 0; W[:] = 0; eA[:] = 0
        if o["fix_pivot"]:
            pv = o["pivot"]
            U[:, :, pv] = 0; eA[:, pv] = 0
            if form == "dense":
                W[:, :, :, pv] = 0
            else:
                W[pv[pb.obs_cam]] = 0
        # (iv) damping, :162-173
        Us = U.copy(order="F")
        for k in range(num_a):
            Us[k, k, :] = (1 + lam) * U[k, k, :]
        Vs = V.copy(order="F")
        for k in range(3):
            Vs[k, k, :] = (1 + lam) * V[k, k, :]
        # (v) V_inv and Y, :178-184
        Vinv = matlab_pinv(Vs) if vinv == "pinv" else pinv3_formula(Vs, lib)
        Vinv = F(Vinv)
        if form == "dense":
            Y = y_dense(W, Vinv)
            S, e_ = mex2(Y, W, Us, eA, eB, lib)
        else:
            Y = sp_y(pb, W, Vinv, num_a, lib)
            S, e_ = sp_schur(pb, Y, W, Us, eA, eB, num_a, lib)
        # (vi) reduced solve, :193
        if solve == "pinv":
            da = matlab_pinv(S) @ e_
        elif solve == "seq":
            da, rc = chol_seq(S, e_, lib)
            if rc:
                da = matlab_pinv(S) @ e_
        else:
            da = chol_solve_fixed(S, e_)
        da = F(da)
        # (vii)-(viii), :204-210
        if form == "dense":
            db, a_new, b_new, X_hat_new = mex3(W, da, eB, Vinv, K, a, b, X, vis, lib)
            e_new = X - X_hat_new
            if sums == "seq":
                old_error = seq_dot(e.reshape(-1, order="F"), lib)
                new_error = seq_dot(e_new.reshape(-1, order="F"), lib)
            else:
                old_error = float(e.reshape(-1, order="F") @ e.reshape(-1, order="F"))
                new_error = float(e_new.reshape(-1, order="F") @ e_new.reshape(-1, order="F"))
        else:
            db, a_new, b_new, xh, _ = sp_update(pb, W, da, eB, Vinv, a, b, num_a, lib,
                                                ndb=num_a if nomex else 6)
            en = pb.obs_x - xh
            if sums == "seq":
                old_error = seq_dot(e[cm].reshape(-1), lib)
                new_error = seq_dot(en[cm].reshape(-1), lib)
            else:
                old_error = float(e.reshape(-1) @ e.reshape(-1))
                new_error = float(en.reshape(-1) @ en.reshape(-1))
        # (ix)-(x), :215-241
        g = np.concatenate([eA.reshape(-1, order="F"), eB.reshape(-1, order="F")])
        dp = np.concatenate([da.reshape(-1, order="F"), db.reshape(-1, order="F")])
        dpg = seq_dpg(dp, g, lam, lib) if sums == "seq" else float(dp @ (lam * dp + g))
        rho = (old_error - new_error) / dpg
        accepted = (old_error - new_error) > 0
        if trace is not None:
            trace.append(dict(lam=lam, accepted=bool(accepted), old=old_error, new=new_error,
                              rho=rho, da=da.copy(), db=db.copy()))
        if accepted:
            old_error /= num_vis
            new_error /= num_vis
            if o["verbose"]:
                print(f"iter {it}: error= {old_error:g} -> {new_error:g}")
            a, b = a_new, b_new
            lam = lam * max(1.0 / 3.0, 1.0 - (2.0 * rho - 1.0) ** 3)
            nu = 2.0
            if len(err) < it:
                err.append(old_error)
            else:
                err[it - 1] = old_error
            it += 1
            err.append(new_error)
            it2 = 0
        else:
            lam = lam * nu
            nu = 2.0 * nu
            it2 += 1
    K_, Te_, w_, Xe_ = unpack(K, a, b, Xe, nvk)
    if nomex:
        Xe_[3] = 1.0
    return K_, Te_, w_, Xe_, np.array(err)
