"""CPU baselines of one LM pass -- TEST / BASELINE INFRASTRUCTURE ONLY.

Two restatements of the reference's pass (bundle_euclid.m:120-249 with the MEX
stages), both built from this repository's C (never the reference's sources):

* ``SparsePort`` -- "ref_sparse_mt" of SURVEY.md sec. 8.d / BASELINE.md sec. 3:
  oracle/ba_cpu_mt.c (the MEX stages' per-element arithmetic and ascending
  reduction orders on the COO observation list, OpenMP over the host cores)
  plus the reduced solve as LAPACK's BANDED Cholesky (dpbtrf / dpbtrs via
  scipy) -- the same exact structure the GPU exploits, so the GPU/CPU ratio
  compares implementations of one algorithm, not a dense vs banded solve.  A
  dense LAPACK Cholesky (dpotrf) is timed beside it for reference.
* ``dense_pass`` -- "ref_dense": the oracle's dense MEX-layout stages
  (oracle_mex1/2/3: every (point, camera) pair, O(m^2 n) Schur, single
  thread, as the reference MEX files run) with MATLAB-pinv (SVD) solves and
  BLAS limited to one thread.  Feasible for configs 1, 2 and 5.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import it.
"""
from __future__ import annotations

import ctypes
import os
import time

import numpy as np

import bundle_euclid_ref as ref

_HERE = os.path.dirname(os.path.abspath(__file__))
_P = lambda arr: arr.ctypes.data_as(ctypes.c_void_p)   # noqa: E731
_MT = None


def mt_lib():
    global _MT
    if _MT is None:
        ref._lib()   # builds oracle/build if needed
        L = ctypes.CDLL(os.path.join(_HERE, "build", "libba_cpu_mt.so"))
        L.mt_linearize.restype = ctypes.c_double
        L.mt_update.restype = ctypes.c_double
        _MT = L
    return _MT


def host_info():
    """nproc, CPU model, OpenMP threads of the port, BLAS of numpy / scipy."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    blas = ""
    try:
        import threadpoolctl
        for p in threadpoolctl.threadpool_info():
            if p.get("user_api") == "blas":
                blas = f"{p.get('internal_api')} {p.get('version')} ({p.get('num_threads')} threads)"
                break
    except Exception:   # noqa: BLE001 -- informational only
        pass
    quota = None   # the cgroup's CPU bandwidth limit, in CPUs (None = unlimited / unknown)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "cgroup_cpus": quota, "omp_threads": int(mt_lib().mt_threads()),
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"), "cpu_model": model,
            "blas": blas}


def band_cholesky_solve(S, e_, bw=None):
    """da = S \\ e_ with LAPACK's banded Cholesky (dpbtrf / dpbtrs) on the band
    of the lower triangle of S (lower bandwidth bw; from S's non-zeros if
    None); exactly-zero rows fixed (unit diagonal, rhs 0: the pinv rule of
    App. A Q2 / Q8).  Returns (da, lower bandwidth)."""
    import scipy.linalg as sl
    ld = S.shape[0]
    if bw is None:
        rows, cols = np.nonzero(S)
        bw = int((rows - cols).max()) if rows.size else 0
    ab = np.zeros((bw + 1, ld))
    for d in range(bw + 1):
        ab[d, :ld - d] = np.diagonal(S, -d)
    rhs = np.array(e_, dtype=np.float64).reshape(-1).copy()
    zero = ab[0] == 0.0
    ab[0, zero] = 1.0
    rhs[zero] = 0.0
    c = sl.cholesky_banded(ab, lower=True, check_finite=False)
    return sl.cho_solve_banded((c, True), rhs, check_finite=False), bw


class SparsePort:
    """oracle/ba_cpu_mt.c over a COO scene (num_a = 6, the config-3 workload)."""

    def __init__(self, m, n, obs_pt, obs_cam, obs_x, K):
        i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32)   # noqa: E731
        f64 = lambda a: np.ascontiguousarray(a, dtype=np.float64)   # noqa: E731
        order = np.lexsort((obs_cam, obs_pt))          # point-major, cameras ascending
        self.m, self.n = int(m), int(n)
        self.pt, self.cam = i32(np.asarray(obs_pt)[order]), i32(np.asarray(obs_cam)[order])
        self.x = f64(np.asarray(obs_x).reshape(-1, 2)[order])
        self.N = len(self.pt)
        self.pt_ptr = i32(np.concatenate([[0], np.cumsum(np.bincount(self.pt, minlength=n))]))
        self.cam_obs = i32(np.argsort(self.cam, kind="stable"))   # camera-major, points asc.
        self.cam_ptr = i32(np.concatenate([[0], np.cumsum(np.bincount(self.cam, minlength=m))]))
        self.K = f64(np.asarray(K).T.reshape(-1))
        N, n, m = self.N, self.n, self.m
        self.jrec, self.W, self.Y = np.empty(20 * N), np.empty(18 * N), np.empty(18 * N)
        self.V, self.eB, self.Vinv = np.empty(9 * n), np.empty(3 * n), np.empty(9 * n)
        self.U, self.eA = np.empty(36 * m), np.empty(6 * m)
        self.S = np.empty((6 * m, 6 * m), order="F")
        self.e_ = np.empty(6 * m)
        self.db, self.b_new, self.a_new = np.empty(3 * n), np.empty(3 * n), np.empty(6 * m)
        # lower bandwidth of S from the co-visibility (the widest camera span of
        # a point's track): S_jk != 0 only for cameras seen by a common point
        lo = np.minimum.reduceat(self.cam, self.pt_ptr[:-1]) if n else np.zeros(0, np.int32)
        hi = np.maximum.reduceat(self.cam, self.pt_ptr[:-1]) if n else np.zeros(0, np.int32)
        has = np.diff(self.pt_ptr) > 0
        self.bw = int(6 * (hi[has] - lo[has]).max() + 5) if has.any() else 5

    def one_pass(self, a0, b0, lam=1e-3, solve="band", vinv="formula", relin=True):
        """One LM pass at (a0 6 x m, b0 3 x n): dict of old / new SSE, S, e_,
        da, db and the seconds of each phase (the timed region is the whole
        pass: stage 1, damping + Schur, the reduced solve, stage 3).
        vinv="pinv": V*_i^-1 by MATLAB's pinv rule (mt_damp_y_pinv) instead of
        the closed form; relin=False reuses the last pass's stage 1 (a
        rejected step's identical linearisation, App. A Q12)."""
        L = mt_lib()
        f64 = lambda a: np.ascontiguousarray(a, dtype=np.float64)   # noqa: E731
        a = f64(np.asarray(a0).T.reshape(-1))
        b = f64(np.asarray(b0).T.reshape(-1))
        m, n = self.m, self.n
        t = [time.perf_counter()]
        if relin or not hasattr(self, "_old"):
            self._old = L.mt_linearize(n, _P(self.pt_ptr), _P(self.cam), _P(self.x), _P(self.K),
                                       _P(a), _P(b), _P(self.jrec), _P(self.W), _P(self.V),
                                       _P(self.eB))
            L.mt_camera_reduce(m, _P(self.cam_ptr), _P(self.cam_obs), _P(self.jrec), _P(self.U),
                               _P(self.eA))
        old = self._old
        t.append(time.perf_counter())
        damp = L.mt_damp_y_pinv if vinv == "pinv" else L.mt_damp_y
        damp(n, _P(self.pt_ptr), ctypes.c_double(lam), _P(self.V), _P(self.W), _P(self.Vinv),
             _P(self.Y))
        L.mt_schur(m, _P(self.cam_ptr), _P(self.cam_obs), _P(self.pt), _P(self.pt_ptr),
                   _P(self.cam), _P(self.Y), _P(self.W), _P(self.U), ctypes.c_double(lam),
                   _P(self.eA), _P(self.eB), _P(self.S), _P(self.e_))
        t.append(time.perf_counter())
        bw = None
        if solve == "band":
            da, bw = band_cholesky_solve(self.S, self.e_, self.bw)
        else:
            da = ref.chol_solve_fixed(self.S, self.e_).reshape(-1)
        da = f64(da)
        t.append(time.perf_counter())
        new = L.mt_update(m, n, _P(self.pt_ptr), _P(self.cam), _P(self.x), _P(self.K),
                          _P(self.W), _P(da), _P(self.eB), _P(self.Vinv), _P(a), _P(b),
                          _P(self.db), _P(self.a_new), _P(self.b_new))
        t.append(time.perf_counter())
        return {"old_sse": old, "new_sse": new, "S": self.S, "e_": self.e_, "da": da,
                "db": self.db.reshape(n, 3).T, "bandwidth": bw, "a_new": self.a_new,
                "b_new": self.b_new,
                "seconds": {"linearize": t[1] - t[0], "schur": t[2] - t[1],
                            "solve": t[3] - t[2], "update": t[4] - t[3], "total": t[4] - t[0]}}


    def lm(self, a0, b0, *, stop_rel=1e-3, max_iter=20, max_iter2=10, lambda0=1e-3,
           vinv="pinv", solve="band", check_pinv=1):
        """The whole LM loop of bundle_euclid.m:111-249 (fix_calibration) with
        the reference's MATLAB semantics: V*_i^-1 = pinv(V*_i) (mt_damp_y_pinv)
        and da = pinv(S) e_.  The reduced solve is LAPACK's banded Cholesky on
        S with its exactly-zero rows fixed (App. A Q2 / Q8); that IS pinv(S) e_
        when no eigenvalue of S falls below pinv's tolerance ld * eps(max
        eigenvalue) (none is truncated), which check_pinv verifies on every
        check_pinv-th pass and the last (sparse shift-invert Lanczos for the
        extreme eigenvalues of the band; 0 = never).  Returns (error_, a, b, info) with info = passes, accepted and
        the smallest lambda_min / tol seen."""
        a = np.array(a0, dtype=np.float64, order="F")
        b = np.array(b0, dtype=np.float64, order="F")
        lam, nu, it, it2 = lambda0, 2.0, 1, 0
        err, passes, acc, relin = [], 0, 0, True
        worst = np.inf

        def cont():
            if not (it < max_iter and it2 < max_iter2):
                return False
            if it < 3:
                return True
            return err[it - 1] > 1e-20 and err[it - 2] - err[it - 1] > stop_rel * err[it - 2]

        while cont():
            r = self.one_pass(a, b, lam, solve=solve, vinv=vinv, relin=relin)
            passes += 1
            if check_pinv and (passes - 1) % check_pinv == 0:
                worst = min(worst, pinv_margin(self.S))
            old, new = r["old_sse"], r["new_sse"]
            g = np.concatenate([self.eA, self.eB])
            dp = np.concatenate([r["da"], self.db])
            rho = (old - new) / float(dp @ (lam * dp + g))
            if old - new > 0:                         # bundle_euclid.m:218-232
                a = r["a_new"].reshape(self.m, 6).T.copy(order="F")
                b = r["b_new"].reshape(self.n, 3).T.copy(order="F")
                lam = lam * max(1.0 / 3.0, 1.0 - (2.0 * rho - 1.0) ** 3)
                nu = 2.0
                if len(err) < it:
                    err.append(old / self.N)
                else:
                    err[it - 1] = old / self.N
                it += 1
                err.append(new / self.N)
                it2 = 0
                acc += 1
                relin = True
            else:                                     # :233-241
                lam, nu = lam * nu, 2.0 * nu
                it2 += 1
                relin = False
        if check_pinv:   # the last pass's system
            worst = min(worst, pinv_margin(self.S))
        return np.array(err), a, b, {"passes": passes, "accepted": acc, "pinv_margin": worst}


def pinv_margin(S):
    """lambda_min / tol of S restricted to its non-zero rows, tol = MATLAB
    pinv's ld * eps(sigma_max): > 1 means pinv(S) e_ equals the Cholesky
    solve with the zero rows fixed (no singular value is truncated).  S is
    symmetric; sparse shift-invert Lanczos on the band."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as sla
    d = np.diag(S)
    keep = d != 0.0
    A = sp.csc_matrix(S[np.ix_(keep, keep)])
    lmax = sla.eigsh(A, k=1, which="LA", return_eigenvectors=False, tol=1e-6)[0]
    lmin = sla.eigsh(A, k=1, sigma=0.0, which="LM", return_eigenvectors=False, tol=1e-6)[0]
    tol = S.shape[0] * np.spacing(lmax)
    return float(lmin / tol)


def dense_pass(K, a, b, X, vis, lam=1e-3):
    """ref_dense: one pass of the reference's dense MEX loops (oracle_mex1/2/3,
    single thread) with MATLAB-pinv (SVD) solves, BLAS on one thread.
    Returns (seconds, old_sse, new_sse)."""
    import threadpoolctl
    with threadpoolctl.threadpool_limits(1):
        t0 = time.perf_counter()
        X_hat, A, B, e, U, V, W, eA, eB = ref.mex1(K, a, b, X, vis)
        num_a = a.shape[0]
        Us = U.copy(order="F")
        for k in range(num_a):
            Us[k, k] = (1 + lam) * U[k, k]
        Vs = V.copy(order="F")
        for k in range(3):
            Vs[k, k] = (1 + lam) * V[k, k]
        Vinv = ref.F(ref.matlab_pinv(Vs))
        Y = ref.y_dense(W, Vinv)
        S, e_ = ref.mex2(Y, W, Us, eA, eB)
        da = ref.F(ref.matlab_pinv(S) @ e_)
        db, a_new, b_new, X_hat_new = ref.mex3(W, da, eB, Vinv, K, a, b, X, vis)
        e_new = X - X_hat_new
        old = float(e.reshape(-1) @ e.reshape(-1))
        new = float(e_new.reshape(-1) @ e_new.reshape(-1))
        return time.perf_counter() - t0, old, new
