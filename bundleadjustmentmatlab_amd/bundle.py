"""Host mirror of the reference's MATLAB entry points, running on libvlgba.

``bundle_euclid`` keeps the signature, option names, argument meaning and
output semantics of toolbox/bundle/bundle_euclid.m:1-269::

    K_, Te_, w_, Xe_, error_ = bundle_euclid(K, Te, w, Xe, x, 'fix_calibration',
                                             'visibility', vis, 'verbose')

with arrays MATLAB-shaped (K 4xm, Te 3xm, w 3xm, Xe 4xn, x 3xnxm).  The whole
LM loop (bundle_euclid.m:111-249) runs on the GPU through ``vlgba_solve``.

``bundle_euclid_obs`` takes the same problem as a COO observation list, the
form that scales to the 1000-camera / 500k-point configs (a dense x at that
size is 12 GB).

``bundle_euclid_nomex`` is the same drop-in for the reference's pure-MATLAB
twin toolbox/bundle/bundle_euclid_nomex.m (full-da back substitution, no
'fix_pivot', Xe_(4,:) = 1).

``mex_bundle_1_XABeUVWeAeB`` / ``mex_bundle_2_Se_`` / ``mex_bundle_3_db_new``
mirror the three MEX stages with their exact argument layouts.
"""
from __future__ import annotations

import ctypes
import numpy as np

from ._lib import (ALLREDUCE_FN, MODEL_EUCLIDEAN, MODEL_PROJECTIVE, NKERNELS, ON_PASS_FN,
                   VlgbaOptions,
                   VlgbaProblem, VlgbaResectProblem, VlgbaStats,
                   VlgbaStepInfo, c_dp, c_ip, c_up, check, lib)

__all__ = ["bundle_euclid", "bundle_euclid_nomex", "bundle_euclid_obs", "BundleAdjuster",
           "bundle_euclid_resect",
           "parse_options", "pivot_mask",
           "mex_bundle_1_XABeUVWeAeB", "mex_bundle_2_Se_", "mex_bundle_3_db_new"]


def _F(a):
    return np.asfortranarray(a, dtype=np.float64)


def _dp(a):
    return a.ctypes.data_as(c_dp)


# ---------------------------------------------------------------------------
# options (bundle_euclid.m:44-82)
# ---------------------------------------------------------------------------
def pivot_mask(pivot, m):
    """The cameras ``U(:,:,pivot) = 0`` fixes (bundle_euclid.m:150-153), read
    the way MATLAB indexes with ``pivot``: a logical mask (bool dtype) of any
    length -- entries past m must be false -- or a list of 1-based camera
    numbers (``'fix_pivot', 1`` or ``[1 3]``; duplicates allowed).  MATLAB
    would grow U / W / eA for a true entry or an index past m, and errors on
    an index that is not a positive integer; both are errors here.  Returns
    the (m,) bool mask."""
    p = np.asarray(pivot)
    mask = np.zeros(m, dtype=bool)
    flat = p.reshape(-1)
    if p.dtype == bool:
        if flat[m:].any():
            raise ValueError("fix_pivot: logical index past the camera count")
        mask[:min(flat.size, m)] = flat[:m]
        return mask
    if flat.size == 0:
        return mask
    v = flat.astype(np.float64)
    if not np.all(np.isfinite(v)) or np.any(v != np.floor(v)) or v.min() < 1 or v.max() > m:
        raise ValueError("fix_pivot: camera indices must be integers in 1..m")
    mask[v.astype(np.int64) - 1] = True
    return mask


def parse_options(m, n, varargin, x=None, nomex=False):
    """Name/value options of bundle_euclid.m:53-78.  Unknown names are
    ignored, as the reference's switch statement ignores them.  'fix_pivot'
    takes a logical mask or 1-based camera numbers (pivot_mask).  nomex=True
    parses bundle_euclid_nomex.m:50-70 instead, which has no 'fix_pivot': the
    name and its argument fall through its switch and are ignored."""
    o = dict(fix_structure=False, fix_motion=False, fix_pivot=False,
             pivot=np.zeros(m, dtype=bool), num_variableK=4, visible=None, verbose=False)
    k = 0
    varargin = list(varargin)
    while k < len(varargin):
        name = varargin[k]
        name = name.lower() if isinstance(name, str) else name
        if name == "fix_structure":
            o["fix_structure"] = True
        elif name == "fix_motion":
            o["fix_motion"] = True
        elif name == "fix_pivot":
            if not nomex:
                o["fix_pivot"] = True
                o["pivot"] = pivot_mask(varargin[k + 1], m)
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
    if o["visible"] is None and x is not None:
        o["visible"] = (x[0] != 0) | (x[1] != 0)          # bundle_euclid.m:50
    if o["visible"] is not None:
        o["visible"] = np.asarray(o["visible"], dtype=np.float64).reshape(n, m, order="F")
    return o


def pack_a(K, Te, w, nvk):
    """a = [w; T; (K)] (bundle_euclid.m:89-96)."""
    m = w.shape[1]
    a = np.zeros((6 + nvk, m), order="F")
    a[0:3] = w
    a[3:6] = Te
    if nvk == 1:
        a[6] = K[0]
    elif nvk == 4:
        a[6:10] = K
    return a


def unpack(K, a, b, Xe4, nvk):
    """bundle_euclid.m:255-267 (Xe_(4,:) is the input Xe(4,:), App. A Q5)."""
    K_ = np.array(K, dtype=np.float64, order="F")
    if nvk == 1:
        K_[0] = a[6]
        K_[1] = a[6]
    elif nvk == 4:
        K_[:] = a[6:10]
    return K_, a[3:6].copy(order="F"), a[0:3].copy(order="F"), np.vstack([b, Xe4])


# ---------------------------------------------------------------------------
# per-pass JSON log ("Tracing")
# ---------------------------------------------------------------------------
class _PassLog:
    """Callable for vlgba_options.on_pass: one JSON line per LM pass."""

    def __init__(self, sink, num_vis, projective):
        import json
        self._json = json
        self._own = False
        self._fn = None
        self._fh = None
        if callable(sink) and not hasattr(sink, "write"):
            self._fn = sink
        elif hasattr(sink, "write"):
            self._fh = sink
        else:
            self._fh = open(sink, "a", encoding="utf-8")
            self._own = True
        self.num_vis = float(num_vis)
        self.projective = projective
        self.records = []

    def __call__(self, npass, it, info_p, _user):
        i = info_p.contents
        # bundle_euclid.m:219-220 error_ = SSE / num_vis (projective: SSE * (1 / num_vis))
        sc = (lambda v: 1 / self.num_vis * v) if self.projective else (lambda v: v / self.num_vis)
        rec = {"pass": int(npass), "iter": int(it), "lambda": i.lambda_,
               "old_sse": i.old_sse, "new_sse": i.new_sse, "error_old": sc(i.old_sse),
               "error_new": sc(i.new_sse), "dpg": i.dpg, "rho": i.rho,
               "accepted": bool(i.accepted), "chol_failed": bool(i.chol_failed),
               "pinv": bool(i.pinv), "spin_retry": bool(i.spin_retry)}
        self.records.append(rec)
        try:
            if self._fn is not None:
                self._fn(rec)
            else:
                self._fh.write(self._json.dumps(rec) + "\n")
        except Exception:   # noqa: BLE001 -- a failing log must not abort the solve
            pass

    def close(self):
        if self._own and self._fh is not None:
            self._fh.close()
            self._fh = None


# ---------------------------------------------------------------------------
# the GPU solver handle
# ---------------------------------------------------------------------------
class BundleAdjuster:
    """One problem resident on one GPU (vlgba_ctx).

    obs_pt / obs_cam (0-based) and obs_x (N, 2) describe the visible
    observations; K is 4 x m; num_a is 6 (fix_calibration), 7 (fix_principal)
    or 10 (variable K).  Options follow bundle_euclid.m's names.  ``solver``
    picks the reduced-camera solve: "auto" (cyclic reduction when S is
    tile-tridiagonal, else envelope Cholesky -- on a nested-dissection camera
    order when that shortens its chain of steps), "envelope", "nd" (the
    nested-dissection order whenever the cameras split) or "dense";
    ``dense_solve=True`` is the same as solver="dense".  ``schur_kernel``
    picks the fast-path Schur complement kernel: "auto" (dense per-chunk
    products on fp64 MFMA when the tracks fit) or "terms" (per-term sums).
    ``semantics`` is "mex" (bundle_euclid.m) or "nomex" (bundle_euclid_nomex.m).
    ``parity=True`` runs the parity mode (vlgba_options.ordered = 2: ordered
    sums, sequential Cholesky, LM scalars in the reference's flat order --
    the LM trajectory is bit-identical to the CPU oracle's).  ``stop_rel``
    replaces the 1e-3 of the stop rule (bundle_euclid.m:123).
    ``log`` (a path, a text file or a callable) receives one JSON record per
    LM pass of run() (vlgba_options.on_pass): pass, iter, lambda, old / new
    SSE, error_ values (SSE / num_vis), rho, accepted, chol_failed, pinv.
    ``model="projective"`` solves bundle_projective.m instead: num_a = 12
    (a = P(:) per camera), K is None and ``m`` gives the camera count.
    """
    SOLVERS = {"auto": 0, "dense": 1, "envelope": 2, "sequential": 3, "nd": 4}
    SCHUR_KERNELS = {"auto": 0, "terms": 1}
    SEMANTICS = {"mex": 0, "nomex": 1}
    MODELS = {"euclidean": MODEL_EUCLIDEAN, "projective": MODEL_PROJECTIVE}

    def __init__(self, K, obs_pt, obs_cam, obs_x, n, num_a=6, *, fix_structure=False,
                 fix_motion=False, pivot=None, verbose=False, num_vis=0.0, device=0,
                 rank=0, world_size=1, comm_id=None, max_iter=0, max_iter2=0, lambda0=0.0,
                 dense_solve=False, ordered=False, allreduce=None, solver=None,
                 schur_kernel="auto", semantics="mex", model="euclidean", m=None,
                 parity=False, stop_rel=0.0, log=None):
        L = lib()
        solve_mode = self.SOLVERS[solver] if solver is not None else int(bool(dense_solve))
        self.K = _F(K) if K is not None else None
        self.m = int(m) if m is not None else self.K.shape[1]
        self.n = int(n)
        self.num_a = int(num_a)
        self.max_iter = int(max_iter) if max_iter > 0 else 20   # bundle_euclid.m:117
        self._pt = np.ascontiguousarray(obs_pt, dtype=np.int32)
        self._cam = np.ascontiguousarray(obs_cam, dtype=np.int32)
        self._x = np.ascontiguousarray(obs_x, dtype=np.float64).reshape(-1, 2)
        self.num_obs = len(self._pt)
        prob = VlgbaProblem(self.m, self.n, self.num_a, self.num_obs,
                            self._pt.ctypes.data_as(c_ip), self._cam.ctypes.data_as(c_ip),
                            _dp(self._x), _dp(self.K) if self.K is not None else None,
                            float(num_vis), self.MODELS[model])
        self._pivot = None
        if pivot is not None:
            self._pivot = np.ascontiguousarray(np.asarray(pivot, dtype=bool).reshape(-1),
                                               dtype=np.uint8)
        self._comm = None
        if comm_id is not None:
            self._comm = ctypes.create_string_buffer(bytes(comm_id), 128)
        self._ar = None
        if allreduce is not None:
            # host collective: allreduce(np.ndarray) sums in place over ranks
            def _cb(buf, count, _user, fn=allreduce):
                try:
                    fn(np.ctypeslib.as_array(buf, shape=(count,)))
                    return 0
                except Exception:   # noqa: BLE001 -- reported to the library as failure
                    return 1
            self._ar = ALLREDUCE_FN(_cb)
        self._log = self._log_fn = None
        if log is not None:
            self._log = _PassLog(log, num_vis if num_vis > 0 else float(self.num_obs),
                                 model == "projective")
            self._log_fn = ON_PASS_FN(self._log)
        opt = VlgbaOptions(int(fix_structure), int(fix_motion),
                           self._pivot.ctypes.data_as(c_up) if self._pivot is not None else None,
                           int(verbose), int(max_iter), int(max_iter2), float(lambda0),
                           int(device), int(rank), int(world_size),
                           ctypes.cast(self._comm, ctypes.c_void_p) if self._comm else None,
                           solve_mode, 2 if parity else int(ordered),
                           ctypes.cast(self._ar, ctypes.c_void_p) if self._ar else None, None,
                           self.SCHUR_KERNELS[schur_kernel], self.SEMANTICS[semantics],
                           float(stop_rel),
                           ctypes.cast(self._log_fn, ctypes.c_void_p) if self._log_fn else None,
                           None)
        h = ctypes.c_void_p()
        check(L.vlgba_create(ctypes.byref(prob), ctypes.byref(opt), ctypes.byref(h)),
              "vlgba_create")
        self._h = h
        self._L = L

    def close(self):
        if getattr(self, "_h", None):
            self._L.vlgba_destroy(self._h)
            self._h = None
        if getattr(self, "_log", None) is not None:
            self._log.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_params(self, a, b):
        a = np.ascontiguousarray(_F(a).reshape(-1, order="F"))
        b = np.ascontiguousarray(_F(b).reshape(-1, order="F"))
        assert a.size == self.num_a * self.m and b.size == 3 * self.n
        check(self._L.vlgba_set_params(self._h, _dp(a), _dp(b)), "vlgba_set_params")

    def get_params(self):
        a = np.zeros(self.num_a * self.m)
        b = np.zeros(3 * self.n)
        check(self._L.vlgba_get_params(self._h, _dp(a), _dp(b)), "vlgba_get_params")
        return a.reshape(self.num_a, self.m, order="F"), b.reshape(3, self.n, order="F")

    def force_status(self, word, passes=1):
        """Fault injection: the next ``passes`` passes report a non-positive
        pivot (word 4: pinv step) or a hand-off timeout (word 5: re-solve);
        word 6: the next ``passes`` starts of the envelope runner fail (the
        factorization then runs with the column launches alone)."""
        check(self._L.vlgba_debug_force_status(self._h, int(word), int(passes)),
              "vlgba_debug_force_status")

    def step(self, relinearize=True, update_lm=True):
        info = VlgbaStepInfo()
        check(self._L.vlgba_step(self._h, int(relinearize), int(update_lm), ctypes.byref(info)),
              "vlgba_step")
        return info

    def passes(self, n):
        """n full passes at the current parameters and lambda, each
        relinearising, none changing the state (vlgba_run_passes); the last
        pass's info."""
        info = VlgbaStepInfo()
        check(self._L.vlgba_run_passes(self._h, int(n), ctypes.byref(info)), "vlgba_run_passes")
        return info

    def run(self):
        """The LM loop (vlgba_run): (error_, stats).  error_ has at most
        max_iter entries (bundle_euclid.m:117-123)."""
        err = np.zeros(self.max_iter + 1)
        st = VlgbaStats()
        check(self._L.vlgba_run(self._h, _dp(err), err.size, ctypes.byref(st)), "vlgba_run")
        assert st.num_error <= err.size
        return err[: st.num_error].copy(), st

    def last_step(self):
        """(da (num_a, m), db (3, n)) of the last pass (vlgba_get_step)."""
        da = np.zeros(self.num_a * self.m)
        db = np.zeros(3 * self.n)
        check(self._L.vlgba_get_step(self._h, _dp(da), _dp(db)), "vlgba_get_step")
        return da.reshape(self.num_a, self.m, order="F"), db.reshape(3, self.n, order="F")

    def reduced_system(self, dense=True):
        """S (lower triangle: blocks j >= k; dense (na m) x (na m) if dense,
        else (blk_jk (nb, 2), blocks (nb, na, na))) and e_ at the current
        lambda (vlgba_get_reduced_system)."""
        nb = self.plan_info()["blocks"]
        na = self.num_a
        jk = np.zeros(2 * nb, dtype=np.int32)
        blocks = np.zeros(na * na * nb)
        e_ = np.zeros(na * self.m)
        check(self._L.vlgba_get_reduced_system(self._h, jk.ctypes.data_as(c_ip), _dp(blocks),
                                               _dp(e_)), "vlgba_get_reduced_system")
        jk = jk.reshape(nb, 2)
        blocks = blocks.reshape(nb, na, na).transpose(0, 2, 1)   # [b, r, c]
        if not dense:
            return jk, blocks, e_
        S = np.zeros((na * self.m, na * self.m))
        for (j, k), B in zip(jk, blocks):
            if j == k:
                S[na * j:na * j + na, na * k:na * k + na] = np.tril(B)
            else:
                S[na * j:na * j + na, na * k:na * k + na] = B
        return S, e_

    def sync(self):
        check(self._L.vlgba_sync(self._h), "vlgba_sync")

    def linearization(self):
        """Stage 1 at the current parameters: dict of U (na, na, m), eA (na, m),
        V (3, 3, n), eB (3, n) and W (na, 3, N) with observations point-major
        (points ascending, cameras ascending within a point)."""
        na, m, n, N = self.num_a, self.m, self.n, self.num_obs
        U = np.zeros((na, na, m), order="F")
        eA = np.zeros((na, m), order="F")
        V = np.zeros((3, 3, n), order="F")
        eB = np.zeros((3, n), order="F")
        W = np.zeros((na, 3, N), order="F")
        check(self._L.vlgba_get_linearization(self._h, _dp(U), _dp(eA), _dp(V), _dp(eB),
                                              _dp(W)), "vlgba_get_linearization")
        return dict(U=U, eA=eA, V=V, eB=eB, W=W)

    def set_timing(self, on=True):
        check(self._L.vlgba_set_timing(self._h, int(on)), "vlgba_set_timing")

    def kernel_ms(self, reset=True):
        """{kernel: (total ms, launches)} accumulated since the last reset over
        the passes run with set_timing(True)."""
        n = NKERNELS
        ms = np.zeros(n)
        calls = (ctypes.c_longlong * n)()
        check(self._L.vlgba_kernel_ms(self._h, _dp(ms), calls, int(reset)), "vlgba_kernel_ms")
        return {self._L.vlgba_kernel_name(k).decode(): (float(ms[k]), int(calls[k]))
                for k in range(n) if calls[k] > 0}

    PLAN_KEYS = ("obs", "points", "cameras", "num_a", "chunks", "chunk_slots",
                 "chunk_eslots", "groups", "group_slots", "group_eslots", "blocks",
                 "tiles", "cr_levels", "cr_elim", "cr_keep", "ordered", "schur_terms",
                 "blob_words", "mfma", "cr_rows", "mfma_groups", "reordered", "long_points",
                 "nd_arcs", "nd_sep_tiles", "solve_flops_factor", "solve_flops_syrk",
                 "solve_flops_back", "env_runner_runs")

    def plan_info(self):
        """Execution-plan sizes of this rank (vlgba_plan_info)."""
        n = len(self.PLAN_KEYS)
        buf = (ctypes.c_longlong * n)()
        rc = self._L.vlgba_plan_info(self._h, buf, n)
        check(min(rc, 0), "vlgba_plan_info")
        return dict(zip(self.PLAN_KEYS, [int(v) for v in buf]))

    def phase_ms(self):
        ms = np.zeros(7)
        check(self._L.vlgba_phase_ms(self._h, _dp(ms)), "vlgba_phase_ms")
        return dict(zip(["linearize", "camera_reduce", "damp_y", "schur", "assemble",
                         "cholesky_solve", "update"], ms.tolist()))


# ---------------------------------------------------------------------------
# drop-in drivers
# ---------------------------------------------------------------------------
def euclid_obs_adjuster(K, m, n, obs_pt, obs_cam, obs_x, *varargin, num_vis=0.0, device=0,
                        rank=0, world_size=1, comm_id=None, semantics="mex", **solver):
    """The BundleAdjuster that bundle_euclid_obs would create for this problem
    and these options (its structure only: no parameter values), so a caller
    can build it ahead of time -- the host plan of vlgba_create runs with the
    GIL released (ctypes), e.g. on a worker thread while the previous solve
    runs (incremental.py) -- and hand it to bundle_euclid_obs(adjuster=...)."""
    o = parse_options(m, n, varargin, nomex=semantics == "nomex")
    ba = BundleAdjuster(K, obs_pt, obs_cam, obs_x, n, 6 + o["num_variableK"],
                        fix_structure=o["fix_structure"], fix_motion=o["fix_motion"],
                        pivot=o["pivot"] if o["fix_pivot"] else None, verbose=o["verbose"],
                        num_vis=num_vis, device=device, rank=rank, world_size=world_size,
                        comm_id=comm_id, semantics=semantics, **solver)
    ba.fingerprint = _adjuster_fingerprint(K, m, n, obs_pt, obs_cam, obs_x, o, num_vis,
                                           semantics, rank, world_size, device, comm_id)
    return ba


def _adjuster_fingerprint(K, m, n, obs_pt, obs_cam, obs_x, o, num_vis, semantics, rank,
                          world_size, device, comm_id):
    """What a prebuilt adjuster was made for: sizes, the parsed
    options, K, a hash of the observation list, the device and the RCCL id
    -- a context built for another subset, other options, another GPU or
    another communicator with the same counts must not be used."""
    # xxh3 (~25x blake2b's speed; the growing replay fingerprints every solve's
    # observations twice, at build and at use), over the arrays' own buffers
    try:
        import xxhash
        h = xxhash.xxh3_128()
    except ImportError:
        import hashlib
        h = hashlib.blake2b(digest_size=16)
    for arr, dt in ((obs_pt, np.int32), (obs_cam, np.int32), (obs_x, np.float64),
                    (K, np.float64)):
        h.update(memoryview(np.ascontiguousarray(arr, dtype=dt)).cast("B"))
    piv = o["pivot"] if o["fix_pivot"] else None
    if piv is not None:
        h.update(np.asarray(piv, dtype=bool).tobytes())
    if comm_id is not None:
        h.update(bytes(comm_id))
    return (int(m), int(n), int(o["num_variableK"]), bool(o["fix_structure"]),
            bool(o["fix_motion"]), bool(o["fix_pivot"]), bool(o["verbose"]), float(num_vis),
            semantics, int(rank), int(world_size), int(device), comm_id is not None,
            h.hexdigest())


def bundle_euclid_obs(K, Te, w, Xe, obs_pt, obs_cam, obs_x, *varargin, num_vis=0.0, device=0,
                      rank=0, world_size=1, comm_id=None, return_stats=False,
                      semantics="mex", adjuster=None, **solver):
    """bundle_euclid on a COO observation list (0-based point / camera ids).
    ``solver`` keywords go to BundleAdjuster (parity, stop_rel, max_iter,
    max_iter2, lambda0, solver, ordered, schur_kernel).  ``adjuster``: a handle
    made beforehand by euclid_obs_adjuster for the same problem and options
    (or a concurrent.futures.Future of one); it is used and closed here."""
    K, Te, w, Xe = _F(K), _F(Te), _F(w), _F(Xe)
    m, n = w.shape[1], Xe.shape[1]
    nomex = semantics == "nomex"
    o = parse_options(m, n, varargin, nomex=nomex)
    nvk = o["num_variableK"]
    num_a = 6 + nvk
    a = pack_a(K, Te, w, nvk)
    b = _F(Xe[0:3])
    if adjuster is not None:
        if solver:
            raise ValueError("bundle_euclid_obs: solver options belong to the prebuilt adjuster")
        ba = adjuster.result() if hasattr(adjuster, "result") else adjuster
        want = _adjuster_fingerprint(K, m, n, obs_pt, obs_cam, obs_x, o, num_vis, semantics,
                                     rank, world_size, device, comm_id)
        if getattr(ba, "fingerprint", None) != want:
            ba.close()
            raise ValueError("bundle_euclid_obs: the prebuilt adjuster is for another problem "
                             "or other options (make it with euclid_obs_adjuster)")
    else:
        ba = euclid_obs_adjuster(K, m, n, obs_pt, obs_cam, obs_x, *varargin, num_vis=num_vis,
                                 device=device, rank=rank, world_size=world_size,
                                 comm_id=comm_id, semantics=semantics, **solver)
    with ba:
        ba.set_params(a, b)
        err, st = ba.run()
        a, b = ba.get_params()
    # Xe_(4,:): the input's (bundle_euclid.m:267) or ones (bundle_euclid_nomex.m:364)
    out = unpack(K, a, b, np.ones((1, n)) if nomex else Xe[3:4], nvk) + (err,)
    return out + (st,) if return_stats else out


def bundle_euclid(K, Te, w, Xe, x, *varargin, device=0, return_stats=False, semantics="mex",
                  **solver):
    """[K_ Te_ w_ Xe_ error_] = bundle_euclid(K, Te, w, Xe, x, ...)  (bundle_euclid.m:1)."""
    x = _F(x)
    m, n = np.shape(w)[1], x.shape[1]
    o = parse_options(m, n, varargin, x=x, nomex=semantics == "nomex")
    vis = o["visible"]
    num_vis = float(vis.sum())                                     # bundle_euclid.m:82
    pt, cam = np.nonzero(vis)                                      # point-major
    obs_x = np.stack([x[0, pt, cam], x[1, pt, cam]], axis=1)
    # re-emit the options without 'visibility' (already applied)
    rest, k = [], 0
    while k < len(varargin):
        nm = varargin[k].lower() if isinstance(varargin[k], str) else varargin[k]
        if nm == "visibility":
            k += 2
            continue
        if nm == "fix_pivot":
            rest += [varargin[k], varargin[k + 1]]
            k += 2
            continue
        rest.append(varargin[k])
        k += 1
    return bundle_euclid_obs(K, Te, w, Xe, pt, cam, obs_x, *rest, num_vis=num_vis,
                             device=device, return_stats=return_stats, semantics=semantics,
                             **solver)


def bundle_euclid_nomex(K, Te, w, Xe, x, *varargin, device=0, return_stats=False, **solver):
    """[K_ Te_ w_ Xe_ error_] = bundle_euclid_nomex(K, Te, w, Xe, x, ...)
    (bundle_euclid_nomex.m:1): the same LM loop with the twin's semantics --
    db from every camera parameter (:268-277), no 'fix_pivot', Xe_(4,:) = 1."""
    return bundle_euclid(K, Te, w, Xe, x, *varargin, device=device,
                         return_stats=return_stats, semantics="nomex", **solver)


def bundle_euclid_resect(K, Te, w, Xs, xs, *varargin, device=0, max_iter=0, max_iter2=0,
                         lambda0=0.0, stop_rel=0.0, return_stats=False):
    """Batched one-camera refinement with the structure fixed -- the call of
    estimate_camera.m:247-253,

        [K T Omega] = bundle_euclid(K, T, Omega, X, x0, 'fix_calibration',
                                    'fix_structure', 'visibility', inlier')

    for every camera q at once on the GPU (vlgba_resect).  K (4 x c), Te, w
    (3 x c); Xs[q] the fixed points camera q sees (3 or 4 x n_q), xs[q] their
    measured image points (2 or 3 x n_q; only the inliers).  Options as
    bundle_euclid.m: 'fix_calibration' (num_a 6), 'fix_principal' (7), neither
    (10); 'fix_structure' is implied.  Returns K_, Te_, w_ and the list of
    per-camera error_ (SSE / n_q per accepted step)."""
    K, Te, w = _F(K), _F(Te), _F(w)
    c = w.shape[1]
    o = parse_options(c, 0, varargin)
    nvk = o["num_variableK"]
    na = 6 + nvk
    a = np.ascontiguousarray(pack_a(K, Te, w, nvk).reshape(-1, order="F"))
    assert len(Xs) == len(xs) == c
    cnt = [np.shape(X)[1] for X in Xs]
    assert all(np.shape(x)[1] == k for x, k in zip(xs, cnt))
    ptr = np.ascontiguousarray(np.concatenate([[0], np.cumsum(cnt)]), dtype=np.int64)
    Xo = np.ascontiguousarray(np.concatenate([np.asarray(X, dtype=np.float64)[:3].T for X in Xs]
                                             if c else np.zeros((0, 3))))
    xo = np.ascontiguousarray(np.concatenate([np.asarray(x, dtype=np.float64)[:2].T for x in xs]
                                             if c else np.zeros((0, 2))))
    cap = (max_iter if max_iter > 0 else 20) + 1
    err = np.zeros((c, cap))
    nerr = np.zeros(c, dtype=np.int32)
    pr = VlgbaResectProblem(c, na, ptr.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)),
                            _dp(Xo), _dp(xo), _dp(np.ascontiguousarray(K.reshape(-1, order="F"))))
    opt = VlgbaOptions()
    opt.max_iter, opt.max_iter2, opt.lambda0 = int(max_iter), int(max_iter2), float(lambda0)
    opt.device, opt.stop_rel = int(device), float(stop_rel)
    st = VlgbaStats()
    check(lib().vlgba_resect(ctypes.byref(pr), ctypes.byref(opt), _dp(a), _dp(err), cap,
                             nerr.ctypes.data_as(c_ip), ctypes.byref(st)), "vlgba_resect")
    a = a.reshape(na, c, order="F")
    K_, Te_, w_, _ = unpack(K, a, np.zeros((3, 0)), np.zeros((1, 0)), nvk)
    errs = [err[q, : nerr[q]].copy() for q in range(c)]
    return (K_, Te_, w_, errs, st) if return_stats else (K_, Te_, w_, errs)


# ---------------------------------------------------------------------------
# MEX stage mirrors (exact argument layouts of the reference MEX files)
# ---------------------------------------------------------------------------
def mex_bundle_1_XABeUVWeAeB(K, a, b, X, visible):
    """[X_hat A B e U V W eA eB] = mex_bundle_1_XABeUVWeAeB(K, a, b, X, visible)."""
    K, a, b, X, vis = map(_F, (K, a, b, X, visible))
    num_a, m = a.shape
    n = b.shape[1]
    z = lambda *s: np.zeros(s, order="F")
    out = [z(2, n, m), z(2, num_a, n, m), z(2, 3, n, m), z(2, n, m), z(num_a, num_a, m),
           z(3, 3, n), z(num_a, 3, n, m), z(num_a, m), z(3, n)]
    check(lib().vlgba_mex_bundle_1(m, n, num_a, _dp(K), _dp(a), _dp(b), _dp(X), _dp(vis),
                                   *[_dp(q) for q in out]), "mex_bundle_1_XABeUVWeAeB")
    return tuple(out)


def mex_bundle_2_Se_(Y, W, U, eA, eB):
    """[S e_] = mex_bundle_2_Se_(Y, W, U, eA, eB)."""
    Y, W, U, eA, eB = map(_F, (Y, W, U, eA, eB))
    num_a, m = eA.shape
    n = eB.shape[1]
    S = np.zeros((num_a * m, num_a * m), order="F")
    e_ = np.zeros((num_a * m, 1), order="F")
    check(lib().vlgba_mex_bundle_2(m, n, num_a, _dp(Y), _dp(W), _dp(U), _dp(eA), _dp(eB),
                                   _dp(S), _dp(e_)), "mex_bundle_2_Se_")
    return S, e_


def mex_bundle_3_db_new(W, da, eB, V_inv, K, a, b, X, visible):
    """[db a_new b_new X_hat] = mex_bundle_3_db_new(W, da, eB, V_inv, K, a, b, X, visible)."""
    W, da, eB, Vinv, K, a, b, X, vis = map(_F, (W, da, eB, V_inv, K, a, b, X, visible))
    num_a, m = a.shape
    n = b.shape[1]
    db = np.zeros((3, n), order="F")
    a_new = np.zeros((num_a, m), order="F")
    b_new = np.zeros((3, n), order="F")
    X_hat = np.zeros((2, n, m), order="F")
    check(lib().vlgba_mex_bundle_3(m, n, num_a, _dp(W), _dp(da), _dp(eB), _dp(Vinv), _dp(K),
                                   _dp(a), _dp(b), _dp(X), _dp(vis), _dp(db), _dp(a_new),
                                   _dp(b_new), _dp(X_hat)), "mex_bundle_3_db_new")
    return db, a_new, b_new, X_hat
