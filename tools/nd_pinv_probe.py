"""Why the nested-dissection envelope meets non-positive pivots on the scaled
growing replay (cfg5x) where the natural order does not.

Replays cfg5x with the default solver; every solve that took a pinv step is
saved (inputs + per-pass log) under OUT/solve_<k>.npz.  For each such solve the
failing pass is then re-created (a fresh handle stepped to the pass before it,
so the state and lambda are the ones the failing pass saw) for the ND and the
natural order, and on the reduced system S of that pass (numpy, this host):
  * the eigenvalues of S against MATLAB pinv's tolerance (bundle_euclid.m:193),
  * LAPACK dpotrf on the natural and on the ND row order: the first failing
    leading minor, its camera, arc / separator, and the pivot's value left
    after elimination relative to the diagonal entry it started from.

usage: python tools/nd_pinv_probe.py [OUT] [max_solves]
"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import scipy.linalg.lapack as lapack  # noqa: E402

import bundleadjustmentmatlab_amd as pkg  # noqa: E402
import bundleadjustmentmatlab_amd.incremental as inc  # noqa: E402
from bundleadjustmentmatlab_amd._lib import lib  # noqa: E402
from bundleadjustmentmatlab_amd.bundle import pack_a  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402

NB = 64


def nd_rows(m, na, jk):
    """camera -> first row of the ND order (ba_chol_setup), the separator's
    first row, and the arcs' boundaries"""
    flat = np.ascontiguousarray(jk.reshape(-1), dtype=np.int32)
    bnd = np.zeros(9, dtype=np.int32)
    crit = ctypes.c_int(0)
    P = ctypes.POINTER(ctypes.c_int)
    K = lib().vlgba_debug_nd_plan(m, na, flat.ctypes.data_as(P), len(jk),
                                  bnd.ctypes.data_as(P), ctypes.byref(crit))
    if K <= 0:
        return None, None, None
    minK = np.arange(m)
    for j, k in jk:
        minK[j] = min(minK[j], k)
    crow = np.full(m, -1)
    row = 0
    for t in range(K):
        for j in range(bnd[t], bnd[t + 1]):
            if minK[j] >= bnd[t]:
                crow[j] = row
                row += na
        row = (row + NB - 1) // NB * NB
    s0 = row
    for t in range(K):
        for j in range(bnd[t], bnd[t + 1]):
            if minK[j] < bnd[t]:
                crow[j] = row
                row += na
    return crow, s0, bnd[:K + 1].tolist()


def potrf_probe(S, order):
    """dpotrf of S[order][:, order]: (info, pivot left / starting diagonal)"""
    A = np.asfortranarray(S[np.ix_(order, order)])
    c, info = lapack.dpotrf(A, lower=1, clean=0, overwrite_a=0)
    if info <= 0:
        return 0, None
    i = info - 1
    L = np.tril(c[:i, :i])
    r = A[i, :i]
    y = np.linalg.solve(L, r) if i else r
    left = A[i, i] - y @ y
    return info, float(left / A[i, i])


def analyse(tag, args, kw, fail_pass, solver):
    K, T, w, X, pt, cam, x = args
    a = pack_a(K, T, w, 0)
    b = np.asfortranarray(X[:3])
    out = {"solver": solver}
    with pkg.BundleAdjuster(K, pt, cam, x, X.shape[1], 6, solver=solver,
                            num_vis=kw.get("num_vis", 0.0)) as ba:
        ba.set_params(a, b)
        lam = None
        for _ in range(fail_pass - 1):
            info = ba.step(relinearize=False, update_lm=True)
        jk, blocks, e_ = ba.reduced_system(dense=False)
        S, e = ba.reduced_system(dense=True)
        info = ba.step(relinearize=False, update_lm=False)
        out["pinv_here"] = bool(info.pinv)
        out["lambda"] = info.lambda_
        plan = ba.plan_info()
        out["nd_arcs"], out["nd_sep_tiles"], out["tiles"] = (plan["nd_arcs"], plan["nd_sep_tiles"],
                                                            plan["tiles"])
    m = K.shape[1]
    na = 6
    S = np.tril(S) + np.tril(S, -1).T
    d = np.diag(S).copy()
    z = np.flatnonzero(d == 0.0)
    S[z, z] = 1.0
    ev = np.linalg.eigvalsh(S)
    tol = S.shape[0] * np.spacing(np.abs(ev).max())
    out["eig_min"], out["eig_max"] = float(ev[0]), float(ev[-1])
    out["eig_below_pinv_tol"] = int((np.abs(ev) <= tol).sum())
    out["eig_neg"] = int((ev < 0).sum())
    out["eig_low8"] = [float(v) for v in ev[:8]]
    nat = np.arange(S.shape[0])
    info_n, rel_n = potrf_probe(S, nat)
    out["potrf_natural"] = {"info": int(info_n), "pivot_rel": rel_n,
                            "camera": int((info_n - 1) // na) if info_n else None}
    crow, s0, bnd = nd_rows(m, na, jk)
    if crow is not None:
        # ND row r -> original row (the padding rows between parts dropped)
        perm = np.full(int(crow.max()) + na, -1, dtype=np.int64)
        for j in range(m):
            perm[crow[j]:crow[j] + na] = np.arange(na * j, na * j + na)
        perm = perm[perm >= 0]
        info_d, rel_d = potrf_probe(S, perm)
        cam_d = int(perm[info_d - 1] // na) if info_d else None
        out["potrf_nd"] = {"info": int(info_d), "pivot_rel": rel_d, "camera": cam_d,
                           "in_separator": bool(info_d and crow[cam_d] >= s0), "bnd": bnd,
                           "sep_first_row": int(s0),
                           "sep_cams": int((crow >= s0).sum())}
    print(f"[probe] {tag} {solver}: {json.dumps(out)}", flush=True)
    return out


def main():
    outdir = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/nd_probe"
    maxs = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    os.makedirs(outdir, exist_ok=True)
    sc = make_config("cfg5x")
    orig = inc.bundle_euclid_obs
    failed = []
    count = [0]

    def wrapped(*args, **kw):
        recs = []
        kw2 = dict(kw)
        kw2["log"] = recs.append
        r = orig(*args, **kw2)
        k = count[0]
        count[0] += 1
        if any(q["pinv"] for q in recs):
            K, T, w, X, pt, cam, x = args[:7]
            p = 1 + next(i for i, q in enumerate(recs) if q["pinv"])
            np.savez_compressed(os.path.join(outdir, f"solve_{k}.npz"), K=K, T=T, w=w, X=X,
                                pt=pt, cam=cam, x=x, num_vis=kw.get("num_vis", 0.0),
                                log=json.dumps(recs))
            print(f"[probe] solve {k}: {K.shape[1]} cams {len(pt)} obs, pinv at pass {p} "
                  f"of {len(recs)} (lambda {recs[p - 1]['lambda']:.3g}); "
                  f"passes {[(q['lambda'], q['accepted'], q['pinv']) for q in recs]}", flush=True)
            failed.append((k, tuple(np.array(a, copy=True) for a in args[:7]), dict(kw), p))
        return r

    inc.bundle_euclid_obs = wrapped
    t0 = time.perf_counter()
    res = inc.incremental_bundle(sc, devices=[0])
    sol = res["solves"]
    print(f"[probe] replay {time.perf_counter() - t0:.1f} s, {len(sol)} solves, "
          f"{len(failed)} with a pinv step, final error "
          f"{next(q['error'][-1] for q in reversed(sol) if len(q['error'])):.6f}", flush=True)
    inc.bundle_euclid_obs = orig
    summary = []
    for k, args, kw, p in failed[:maxs]:
        for solver in ("auto", "envelope"):
            summary.append(dict(solve=k, pass_=p, **analyse(f"solve {k} pass {p}", args, kw, p,
                                                              solver)))
    with open(os.path.join(outdir, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
