"""One growing-replay solve where the nested-dissection envelope and the
natural order part: the cfg5x replay (default solver) up
to solve K, that solve's inputs saved, then the solve re-run pass by pass for
the ND / natural / dense solvers, each pass's da checked against numpy's solve
of the same reduced system (relative residual, difference).

usage: python tools/nd_solve_debug.py [K] [OUT]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bundleadjustmentmatlab_amd as pkg  # noqa: E402
import bundleadjustmentmatlab_amd.incremental as inc  # noqa: E402
from bundleadjustmentmatlab_amd.bundle import pack_a  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402


class Stop(Exception):
    pass


def capture(sc, K):
    orig = inc.bundle_euclid_obs
    cnt = [0]
    got = {}

    def wrapped(*a, **kw):
        if cnt[0] == K:
            got["args"] = tuple(np.array(v, copy=True) for v in a[:7])
            got["opts"] = a[7:]
            got["kw"] = kw
            raise Stop()
        cnt[0] += 1
        return orig(*a, **kw)
    inc.bundle_euclid_obs = wrapped
    try:
        inc.incremental_bundle(sc, devices=[0])
    except Stop:
        pass
    finally:
        inc.bundle_euclid_obs = orig
    return got


def run(args, kw, solver, npass=40):
    Kc, T, w, X, pt, cam, x = args
    a = pack_a(Kc, T, w, 0)
    b = np.asfortranarray(X[:3])
    rows = []
    with pkg.BundleAdjuster(Kc, pt, cam, x, X.shape[1], 6, solver=solver,
                            num_vis=kw.get("num_vis", 0.0)) as ba:
        ba.set_params(a, b)
        plan = ba.plan_info()
        for p in range(npass):
            S, e = ba.reduced_system(dense=True)
            S = np.tril(S) + np.tril(S, -1).T
            e = e.reshape(-1).copy()
            z = np.flatnonzero(np.diag(S) == 0.0)
            S[z, z] = 1.0
            e[z] = 0.0
            info = ba.step(relinearize=False, update_lm=True)
            da, _ = ba.last_step()
            d = da.reshape(-1, order="F")
            ref = np.linalg.solve(S, e)
            res = np.linalg.norm(S @ d - e) / np.linalg.norm(e)
            rows.append(dict(p=p, lam=info.lambda_, acc=int(info.accepted), rho=info.rho,
                             old=info.old_sse, new=info.new_sse, pinv=int(info.pinv),
                             res=float(res),
                             diff=float(np.abs(d - ref).max() / np.abs(ref).max()),
                             dmax=float(np.abs(d).max()), refmax=float(np.abs(ref).max()),
                             cond=float(np.linalg.cond(S)) if p < 3 or not info.accepted else None))
    return plan, rows


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 823
    out = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/nd_solve_debug"
    os.makedirs(out, exist_ok=True)
    sc = make_config("cfg5x")
    got = capture(sc, K)
    args, kw = got["args"], got["kw"]
    np.savez_compressed(os.path.join(out, f"solve_{K}.npz"), *args, num_vis=kw.get("num_vis", 0.0))
    print(f"solve {K}: {args[0].shape[1]} cams, {args[3].shape[1]} pts, {len(args[4])} obs, "
          f"opts {got['opts']}", flush=True)
    summary = {}
    for solver in ("nd", "envelope", "dense"):
        plan, rows = run(args, kw, solver)
        summary[solver] = rows
        print(f"--- {solver}: arcs {plan['nd_arcs']} sep tiles {plan['nd_sep_tiles']} tiles "
              f"{plan['tiles']}", flush=True)
        for r in rows:
            c = f"{r['cond']:.1e}" if r["cond"] else "   -   "
            print(f"  pass {r['p']:2d} lam {r['lam']:.3e} acc {r['acc']} rho {r['rho']:+.3e} "
                  f"old {r['old']:.6e} new {r['new']:.6e} res {r['res']:.1e} diff {r['diff']:.1e} "
                  f"|da| {r['dmax']:.2e} |ref| {r['refmax']:.2e} cond {c}", flush=True)
    with open(os.path.join(out, f"solve_{K}.json"), "w") as f:
        json.dump(summary, f)


if __name__ == "__main__":
    main()
