"""Is the default fast path's converged cost biased against the reference's?


For many independent LM solves, each started from the SAME point on the GPU
(default fast path) and on the oracle with the reference's MATLAB semantics
(SVD pinv for V*_i and S: oracle/bundle_euclid_ref.py, or the CPU port's
banded-Cholesky pinv at cfg2 / cfg3 sizes), under the tightened stop rule,
record the SIGNED relative difference (GPU final - oracle final) / oracle
final.  Beside it, the reference's own floor: the same oracle with lambda0
moved by 1 part in 1e9 (a rounding-size change to the start of the same
algorithm) against the unmoved oracle, and the GPU against itself the same
way.

Sets:
  small   6 cameras x 30-60 points (tests/test_gpu_lm_parity.py's "small"
          model), seeds 100 ..
  cfg1    config 1's model (10 x 100-200), seeds 100 ..
  banded  24 x 1500 banded (the "banded" model), seeds 100 ..
  cfg5    every solve of the 50-camera growing replay (config 5), re-run
          from its own inputs
  cfg2    config 2's model at full size (50 x 10k x 60k), seeds 2 ..
  cfg3    config 3 (1000 x 500k x 3M), seeds 3 ..

Usage (GPU box): python tools/converged_bias.py --out gpurun_out/bias.json
  [--sets small,cfg1,banded,cfg5,cfg2,cfg3] [--nseed 30] [--big-seeds 4]
Oracle work runs in a spawned process pool beside the GPU solves.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor
import multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

KW = dict(stop_rel=1e-9, max_iter=100, max_iter2=30)          # test_gpu_lm_parity.py
STOP_BIG = dict(stop_rel=1e-12, max_iter=200, max_iter2=30)   # test_gpu_converged.py
EPS_L0 = 1e-9                                                 # the floor's lambda0 move


def small_scene(kind, seed):
    from bundleadjustmentmatlab_amd.scene import make_config
    if kind == "small":
        return make_config("cfg1", m=6, min_n=30, max_n=60, seed=seed)
    if kind == "cfg1":
        return make_config("cfg1", seed=seed)
    if kind == "banded":
        return make_config("cfg2", m=24, n=1500, seed=seed)
    raise ValueError(kind)


# ---------------------------------------------------------------- oracle side
def oracle_small(kind, seed):
    import bundle_euclid_ref as ref
    sc = small_scene(kind, seed)
    x, vis = sc.dense()
    out = {}
    for nm, l0 in (("ref", 1e-3), ("ref_l0", 1e-3 * (1 + EPS_L0))):
        r = ref.bundle_euclid_ref(sc.K, sc.T0, sc.w0, sc.X0, x, "visibility", vis,
                                  "fix_calibration", form="sparse", vinv="pinv", solve="pinv",
                                  lambda0=l0, **KW)
        out[nm] = float(r[4][-1])
        out[nm + "_n"] = len(r[4])
    return (kind, seed), out


def oracle_call(q, c):
    """one replay solve on the oracle (MATLAB semantics) from its inputs"""
    import bundle_euclid_ref as ref
    from test_gpu_full_configs import _dense
    x, vis = _dense(c)
    out = {}
    for nm, l0 in (("ref", 1e-3), ("ref_l0", 1e-3 * (1 + EPS_L0))):
        r = ref.bundle_euclid_ref(c["K"], c["T"], c["w"], c["X"], x, "visibility", vis,
                                  *c["opts"], form="sparse", vinv="pinv", solve="pinv",
                                  lambda0=l0, **KW)
        out[nm] = float(r[4][-1]) if len(r[4]) else None
    return ("cfg5", q), out


def oracle_big(name, seed):
    import cpu_port
    from bundleadjustmentmatlab_amd.scene import make_config
    sc = make_config(name, seed=seed)
    a0 = np.vstack([sc.w0, sc.T0])
    b0 = np.asfortranarray(sc.X0[:3])
    port = cpu_port.SparsePort(sc.m, sc.n, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.K)
    out = {}
    for nm, l0 in (("ref", 1e-3), ("ref_l0", 1e-3 * (1 + EPS_L0))):
        e, _, _, info = port.lm(a0, b0, vinv="pinv", solve="band", check_pinv=0, lambda0=l0,
                                **STOP_BIG)
        out[nm] = float(e[-1])
        out[nm + "_n"] = int(info["passes"])
    return (name, seed), out


# ------------------------------------------------------------------- GPU side
def gpu_small(pkg, kind, seed):
    sc = small_scene(kind, seed)
    x, vis = sc.dense()
    out = {}
    for nm, l0 in (("gpu", 1e-3), ("gpu_l0", 1e-3 * (1 + EPS_L0))):
        g = pkg.bundle_euclid(sc.K, sc.T0, sc.w0, sc.X0, x, "visibility", vis, "fix_calibration",
                              lambda0=l0, **KW)
        out[nm] = float(g[4][-1])
        out[nm + "_n"] = len(g[4])
    return out


def gpu_call(c):
    from bundleadjustmentmatlab_amd.bundle import bundle_euclid_obs
    nv = float(len(c["pt"]))
    out = {}
    for nm, l0 in (("gpu", 1e-3), ("gpu_l0", 1e-3 * (1 + EPS_L0))):
        g = bundle_euclid_obs(c["K"], c["T"], c["w"], c["X"], c["pt"], c["cam"], c["ox"],
                              *c["opts"], num_vis=nv, lambda0=l0, **KW)
        out[nm] = float(g[4][-1]) if len(g[4]) else None
    return out


def gpu_big(pkg, name, seed):
    from bundleadjustmentmatlab_amd.scene import make_config
    sc = make_config(name, seed=seed)
    a = np.vstack([sc.w0, sc.T0])
    b = np.asfortranarray(sc.X0[:3])
    out = {}
    for nm, l0 in (("gpu", 1e-3), ("gpu_l0", 1e-3 * (1 + EPS_L0))):
        with pkg.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, 6, lambda0=l0,
                                **STOP_BIG) as ba:
            ba.set_params(a, b)
            err, st = ba.run()
        out[nm] = float(err[-1])
        out[nm + "_n"] = int(st.iterations)
    return out


# ------------------------------------------------------------------ summary
def sign_test_p(pos, neg):
    """two-sided exact binomial p of a sign count (ties dropped)"""
    n = pos + neg
    if n == 0:
        return 1.0
    k = min(pos, neg)
    tail = sum(math.comb(n, i) for i in range(k + 1)) / 2.0 ** n
    return min(1.0, 2 * tail)


def summarize(rows):
    """rows: dicts with gpu, ref, gpu_l0, ref_l0 finals"""
    d = np.array([(r["gpu"] - r["ref"]) / r["ref"] for r in rows
                  if r.get("gpu") is not None and r.get("ref") is not None])
    f_ref = np.array([(r["ref_l0"] - r["ref"]) / r["ref"] for r in rows
                      if r.get("ref_l0") is not None and r.get("ref") is not None])
    f_gpu = np.array([(r["gpu_l0"] - r["gpu"]) / r["gpu"] for r in rows
                      if r.get("gpu_l0") is not None and r.get("gpu") is not None])
    pos, neg = int((d > 0).sum()), int((d < 0).sum())

    def q(v):
        if len(v) == 0:
            return None
        return dict(n=int(len(v)), median=float(np.median(v)), mean=float(v.mean()),
                    median_abs=float(np.median(np.abs(v))), p90_abs=float(np.quantile(np.abs(v), 0.9)),
                    max_abs=float(np.abs(v).max()))
    return dict(gpu_minus_ref=q(d), pos=pos, neg=neg, zero=int((d == 0).sum()),
                sign_test_p=sign_test_p(pos, neg), ref_floor=q(f_ref), gpu_floor=q(f_gpu),
                signed=[float(v) for v in d])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/converged_bias.json")
    ap.add_argument("--sets", default="small,cfg1,banded,cfg5,cfg2,cfg3")
    ap.add_argument("--nseed", type=int, default=30)
    ap.add_argument("--big-seeds", type=int, default=4)
    ap.add_argument("--workers", type=int, default=8)
    args = ap.parse_args()
    sets = args.sets.split(",")
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    t0 = time.time()
    # the oracle pool is spawned before anything touches the GPU
    pool = ProcessPoolExecutor(args.workers, mp_context=mp.get_context("spawn"))
    futs = []
    for kind in ("small", "cfg1", "banded"):
        if kind in sets:
            futs += [pool.submit(oracle_small, kind, 100 + s) for s in range(args.nseed)]
    big = [(nm, s0 + s) for nm, s0 in (("cfg2", 2), ("cfg3", 3)) if nm in sets
           for s in range(args.big_seeds)]
    # the CPU port uses OpenMP: one big oracle at a time beside the small ones
    big_pool = ProcessPoolExecutor(1, mp_context=mp.get_context("spawn")) if big else None
    big_futs = [big_pool.submit(oracle_big, nm, s) for nm, s in big]

    import torch
    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    import bundleadjustmentmatlab_amd as pkg
    rows = {}
    for kind in ("small", "cfg1", "banded"):
        if kind in sets:
            for s in range(args.nseed):
                rows[(kind, 100 + s)] = gpu_small(pkg, kind, 100 + s)
            print(f"[bias] GPU {kind} done {time.time() - t0:.0f}s", flush=True)
    if "cfg5" in sets:
        from test_gpu_full_configs import _replay
        from bundleadjustmentmatlab_amd.scene import make_config
        _, calls = _replay(pkg, make_config("cfg5"))
        for q, c in enumerate(calls):
            c2 = {k: v for k, v in c.items() if k != "out"}
            futs.append(pool.submit(oracle_call, q, c2))
            rows[("cfg5", q)] = gpu_call(c2)
        print(f"[bias] GPU cfg5 {len(calls)} solves done {time.time() - t0:.0f}s", flush=True)
    for nm, s in big:
        rows[(nm, s)] = gpu_big(pkg, nm, s)
        print(f"[bias] GPU {nm} seed {s} done {time.time() - t0:.0f}s", flush=True)
    from concurrent.futures import as_completed
    for f in as_completed(futs + big_futs):   # a line per result: the box's silence watchdog
        key, out = f.result()
        rows[key].update(out)
        print(f"[bias] oracle {key[0]} {key[1]} done {time.time() - t0:.0f}s", flush=True)
    print(f"[bias] oracle done {time.time() - t0:.0f}s", flush=True)
    pool.shutdown()
    if big_pool:
        big_pool.shutdown()
    res = {"what": __doc__.split("\n\n")[0], "stop_small": KW, "stop_big": STOP_BIG,
           "eps_lambda0": EPS_L0, "sets": {}, "rows": {f"{k[0]}:{k[1]}": v for k, v in rows.items()}}
    allrows = []
    for st in sets:
        rs = [v for k, v in rows.items() if k[0] == st]
        if rs:
            res["sets"][st] = summarize(rs)
            allrows += rs
    res["all"] = summarize(allrows)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    for st, sm in list(res["sets"].items()) + [("all", res["all"])]:
        g = sm["gpu_minus_ref"]
        fr, fg = sm["ref_floor"], sm["gpu_floor"]
        print(f"[bias] {st:7s} n={g['n']:3d} +{sm['pos']} -{sm['neg']} ={sm['zero']} "
              f"p={sm['sign_test_p']:.3f} | GPU-ref median {g['median']:+.2e} |med| "
              f"{g['median_abs']:.2e} max {g['max_abs']:.2e} | ref floor |med| "
              f"{fr['median_abs'] if fr else float('nan'):.2e} max "
              f"{fr['max_abs'] if fr else float('nan'):.2e} | GPU floor |med| "
              f"{fg['median_abs'] if fg else float('nan'):.2e}", flush=True)


if __name__ == "__main__":
    main()
