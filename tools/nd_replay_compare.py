"""The scaled growing replay (cfg5x) with the nested-dissection envelope
(default solver) and with the natural camera order (VLGBA_ND=0), solve by
solve: where the two trajectories part, and how the error_ of each solve
compares (final error 0.83 with ND vs 0.55 natural).

Writes OUT/replay_<mode>.json (per solve: cameras, points, observations,
error_ first / last, passes, accepted, pinv passes) and prints the first
solve whose final error differs by > 1e-9 / 1e-6 / 1e-3 relative and a
coarse table of both error traces.

usage: python tools/nd_replay_compare.py [OUT] [config]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bundleadjustmentmatlab_amd.incremental as inc  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402


def replay(sc, nd):
    if nd:
        os.environ.pop("VLGBA_ND", None)
    else:
        os.environ["VLGBA_ND"] = "0"
    orig = inc.bundle_euclid_obs
    extra = []

    def wrapped(*a, **kw):
        r = orig(*a, **kw)
        st = r[-1]
        extra.append(int(st.pinv_passes))
        return r
    inc.bundle_euclid_obs = wrapped
    t0 = time.perf_counter()
    res = inc.incremental_bundle(sc, devices=[0])
    inc.bundle_euclid_obs = orig
    out = []
    for q, pv in zip(res["solves"], extra):
        e = q["error"]
        out.append(dict(tag=q["tag"], camera=q["camera"], cameras=q["cameras"], points=q["points"],
                        observations=q["observations"], e0=float(e[0]) if len(e) else None,
                        e1=float(e[-1]) if len(e) else None, passes=q["passes"],
                        accepted=q["accepted"], pinv=pv))
    print(f"[replay] {'nd' if nd else 'natural'}: {time.perf_counter() - t0:.1f} s, "
          f"{len(out)} solves, pinv passes {sum(extra)}", flush=True)
    return out


def main():
    outdir = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/nd_replay"
    cfg = sys.argv[2] if len(sys.argv) > 2 else "cfg5x"
    os.makedirs(outdir, exist_ok=True)
    sc = make_config(cfg)
    runs = {}
    for nd in (True, False):
        runs[nd] = replay(sc, nd)
        with open(os.path.join(outdir, f"replay_{'nd' if nd else 'natural'}.json"), "w") as f:
            json.dump(runs[nd], f)
    A, B = runs[True], runs[False]
    for tol in (1e-12, 1e-9, 1e-6, 1e-3, 1e-1):
        k = next((i for i, (a, b) in enumerate(zip(A, B))
                  if a["e1"] is not None and b["e1"] is not None and
                  abs(a["e1"] - b["e1"]) > tol * b["e1"]), None)
        print(f"first solve with final error differing by > {tol:g}: {k}"
              + (f" ({A[k]['cameras']} cams, nd {A[k]['e1']:.9g} natural {B[k]['e1']:.9g})"
                 if k is not None else ""), flush=True)
    print(" solve  cams   nd e0      nd e1    | nat e0     nat e1   | nd/nat passes")
    for i in list(range(0, len(A), max(1, len(A) // 40))) + [len(A) - 1]:
        a, b = A[i], B[i]
        f = lambda v: f"{v:9.5f}" if v is not None else "     None"   # noqa: E731
        print(f" {i:5d} {a['cameras']:5d} {f(a['e0'])} {f(a['e1'])} | {f(b['e0'])} {f(b['e1'])} | "
              f"{a['passes']}/{b['passes']}")


if __name__ == "__main__":
    main()
