"""Diagnostic (not part of the library): run the same fast-path solves with
and without VLGBA_POISON=1 (every device block handed out filled with 0xff
bytes) and print the first LM pass whose cost differs, per solver / Schur
kernel variant.  A difference means some kernel reads memory it never wrote.

  python tools/poison_diff.py            # parent: runs both children
"""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

VARIANTS = [(kind, solver, sk) for kind in ("small", "banded")
            for solver in ("dense", "envelope", "auto") for sk in ("auto", "terms")]


def child():
    import numpy as np
    import bundleadjustmentmatlab_amd as ba
    from bundleadjustmentmatlab_amd.scene import make_config
    out = {}
    for kind, solver, sk in VARIANTS:
        sc = (make_config("cfg1", m=6, min_n=30, max_n=60, seed=7) if kind == "small"
              else make_config("cfg2", m=24, n=1500, seed=9))
        x, vis = sc.dense()
        recs = []
        got = ba.bundle_euclid(sc.K, sc.T0, sc.w0, sc.X0, x, "visibility", vis,
                               "fix_calibration", stop_rel=1e-9, max_iter=100, max_iter2=30,
                               solver=solver, schur_kernel=sk, log=recs.append)
        out[f"{kind}/{solver}/{sk}"] = {
            "err": [float(v).hex() for v in np.asarray(got[4]).ravel()],
            "pass": [[r.get("pass"), r.get("pinv"), r.get("chol_failed"), r.get("accepted"),
                      float(r.get("new_sse", 0.0)).hex()] for r in recs]}
    print("JSON" + json.dumps(out))


def main():
    res = {}
    runs = [("plain", {}), ("poison", {"VLGBA_POISON": "1"})]
    runs += [(f"plain{i}", {}) for i in range(2, 2 + int(os.environ.get("PDIFF_REPEAT", "0")))]
    for tag, env in runs:
        e = dict(os.environ, **env)
        p = subprocess.run([sys.executable, "-u", __file__, "--child"], env=e,
                           capture_output=True, text=True, timeout=600)
        line = [l for l in p.stdout.splitlines() if l.startswith("JSON")]
        if p.returncode != 0 or not line:
            print(tag, "child failed", p.returncode, p.stderr[-3000:])
            return 1
        res[tag] = json.loads(line[-1][4:])
    for tag in [t for t, _ in runs[1:]]:
      print("--- plain vs", tag)
      for k in res["plain"]:
        a, b = res["plain"][k], res[tag][k]
        first = next((i for i, (u, v) in enumerate(zip(a["pass"], b["pass"])) if u != v), None)
        same = a["err"] == b["err"]
        print(f"{k:28s} {'same' if same else 'DIFFERS'}  passes {len(a['pass'])}/{len(b['pass'])}"
              f"  first differing pass {first}  final {float.fromhex(a['err'][-1]):.12g} / {float.fromhex(b['err'][-1]):.12g}")
        if first is not None:
            print("   plain ", a["pass"][first])
            print("   poison", b["pass"][first])
    return 0


if __name__ == "__main__":
    if "--child" in sys.argv:
        child()
    else:
        sys.exit(main())
