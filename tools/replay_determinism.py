"""Is the growing replay deterministic?  The cfg5x-M segment replayed several
times -- in one process, or each run in a fresh process (--fresh) -- with the
prefetch on (2 or 1 workers) or off: the first solve whose final error differs
from the first run's, and the pinv passes.

usage: python tools/replay_determinism.py [M] [--runs pf2,pf2,none] [--fresh]
  a run spec ending in "@spin" (with --fresh) reports a hand-off timeout on
  every pass (VLGBA_DEBUG_SPIN_TIMEOUT): every pass re-solved without spins
"""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402


def run(M, spec):
    import bundleadjustmentmatlab_amd.incremental as inc
    from bundleadjustmentmatlab_amd.scene import make_config
    sc = make_config("cfg5x", m=M)
    pinv, spin = [], []
    orig = inc.bundle_euclid_obs

    def spy(*a, **kw):
        r = orig(*a, **kw)
        pinv.append(int(r[-1].pinv_passes))
        spin.append(int(r[-1].spin_retries))
        return r
    inc.bundle_euclid_obs = spy
    spec = spec.split("@")[0]
    if spec.startswith("pf"):
        inc.PREFETCH_WORKERS = int(spec[2:] or 2)
    try:
        res = inc.incremental_bundle(sc, devices=[0], prefetch=spec != "none")
    finally:
        inc.bundle_euclid_obs = orig
    e = [float(q["error"][-1]) if len(q["error"]) else float("nan") for q in res["solves"]]
    info = [(q["tag"], q["camera"], int(q["passes"]), float(q["error"][0]) if len(q["error"]) else 0.0)
            for q in res["solves"]]
    return e, pinv, dict(res["prefetch"], spin_retries=sum(spin)), info


def main():
    args = sys.argv[1:]
    M = int(args[0]) if args and args[0].isdigit() else 600
    specs = args[args.index("--runs") + 1].split(",") if "--runs" in args else ["pf2", "pf2", "none"]
    if "--child" in args:
        print("JSON" + json.dumps(run(M, specs[0])))
        return
    out = []
    for spec in specs:
        if "--fresh" in args:
            env = dict(os.environ)
            if spec.endswith("@spin"):
                env["VLGBA_DEBUG_SPIN_TIMEOUT"] = "0:1000000"
            p = subprocess.run([sys.executable, "-u", __file__, str(M), "--runs", spec, "--child"],
                               capture_output=True, text=True, timeout=1000, env=env)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("JSON")]
            if p.returncode != 0 or not line:
                print(spec, "failed", p.returncode, p.stderr[-2000:])
                return
            out.append((spec, json.loads(line[-1][4:])))
        else:
            out.append((spec, run(M, spec)))
    ref_e = np.array(out[0][1][0])
    ref_info = out[0][1][3]
    for spec, (e, p, st, info) in out:
        e = np.array(e)
        d = np.flatnonzero(~((e == ref_e) | (np.isnan(e) & np.isnan(ref_e))))
        f = int(d[0]) if len(d) else None
        print(f"{spec}: final {e[-1]:.9f}, pinv passes {sum(p)} at solves "
              f"{np.flatnonzero(p).tolist()}, prefetch {st}, first solve differing from run 1: {f}",
              flush=True)
        if f is not None:
            print(f"   run 1 solve {f}: {ref_info[f]} final {ref_e[f]!r}")
            print(f"   this  solve {f}: {info[f]} final {e[f]!r}")


if __name__ == "__main__":
    main()
