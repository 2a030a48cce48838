"""Passes of the fast path on small scenes -- the step (da, db), the pass
scalars and the linearisation an accepted step takes (W, V, eB, U, eA) -- saved
to an .npz, and a comparison of two such files: bit-identity checks of a
kernel change between two builds (VLGBA_LIB=...).

usage: python tools/lin_dump.py OUT.npz          (dump, with the library in use)
       python tools/lin_dump.py --compare A.npz B.npz [--sse-tol 1e-13]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

SCENES = [("banded", dict(config="cfg2", m=30, n=3000, seed=17), 6, {}),
          ("fixstruct", dict(config="cfg1", m=12, min_n=150, max_n=250, seed=41), 6,
           dict(fix_structure=True)),
          ("pivot", dict(config="cfg1", m=12, min_n=150, max_n=250, seed=41), 6, "pivot"),
          ("cfg3s", dict(config="cfg2", m=200, n=40000, seed=3), 6, {})]


def dump(out):
    import bundleadjustmentmatlab_amd as pkg
    from bundleadjustmentmatlab_amd.scene import make_config
    res = {}
    for name, sk, na, kw in SCENES:
        sk = dict(sk)
        sc = make_config(sk.pop("config"), **sk)
        if kw == "pivot":
            kw = dict(pivot=np.arange(sc.m) < 2)
        a = np.vstack([sc.w0, sc.T0])
        b = np.asfortranarray(sc.X0[:3])
        with pkg.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, na, **kw) as ba:
            ba.set_params(a, b)
            for p in range(4):
                i = ba.step(relinearize=True, update_lm=True)
                da, db = ba.last_step()
                res[f"{name}_{p}_da"], res[f"{name}_{p}_db"] = da, db
                res[f"{name}_{p}_scal"] = np.array([i.old_sse, i.new_sse, i.dpg, i.accepted,
                                                    i.lambda_])
            for k, v in ba.linearization().items():
                res[f"{name}_lin_{k}"] = v
            pa, pb = ba.get_params()
            res[f"{name}_a"], res[f"{name}_b"] = pa, pb
    np.savez(out, **res)
    print(f"[lin_dump] {len(res)} arrays -> {out}")


def compare(fa, fb, sse_tol):
    A, B = np.load(fa), np.load(fb)
    bad = 0
    for k in sorted(A.files):
        x, y = A[k], B[k]
        if k.endswith("_scal"):
            ok = (x[3] == y[3] and x[4] == y[4] and
                  np.all(np.abs(x[:3] - y[:3]) <= sse_tol * np.abs(y[:3])))
        else:
            ok = np.array_equal(x, y)
        if not ok:
            bad += 1
            d = np.max(np.abs(x - y)) if x.shape == y.shape else "shape"
            print(f"[lin_dump] DIFF {k}: max |d| {d}")
    print(f"[lin_dump] {len(A.files)} arrays compared, {bad} differ "
          f"(scalars to {sse_tol:g} relative, the rest bit for bit)")
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        tol = float(sys.argv[sys.argv.index("--sse-tol") + 1]) if "--sse-tol" in sys.argv else 1e-13
        sys.exit(1 if compare(sys.argv[2], sys.argv[3], tol) else 0)
    dump(sys.argv[1])
