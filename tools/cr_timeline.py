#!/usr/bin/env python3
"""Record timeline of the one-launch cyclic reduction (k_cr32_fused),
diagnostic build.

Build ``make -C bundleadjustmentmatlab_amd/csrc stamps`` (libvlgba_stamps.so,
-DBA_STAMPS), then on the GPU box:  python tools/cr_timeline.py [cfg]
Per level: when its records start, finish waiting, finish computing and have
published (us from the launch's first record, median over the level), and the
mean wait / compute / publish times -- the critical path of the launch.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bundleadjustmentmatlab_amd._lib as L  # noqa: E402

L.LIB_PATH = os.environ.get("VLGBA_LIB") or os.path.join(ROOT, "bundleadjustmentmatlab_amd",
                                                       "libvlgba_stamps.so")
from bundleadjustmentmatlab_amd import BundleAdjuster  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402


def record_levels(nt, ncu=256, roles=None):
    """Block -> (kind, level) of k_cr32_fused, as ba_chol_setup / ba_chol_solve
    lay the records out (``roles``, if given, receives each block's role)."""
    roles = [] if roles is None else roles
    act = list(range(nt))
    levels = []
    while act:
        elim = act[0::2]
        keep = act[1::2]
        levels.append((len(elim), len(keep)))
        act = keep
    kinds = []
    ne0 = levels[0][0]
    per = 2 if 3 * ne0 > ncu else 3
    kinds += [("factor", 0)] * (per * ne0)
    roles[:] = [(2 if (b & 1) else 4) if per == 2 else b % 3 for b in range(per * ne0)]
    for lv in range(1, len(levels)):
        ne = levels[lv][0]
        kinds += [("fused", lv)] * (3 * ne) + [("survivor", lv)] * levels[lv][1]
        roles += [b % 3 for b in range(3 * ne)] + [3] * levels[lv][1]
    kinds += [("back", -1)] * nt
    roles += [-1] * nt
    return kinds


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
    sc = make_config(cfg)
    lib = L.lib()
    fn = lib.vlgba_debug_crstamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    a = np.zeros((6, sc.m), order="F")
    a[0:3], a[3:6] = sc.w0, sc.T0
    b = np.asfortranarray(sc.X0[:3])
    ba = BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, 6)
    ba.set_params(a, b)
    for _ in range(4):
        ba.step(relinearize=True, update_lm=False)
    ba.sync()
    plan = ba.plan_info()
    rows = plan["cr_rows"]
    nt = -(-6 * sc.m // rows)
    roles = []
    kinds = record_levels(nt, roles=roles)
    roles = np.array(roles)
    nrec = len(kinds)
    st = (ctypes.c_ulonglong * (12 * nrec))()
    assert fn(st, nrec) == 0
    t8 = np.array(st, dtype=np.float64).reshape(nrec, 12)[:, :8] / 100.0   # us
    fch = lib.vlgba_debug_chstamps
    fch.restype = ctypes.c_int
    fch.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    sc2 = (ctypes.c_ulonglong * (2 * nrec))()
    assert fch(sc2, nrec) == 0
    tch = np.array(sc2, dtype=np.float64).reshape(nrec, 2) / 100.0
    t0 = t8[:, 0].min()
    t8 -= t0
    tch -= t0
    t = t8[:, :4]
    print(f"{cfg}: {nt} tiles of {rows} rows, {nrec} records; launch span "
          f"{t[:, 3].max():.1f} us")
    print("   kind     lvl  n   start  waited  computed  published | wait  compute  publish (us)")
    groups = {}
    for i, k in enumerate(kinds):
        groups.setdefault(k, []).append(i)
    for k in sorted(groups, key=lambda k: (k[0] == "back", k[1], k[0] != "factor",
                                          k[0] == "survivor")):
        idx = groups[k]
        tt = t[idx]
        med = np.median(tt, axis=0)
        d = np.mean(tt[:, 1:] - tt[:, :-1], axis=0)
        print(f"  {k[0]:9s} {k[1]:3d} {len(idx):4d} {med[0]:7.1f} {med[1]:7.1f} {med[2]:9.1f} "
              f"{med[3]:9.1f} | {d[0]:5.1f} {d[1]:7.1f} {d[2]:7.1f}")
    # inside the level body of the panel roles (1, 2: the next level's inputs)
    print("   panel records (roles 1/2)  | wait  loads  update  factor+panel  panel  store+publish (us)"
          "  [F0  M  F1]")
    for lv in sorted({k[1] for k in kinds if k[0] in ("factor", "fused")}):
        idx = [i for i, k in enumerate(kinds) if k[1] == lv and k[0] in ("factor", "fused")
               and roles[i] in (1, 2, 4)]
        if not idx:
            continue
        x = np.concatenate([t8[idx], tch[idx]], axis=1)
        # records whose role skipped the body (no neighbour on that side) leave
        # stale sub-stamps: only stamps inside [entry, published] count
        for c in range(4, 10):
            bad = (x[:, c] < x[:, 0]) | (x[:, c] > x[:, 3])
            x[bad, c] = np.nan
        seq = [x[:, 1] - x[:, 0], x[:, 4] - x[:, 1], x[:, 5] - x[:, 4], x[:, 6] - x[:, 5],
               x[:, 7] - x[:, 6], x[:, 3] - x[:, 7]]
        sub = [x[:, 8] - x[:, 5], x[:, 9] - x[:, 8], x[:, 6] - x[:, 9]]
        print(f"   level {lv:2d} ({len(idx):3d} records)      | " +
              "  ".join(f"{np.nanmedian(v):5.2f}" for v in seq) + "  [" +
              "  ".join(f"{np.nanmedian(v):4.2f}" for v in sub) + "]")
    ba.close()


if __name__ == "__main__":
    main()
