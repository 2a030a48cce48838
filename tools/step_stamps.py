"""Per-column timeline of the envelope Cholesky (k_factor_step /
k_factor_multi) from the BA_STAMPS build (tools/ab_build.sh stamps
-DBA_STAMPS=1): workgroup 0 (diagonal) and 1 (first panel tile) entry,
factor start / end, exit, and the last workgroup's exit, per tile column.

usage: VLGBA_LIB=tools/build/ab/stamps/libvlgba.so python tools/step_stamps.py [config] [solver]
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bundleadjustmentmatlab_amd as gpu  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "ladybug"
solver = sys.argv[2] if len(sys.argv) > 2 else "auto"
if cfg.startswith("cfg5x:"):   # the first M cameras of cfg5x (tools/prof_cfg5x_solve.py)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from prof_cfg5x_solve import sub_problem
    M = int(cfg.split(":")[1])
    full = make_config("cfg5x")
    used, pt, cam, x = sub_problem(full, M)
    K, n = full.K[:, :M], len(used)
    a = np.vstack([full.w0[:, :M], full.T0[:, :M]])
    b = np.asfortranarray(full.X0[:3, used])
else:
    sc = make_config(cfg)
    K, n, pt, cam, x = sc.K, sc.n, sc.obs_pt, sc.obs_cam, sc.obs_x
    a = np.vstack([sc.w0, sc.T0])
    b = np.asfortranarray(sc.X0[:3])
L = ctypes.CDLL(os.environ["VLGBA_LIB"])
with gpu.BundleAdjuster(K, pt, cam, x, n, 6, solver=solver) as ba:
    ba.set_params(a, b)
    for _ in range(3):
        ba.step(relinearize=True, update_lm=False)
    ba.sync()
    plan = ba.plan_info()
    nt = plan["tiles"]
    buf = (ctypes.c_ulonglong * (9 * nt))()
    assert L.vlgba_debug_fstamps(buf, nt) == 0
st = np.array(buf, dtype=np.float64).reshape(nt, 9)
print(f"{cfg}: tiles {nt}, arcs {plan['nd_arcs']}, separator tiles {plan['nd_sep_tiles']}")
order = np.argsort(st[:, 0])
t0 = st[order[0], 0]
us = lambda v: (v - t0) / 100.0   # s_memrealtime: 100 MHz
prev_end = None
rows = []
for k in order:
    s = st[k]
    gap = (s[0] - prev_end) / 100.0 if prev_end is not None else 0.0
    rows.append((k, us(s[0]), gap, (s[1] - s[0]) / 100, (s[2] - s[1]) / 100, (s[3] - s[2]) / 100,
                 (s[5] - s[4]) / 100 if s[5] else -1, (s[6] - s[5]) / 100 if s[6] else -1,
                 (s[7] - s[6]) / 100 if s[7] else -1, (s[8] - s[0]) / 100))
    prev_end = max(prev_end or 0, s[8])
print(" col   start    gap | wg0: pre  potrf  post | wg1: pre  potrf  post | span")
for r in rows:
    print("%4d %7.1f %6.1f | %8.1f %6.1f %5.1f | %8.1f %6.1f %5.1f | %5.1f" % r)
R = np.array(rows)
print("mean: gap %.1f, wg0 pre %.1f potrf %.1f post %.1f, wg1 pre %.1f potrf %.1f post %.1f, span %.1f us"
      % tuple(R[1:, 2:].mean(axis=0)))
