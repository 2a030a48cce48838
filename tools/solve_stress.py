"""Diagnostic (GPU box): run-to-run determinism of single solves of the
growing replay.  The cfg5x-M replay runs as usual; every solve whose index is
in [lo, hi) is solved R more times from the same inputs on fresh contexts
(optionally while another stream keeps the GPU busy: --load) and each
replica's error_ trace and parameters are compared bit for bit with the
replay's own solve.

usage: python tools/solve_stress.py [M] [lo] [hi] [R] [--load]
"""
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bundleadjustmentmatlab_amd.incremental as inc  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
M = int(args[0]) if len(args) > 0 else 600
lo = int(args[1]) if len(args) > 1 else 900
hi = int(args[2]) if len(args) > 2 else 1100
R = int(args[3]) if len(args) > 3 else 2
load = "--load" in sys.argv

stop = threading.Event()
if load:
    import torch

    def burn():
        s = torch.cuda.Stream()
        a = torch.randn(4096, 4096, device="cuda")
        with torch.cuda.stream(s):
            while not stop.is_set():
                for _ in range(20):
                    a = torch.tanh(a @ a * 1e-4)
                s.synchronize()
    th = threading.Thread(target=burn, daemon=True)
    th.start()

sc = make_config("cfg5x", m=M)
orig = inc.bundle_euclid_obs
count = [0]
bad = []


def same(r1, r2):
    return all(np.array_equal(np.asarray(u), np.asarray(v)) for u, v in zip(r1[:5], r2[:5]))


def spy(*a, **kw):
    r = orig(*a, **kw)
    k = count[0]
    count[0] += 1
    if lo <= k < hi:
        kw2 = {q: v for q, v in kw.items() if q != "adjuster"}
        for rep in range(R):
            r2 = orig(*a, **kw2)
            if not same(r, r2):
                e1, e2 = np.asarray(r[4]), np.asarray(r2[4])
                first = next((i for i in range(min(len(e1), len(e2))) if e1[i] != e2[i]), None)
                bad.append((k, rep))
                print(f"solve {k} replica {rep}: DIFFERS (cameras {a[0].shape[1]}, passes "
                      f"{len(e1)}/{len(e2)}, first differing error_ entry {first}: "
                      f"{e1[first] if first is not None else None!r} vs "
                      f"{e2[first] if first is not None else None!r}; pinv {r[-1].pinv_passes}/"
                      f"{r2[-1].pinv_passes}, spin {r[-1].spin_retries}/{r2[-1].spin_retries})",
                      flush=True)
    if k % 200 == 0:
        print(f"... solve {k}", flush=True)
    return r


inc.bundle_euclid_obs = spy
try:
    inc.incremental_bundle(sc, devices=[0])
finally:
    inc.bundle_euclid_obs = orig
    stop.set()
    if load:
        th.join()
print(f"checked solves [{lo}, {hi}) x {R} replicas{' under load' if load else ''}: "
      f"{len(bad)} differing")
