"""Where the growing replay waits for its prefetched contexts: per solve kind
and camera-count bucket, the wait, the worker's creation time and the LM loop
of the solve before (the time the creation had to hide behind).
usage: python tools/replay_waits.py [M]"""
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bundleadjustmentmatlab_amd.incremental as inc  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
sc = make_config("cfg5x", m=M) if M != 1000 else make_config("cfg5x")
res = inc.incremental_bundle(sc, devices=[0])
sol = res["solves"]
agg = defaultdict(lambda: np.zeros(5))
for q, s in enumerate(sol):
    b = (s["tag"][:6], min(s["cameras"] // 250, 3))
    prev = sol[q - 1]["lm_seconds"] if q else 0.0
    agg[b] += [1, s["wait_create"], s["create"] or 0.0, s["lm_seconds"], prev]
print("kind    cams      n   wait_s  create_s  lm_s  lm_prev_s")
for (tag, bk), v in sorted(agg.items()):
    print(f"{tag:7s} {250 * bk:4d}+ {int(v[0]):5d} {v[1]:8.3f} {v[2]:9.3f} {v[3]:6.3f} {v[4]:8.3f}")
print("total wait", sum(s["wait_create"] for s in sol), "prefetch", res["prefetch"])
