"""Where a config-5 growing-BA replay spends its time (GPU box)."""
import sys
import time
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from bundleadjustmentmatlab_amd.incremental import incremental_bundle
from bundleadjustmentmatlab_amd.scene import make_config

sc = make_config("cfg5")
incremental_bundle(sc)
for _ in range(3):
    t0 = time.perf_counter()
    r = incremental_bundle(sc)
    dt = time.perf_counter() - t0
    ss = sum(q["seconds"] for q in r["solves"])
    rs = sum(q["seconds"] for q in r["resections"])
    print(f"replay {1e3*dt:.1f} ms: {len(r['solves'])} solves {1e3*ss:.1f} ms, "
          f"{len(r['resections'])} resections {1e3*rs:.1f} ms, host rest {1e3*(dt-ss-rs):.1f} ms; "
          f"passes {sum(q['passes'] for q in r['solves'])}")
big = max(r["solves"], key=lambda q: q["observations"])
print("largest solve", big["observations"], "obs", big["passes"], "passes", f"{1e3*big['seconds']:.2f} ms")
