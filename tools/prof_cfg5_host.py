"""Host-side profile of the cfg5 growing replay (GPU box): cProfile of one
replay after a warm-up replay, sorted by own time and by cumulative time."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.getcwd())
from bundleadjustmentmatlab_amd.incremental import incremental_bundle  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402

sc = make_config(sys.argv[1] if len(sys.argv) > 1 else "cfg5")
incremental_bundle(sc)
t0 = time.perf_counter()
incremental_bundle(sc)
print(f"replay {1e3 * (time.perf_counter() - t0):.1f} ms (unprofiled)")
cProfile.run("incremental_bundle(sc)", "/tmp/p5")
st = pstats.Stats("/tmp/p5")
st.sort_stats("tottime").print_stats(25)
st.sort_stats("cumulative").print_stats(40)
