import cProfile, pstats, sys, os
sys.path.insert(0, os.getcwd())
from bundleadjustmentmatlab_amd.incremental import incremental_bundle
from bundleadjustmentmatlab_amd.scene import make_config
sc = make_config("cfg5"); incremental_bundle(sc)
cProfile.run("incremental_bundle(sc)", "/tmp/p5")
pstats.Stats("/tmp/p5").sort_stats("tottime").print_stats(18)
