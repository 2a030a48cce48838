#!/bin/bash
# Build tools/build/bench_plan (the CPU harness of the context's host planner,
# tools/bench_plan.cpp) against the library's kernel objects, and write the
# problem files it reads (tools/build/plan_*.bin).
set -e
cd "$(dirname "$0")/.."
make -s -C bundleadjustmentmatlab_amd/csrc -j8
mkdir -p tools/build
O=bundleadjustmentmatlab_amd/csrc/build
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -DBA_PLAN_TIMING -I include \
  -x hip tools/bench_plan.cpp -x none $O/ba_kernels.hip.o $O/ba_chol.hip.o $O/ba_resect.hip.o \
  $O/ba_scene.hip.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o tools/build/bench_plan
python3 - <<'PY'
import sys
import numpy as np
sys.path[:0] = [".", "tools"]
from bundleadjustmentmatlab_amd.scene import make_config
from prof_cfg5x_solve import sub_problem


def write(name, m, n, pt, cam):
    with open(f"tools/build/plan_{name}.bin", "wb") as f:
        np.array([m, n, len(pt)], np.int32).tofile(f)
        np.asarray(pt, np.int32).tofile(f)
        np.asarray(cam, np.int32).tofile(f)


sc = make_config("cfg5x")
for M in (300, 900):
    used, pt, cam, _ = sub_problem(sc, M)
    write(f"cfg5x_{M}", M, len(used), pt, cam)
for name in ("cfg2", "ladybug"):
    s = make_config(name)
    write(name, s.m, s.n, s.obs_pt, s.obs_cam)
s = make_config("cfg3")
write("cfg3", s.m, s.n, s.obs_pt, s.obs_cam)
PY
