"""The host plan built on several threads is the single-threaded plan, bit for
bit (ba_solver.cpp plan_host: chunk lists, long-track slots, term records and
bucket sorts in work-balanced thread ranges).  CPU only: tools/bench_plan.cpp
runs plan_host on a problem file and hashes every plan vector."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    out = tmp_path_factory.mktemp("plan")
    exe = str(out / "bench_plan")
    lib = os.path.join(ROOT, "bundleadjustmentmatlab_amd", "csrc")
    subprocess.run(["make", "-s", "-C", lib, "-j8"], check=True)
    objs = [os.path.join(lib, "build", f) for f in
            ("ba_kernels.hip.o", "ba_chol.hip.o", "ba_resect.hip.o", "ba_scene.hip.o")]
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                    "-ffp-contract=off", "-I", os.path.join(ROOT, "include"), "-x", "hip",
                    os.path.join(ROOT, "tools", "bench_plan.cpp"), "-x", "none", *objs,
                    "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib", "-o", exe],
                   check=True, capture_output=True)
    return exe, out


def _write(path, m, n, pt, cam):
    with open(path, "wb") as f:
        np.array([m, n, len(pt)], np.int32).tofile(f)
        np.asarray(pt, np.int32).tofile(f)
        np.asarray(cam, np.int32).tofile(f)


def _hash(exe, path, threads):
    env = dict(os.environ, VLGBA_HOST_THREADS=str(threads))
    r = subprocess.run([exe, path, "1"], check=True, capture_output=True, text=True, env=env)
    return re.search(r"hash ([0-9a-f]+)", r.stdout).group(1), r.stdout


@pytest.mark.parametrize("name", ["cfg5x_300", "ladybug_small", "banded"])
def test_plan_identical_on_threads(harness, name):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from bundleadjustmentmatlab_amd.scene import make_config
    exe, out = harness
    if name == "cfg5x_300":      # short, per-term and long tracks (up to 76 views), re-detections
        from prof_cfg5x_solve import sub_problem
        sc = make_config("cfg5x")
        used, pt, cam, _ = sub_problem(sc, 300)
        m, n = 300, len(used)
    elif name == "ladybug_small":   # loop closures + long tracks past a chunk (segment chunks)
        sc = make_config("ladybug", m=200, n=20_000, long_frac=0.01, long_len=(130, 180))
        m, n, pt, cam = sc.m, sc.n, sc.obs_pt, sc.obs_cam
    else:
        sc = make_config("cfg2")
        m, n, pt, cam = sc.m, sc.n, sc.obs_pt, sc.obs_cam
    path = str(out / f"{name}.bin")
    _write(path, m, n, pt, cam)
    h1, log1 = _hash(exe, path, 1)
    h8, log8 = _hash(exe, path, 8)
    assert "fast 1" in log1, log1          # the chunked (fast) plan, not the ordered fallback
    assert h1 == h8, (log1, log8)
