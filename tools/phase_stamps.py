#!/usr/bin/env python3
"""Per-phase cycle split of the fast-path kernels (diagnostic build).

Build ``make -C bundleadjustmentmatlab_amd/csrc stamps`` (libvlgba_stamps.so,
-DBA_STAMPS), then run on the GPU box:  python tools/phase_stamps.py [cfg]
Prints, per stamped phase, the s_memtime cycles summed over workgroups and
per chunk (thread 0 of each workgroup stamps at its phase boundaries).
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bundleadjustmentmatlab_amd._lib as L  # noqa: E402

L.LIB_PATH = os.path.join(ROOT, "bundleadjustmentmatlab_amd", "libvlgba_stamps.so")
from bundleadjustmentmatlab_amd import BundleAdjuster  # noqa: E402
from bundleadjustmentmatlab_amd.scene import make_config  # noqa: E402

PHASES = {"k_schur_group": ["prologue", "stage+pinv", "Y", "slots+e", "barrier", "epilogue"],
          "k_schur_mfma": ["prologue", "stage+pinv", "W scatter", "Y", "mfma+e+flush",
                           "final barrier", "epilogue"]}


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
    sc = make_config(cfg)
    lib = L.lib()
    fn = lib.vlgba_debug_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    a = np.zeros((6, sc.m), order="F")
    a[0:3], a[3:6] = sc.w0, sc.T0
    b = np.asfortranarray(sc.X0[:3])
    ba = BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, 6)
    ba.set_params(a, b)
    st = (ctypes.c_ulonglong * 32)()
    ba.step(relinearize=True, update_lm=False)
    ba.sync()
    fn(st, 1)
    reps = 5
    for _ in range(reps):
        ba.step(relinearize=True, update_lm=False)
    ba.sync()
    fn(st, 1)
    v = [st[i] / reps for i in range(32)]
    kern = "k_schur_mfma" if ba.plan_info()["mfma"] else "k_schur_group"
    names = PHASES[kern]
    chunks, wgs = (v[8], v[9]) if kern == "k_schur_mfma" else (v[6], v[7])
    print(f"{kern}: {wgs:.0f} workgroups, {chunks:.0f} chunks per pass")
    tot = sum(v[:len(names)])
    for i, name in enumerate(names):
        print(f"  {name:12s} {v[i] / 1e6:9.2f} Mcycles  {100 * v[i] / max(tot, 1):5.1f}%  "
              f"{v[i] / max(chunks, 1):9.0f} cycles/chunk")
    if kern == "k_schur_mfma" and v[11] > 0:
        # s_memrealtime runs at 100 MHz: calibrates s_memtime and the WG lifetime
        ghz = v[10] / v[11] * 0.1
        life_us = v[11] / wgs / 100.0
        print(f"  s_memtime clock {ghz:.2f} GHz; mean workgroup lifetime {life_us:.1f} us; "
              f"sum of lifetimes {v[11] / 100.0:.0f} us")
    # the linearisation body (k_linearize_chunk, or the fused k_update_linearize:
    # its update phase is stamp 23, between the prologue and the projections)
    lin = [(16, "prologue"), (23, "update (fused)"), (17, "projections"), (18, "W"),
           (19, "V/eB"), (20, "U/eA partials"), (21, "sse reduce")]
    tot = sum(v[i] for i, _ in lin)
    print(f"linearisation body: {v[22]:.0f} workgroups per pass")
    for i, name in lin:
        print(f"  {name:14s} {v[i] / 1e6:9.2f} Mcycles  {100 * v[i] / max(tot, 1):5.1f}%  "
              f"{v[i] / max(v[22], 1):9.0f} cycles/workgroup")
    ba.close()


if __name__ == "__main__":
    main()
