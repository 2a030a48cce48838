#!/usr/bin/env python3
"""Benchmark: Euclidean LM iterations/s on the BASELINE.json workload.

A "step" is one full Levenberg-Marquardt pass of bundle_euclid.m:120-249 on
the GPU: rotations + linearisation (10 projections / observation, FD
Jacobians) + U/V/W/eA/eB + damping / V*^-1 / Y + Schur complement + dense fp64
MFMA Cholesky solve + back-substitution / update / new cost.  Every timed
step relinearises (the accepted-step cost, the most expensive pass).

Workload at N=1: config 3, 1000 cameras x 500k points x 3M observations
(synthetic, seeded; BASELINE.json configs[2]).  With --gpus N the same scene
is point-sharded over N ranks (strong scaling, RCCL all-reduce of the
reduced camera system).

Run:  python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md; fp64 matrix = vendor spec)
PEAK_HBM_GBS = 8000.0
PEAK_F64_TFLOPS = 78.6


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-points", type=int, default=0,
                    help="points of the CPU-baseline sample (0 = full scene)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    torch.cuda.set_device(local)

    import bundleadjustmentmatlab_amd as pkg
    from bundleadjustmentmatlab_amd.scene import make_config

    t0 = time.time()
    sc = make_config(args.config)
    log(f"[bench] scene {args.config}: m={sc.m} n={sc.n} N={sc.num_obs} ({time.time()-t0:.1f}s)")
    num_a = 6
    a0 = np.zeros((num_a, sc.m), order="F")
    a0[0:3], a0[3:6] = sc.w0, sc.T0
    b0 = np.asfortranarray(sc.X0[:3])

    comm_id = None
    if world > 1:
        from bundleadjustmentmatlab_amd.dist import unique_id_bytes
        buf = [unique_id_bytes() if rank == 0 else None]
        dist.broadcast_object_list(buf, src=0)
        comm_id = buf[0]
    t0 = time.time()
    ba = pkg.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, num_a, device=local,
                            rank=rank, world_size=world, comm_id=comm_id)
    ba.set_params(a0, b0)
    log(f"[bench] setup {time.time()-t0:.1f}s")

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        ba.step(relinearize=True, update_lm=False)
    ba.sync()
    # per-phase device timing (HIP events on the library stream), untimed pass
    ba.set_timing(True)
    phases = []
    for _ in range(max(1, min(3, args.steps))):
        ba.step(relinearize=True, update_lm=False)
        phases.append(ba.phase_ms())
    ba.set_timing(False)
    ph = {k: float(np.median([p[k] for p in phases])) for k in phases[0]}

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    info = None
    for _ in range(args.steps):
        info = ba.step(relinearize=True, update_lm=False)
    ba.sync()
    barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms_step = 1e3 * dt / args.steps
    its = args.steps / dt
    log(f"[bench] {ms_step:.3f} ms/iteration  phases(ms): " +
        " ".join(f"{k}={v:.3f}" for k, v in ph.items()))
    log(f"[bench] last pass: old_sse={info.old_sse:.9g} new_sse={info.new_sse:.9g} "
        f"rho={info.rho:.4g}")

    # ---- roofline of the dominant phase -----------------------------------
    n_s = num_a * sc.m
    dom = max(ph, key=ph.get)
    N = sc.num_obs
    if dom == "cholesky_solve":
        flops = n_s ** 3 / 3.0 + 2.0 * n_s ** 2
        roof = dict(bound="mfma", achieved=flops / (ph[dom] * 1e-3) / 1e12,
                    peak=PEAK_F64_TFLOPS, unit="TFLOP/s")
    else:
        # algorithmic HBM bytes of the phase (DESIGN.md "Roofline")
        per_obs = {"linearize": 16 + 4 + 8 * (2 * num_a + 2) + 8 * 3 * num_a,
                   "camera_reduce": 8 * (2 * num_a + 2) + 4,
                   "damp_y": 8 * 3 * num_a * 2 + 8 * num_a,
                   "schur": 8 * 3 * num_a * 2,
                   "update": 8 * 3 * num_a + 16 + 4,
                   "assemble": 0}.get(dom, 0)
        nbytes = per_obs * N
        roof = dict(bound="hbm", achieved=nbytes / (ph[dom] * 1e-3) / 1e9,
                    peak=PEAK_HBM_GBS, unit="GB/s")
    roof["frac"] = roof["achieved"] / roof["peak"]
    roof["traffic"] = None
    roof["kernel"] = dom

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(sc, a0, b0, num_a, args.cpu_sample_points)

    out = {
        "metric": "LM iterations/sec + observations/sec, 1000-cam/500k-pt synthetic",
        "value": its,
        "unit": "LM iterations/s",
        "observations_per_s": its * N,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded banded scene, SURVEY.md 8.d)",
        "config": {"workload": f"{args.config}: {sc.m} cams x {sc.n} pts x {N} obs, "
                               "fix_calibration (num_a=6), full LM pass per step",
                   "cameras": sc.m, "points": sc.n, "observations": N,
                   "parallelism": f"point-shard x{world}"},
        "phases_ms": ph,
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    ba.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(sc, a0, b0, num_a, sample_points):
    """One LM pass of the oracle restatement (C stages, single thread, + MATLAB
    pinv of S via numpy/OpenBLAS) on the host cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bundle_euclid_ref as ref
    if sample_points and sample_points < sc.n:
        keep = sc.obs_pt < sample_points
        pt, cam, x = sc.obs_pt[keep], sc.obs_cam[keep], sc.obs_x[keep]
        n = sample_points
        b = np.asfortranarray(b0[:, :n])
        desc = f"1 LM pass, first {n} points ({keep.sum()} obs) of the scene"
    else:
        pt, cam, x, n, b = sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, b0
        desc = f"1 full LM pass of the scene ({len(pt)} obs)"
    t0 = time.perf_counter()
    pb = ref.SparseProblem(sc.m, n, pt, cam, x, sc.K)
    L = ref.sp_linearize(pb, a0, b, num_a)
    lam = 1e-3
    Us = L["U"].copy(order="F")
    for k in range(num_a):
        Us[k, k] = (1 + lam) * L["U"][k, k]
    Vs = L["V"].copy(order="F")
    for k in range(3):
        Vs[k, k] = (1 + lam) * L["V"][k, k]
    Vinv = ref.matlab_pinv(Vs)
    Y = ref.sp_y(pb, L["W"], np.asfortranarray(Vinv), num_a)
    S, e_ = ref.sp_schur(pb, Y, L["W"], Us, L["eA"], L["eB"], num_a)
    da = ref.matlab_pinv(S) @ e_
    ref.sp_update(pb, L["W"], da, L["eB"], Vinv, a0, b, num_a)
    dt = time.perf_counter() - t0
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": 1.0 / dt, "unit": "LM iterations/s", "cores": threads, "kind": "port",
            "sample": desc + f"; stages single-threaded C, pinv(S) OpenBLAS "
                             f"({threads} threads); {dt:.2f} s"}


if __name__ == "__main__":
    main()
