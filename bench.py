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
    # per-phase and per-kernel device timing (HIP events around every launch on
    # the library stream), in untimed passes
    ba.set_timing(True)
    ba.kernel_ms(reset=True)
    phases = []
    n_timed = max(1, min(3, args.steps))
    for _ in range(n_timed):
        ba.step(relinearize=True, update_lm=False)
        phases.append(ba.phase_ms())
    kms = ba.kernel_ms(reset=True)
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

    N = sc.num_obs
    # ---- roofline of the dominant kernel -----------------------------------
    roofs = {k: kernel_roofline(k, tot, calls, sc, num_a, world) for k, (tot, calls) in
             kms.items()}
    dom = max(kms, key=lambda k: kms[k][0])
    roof = roofs[dom]
    log("[bench] kernels (avg us/launch, launches/pass, roofline frac): " +
        "  ".join(f"{k}={1e3 * t / c:.1f}us x{c / n_timed:.0f} "
                  f"{roofs[k]['frac']:.3f}" for k, (t, c) in
                  sorted(kms.items(), key=lambda kv: -kv[1][0])))

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


def envelope_panels(sc, num_a):
    """Panel tiles per Cholesky step of the tile envelope (ba_chol.hip)."""
    NB = 64
    n_s = num_a * sc.m
    nt = (n_s + NB - 1) // NB
    tfirst = np.arange(nt)
    ptr = np.concatenate([[0], np.cumsum(np.bincount(sc.obs_pt, minlength=sc.n))])
    cnt = np.diff(ptr)
    cmin = np.minimum.reduceat(sc.obs_cam, ptr[:-1][cnt > 0])
    lo = np.repeat(cmin, cnt[cnt > 0])           # smallest camera of each obs' point
    for r in range(num_a):                        # every row of camera j couples with it
        np.minimum.at(tfirst, (num_a * sc.obs_cam + r) // NB, (num_a * lo) // NB)
    T = np.array([(tfirst[k + 1:] <= k).sum() for k in range(nt)])
    return nt, T


def kernel_roofline(name, tot_ms, calls, sc, num_a, world):
    """Algorithmic bytes (HBM-bound kernels) or flops (MFMA kernels) per launch
    divided by the measured average launch time (DESIGN.md 'Roofline')."""
    N = sc.num_obs / world
    n = sc.n / world
    avg_s = tot_ms * 1e-3 / calls
    NB = 64
    if name in ("k_factor_panel", "k_syrk", "k_backward"):
        nt, T = envelope_panels(sc, num_a)
        if name == "k_factor_panel":
            # potrf + trtri of the diagonal tile, T panel GEMMs, fused syrk if T == 1
            fl = sum(2 * NB ** 3 / 3 + t * 2 * NB ** 3 + (NB ** 3 if t == 1 else 0) for t in T)
        elif name == "k_syrk":
            fl = sum(t * (t + 1) / 2 * 2 * NB ** 3 for t in T if t > 1)
        else:
            fl = sum(2 * NB * NB * (1 + t) for t in T)
        passes = calls / max(1, (len(T) if name != "k_syrk" else sum(1 for t in T if t > 1)))
        per = fl / (calls / passes)                 # flops per launch
        achieved = per / avg_s / 1e12
        return dict(bound="mfma", achieved=achieved, peak=PEAK_F64_TFLOPS, unit="TFLOP/s",
                    frac=achieved / PEAK_F64_TFLOPS, traffic=None, kernel=name,
                    per_launch=f"{per:.3g} flop")
    JS = 8 * (2 * num_a + 2)
    WS = 8 * 3 * num_a
    per_obs = {"k_linearize": 16 + 4 + JS + WS,          # obs (x, cam) in; jrec, W out
               "k_camera_reduce": JS + 4,                 # jrec + cam_obs in
               "k_damp_point": 2 * WS + 8 * num_a,        # W in; Y, t out
               "k_schur": 2 * WS,                         # Y, W per term (>= once)
               "k_schur_chunk": WS,                       # W in (once, contiguous)
               "k_point_update": WS + 16 + 4}.get(name, 0)
    per_pt = {"k_linearize": 24 + 72 + 24 + 4,           # b in; V, eB out
              "k_damp_point": 72 + 24 + 72,
              "k_schur_chunk": 72 + 24 + 72,             # V, eB in; V*^-1 out
              "k_point_update": 24 + 72 + 24 + 48 + 4}.get(name, 0)
    # every such kernel runs once per pass: bytes per launch = bytes per pass
    nbytes = per_obs * N + per_pt * n
    achieved = nbytes / avg_s / 1e9 if nbytes else 0.0
    return dict(bound="hbm", achieved=achieved, peak=PEAK_HBM_GBS, unit="GB/s",
                frac=achieved / PEAK_HBM_GBS, traffic=None, kernel=name,
                per_launch=f"{nbytes:.3g} B")


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
