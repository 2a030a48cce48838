#!/usr/bin/env python3
"""Benchmark: Euclidean LM iterations/s on the BASELINE.json workload.

A "step" is one full Levenberg-Marquardt pass of bundle_euclid.m:120-249 on
the GPU: linearisation (10 projections / observation, FD Jacobians) +
U/V/W/eA/eB + damping / V*^-1 / Y + Schur complement + fp64 MFMA reduced
solve + back-substitution / update / new cost.  Every timed step linearises
once (the accepted-step cost, the most expensive pass): on the default fast
path the update kernel linearises at the new point in the same pass over the
observations (k_update_linearize), so a step is camera
reduction + Schur + solve + that fused update -- exactly the work of an
accepted pass, whose linearisation the next pass starts from.

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
# VALU issue: one fp64 wave64 instruction per 4 cycles per SIMD, 4 SIMDs x 256 CUs,
# 2.4 GHz peak clock (MI355X_MICROARCH.md) -> wave-instructions per second
PEAK_VALU_WINST = 256 * 4 * 2.4e9 / 4


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 100; 5 for the growing replay cfg5, 1 for cfg5x)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed steps first (default 50: ~30 ms of passes, so the GPU's "
                         "clocks have ramped -- a 20-step region right after 3 warmups "
                         "measured 0.66 ms/pass against 0.62 steady, tools/step_times.py; "
                         "2 for cfg5, 0 for cfg5x)")
    ap.add_argument("--clock-ramp", type=float, default=0.25,
                    help="pass/solve modes: seconds of untimed passes before the W warmup "
                         "steps (default 0.25; 0: none), so the timed steps see the clock "
                         "the GPU holds under load (DVFS: the first ~30 ms of passes run "
                         "slower whatever W is; recorded in the line as clock_ramp)")
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="cfg3: skip the config-5 replay carried in the line")
    ap.add_argument("--host-scene", action="store_true",
                    help="generate the banded configs with numpy instead of on the GPU")
    ap.add_argument("--cpu-sample-points", type=int, default=0,
                    help="points of the CPU-baseline sample (0 = full scene)")
    ap.add_argument("--mode", choices=["pass", "solve"], default="pass",
                    help="pass: one LM pass per step (headline); solve: one full LM "
                         "solve to convergence per step (bundle_euclid.m:111-249)")
    ap.add_argument("--time-fallbacks", action="store_true",
                    help="also time one forced pinv pass and one forced re-solve "
                         "(loads rocSOLVER; outside the timed region)")
    ap.add_argument("--spawn-selftest", action="store_true",
                    help="launch only: every rank joins the gloo group and reports (no GPU)")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = {"cfg5": 5, "cfg5x": 1}.get(args.config, 100)
    if args.warmup is None:
        args.warmup = {"cfg5": 2, "cfg5x": 0}.get(args.config, 50)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # not under torch.distributed.run: start one process per GPU ourselves,
        # before this process touches the GPU
        return spawn_ranks(args)
    if args.spawn_selftest:
        return spawn_selftest()
    if args.config in ("cfg5", "cfg5x"):
        return bench_incremental(args)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    import bundleadjustmentmatlab_amd as pkg
    from bundleadjustmentmatlab_amd.dist import rank_collective
    from bundleadjustmentmatlab_amd.scene import make_config
    # one GPU per rank with RCCL; more ranks than GPUs share them over gloo
    ndev = torch.cuda.device_count()   # (counting does not initialise the GPU)
    comm_id, host_ar, local = (rank_collective(dist, rank, world, ndev) if world > 1
                               else (None, None, local))
    torch.cuda.set_device(local)

    t0 = time.time()
    sc = make_config(args.config, gpu=not args.host_scene, **({"device": local} if
                     not args.host_scene and args.config in ("cfg2", "cfg3") else {}))
    log(f"[bench] scene {args.config}: m={sc.m} n={sc.n} N={sc.num_obs} ({time.time()-t0:.1f}s, "
        f"{'numpy' if args.host_scene or args.config not in ('cfg2', 'cfg3') else 'GPU'})")
    num_a = 6
    a0 = np.zeros((num_a, sc.m), order="F")
    a0[0:3], a0[3:6] = sc.w0, sc.T0
    b0 = np.asfortranarray(sc.X0[:3])

    t0 = time.time()
    ba = pkg.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, num_a, device=local,
                            rank=rank, world_size=world, comm_id=comm_id, allreduce=host_ar)
    ba.set_params(a0, b0)
    log(f"[bench] setup {time.time()-t0:.1f}s")

    def barrier():
        if world > 1:
            dist.barrier()

    ba.step(relinearize=True, update_lm=False)   # first touch, outside everything
    ba.sync()
    # clock ramp: untimed passes for --clock-ramp seconds (every one a full
    # pass, like the timed ones), so the measurement is the steady state and
    # not the GPU's DVFS ramp from idle (a 20-step region right after a few
    # warmups ran ~6 % slow: 0.609 vs 0.573 ms, BENCH_r05 against the 100 / 50
    # runs); then the W warmup steps: the first passes after switching the
    # timing mode off carry one-time costs (measured: ~0.8 ms over a 20-step
    # region when the timed steps followed it directly)
    # (a pass count, the same on every rank: each pass holds collectives)
    ramp = {"seconds": 0.0, "passes": 0}

    def clock_ramp():
        if args.clock_ramp <= 0:
            return
        t_r = time.perf_counter()
        for _ in range(3):
            ba.step(relinearize=True, update_lm=False)
        ba.sync()
        t_pass = max((time.perf_counter() - t_r) / 3, 1e-5)
        n_ramp = int(min(args.clock_ramp / t_pass, 20000))
        if world > 1:
            tt = torch.tensor([n_ramp], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            n_ramp = int(tt.item())
        for _ in range(n_ramp):
            ba.step(relinearize=True, update_lm=False)
        ba.sync()
        ramp["seconds"] += time.perf_counter() - t_r
        ramp["passes"] += 3 + n_ramp
    clock_ramp()
    # per-phase and per-kernel device timing (HIP events around every launch on
    # the library stream), in untimed passes after the clock ramp (at the
    # steady-state clock, as the timed steps and rocprofv3's kernel trace see
    # it: taken before the ramp they read the fused kernel ~8 % slow, 278 vs
    # 258 us, profiles/r06/r06b_cfg3_kernel_stats.csv)
    ba.set_timing(True)
    ba.kernel_ms(reset=True)
    phases = []
    n_timed = max(1, min(10, args.steps))
    for _ in range(n_timed):
        ba.step(relinearize=True, update_lm=False)
        phases.append(ba.phase_ms())
    kms = ba.kernel_ms(reset=True)
    ba.set_timing(False)
    ph = {k: float(np.median([p[k] for p in phases])) for k in phases[0]}
    # and the ramp again: the timing passes synchronise after every pass, the
    # GPU idles between them and its clock drops (a 20-step region right
    # after them ran 0.562 against 0.526 ms/pass)
    clock_ramp()
    for _ in range(args.warmup):
        ba.step(relinearize=True, update_lm=False)
    ba.sync()

    if args.mode == "solve":
        return bench_solve(args, ba, sc, a0, b0, world, rank, barrier, torch, dist)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    info = None
    n_pinv = n_retry = 0
    for _ in range(args.steps):
        info = ba.step(relinearize=True, update_lm=False)
        n_pinv += info.pinv
        n_retry += info.spin_retry
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
    plan = ba.plan_info()
    log("[bench] plan: " + " ".join(f"{k}={v}" for k, v in plan.items()))
    roofs = {k: kernel_roofline(k, tot, calls, plan, n_timed) for k, (tot, calls) in
             kms.items()}
    traffic, valu = pmc_traffic(args.config, plan)
    for k, r in roofs.items():
        r["traffic"] = traffic.get(k)
        if k in valu:   # the VALU-issue roof beside the HBM / MFMA one
            w = valu[k] / (r["avg_launch_us"] * 1e-6)
            r["valu_issue"] = {"winst_per_launch": valu[k], "achieved": w,
                               "peak": PEAK_VALU_WINST, "unit": "wave-instr/s",
                               "frac": w / PEAK_VALU_WINST,
                               "source": f"SQ_INSTS_VALU, profiles/pmc_traffic_{args.config}.json"}
    dom = max(kms, key=lambda k: kms[k][0])
    roof = roofs[dom]
    log("[bench] kernels (avg us/launch, launches/pass, roofline frac): " +
        "  ".join(f"{k}={1e3 * t / c:.1f}us x{c / n_timed:.0f} "
                  f"{roofs[k]['frac']:.3f}" for k, (t, c) in
                  sorted(kms.items(), key=lambda kv: -kv[1][0])))

    # the solve's fallbacks, outside the timed region: their count in the timed
    # passes, and one pass of each forced (vlgba_debug_force_status) -- the
    # pinv step (rocSOLVER dsyevd on the dense S; its first call also loads
    # the library) and the re-solve without spins after a hand-off timeout
    fallbacks = {"pinv_passes_timed": n_pinv, "spin_retries_timed": n_retry}
    if args.time_fallbacks:
        for word, key in ((4, "pinv_pass_ms"), (5, "nospin_resolve_pass_ms")):
            ts = []
            for _ in range(2):                      # the first pinv pass loads rocSOLVER
                barrier()
                t1 = time.perf_counter()
                ba.force_status(word, 1)
                fi = ba.step(relinearize=True, update_lm=False)
                ba.sync()
                ts.append(1e3 * (time.perf_counter() - t1))
                assert (fi.pinv if word == 4 else fi.spin_retry) == 1
            fallbacks[key] = ts[-1]
            if word == 4:
                fallbacks["pinv_first_call_ms"] = ts[0]
        log(f"[bench] fallbacks: {fallbacks}")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(sc, a0, b0, num_a, args.cpu_sample_points,
                           dense=args.config in ("cfg1", "cfg2"))

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
        "data": ("synthetic (seeded banded scene, SURVEY.md 8.d, generated on the GPU: "
                 "csrc/ba_scene.hip)" if not args.host_scene and args.config in ("cfg2", "cfg3")
                 else "synthetic (seeded scene, SURVEY.md 8.d, numpy)"),
        "config": {"workload": f"{args.config}: {sc.m} cams x {sc.n} pts x {N} obs, "
                               "fix_calibration (num_a=6), full LM pass per step, one "
                               "linearisation per step" + (
                                   " (fused into the update: k_update_linearize)"
                                   if "k_update_linearize" in kms else ""),
                   "cameras": sc.m, "points": sc.n, "observations": N,
                   "parallelism": f"point-shard x{world}",
                   "collective": "rccl" if comm_id is not None else
                                 ("gloo host all-reduce (ranks share a GPU)" if world > 1 else
                                  None)},
        "phases_ms": ph,
        "clock_ramp": ramp,
        "roofline": roof,
        "whole_pass": whole_pass(plan, ms_step),
        "solve_roofline": {k: roofs[k] for k in SOLVE_FLOPS if k in roofs},
        "solve_fallbacks": fallbacks,
        "cpu_baseline": cpu,
    }
    ba.close()
    if rank == 0 and world == 1 and args.config == "cfg3" and not args.no_other_configs:
        # config 5 (the growing replay) measured in the same driver run: three
        # timed replays after one untimed, its CPU baseline beside it
        try:
            out["other_configs"] = {"cfg5": replay_summary(
                replay_line("cfg5", 3, 1, not args.no_cpu_baseline))}
        except Exception as e:   # noqa: BLE001 -- the cfg3 line stands on its own
            log(f"[bench] cfg5 replay failed: {e!r}")
            out["other_configs"] = {"cfg5": {"error": repr(e)}}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def spawn_ranks(args):
    """bench.py --gpus N outside torch.distributed.run: N child processes of
    this script with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT
    set (the contract torchrun provides); rank 0 prints the JSON line.  The
    parent never initialises the GPU.  Exit status: the first failing rank's."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        sys.exit(bad[0])


def spawn_selftest():
    """Each rank joins the gloo process group; rank 0 prints the gathered ranks."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.tensor([float(dist.get_rank())])
    dist.all_reduce(t)
    world = dist.get_world_size()
    if dist.get_rank() == 0:
        print(json.dumps({"world": world, "rank_sum": float(t.item()),
                          "expected": world * (world - 1) / 2}), flush=True)
    dist.destroy_process_group()


def bench_solve(args, ba, sc, a0, b0, world, rank, barrier, torch, dist):
    """--mode solve: K full LM solves to convergence from the same start
    (set_params + vlgba_run each; the parameter upload is inside the timed
    region).  value = LM passes/s over the whole solves."""
    for _ in range(args.warmup):
        ba.set_params(a0, b0)
        ba.run()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    passes = 0
    err = st = None
    for _ in range(args.steps):
        ba.set_params(a0, b0)
        err, st = ba.run()
        passes += st.iterations
    barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    out = {
        "metric": "LM iterations/sec (full solves to convergence)",
        "value": passes / dt, "unit": "LM iterations/s",
        "observations_per_s": passes / dt * sc.num_obs,
        "solves_per_s": args.steps / dt, "ms_per_solve": 1e3 * dt / args.steps,
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * dt / args.steps, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (seeded, SURVEY.md 8.d)",
        "config": {"workload": f"{args.config}: {sc.m} cams x {sc.n} pts x {sc.num_obs} obs, "
                               "fix_calibration, bundle_euclid.m LM to convergence per step",
                   "cameras": sc.m, "points": sc.n, "observations": sc.num_obs,
                   "parallelism": f"point-shard x{world}"},
        "lm": {"passes_per_solve": st.iterations, "accepted": st.accepted,
               "error_first": float(err[0]), "error_final": float(err[-1])},
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    ba.close()
    if world > 1:
        dist.destroy_process_group()


def bench_incremental(args):
    """--config cfg5 (BASELINE.json configs[4]): replay the growing-BA call
    sequence of incr_reconstruction.m:223-341 (two bundle_euclid solves per
    added camera) on the seeded 50-camera test_incremental scene; --config
    cfg5x: the same on the scaled 1000-camera variant (scene.growing_scene).
    Each solve picks its shard count with dist.choose_shards over the GPUs
    present (1 -> 8 elastic point sharding: rank threads, RCCL between
    distinct GPUs).  A step is one whole replay; value = BA solves/s."""
    print(json.dumps(replay_line(args.config, args.steps, args.warmup,
                                 not args.no_cpu_baseline)), flush=True)


def replay_summary(line):
    """The config-5 replay's headline fields, carried in the default (cfg3)
    bench line so that the driver's run measures config 5 too."""
    keep = ("metric", "value", "unit", "lm_iterations_per_s", "ms_per_step", "steps", "warmup")
    out = {k: line[k] for k in keep}
    out["workload"] = line["config"]["workload"]
    cb = line.get("cpu_baseline")
    if cb:
        out["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample")}
    rf = line.get("roofline") or {}
    out["roofline"] = {k: rf.get(k) for k in ("device_busy_frac", "kernel", "bound", "frac")}
    out["host_device_split_s"] = line["host_device_split_s"]
    out["prefetch"] = line.get("prefetch")
    return out


def replay_line(config, steps, warmup, with_cpu):
    """One growing-replay bench line (dict): `steps` timed replays after
    `warmup` untimed ones."""
    import torch
    from bundleadjustmentmatlab_amd.dist import OBS_PER_SHARD
    from bundleadjustmentmatlab_amd.incremental import incremental_bundle
    from bundleadjustmentmatlab_amd.scene import make_config
    ndev = max(1, torch.cuda.device_count())
    torch.cuda.set_device(0)
    sc = make_config(config)
    devices = list(range(ndev))
    t_start = time.perf_counter()

    def progress(solves):   # a line every 200 solves (long replays)
        if len(solves) % 200 == 0:
            q = solves[-1]
            log(f"[bench] {len(solves)} solves, {time.perf_counter() - t_start:.1f} s: "
                f"{q['cameras']} cams {q['observations']} obs, solve {1e3 * q['seconds']:.1f} ms "
                f"(solve time so far {sum(s['seconds'] for s in solves):.1f} s)")
    for _ in range(warmup):
        incremental_bundle(sc, devices=devices, progress=progress)
    # the CPU baseline's sample: every k-th BA call of the last timed replay
    # (its inputs by reference -- the replay builds them fresh per call -- and
    # the wall time of the GPU call), re-solved on the host afterwards
    import bundleadjustmentmatlab_amd.incremental as inc
    ncalls = 2 * (sc.m - 2)
    k_every = max(1, -(-ncalls // 48))
    sample, spy_on = [], [False]
    orig = inc.bundle_euclid_obs

    def spy(K, T, w, X, pt, cam, ox, *opts, **kw):
        t1 = time.perf_counter()
        out = orig(K, T, w, X, pt, cam, ox, *opts, **kw)
        if spy_on[0] and spy.count % k_every == 0:
            sample.append(dict(K=K, T=T, w=w, X=X, pt=pt, cam=cam, ox=ox, opts=opts,
                               gpu_s=time.perf_counter() - t1, passes=out[-1].iterations))
        spy.count += 1
        return out
    spy.count = 0
    inc.bundle_euclid_obs = spy
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = None
    try:
        for q in range(steps):
            spy_on[0] = q == steps - 1
            spy.count = 0
            res = incremental_bundle(sc, devices=devices, progress=progress)
    finally:
        inc.bundle_euclid_obs = orig
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    sol = res["solves"]
    shards = {}
    for q in sol:
        shards[str(q["shards"])] = shards.get(str(q["shards"]), 0) + 1
    passes = sum(q["passes"] for q in sol)
    obs_passes = sum(q["passes"] * q["observations"] for q in sol)
    out = {
        "metric": "incremental BA solves/sec (test_incremental-style growing BA)",
        "value": steps * len(sol) / dt, "unit": "BA solves/s",
        "lm_iterations_per_s": steps * passes / dt,
        "observations_per_s": steps * obs_passes / dt,
        "n_gpus": 1, "steps": steps, "warmup": warmup,
        "ms_per_step": 1e3 * dt / steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded generate_scene_and_motion restatement, SURVEY.md 8.d)",
        "config": {"workload": f"{config}: {sc.m} cams x {sc.n} pts x {sc.num_obs} obs, "
                               f"{len(sol)} growing solves per replay",
                   "cameras": sc.m, "points": sc.n, "observations": sc.num_obs,
                   "parallelism": f"elastic point shard over {ndev} GPU(s)",
                   "solves_by_shard_count": shards},
        "final": {"cameras": sol[-1]["cameras"], "points": sol[-1]["points"],
                  "observations": sol[-1]["observations"],
                  # (a solve whose every step is rejected returns an empty error_,
                  # as bundle_euclid.m does: the last solve that moved)
                  "error_final": float(next(q["error"][-1] for q in reversed(sol)
                                            if len(q["error"])))},
        "time_split_s": {"solves": sum(q["seconds"] for q in sol),
                         "resections": sum(q["seconds"] for q in res["resections"]),
                         "replay": dt / steps},
        # where a replay's solve time goes: the LM loops (vlgba_run: device passes
        # + the host's per-pass decisions), the wait for the context the worker
        # thread built ahead (its host plan + uploads; create_worker is the
        # worker's own time, overlapped with the previous solve), and the rest
        # of the solve calls on the replay thread (parameter upload / download,
        # packing); host_glue = the replay's numpy stand-ins around the solves
        "host_device_split_s": {
            "lm_loops": sum(q["lm_seconds"] for q in sol),
            "wait_for_context": sum(q["wait_create"] for q in sol),
            "create_worker": sum(q["create"] or 0.0 for q in sol),
            "solve_calls_rest": sum(q["seconds"] - q["lm_seconds"] - q["wait_create"]
                                    for q in sol),
            "host_glue": dt / steps - sum(q["seconds"] for q in sol) -
                         sum(q["seconds"] for q in res["resections"])},
        "elastic": {"obs_per_shard": OBS_PER_SHARD, "max_solve_observations":
                    max(q["observations"] for q in sol),
                    "note": "a solve shards only above 2 x obs_per_shard observations "
                            "(dist.py: the crossover of the sharded kernels' 0.18 us/obs "
                            "against two all-reduces per pass)" +
                            ("; every solve of this scene is below it, so the elastic "
                             "count is 1 throughout" if max(q["observations"] for q in sol)
                             < 2 * OBS_PER_SHARD else "")},
        # the prefetch workers (incremental.py): contexts used as built ahead,
        # rebuilt after a wrong prediction, built on the replay thread, and the
        # replay thread's wait for them by solve kind
        "prefetch": res.get("prefetch"),
        "cpu_baseline": replay_cpu_baseline(sample, k_every, ncalls) if with_cpu else None,
    }
    out["roofline"] = replay_roofline(sc, devices, dt / steps)
    return out


def replay_roofline(sc, devices, replay_s):
    """Where the device time of a growing replay goes: one more replay (after
    the timed ones) with every context timing its kernels (VLGBA_KTIME_ALL=1:
    HIP events around each launch, summed over the destroyed contexts by
    vlgba_kernel_ms(NULL)); device_busy_frac = the summed kernel time over the
    timed replay's wall time; the dominant kernel against its roof -- a solve
    kernel against the fp64 matrix peak with the library's own count of the
    solve's algorithmic flops (vlgba_kernel_flops), the others as busy time
    only (their bytes vary per solve)."""
    import ctypes
    from bundleadjustmentmatlab_amd._lib import NKERNELS, lib
    from bundleadjustmentmatlab_amd.incremental import incremental_bundle
    L = lib()
    ms = np.zeros(NKERNELS)
    calls = (ctypes.c_longlong * NKERNELS)()
    fl = np.zeros(NKERNELS)
    dp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))   # noqa: E731
    L.vlgba_kernel_ms(None, dp(ms), calls, 1)
    os.environ["VLGBA_KTIME_ALL"] = "1"
    try:
        t0 = time.perf_counter()
        incremental_bundle(sc, devices=devices)
        t_timed = time.perf_counter() - t0
    finally:
        del os.environ["VLGBA_KTIME_ALL"]
    L.vlgba_kernel_ms(None, dp(ms), calls, 0)
    L.vlgba_kernel_flops(None, dp(fl))
    names = [L.vlgba_kernel_name(k).decode() for k in range(NKERNELS)]
    busy = float(ms.sum()) * 1e-3
    dom = int(np.argmax(ms))
    per = {names[k]: {"ms": float(ms[k]), "launches": int(calls[k])}
           for k in np.argsort(-ms) if calls[k] > 0}
    out = {"device_busy_s": busy, "replay_s": replay_s,
           "device_busy_frac": busy / replay_s,
           "timing_replay_s": t_timed, "kernel": names[dom], "kernels": per}
    if fl[dom] > 0:
        tfs = fl[dom] / (ms[dom] * 1e-3) / 1e12
        out.update(bound="mfma", achieved=tfs, peak=PEAK_F64_TFLOPS, unit="TFLOP/s",
                   frac=tfs / PEAK_F64_TFLOPS, traffic=None,
                   per_launch=f"{fl[dom] / max(1, calls[dom]):.4g} flop")
    # every solve kernel's rate (the replay's reduced solves are its MFMA work)
    out["solve_kernels"] = {names[k]: {"achieved_tflops": fl[k] / (ms[k] * 1e-3) / 1e12,
                                       "frac": fl[k] / (ms[k] * 1e-3) / 1e12 / PEAK_F64_TFLOPS}
                            for k in range(NKERNELS) if fl[k] > 0 and ms[k] > 0}
    log(f"[bench] replay device time {busy:.2f} s of {replay_s:.2f} s "
        f"({100 * busy / replay_s:.0f} %), dominant {names[dom]} {ms[dom] * 1e-3:.2f} s")
    return out


def replay_cpu_baseline(sample, k_every, ncalls):
    """The growing replay's BA solves on the host (SURVEY.md 8.d ref_sparse_mt;
    the reference's own timing point is test_incremental.m:42-44's tic / toc
    around the growing reconstruction): every k-th call of the timed replay
    re-solved from its own inputs by oracle/cpu_port.py SparsePort.lm -- the
    OpenMP C port of the MEX stages with the reference's MATLAB semantics
    (pinv V*_i, pinv(S) e_ as LAPACK's banded Cholesky), the same LM rule and
    stop -- against the GPU's wall time for the same calls (context wait,
    upload, LM loop, download).  Bounded: the sample is at most 48 calls."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_port
    if not sample:
        return None
    cpu_port.band_cholesky_solve(np.eye(12) * 2.0, np.ones(12))   # first-call costs
    t_cpu, passes, worst = 0.0, 0, 0.0
    # in a fixed shuffled order until ~30 s of CPU work (a spread subset of the
    # sample when the large solves are slow); the GPU side is summed over the
    # same calls
    order = np.random.default_rng(0).permutation(len(sample))
    done = []
    for q in order:
        if t_cpu > 30.0:
            break
        c = sample[q]
        done.append(c)
        assert c["opts"] == ("fix_calibration",), c["opts"]
        t1 = time.perf_counter()
        port = cpu_port.SparsePort(c["K"].shape[1], c["X"].shape[1], c["pt"], c["cam"], c["ox"],
                                   c["K"])
        e, _, _, info = port.lm(np.vstack([c["w"], c["T"]]), np.asfortranarray(c["X"][:3]),
                                vinv="pinv", solve="band", check_pinv=0)
        t_cpu += time.perf_counter() - t1
        passes += info["passes"]
        worst = max(worst, 6 * c["K"].shape[1])
    t_gpu = sum(c["gpu_s"] for c in done)
    info = cpu_port.host_info()
    n = len(done)
    log(f"[bench] cpu replay sample: {n} solves, CPU {t_cpu:.2f} s, GPU {t_gpu:.3f} s "
        f"(x{t_cpu / t_gpu:.1f}) {info}")
    return {"value": n / t_cpu, "unit": "BA solves/s", "cores": info["omp_threads"],
            "kind": "port",
            "sample": f"{n} of every-{k_every}th of the replay's {ncalls} BA calls ({n} solves, "
                      f"{passes} LM passes, reduced systems up to {worst} rows) re-solved "
                      f"from their own inputs: OpenMP C port of the MEX stages "
                      f"({info['omp_threads']} threads), pinv V*_i, LAPACK banded Cholesky "
                      f"of S; port construction included",
            "seconds": t_cpu, "gpu_same_calls_s": t_gpu, "gpu_same_calls_solves_per_s": n / t_gpu,
            "host": info}


# timer name (vlgba_kernel_name) -> device kernel name in the rocprofv3 output
# (tools/kstats.py / pmc_traffic.py key the linearisation by its template flag)
PMC_ALIAS = {"k_linearize": "k_linearize_chunk", "k_camera_reduce": "k_camera_reduce_chunks",
             "k_update_linearize": "k_update_linearize"}


def pmc_traffic(config, plan):
    """HBM bytes per launch of each kernel from the committed PMC passes
    (profiles/pmc_traffic_<config>.json, tools/pmc_traffic.py: FETCH_SIZE x 2 +
    WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md) and VALU wave-
    instructions per launch (SQ_INSTS_VALU), or ({}, {}) if absent.
    Valid for the fast (chunked) single-rank path it was collected on."""
    path = os.path.join(ROOT, "profiles", f"pmc_traffic_{config}.json")
    if plan.get("ordered") or not os.path.exists(path):
        return {}, {}
    with open(path) as f:
        kern = json.load(f)["kernels"]
    out, valu = {}, {}
    for name in list(PMC_ALIAS) + [k for k in kern if k.startswith("k_")]:
        base = PMC_ALIAS.get(name, name)
        if base in kern:
            out[name] = kern[base]["bytes"]
            if "valu_winst" in kern[base]:
                valu[name] = kern[base]["valu_winst"]
    return out, valu


# solve timers (vlgba_kernel_name) -> their flop entry of the plan (vlgba_plan_info)
SOLVE_FLOPS = {"k_factor_step": "solve_flops_factor", "k_cr_factor": "solve_flops_factor",
               "k_syrk": "solve_flops_syrk", "k_backward": "solve_flops_back",
               "k_cr_back": "solve_flops_back"}


def whole_pass(plan, ms_per_pass):
    """SURVEY.md 8.d's algorithmic bytes of one whole LM pass (phases (i) + (iv):
    observations, point / camera gathers and arrays, W written once and read
    twice, the per-point V / V*^-1 / eB arrays) against the pass time and the
    HBM peak -- the whole-iteration fraction beside the dominant kernel's."""
    NA = plan["num_a"]
    N, n, m = plan["obs"], plan["points"], plan["cameras"]
    nbytes = (2 * (N * 24 + N * 24 + n * 24 + m * 8 * NA) + N * 8 * 3 * NA * 3 +
              n * 8 * (9 + 3 + 9) * 2)
    gbs = nbytes / (ms_per_pass * 1e-3) / 1e9
    return {"bytes": nbytes, "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": gbs / PEAK_HBM_GBS,
            "source": "SURVEY.md 8.d algorithmic bytes per iteration / ms_per_step"}


def kernel_roofline(name, tot_ms, calls, plan, n_passes):
    """Algorithmic bytes (HBM-bound kernels) or flops (MFMA / VALU kernels) per
    launch divided by the measured average launch duration.
    Sizes come from the library's own execution plan (vlgba_plan_info), so the
    figures follow the chunk / group / tile counts actually launched."""
    NA = plan["num_a"]
    N, n, m = plan["obs"], plan["points"], plan["cameras"]
    NU = NA * (NA + 1) // 2
    WS = 8 * 3 * NA                         # W_ij, NA x 3 fp64
    avg_s = tot_ms * 1e-3 / calls
    per_pass = calls / n_passes             # launches per LM pass
    nbytes, flops = 0.0, 0.0
    if name == "k_linearize":
        # obs (cam, u, v) + chunk-local ids in; W out; b in; V, eB out; U / eA partials out
        nbytes = (N * (4 + 16 + 2 + WS) + n * (4 + 24 + 72 + 24) +
                  plan["chunk_eslots"] * (8 * (NU + NA) + 4) + plan["chunks"] * 20)
        # 1 + NA + 3 projections per observation (~53 flop each) + 2(NA+3) FD divides
        flops = N * ((1 + NA + 3) * 53 + 2 * (NA + 3) * 2 + 3 * NA * 3)
    elif name == "k_update_linearize":
        # the point update (W rows of the pass read once, da rows, eB / V*^-1 / b
        # in, db / b_new out) + the linearisation at (a_new, b_new) as above
        # (b_new read back; the SSE partials are the pass's new SSE)
        nbytes = (N * (4 + 16 + 2 + WS + WS) + n * (4 + 24 + 72 + 24) +
                  n * (24 + 72 + 24 + 24 + 24) + m * 8 * NA +
                  plan["chunk_eslots"] * (8 * (NU + NA) + 4) + plan["chunks"] * 28)
        flops = N * ((1 + NA + 3) * 53 + 2 * (NA + 3) * 2 + 3 * NA * 3 + 3 * 6 * 2) + n * 30
    elif name == "k_camera_reduce":
        nbytes = plan["chunk_eslots"] * (8 * (NU + NA) + 4) + m * 8 * (NA * NA + NA)
    elif name in ("k_schur_group", "k_schur_mfma"):
        # W, V, eB, metadata in; V*^-1 out; LDS-accumulated block / camera partials out
        # (in a mixed plan both kernels run, each over its own groups: the
        # per-kernel byte split is not tracked, the sum is attributed to each)
        nbytes = (N * WS + n * (72 + 24 + 72) + 4 * plan["blob_words"] +
                  8 * NA * NA * plan["group_slots"] + 8 * NA * plan["group_eslots"])
        # S terms (NA x NA x 3 fma each), Y = W V*^-1, e_ terms
        flops = 2 * (plan["schur_terms"] * NA * NA * 3 + N * NA * 9 + N * NA * 3)
    elif name == "k_schur_reduce":
        nbytes = (8 * NA * NA * plan["group_slots"] + 8 * NA * plan["group_eslots"] +
                  8 * (NA * NA + 1) * plan["blocks"] + 8 * NA * m)
    elif name == "k_point_update":
        nbytes = N * (WS + 4 + 16) + n * (4 + 24 + 72 + 24 + 24 + 24)
    elif name == "k_rotations":
        nbytes = m * 8 * (NA + 45)
    elif name == "k_camera_update":
        nbytes = m * 8 * (3 * NA + 9)
    elif name in SOLVE_FLOPS:
        # the reduced solve: the library's own count of its algorithmic flops
        # per pass (vlgba_plan_info [25..27], ba_chol_setup: tile-dense potrf +
        # trtri, GEMMs, GEMVs), spread over the pass's launches of that timer
        flops = plan[SOLVE_FLOPS[name]]
    else:
        nbytes = 0.0
    nbytes /= per_pass                      # per launch (the timers count every launch)
    flops /= per_pass
    gbs = nbytes / avg_s / 1e9 if nbytes else 0.0
    tfs = flops / avg_s / 1e12 if flops else 0.0
    hbm = dict(bound="hbm", achieved=gbs, peak=PEAK_HBM_GBS, unit="GB/s",
               frac=gbs / PEAK_HBM_GBS, traffic=None, kernel=name,
               per_launch=f"{nbytes:.4g} B", avg_launch_us=avg_s * 1e6)
    fl = dict(bound="mfma", achieved=tfs, peak=PEAK_F64_TFLOPS, unit="TFLOP/s",
              frac=tfs / PEAK_F64_TFLOPS, traffic=None, kernel=name,
              per_launch=f"{flops:.4g} flop", avg_launch_us=avg_s * 1e6)
    if name in SOLVE_FLOPS:
        return fl
    # a kernel with both figures is reported against the roof it is closer to
    return hbm if hbm["frac"] >= fl["frac"] else fl


def cpu_baseline(sc, a0, b0, num_a, sample_points, dense=False):
    """One LM pass of the CPU port on the GPU box's host (oracle/cpu_port.py,
    SURVEY.md 8.d "ref_sparse_mt"): oracle/ba_cpu_mt.c -- the MEX stages'
    per-element arithmetic and reduction orders, OpenMP over the host cores --
    and the reduced solve as LAPACK's banded Cholesky (dpbtrf), the same exact
    band structure the GPU's cyclic reduction uses.  dense=True adds "ref_dense"
    (the reference's dense single-thread MEX loops + SVD pinv; configs 1-2)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_port
    if sample_points and sample_points < sc.n:
        keep = sc.obs_pt < sample_points
        pt, cam, x = sc.obs_pt[keep], sc.obs_cam[keep], sc.obs_x[keep]
        n = sample_points
        desc = f"1 LM pass, first {n} points ({keep.sum()} obs) of the scene"
    else:
        pt, cam, x, n = sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n
        desc = f"1 full LM pass of the scene ({len(pt)} obs)"
    port = cpu_port.SparsePort(sc.m, n, pt, cam, x, sc.K)
    b = np.asarray(b0)[:, :n]
    # warm-up: OpenMP pool, LAPACK / scipy first-call costs
    cpu_port.band_cholesky_solve(np.eye(12) * 2.0, np.ones(12))
    port.one_pass(a0, b)
    r = port.one_pass(a0, b)
    dt = r["seconds"]["total"]
    rd = port.one_pass(a0, b, solve="dense")
    info = cpu_port.host_info()
    log(f"[bench] cpu port: old_sse={r['old_sse']:.9g} new_sse={r['new_sse']:.9g} {dt:.3f} s "
        f"(banded solve {r['seconds']['solve']:.4f} s, bandwidth {r['bandwidth']}; dense "
        f"dpotrf {rd['seconds']['solve']:.3f} s) {info}")
    out = {"value": 1.0 / dt, "unit": "LM iterations/s", "cores": info["omp_threads"],
           "kind": "port",
           "sample": desc + f"; OpenMP C port of the MEX stages ({info['omp_threads']} threads) "
                            f"+ LAPACK banded Cholesky of S (bandwidth {r['bandwidth']}); "
                            f"{dt:.3f} s",
           "phases_s": r["seconds"], "dense_lapack_solve_s": rd["seconds"]["solve"],
           "host": info, "old_sse": r["old_sse"], "new_sse": r["new_sse"]}
    if dense:
        x, vis = sc.dense()
        a = np.asfortranarray(a0)
        t, o, nw = cpu_port.dense_pass(sc.K, a, np.asfortranarray(b0), np.asfortranarray(x[0:2]),
                                       vis.astype(np.float64))
        out["ref_dense"] = {"value": 1.0 / t, "unit": "LM iterations/s", "cores": 1,
                            "sample": "1 LM pass of the reference's dense n x m MEX loops "
                                      "(oracle_mex1/2/3) + SVD pinv, one thread",
                            "seconds": t, "old_sse": o, "new_sse": nw}
        log(f"[bench] ref_dense: {t:.3f} s/pass")
    return out


if __name__ == "__main__":
    main()
