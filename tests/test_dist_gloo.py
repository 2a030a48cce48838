"""World-size-2 gloo rehearsal (CPU) of the native point-sharded LM pass.

Mirrors ba_solver.cpp's multi-GPU data path with the oracle as the compute:
each rank linearises its contiguous point range (dist.shard_points) and adds
its own partial U* and eA into its partial reduced system (damping is linear
in U), [S | e_ | old SSE] is all-reduced once, every rank solves the same
system, and the new SSE is all-reduced (two collectives per pass).
The result must match the single-process pass (summation order differs, so
to 1e-12 relative, not bits).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pass(ref, pb_full, lo, hi, a, b, num_a, lam, world, rank):
    """One LM pass on points [lo, hi) with all-reduces (world > 1)."""
    sc_pt = pb_full.obs_pt
    keep = (sc_pt >= lo) & (sc_pt < hi)
    pb = ref.SparseProblem(pb_full.m, hi - lo, sc_pt[keep] - lo, pb_full.obs_cam[keep],
                           pb_full.obs_x[keep], pb_full.K)
    bl = np.asfortranarray(b[:, lo:hi])
    L = ref.sp_linearize(pb, a, bl, num_a)
    old = float(L["e"].reshape(-1) @ L["e"].reshape(-1))
    # every rank adds its own partial U* and eA into its partial reduced system
    # (damping is linear in U); one all-reduce of [S | e_ | old SSE]
    U, eA = L["U"], L["eA"]
    Us = U.copy(order="F")
    for k in range(num_a):
        Us[k, k] = (1 + lam) * U[k, k]
    Vs = L["V"].copy(order="F")
    for k in range(3):
        Vs[k, k] = (1 + lam) * L["V"][k, k]
    Vinv = ref.pinv3_formula(Vs)
    Y = ref.sp_y(pb, L["W"], Vinv, num_a)
    S, e_ = ref.sp_schur(pb, Y, L["W"], Us, eA, L["eB"], num_a)
    if world > 1:
        t = torch.from_numpy(np.concatenate([S.reshape(-1, order="F"), e_.reshape(-1), [old]]))
        dist.all_reduce(t)
        v = t.numpy()
        S = v[: S.size].reshape(S.shape, order="F")
        e_ = v[S.size:S.size + e_.size].reshape(-1, 1)
        old = float(v[-1])
    da = ref.chol_solve_fixed(S, e_)
    _, a_new, b_new, _, sse = ref.sp_update(pb, L["W"], da, L["eB"], Vinv, a, bl, num_a)
    if world > 1:
        t = torch.tensor([sse], dtype=torch.float64)
        dist.all_reduce(t)
        sse = float(t.item())
    return dict(S=S, e_=e_, da=da, old=old, new=sse, a_new=a_new, b_new=b_new)


def _worker(rank, world, port, outdir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import bundle_euclid_ref as ref
    from bundleadjustmentmatlab_amd.dist import shard_points
    from bundleadjustmentmatlab_amd.scene import make_config
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    sc = make_config("cfg2", n=3000, m=30)
    num_a = 6
    a = np.zeros((num_a, sc.m), order="F")
    a[0:3], a[3:6] = sc.w0, sc.T0
    b = np.asfortranarray(sc.X0[:3])
    pb = ref.SparseProblem(sc.m, sc.n, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.K)
    lo, hi = shard_points(pb.pt_ptr, world, rank)
    r = _pass(ref, pb, lo, hi, a, b, num_a, 1e-3, world, rank)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), lo=lo, hi=hi, **r)
    dist.destroy_process_group()


@pytest.mark.slow
def test_two_rank_pass_matches_single(tmp_path, oracle):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    from bundleadjustmentmatlab_amd.scene import make_config
    sc = make_config("cfg2", n=3000, m=30)
    num_a = 6
    a = np.zeros((num_a, sc.m), order="F")
    a[0:3], a[3:6] = sc.w0, sc.T0
    b = np.asfortranarray(sc.X0[:3])
    pb = oracle.SparseProblem(sc.m, sc.n, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.K)
    full = _pass(oracle, pb, 0, sc.n, a, b, num_a, 1e-3, 1, 0)
    r0 = np.load(tmp_path / "rank0.npz")
    r1 = np.load(tmp_path / "rank1.npz")
    assert r0["hi"] == r1["lo"] and r0["lo"] == 0 and r1["hi"] == sc.n
    for r in (r0, r1):
        assert np.allclose(r["S"], full["S"], rtol=0, atol=1e-12 * np.abs(full["S"]).max())
        assert np.allclose(r["e_"], full["e_"], rtol=0, atol=1e-12 * np.abs(full["e_"]).max())
        assert np.allclose(r["da"], full["da"], rtol=0, atol=1e-8 * np.abs(full["da"]).max())
        assert abs(r["old"] - full["old"]) <= 1e-12 * full["old"]
        assert abs(r["new"] - full["new"]) <= 1e-9 * full["new"]
    assert np.array_equal(r0["da"], r1["da"])         # every rank solves the same system
    b_new = np.concatenate([r0["b_new"], r1["b_new"]], axis=1)
    assert np.allclose(b_new, full["b_new"], rtol=0, atol=1e-9)


def test_bench_spawns_ranks():
    """bench.py --gpus 2 outside torch.distributed.run launches two ranks that
    rendezvous over gloo on 127.0.0.1 (no GPU touched: --spawn-selftest)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                          "--spawn-selftest"], capture_output=True, text=True, env=env,
                         timeout=240, check=True)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, out.stdout + out.stderr
    rec = json.loads(line[0])
    assert rec["world"] == 2 and rec["rank_sum"] == rec["expected"] == 1.0
