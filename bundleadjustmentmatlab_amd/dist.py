"""Point sharding over ranks (one process per GPU).

The native solver (libvlgba) owns the data path: it splits the points into
contiguous ranges of balanced observation count and all-reduces the reduced
camera system over RCCL.  This module holds the host-side pieces: the RCCL id
exchange and the shard rule, restated in numpy so CPU (gloo) tests can check
it without a GPU.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, lib


def unique_id_bytes() -> bytes:
    """A fresh 128-byte RCCL unique id (call on rank 0, then broadcast)."""
    buf = ctypes.create_string_buffer(128)
    check(lib().vlgba_get_unique_id(buf), "vlgba_get_unique_id")
    return buf.raw


def shard_points(pt_ptr: np.ndarray, world: int, rank: int) -> tuple[int, int]:
    """[p0, p1) of rank: same rule as ctx_create in ba_solver.cpp (lower_bound of
    N*r/world in the point offsets)."""
    n = len(pt_ptr) - 1
    N = int(pt_ptr[-1])
    if world <= 1:
        return 0, n

    def bound(r):
        target = (N * r) // world
        return min(int(np.searchsorted(pt_ptr, target, side="left")), n)

    p0 = 0 if rank == 0 else bound(rank)
    p1 = n if rank == world - 1 else bound(rank + 1)
    return p0, p1


def rank_collective(pg, rank: int, world: int, ndev: int):
    """The collective of one process per rank (torch.distributed group pg
    already initialised): RCCL when every rank has a GPU of its own (world <=
    ndev; rank 0 makes the unique id and the group broadcasts it), else --
    ranks sharing a device, where RCCL refuses a second rank -- the host
    all-reduce over pg (gloo).  Returns (comm_id, allreduce, device): pass
    comm_id / allreduce to BundleAdjuster and run on `device`."""
    if world <= 1:
        return None, None, 0
    if world <= ndev:
        buf = [unique_id_bytes() if rank == 0 else None]
        pg.broadcast_object_list(buf, src=0)
        return buf[0], None, rank
    import torch

    def allreduce(arr):
        pg.all_reduce(torch.from_numpy(arr))
    return None, allreduce, rank % max(1, ndev)


# ---------------------------------------------------------------------------
# Elastic shard count (BASELINE.json config 5: "1 -> 8 GPU elastic point
# shard"): each growing-BA call picks its own number of ranks from its size,
# and the ranks run as threads of one process, one libvlgba context per rank
# on device rank % ndev, their collectives through host memory.
# ---------------------------------------------------------------------------
# The threshold, from measured per-pass times: the sharded
# kernels (linearisation, V*^-1 + Schur, point update) cost ~0.18 us per
# observation per pass (540 us for config 3's 3M observations on one MI355X,
# profiles/r03b_cfg3_kernel_stats.txt); the reduced solve does not shrink with
# the rank count; sharding adds two all-reduces per pass (~30-60 us by RCCL's
# per-call latency over xGMI, ~45 us taken).  Going from 1 to 2 ranks saves
# 0.09 us x N per pass, so it pays only above N ~ 500k observations -- 250k per
# rank -- and every further doubling needs the same per-rank count.  Config
# 5's solves stay below it (the 50-camera replay: < 2k observations; the
# 1000-camera cfg5x: at most 175k), so on these scenes the elastic count is
# always 1: the 1 -> 8 path is exercised only with a lowered threshold
# (tests/test_gpu_incremental.py).
OBS_PER_SHARD = 250_000


def choose_shards(num_obs: int, ndev: int, obs_per_shard: int = OBS_PER_SHARD) -> int:
    """Ranks for one solve: the largest power of two <= ndev that keeps at
    least obs_per_shard observations per rank (1 for the small early solves
    of a growing reconstruction, up to ndev for the large ones)."""
    k = 1
    while k * 2 <= max(1, ndev) and num_obs // (k * 2) >= obs_per_shard:
        k *= 2
    return k


class HostGroup:
    """In-process all-reduce for `world` rank threads: each rank's
    allreduce(buf) blocks until every rank has contributed, then every rank
    receives the element-wise sum in rank order (deterministic)."""

    def __init__(self, world: int):
        import threading
        self.world = world
        self._bar = threading.Barrier(world)
        self._bufs = [None] * world
        self._sum = None

    def allreduce_fn(self, rank: int):
        def ar(buf: np.ndarray):
            self._bufs[rank] = buf.copy()
            if self._bar.wait() == 0:
                s = self._bufs[0].copy()
                for r in range(1, self.world):
                    s += self._bufs[r]
                self._sum = s
            self._bar.wait()
            buf[:] = self._sum
            self._bar.wait()
        return ar


_COMM_IDS: dict = {}   # device tuple -> RCCL unique id (libvlgba caches the communicators)


def release_comms() -> int:
    """Forget every RCCL id run_sharded made: libvlgba destroys the idle
    communicators bootstrapped from them (vlgba_comm_release).  An id is never
    passed again after this, so no later context waits in ncclCommInitRank on
    a spent id.  Returns the number of communicators destroyed."""
    L = lib()
    n = 0
    for key in list(_COMM_IDS):
        n += max(0, int(L.vlgba_comm_release(_COMM_IDS.pop(key))))
    return n


def run_sharded(K, obs_pt, obs_cam, obs_x, n, num_a, a, b, world, *, devices=None, **kw):
    """One LM solve (vlgba_run) over `world` rank threads, rank r on device
    devices[r % len(devices)].  Ranks on distinct GPUs share one RCCL
    communicator (one unique id per device set, ncclCommInitRank per thread
    on its first use; libvlgba keeps the communicators for the next solve);
    ranks that share a GPU (RCCL refuses two ranks on one device) use the
    host-memory all-reduce (HostGroup).  Returns (a, b, error_, stats) of
    rank 0 (every rank holds the same a, b, error_)."""
    import threading
    from .bundle import BundleAdjuster
    if world <= 1:
        with BundleAdjuster(K, obs_pt, obs_cam, obs_x, n, num_a, **kw) as ba:
            ba.set_params(a, b)
            err, st = ba.run()
            a2, b2 = ba.get_params()
        return a2, b2, err, st
    devices = devices or [0]
    devs = [devices[r % len(devices)] for r in range(world)]
    comm = None
    if len(set(devs)) == world:   # one RCCL id per device set: the library keeps its
        comm = _COMM_IDS.get(tuple(devs))   # communicators for the next solve
        if comm is None:
            comm = _COMM_IDS[tuple(devs)] = unique_id_bytes()
    grp = None if comm else HostGroup(world)
    out = [None] * world
    errs = []

    def rank_main(r):
        try:
            with BundleAdjuster(K, obs_pt, obs_cam, obs_x, n, num_a, rank=r, world_size=world,
                                comm_id=comm, allreduce=grp.allreduce_fn(r) if grp else None,
                                device=devs[r], **kw) as ba:
                ba.set_params(a, b)
                err, st = ba.run()
                out[r] = ba.get_params() + (err, st)
        except Exception as e:   # noqa: BLE001 -- re-raised below
            errs.append(e)
            if grp:
                grp._bar.abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    return out[0]
