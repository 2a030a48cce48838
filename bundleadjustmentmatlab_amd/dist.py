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
