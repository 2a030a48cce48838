"""The nested-dissection planner of the envelope solve (ba_chol.hip
nd_choose, through the host-only vlgba_debug_nd_plan: no GPU).  The cameras
split into arcs [bnd[t], bnd[t+1]); a camera co-visible with a camera of an
earlier arc joins the separator.  Checked: no co-visible pair crosses two
arcs outside the separator (what lets the arcs be factored side by side),
the predicted chain matches its definition, and it is shorter than the
natural order's column count."""
import ctypes

import numpy as np
import pytest

from bundleadjustmentmatlab_amd import lib
from bundleadjustmentmatlab_amd.scene import make_config


def _blocks(obs_pt, obs_cam):
    order = np.lexsort((obs_cam, obs_pt))
    pt, cam = obs_pt[order], obs_cam[order]
    cuts = np.r_[0, np.flatnonzero(np.diff(pt)) + 1, len(pt)]
    pairs = set()
    for a, b in zip(cuts[:-1], cuts[1:]):
        cs = np.unique(cam[a:b])
        for x in range(len(cs)):
            for y in range(x + 1):
                pairs.add((int(cs[x]), int(cs[y])))
    return np.array(sorted(pairs), dtype=np.int32).reshape(-1, 2)


def _plan(m, na, jk):
    bnd = (ctypes.c_int * 9)()
    crit = ctypes.c_int(0)
    flat = np.ascontiguousarray(jk.reshape(-1), dtype=np.int32)
    K = lib().vlgba_debug_nd_plan(m, na, flat.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                  len(jk), bnd, ctypes.byref(crit))
    return K, list(bnd)[:K + 1] if K > 0 else [], crit.value


def _check(m, na, jk, K, bnd, crit):
    minK = np.arange(m)
    np.minimum.at(minK, jk[:, 0], jk[:, 1])
    part = np.empty(m, dtype=np.int64)
    for t in range(K):
        part[bnd[t]:bnd[t + 1]] = t
    sep = minK < np.asarray(bnd)[part]
    arc = np.where(sep, -1, part)
    j, k = jk[:, 0], jk[:, 1]
    cross = (arc[j] >= 0) & (arc[k] >= 0) & (arc[j] != arc[k])
    assert not cross.any()
    cnt = [int(((arc == t)).sum()) for t in range(K)]
    ns = -(-na * int(sep.sum()) // 64)
    want = max(-(-na * c // 64) for c in cnt) + ns + (2 if ns else 0)
    assert crit == want
    assert bnd[0] == 0 and bnd[-1] == m and all(a < b for a, b in zip(bnd, bnd[1:]))


@pytest.mark.parametrize("kind,m", [("ladybug", 300), ("ladybug", 120), ("cfg2", 200)])
def test_nd_plan_splits_the_cameras(kind, m):
    sc = make_config(kind, m=m, n=60 * m, seed=11)
    jk = _blocks(sc.obs_pt, sc.obs_cam)
    K, bnd, crit = _plan(m, 6, jk)
    assert 2 <= K <= 8, K
    _check(m, 6, jk, K, bnd, crit)
    natural = -(-6 * m // 64)
    assert crit < natural


def test_nd_plan_disconnected_and_bad_input():
    # two camera groups that never share a point: no separator at all
    jk = np.array([[0, 0], [1, 0], [1, 1], [2, 2], [3, 2], [3, 3]], dtype=np.int32)
    K, bnd, crit = _plan(4, 6, jk)
    assert K >= 2
    _check(4, 6, jk, K, bnd, crit)
    bad = np.array([[0, 1]], dtype=np.int32)      # j < k
    assert _plan(4, 6, bad)[0] == -1
    assert _plan(1, 6, jk[:1])[0] == -1
