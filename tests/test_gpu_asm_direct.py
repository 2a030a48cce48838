"""Direct assembly (ba_dev::asm_direct): on the
camera-aligned cyclic reduction of one rank, k_schur_reduce writes each
co-visible block's lower entries straight into S -- and applies the pinv rule
of an exactly-zero diagonal (unit pivot, zero rhs; bundle_euclid.m:193, App. A
Q8) -- instead of k_assemble_tiles gathering the block sums into the tiles.

Against k_assemble_tiles (VLGBA_ASM_DIRECT=0), from the same start: every
step (da, db), the pass scalars, the whole LM run (error_ trace and the
returned parameters) are bit-identical; with the pass timers on, the direct
context launches no k_assemble.  Scenes: plain banded (the config-2 / 3
model), fix_pivot (the pivot cameras' diagonals are exactly zero: the rule),
fix_motion (every camera's), nomex semantics; and a banded scene whose
five-camera groups are not fully co-visible, where the direct mode must stay
off (the CR writes whole diagonal tiles back, so every lower entry of them
has to be rewritten each pass).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _banded(track=6, m=30, n=3000, seed=17):
    from bundleadjustmentmatlab_amd.scene import banded_scene
    return banded_scene(m=m, n=n, track=track, seed=seed)


CASES = [("plain", {}), ("pivot", dict(pivot="first2")), ("fixmotion", dict(fix_motion=True)),
         ("nomex", dict(semantics="nomex"))]


def _make(gpu, sc, kw, direct):
    kw = dict(kw)
    if kw.get("pivot") == "first2":
        kw["pivot"] = np.arange(sc.m) < 2
    old = os.environ.pop("VLGBA_ASM_DIRECT", None)
    if not direct:
        os.environ["VLGBA_ASM_DIRECT"] = "0"
    try:
        return gpu.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, 6, **kw)
    finally:
        os.environ.pop("VLGBA_ASM_DIRECT", None)
        if old is not None:
            os.environ["VLGBA_ASM_DIRECT"] = old


def _start(sc):
    a = np.zeros((6, sc.m), order="F")
    a[0:3], a[3:6] = sc.w0, sc.T0
    return a, np.asfortranarray(sc.X0[:3])


def _assemble_launches(ba):
    ba.set_timing(True)
    ba.kernel_ms(reset=True)
    ba.step(relinearize=True, update_lm=False)
    k = ba.kernel_ms(reset=True)
    ba.set_timing(False)
    return k.get("k_assemble", (0.0, 0))[1]


@pytest.mark.parametrize("kind,kw", CASES)
def test_direct_assembly_bit_identical(gpu, kind, kw):
    sc = _banded()
    a, b = _start(sc)
    res = {}
    for direct in (True, False):
        ba = _make(gpu, sc, kw, direct)
        plan = ba.plan_info()
        assert plan["cr_levels"] > 0 and plan["cr_rows"] == 30, plan   # camera-aligned CR
        ba.set_params(a, b)
        steps = []
        for _ in range(4):
            i = ba.step(relinearize=False, update_lm=True)
            da, db = ba.last_step()
            steps.append((i.old_sse, i.new_sse, i.dpg, i.accepted, i.lambda_, i.pinv,
                          da.copy(), db.copy()))
        launches = _assemble_launches(ba)
        ba.set_params(a, b)
        err, st = ba.run()
        res[direct] = (steps, err, ba.get_params(), launches, st.pinv_passes)
        ba.close()
    (s1, e1, p1, l1, pv1), (s0, e0, p0, l0, pv0) = res[True], res[False]
    assert l1 == 0 and l0 == 1, (l1, l0)          # no k_assemble launch in the direct mode
    for u, v in zip(s1, s0):
        assert u[:6] == v[:6], (kind, u[:6], v[:6])
        assert np.array_equal(u[6], v[6]) and np.array_equal(u[7], v[7]), kind
    assert np.array_equal(e1, e0), (e1, e0)
    assert all(np.array_equal(x, y) for x, y in zip(p1, p0))
    assert pv1 == pv0


def test_direct_assembly_off_without_full_groups(gpu):
    """Tracks of 3 views: cameras 4 apart in one five-camera group share no
    point, so the group's diagonal tile has lower entries no block covers; the
    context keeps k_assemble_tiles (one launch per pass)."""
    sc = _banded(track=3, m=30, n=3000, seed=5)
    a, b = _start(sc)
    ba = _make(gpu, sc, {}, True)
    plan = ba.plan_info()
    assert plan["cr_levels"] > 0, plan
    ba.set_params(a, b)
    assert _assemble_launches(ba) == 1
    ba.close()
