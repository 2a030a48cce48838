"""k_reduce_assemble (ba_chol.hip, opt-in VLGBA_FUSE_REDUCE=1: measured no
faster than the two launches it replaces): on a single rank without long
tracks the block sums of the reduced system (k_schur_reduce: the damped U_j
term, then the group partials in slot order; the rhs from eA_j and the group
e-partials) are formed inside the envelope-tile assembly launch instead of a
launch of their own.  Same operations in the same order: every pass's step
and LM trajectory is bit-identical to the separate kernels' (the default), on
the cyclic-reduction path (banded), the envelope and the nested-dissection
order (ladybug), with the fix masks and num_a 7 / 10."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _scene(kind):
    from bundleadjustmentmatlab_amd.scene import make_config
    if kind == "ladybug":
        return make_config("ladybug", m=120, n=12000, seed=3)
    if kind == "small":
        return make_config("cfg1", m=12, min_n=150, max_n=250, seed=41)
    return make_config("cfg2", m=40, n=4000, seed=5)


def _start(sc, num_a):
    a = np.zeros((num_a, sc.m), order="F")
    a[0:3], a[3:6] = sc.w0, sc.T0
    if num_a == 7:
        a[6] = sc.K[0]
    elif num_a == 10:
        a[6:10] = sc.K
    return a, np.asfortranarray(sc.X0[:3])


def _run(gpu, sc, num_a, kw):
    a, b = _start(sc, num_a)
    with gpu.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, num_a,
                            stop_rel=1e-9, max_iter=10, **kw) as ba:
        ba.set_params(a, b)
        i1 = ba.step(relinearize=True, update_lm=False)
        da, db = ba.last_step()
        first = (i1.old_sse, i1.new_sse, da.copy(), db.copy())
        err, st = ba.run()
        return first, err.copy(), [x.copy() for x in ba.get_params()], ba.plan_info()


@pytest.mark.parametrize("kind,num_a,kw", [
    ("banded", 6, {}), ("ladybug", 6, {}), ("ladybug", 6, dict(solver="envelope")),
    ("ladybug", 6, dict(solver="nd")), ("small", 7, {}), ("small", 10, {}),
    ("small", 6, dict(fix_structure=True)), ("banded", 6, dict(fix_motion=True))])
def test_fused_reduce_bit_identical(gpu, monkeypatch, kind, num_a, kw):
    sc = _scene(kind)
    f0, e0, p0, _ = _run(gpu, sc, num_a, kw)
    monkeypatch.setenv("VLGBA_FUSE_REDUCE", "1")
    f1, e1, p1, plan = _run(gpu, sc, num_a, kw)
    assert f1[0] == f0[0] and f1[1] == f0[1]
    assert np.array_equal(f1[2], f0[2]) and np.array_equal(f1[3], f0[3])
    assert np.array_equal(e1, e0), (e1, e0)
    for x, y in zip(p1, p0):
        assert np.array_equal(x, y)
