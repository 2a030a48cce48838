"""k_schur_long_acc (ba_kernels.hip): the long tracks' (obs, obs) terms of
the co-visible blocks, subtracted after k_schur_reduce has written the blocks'
slot sums -- four lanes per block, each a quarter of S_jk, the Y / W rows
straight from global memory -- against k_schur_reduce streaming the pairs
itself through LDS (VLGBA_LONG_ACC=0).  Each entry takes the same terms in the
same (track) order with the same expression, so every pass's step and the
whole LM trajectory are bit-identical.  (An XCD-range order of
k_schur_reduce's blocks was tried beside it and measured slower: DESIGN.md
sec. 5.)"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _scene():
    from bundleadjustmentmatlab_amd.scene import make_config
    return make_config("ladybug", m=300, n=5000, max_track=30, radius=150.0, seed=29,
                       long_frac=0.01, long_len=(100, 220))


@pytest.mark.parametrize("num_a", [6, 7])
def test_long_acc_bit_identical(gpu, monkeypatch, num_a):
    sc = _scene()

    def run():
        a = np.zeros((num_a, sc.m), order="F")
        a[0:3], a[3:6] = sc.w0, sc.T0
        if num_a == 7:
            a[6] = sc.K[0]
        b = np.asfortranarray(sc.X0[:3])
        with gpu.BundleAdjuster(sc.K, sc.obs_pt, sc.obs_cam, sc.obs_x, sc.n, num_a,
                                stop_rel=1e-9, max_iter=6) as ba:
            ba.set_params(a, b)
            ba.step(relinearize=True, update_lm=False)
            da, db = ba.last_step()
            err, st = ba.run()
            return da.copy(), db.copy(), err.copy(), [x.copy() for x in ba.get_params()], \
                ba.plan_info()
    monkeypatch.setenv("VLGBA_LONG_ACC", "0")
    r0 = run()
    monkeypatch.setenv("VLGBA_LONG_ACC", "1")
    r1 = run()
    assert r1[4]["long_points"] > 10, r1[4]
    for x, y in zip(r0[:3], r1[:3]):
        assert np.array_equal(x, y)
    for x, y in zip(r0[3], r1[3]):
        assert np.array_equal(x, y)
