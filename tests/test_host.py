"""Host-side logic (no GPU): option parsing, packing, scenes, shard rule."""
import numpy as np
import pytest

from bundleadjustmentmatlab_amd.bundle import pack_a, parse_options, unpack
from bundleadjustmentmatlab_amd.dist import shard_points
from bundleadjustmentmatlab_amd.scene import make_config


def test_parse_options_defaults_and_names():
    m, n = 3, 4
    x = np.zeros((3, n, m))
    x[0, 1, 2] = 5.0
    x[1, 3, 0] = -1.0
    o = parse_options(m, n, [], x=x)
    assert o["num_variableK"] == 4 and not o["fix_structure"] and not o["verbose"]
    vis = o["visible"]                      # bundle_euclid.m:50 default
    assert vis.dtype == np.float64 and vis.sum() == 2 and vis[1, 2] == 1 and vis[3, 0] == 1
    pv = np.array([True, False, True])
    o = parse_options(m, n, ["FIX_CALIBRATION", "fix_structure", "fix_pivot", pv, "verbose",
                             "unknown_option", "visibility", np.ones((n, m)) * 2], x=x)
    assert o["num_variableK"] == 0 and o["fix_structure"] and o["fix_pivot"] and o["verbose"]
    assert np.array_equal(o["pivot"], pv)
    assert o["visible"].sum() == 2 * n * m          # num_vis sums values (App. A Q10)
    assert parse_options(m, n, ["fix_principal"], x=x)["num_variableK"] == 1


def test_pivot_mask_matlab_indexing():
    """'fix_pivot' as bundle_euclid.m:150-153 indexes with it: a logical mask
    of any length (none true past m) or 1-based camera numbers."""
    from bundleadjustmentmatlab_amd.bundle import pivot_mask
    m = 5
    assert pivot_mask(np.array([True, False, True]), m).tolist() == [1, 0, 1, 0, 0]
    assert pivot_mask(np.array([True, False, False, False, False, False]), m).tolist() == \
        [1, 0, 0, 0, 0]
    assert pivot_mask(1, m).tolist() == [1, 0, 0, 0, 0]
    assert pivot_mask([1, 3, 3], m).tolist() == [1, 0, 1, 0, 0]
    assert pivot_mask(np.array([[2.0], [5.0]]), m).tolist() == [0, 1, 0, 0, 1]
    assert not pivot_mask(np.zeros(0), m).any()
    for bad in (0, 6, 1.5, [-1], np.array([False] * 5 + [True])):
        with pytest.raises(ValueError):
            pivot_mask(bad, m)
    o = parse_options(m, 2, ["fix_pivot", [2, 4]])
    assert o["fix_pivot"] and o["pivot"].tolist() == [0, 1, 0, 1, 0]


def test_oracle_pivot_matches_host(oracle):
    from bundleadjustmentmatlab_amd.bundle import pivot_mask
    for pv in ([1, 3], np.array([True, False]), 2, np.array([1.0, 1.0, 4.0])):
        assert np.array_equal(oracle._matlab_index_mask(pv, 4), pivot_mask(pv, 4))


@pytest.mark.parametrize("nvk", [0, 1, 4])
def test_pack_unpack_roundtrip(nvk):
    rng = np.random.default_rng(0)
    m, n = 4, 5
    K = rng.normal(size=(4, m))
    T, w = rng.normal(size=(3, m)), rng.normal(size=(3, m))
    Xe = rng.normal(size=(4, n))
    a = pack_a(K, T, w, nvk)
    assert a.shape == (6 + nvk, m)
    K_, T_, w_, Xe_ = unpack(K, a, Xe[:3], Xe[3:4], nvk)
    assert np.array_equal(T_, T) and np.array_equal(w_, w)
    assert np.array_equal(Xe_, Xe)                  # Xe_(4,:) = input Xe(4,:) (Q5)
    if nvk == 4:
        assert np.array_equal(K_, K)
    elif nvk == 1:
        assert np.array_equal(K_[0], K[0]) and np.array_equal(K_[1], K[0])
    else:
        assert np.array_equal(K_, K)


@pytest.mark.parametrize("name", ["cfg1", "cfg2"])
def test_scene_properties(name):
    sc = make_config(name)
    # point-major, cameras ascending inside a point, no duplicates
    key = sc.obs_pt.astype(np.int64) * sc.m + sc.obs_cam
    assert np.all(np.diff(key) > 0)
    assert sc.obs_pt.min() >= 0 and sc.obs_pt.max() < sc.n
    if name == "cfg2":
        assert (sc.m, sc.n, sc.num_obs) == (50, 10_000, 60_000)
        assert np.all(np.bincount(sc.obs_pt) == 6)
    # seeded: identical on regeneration
    sc2 = make_config(name)
    assert np.array_equal(sc.obs_x, sc2.obs_x) and np.array_equal(sc.w0, sc2.w0)
    x, vis = sc.dense()
    assert vis.sum() == sc.num_obs and x.shape == (3, sc.n, sc.m)


def test_cfg1_first_camera_has_zero_rotation():
    sc = make_config("cfg1")
    assert np.all(sc.w0[:, 0] == 0.0)       # the test_mview path (App. A Q2)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_points_cover_and_balance(world):
    sc = make_config("cfg2")
    ptr = np.concatenate([[0], np.cumsum(np.bincount(sc.obs_pt, minlength=sc.n))])
    ranges = [shard_points(ptr, world, r) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == sc.n
    for (a0, a1), (b0, b1) in zip(ranges, ranges[1:]):
        assert a1 == b0
    obs = [ptr[p1] - ptr[p0] for p0, p1 in ranges]
    assert max(obs) - min(obs) <= 6 * 2 + 1
