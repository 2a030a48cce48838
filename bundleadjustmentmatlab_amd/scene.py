"""Seeded synthetic scenes for the Euclidean BA path.

The reference generates scenes with unseeded MATLAB randn/rand
(toolbox/test/generate_scene_and_motion.m:1-122) and perturbs them as in
toolbox/test/demo_bundle_euclid.m:29-31.  Here every config is seeded
(numpy PCG64) so runs are reproducible:

* ``mview_scene``  -- a seeded restatement of generate_scene_and_motion.m:36-117
  (f = 500, c = (250, 250), 500x500 image, random-walk camera motion,
  tracked / re-detected / new features), used for config 1 (m = 10, <= 200
  points, the test_mview.m:19-26 setting) and config 5 (test_incremental).
* ``banded_scene`` -- configs 2-4: every point is seen by ``track`` consecutive
  cameras (start camera uniform), i.e. video-like banded co-visibility; a damped
  random-walk camera path keeps each point in front of all its cameras at any
  sequence length (the reference's undamped walk diverges over 1000 frames).

Both return a :class:`Scene` with ground truth, the observation list sorted
point-major (point ascending, camera ascending: the order of the reference's
column-major n x m loops), and the perturbed initial parameters.
"""
from __future__ import annotations

from dataclasses import dataclass
import numpy as np


def rodrigues(w):
    """Rotation matrices for rotation vectors w (3, k) -> (k, 3, 3), numpy/libm.

    Same formula as vl_rodrigues; used only to synthesise
    scenes, never on the solve path."""
    w = np.asarray(w, dtype=np.float64).reshape(3, -1)
    th = np.sqrt((w * w).sum(0))
    small = th < 1e-6
    ths = np.where(small, 1.0, th)
    x, y, z = w / ths
    s, c = np.sin(th), np.cos(th)
    mc = 1.0 - c
    R = np.empty((w.shape[1], 3, 3))
    R[:, 0, 0] = 1 - mc * (y * y + z * z)
    R[:, 1, 0] = s * z + mc * x * y
    R[:, 2, 0] = -s * y + mc * x * z
    R[:, 0, 1] = -s * z + mc * x * y
    R[:, 1, 1] = 1 - mc * (z * z + x * x)
    R[:, 2, 1] = s * x + mc * y * z
    R[:, 0, 2] = s * y + mc * x * z
    R[:, 1, 2] = -s * x + mc * y * z
    R[:, 2, 2] = 1 - mc * (x * x + y * y)
    R[small] = np.eye(3)
    return R


def project(K, w, T, X, cam, pt):
    """Pinhole projection of points X[:, pt] in cameras cam -> (k, 2) and depth."""
    R = rodrigues(w)
    Xc = np.einsum("kij,jk->ki", R[cam], X[:3, pt]) + T[:, cam].T
    u = (K[0, cam] * Xc[:, 0] + K[2, cam] * Xc[:, 2]) / Xc[:, 2]
    v = (K[1, cam] * Xc[:, 1] + K[3, cam] * Xc[:, 2]) / Xc[:, 2]
    return np.stack([u, v], 1), Xc[:, 2]


@dataclass
class Scene:
    K: np.ndarray        # (4, m) fx fy cx cy
    T: np.ndarray        # (3, m) ground-truth translation
    w: np.ndarray        # (3, m) ground-truth rotation vector
    X: np.ndarray        # (4, n) ground-truth homogeneous points
    obs_pt: np.ndarray   # (N,) int32, point-major order
    obs_cam: np.ndarray  # (N,) int32
    obs_x: np.ndarray    # (N, 2) measured pixels (noisy)
    T0: np.ndarray       # (3, m) perturbed initial translation
    w0: np.ndarray       # (3, m) perturbed initial rotation
    X0: np.ndarray       # (4, n) perturbed initial points

    @property
    def m(self):
        return self.K.shape[1]

    @property
    def n(self):
        return self.X.shape[1]

    @property
    def num_obs(self):
        return len(self.obs_pt)

    def dense(self):
        """MATLAB-shaped x (3, n, m) and visibility (n, m), bundle_euclid.m:9,50."""
        x = np.zeros((3, self.n, self.m), order="F")
        x[0, self.obs_pt, self.obs_cam] = self.obs_x[:, 0]
        x[1, self.obs_pt, self.obs_cam] = self.obs_x[:, 1]
        x[2, self.obs_pt, self.obs_cam] = 1.0
        vis = np.zeros((self.n, self.m), order="F")
        vis[self.obs_pt, self.obs_cam] = 1.0
        return x, vis


def _perturb(rng, w, T, X, keep_first_rotation):
    """demo_bundle_euclid.m:29-31: w + 1e-3 N, T + 1e-4 N, X(1:3) + 1e-3 N."""
    w0 = w + rng.standard_normal(w.shape) * 1e-3
    if keep_first_rotation:
        w0[:, 0] = w[:, 0]       # camera 1 keeps w = 0 (App. A Q2, test_mview path)
    T0 = T + rng.standard_normal(T.shape) * 1e-4
    X0 = X.copy()
    X0[:3] += rng.standard_normal(X[:3].shape) * 1e-3
    return w0, T0, X0


def _sort_point_major(pt, cam, x):
    order = np.lexsort((cam, pt))
    return (pt[order].astype(np.int32), cam[order].astype(np.int32),
            np.ascontiguousarray(x[order]))


def mview_scene(m=10, min_n=100, max_n=200, depth=100.0, noise=0.5, seed=1,
                keep_first_rotation=True):
    """Seeded restatement of generate_scene_and_motion.m:36-117 (+ noise as
    test_mview.m:45, perturbation as demo_bundle_euclid.m:29-31)."""
    rng = np.random.default_rng(seed)
    width = height = 500.0
    f, cx, cy = width, width / 2, height / 2
    K = np.tile(np.array([[f], [f], [cx], [cy]]), (1, m))
    w = np.zeros((3, m))
    T = np.zeros((3, m))
    vw, vT = np.zeros(3), np.zeros(3)
    for j in range(1, m):
        vw = vw + 1e-2 * rng.standard_normal(3)
        vT = vT + 1e-0 * rng.standard_normal(3)
        w[:, j] = w[:, j - 1] + vw
        T[:, j] = T[:, j - 1] + vT
    R = rodrigues(w)
    Kinv = np.linalg.inv(np.array([[f, 0, cx], [0, f, cy], [0, 0, 1.0]]))
    Xs, xs = [], {}
    vis = {}

    def proj(j, i):
        p = np.array([[f, 0, cx], [0, f, cy], [0, 0, 1.0]]) @ (R[j] @ Xs[i] + T[:, j])
        return p

    for j in range(m):
        tracked = 0
        for i in range(len(Xs)):                   # track previous features (:62-79)
            if j > 0 and vis.get((i, j - 1), 0):
                p = proj(j, i)
                if p[2] > 0.01 * depth and 1 < p[0] / p[2] < width and 1 < p[1] / p[2] < height:
                    tracked += 1
                    xs[(i, j)] = p[:2] / p[2]
                    vis[(i, j)] = 1
        if tracked < min_n:                         # re-detect stored features (:81-97)
            for i in range(len(Xs)):
                if not vis.get((i, j), 0):
                    p = proj(j, i)
                    if (tracked < max_n and p[2] > 0.01 * depth and
                            1 < p[0] / p[2] < width and 1 < p[1] / p[2] < height):
                        tracked += 1
                        xs[(i, j)] = p[:2] / p[2]
                        vis[(i, j)] = 1
        if tracked < min_n:                         # new features (:99-117)
            n_new = max_n - tracked
            xi = rng.random((2, n_new)) * np.array([[width], [height]])
            d = (1 + 0.5 * rng.standard_normal(n_new)) * depth
            for k in range(n_new):
                if d[k] > 0:
                    Xi = R[j].T @ (d[k] * Kinv @ np.array([xi[0, k], xi[1, k], 1.0]) - T[:, j])
                    Xs.append(Xi)
                    i = len(Xs) - 1
                    xs[(i, j)] = xi[:, k].copy()
                    vis[(i, j)] = 1
    n = len(Xs)
    X = np.vstack([np.array(Xs).T, np.ones((1, n))])
    keys = sorted(vis.keys())
    pt = np.array([k[0] for k in keys])
    cam = np.array([k[1] for k in keys])
    x = np.array([xs[k] for k in keys]) + rng.standard_normal((len(keys), 2)) * noise
    pt, cam, x = _sort_point_major(pt, cam, x)
    w0, T0, X0 = _perturb(rng, w, T, X, keep_first_rotation)
    return Scene(K, T, w, X, pt, cam, x, T0, w0, X0)


def growing_scene(m=1000, min_n=300, max_n=500, depth=100.0, noise=0.5, seed=15,
                  keep_first_rotation=True):
    """generate_scene_and_motion.m:36-117's model (mview_scene) with every
    per-frame step vectorised over the points, for long sequences (config 5's
    scaled 1000-camera variant): frame j keeps the points tracked from frame
    j-1 that still project inside the image in front of the camera, re-detects
    stored points in index order while fewer than min_n are seen (up to max_n),
    and creates max_n - tracked new points when still below min_n.  Same model
    and parameters as mview_scene, not the same random stream."""
    rng = np.random.default_rng(seed)
    width = height = 500.0
    f, cx, cy = width, width / 2, height / 2
    Kmat = np.array([[f, 0, cx], [0, f, cy], [0, 0, 1.0]])
    K = np.tile(np.array([[f], [f], [cx], [cy]]), (1, m))
    w = np.zeros((3, m))
    T = np.zeros((3, m))
    vw, vT = np.zeros(3), np.zeros(3)
    for j in range(1, m):
        vw = vw + 1e-2 * rng.standard_normal(3)
        vT = vT + 1e-0 * rng.standard_normal(3)
        w[:, j] = w[:, j - 1] + vw
        T[:, j] = T[:, j - 1] + vT
    R = rodrigues(w)
    Kinv = np.linalg.inv(Kmat)
    cap = 1 << 16
    Xs = np.zeros((3, cap))
    n = 0
    prev = np.zeros(0, dtype=np.int64)                # points seen in frame j-1
    obs_pt, obs_cam, obs_x = [], [], []

    def inside(j, idx):
        P = Kmat @ (R[j] @ Xs[:, idx] + T[:, j:j + 1])
        z = P[2]
        with np.errstate(divide="ignore", invalid="ignore"):
            u, v = P[0] / z, P[1] / z
        ok = (z > 0.01 * depth) & (u > 1) & (u < width) & (v > 1) & (v < height)
        return ok, np.stack([u, v], 1)

    for j in range(m):
        ok, uv = inside(j, prev)
        vis_idx, vis_uv = [prev[ok]], [uv[ok]]
        tracked = int(ok.sum())
        if tracked < min_n and n > 0:                 # re-detect stored points, in order
            seen = np.zeros(n, dtype=bool)
            seen[prev[ok]] = True
            cand = np.nonzero(~seen)[0]
            ok2, uv2 = inside(j, cand)
            take = np.nonzero(ok2)[0][:max_n - tracked]
            vis_idx.append(cand[take])
            vis_uv.append(uv2[take])
            tracked += len(take)
        if tracked < min_n:                           # new points
            n_new = max_n - tracked
            xi = rng.random((2, n_new)) * np.array([[width], [height]])
            d = (1 + 0.5 * rng.standard_normal(n_new)) * depth
            keep = d > 0
            xi, d = xi[:, keep], d[keep]
            ray = (Kinv @ np.vstack([xi, np.ones(xi.shape[1])])) * d
            Xn = R[j].T @ (ray - T[:, j:j + 1])
            k = Xn.shape[1]
            while n + k > Xs.shape[1]:
                Xs = np.hstack([Xs, np.zeros_like(Xs)])
            Xs[:, n:n + k] = Xn
            vis_idx.append(np.arange(n, n + k))
            vis_uv.append(xi.T)
            n += k
        idx = np.concatenate(vis_idx)
        uvs = np.concatenate(vis_uv)
        order = np.argsort(idx, kind="stable")
        prev = idx[order]
        obs_pt.append(prev)
        obs_cam.append(np.full(len(prev), j))
        obs_x.append(uvs[order])
    X = np.vstack([Xs[:, :n], np.ones((1, n))])
    pt = np.concatenate(obs_pt)
    cam = np.concatenate(obs_cam)
    x = np.concatenate(obs_x) + rng.standard_normal((len(pt), 2)) * noise
    pt, cam, x = _sort_point_major(pt, cam, x)
    w0, T0, X0 = _perturb(rng, w, T, X, keep_first_rotation)
    return Scene(K, T, w, X, pt, cam, x, T0, w0, X0)


def banded_scene(m=50, n=10_000, track=6, depth=(80.0, 120.0), noise=0.5, seed=2,
                 keep_first_rotation=False):
    """Configs 2-4: point i is seen by ``track`` consecutive
    cameras starting at a uniform camera; N = track * n observations."""
    rng = np.random.default_rng(seed)
    track = min(track, m)
    width = height = 500.0
    f, cx, cy = width, width / 2, height / 2
    K = np.tile(np.array([[f], [f], [cx], [cy]]), (1, m))
    w = np.zeros((3, m))
    T = np.zeros((3, m))
    vw, vT = np.zeros(3), np.zeros(3)
    for j in range(1, m):                            # damped random walk
        vw = 0.8 * vw + 2e-3 * rng.standard_normal(3)
        vT = 0.8 * vT + 2e-1 * rng.standard_normal(3)
        w[:, j] = w[:, j - 1] + vw
        T[:, j] = T[:, j - 1] + vT
    R = rodrigues(w)
    # points numbered in order of creation (first camera), as
    # generate_scene_and_motion.m:99-116 appends new features frame by frame
    start = np.sort(rng.integers(0, m - track + 1, size=n))
    # place each point in front of its first camera, then check all cameras
    uv = rng.random((n, 2)) * np.array([width, height])
    d = rng.uniform(depth[0], depth[1], size=n)
    ray = np.stack([(uv[:, 0] - cx) / f, (uv[:, 1] - cy) / f, np.ones(n)], 1) * d[:, None]
    Xw = np.einsum("kji,kj->ki", R[start], ray - T[:, start].T)   # R^T (ray - T)
    X = np.vstack([Xw.T, np.ones((1, n))])
    pt = np.repeat(np.arange(n), track)
    cam = (start[:, None] + np.arange(track)[None, :]).reshape(-1)
    x, z = project(K, w, T, X, cam, pt)
    assert np.all(z > 0.01 * depth[0]), "synthetic point behind a camera"
    x = x + rng.standard_normal(x.shape) * noise
    pt, cam, x = _sort_point_major(pt, cam, x)
    w0, T0, X0 = _perturb(rng, w, T, X, keep_first_rotation)
    return Scene(K, T, w, X, pt, cam, x, T0, w0, X0)


def ladybug_scene(m=1000, n=200_000, mean_extra=3.0, max_track=60, loop=0.05,
                  radius=300.0, depth=(80.0, 120.0), noise=0.5, seed=6, long_frac=0.0,
                  long_len=(100, 200)):
    """A BAL-"ladybug"-like scene (the plan cliffs): cameras drive
    (1 + loop) times round a circle of ``radius`` looking at its centre, so
    the last ``loop`` fraction of the frames revisits the first; every point is
    tracked by 2 + Geometric(1 / (1 + mean_extra)) consecutive cameras (capped
    at ``max_track``: long tracks beside short ones), and a point created in
    the first ``loop`` part is seen again, by 1-3 consecutive cameras, one
    revolution later (loop-closure observations: S is no longer banded).
    ``long_frac`` of the points are landmarks near the circle's centre (depth
    ~ radius) tracked by U(long_len) consecutive cameras: tracks longer than a
    Schur chunk holds."""
    rng = np.random.default_rng(seed)
    width = height = 500.0
    f, cx, cy = width, width / 2, height / 2
    K = np.tile(np.array([[f], [f], [cx], [cy]]), (1, m))
    per_rev = int(round(m / (1.0 + loop)))
    ang = 2 * np.pi * np.arange(m) / per_rev
    C = np.stack([radius * np.cos(ang), radius * np.sin(ang), np.zeros(m)])   # centres
    Rm = np.zeros((m, 3, 3))
    for j in range(m):   # rows: camera axes in world coordinates, z towards the centre
        z = -C[:, j] / np.linalg.norm(C[:, j])
        x = np.cross(np.array([0.0, 0.0, 1.0]), z)
        x /= np.linalg.norm(x)
        Rm[j] = np.stack([x, np.cross(z, x), z])
    w = np.zeros((3, m))
    for j in range(m):
        # rotation vector of Rm[j] (log map), small enough for vl_rodrigues' branch
        Rj = Rm[j]
        th = np.arccos(np.clip((np.trace(Rj) - 1) / 2, -1, 1))
        if th < 1e-12:
            continue
        v = np.array([Rj[2, 1] - Rj[1, 2], Rj[0, 2] - Rj[2, 0], Rj[1, 0] - Rj[0, 1]])
        if np.pi - th < 1e-6:   # ~pi: axis from the symmetric part
            ax = np.sqrt(np.maximum((np.diag(Rj) + 1) / 2, 0))
            ax *= np.sign(np.where(v == 0, 1.0, v))
            w[:, j] = th * ax / np.linalg.norm(ax)
        else:
            w[:, j] = th * v / (2 * np.sin(th))
    R = rodrigues(w)
    T = -np.einsum("kij,jk->ik", R, C)                     # T = -R C
    start = np.sort(rng.integers(0, m - 1, size=n))
    L = 2 + rng.geometric(1.0 / (1.0 + mean_extra), size=n) - 1
    L = np.minimum(L, max_track)
    uv = rng.random((n, 2)) * np.array([width, height])
    d = rng.uniform(depth[0], depth[1], size=n)
    if long_frac > 0:
        lm = rng.random(n) < long_frac
        L = np.where(lm, rng.integers(long_len[0], long_len[1] + 1, size=n), L)
        d = np.where(lm, rng.uniform(0.9 * radius, 1.05 * radius, size=n), d)
    L = np.minimum(L, m - start)
    ray = np.stack([(uv[:, 0] - cx) / f, (uv[:, 1] - cy) / f, np.ones(n)], 1) * d[:, None]
    Xw = np.einsum("kji,kj->ki", R[start], ray - T[:, start].T)
    X = np.vstack([Xw.T, np.ones((1, n))])
    pt = np.repeat(np.arange(n), L)
    cam = np.concatenate([np.arange(s0, s0 + k) for s0, k in zip(start, L)])
    # loop closures: one revolution later, 1-3 cameras
    lc = np.nonzero(start + per_rev < m)[0]
    L2 = np.minimum(rng.integers(1, 4, size=lc.size), m - (start[lc] + per_rev))
    pt = np.concatenate([pt, np.repeat(lc, L2)])
    cam = np.concatenate([cam, np.concatenate([np.arange(s0 + per_rev, s0 + per_rev + k)
                                               for s0, k in zip(start[lc], L2)])
                          if lc.size else np.zeros(0, dtype=int)])
    x, z = project(K, w, T, X, cam, pt)
    keep = z > 0.01 * depth[0]
    pt, cam, x = pt[keep], cam[keep], x[keep]
    x = x + rng.standard_normal(x.shape) * noise
    pt, cam, x = _sort_point_major(pt, cam, x)
    w0, T0, X0 = _perturb(rng, w, T, X, False)
    return Scene(K, T, w, X, pt, cam, x, T0, w0, X0)


def projective_from(sc):
    """Projective BA input (bundle_projective.m:1-8) from a Euclidean scene:
    Pp(:,:,j) = K_j [R(w0_j) | T0_j] / f_j at the perturbed start (a 3 x 4 x m
    projective reconstruction of arbitrary per-camera scale, as
    mview_reconstruction.m:148 hands over), Xp = X0 with Xp(4,:) = 1, and the
    scene's observations.  Returns (Pp, Xp)."""
    R = rodrigues(sc.w0)
    m = sc.m
    Pp = np.zeros((3, 4, m), order="F")
    for j in range(m):
        fx, fy, cx, cy = sc.K[:, j]
        Kj = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1.0]])
        Pp[:, :, j] = Kj @ np.hstack([R[j], sc.T0[:, j:j + 1]]) / fx
    Xp = np.asfortranarray(sc.X0.copy())
    return Pp, Xp


CONFIGS = {
    # name: (factory, kwargs)   -- BASELINE.json "configs"
    "cfg1": (mview_scene, dict(m=10, min_n=100, max_n=200, depth=100.0, seed=1)),
    "cfg2": (banded_scene, dict(m=50, n=10_000, track=6, seed=2)),
    "cfg3": (banded_scene, dict(m=1000, n=500_000, track=6, seed=3)),
    "cfg5": (mview_scene, dict(m=50, min_n=100, max_n=200, depth=100.0, seed=5)),
    # config 5's scaled 1000-camera variant
    # (test_incremental.m's 100 .. 200 tracked features per frame, 1000 frames)
    "cfg5x": (growing_scene, dict(m=1000, min_n=100, max_n=200, depth=100.0, seed=15)),
    # not a BASELINE config: irregular tracks + loop closures
    "ladybug": (ladybug_scene, dict(m=1000, n=200_000, seed=6)),
}


def gpu_banded_scene(m=50, n=10_000, track=6, depth=(80.0, 120.0), noise=0.5, seed=2,
                     keep_first_rotation=False, device=0):
    """banded_scene's model generated on the GPU (vlgba_scene_banded,
    csrc/ba_scene.hip: counter-based Philox streams, so the scene is the same
    for a seed on any device).  Same statistics as banded_scene, a different
    random stream (and the first cameras as jittered strata: uniform marginal,
    numbered in camera order)."""
    import ctypes
    from ._lib import VlgbaSceneOut, VlgbaSceneSpec, check, lib
    track = min(track, m)
    N = n * track
    out = dict(K=np.zeros((4, m), order="F"), w=np.zeros((3, m), order="F"),
               T=np.zeros((3, m), order="F"), X=np.zeros((4, n), order="F"),
               w0=np.zeros((3, m), order="F"), T0=np.zeros((3, m), order="F"),
               X0=np.zeros((4, n), order="F"), obs_pt=np.zeros(N, np.int32),
               obs_cam=np.zeros(N, np.int32), obs_x=np.zeros((N, 2)))
    dp = lambda k: out[k].ctypes.data_as(ctypes.POINTER(ctypes.c_double))   # noqa: E731
    ip = lambda k: out[k].ctypes.data_as(ctypes.POINTER(ctypes.c_int))      # noqa: E731
    spec = VlgbaSceneSpec(int(m), int(n), int(track), float(depth[0]), float(depth[1]),
                          float(noise), int(seed), int(keep_first_rotation), 0.0, 0.0)
    so = VlgbaSceneOut(dp("K"), dp("w"), dp("T"), dp("X"), dp("w0"), dp("T0"), dp("X0"),
                       ip("obs_pt"), ip("obs_cam"), dp("obs_x"), N, 0, 0)
    check(lib().vlgba_scene_banded(ctypes.byref(spec), int(device), ctypes.byref(so)),
          "vlgba_scene_banded")
    if so.behind:
        raise RuntimeError(f"synthetic scene: {so.behind} observations behind their camera")
    return Scene(out["K"], out["T"], out["w"], out["X"], out["obs_pt"], out["obs_cam"],
                 out["obs_x"], out["T0"], out["w0"], out["X0"])


def make_config(name, gpu=False, **over):
    """The named config's scene; gpu=True generates the banded configs on the
    GPU (gpu_banded_scene: same model, counter-based random streams)."""
    fn, kw = CONFIGS[name]
    kw = dict(kw, **over)
    if gpu and fn is banded_scene:
        return gpu_banded_scene(**kw)
    return fn(**kw)
