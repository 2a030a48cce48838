"""Projective bundle adjustment on the GPU -- drop-in for
toolbox/bundle/bundle_projective.m and its three MEX stages.

``bundle_projective(Pp, Xp, x, 'fix_structure', 'visibility', vis, ...)`` keeps
the reference signature (bundle_projective.m:1-18): Pp is 3 x 4 x m, Xp 4 x n
(homogeneous; Xp(4,:) is ignored on input and copied to the output, :76,227),
x 3 x n x m.  It returns ``(Pp_, Xp_, error_)``.  The whole LM loop
(bundle_projective.m:86-215) runs in libvlgba with the projective camera
model (num_a = 12): the same fused linearisation / Schur / reduced-solve /
update kernels as the Euclidean path, the projection of
mex_bundle_proj_1_XABeUVWeAeB.c:13-32 and the projective LM rule (errors
normalised by num_vis before the comparison, lambda / 10 on accept, * 10 on
reject, :182-207).

``bundle_projective_nomex`` is the drop-in for the pure-MATLAB twin
bundle_projective_nomex.m: identical except that the back substitution uses
all 12 camera parameters (:247-256) instead of the MEX file's first six
(mex_bundle_proj_3_db_new.c:107-121, App. A Q3).

Callers in the reference: toolbox/geometry/multi_view.m:190
(``'fix_structure'``) and mview_reconstruction.m:148.
"""
from __future__ import annotations

import numpy as np

from ._lib import check, lib
from .bundle import BundleAdjuster, _dp, _F

__all__ = ["bundle_projective", "bundle_projective_nomex", "bundle_projective_obs",
           "parse_options", "pack_a", "unpack", "mex_bundle_proj_1_XABeUVWeAeB",
           "mex_bundle_proj_2_Se_", "mex_bundle_proj_3_db_new"]

NUM_A = 12


def parse_options(m, n, varargin, x=None):
    """Name/value options of bundle_projective.m:36-63 ('fix_structure',
    'fix_motion', 'visibility', vis, 'verbose'); unknown names are ignored
    as the reference's switch ignores them."""
    o = dict(fix_structure=False, fix_motion=False, visible=None, verbose=False)
    k = 0
    while k < len(varargin):
        name = str(varargin[k]).lower()
        if name == "fix_structure":
            o["fix_structure"] = True
        elif name == "fix_motion":
            o["fix_motion"] = True
        elif name == "visibility":
            o["visible"] = np.asarray(varargin[k + 1])
            k += 1
        elif name == "verbose":
            o["verbose"] = True
        k += 1
    if o["visible"] is None:
        if x is None:
            raise ValueError("visibility needs x")
        o["visible"] = (x[0] != 0) | (x[1] != 0)                    # :39
    o["visible"] = np.asarray(o["visible"], dtype=np.float64).reshape(n, m)   # :62
    return o


def pack_a(Pp):
    """a(1:12, j) = reshape(Pp(:,:,j), 12, 1) (bundle_projective.m:70-73)."""
    Pp = _F(Pp)
    return _F(Pp.reshape(NUM_A, Pp.shape[2], order="F"))


def unpack(a, b, Xp4):
    """Pp_(:,:,j) = reshape(a(:,j), 3, 4); Xp_ = [b; Xp(4,:)] (:221-227)."""
    m = a.shape[1]
    return _F(a.reshape(3, 4, m, order="F")), np.vstack([b, Xp4])


def bundle_projective_obs(Pp, Xp, obs_pt, obs_cam, obs_x, *varargin, num_vis=0.0, device=0,
                          rank=0, world_size=1, comm_id=None, return_stats=False,
                          semantics="mex", **solver_kw):
    """bundle_projective on a COO observation list (0-based point / camera ids);
    varargin takes 'fix_structure', 'fix_motion', 'verbose' (visibility is the
    list itself)."""
    Pp, Xp = _F(Pp), _F(Xp)
    m, n = Pp.shape[2], Xp.shape[1]
    o = parse_options(m, n, varargin, x=np.zeros((2, n, m)))
    a = pack_a(Pp)
    b = _F(Xp[0:3])                                                 # :76
    with BundleAdjuster(None, obs_pt, obs_cam, obs_x, n, NUM_A, m=m, model="projective",
                        fix_structure=o["fix_structure"], fix_motion=o["fix_motion"],
                        verbose=o["verbose"], num_vis=num_vis, device=device, rank=rank,
                        world_size=world_size, comm_id=comm_id, semantics=semantics,
                        **solver_kw) as ba:
        ba.set_params(a, b)
        err, st = ba.run()
        a, b = ba.get_params()
    out = unpack(a, b, Xp[3:4]) + (err,)
    return out + (st,) if return_stats else out


def bundle_projective(Pp, Xp, x, *varargin, device=0, return_stats=False, semantics="mex",
                      **solver_kw):
    """[Pp_ Xp_ error_] = bundle_projective(Pp, Xp, x, ...) (bundle_projective.m:1)."""
    x, Pp = _F(x), _F(Pp)
    m, n = Pp.shape[2], x.shape[1]
    o = parse_options(m, n, varargin, x=x)
    vis = o["visible"]
    num_vis = float(vis.sum())                                      # :63
    pt, cam = np.nonzero(vis)                                       # point-major
    obs_x = np.stack([x[0, pt, cam], x[1, pt, cam]], axis=1)
    rest = []
    k = 0
    while k < len(varargin):                     # the visibility is the observation list
        if str(varargin[k]).lower() == "visibility":
            k += 2
            continue
        rest.append(varargin[k])
        k += 1
    return bundle_projective_obs(Pp, Xp, pt, cam, obs_x, *rest, num_vis=num_vis, device=device,
                                 return_stats=return_stats, semantics=semantics, **solver_kw)


def bundle_projective_nomex(Pp, Xp, x, *varargin, device=0, return_stats=False, **solver_kw):
    """[Pp_ Xp_ error_] = bundle_projective_nomex(Pp, Xp, x, ...)
    (bundle_projective_nomex.m:1): db from all 12 camera parameters (:247-256)."""
    return bundle_projective(Pp, Xp, x, *varargin, device=device, return_stats=return_stats,
                             semantics="nomex", **solver_kw)


# ---------------------------------------------------------------------------
# MEX stage mirrors (mex_bundle_proj_*.c argument layouts, num_a = 12)
# ---------------------------------------------------------------------------
def mex_bundle_proj_1_XABeUVWeAeB(a, b, X, visible):
    """[X_hat A B e U V W eA eB] = mex_bundle_proj_1_XABeUVWeAeB(a, b, X, visible)."""
    a, b, X, vis = map(_F, (a, b, X, visible))
    m = a.shape[1]
    n = b.shape[1]
    z = lambda *s: np.zeros(s, order="F")
    out = [z(2, n, m), z(2, NUM_A, n, m), z(2, 3, n, m), z(2, n, m), z(NUM_A, NUM_A, m),
           z(3, 3, n), z(NUM_A, 3, n, m), z(NUM_A, m), z(3, n)]
    check(lib().vlgba_mex_bundle_proj_1(m, n, _dp(a), _dp(b), _dp(X), _dp(vis),
                                        *[_dp(q) for q in out]),
          "mex_bundle_proj_1_XABeUVWeAeB")
    return tuple(out)


def mex_bundle_proj_2_Se_(Y, W, U, eA, eB):
    """[S e_] = mex_bundle_proj_2_Se_(Y, W, U, eA, eB)."""
    Y, W, U, eA, eB = map(_F, (Y, W, U, eA, eB))
    m = eA.shape[1]
    n = eB.shape[1]
    S = np.zeros((NUM_A * m, NUM_A * m), order="F")
    e_ = np.zeros((NUM_A * m, 1), order="F")
    check(lib().vlgba_mex_bundle_proj_2(m, n, _dp(Y), _dp(W), _dp(U), _dp(eA), _dp(eB), _dp(S),
                                        _dp(e_)), "mex_bundle_proj_2_Se_")
    return S, e_


def mex_bundle_proj_3_db_new(W, da, eB, V_inv, a, b, X, visible):
    """[db a_new b_new X_hat] = mex_bundle_proj_3_db_new(W, da, eB, V_inv, a, b, X, visible)."""
    W, da, eB, Vinv, a, b, X, vis = map(_F, (W, da, eB, V_inv, a, b, X, visible))
    m = a.shape[1]
    n = b.shape[1]
    db = np.zeros((3, n), order="F")
    a_new = np.zeros((NUM_A, m), order="F")
    b_new = np.zeros((3, n), order="F")
    X_hat = np.zeros((2, n, m), order="F")
    check(lib().vlgba_mex_bundle_proj_3(m, n, _dp(W), _dp(da), _dp(eB), _dp(Vinv), _dp(a),
                                        _dp(b), _dp(X), _dp(vis), _dp(db), _dp(a_new),
                                        _dp(b_new), _dp(X_hat)), "mex_bundle_proj_3_db_new")
    return db, a_new, b_new, X_hat
