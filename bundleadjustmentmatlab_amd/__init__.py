"""bundleadjustmentmatlab_amd -- MI355X-native bundle adjustment.

Drop-in for the Levenberg-Marquardt paths of caomw/BundleAdjustmentMatlab
(VLG toolbox/bundle: bundle_euclid.m + mex_bundle_{1,2,3}*.c, bundle_projective.m
+ mex_bundle_proj_{1,2,3}*.c, the *_nomex.m twins), built on
hand-written gfx950 HIP kernels behind the C ABI in include/vlgba.h
(libvlgba.so, built in-tree).
"""
from .bundle import (BundleAdjuster, bundle_euclid, bundle_euclid_nomex,  # noqa: F401
                     bundle_euclid_obs, bundle_euclid_resect,
                     mex_bundle_1_XABeUVWeAeB, mex_bundle_2_Se_, mex_bundle_3_db_new,
                     parse_options)
from .projective import (bundle_projective, bundle_projective_nomex,  # noqa: F401
                         bundle_projective_obs, mex_bundle_proj_1_XABeUVWeAeB,
                         mex_bundle_proj_2_Se_, mex_bundle_proj_3_db_new)
from ._lib import LIB_PATH, VlgbaError, lib  # noqa: F401

__version__ = "0.1.0"
