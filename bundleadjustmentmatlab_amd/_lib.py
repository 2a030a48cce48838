"""ctypes binding of libvlgba.so (include/vlgba.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make -C bundleadjustmentmatlab_amd/csrc``).  There is no fallback: if the
library is missing or cannot be loaded, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# VLGBA_LIB: an alternative build of the same library (A/B timing of a kernel
# variant, tools/ab_build.sh); the package's own build otherwise
LIB_PATH = os.environ.get("VLGBA_LIB") or os.path.join(_HERE, "libvlgba.so")

ABI_VERSION = 5   # VLGBA_ABI_VERSION: the struct layouts below

c_int, c_double, c_ll = ctypes.c_int, ctypes.c_double, ctypes.c_longlong
c_dp = ctypes.POINTER(ctypes.c_double)
c_ip = ctypes.POINTER(ctypes.c_int)
c_up = ctypes.POINTER(ctypes.c_ubyte)


class VlgbaProblem(ctypes.Structure):
    _fields_ = [("m", c_int), ("n", c_int), ("num_a", c_int), ("num_obs", c_ll),
                ("obs_pt", c_ip), ("obs_cam", c_ip), ("obs_x", c_dp), ("K", c_dp),
                ("num_vis", c_double), ("model", c_int)]


MODEL_EUCLIDEAN, MODEL_PROJECTIVE = 0, 1   # VLGBA_MODEL_*


class VlgbaOptions(ctypes.Structure):
    _fields_ = [("fix_structure", c_int), ("fix_motion", c_int), ("pivot", c_up),
                ("verbose", c_int), ("max_iter", c_int), ("max_iter2", c_int),
                ("lambda0", c_double), ("device", c_int), ("rank", c_int),
                ("world_size", c_int), ("comm_id", ctypes.c_void_p), ("dense_solve", c_int),
                ("ordered", c_int), ("allreduce", ctypes.c_void_p),
                ("allreduce_user", ctypes.c_void_p), ("schur_kernel", c_int),
                ("semantics", c_int), ("stop_rel", c_double),
                ("on_pass", ctypes.c_void_p), ("on_pass_user", ctypes.c_void_p)]


NKERNELS = 18   # VLGBA_NKERNELS

# int (*allreduce)(double *buf, long long count, void *user)
ALLREDUCE_FN = ctypes.CFUNCTYPE(c_int, c_dp, c_ll, ctypes.c_void_p)


class VlgbaResectProblem(ctypes.Structure):
    _fields_ = [("nprob", c_int), ("num_a", c_int), ("obs_ptr", ctypes.POINTER(c_ll)),
                ("X", c_dp), ("x", c_dp), ("K", c_dp)]


class VlgbaStats(ctypes.Structure):
    _fields_ = [("iterations", c_int), ("accepted", c_int), ("num_error", c_int),
                ("lambda_", c_double), ("seconds", c_double), ("pinv_passes", c_int),
                ("spin_retries", c_int), ("nd_retries", c_int)]


class VlgbaStepInfo(ctypes.Structure):
    _fields_ = [("old_sse", c_double), ("new_sse", c_double), ("dpg", c_double),
                ("rho", c_double), ("lambda_", c_double), ("accepted", c_int),
                ("chol_failed", c_int), ("pinv", c_int), ("spin_retry", c_int),
                ("nd_retry", c_int)]


class VlgbaSceneSpec(ctypes.Structure):
    _fields_ = [("m", c_int), ("n", c_int), ("track", c_int), ("depth_lo", c_double),
                ("depth_hi", c_double), ("noise", c_double), ("seed", ctypes.c_ulonglong),
                ("keep_first_rotation", c_int), ("width", c_double), ("height", c_double)]


class VlgbaSceneOut(ctypes.Structure):
    _fields_ = [("K", c_dp), ("w", c_dp), ("T", c_dp), ("X", c_dp), ("w0", c_dp), ("T0", c_dp),
                ("X0", c_dp), ("obs_pt", c_ip), ("obs_cam", c_ip), ("obs_x", c_dp),
                ("num_obs_cap", c_ll), ("num_obs", c_ll), ("behind", c_ll)]


# vlgba_options.on_pass(pass, iter, const vlgba_step_info *, user)
ON_PASS_FN = ctypes.CFUNCTYPE(None, c_int, c_int, ctypes.POINTER(VlgbaStepInfo), ctypes.c_void_p)


# name -> (restype, argtypes); must match include/vlgba.h exactly
SIGNATURES = {
    "vlgba_solve": (c_int, [ctypes.POINTER(VlgbaProblem), ctypes.POINTER(VlgbaOptions), c_dp,
                            c_dp, c_dp, c_int, ctypes.POINTER(VlgbaStats)]),
    "vlgba_create": (c_int, [ctypes.POINTER(VlgbaProblem), ctypes.POINTER(VlgbaOptions),
                             ctypes.POINTER(ctypes.c_void_p)]),
    "vlgba_set_params": (c_int, [ctypes.c_void_p, c_dp, c_dp]),
    "vlgba_get_params": (c_int, [ctypes.c_void_p, c_dp, c_dp]),
    "vlgba_step": (c_int, [ctypes.c_void_p, c_int, c_int, ctypes.POINTER(VlgbaStepInfo)]),
    "vlgba_run": (c_int, [ctypes.c_void_p, c_dp, c_int, ctypes.POINTER(VlgbaStats)]),
    "vlgba_run_passes": (c_int, [ctypes.c_void_p, c_int, ctypes.POINTER(VlgbaStepInfo)]),
    "vlgba_get_step": (c_int, [ctypes.c_void_p, c_dp, c_dp]),
    "vlgba_get_reduced_system": (c_int, [ctypes.c_void_p, c_ip, c_dp, c_dp]),
    "vlgba_get_linearization": (c_int, [ctypes.c_void_p, c_dp, c_dp, c_dp, c_dp, c_dp]),
    "vlgba_sync": (c_int, [ctypes.c_void_p]),
    "vlgba_destroy": (None, [ctypes.c_void_p]),
    "vlgba_set_timing": (c_int, [ctypes.c_void_p, c_int]),
    "vlgba_phase_ms": (c_int, [ctypes.c_void_p, c_dp]),
    "vlgba_kernel_ms": (c_int, [ctypes.c_void_p, c_dp, ctypes.POINTER(c_ll), c_int]),
    "vlgba_kernel_name": (ctypes.c_char_p, [c_int]),
    "vlgba_kernel_flops": (c_int, [ctypes.c_void_p, c_dp]),
    "vlgba_plan_info": (c_int, [ctypes.c_void_p, ctypes.POINTER(c_ll), c_int]),
    "vlgba_mex_bundle_1": (c_int, [c_int, c_int, c_int] + [c_dp] * 14),
    "vlgba_mex_bundle_2": (c_int, [c_int, c_int, c_int] + [c_dp] * 7),
    "vlgba_mex_bundle_3": (c_int, [c_int, c_int, c_int] + [c_dp] * 13),
    "vlgba_mex_bundle_proj_1": (c_int, [c_int, c_int] + [c_dp] * 13),
    "vlgba_mex_bundle_proj_2": (c_int, [c_int, c_int] + [c_dp] * 7),
    "vlgba_mex_bundle_proj_3": (c_int, [c_int, c_int] + [c_dp] * 12),
    "vlgba_resect": (c_int, [ctypes.POINTER(VlgbaResectProblem), ctypes.POINTER(VlgbaOptions),
                             c_dp, c_dp, c_int, c_ip, ctypes.POINTER(VlgbaStats)]),
    "vlgba_scene_banded": (c_int, [ctypes.POINTER(VlgbaSceneSpec), c_int,
                                   ctypes.POINTER(VlgbaSceneOut)]),
    "vlgba_version": (c_int, [ctypes.c_char_p, c_int]),
    "vlgba_abi_check": (c_int, [c_int, c_ll, c_ll, c_ll, c_ll, c_ll]),
    "vlgba_get_unique_id": (c_int, [ctypes.c_void_p]),
    "vlgba_comm_release": (c_int, [ctypes.c_void_p]),
    "vlgba_device_count": (c_int, []),
    "vlgba_debug_sincos": (c_int, [c_dp, c_dp, c_dp, c_ll]),
    "vlgba_debug_pinv_solve": (c_int, [c_int, c_dp, c_dp, c_dp]),
    "vlgba_debug_force_status": (c_int, [ctypes.c_void_p, c_int, c_int]),
    "vlgba_debug_nd_plan": (c_int, [c_int, c_int, c_ip, c_int, c_ip, c_ip]),
}

ERRORS = {-1001: "bad argument",
          -1002: "num_a must be 6, 7 or 10 (Euclidean) or 12 (projective)",
          -1003: "duplicate (point, camera) observation", -1004: "out of host memory",
          -1005: "RCCL communicator failure",
          -1006: "library / header ABI mismatch"}

_lib = None


class VlgbaError(RuntimeError):
    pass


def lib():
    """The loaded libvlgba (raises if the HIP library is not built / loadable)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise VlgbaError(f"{LIB_PATH} not built: run __graft_entry__.build() or "
                             "make -C bundleadjustmentmatlab_amd/csrc")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("VLGBA_LIB") and not hasattr(L, name):
                continue   # an older build under A/B timing (tools/ab_run.sh)
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if hasattr(L, "vlgba_abi_check") or not os.environ.get("VLGBA_LIB"):
            rc = L.vlgba_abi_check(ABI_VERSION, *(ctypes.sizeof(s) for s in (
                VlgbaProblem, VlgbaOptions, VlgbaStats, VlgbaStepInfo, VlgbaResectProblem)))
            if rc != 0:
                raise VlgbaError(f"{LIB_PATH} does not match this binding (ABI {ABI_VERSION}): "
                                 "rebuild it with __graft_entry__.build()")
        _lib = L
    return _lib


def check(rc: int, what: str = "vlgba"):
    if rc != 0:
        msg = ERRORS.get(rc, f"HIP error {-rc}" if -1000 < rc < 0 else f"code {rc}")
        raise VlgbaError(f"{what} failed: {msg} ({rc})")
