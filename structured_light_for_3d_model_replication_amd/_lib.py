"""ctypes binding of libslgpu.so (include/slgpu.h).

The shared library is built in-tree by ``__graft_entry__.build()``.  There is no
fallback: if the library is missing or has no device, every product entry point
raises instead of silently computing on the CPU.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# SLGPU_LIB selects an alternative build (measurement of build variants only)
LIB_PATH = os.environ.get("SLGPU_LIB") or os.path.join(_HERE, "libslgpu.so")

SL_OK = 0
SL_EINVAL = -1
SL_EINDEX = -2
SL_EHIP = -3
SL_ENOCALIB = -4
SL_ETIMEOUT = -5
SL_ECAPACITY = -6
SL_EIO = -7

SL_MASK_ADAPTIVE = 0
SL_MASK_FIXED = 1
SL_XYZ_F32 = 0
SL_XYZ_F64 = 1
SL_XYZ_F32_FAST = 2

# every symbol include/slgpu.h declares
EXPORTS = ("sl_abi_version", "sl_ctx_create", "sl_ctx_destroy", "sl_ctx_last_error", "sl_ctx_reserve",
           "sl_set_calib", "sl_decode_triangulate", "sl_mask_counts_to", "sl_stack_ready", "sl_stack_next", "sl_call_prepare", "sl_call_run", "sl_call_destroy", "sl_triangulate_maps", "sl_sync",
           "sl_last_thresholds", "sl_last_launch_info", "sl_profile_enable", "sl_profile_read", "sl_time_kernels", "sl_format_ply", "sl_write_ply",
           "sl_write_ply_device", "sl_write_ply_binary", "sl_voxel_downsample", "sl_statistical_outliers", "sl_select_by_index",
           "sl_transform_points", "sl_estimate_normals", "sl_icp_point_to_plane", "sl_radius_search", "sl_compute_fpfh",
           "sl_feature_nn", "sl_ransac_feature_matching", "sl_merge_pool_trim", "sl_calib_products", "sl_gather_unique_id", "sl_gather_init", "sl_gather_counts",
           "sl_gather",
           "sl_decode_triangulate_batch", "sl_last_error")

_vp = ctypes.c_void_p
_i32 = ctypes.c_int
_i64 = ctypes.c_int64
_SIGS = {
    "sl_abi_version": (_i32, []),
    "sl_ctx_create": (_i32, [_i32, ctypes.POINTER(_vp)]),
    "sl_ctx_destroy": (None, [_vp]),
    "sl_ctx_last_error": (ctypes.c_char_p, [_vp]),
    "sl_ctx_reserve": (_i32, [_vp, _i64, _i64]),
    "sl_set_calib": (_i32, [_vp, _i32, _i32, _vp, _vp, _vp, _i32, _vp]),
    "sl_decode_triangulate": (_i32, [_vp, _vp, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _i64, _i32,
                                     _vp, _vp, _vp, _vp, _vp, _i32, _vp, _i64, _vp, _vp]),
    "sl_mask_counts_to": (_i32, [_vp, _vp]),
    "sl_stack_ready": (_i32, [_vp, _vp]),
    "sl_stack_next": (_i32, [_vp, _vp, _i64, _i32]),
    "sl_call_prepare": (_i32, [_vp, _vp, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _i64, _i32,
                               _vp, _vp, _vp, _vp, _vp, _i32, _vp, _i64, _vp, ctypes.POINTER(_vp)]),
    "sl_call_run": (_i32, [_vp, _vp]),
    "sl_call_destroy": (None, [_vp]),
    "sl_triangulate_maps": (_i32, [_vp, _vp, _vp, _vp, _i32, _i32, _i32, _vp, _vp, _i32, _vp, _i64, _vp,
                                   _vp]),
    "sl_sync": (_i32, [_vp, _vp]),
    "sl_last_thresholds": (_i32, [_vp, _i32, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
                                  ctypes.POINTER(_i32), ctypes.POINTER(_i32)]),
    "sl_last_launch_info": (_i32, [_vp, ctypes.POINTER(_i32), ctypes.POINTER(_i64), ctypes.POINTER(_i64)]),
    "sl_profile_enable": (_i32, [_vp, _i32]),
    "sl_profile_read": (_i32, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_i32)]),
    "sl_time_kernels": (_i32, [_vp, _i32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(ctypes.c_double)]),
    "sl_format_ply": (_i32, [_vp, _i32, _vp, _i64, _i32, _vp, _i64, ctypes.POINTER(_i64)]),
    "sl_write_ply": (_i32, [ctypes.c_char_p, _vp, _i32, _vp, _i64, _i32]),
    "sl_write_ply_device": (_i32, [_vp, ctypes.c_char_p, _vp, _i32, _vp, _i64, _vp]),
    "sl_write_ply_binary": (_i32, [ctypes.c_char_p, _vp, _i32, _vp, _i64, _i32]),
    "sl_voxel_downsample": (_i32, [_vp, _vp, _vp, _i64, ctypes.c_double, _vp, _vp, ctypes.POINTER(_i64), _vp]),
    "sl_statistical_outliers": (_i32, [_vp, _vp, _i64, _i32, ctypes.c_double, _vp, _vp, ctypes.POINTER(_i64), _vp]),
    "sl_select_by_index": (_i32, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp]),
    "sl_transform_points": (_i32, [_vp, _vp, _i64, _vp, _vp]),
    "sl_estimate_normals": (_i32, [_vp, _vp, _i64, ctypes.c_double, _i32, _vp, _vp]),
    "sl_icp_point_to_plane": (_i32, [_vp, _vp, _i64, _vp, _vp, _i64, ctypes.c_double, _vp, _i32, ctypes.c_double,
                                      ctypes.c_double, _vp, ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_i32), _vp]),
    "sl_radius_search": (_i32, [_vp, _vp, _i64, ctypes.c_double, _i32, _vp, _vp, _vp, _vp]),
    "sl_compute_fpfh": (_i32, [_vp, _vp, _vp, _i64, ctypes.c_double, _i32, _vp, _vp]),
    "sl_feature_nn": (_i32, [_vp, _vp, _i64, _vp, _i64, _i32, _vp, _vp]),
    "sl_ransac_feature_matching": (_i32, [_vp, _vp, _i64, _vp, _i64, _vp, _vp, _i32, ctypes.c_double,
                                           ctypes.c_double, _i32, ctypes.c_double, ctypes.c_uint64, _vp,
                                           ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(_i32), ctypes.POINTER(_i32), ctypes.POINTER(_i64), _vp]),
    "sl_merge_pool_trim": (_i32, [_i32, ctypes.POINTER(_i64)]),
    "sl_gather_unique_id": (_i32, [_vp]),
    "sl_gather_init": (_i32, [_vp, _i32, _i32, _vp]),
    "sl_gather_counts": (_i32, [_vp, _i64, _vp, _vp]),
    "sl_gather": (_i32, [_vp, _vp, _i32, _vp, _vp, _i32, _vp, _vp, _vp]),
    "sl_decode_triangulate_batch": (_i32, [_vp, _vp, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _i64, _i32,
                                           _vp, _vp, _vp, _vp, _vp, _i32, _vp, _i64, _vp, _vp]),
    "sl_last_error": (ctypes.c_char_p, [_vp]),
    "sl_calib_products": (_i32, [_vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp]),
}

_lock = threading.Lock()
_lib = None


def load() -> ctypes.CDLL:
    """Load libslgpu.so (raises RuntimeError if it has not been built)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -c 'import "
                                   f"__graft_entry__ as g; g.build()'` (hipcc, gfx950)")
            lib = ctypes.CDLL(LIB_PATH)
            variant = bool(os.environ.get("SLGPU_LIB"))
            for name, (res, args) in _SIGS.items():
                try:
                    fn = getattr(lib, name)
                except AttributeError:
                    if variant:  # an older measurement build (SLGPU_LIB): entry points it predates are absent
                        continue
                    raise
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


class SLError(RuntimeError):
    pass


def check(code: int, ctx=None, what: str = "") -> None:
    """Map an SL_E* status to the exception type the reference raises."""
    if code == SL_OK:
        return
    msg = what
    if ctx is not None:
        raw = load().sl_ctx_last_error(ctx)
        msg = raw.decode() if raw else what
    if code in (SL_EINVAL, SL_ENOCALIB, SL_ECAPACITY):
        raise ValueError(msg)
    if code == SL_EINDEX:
        raise IndexError(msg)
    if code == SL_EIO:
        raise OSError(msg)
    raise SLError(f"libslgpu error {code}: {msg}")
