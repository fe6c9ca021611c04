"""ctypes binding of ``lib/libgsplat_hip.so`` (the C ABI declared in ``include/gsplat.h``).

The shared library is the product: hand-written HIP for gfx950.  There is no fallback --
if the library is missing, importing a renderer entry point raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libgsplat_hip.so")

GS_OK = 0
GS_ERR_INVALID = -1
GS_ERR_HIP = -2
GS_ERR_IO = -3
GS_ERR_NOMEM = -4
GS_ERR_STATE = -5

GS_FLAG_CLEAN = 1
GS_FLAG_FAST_EXP = 2
GS_FLAG_TIMING = 4
GS_FLAG_NO_CULL = 8
GS_FLAG_DRAW_STATS = 16
GS_FLAG_DRAW_TRACE = 128  # with GS_FLAG_DRAW_STATS: per-block times and counts only
GS_FLAG_SH = 64

GS_READ_KEYS = 1
GS_READ_VALS = 2
GS_READ_BINS = 3
GS_TIMING_FRAME = 0
GS_TIMING_DRAW = 1
GS_TIMING_STAGES = 2
GS_READ_MEANS2D = 4
GS_READ_CONICS = 5
GS_READ_CULLBOX = 6


GS_KERNEL_DRAW = 1
GS_KERNEL_SORT = 2


class gs_uniforms(ctypes.Structure):
    _fields_ = [
        ("view", ctypes.c_float * 16),
        ("vp", ctypes.c_float * 16),
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("focal_x", ctypes.c_float),
        ("focal_y", ctypes.c_float),
        ("tan_fov_x", ctypes.c_float),
        ("tan_fov_y", ctypes.c_float),
    ]


class gs_frame_stats(ctypes.Structure):
    _fields_ = [
        ("num_splats", ctypes.c_int64),
        ("visible", ctypes.c_int64),
        ("duplicates", ctypes.c_int64),
        ("entries", ctypes.c_int64),
        ("ms_preprocess", ctypes.c_float),
        ("ms_sort", ctypes.c_float),
        ("ms_bins", ctypes.c_float),
        ("ms_draw", ctypes.c_float),
        ("ms_total", ctypes.c_float),
    ]


class gs_camera(ctypes.Structure):
    _fields_ = [
        ("position", ctypes.c_float * 3),
        ("rotation", ctypes.c_float * 3),
        ("fovy", ctypes.c_float),
        ("near_plane", ctypes.c_float),
        ("far_plane", ctypes.c_float),
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
    ]


class gs_timing(ctypes.Structure):
    _fields_ = [
        ("frames", ctypes.c_int64),
        ("ms_preprocess", ctypes.c_double),
        ("ms_emit", ctypes.c_double),
        ("ms_sort", ctypes.c_double),
        ("ms_bins", ctypes.c_double),
        ("ms_draw", ctypes.c_double),
        ("ms_frame", ctypes.c_double),
        ("ms_host_render", ctypes.c_double),
        ("ms_host_wait", ctypes.c_double),
        ("host_renders", ctypes.c_int64),
    ]


_vp = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64
_u32 = ctypes.c_uint32
_f = ctypes.c_float
_fp = ctypes.POINTER(ctypes.c_float)
_sz = ctypes.c_size_t

# name -> (restype, argtypes); every symbol include/gsplat.h declares
SIGNATURES = {
    "gs_version": (ctypes.c_char_p, []),
    "gs_device_count": (_i, [ctypes.POINTER(_i)]),
    "gs_last_error": (ctypes.c_char_p, [_vp]),
    "gs_ctx_create": (_i, [_i, ctypes.POINTER(_vp)]),
    "gs_ctx_destroy": (None, [_vp]),
    "gs_sync": (_i, [_vp]),
    "gs_stream": (_vp, [_vp]),
    "gs_ctx_set_lanes": (_i, [_vp, _i]),
    "gs_ctx_set_sort_prefix": (_i, [_vp, _i, ctypes.POINTER(_i)]),
    "gs_ctx_set_draw_sub": (_i, [_vp, _i, ctypes.POINTER(_i)]),
    "gs_ctx_set_small_limits": (_i, [_vp, ctypes.c_int64, ctypes.c_int64]),
    "gs_ctx_set_bucket_sort": (_i, [_vp, _i]),
    "gs_ctx_set_kept_emission": (_i, [_vp, _i, ctypes.POINTER(ctypes.c_uint64)]),
    "gs_ctx_set_lookback_spin": (_i, [_vp, _i, ctypes.POINTER(ctypes.c_uint64)]),
    "gs_prefix_stats": (_i, [_vp, _vp, _i]),
    "gs_malloc": (_i, [_vp, _sz, ctypes.POINTER(_vp)]),
    "gs_free": (_i, [_vp, _vp]),
    "gs_memcpy_h2d": (_i, [_vp, _vp, _vp, _sz]),
    "gs_memcpy_d2h": (_i, [_vp, _vp, _vp, _sz]),
    "gs_memset": (_i, [_vp, _vp, _i, _sz]),
    "gs_stream_copy_gbs": (_i, [_vp, _sz, _i, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "gs_ply_count": (_i, [ctypes.c_char_p, ctypes.POINTER(_i)]),
    "gs_ply_load": (_i, [ctypes.c_char_p, _i, _vp, _vp, _vp, _vp, _vp]),
    "gs_ply_write": (_i, [ctypes.c_char_p, _i, _vp, _vp, _vp, _vp, _vp]),
    "gs_save_png": (_i, [ctypes.c_char_p, _i, _i, _vp, _i]),
    "gs_activate": (_i, [_i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gs_covariance3d": (_i, [_i, _vp, _vp, _vp]),
    "gs_camera_update": (_i, [ctypes.POINTER(gs_camera), _vp, _vp, _fp, _fp, _fp, _fp]),
    "gs_camera_uniforms": (_i, [ctypes.POINTER(gs_camera), ctypes.POINTER(gs_uniforms)]),
    "gs_scene_create": (_i, [_vp, _i, _vp, _vp, _vp, _vp, ctypes.POINTER(_vp)]),
    "gs_scene_load_ply": (_i, [_vp, ctypes.c_char_p, ctypes.POINTER(_vp)]),
    "gs_scene_download": (_i, [_vp, _vp, _vp, _vp, _vp]),
    "gs_scene_set_sh": (_i, [_vp, _vp, _vp]),
    "gs_ply_load_sh": (_i, [ctypes.c_char_p, _i, _vp, _vp]),
    "gs_scene_destroy": (None, [_vp]),
    "gs_scene_count": (_i, [_vp]),
    "gs_render": (_i, [_vp, _vp, ctypes.POINTER(gs_uniforms), _u32, _vp, _i, ctypes.POINTER(gs_frame_stats)]),
    "gs_last_stats": (_i, [_vp, _vp]),
    "gs_seen_stats": (_i, [_vp, _vp]),
    "gs_preprocess": (_i, [_vp, _vp, ctypes.POINTER(gs_uniforms), _u32, ctypes.POINTER(gs_frame_stats)]),
    "gs_sort": (_i, [_vp]),
    "gs_compute_bins": (_i, [_vp]),
    "gs_draw": (_i, [_vp, _vp, _i, _i, _f, _f, _u32, _vp, _i]),
    "gs_frame_read": (_i, [_vp, _i, _vp, _sz]),
    "gs_argsort_f32": (_i, [_vp, _vp, _vp, _i64]),
    "gs_sort_pairs_u32": (_i, [_vp, _vp, _vp, _i64]),
    "gs_pad_buffer": (_i, [_i, _i]),
    "gs_last_kernel_ms": (_i, [_vp, _i, _fp]),
    "gs_timing_reset": (_i, [_vp]),
    "gs_timing_enable": (_i, [_vp, _i]),
    "gs_draw_stats": (_i, [_vp, _vp, _i]),
    "gs_draw_block_trace": (_i, [_vp, _vp, _i]),
    "gs_timing_read": (_i, [_vp, ctypes.POINTER(gs_timing)]),
}

_lib = None


class GsError(RuntimeError):
    """A libgsplat_hip call returned a negative status."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def lib() -> ctypes.CDLL:
    """Load libgsplat_hip.so once.  Raises if it has not been built -- no fallback."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(make -C openglgaussiansplattingrenderer_amd). There is no CPU fallback."
            )
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, ctx=None) -> int:
    if rc < 0:
        msg = lib().gs_last_error(ctx)
        raise GsError(rc, msg.decode() if msg else "")
    return rc


def ptr(a) -> ctypes.c_void_p:
    """data pointer of a numpy array (or None)"""
    if a is None:
        return None
    return ctypes.c_void_p(a.ctypes.data)
