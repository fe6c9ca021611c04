"""MI355X-native (gfx950) Gaussian-splat forward renderer + radix sort.

Drop-in for the hot path of thomas-chernaik/OpenGLGaussianSplattingRenderer: preprocess ->
depth radix sort -> per-tile front-to-back alpha blend, as hand-written HIP kernels behind
the C ABI in include/gsplat.h (lib/libgsplat_hip.so).  This package mirrors the reference's
C++ API (Splats, GPURadixSort, PadBuffer, Camera) on top of that ABI.
"""
from ._native import (GS_FLAG_CLEAN, GS_FLAG_DRAW_STATS, GS_FLAG_DRAW_TRACE, GS_FLAG_FAST_EXP, GS_FLAG_NO_CULL, GS_FLAG_SH, GS_FLAG_TIMING,
                      GS_KERNEL_DRAW,
                      GS_KERNEL_SORT, GS_READ_BINS, GS_READ_CONICS, GS_READ_CULLBOX, GS_READ_KEYS,
                      GS_READ_MEANS2D, GS_READ_VALS, GS_TIMING_DRAW, GS_TIMING_FRAME, GS_TIMING_STAGES, GsError,
                      LIB_PATH, lib)
from .splats import (Camera, Context, DeviceBuffer, GPURadixSort, PadBuffer, Splats, activate,
                     covariance3d, createAndLinkSortAndHistogramShaders, createRandomNumbersFloat, load_ply,
                     load_ply_sh, main_camera, make_uniforms, save_ply, save_png, sort_pairs)

__all__ = [
    "Camera", "Context", "DeviceBuffer", "GPURadixSort", "PadBuffer", "Splats", "activate", "covariance3d",
    "createAndLinkSortAndHistogramShaders", "createRandomNumbersFloat", "load_ply", "main_camera",
    "make_uniforms", "save_ply", "save_png", "sort_pairs", "lib", "LIB_PATH", "GsError",
    "GS_FLAG_CLEAN", "GS_FLAG_DRAW_STATS", "GS_FLAG_DRAW_TRACE", "GS_FLAG_FAST_EXP", "GS_FLAG_TIMING", "GS_FLAG_NO_CULL", "GS_FLAG_SH",
    "load_ply_sh",
    "GS_READ_KEYS", "GS_READ_VALS", "GS_READ_BINS", "GS_READ_MEANS2D", "GS_READ_CONICS", "GS_READ_CULLBOX",
    "GS_KERNEL_DRAW", "GS_KERNEL_SORT", "GS_TIMING_FRAME", "GS_TIMING_DRAW", "GS_TIMING_STAGES",
]
