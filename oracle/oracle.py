"""ctypes wrapper of the CPU oracle (oracle/_build/libgsoracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg -- never by the product package.  See gs_oracle.h for what each function
restates (reference file:line) and how parity is pinned.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libgsoracle.so")
FLAG_CLEAN = 1

_L = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        vp = ctypes.c_void_p
        sig = {
            "ora_gen_sort_keys": (None, [ctypes.c_int, vp]),
            "ora_fnv1a64_words": (ctypes.c_uint64, [vp, ctypes.c_uint64]),
            "ora_argsort_f32": (None, [vp, vp, ctypes.c_int]),
            "ora_sort_pairs": (None, [vp, vp, ctypes.c_int64]),
            "ora_ply_count": (ctypes.c_int, [ctypes.c_char_p]),
            "ora_ply_load": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, vp, vp, vp, vp, vp]),
            "ora_cov3d": (None, [ctypes.c_int, vp, vp, vp]),
            "ora_sh_colours": (None, [ctypes.c_int, vp, vp, vp, vp, vp, vp]),
            "ora_preprocess": (None, [ctypes.c_int, vp, vp, vp, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                      ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_uint32,
                                      vp, vp, vp, vp, vp, vp]),
            "ora_emit": (ctypes.c_int64, [ctypes.c_int, vp, vp, vp, vp, vp, vp, ctypes.c_int64]),
            "ora_bins": (None, [vp, ctypes.c_int64, vp]),
            "ora_draw": (None, [ctypes.c_int, ctypes.c_int, ctypes.c_uint32, vp, vp, ctypes.c_int64, vp, vp, vp, vp]),
            "ora_draw_rows": (None, [ctypes.c_int, ctypes.c_int, ctypes.c_uint32, vp, vp, ctypes.c_int64, vp, vp, vp,
                                     vp, ctypes.c_int, ctypes.c_int]),
            "ora_expf": (ctypes.c_float, [ctypes.c_float]),
            "ora_num_threads": (ctypes.c_int, []),
        }
        for k, (r, a) in sig.items():
            f = getattr(L, k)
            f.restype = r
            f.argtypes = a
        _L = L
    return _L


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def gen_sort_keys(n: int) -> np.ndarray:
    out = np.empty(n, np.float32)
    lib().ora_gen_sort_keys(n, _p(out))
    return out


def fnv1a64_words(a: np.ndarray) -> int:
    w = np.ascontiguousarray(a).view(np.uint32)
    return int(lib().ora_fnv1a64_words(_p(w), w.size))


def argsort_f32(keys: np.ndarray, order: np.ndarray | None = None) -> np.ndarray:
    keys = np.ascontiguousarray(keys, np.float32)
    o = np.arange(len(keys), dtype=np.int32) if order is None else np.array(order, np.int32)
    lib().ora_argsort_f32(_p(keys), _p(o), len(keys))
    return o


def sort_pairs(keys: np.ndarray, vals: np.ndarray):
    k = np.array(keys, np.uint32)
    v = np.array(vals, np.uint32)
    lib().ora_sort_pairs(_p(k), _p(v), len(k))
    return k, v


def ply_load(path: str):
    n = lib().ora_ply_count(path.encode())
    if n < 0:
        raise IOError(path)
    means = np.zeros((n, 4), np.float32)
    cols = np.zeros((n, 4), np.float32)
    op = np.zeros(n, np.float32)
    sc = np.zeros((n, 3), np.float32)
    rot = np.zeros((n, 4), np.float32)
    if lib().ora_ply_load(path.encode(), n, _p(means), _p(cols), _p(op), _p(sc), _p(rot)) != 0:
        raise IOError(path)
    return means, cols, op, sc, rot


def cov3d(scales, rots) -> np.ndarray:
    s = np.ascontiguousarray(scales, np.float32)
    r = np.ascontiguousarray(rots, np.float32)
    out = np.zeros(6 * len(s), np.float32)
    lib().ora_cov3d(len(s), _p(s), _p(r), _p(out))
    return out


def sh_colours(means4, f_dc3, f_rest45, view16, visible, colours4) -> np.ndarray:
    """SURVEY f3 colours (GS_FLAG_SH) of the visible splats; others keep colours4's values"""
    m = np.ascontiguousarray(means4, np.float32)
    d = np.ascontiguousarray(f_dc3, np.float32)
    r = np.ascontiguousarray(f_rest45, np.float32)
    v = np.ascontiguousarray(view16, np.float32)
    vis = np.ascontiguousarray(visible, np.uint8)
    out = np.array(colours4, np.float32, copy=True, order="C")
    lib().ora_sh_colours(len(m), _p(m), _p(d), _p(r), _p(v), _p(vis), _p(out))
    return out


def expf(x: float) -> float:
    return lib().ora_expf(x)


KEY_CULLED = np.float32(1000000.0).view(np.uint32)  # preprocess.glsl:83 depth of a culled splat


def reference_draw_list(keys, vals, culled: int, flags: int):
    """The sorted list the reference's draw walks (ref mode).  preprocess.glsl:80-88 leaves every
    culled splat i in the sorted range with depth 1e6 and splatKeys[i] = 0, so after the sort it
    sits, as splat 0 (draw.glsl:97-98 reads splatKeys[indices[pos]]), among the entries: after
    every key whose bits are <= bits(1e6) (the emitted entries come first in the sort's input, so
    equal keys keep them ahead), before the larger bit patterns (negative keys, Q6).  countBins
    never bins 1e6, so only a Q10 over-read window reaches them.  `culled` = splats without
    entries (NDC-culled; det == 0, Q7, is placed the same way).  Clean mode: no such entries."""
    if flags & FLAG_CLEAN or culled <= 0:
        return vals, len(vals)
    P = int(np.searchsorted(keys, KEY_CULLED, side="right"))
    out = np.concatenate([vals[:P], np.zeros(culled, np.uint32), vals[P:]])
    return out, len(out)


def render(means4, cov6, opacity, colours4, u, flags: int = 0, stages: bool = True, draw: bool = True):
    """Full frame in the oracle: preprocess -> emit -> stable sort -> bins -> draw.
    ``u`` is a gs_uniforms-like object (view, vp, width, height, focal_x, ...)."""
    L = lib()
    means4 = np.ascontiguousarray(means4, np.float32)
    cov6 = np.ascontiguousarray(cov6, np.float32)
    opacity = np.ascontiguousarray(opacity, np.float32)
    colours4 = np.ascontiguousarray(colours4, np.float32)
    n = len(opacity)
    view = np.array(u.view[:], np.float32)
    vp = np.array(u.vp[:], np.float32)
    W, H = int(u.width), int(u.height)
    m2d = np.zeros(2 * n, np.float32)
    conic = np.zeros(4 * n, np.float32)
    z01 = np.zeros(n, np.float32)
    txy = np.zeros(2 * n, np.int32)
    rect = np.zeros(4 * n, np.int32)
    cnt = np.zeros(2 * n, np.int32)
    L.ora_preprocess(n, _p(means4), _p(cov6), _p(opacity), _p(view), _p(vp), W, H, u.focal_x, u.focal_y,
                     u.tan_fov_x, u.tan_fov_y, flags, _p(m2d), _p(conic), _p(z01), _p(txy), _p(rect), _p(cnt))
    E = int(L.ora_emit(n, _p(z01), _p(txy), _p(rect), _p(cnt), None, None, 0))
    keys = np.zeros(max(E, 1), np.uint32)
    vals = np.zeros(max(E, 1), np.uint32)
    L.ora_emit(n, _p(z01), _p(txy), _p(rect), _p(cnt), _p(keys), _p(vals), E)
    keys, vals = keys[:E], vals[:E]
    emitted = (keys.copy(), vals.copy()) if stages else None
    L.ora_sort_pairs(_p(keys), _p(vals), E)
    bins = np.zeros(256, np.uint32)
    L.ora_bins(_p(keys), E, _p(bins))
    img = None
    dvals, dE = reference_draw_list(keys, vals, n - int(cnt[0::2].sum()), flags)
    if draw:
        img = np.zeros((H, W, 4), np.uint8)
        L.ora_draw(W, H, flags, _p(bins), _p(dvals), dE, _p(m2d), _p(conic), _p(colours4), _p(img))
    out = dict(image=img, keys=keys, vals=vals, bins=bins, means2d=m2d, conics=conic, V=int(cnt[0::2].sum()),
               D=int(cnt[1::2].sum()), E=E, counts=cnt, z01=z01, tilexy=txy, rect=rect)
    if stages:
        out["emitted_keys"], out["emitted_vals"] = emitted
    return out


def time_frame(means4, cov6, opacity, colours4, u, flags: int = 0, row_step: int = 1) -> dict:
    """Time the oracle's frame stages (wall clock, host cores).  The blend is run on every
    ``row_step``-th pixel row only and its time scaled by row_step (a bounded sample)."""
    import time
    L = lib()
    means4 = np.ascontiguousarray(means4, np.float32)
    cov6 = np.ascontiguousarray(cov6, np.float32)
    opacity = np.ascontiguousarray(opacity, np.float32)
    colours4 = np.ascontiguousarray(colours4, np.float32)
    n = len(opacity)
    view = np.array(u.view[:], np.float32)
    vp = np.array(u.vp[:], np.float32)
    W, H = int(u.width), int(u.height)
    m2d = np.zeros(2 * n, np.float32)
    conic = np.zeros(4 * n, np.float32)
    z01 = np.zeros(n, np.float32)
    txy = np.zeros(2 * n, np.int32)
    rect = np.zeros(4 * n, np.int32)
    cnt = np.zeros(2 * n, np.int32)
    t0 = time.perf_counter()
    L.ora_preprocess(n, _p(means4), _p(cov6), _p(opacity), _p(view), _p(vp), W, H, u.focal_x, u.focal_y,
                     u.tan_fov_x, u.tan_fov_y, flags, _p(m2d), _p(conic), _p(z01), _p(txy), _p(rect), _p(cnt))
    E = int(L.ora_emit(n, _p(z01), _p(txy), _p(rect), _p(cnt), None, None, 0))
    keys = np.zeros(max(E, 1), np.uint32)
    vals = np.zeros(max(E, 1), np.uint32)
    L.ora_emit(n, _p(z01), _p(txy), _p(rect), _p(cnt), _p(keys), _p(vals), E)
    t1 = time.perf_counter()
    L.ora_sort_pairs(_p(keys), _p(vals), E)
    t2 = time.perf_counter()
    bins = np.zeros(256, np.uint32)
    L.ora_bins(_p(keys), E, _p(bins))
    t3 = time.perf_counter()
    img = np.zeros((H, W, 4), np.uint8)
    dvals, dE = reference_draw_list(keys[:E], vals[:E], n - int(cnt[0::2].sum()), flags)
    L.ora_draw_rows(W, H, flags, _p(bins), _p(dvals), dE, _p(m2d), _p(conic), _p(colours4), _p(img), 0, row_step)
    t4 = time.perf_counter()
    draw_full = (t4 - t3) * row_step
    total = (t1 - t0) + (t2 - t1) + (t3 - t2) + draw_full
    return dict(preprocess_s=t1 - t0, sort_s=t2 - t1, bins_s=t3 - t2, draw_sample_s=t4 - t3, draw_est_s=draw_full,
                frame_est_s=total, E=E, row_step=row_step, threads=L.ora_num_threads())
