"""Host-side mirror of the reference's C++ API for the hot path.

Reference (thomas-chernaik/OpenGLGaussianSplattingRenderer):
  include/Splats.h:29-124 / src/Splats.cpp   -> class Splats
  include/sort.h:15-23    / src/sort.cpp     -> GPURadixSort, PadBuffer,
                                                createAndLinkSortAndHistogramShaders
  include/Camera.h / src/Camera.cpp          -> class Camera
  src/utils.cpp:49-63                        -> createRandomNumbersFloat

Same names, argument meaning and error behaviour; the GL objects become device buffers
owned by a ``Context`` (one per GPU) and every stage runs as HIP kernels through
``libgsplat_hip.so``.  Matrices are numpy float32 (4,4) arrays indexed like glm,
``M[c, r] == glm m[c][r]`` (column-major memory).
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

from . import _native as N
from ._native import check, lib, ptr


class Context:
    """A device + HIP stream (replaces the GL context; one per GPU, not thread-safe)."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        check(lib().gs_ctx_create(int(device), ctypes.byref(h)))
        self.handle = h
        self.device = device

    def close(self):
        if self.handle:
            lib().gs_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        check(lib().gs_sync(self.handle), self.handle)

    def set_lanes(self, lanes: int):
        """frames in flight on the device (gs_ctx_set_lanes): 2 (default) overlaps frame k+1's
        preprocess / emission / sort with frame k's blend; 3 keeps one more frame in flight
        (throughput +1-2 % at C3); 1 runs frames one after the other"""
        check(lib().gs_ctx_set_lanes(self.handle, int(lanes)), self.handle)

    def set_sort_prefix(self, target: int = -1) -> int:
        """prefix sort of frames enqueued without a round trip (gs_ctx_set_sort_prefix): every
        tile list sorted at least `target` entries deep (0: always the full sort; < 0: leave it);
        returns the current target"""
        cur = ctypes.c_int()
        check(lib().gs_ctx_set_sort_prefix(self.handle, int(target), ctypes.byref(cur)), self.handle)
        return cur.value

    def set_small_limits(self, draw_entries: int = -1, sort_entries: int = -1):
        """gs_ctx_set_small_limits: entry counts below which frames blend in 8x8 sub-blocks /
        sort in 8 launches (-1 leaves a limit)"""
        check(lib().gs_ctx_set_small_limits(self.handle, int(draw_entries), int(sort_entries)), self.handle)

    def set_bucket_sort(self, on: int = -1) -> int:
        """gs_ctx_set_bucket_sort: the small sort by tile then per tile (1, default) or in four
        8-bit passes (0); -1 leaves it.  Returns the form set."""
        r = lib().gs_ctx_set_bucket_sort(self.handle, int(on))
        check(min(r, 0), self.handle)
        return r

    def set_kept_emission(self, on: int = -1):
        """gs_ctx_set_kept_emission: prefix-sorted frames emit and sort only the entries within
        the previous frame's key bounds (1) or every entry (0, default); -1 leaves it.  Returns
        (setting, frames emitted that way so far)."""
        n = ctypes.c_uint64()
        r = lib().gs_ctx_set_kept_emission(self.handle, int(on), ctypes.byref(n))
        check(min(r, 0), self.handle)
        return r, int(n.value)

    def set_lookback_spin(self, limit: int = -1):
        """gs_ctx_set_lookback_spin: polls the fused preprocess + emission's look-back waits before
        it gives up and the frame is rendered again (0: at once, a test hook; -1 leaves it).
        Returns (limit, frames rendered again for it)."""
        red = ctypes.c_uint64()
        r = lib().gs_ctx_set_lookback_spin(self.handle, int(limit), ctypes.byref(red))
        check(min(r, 0), self.handle)
        return r, int(red.value)

    def set_draw_sub(self, sub: int = -1) -> int:
        """the blend's sub-block form (gs_ctx_set_draw_sub): 0 by entry count (default), 8 (one
        pixel per lane, small frames) or 16 (2x2 quads per lane, large frames); -1 leaves it.
        Returns the form the newest frame's blend used (0 before any)."""
        cur = ctypes.c_int()
        check(lib().gs_ctx_set_draw_sub(self.handle, int(sub), ctypes.byref(cur)), self.handle)
        return cur.value

    def prefix_stats(self, reset: bool = False) -> dict:
        """gs_prefix_stats: frames prefix-sorted, of them rendered again, entries kept / entries of
        the newest retired prefix-sorted frame"""
        a = np.zeros(4, np.uint64)
        check(lib().gs_prefix_stats(self.handle, ptr(a), int(reset)), self.handle)
        return dict(frames=int(a[0]), redone=int(a[1]), kept=int(a[2]), entries=int(a[3]))

    def timing_reset(self):
        check(lib().gs_timing_reset(self.handle), self.handle)

    def timing_read(self) -> dict:
        t = N.gs_timing()
        check(lib().gs_timing_read(self.handle, ctypes.byref(t)), self.handle)
        return {k: getattr(t, k) for k, _ in N.gs_timing._fields_}

    def timing_enable(self, mode: int):
        """GS_TIMING_FRAME / GS_TIMING_DRAW / GS_TIMING_STAGES (gs_timing_enable)"""
        check(lib().gs_timing_enable(self.handle, int(mode)), self.handle)

    def draw_stats(self, reset: bool = True) -> dict:
        a = np.zeros(16, np.uint64)
        check(lib().gs_draw_stats(self.handle, ptr(a), int(reset)), self.handle)
        return dict(blocks=int(a[0]), iterations=int(a[1]), survivors=int(a[2]), list_entries=int(a[3]),
                    max_iterations=int(a[4]), max_survivors=int(a[5]), max_cycles=int(a[6]), sum_cycles=int(a[7]),
                    wave_steps=int(a[8]), steps_any_need=int(a[9]), pixel_needs=int(a[10]))

    def draw_block_trace(self, blocks: int) -> np.ndarray:
        """[blocks, 16] uint32 per draw block (gs_draw_block_trace): start, end (100 MHz ticks),
        iterations, survivors, survivor steps, steps with a needing pixel, pixel needs, list
        entries, steps while <= 64 / <= 128 pixels active, events while <= 64, done-mask refreshes,
        dense-phase steps with > 192 / 129-192 / 65-128 active pixels, dense-phase events."""
        a = np.zeros((blocks, 16), np.uint32)
        n = lib().gs_draw_block_trace(self.handle, ptr(a), int(blocks))
        check(n, self.handle)
        return a[:n]

    def last_kernel_ms(self, kernel: int) -> float:
        ms = ctypes.c_float()
        check(lib().gs_last_kernel_ms(self.handle, kernel, ctypes.byref(ms)), self.handle)
        return ms.value


class DeviceBuffer:
    """A device allocation (stands in for a GL shader-storage buffer object)."""

    def __init__(self, ctx: Context, nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        check(lib().gs_malloc(ctx.handle, self.nbytes, ctypes.byref(p)), ctx.handle)
        self.ptr = p

    @classmethod
    def from_array(cls, ctx: Context, a: np.ndarray) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        b = cls(ctx, a.nbytes)
        b.upload(a)
        return b

    def upload(self, a: np.ndarray):
        a = np.ascontiguousarray(a)
        if a.nbytes > self.nbytes:
            raise ValueError("array larger than the buffer")
        check(lib().gs_memcpy_h2d(self.ctx.handle, self.ptr, ptr(a), a.nbytes), self.ctx.handle)

    def download(self, dtype, count: int) -> np.ndarray:
        out = np.empty(count, dtype=dtype)
        if out.nbytes > self.nbytes:
            raise ValueError("read past the buffer")
        check(lib().gs_memcpy_d2h(self.ctx.handle, ptr(out), self.ptr, out.nbytes), self.ctx.handle)
        return out

    def free(self):
        if self.ptr:
            lib().gs_free(self.ctx.handle, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


# --------------------------------------------------------------------- sort API
def createAndLinkSortAndHistogramShaders():
    """src/sort.cpp:15-124.  Nothing to compile at run time (kernels are built ahead of
    time for gfx950); returns placeholder program handles (histogram, sort, sum)."""
    print("compiling sorting shaders", file=sys.stderr)
    print("compiled and linked sorting shaders", file=sys.stderr)
    return 1, 2, 3


def PadBuffer(size: int, unitWidth: int) -> int:
    """src/sort.cpp:127-137"""
    return int(lib().gs_pad_buffer(int(size), int(unitWidth)))


def GPURadixSort(histogramProgram, prefixSumProgram, sortProgram, intermediateBuffer, orderBuffer: DeviceBuffer,
                 histogramBuffer, size: int, workGroupCount: int, workGroupSize: int, buffer: DeviceBuffer):
    """src/sort.cpp:139-203: stable argsort of the float keys in ``buffer`` by their bits.

    ``orderBuffer`` (int32[size]) is read as the initial order and receives the sorted
    order; the keys are not moved.  Program handles, ``intermediateBuffer``,
    ``histogramBuffer`` and the workgroup shape are accepted for signature parity; the
    HIP sort keeps its own scratch in the context.
    """
    number_of_sections = workGroupCount * workGroupSize
    if number_of_sections <= 0:
        print(f"Size must be a multiple of {number_of_sections}", file=sys.stderr)
        return
    ctx = orderBuffer.ctx
    check(lib().gs_argsort_f32(ctx.handle, buffer.ptr, orderBuffer.ptr, int(size)), ctx.handle)


def sort_pairs(ctx: Context, keys: DeviceBuffer, vals: DeviceBuffer, n: int):
    """Stable in-place sort of (uint32 key, uint32 value) pairs by key."""
    check(lib().gs_sort_pairs_u32(ctx.handle, keys.ptr, vals.ptr, int(n)), ctx.handle)


# ------------------------------------------------------------------- test RNG
def createRandomNumbersFloat(size: int) -> np.ndarray:
    """src/utils.cpp:49-63 -- srand(20), glibc rand(): rand()%255 + rand()/RAND_MAX + 0.5"""
    if size < 1:
        print("Error: size must be greater than 0", file=sys.stderr)
        return np.zeros(0, np.float32)
    libc = ctypes.CDLL("libc.so.6")
    libc.rand.restype = ctypes.c_int
    libc.srand(20)
    raw = np.fromiter((libc.rand() for _ in range(2 * size)), dtype=np.int64, count=2 * size)
    random = (raw[0::2] % 255).astype(np.float32)
    frac = raw[1::2].astype(np.float32) / np.float32(2147483647)
    return (frac + random) + np.float32(0.5)


# --------------------------------------------------------------------- camera
class Camera:
    """src/Camera.cpp restatement (uniform generator).  Keeps the reference's quirks:
    tan() of degrees in getTanFovx/y (Q1) and focal_x from fovy (Q3)."""

    def __init__(self, x: float = 0.0, y: float = 0.0, z: float = 0.0, *, width: int = 1024, height: int = 512,
                 near: float | None = None):
        self.position = np.array([x, y, z], np.float32)
        self.rotation = np.zeros(3, np.float32)
        self.fovy = 60.0
        # Camera() uses near 0.0001, Camera(x,y,z) uses 0.1 (src/Camera.cpp:13,25)
        self.near = 0.1 if near is None else near
        self.far = 10000.0
        self.width, self.height = int(width), int(height)

    def _c(self) -> N.gs_camera:
        c = N.gs_camera()
        for k in range(3):
            c.position[k] = float(self.position[k])
            c.rotation[k] = float(self.rotation[k])
        c.fovy, c.near_plane, c.far_plane = self.fovy, self.near, self.far
        c.width, c.height = self.width, self.height
        return c

    def _update(self):
        view = np.zeros(16, np.float32)
        proj = np.zeros(16, np.float32)
        fx, fy, tx, ty = (ctypes.c_float() for _ in range(4))
        check(lib().gs_camera_update(ctypes.byref(self._c()), ptr(view), ptr(proj), ctypes.byref(fx), ctypes.byref(fy),
                                     ctypes.byref(tx), ctypes.byref(ty)))
        return view.reshape(4, 4), proj.reshape(4, 4), fx.value, fy.value, tx.value, ty.value

    def update(self):
        pass  # state is recomputed on demand

    def setWidthHeight(self, width: int, height: int):
        self.width, self.height = int(width), int(height)

    def getWidth(self) -> int:
        return self.width

    def getHeight(self) -> int:
        return self.height

    def getViewMatrix(self) -> np.ndarray:
        return self._update()[0]

    def getProjectionMatrix(self) -> np.ndarray:
        return self._update()[1]

    def getFocalX(self) -> float:
        return self._update()[2]

    def getFocalY(self) -> float:
        return self._update()[3]

    def getTanFovx(self) -> float:
        return self._update()[4]

    def getTanFovy(self) -> float:
        return self._update()[5]

    def rotateRight(self, angle: float):
        self.rotation[1] = np.float32(self.rotation[1] + np.float32(angle))

    def rotateLeft(self, angle: float):
        self.rotateRight(-angle)

    def rotateUp(self, angle: float):
        self.rotation[0] = np.float32(self.rotation[0] + np.float32(angle))

    def rotateDown(self, angle: float):
        self.rotateUp(-angle)

    def moveForward(self, distance: float):
        v = self.getViewMatrix()  # upper-left 3x3 of view == rotationMatrix (view = R * T)
        d = np.float32(distance)
        self.position = (self.position + np.array([v[0, 2] * d, v[1, 2] * d, v[2, 2] * d], np.float32)).astype(np.float32)

    def moveBackward(self, distance: float):
        self.moveForward(-distance)

    def moveLeft(self, distance: float):
        v = self.getViewMatrix()
        d = np.float32(distance)
        self.position = (self.position + np.array([v[0, 0] * d, v[1, 0] * d, v[2, 0] * d], np.float32)).astype(np.float32)

    def moveRight(self, distance: float):
        self.moveLeft(-distance)

    def moveUp(self, distance: float):
        self.position = (self.position + np.array([0, distance, 0], np.float32)).astype(np.float32)

    def moveDown(self, distance: float):
        self.moveUp(-distance)

    def uniforms(self) -> N.gs_uniforms:
        """The gpuRender arguments exactly as main.cpp:62-64 passes them (tan x/y swapped, Q2)."""
        u = N.gs_uniforms()
        check(lib().gs_camera_uniforms(ctypes.byref(self._c()), ctypes.byref(u)))
        return u


def main_camera(width: int = 1024, height: int = 512) -> Camera:
    """main.cpp:40-45 pose: Camera(5, 0.5, -4); rotateDown(20); rotateRight(40)."""
    cam = Camera(5.0, 0.5, -4.0)
    cam.rotateDown(20.0)
    cam.rotateRight(40.0)
    cam.setWidthHeight(width, height)
    return cam


def make_uniforms(view, width, height, focal_x, focal_y, tan_fov_x, tan_fov_y, vp) -> N.gs_uniforms:
    u = N.gs_uniforms()
    v = np.ascontiguousarray(view, np.float32).reshape(16)
    p = np.ascontiguousarray(vp, np.float32).reshape(16)
    for k in range(16):
        u.view[k] = float(v[k])
        u.vp[k] = float(p[k])
    u.width, u.height = int(width), int(height)
    u.focal_x, u.focal_y = float(focal_x), float(focal_y)
    u.tan_fov_x, u.tan_fov_y = float(tan_fov_x), float(tan_fov_y)
    return u


# ------------------------------------------------------------- loader helpers
def load_ply_sh(path: str, n: int):
    """raw (f_dc3 (n,3), f_rest45 (n,45)) of a ply -- the fields loadSplats drops"""
    d = np.zeros((n, 3), np.float32)
    r = np.zeros((n, 45), np.float32)
    check(lib().gs_ply_load_sh(os.fsencode(path), int(n), ptr(d), ptr(r)))
    return d, r


def save_png(filename: str, rgba8: np.ndarray, flip_y: bool = False):
    """RGBA8 image (H, W, 4), row 0 = GL row 0, to PNG (gs_save_png)."""
    img = np.ascontiguousarray(rgba8, np.uint8)
    H, W = img.shape[0], img.shape[1]
    check(lib().gs_save_png(os.fsencode(filename), int(W), int(H), ptr(img), int(flip_y)))


def load_ply(filePath: str):
    """src/Splats.cpp:174-344 through the library's C++ loader.
    Returns means3D (N,4), colours (N,4), opacities (N,), scales (N,3), rotations (N,4)."""
    n = ctypes.c_int()
    check(lib().gs_ply_count(filePath.encode(), ctypes.byref(n)))
    N_ = n.value
    means = np.zeros((N_, 4), np.float32)
    cols = np.zeros((N_, 4), np.float32)
    op = np.zeros(N_, np.float32)
    sc = np.zeros((N_, 3), np.float32)
    rot = np.zeros((N_, 4), np.float32)
    check(lib().gs_ply_load(filePath.encode(), N_, ptr(means), ptr(cols), ptr(op), ptr(sc), ptr(rot)))
    return means, cols, op, sc, rot


def save_ply(path: str, means, rotations, scales, opacities, colours):
    """tests/plyFileGenerator.py:155-249 byte layout, via the library's C++ writer."""
    m = np.ascontiguousarray(means, np.float32).reshape(-1, 3)
    r = np.ascontiguousarray(rotations, np.float32).reshape(-1, 4)
    s = np.ascontiguousarray(scales, np.float32).reshape(-1, 3)
    o = np.ascontiguousarray(opacities, np.float32).reshape(-1)
    c = np.ascontiguousarray(colours, np.float32).reshape(-1, 3)
    check(lib().gs_ply_write(path.encode(), len(m), ptr(m), ptr(r), ptr(s), ptr(o), ptr(c)))


def activate(f_dc, opacity_logit, log_scale, rot_raw):
    """the loader's activations on raw records (same arithmetic as loadSplats)"""
    f = np.ascontiguousarray(f_dc, np.float32).reshape(-1, 3)
    n = len(f)
    o = np.ascontiguousarray(opacity_logit, np.float32).reshape(-1)
    s = np.ascontiguousarray(log_scale, np.float32).reshape(-1, 3)
    r = np.ascontiguousarray(rot_raw, np.float32).reshape(-1, 4)
    cols = np.zeros((n, 4), np.float32)
    op = np.zeros(n, np.float32)
    sc = np.zeros((n, 3), np.float32)
    rot = np.zeros((n, 4), np.float32)
    check(lib().gs_activate(n, ptr(f), ptr(o), ptr(s), ptr(r), ptr(cols), ptr(op), ptr(sc), ptr(rot)))
    return cols, op, sc, rot


def covariance3d(scales, rotations) -> np.ndarray:
    """src/Splats.cpp:414-479 -> flat float32[6N]"""
    s = np.ascontiguousarray(scales, np.float32).reshape(-1, 3)
    r = np.ascontiguousarray(rotations, np.float32).reshape(-1, 4)
    out = np.zeros(6 * len(s), np.float32)
    check(lib().gs_covariance3d(len(s), ptr(s), ptr(r), ptr(out)))
    return out


# --------------------------------------------------------------------- Splats
class Splats:
    """include/Splats.h:29-124.  ``Splats(path, width, height)`` loads the ply, computes the
    3D covariances on the host and uploads the scene; ``gpuRender`` runs the frame as HIP
    kernels.  ``flags`` selects ref (default: the reference's deterministic quirks kept) or
    GS_FLAG_CLEAN, and the blend's exp (bit-exact polynomial or GS_FLAG_FAST_EXP)."""

    def __init__(self, filePath: str | None, width: int, height: int, *, ctx: Context | None = None,
                 device: int = 0, flags: int = 0, arrays=None, gpu_load: bool = False, sh: bool = False):
        self.ctx = ctx if ctx is not None else Context(device)
        self.flags = int(flags)
        print("setting up splats", file=sys.stderr)
        if gpu_load:  # activations + covariance on the GPU (gs_scene_load_ply)
            self._load_gpu(filePath, width, height)
            if sh:
                self.set_sh(*load_ply_sh(filePath, self.numSplats))
            print("finished setting up splats", file=sys.stderr)
            return
        if arrays is None:
            self.loadSplats(filePath)
        else:
            self.means3D, self.colours, self.opacities, self.scales, self.rotations = arrays
            self.numSplats = len(self.means3D)
        self.sphericalHarmonics = np.zeros(0, np.float32)  # never filled (include/Splats.h:59)
        self.computeCovarianceMatrices()
        self._scene = None
        self.loadToGPU(width, height)
        if sh and filePath is not None:  # keep the f_rest the reference discards
            self.set_sh(*load_ply_sh(filePath, self.numSplats))
        print("finished setting up splats", file=sys.stderr)

    def set_sh(self, f_dc3, f_rest45):
        """attach degree-3 SH (raw f_dc, f_rest in ply layout) for GS_FLAG_SH frames"""
        d = np.ascontiguousarray(f_dc3, np.float32).reshape(-1, 3)
        r = np.ascontiguousarray(f_rest45, np.float32).reshape(-1, 45)
        assert len(d) == len(r) == self.numSplats
        check(lib().gs_scene_set_sh(self._scene, ptr(d), ptr(r)), self.ctx.handle)
        self.sphericalHarmonics = np.concatenate([d, r], axis=1)

    @classmethod
    def from_raw(cls, means3, f_dc, opacity_logit, log_scale, rot_raw, width, height, **kw) -> "Splats":
        """Scene from raw (pre-activation) ply fields -- what loadSplats would read from a file."""
        cols, op, sc, rot = activate(f_dc, opacity_logit, log_scale, rot_raw)
        m = np.ascontiguousarray(means3, np.float32).reshape(-1, 3)
        means4 = np.concatenate([m, np.ones((len(m), 1), np.float32)], axis=1)
        return cls(None, width, height, arrays=(means4, cols, op, sc, rot), **kw)

    def _load_gpu(self, filePath: str, width: int, height: int):
        h = ctypes.c_void_p()
        check(lib().gs_scene_load_ply(self.ctx.handle, os.fsencode(filePath), ctypes.byref(h)), self.ctx.handle)
        self._scene = h
        self.numSplats = int(lib().gs_scene_count(h))
        empty = np.zeros((0, 4), np.float32)
        self.means3D = self.colours = self.rotations = empty
        self.opacities, self.scales = np.zeros(0, np.float32), np.zeros((0, 3), np.float32)
        self.covarianceMatrices = np.zeros(0, np.float32)
        self.sphericalHarmonics = np.zeros(0, np.float32)
        self.width, self.height = int(width), int(height)
        self._texture = DeviceBuffer(self.ctx, self.width * self.height * 4)
        self._stats = N.gs_frame_stats()

    def download(self):
        """(means4, cov6, opacity, colours4) of the device scene (gs_scene_download)"""
        n = self.numSplats
        m, c, o, col = (np.zeros(4 * n, np.float32), np.zeros(6 * n, np.float32), np.zeros(n, np.float32),
                        np.zeros(4 * n, np.float32))
        check(lib().gs_scene_download(self._scene, ptr(m), ptr(c), ptr(o), ptr(col)), self.ctx.handle)
        return m.reshape(n, 4), c, o, col.reshape(n, 4)

    # src/Splats.cpp:174-344
    def loadSplats(self, filePath: str):
        print("Loading splats from file", file=sys.stderr)
        self.means3D, self.colours, self.opacities, self.scales, self.rotations = load_ply(filePath)
        self.numSplats = len(self.means3D)
        print(f"num splats: {self.numSplats}", file=sys.stderr)
        print("Finished loading splats from file", file=sys.stderr)

    # src/Splats.cpp:414-438
    def computeCovarianceMatrices(self):
        self.covarianceMatrices = covariance3d(self.scales, self.rotations)

    def loadShaders(self):
        """src/Splats.cpp:156-172 -- kernels are compiled ahead of time; nothing to do."""

    # src/Splats.cpp:61-154
    def loadToGPU(self, width: int, height: int):
        if self._scene is not None:
            lib().gs_scene_destroy(self._scene)
            self._scene = None
        h = ctypes.c_void_p()
        check(lib().gs_scene_create(self.ctx.handle, self.numSplats, ptr(np.ascontiguousarray(self.means3D, np.float32)),
                                    ptr(self.covarianceMatrices), ptr(np.ascontiguousarray(self.opacities, np.float32)),
                                    ptr(np.ascontiguousarray(self.colours, np.float32)), ctypes.byref(h)), self.ctx.handle)
        self._scene = h
        self.width, self.height = int(width), int(height)
        self._texture = DeviceBuffer(self.ctx, self.width * self.height * 4)
        self._stats = N.gs_frame_stats()

    @property
    def stats(self) -> N.gs_frame_stats:
        """counts of the newest frame (gs_last_stats: waits for it)"""
        st = N.gs_frame_stats()
        check(lib().gs_last_stats(self.ctx.handle, ctypes.byref(st)), self.ctx.handle)
        return st

    @property
    def numDuplicates(self) -> int:
        """include/Splats.h:56 -- duplicate entries of the newest frame"""
        return int(self.stats.duplicates)

    def __del__(self):
        try:
            if self._scene is not None:
                lib().gs_scene_destroy(self._scene)  # safe after the ctx is gone (detached)
                self._scene = None
        except Exception:
            pass

    # src/Splats.cpp:542-585
    def preprocess(self, viewMatrix, width, height, focal_x, focal_y, tan_fov_x, tan_fov_y, vpMatrix):
        u = make_uniforms(viewMatrix, width, height, focal_x, focal_y, tan_fov_x, tan_fov_y, vpMatrix)
        self._preprocess_u(u)

    def _preprocess_u(self, u: N.gs_uniforms):
        check(lib().gs_preprocess(self.ctx.handle, self._scene, ctypes.byref(u), self.flags, ctypes.byref(self._stats)),
              self.ctx.handle)
        self._sorted = False

    # src/Splats.cpp:346-354
    def sort(self):
        if getattr(self, "_sorted", False):
            return  # already sorted this frame (computeBins ran first)
        check(lib().gs_sort(self.ctx.handle), self.ctx.handle)
        self._sorted = True

    # src/Splats.cpp:481-512.  Tile ranges come from the sorted entries, so with the
    # reference's call order (computeBins before sort, src/Splats.cpp:593-594) sort runs first.
    def computeBins(self):
        self.sort()
        check(lib().gs_compute_bins(self.ctx.handle), self.ctx.handle)

    # src/Splats.cpp:356-381
    def draw(self, width: int, height: int, tileWidth: float, tileHeight: float):
        if width * height * 4 > self._texture.nbytes:
            self._texture = DeviceBuffer(self.ctx, width * height * 4)
        self.width, self.height = int(width), int(height)
        check(lib().gs_draw(self.ctx.handle, self._scene, int(width), int(height), float(tileWidth), float(tileHeight),
                            self.flags, self._texture.ptr, 1), self.ctx.handle)

    # src/Splats.cpp:587-597
    def gpuRender(self, viewMatrix, width, height, focal_x, focal_y, tan_fov_x, tan_fov_y, vpMatrix):
        u = make_uniforms(viewMatrix, width, height, focal_x, focal_y, tan_fov_x, tan_fov_y, vpMatrix)
        self.render_uniforms(u)

    def render_uniforms(self, u: N.gs_uniforms):
        """One frame into the back texture, which then becomes the texture (double buffering: a
        frame's blend need not wait for the previous frame's, gs_render orders blends per
        output only)."""
        nbytes = u.width * u.height * 4
        backs = getattr(self, "_backs", None)
        if backs is None:
            backs = self._backs = [None, None]  # a ring of three textures (one per frame lane)
        back = backs[0]  # the oldest texture
        if back is None or nbytes > back.nbytes:
            back = DeviceBuffer(self.ctx, max(nbytes, self._texture.nbytes))
        self.width, self.height = int(u.width), int(u.height)
        # no stats pointer: the frame is enqueued without a host round trip (gs_render)
        check(lib().gs_render(self.ctx.handle, self._scene, ctypes.byref(u), self.flags, back.ptr, 1, None),
              self.ctx.handle)
        self._backs = backs[1:] + [self._texture]
        self._texture = back

    def saveImage(self, filename: str, flip_y: bool = False):
        """saveImage (src/Splats.cpp:516-540) of the current texture: RGBA PNG, row 0 = GL row 0
        (flip_y=True: screen orientation)."""
        save_png(filename, self.texture(), flip_y)

    def texture(self) -> np.ndarray:
        """RGBA8 image (H, W, 4); row 0 = GL row 0 (bottom of the screen)."""
        return self._texture.download(np.uint8, self.width * self.height * 4).reshape(self.height, self.width, 4)

    def display(self) -> np.ndarray:
        """src/Splats.cpp:383-412 presents the texture with a y-flip (renderTexture.vert:11);
        headless: returns the top-down image."""
        return self.texture()[::-1]

    # frame-state readback (parity tests)
    def read(self, what: int, count: int, dtype=np.uint32) -> np.ndarray:
        out = np.empty(count, dtype=dtype)
        check(lib().gs_frame_read(self.ctx.handle, what, ptr(out), count), self.ctx.handle)
        return out
