"""Static-camera prefix frames in phases (ref mode, clean mode, ref mode again, each after a
synchronous frame): prefix frames, frames rendered again and the newest kept count per phase,
and whether every image equals the synchronous frame's.  Run with a GS_PREFIX_TRACE build for
the per-frame miss lines.  python tools/diag/kept_miss.py [frames]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import openglgaussiansplattingrenderer_amd as g  # noqa: E402
from openglgaussiansplattingrenderer_amd import _native as N  # noqa: E402
from openglgaussiansplattingrenderer_amd._native import check, lib  # noqa: E402
from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw  # noqa: E402

W, H = 1920, 1080
frames = int(sys.argv[1]) if len(sys.argv) > 1 else 6
ctx = g.Context(0)
sp = g.Splats.from_raw(*bicycle_standin_raw(), W, H, ctx=ctx)
u = g.main_camera(W, H).uniforms()
ref = g.DeviceBuffer(ctx, W * H * 4)
outs = [g.DeviceBuffer(ctx, W * H * 4) for _ in range(frames)]
ctx.set_sort_prefix()
for phase, flags in enumerate([0, g.GS_FLAG_CLEAN, 0, g.GS_FLAG_CLEAN]):
    sp.flags = flags
    st = N.gs_frame_stats()
    check(lib().gs_render(ctx.handle, sp._scene, ctypes.byref(u), flags, ref.ptr, 1, ctypes.byref(st)), ctx.handle)
    img = ref.download(np.uint8, W * H * 4)
    ctx.prefix_stats(reset=True)
    print(f"phase {phase} flags {flags}: sync frame done", file=sys.stderr, flush=True)
    for k in range(frames):
        check(lib().gs_render(ctx.handle, sp._scene, ctypes.byref(u), flags, outs[k].ptr, 1, None), ctx.handle)
    ctx.sync()
    ps = ctx.prefix_stats()
    same = []
    for k, o in enumerate(outs):
        a = o.download(np.uint8, W * H * 4).reshape(H, W, 4)
        b = img.reshape(H, W, 4)
        bad = np.argwhere((a != b).any(axis=2))
        same.append(len(bad) == 0)
        if len(bad):
            tiles = sorted({(int(x * 16 // W), int(y * 16 // H)) for y, x in bad})
            print(f"  frame {k}: {len(bad)} pixels differ, tiles (x, y) {tiles[:12]}{' ...' if len(tiles) > 12 else ''}",
                  flush=True)
    print(f"phase {phase} flags {flags}: {ps} images equal {all(same)}", flush=True)
ctx.close()
