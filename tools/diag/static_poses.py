"""Diagnostic: frames/s of single poses of the camera sweep rendered without motion (the bench's
static_same_poses_fps, per pose), with the prefix-sort counters of each.
  python tools/diag/static_poses.py [deg] [frames]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import openglgaussiansplattingrenderer_amd as g  # noqa: E402
from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw  # noqa: E402

deg = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
W, H = 1920, 1080
ctx = g.Context(0)
sp = g.Splats.from_raw(*bicycle_standin_raw(), W, H, ctx=ctx)
base = ctx.set_sort_prefix()
ctx.set_lanes(3)
for k in sorted({0, (steps - 1) // 4, (steps - 1) // 2, 3 * (steps - 1) // 4, steps - 1}):
    cam = g.main_camera(W, H)
    cam.rotateRight(deg * k)
    u = cam.uniforms()
    ctx.set_sort_prefix(base)
    for _ in range(10):
        sp.render_uniforms(u)
    ctx.sync()
    ctx.prefix_stats(reset=True)
    t0 = time.perf_counter()
    for _ in range(60):
        sp.render_uniforms(u)
    ctx.sync()
    dt = time.perf_counter() - t0
    print(f"pose {k} ({deg * k:.1f} deg): {60 / dt:.1f} frames/s E {sp.stats.entries} prefix {ctx.prefix_stats()}",
          flush=True)
