"""Diagnostic: a 3 deg/frame camera sweep with the prefix sort, then 70 static frames of its first
pose -- the prefix bookkeeping of the static frames after a sweep (run on a GS_PREFIX_TRACE build:
the per-frame trace goes to stderr).
  python tools/diag/seq_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import openglgaussiansplattingrenderer_amd as g  # noqa: E402
from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw  # noqa: E402

W, H = 1920, 1080
ctx = g.Context(0)
sp = g.Splats.from_raw(*bicycle_standin_raw(), W, H, ctx=ctx)
base = ctx.set_sort_prefix()
ctx.set_lanes(3)
poses = []
for k in range(100):
    cam = g.main_camera(W, H)
    cam.rotateRight(3.0 * k)
    poses.append(cam.uniforms())
print("== sweep", file=sys.stderr, flush=True)
for u in poses:
    sp.render_uniforms(u)
ctx.sync()
print("== static pose 0", file=sys.stderr, flush=True)
ctx.set_sort_prefix(base)
t0 = time.perf_counter()
for _ in range(70):
    sp.render_uniforms(poses[0])
ctx.sync()
print("static frames/s", 70 / (time.perf_counter() - t0), ctx.prefix_stats(), flush=True)
