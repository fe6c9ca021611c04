"""Diagnostic: the 0.5 deg/frame camera sweep (bench.py camera_sweep's poses) with the prefix sort,
printing per-frame prefix bookkeeping from a GS_PREFIX_TRACE build (stderr) -- which frames miss
(a blend reached an unsorted position) or overflow their kept capacity, and when the cooldown runs.
  tools/variants.sh trace -DGS_PREFIX_TRACE && cp .../variants/trace.so .../libgsplat_hip.so
  python tools/diag/prefix_sweep.py [deg] [frames]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import openglgaussiansplattingrenderer_amd as g  # noqa: E402
from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw  # noqa: E402

deg = float(sys.argv[1]) if len(sys.argv) > 1 else 0.5
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 100
W, H = 1920, 1080
ctx = g.Context(0)
sp = g.Splats.from_raw(*bicycle_standin_raw(), W, H, ctx=ctx)
poses = []
for k in range(frames):
    cam = g.main_camera(W, H)
    cam.rotateRight(deg * k)
    poses.append(cam.uniforms())
base = ctx.set_sort_prefix()
ctx.set_sort_prefix(0)
sp.render_uniforms(poses[0])
ctx.sync()
ctx.set_sort_prefix(base)
ctx.set_lanes(3)
ctx.prefix_stats(reset=True)
for k, u in enumerate(poses):
    print(f"frame {k}", file=sys.stderr, flush=True)
    sp.render_uniforms(u)
ctx.sync()
print(ctx.prefix_stats(), flush=True)
