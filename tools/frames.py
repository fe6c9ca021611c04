"""Render K frames of a config with given flags (for rocprofv3 runs).
python tools/frames.py c3 FLAGS K [LANES]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import openglgaussiansplattingrenderer_amd as g  # noqa: E402
from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw  # noqa: E402

cfg, flags, k = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
W, H = (1920, 1080) if cfg == "c3" else (3840, 2160)
ctx = g.Context(0)
if len(sys.argv) > 4:
    ctx.set_lanes(int(sys.argv[4]))
sp = g.Splats.from_raw(*bicycle_standin_raw(), W, H, ctx=ctx, flags=flags)
u = g.main_camera(W, H).uniforms()
for _ in range(k):
    sp.render_uniforms(u)
ctx.sync()
