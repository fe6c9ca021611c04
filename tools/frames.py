"""Render K frames of a config with given flags / draw_q (for rocprofv3 runs).
python tools/frames.py c3 FLAGS Q K"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import openglgaussiansplattingrenderer_amd as g  # noqa: E402
from openglgaussiansplattingrenderer_amd._native import GS_PARAM_DRAW_Q  # noqa: E402
from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw  # noqa: E402

cfg, flags, q, k = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
W, H = (1920, 1080) if cfg == "c3" else (3840, 2160)
ctx = g.Context(0)
ctx.set_param(GS_PARAM_DRAW_Q, q)
sp = g.Splats.from_raw(*bicycle_standin_raw(), W, H, ctx=ctx, flags=flags)
u = g.main_camera(W, H).uniforms()
for _ in range(k):
    sp.render_uniforms(u)
ctx.sync()
