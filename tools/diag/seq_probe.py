import os, sys, time
sys.path.insert(0, '/root/repo' if os.path.exists('/root/repo') else os.getcwd())
import openglgaussiansplattingrenderer_amd as g
from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw
W, H = 1920, 1080
ctx = g.Context(0)
sp = g.Splats.from_raw(*bicycle_standin_raw(), W, H, ctx=ctx)
base = ctx.set_sort_prefix()
ctx.set_lanes(3)
poses = []
for k in range(100):
    cam = g.main_camera(W, H); cam.rotateRight(3.0 * k); poses.append(cam.uniforms())
print("== sweep", file=sys.stderr, flush=True)
for u in poses: sp.render_uniforms(u)
ctx.sync()
print("== static pose 0", file=sys.stderr, flush=True)
ctx.set_sort_prefix(base)
t0 = time.perf_counter()
for i in range(70):
    sp.render_uniforms(poses[0])
ctx.sync()
print("static fps", 70 / (time.perf_counter() - t0), ctx.prefix_stats(), flush=True)
