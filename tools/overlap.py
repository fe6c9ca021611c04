"""Frames of one view from C ctxs on one GPU, round robin, no sync between frames: does running
two frames' kernels concurrently (separate streams and buffers) raise throughput?
python tools/overlap.py [ctxs] [frames]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import openglgaussiansplattingrenderer_amd as g  # noqa: E402
from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 2
K = int(sys.argv[2]) if len(sys.argv) > 2 else 40
W, H = 1920, 1080
raw = bicycle_standin_raw()
ctxs = [g.Context(0) for _ in range(C)]
sps = [g.Splats.from_raw(*raw, W, H, ctx=c) for c in ctxs]
u = g.main_camera(W, H).uniforms()
for c in ctxs:
    c.timing_enable(0)
for rep in range(3):
    for k in range(10):
        sps[k % C].render_uniforms(u)
    for c in ctxs:
        c.sync()
    t0 = time.perf_counter()
    for k in range(K):
        sps[k % C].render_uniforms(u)
    for c in ctxs:
        c.sync()
    dt = time.perf_counter() - t0
    print(f"ctxs={C} frames={K}: {dt / K * 1e3:.4f} ms/frame  {K / dt:.1f} frames/s", flush=True)
img = [sp.texture() for sp in sps]
print("images equal across ctxs:", all((i == img[0]).all() for i in img))
