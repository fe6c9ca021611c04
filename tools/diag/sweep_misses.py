"""Frames rendered again under bench.py's camera pans, counted over repeated runs: each run
starts cold (gs_ctx_set_sort_prefix clears the per-tile depths), renders the first pose alone,
then the 20 poses of the pan on three lanes (bench.py camera_sweep's prefix leg).
python tools/diag/sweep_misses.py [runs]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import openglgaussiansplattingrenderer_amd as g  # noqa: E402
from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw  # noqa: E402

W, H = 1920, 1080
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
ctx = g.Context(0)
sp = g.Splats.from_raw(*bicycle_standin_raw(), W, H, ctx=ctx)
base = ctx.set_sort_prefix()
for d in (0.5, 3.0):
    poses = []
    for k in range(20):
        cam = g.main_camera(W, H)
        cam.rotateRight(d * k)
        poses.append(cam.uniforms())
    redone, fps = [], []
    for _ in range(runs):
        ctx.set_sort_prefix(0)
        ctx.set_lanes(1)
        sp.render_uniforms(poses[0])
        ctx.sync()
        ctx.set_sort_prefix(base)
        sp.render_uniforms(poses[0])
        ctx.sync()
        ctx.set_lanes(3)
        ctx.prefix_stats(reset=True)
        t0 = time.perf_counter()
        for u in poses:
            sp.render_uniforms(u)
        ctx.sync()
        fps.append(len(poses) / (time.perf_counter() - t0))
        redone.append(ctx.prefix_stats()["redone"])
    print(f"{d} deg/frame: rendered again per run {redone} (total {sum(redone)} of {20 * runs} frames), "
          f"frames/s median {sorted(fps)[len(fps) // 2]:.0f}", flush=True)
ctx.close()
