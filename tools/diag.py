"""Diagnostics on the GPU box: per-stage times and blend work counters for the C3/C4 frames
in each mode.  python tools/diag.py [c3|c4] [frames] [mode,mode,...]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import openglgaussiansplattingrenderer_amd as g  # noqa: E402
from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 10
W, H = (1920, 1080) if cfg == "c3" else (3840, 2160)
ctx = g.Context(0)
t = time.time()
sp = g.Splats.from_raw(*bicycle_standin_raw(), W, H, ctx=ctx)
print(f"scene up in {time.time() - t:.1f}s", flush=True)
u = g.main_camera(W, H).uniforms()
variants = [("ref", 0), ("ref+fast", g.GS_FLAG_FAST_EXP), ("clean", g.GS_FLAG_CLEAN),
            ("clean+fast", g.GS_FLAG_CLEAN | g.GS_FLAG_FAST_EXP), ("nocull", g.GS_FLAG_NO_CULL)]
only = sys.argv[3].split(",") if len(sys.argv) > 3 else None
for name, fl in variants:
    if only and name not in only:
        continue
    sp.flags = fl | g.GS_FLAG_DRAW_STATS
    sp.render_uniforms(u)
    ctx.draw_stats(reset=True)
    sp.render_uniforms(u)
    st = ctx.draw_stats(reset=True)
    sp.flags = fl
    for _ in range(3):
        sp.render_uniforms(u)
    ctx.timing_enable(g.GS_TIMING_DRAW)  # wall time as bench.py measures it
    ctx.timing_reset()
    t0 = time.perf_counter()
    for _ in range(frames):
        sp.render_uniforms(u)
    ctx.sync()
    dt = (time.perf_counter() - t0) / frames * 1e3
    ctx.timing_enable(g.GS_TIMING_STAGES)  # stage breakdown from a second pass
    ctx.timing_reset()
    for _ in range(frames):
        sp.render_uniforms(u)
    tm = ctx.timing_read()
    nf = tm["frames"]
    s = " ".join(f"{k[3:]}={tm[k] / nf:.3f}" for k in ("ms_preprocess", "ms_emit", "ms_sort", "ms_bins", "ms_draw"))
    print(f"{name:11s} wall {dt:.3f} ms/frame  {s}  E={sp.stats.entries} draw: {st}", flush=True)
