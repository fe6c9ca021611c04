"""Two frames in flight: one ctx with 2 lanes vs 2 ctxs with 1 lane each; host enqueue time per
frame.  python tools/overlap2.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import openglgaussiansplattingrenderer_amd as g  # noqa: E402
from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw  # noqa: E402

W, H, K = 1920, 1080, 40
raw = bicycle_standin_raw()
u = g.main_camera(W, H).uniforms()


def run(sps, ctxs, label, tmode=0):
    for c in ctxs:
        c.timing_enable(tmode)
    for rep in range(2):
        for k in range(8):
            sps[k % len(sps)].render_uniforms(u)
        for c in ctxs:
            c.sync()
        enq = []
        t0 = time.perf_counter()
        for k in range(K):
            a = time.perf_counter()
            sps[k % len(sps)].render_uniforms(u)
            enq.append(time.perf_counter() - a)
        for c in ctxs:
            c.sync()
        dt = time.perf_counter() - t0
        print(f"{label} timing={tmode}: {dt / K * 1e3:.4f} ms/frame; host enqueue per frame median "
              f"{np.median(enq) * 1e3:.4f} ms, first 4: {[round(x * 1e3, 3) for x in enq[:4]]}", flush=True)


c1 = g.Context(0)
s1 = g.Splats.from_raw(*raw, W, H, ctx=c1)
for lanes in (1, 2):
    c1.set_lanes(lanes)
    run([s1], [c1], f"1 ctx, {lanes} lane(s)")
    run([s1], [c1], f"1 ctx, {lanes} lane(s)", 1)
c2 = g.Context(0)
s2 = g.Splats.from_raw(*raw, W, H, ctx=c2)
c1.set_lanes(1)
c2.set_lanes(1)
run([s1, s2], [c1, c2], "2 ctxs x 1 lane")
c1.set_lanes(2)
c2.set_lanes(2)
run([s1, s2], [c1, c2], "2 ctxs x 2 lanes")
