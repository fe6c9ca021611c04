"""probe: which depth-range scenes keep a cut prefix without misses (test design aid)"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import openglgaussiansplattingrenderer_amd as g
from tests.test_gpu_render import depth_range_scene
for W, H in [(512, 512), (1920, 1080)]:
    for ls, ob in [(-4.5, 4.0), (-3.5, 4.0), (-2.5, 4.0), (-2.5, 6.0)]:
        for target in (1024, 4096):
            ctx = g.Context(0)
            ctx.set_small_limits(-1, 0)
            ctx.set_sort_prefix(target)
            u = g.main_camera(W, H).uniforms()
            sp = g.Splats.from_raw(*depth_range_scene(u, 80_000, log_scale=ls, opacity_bias=ob), W, H, ctx=ctx)
            res = []
            for f in range(6):
                sp.render_uniforms(u)
                ctx.sync()
                ps = ctx.prefix_stats()
                res.append((ps["frames"], ps["redone"], ps["kept"], ps["entries"]))
            print(W, ls, ob, target, res, flush=True)
            ctx.close()
