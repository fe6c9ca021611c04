"""Blend-work diagnostics of the C5 views on the GPU box: tile list lengths (bins), and the
per-block trace of a GS_FLAG_DRAW_STATS draw (duration, iterations, survivors, list entries).
python tools/view_diag.py [view ...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import openglgaussiansplattingrenderer_amd as g  # noqa: E402
from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw  # noqa: E402

W, H = 1920, 1080
ctx = g.Context(0)
sp = g.Splats.from_raw(*bicycle_standin_raw(), W, H, ctx=ctx)
views = [int(v) for v in sys.argv[1:]] or [4]
for v in views:
    cam = g.main_camera(W, H)
    cam.rotateRight(45.0 * v)
    u = cam.uniforms()
    sp.flags = 0
    sp.render_uniforms(u)
    sp.render_uniforms(u)
    bins = sp.read(g.GS_READ_BINS, 256).astype(np.int64)
    cnt = np.diff(np.concatenate([[0], bins[:256]]))
    sp.flags = g.GS_FLAG_DRAW_STATS
    sp.render_uniforms(u)
    ctx.draw_stats(reset=True)
    sp.render_uniforms(u)
    st = ctx.draw_stats(reset=True)
    tr = ctx.draw_block_trace(65536)
    dur = (tr[:, 1].astype(np.int64) - tr[:, 0].astype(np.int64)) & 0xffffffff
    t0 = tr[:, 0].astype(np.int64).min()
    end = ((tr[:, 1].astype(np.int64) - t0) & 0xffffffff)
    q = lambda a: np.percentile(a, [50, 90, 99, 100]).round(1).tolist()
    print(f"view {v}: E={sp.stats.entries} tiles: nonempty {int((cnt > 0).sum())} list len pct50/90/99/max {q(cnt)}")
    print(f"  blocks {len(tr)} dur us pct {q(dur / 100.0)} span us {end.max() / 100.0:.1f}")
    print(f"  iterations pct {q(tr[:, 2])} survivors pct {q(tr[:, 3])} list entries pct {q(tr[:, 7])}")
    top = np.argsort(-dur)[:8]
    for b in top:
        print(f"   block {b}: dur {dur[b] / 100:.1f} us it {tr[b, 2]} surv {tr[b, 3]} steps {tr[b, 4]} list {tr[b, 7]} start {((tr[b, 0] - t0) & 0xffffffff) / 100:.1f}")
    print(f"  stats {st}", flush=True)
