"""Per-block timeline of one draw (GS_FLAG_DRAW_STATS): how long the sub-blocks run, how many
are resident over time, and whether the kernel's span is set by a few long blocks.
python tools/timeline.py [c2|c3|c4] [flags]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import openglgaussiansplattingrenderer_amd as g  # noqa: E402
from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
flags = int(sys.argv[2]) if len(sys.argv) > 2 else 0
view = int(cfg[1:]) if cfg.startswith("v") else 0  # vK: C5 pose K at 1080p
W, H = {"c2": (512, 512), "c3": (1920, 1080)}.get(cfg, (1920, 1080) if view or cfg == "v0" else (3840, 2160))
ctx = g.Context(0)
if cfg == "c2":
    from openglgaussiansplattingrenderer_amd.scenes import c2_scene
    means, rot, sc, op, col = c2_scene()
    sp = g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, W, H, ctx=ctx)
else:
    sp = g.Splats.from_raw(*bicycle_standin_raw(), W, H, ctx=ctx)
cam = g.main_camera(W, H)
cam.rotateRight(45.0 * view)
u = cam.uniforms()
# GS_LIGHT_TRACE=1 (environment): GS_FLAG_DRAW_TRACE -- per-block times and counts only (the full
# per-survivor counters about double the blend's span)
light = bool(os.environ.get("GS_LIGHT_TRACE"))
sp.flags = flags | g.GS_FLAG_DRAW_STATS | (g.GS_FLAG_DRAW_TRACE if light else 0)
for _ in range(3):
    sp.render_uniforms(u)
ctx.draw_stats(reset=True)
sp.render_uniforms(u)
st = ctx.draw_stats(reset=False)
tr = ctx.draw_block_trace(65536).astype(np.int64)
if len(sys.argv) > 3:  # save the raw trace and the bins (tile order) for offline analysis
    np.savez(sys.argv[3], trace=tr, bins=sp.read(g.GS_READ_BINS, 256))
live = tr[:, 1] != 0
tr = tr[live]
t0 = tr[:, 0].min()
s, e = (tr[:, 0] - t0) * 0.01, (tr[:, 1] - t0) * 0.01  # us
d = e - s
print(f"{cfg} flags={flags} blocks={len(tr)} span={e.max():.1f} us  start spread={s.max():.1f} us")
print("block duration us: " + " ".join(f"p{p}={np.percentile(d, p):.1f}" for p in (10, 50, 90, 99, 100)))
print("iterations: " + " ".join(f"p{p}={np.percentile(tr[:, 2], p):.0f}" for p in (50, 90, 99, 100)) +
      "  survivors: " + " ".join(f"p{p}={np.percentile(tr[:, 3], p):.0f}" for p in (50, 90, 99, 100)))
grid = np.linspace(0, e.max(), 21)
act = [int(((s <= x) & (e > x)).sum()) for x in grid[:-1]]
print("resident blocks at 5% steps:", act)
o = np.argsort(-d)[:8]
for i in o:
    print(f"  long block: {d[i]:.1f} us start {s[i]:.1f} iters {tr[i, 2]} surv {tr[i, 3]}")
A = np.stack([tr[:, 2], tr[:, 3], np.ones(len(tr))], 1).astype(float)
coef, *_ = np.linalg.lstsq(A, d, rcond=None)
print(f"duration ~ {coef[0]:.3f} us/iteration + {coef[1]:.3f} us/survivor + {coef[2]:.1f} us")
# event passes: a survivor with k needing pixels runs ceil(k/64) passes; per block only the sum
A = np.stack([tr[:, 2], tr[:, 5], tr[:, 6] / 64.0, np.ones(len(tr))], 1).astype(float)
coef, *_ = np.linalg.lstsq(A, d, rcond=None)
res = d - A @ coef
print(f"duration ~ {coef[0]:.3f} us/iteration + {coef[1]:.3f} us/needing survivor + {coef[2]:.3f} us/64 events"
      f" + {coef[3]:.1f} us  (residual rms {res.std():.1f} us)")
for lo, hi in ((0, 25), (25, 50), (50, 75), (75, 100)):
    m = (s >= np.percentile(s, lo)) & (s <= np.percentile(s, hi))
    print(f"  start pct {lo}-{hi}: mean dur {d[m].mean():.1f} us  iters {tr[m, 2].mean():.1f}  need-surv {tr[m, 5].mean():.1f}"
          f"  events {tr[m, 6].mean():.0f}")
for i in o:
    print(f"  long block {i}: {d[i]:.1f} us  steps {tr[i, 4]} needing {tr[i, 5]} events {tr[i, 6]} entries {tr[i, 7]}")
short = np.argsort(d)[:5]
for i in short:
    print(f"  short block {i}: {d[i]:.1f} us  start {s[i]:.1f} iters {tr[i, 2]} surv {tr[i, 3]} events {tr[i, 6]}")
k64, k128, ev64, refr = tr[:, 8].sum(), tr[:, 9].sum(), tr[:, 10].sum(), tr[:, 11].sum()
if tr[:, 4].sum() == 0:  # a light trace (GS_LIGHT_TRACE): times, list steps and survivors only
    print("per-survivor counters not recorded (light trace)")
else:
    ns, ne = tr[:, 4].sum(), max(1, tr[:, 6].sum())
    print(f"survivor steps {ns}: with <=64 active px {k64} ({k64 / ns:.1%}), <=128 {k128}"
          f" ({k128 / ns:.1%}); events with <=64 active {ev64} ({ev64 / ne:.1%})")
    print(f"done-mask refreshes (a pixel saturated): {refr} ({refr / max(1, tr[:, 12:15].sum()):.2f} per dense step)")
    a192, a128, a64, dev = (tr[:, k].sum() for k in (12, 13, 14, 15))
    nd = max(1, a192 + a128 + a64)
    print(f"dense steps {a192 + a128 + a64}: >192 active {a192} ({a192 / nd:.1%}), 129-192 {a128} ({a128 / nd:.1%}), "
          f"65-128 {a64} ({a64 / nd:.1%}); events per dense step {dev / nd:.1f}")
print("counters:", st)
