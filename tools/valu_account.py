"""The blend's VALU account: where k_draw's vector instructions go at C3.
Dynamic counts from one GS_FLAG_DRAW_STATS frame (per-block trace: chunk steps, batches, dense /
sparse survivor steps with and without events, extra event passes, done-mask refreshes), times
the per-instance VALU of each code region read off the gfx950 listing of k_draw<false,false,false>
(tools/isa_blocks.py; profiles/r05/draw_isa_blocks.txt): the account sums to the SQ_INSTS_VALU
the counters measure (profiles/rNN/pmc_summary.json) within the listed bounds.
python tools/valu_account.py [c3|c4|vK]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import openglgaussiansplattingrenderer_amd as g  # noqa: E402
from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw  # noqa: E402

# per-instance VALU of k_draw<false,false,false> (isa_blocks.py block names of this build)
COST = {
    "chunk step (index load, box gather, box test, queue; loop tail)": 30,   # .LBB_51 19 + queue 4 + tail 7
    "batch (threshold, finite check, exact cull, gather issue)": 93,        # 28 + exact cull 61 + issue 4
    "dense step: broadcast, 4 powers (packed), need test": 29,               # .LBB_79
    "dense step with events: compaction, exp, blend, saturation": 42,        # ~9 + 20 + 12 + 1
    "dense extra event pass (> 64 events)": 30,                              # .LBB_91 17 + 12 + 1
    "done-mask refresh": 5,
    "sparse step: broadcast, power, need test": 19,                          # .LBB_71
    "sparse step with events: exp, blend": 34,                               # 17 + 12 + 5
    "block setup and epilogue (upper bound)": 400,
}


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    view = int(cfg[1:]) if cfg.startswith("v") else 0
    W, H = (3840, 2160) if cfg == "c4" else (1920, 1080)
    ctx = g.Context(0)
    sp = g.Splats.from_raw(*bicycle_standin_raw(), W, H, ctx=ctx)
    cam = g.main_camera(W, H)
    cam.rotateRight(45.0 * view)
    u = cam.uniforms()
    sp.flags = g.GS_FLAG_DRAW_STATS
    for _ in range(3):
        sp.render_uniforms(u)
    ctx.draw_stats(reset=True)
    sp.render_uniforms(u)
    ctx.draw_stats(reset=False)
    tr = ctx.draw_block_trace(65536).astype(np.int64)
    tr = tr[tr[:, 1] != 0]
    steps, kit, sparse = tr[:, 4].sum(), tr[:, 4].sum(), tr[:, 8].sum()
    dense = kit - sparse
    n = {
        "chunk step (index load, box gather, box test, queue; loop tail)": tr[:, 2].sum(),
        "batch (threshold, finite check, exact cull, gather issue)": tr[:, 15].sum(),
        "dense step: broadcast, 4 powers (packed), need test": dense,
        "dense step with events: compaction, exp, blend, saturation": tr[:, 12].sum(),
        "dense extra event pass (> 64 events)": tr[:, 13].sum(),
        "done-mask refresh": tr[:, 11].sum(),
        "sparse step: broadcast, power, need test": sparse,
        "sparse step with events: exp, blend": tr[:, 14].sum(),
        "block setup and epilogue (upper bound)": len(tr),
    }
    rows, tot = [], 0
    for k, c in COST.items():
        v = int(n[k]) * c
        tot += v
        rows.append((k, int(n[k]), c, v))
    pmc = None
    import glob
    for p in sorted(glob.glob(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                                           "r[0-9][0-9]", "pmc_summary.json")))[-1:]:
        pmc = (os.path.relpath(p), json.load(open(p)).get("k_draw", {}).get("sq", {}).get("SQ_INSTS_VALU"))
    print(f"{cfg}: {len(tr)} sub-blocks, {steps} survivor steps ({dense} dense, {sparse} sparse), "
          f"{tr[:, 6].sum()} pixel events")
    print(f"{'region':66s} {'count':>10s} {'VALU/inst':>9s} {'VALU':>12s} {'share':>6s}")
    for k, cnt, c, v in rows:
        print(f"{k:66s} {cnt:10d} {c:9d} {v:12.4g} {v / tot:6.1%}")
    print(f"{'account total':66s} {'':10s} {'':9s} {tot:12.4g}")
    if pmc and pmc[1]:
        print(f"measured SQ_INSTS_VALU per launch ({pmc[0]}): {pmc[1]:.4g}  (account / measured {tot / pmc[1]:.3f})")
    ctx.close()


if __name__ == "__main__":
    main()
