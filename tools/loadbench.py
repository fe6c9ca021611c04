"""Load time of a bicycle-sized ply (6,131,954 splats, 1.52 GB): the host path (ply parse +
activations + covariance on one host thread, then upload; what Splats(path) does, as the
reference does) against the GPU path (gs_scene_load_ply).  python tools/loadbench.py [n]"""
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import openglgaussiansplattingrenderer_amd as g  # noqa: E402
from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 6_131_954
means, f_dc, logit, log_scale, rot = bicycle_standin_raw(n)
cols, op, sc, rt = g.activate(f_dc, logit, log_scale, rot)
with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
    p = os.path.join(td, "bicycle_standin.ply")
    g.save_ply(p, means, rt, sc, op, f_dc)
    size = os.path.getsize(p)
    ctx = g.Context(0)
    for rep in range(2):  # second round: file in the page cache for both
        t0 = time.perf_counter()
        host = g.Splats(p, 1920, 1080, ctx=ctx)
        ctx.sync()
        t1 = time.perf_counter()
        dev = g.Splats(p, 1920, 1080, ctx=ctx, gpu_load=True)
        ctx.sync()
        t2 = time.perf_counter()
        same = all(np.array_equal(a.view(np.uint32), b.view(np.uint32)) for a, b in zip(host.download(), dev.download()))
        print(f"round {rep}: {n} splats, {size / 1e9:.2f} GB ply: host path {t1 - t0:.2f} s, "
              f"GPU path {t2 - t1:.2f} s ({size / (t2 - t1) / 1e9:.2f} GB/s), identical scenes: {same}", flush=True)
        del host, dev
