"""Time the radix sort variants (hipEvents, median of R) and check them against numpy.
python tools/sortbench.py [R]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import openglgaussiansplattingrenderer_amd as g  # noqa: E402
from oracle import oracle as O  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 30
ctx = g.Context(0)
rng = np.random.default_rng(1)
cases = {
    "sortTests 5.12M f32 argsort": ("arg", O.gen_sort_keys(5_119_993)),
    "render-like 10M pairs": ("pairs", (rng.integers(0, 256, 10_000_000) + rng.random(10_000_000) * 0.03 + 0.96)
                              .astype(np.float32).view(np.uint32)),
    "uniform32 10M pairs": ("pairs", rng.integers(0, 2**32, 10_000_000, dtype=np.uint64).astype(np.uint32)),
}
for name, (kind, keys) in cases.items():
    n = len(keys)
    iota = np.arange(n, dtype=np.uint32)
    exp = np.argsort(keys.view(np.uint32), kind="stable")
    for algo in (0,):
        kb = g.DeviceBuffer.from_array(ctx, keys)
        vb = g.DeviceBuffer.from_array(ctx, iota)
        ms = []
        for r in range(R + 3):
            if kind == "arg":
                vb.upload(iota)
                g.GPURadixSort(1, 3, 2, None, vb, None, n, 16, 32, kb)
            else:
                kb.upload(keys)
                vb.upload(iota)
                g.sort_pairs(ctx, kb, vb, n)
            t = ctx.last_kernel_ms(g.GS_KERNEL_SORT)
            if r >= 3:
                ms.append(t)
        out = vb.download(np.uint32, n)
        ok = np.array_equal(out, exp)
        med = float(np.median(ms))
        print(f"{name:28s} algo {algo}: {med * 1e3:8.1f} us  {n / med / 1e6:6.1f} Gkeys/s  "
              f"68B/key -> {68 * n / (med * 1e-3) / 1e12:5.2f} TB/s  ok={ok}", flush=True)
