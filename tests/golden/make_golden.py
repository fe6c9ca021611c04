"""Generate the committed golden fixtures for the render path from the CPU oracle.

    python tests/golden/make_golden.py

C1: testSingleItem.ply (the reference's own fixture, copied here) at 256x256.
C2: 10,000 synthetic splats (tests/plyFileGenerator.py save_ply convention, seed
    20240101) at 512x512.
Both with the main.cpp:40-45 camera pose, in ref mode (flags 0) and clean mode (flags 1).
Each fixture stores the uniforms, the scene hash, V/D/E, the sorted keys/values, bins,
means2D, conics and the RGBA8 image the oracle produces.
"""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402


def uniforms_array(u):
    return np.array(list(u.view) + list(u.vp) + [u.width, u.height, u.focal_x, u.focal_y, u.tan_fov_x, u.tan_fov_y],
                    np.float64)


class U:
    """gs_uniforms-like object rebuilt from a fixture"""

    def __init__(self, a):
        self.view = [float(x) for x in a[0:16]]
        self.vp = [float(x) for x in a[16:32]]
        self.width, self.height = int(a[32]), int(a[33])
        self.focal_x, self.focal_y, self.tan_fov_x, self.tan_fov_y = (float(np.float32(x)) for x in a[34:38])


def scene_c1():
    return O.ply_load(os.path.join(HERE, "testSingleItem.ply"))


def scene_c2(tmpdir):
    import openglgaussiansplattingrenderer_amd as g
    from openglgaussiansplattingrenderer_amd.scenes import c2_scene
    path = os.path.join(tmpdir, "c2.ply")
    g.save_ply(path, *c2_scene())
    return O.ply_load(path)


def scene_hash(means, cols, op, sc, rot):
    return O.fnv1a64_words(np.concatenate([a.reshape(-1).view(np.uint32) for a in (means, cols, op, sc, rot)]))


def make(name, scene, W, H):
    import openglgaussiansplattingrenderer_amd as g
    means, cols, op, sc, rot = scene
    cov = O.cov3d(sc, rot)
    u = g.main_camera(W, H).uniforms()
    out = {"uniforms": uniforms_array(u), "scene_hash": np.uint64(scene_hash(means, cols, op, sc, rot))}
    for mode, flags in (("ref", 0), ("clean", 1)):
        r = O.render(means, cov, op, cols, u, flags=flags)
        for k in ("keys", "vals", "bins", "means2d", "conics", "image"):
            out[f"{mode}_{k}"] = r[k]
        out[f"{mode}_VDE"] = np.array([r["V"], r["D"], r["E"]], np.int64)
        print(name, mode, "V D E", r["V"], r["D"], r["E"], "nonzero px", int((r["image"][..., 3] > 0).sum()))
    np.savez_compressed(os.path.join(HERE, f"golden_{name}.npz"), **out)


def main():
    O.build()
    with tempfile.TemporaryDirectory() as td:
        make("c1", scene_c1(), 256, 256)
        make("c2", scene_c2(td), 512, 512)


if __name__ == "__main__":
    main()
