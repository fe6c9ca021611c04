"""A scene whose last tile's Q10 window reaches the reference's culled entries (SURVEY Q10,
preprocess.glsl:80-88): splat 0 sits in the last non-empty tile, 300 splats are off-screen
(culled: key 1e6, drawn as splat 0), the rest fill the low tiles.  Shared by the oracle test
(the block changes pixels) and the GPU parity test."""
import numpy as np


def culled_scene(g, W=512, H=512, n_lo=600, n_culled=300, seed=3):
    u = g.main_camera(W, H).uniforms()
    VP = np.array(u.vp[:], np.float64).reshape(4, 4).T
    rng = np.random.default_rng(seed)

    def world(sx, sy, z=0.5):
        ndc = np.stack([2 * sx / W - 1, 2 * sy / H - 1, np.full(len(sx), z), np.ones(len(sx))], 1)
        w = (np.linalg.inv(VP) @ ndc.T).T
        return (w[:, :3] / w[:, 3:]).astype(np.float32)

    m0 = world(np.array([W - 20.0]), np.array([H - 20.0]))                    # splat 0: tile 255
    lo = world(rng.uniform(0, W / 2, n_lo), rng.uniform(0, H / 2, n_lo))      # tiles with low indices
    off = world(rng.uniform(1.5 * W, 2.5 * W, n_culled), rng.uniform(0, H, n_culled))  # culled (NDC x > 1)
    means = np.concatenate([m0, lo, off])
    n = len(means)
    rot = rng.normal(size=(n, 4)).astype(np.float32)
    log_sc = rng.uniform(np.log(0.01), np.log(0.05), (n, 3)).astype(np.float32)
    log_sc[0] = np.log(0.08)
    op = np.full(n, -2.5, np.float32)  # opacity ~0.076: many blends before saturation
    col = rng.normal(size=(n, 3)).astype(np.float32)
    return means, col, op, log_sc, rot, u
