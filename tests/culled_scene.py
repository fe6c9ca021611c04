"""A scene whose last tile's Q10 window reaches the reference's culled entries (SURVEY Q10,
preprocess.glsl:80-88): splat 0 sits in the last non-empty tile, 300 splats are off-screen
(culled: key 1e6, drawn as splat 0), the rest fill the low tiles.  Shared by the oracle test
(the block changes pixels) and the GPU parity tests.

n_bulk > 0 adds that many wide splats (~120 px radius) in the upper-left quarter of the image,
each spanning ~40 coarse tiles, so the frame has millions of entries -- enough for the prefix sort
(E >= 64 x its 32768-entry target) -- while tile 255 keeps splat 0's short list, no key falls in
[256, 1e6) and every class from tile 255 on is kept whole (no prefix limit)."""
import numpy as np


def culled_scene(g, W=512, H=512, n_lo=600, n_culled=300, seed=3, n_bulk=0):
    u = g.main_camera(W, H).uniforms()
    VP = np.array(u.vp[:], np.float64).reshape(4, 4).T
    V = np.array(u.view[:], np.float64).reshape(4, 4).T
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
    if n_bulk:
        bm = world(rng.uniform(0, W / 2, n_bulk), rng.uniform(0, H * 0.4, n_bulk))
        depth = -(V @ np.c_[bm, np.ones(n_bulk)].T)[2]  # view-space distance
        sig = 40.0 * depth / u.focal_y                    # ~40 px: 3-sigma radius ~120 px
        means = np.concatenate([means, bm])
        rot = np.concatenate([rot, rng.normal(size=(n_bulk, 4)).astype(np.float32)])
        log_sc = np.concatenate([log_sc, np.repeat(np.log(sig)[:, None], 3, 1).astype(np.float32)])
        op = np.concatenate([op, rng.normal(-1.0, 1.0, n_bulk).astype(np.float32)])
        col = np.concatenate([col, rng.normal(size=(n_bulk, 3)).astype(np.float32)])
    return means, col, op, log_sc, rot, u
