"""Deterministic synthetic scenes for the benchmark configs (BASELINE.md section 2,
SURVEY 8(d)).  Raw fields are generated as the float32 values a .ply would hold, so
``Splats.from_raw`` is bit-identical to writing them into a ply and loading it.

C2: 10,000 splats in tests/plyFileGenerator.py's save_ply convention (activated opacity /
    scale / raw colour written by the writer), seed 20240101.
C3: a seeded synthetic stand-in for the bicycle point_cloud.ply (6,131,954 splats) --
    labelled synthetic; the real file is used when $GS_BICYCLE_PLY points at it.
"""
from __future__ import annotations

import numpy as np

BICYCLE_N = 6_131_954


def c2_scene(n: int = 10_000, seed: int = 20240101):
    """save_ply inputs: means (n,3), rotations (n,4), scales (n,3), opacities (n,), colours (n,3)"""
    rng = np.random.default_rng(seed)
    means = rng.uniform(-2.0, 2.0, size=(n, 3)).astype(np.float32)
    log_scale = rng.uniform(np.log(0.01), np.log(0.2), size=(n, 3))
    scales = np.exp(log_scale).astype(np.float32)
    q = rng.normal(size=(n, 4))
    rotations = (q / np.linalg.norm(q, axis=1, keepdims=True)).astype(np.float32)
    opacities = rng.uniform(0.05, 0.99, size=n).astype(np.float32)
    colours = rng.normal(size=(n, 3)).astype(np.float32)  # f_dc
    return means, rotations, scales, opacities, colours


def bicycle_standin_raw(n: int = BICYCLE_N, seed: int = 6131954):
    """raw ply fields (means3, f_dc3, opacity_logit, log_scale3, rot_raw4) of the C3 stand-in:
    70% of means in a dense central object N(0, 0.7^2)^3, 30% on a background shell of radius
    U[5, 30]; log-scale N(-4.6, 1) clipped to [-9, 0.5]; opacity logit N(0, 3^2);
    f_dc N(0, 0.8^2); quaternion N(0,1)^4 (normalised by the loader)."""
    rng = np.random.default_rng(seed)
    n_obj = int(round(0.7 * n))
    n_sh = n - n_obj
    means = np.empty((n, 3), np.float32)
    means[:n_obj] = rng.normal(0.0, 0.7, size=(n_obj, 3)).astype(np.float32)
    d = rng.normal(size=(n_sh, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = rng.uniform(5.0, 30.0, size=(n_sh, 1))
    means[n_obj:] = (d * r).astype(np.float32)
    log_scale = np.clip(rng.normal(-4.6, 1.0, size=(n, 3)), -9.0, 0.5).astype(np.float32)
    opacity_logit = rng.normal(0.0, 3.0, size=n).astype(np.float32)
    f_dc = rng.normal(0.0, 0.8, size=(n, 3)).astype(np.float32)
    rot = rng.normal(size=(n, 4)).astype(np.float32)
    return means, f_dc, opacity_logit, log_scale, rot


def write_raw_ply(path: str, means3, f_dc3, opacity_logit, log_scale3, rot_raw4, f_rest45=None):
    """a ply of raw (pre-activation) fields in the tests/plyFileGenerator.py layout (x y z, nx ny nz,
    f_dc_0..2, f_rest_0..44, opacity, scale_0..2, rot_0..3): what loadSplats reads and activates,
    so Splats(path, W, H) equals Splats.from_raw(the same fields) bit for bit"""
    means3 = np.asarray(means3, np.float32).reshape(-1, 3)
    n = len(means3)
    hdr = ("ply\nformat binary_little_endian 1.0\nelement vertex %d\n" % n +
           "".join(f"property float {p}\n" for p in ["x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"]) +
           "".join(f"property float f_rest_{k}\n" for k in range(45)) +
           "property float opacity\nproperty float scale_0\nproperty float scale_1\nproperty float scale_2\n"
           "property float rot_0\nproperty float rot_1\nproperty float rot_2\nproperty float rot_3\nend_header\n")
    with open(path, "wb") as f:
        f.write(hdr.encode())
        step = 1 << 20
        for a in range(0, n, step):
            b = min(n, a + step)
            rec = np.zeros((b - a, 62), np.float32)
            rec[:, 0:3] = means3[a:b]
            rec[:, 6:9] = np.asarray(f_dc3, np.float32).reshape(-1, 3)[a:b]
            if f_rest45 is not None:
                rec[:, 9:54] = np.asarray(f_rest45, np.float32).reshape(-1, 45)[a:b]
            rec[:, 54] = np.asarray(opacity_logit, np.float32).reshape(-1)[a:b]
            rec[:, 55:58] = np.asarray(log_scale3, np.float32).reshape(-1, 3)[a:b]
            rec[:, 58:62] = np.asarray(rot_raw4, np.float32).reshape(-1, 4)[a:b]
            f.write(rec.tobytes())
