"""Independent float64 numpy restatement of the reference's GPU shaders, used to check the
C oracle (which is float32, glm operator order).  Written from the GLSL directly with
ordinary matrix algebra -- it shares no code with oracle/gs_oracle.c.

  preprocess   shaders/preprocess.glsl:64-190
  draw         shaders/draw.glsl:70-143 (+ countBins/prefixBins, sort by key)
"""
from __future__ import annotations

import numpy as np


def glm(m16) -> np.ndarray:
    """column-major float[16] -> ordinary 4x4 matrix M[row, col]"""
    return np.array(m16, np.float64).reshape(4, 4).T


def preprocess(means4, cov6, opacity, u, clean=False):
    n = len(opacity)
    V = glm(u.view[:])
    VP = glm(u.vp[:])
    W, H = int(u.width), int(u.height)
    m = np.asarray(means4, np.float64).copy()
    m[:, 3] = 1.0
    p = m @ VP.T
    w = np.maximum(p[:, 3], 1e-4)
    p = p / w[:, None]
    culled = (p[:, 0] < -1) | (p[:, 0] > 1) | (p[:, 1] < -1) | (p[:, 1] > 1)
    sx = (p[:, 0] + 1) * 0.5 * W
    sy = (p[:, 1] + 1) * 0.5 * H
    z01 = (p[:, 2] + 1) * 0.5
    t = m @ V.T
    tx, ty, tz = t[:, 0].copy(), t[:, 1].copy(), t[:, 2].copy()
    limx, limy = -1.3 * u.tan_fov_x, -1.3 * u.tan_fov_y
    tx = np.minimum(limx, np.maximum(-limx, tx / tz)) * tz
    ty = np.minimum(limy, np.maximum(-limy, ty / tz)) * tz
    c = np.asarray(cov6, np.float64).reshape(n, 6)
    Sig = np.stack([c[:, [0, 1, 2]], c[:, [1, 3, 4]], c[:, [2, 4, 5]]], axis=1)
    # GLSL mat3(...) is column-major: J as a math matrix has rows (fx/tz,0,0),(0,fy/tz,0),
    # (-fx tx/tz^2, -fy ty/tz^2, 0)
    J = np.zeros((n, 3, 3))
    J[:, 0, 0] = u.focal_x / tz
    J[:, 1, 1] = u.focal_y / tz
    J[:, 2, 0] = -(u.focal_x * tx) / (tz * tz)
    J[:, 2, 1] = -(u.focal_y * ty) / (tz * tz)
    W3 = V[:3, :3]  # math matrix of mat3(viewMatrix)
    T = W3.T[None] @ J
    C = np.transpose(T, (0, 2, 1)) @ np.transpose(Sig, (0, 2, 1)) @ T
    a = C[:, 0, 0] + 0.3
    b = C[:, 1, 0]  # covariance2D[0][1] = column 0, row 1
    cc = C[:, 1, 1] + 0.3
    det = a * cc - b * b
    conic = np.stack([cc / det, -b / det, a / det], axis=1)
    mid = (cc + a) * 0.5
    l1 = mid + np.sqrt(np.maximum(0.1, mid * mid - det))
    l2 = mid - np.sqrt(np.maximum(0.1, mid * mid - det))
    radius = np.ceil(3 * np.sqrt(np.maximum(l1, l2)))
    return dict(culled=culled, sx=sx, sy=sy, z01=z01, conic=conic, det=det, radius=radius)


def draw(W, H, vals_sorted, bins, means2d, conic4, colours4, clean=False, E=None, keys_sorted=None, culled=0):
    """per-pixel front-to-back blend in float64 (no quirks beyond Q9/Q10 of ref mode, and the
    culled splats' 1e6 entries that a Q10 window can reach: given keys_sorted and the number of
    culled splats, they are placed -- as splat 0 -- after the non-negative keys <= 1e6)"""
    vals_sorted = np.asarray(vals_sorted)[: (len(vals_sorted) if E is None else E)]
    if not clean and culled and keys_sorted is not None:
        kf = np.asarray(keys_sorted[: len(vals_sorted)], np.uint32).view(np.float32)
        P = int(np.count_nonzero(~np.signbit(kf) & (kf <= 1e6)))
        vals_sorted = np.concatenate([vals_sorted[:P], np.zeros(culled, vals_sorted.dtype), vals_sorted[P:]])
    E = len(vals_sorted)
    tw, th = W / 16.0, H / 16.0
    cw = W if clean else (W // 32) * 32
    ch = H if clean else (H // 32) * 32
    img = np.zeros((H, W, 4), np.float64)
    m2 = means2d.reshape(-1, 2).astype(np.float64)
    co = conic4.reshape(-1, 4).astype(np.float64)
    cl = colours4.reshape(-1, 4).astype(np.float64)
    for y in range(ch):
        for x in range(cw):
            t = int(y / th) * 16 + int(x / tw)
            start = 0 if t == 0 else int(bins[t - 1])
            end = int(bins[t])
            if not clean and end > start:
                end = min(E, start + ((end - start + 1023) // 1024) * 1024)
            if end <= start:
                continue
            s = vals_sorted[start:end]
            dx = x - m2[s, 0]
            dy = y - m2[s, 1]
            pw = -0.5 * (co[s, 0] * dx * dx + co[s, 2] * dy * dy) - co[s, 1] * dx * dy
            alpha = np.minimum(0.99, np.exp(np.minimum(pw, 0)) * co[s, 3])
            ok = (pw <= 0) & (alpha >= 1 / 255)
            col = np.zeros(4)
            for k in np.nonzero(ok)[0]:
                aT = alpha[k] * (1 - col[3])
                col[:3] += cl[s[k], :3] * aT
                col[3] += aT
                if col[3] >= 0.99:
                    break
            img[y, x] = col
    out = np.clip(img / 255.0, 0, 1)
    return np.floor(out * 255 + 0.5).astype(np.uint8)
