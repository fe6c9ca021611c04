"""SURVEY f3 (beyond the reference): view-dependent colour from degree-3 SH (GS_FLAG_SH).
CPU: the ply's raw SH fields round-trip through gs_ply_load_sh.  GPU: frames are bit-exact
against the oracle's SH colours rendered by the oracle; with f_rest = 0 the SH path gives the
reference's colour (image identical to the default path)."""
import os

import numpy as np
import pytest

import openglgaussiansplattingrenderer_amd as g
from openglgaussiansplattingrenderer_amd.scenes import c2_scene


def write_ply_with_sh(path, means, f_dc, f_rest, logit, log_scale, rot):
    """ply in the tests/plyFileGenerator.py layout with nonzero f_rest"""
    n = len(means)
    hdr = ("ply\nformat binary_little_endian 1.0\nelement vertex %d\n" % n +
           "".join(f"property float {p}\n" for p in ["x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"]) +
           "".join(f"property float f_rest_{k}\n" for k in range(45)) +
           "property float opacity\nproperty float scale_0\nproperty float scale_1\nproperty float scale_2\n"
           "property float rot_0\nproperty float rot_1\nproperty float rot_2\nproperty float rot_3\nend_header\n")
    rec = np.zeros((n, 62), np.float32)
    rec[:, 0:3] = means
    rec[:, 6:9] = f_dc
    rec[:, 9:54] = f_rest
    rec[:, 54] = logit
    rec[:, 55:58] = log_scale
    rec[:, 58:62] = rot
    with open(path, "wb") as f:
        f.write(hdr.encode())
        f.write(rec.tobytes())


def sh_scene(n=10000, seed=7):
    means, rot, sc, op, col = c2_scene(n)
    rng = np.random.default_rng(seed)
    f_rest = rng.normal(0, 0.3, (n, 45)).astype(np.float32)
    return means, col, f_rest, np.log(op / (1 - op)).astype(np.float32), np.log(sc).astype(np.float32), rot


def test_ply_sh_roundtrip(tmp_path):
    means, f_dc, f_rest, logit, log_scale, rot = sh_scene(300)
    p = str(tmp_path / "sh.ply")
    write_ply_with_sh(p, means, f_dc, f_rest, logit, log_scale, rot)
    d, r = g.load_ply_sh(p, 300)
    assert np.array_equal(d, f_dc) and np.array_equal(r, f_rest)


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, g.GS_FLAG_CLEAN])
def test_sh_frame_matches_oracle(tmp_path, flags):
    from oracle import oracle as O
    O.build()
    W, H = 512, 384
    ctx = g.Context(0)
    means, f_dc, f_rest, logit, log_scale, rot = sh_scene()
    p = str(tmp_path / "sh.ply")
    write_ply_with_sh(p, means, f_dc, f_rest, logit, log_scale, rot)
    sp = g.Splats(p, W, H, ctx=ctx, sh=True)
    u = g.main_camera(W, H).uniforms()
    sp.flags = flags | g.GS_FLAG_SH
    sp.render_uniforms(u)
    img = sp.texture()
    cols = O.sh_colours(sp.means3D, f_dc, f_rest, np.array(u.view, np.float32), np.ones(sp.numSplats, np.uint8),
                        sp.colours)
    ref = O.render(sp.means3D, sp.covarianceMatrices, sp.opacities, cols, u, flags=flags, stages=False)
    assert np.array_equal(img.reshape(-1), ref["image"].reshape(-1))
    # view dependence: another pose changes colours, still bit-exact
    cam = g.main_camera(W, H)
    cam.rotateRight(15.0)
    u2 = cam.uniforms()
    sp.render_uniforms(u2)
    cols2 = O.sh_colours(sp.means3D, f_dc, f_rest, np.array(u2.view, np.float32), np.ones(sp.numSplats, np.uint8),
                         sp.colours)
    ref2 = O.render(sp.means3D, sp.covarianceMatrices, sp.opacities, cols2, u2, flags=flags, stages=False)
    assert np.array_equal(sp.texture().reshape(-1), ref2["image"].reshape(-1))
    ctx.close()


@pytest.mark.gpu
def test_sh_zero_rest_is_reference_colour(tmp_path):
    W, H = 384, 256
    ctx = g.Context(0)
    means, f_dc, f_rest, logit, log_scale, rot = sh_scene(5000)
    f_dc = np.abs(f_dc)  # (0.5 + SH_C0 f_dc) >= 0: the SH path's clamp is inactive
    p = str(tmp_path / "sh0.ply")
    write_ply_with_sh(p, means, f_dc, np.zeros_like(f_rest), logit, log_scale, rot)
    sp = g.Splats(p, W, H, ctx=ctx, sh=True)
    u = g.main_camera(W, H).uniforms()
    sp.render_uniforms(u)
    base = sp.texture()
    sp.flags = g.GS_FLAG_SH
    sp.render_uniforms(u)
    assert np.array_equal(base, sp.texture())
    ctx.close()


@pytest.mark.gpu
def test_sh_flag_needs_sh(tmp_path):
    ctx = g.Context(0)
    means, rot, sc, op, col = c2_scene(100)
    sp = g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, 64, 64, ctx=ctx)
    sp.flags = g.GS_FLAG_SH
    with pytest.raises(g.GsError, match="no SH"):
        sp.render_uniforms(g.main_camera(64, 64).uniforms())
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("target", ["whole", 512])
def test_sh_prefix_sorted_frames_colour_kept_splats(tmp_path, target):
    """a prefix-sorted GS_FLAG_SH frame colours only its kept entries' splats, after the sort
    (k_sh_kept): frames enqueued without a round trip, over two poses, bit-exact against the
    oracle's SH colours -- with every class kept whole (no frame may be redone, so the kept-splat
    colours made the images) and with cut lists (misses re-rendered on the synchronous path)"""
    from oracle import oracle as O
    O.build()
    W, H = 1280, 720
    ctx = g.Context(0)
    means, f_dc, f_rest, logit, log_scale, rot = sh_scene(100_000, seed=11)  # > 64k: not the fused kernel
    p = str(tmp_path / "sh_big.ply")
    write_ply_with_sh(p, means, f_dc, f_rest, logit, log_scale, rot)
    sp = g.Splats(p, W, H, ctx=ctx, sh=True)
    sp.flags = g.GS_FLAG_SH
    poses = []
    for turn in (0.0, 4.0):
        cam = g.main_camera(W, H)
        cam.rotateRight(turn)
        poses.append(cam.uniforms())
    refs = []
    for u in poses:
        cols = O.sh_colours(sp.means3D, f_dc, f_rest, np.array(u.view, np.float32), np.ones(sp.numSplats, np.uint8),
                            sp.colours)
        refs.append(O.render(sp.means3D, sp.covarianceMatrices, sp.opacities, cols, u, flags=0, stages=False))
    E = min(r["E"] for r in refs)
    ctx.set_sort_prefix(E // 64 if target == "whole" else target)
    sp.render_uniforms(poses[0])  # host-synchronous (the context's first frame)
    assert np.array_equal(sp.texture().reshape(-1), refs[0]["image"].reshape(-1))
    ctx.prefix_stats(reset=True)
    for k in range(4):
        sp.render_uniforms(poses[k % 2])
        assert np.array_equal(sp.texture().reshape(-1), refs[k % 2]["image"].reshape(-1)), f"frame {k}"
    ps = ctx.prefix_stats()
    assert ps["frames"] >= 1, ps
    if target == "whole":
        assert ps["redone"] == 0, ps
    ctx.close()


@pytest.mark.gpu
def test_sh_prefix_frame_then_staged_draw():
    """a prefix-sorted GS_FLAG_SH frame colours only its kept entries' splats; a staged
    gs_draw of that frame sorts its lists whole again (resort_full), and must colour every splat
    with entries first.  The staged draw uses tiles twice the frame's size, so pixels read their
    lists past the kept prefix (where the colours would be another pose's); it must equal the same
    staged draw after the host-synchronous frame of that pose."""
    import ctypes
    from openglgaussiansplattingrenderer_amd._native import check, lib
    from openglgaussiansplattingrenderer_amd import _native as N
    from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw
    W, H = 1920, 1080
    ctx = g.Context(0)
    ctx.set_lanes(1)  # one colour buffer: the pose-A colours stay where the B frame does not write
    sp = g.Splats.from_raw(*bicycle_standin_raw(), W, H, ctx=ctx)
    rng = np.random.default_rng(4242)
    f_dc = ((sp.colours[:, :3] / 255.0 - 0.5) / 0.28209479177387814).astype(np.float32)
    sp.set_sh(f_dc, rng.normal(0, 0.1, (sp.numSplats, 45)).astype(np.float32))
    sp.flags = g.GS_FLAG_SH
    uB = g.main_camera(W, H).uniforms()
    camA = g.main_camera(W, H)
    camA.rotateRight(20.0)
    uA = camA.uniforms()
    out = g.DeviceBuffer(ctx, W * H * 4)
    dst = g.DeviceBuffer(ctx, W * H * 4)

    def frame(u, sync):
        st = N.gs_frame_stats()
        check(lib().gs_render(ctx.handle, sp._scene, ctypes.byref(u), sp.flags, out.ptr, 1,
                              ctypes.byref(st) if sync else None), ctx.handle)

    def staged_draw():
        check(lib().gs_draw(ctx.handle, sp._scene, W, H, ctypes.c_float(W / 8.0), ctypes.c_float(H / 8.0),
                            g.GS_FLAG_SH, dst.ptr, 1), ctx.handle)
        return dst.download(np.uint8, W * H * 4)

    frame(uB, True)
    ref_img = staged_draw()
    frame(uA, True)  # every splat visible at A now holds A's colour
    assert ctx.set_sort_prefix() == 32768
    ctx.prefix_stats(reset=True)
    frame(uB, False)  # prefix-sorted: B's colours for the kept entries' splats only
    ctx.sync()
    ps = ctx.prefix_stats()
    assert ps["frames"] == 1 and ps["redone"] == 0 and ps["kept"] < ps["entries"] // 2, ps
    assert np.array_equal(staged_draw(), ref_img)
    ctx.close()
