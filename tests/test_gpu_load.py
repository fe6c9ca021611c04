"""the GPU load path (gs_scene_load_ply) against the host loader
(gs_ply_load + gs_covariance3d + gs_scene_create, itself checked against the reference's
fixture in test_oracle): the device scenes are identical bit for bit, and so are the frames."""
import os

import numpy as np
import pytest

import openglgaussiansplattingrenderer_amd as g

pytestmark = pytest.mark.gpu


def write_scene(path, n, seed):
    rng = np.random.default_rng(seed)
    means = rng.normal(0, 1.5, (n, 3)).astype(np.float32)
    rot = rng.normal(size=(n, 4)).astype(np.float32)  # raw, unnormalised (the loader normalises)
    sc = np.exp(rng.uniform(-9, 1, (n, 3))).astype(np.float32)
    op = rng.uniform(1e-4, 1 - 1e-4, n).astype(np.float32)
    col = rng.normal(0, 2, (n, 3)).astype(np.float32)
    # extremes through exp: very large / small logits and log-scales
    k = min(n, 4)
    op[:k] = np.array([1e-30, 1 - 1e-7, 0.5, 1e-7], np.float32)[:k]
    sc[:k] = np.array([[1e-30, 1e-20, 1e-10], [1e3, 1e6, 1e9], [1, 1, 1], [1e-38, 1e-38, 1e-38]], np.float32)[:k]
    g.save_ply(path, means, rot, sc, op, col)


@pytest.mark.parametrize("n", [1, 1000, 300_001])  # 300k spans two staging chunks
def test_gpu_load_matches_host(tmp_path, n):
    ctx = g.Context(0)
    p = str(tmp_path / "s.ply")
    write_scene(p, n, n)
    host = g.Splats(p, 320, 240, ctx=ctx)
    dev = g.Splats(p, 320, 240, ctx=ctx, gpu_load=True)
    assert dev.numSplats == host.numSplats == n
    for a, b, what in zip(host.download(), dev.download(), ("means", "cov", "opacity", "colour")):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), what
    u = g.main_camera(320, 240).uniforms()
    host.render_uniforms(u)
    dev.render_uniforms(u)
    assert np.array_equal(host.texture(), dev.texture())
    ctx.close()


def test_gpu_load_errors(tmp_path):
    ctx = g.Context(0)
    p = str(tmp_path / "s.ply")
    write_scene(p, 100, 1)
    raw = open(p, "rb").read()
    open(p, "wb").write(raw[:-10])  # truncated body
    with pytest.raises(g.GsError, match="failed to read all splats"):
        g.Splats(p, 64, 64, ctx=ctx, gpu_load=True)
    open(p, "wb").write(raw + b"x")  # trailing data (src/Splats.cpp:333-340)
    with pytest.raises(g.GsError, match="failed to read all splats"):
        g.Splats(p, 64, 64, ctx=ctx, gpu_load=True)
    with pytest.raises(g.GsError):
        g.Splats(str(tmp_path / "missing.ply"), 64, 64, ctx=ctx, gpu_load=True)
    ctx.close()


@pytest.mark.parametrize("n", [1, 3, 4099])  # odd counts: 28-byte shape records straddle 16-byte lines
def test_scene_roundtrip_bits(n):
    """gs_scene_create -> gs_scene_download returns every uploaded word unchanged (mean planes and the
    28-byte cov6 + opacity records, gs_internal.hpp kShapeFloats), including -0, subnormals, inf, NaN."""
    ctx = g.Context(0)
    rng = np.random.default_rng(n)
    means = rng.integers(0, 2**32, (n, 4), dtype=np.uint32).view(np.float32).copy()
    cov = rng.integers(0, 2**32, 6 * n, dtype=np.uint32).view(np.float32).copy()
    op = rng.integers(0, 2**32, n, dtype=np.uint32).view(np.float32).copy()
    col = rng.integers(0, 2**32, (n, 4), dtype=np.uint32).view(np.float32).copy()
    special = np.array([0x80000000, 0x00000001, 0x7F800000, 0x7FC00001], np.uint32).view(np.float32)
    cov[:min(6 * n, 4)] = special[:min(6 * n, 4)]
    op[-1] = special[3]
    means[0, :3] = special[:3]
    s = g.Splats(None, 64, 64, ctx=ctx, arrays=(np.zeros((n, 4), np.float32), np.zeros((n, 4), np.float32),
                                               np.zeros(n, np.float32), np.ones((n, 3), np.float32),
                                               np.tile(np.float32([1, 0, 0, 0]), (n, 1))))
    s.means3D, s.covarianceMatrices, s.opacities, s.colours = means, cov, op, col
    s.loadToGPU(64, 64)
    m, c, o, cl = s.download()
    assert np.array_equal(m[:, :3].view(np.uint32), means[:, :3].view(np.uint32))
    assert np.all(m[:, 3] == 1.0)  # w is not stored (the reference's means are homogeneous points)
    assert np.array_equal(c.view(np.uint32), cov.view(np.uint32))
    assert np.array_equal(o.view(np.uint32), op.view(np.uint32))
    assert np.array_equal(cl.view(np.uint32), col.view(np.uint32))
    ctx.close()
