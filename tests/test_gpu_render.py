"""GPU parity of the frame (preprocess -> sort -> bins -> blend) against the CPU oracle and
the committed golden fixtures.

Bar: means2D, conics, keys, sorted entries and bins bit-exact; RGBA8 bit-exact
with the defined exp (default), and >= 99.9% of covered pixels within +-1 LSB, max +-2 LSB
with GS_FLAG_FAST_EXP (hardware v_exp_f32)."""
import ctypes
import os
import tempfile

import numpy as np
import pytest

import openglgaussiansplattingrenderer_amd as g
from openglgaussiansplattingrenderer_amd import _native as N
from tests.golden.make_golden import U

pytestmark = pytest.mark.gpu

FAST_TOL_FRAC = 0.999
FAST_TOL_MAX = 2


@pytest.fixture(scope="module")
def ctx():
    c = g.Context(0)
    yield c
    c.close()


def c2_path(td):
    from openglgaussiansplattingrenderer_amd.scenes import c2_scene
    p = os.path.join(td, "c2.ply")
    g.save_ply(p, *c2_scene())
    return p


def scene_path(name, td, golden_dir):
    return os.path.join(golden_dir, "testSingleItem.ply") if name == "c1" else c2_path(td)


def gpu_frame(sp: g.Splats, u, flags):
    sp.flags = flags
    sp.render_uniforms(u)
    n, E = sp.numSplats, int(sp.stats.entries)
    # the values first, as the frame's sort left them (its last passes carry no keys); reading
    # the keys then sorts the frame's entries again, with keys
    vals = sp.read(g.GS_READ_VALS, E)
    return dict(image=sp.texture(), keys=sp.read(g.GS_READ_KEYS, E), vals=vals,
                bins=sp.read(g.GS_READ_BINS, 256), means2d=sp.read(g.GS_READ_MEANS2D, 2 * n, np.float32),
                conics=sp.read(g.GS_READ_CONICS, 4 * n, np.float32), V=int(sp.stats.visible),
                D=int(sp.stats.duplicates), E=E)


def assert_bits(a, b, what):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    assert a.shape == b.shape, what
    bad = np.nonzero(a.view(np.uint32 if a.dtype.itemsize == 4 else np.uint8) !=
                     b.view(np.uint32 if b.dtype.itemsize == 4 else np.uint8))[0]
    assert bad.size == 0, f"{what}: {bad.size} mismatches, first at {bad[:5]}"


def assert_image_tol(got, ref, what):
    d = np.abs(got.astype(int) - ref.astype(int))
    frac = np.mean(d.max(axis=-1) <= 1)
    assert d.max() <= FAST_TOL_MAX and frac >= FAST_TOL_FRAC, f"{what}: max {d.max()} within1 {frac}"


@pytest.fixture(params=[16, 8], ids=["sub16", "sub8"])
def sub(ctx, request):
    """the blend's sub-block form, forced (gs_ctx_set_draw_sub): both forms give the same image"""
    ctx.set_draw_sub(request.param)
    yield request.param
    ctx.set_draw_sub(0)


@pytest.mark.parametrize("name", ["c1", "c2"])
@pytest.mark.parametrize("mode,flags", [("ref", 0), ("clean", g.GS_FLAG_CLEAN)])
def test_golden_configs(ctx, golden_dir, name, mode, flags, sub):
    z = np.load(os.path.join(golden_dir, f"golden_{name}.npz"))
    u = U(z["uniforms"])
    uu = g.make_uniforms(np.array(u.view, np.float32).reshape(4, 4), u.width, u.height, u.focal_x, u.focal_y,
                         u.tan_fov_x, u.tan_fov_y, np.array(u.vp, np.float32).reshape(4, 4))
    with tempfile.TemporaryDirectory() as td:
        sp = g.Splats(scene_path(name, td, golden_dir), u.width, u.height, ctx=ctx)
    r = gpu_frame(sp, uu, flags)
    assert [r["V"], r["D"], r["E"]] == list(z[f"{mode}_VDE"])
    for k in ("means2d", "conics", "keys", "vals", "bins"):
        assert_bits(r[k], z[f"{mode}_{k}"], f"{name}/{mode}/{k}")
    assert_bits(r["image"].reshape(-1), z[f"{mode}_image"].reshape(-1), f"{name}/{mode}/image")
    assert ctx.set_draw_sub() == sub
    # fast exp: tolerance parity
    rf = gpu_frame(sp, uu, flags | g.GS_FLAG_FAST_EXP)
    assert_image_tol(rf["image"], z[f"{mode}_image"], f"{name}/{mode}/fast")


@pytest.mark.parametrize("W,H,n", [(1920, 1080, 20_000), (3840, 2160, 4_000), (1000, 600, 15_000),
                                   (12, 40, 3_000)])  # 12 px: reference tile width 0 (16-byte records)
@pytest.mark.parametrize("flags", [0, g.GS_FLAG_CLEAN])
def test_non_multiple_of_16_resolutions(ctx, oracle, W, H, n, flags, sub):
    """1080p / 4K / odd sizes: Q4 (int vs float tile dims), Q5 (unclamped main tile),
    Q9 (partial coverage) and Q18 (tile-straddling blocks) -- against the oracle live."""
    from openglgaussiansplattingrenderer_amd.scenes import c2_scene
    means, rot, sc, op, col = c2_scene(n, seed=n)
    sp = g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, W, H, ctx=ctx)
    u = g.main_camera(W, H).uniforms()
    r = gpu_frame(sp, u, flags)
    o = oracle.render(sp.means3D, sp.covarianceMatrices, sp.opacities, sp.colours, u, flags=flags)
    assert [r["V"], r["D"], r["E"]] == [o["V"], o["D"], o["E"]]
    for k in ("means2d", "conics", "keys", "vals", "bins"):
        assert_bits(r[k], o[k], f"{W}x{H}/{k}")
    assert_bits(r["image"].reshape(-1), o["image"].reshape(-1), f"{W}x{H}/image")
    assert ctx.set_draw_sub() == sub


@pytest.mark.parametrize("W,H,turn,flags", [(1920, 1080, 60, 0), (1920, 1080, 60, g.GS_FLAG_CLEAN),
                                             (12, 40, 30, 0)])  # 12 px: 16-byte records
def test_queued_preprocess_on_mostly_culled_frames(oracle, W, H, turn, flags):
    """a frame that follows one with fewer than half its splats inside the NDC square runs the
    queued preprocess (k_preprocess_q: the bulk of the preprocess on the NDC survivors only), the
    first frame of a context the straight-line one: both bit-exact against the oracle (100k
    splats, above the fused preprocess + emission's size)"""
    from openglgaussiansplattingrenderer_amd.scenes import c2_scene
    ctx = g.Context(0)
    means, rot, sc, op, col = c2_scene(100_000, seed=9)  # > 64 preprocess blocks: not the fused form
    sp = g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, W, H, ctx=ctx)
    cam = g.main_camera(W, H)
    cam.rotateRight(float(turn))
    u = cam.uniforms()
    o = oracle.render(sp.means3D, sp.covarianceMatrices, sp.opacities, sp.colours, u, flags=flags)
    assert 0 < o["V"] * 2 < sp.numSplats  # the second frame takes the queued form
    for frame in ("straight", "queued"):
        r = gpu_frame(sp, u, flags)
        assert [r["V"], r["D"], r["E"]] == [o["V"], o["D"], o["E"]], frame
        for k in ("means2d", "conics", "keys", "vals", "bins"):
            assert_bits(r[k], o[k], f"{frame}/{k}")
        assert_bits(r["image"].reshape(-1), o["image"].reshape(-1), f"{frame}/image")


def depth_range_scene(u, n=20_000, seed=5, log_scale=-7.0, opacity_bias=0.0):
    """n tiny splats at random NDC x, y in [-0.95, 0.95] and NDC depth in [-1.5, 2.5]: in ref mode
    there is no near/far cull (preprocess.glsl:77-89), so the keys tile + z01 (:154) run outside
    [tile, tile + 1) -- below their tile, negative floats (which sort last as words but bin to
    tile 0, countBins.glsl:25-29) and past tile + 1 into the next tiles' ranges"""
    rng = np.random.default_rng(seed)
    VP = np.array(u.vp[:], np.float64).reshape(4, 4).T
    ndc = np.stack([rng.uniform(-0.95, 0.95, n), rng.uniform(-0.95, 0.95, n), rng.uniform(-1.5, 2.5, n),
                    np.ones(n)], 1)
    w = (np.linalg.inv(VP) @ ndc.T).T
    means = (w[:, :3] / w[:, 3:]).astype(np.float32)
    col = rng.normal(0, 0.8, (n, 3)).astype(np.float32)
    op = (rng.normal(0, 2, n) + opacity_bias).astype(np.float32)
    return means, col, op, np.full((n, 3), log_scale, np.float32), rng.normal(size=(n, 4)).astype(np.float32)


# the frame sort's forms: (bucket sort, small-sort entry limit, prefix target)
SORT_FORMS = {
    "bucket": (1, 512 << 10, 0),      # by tile, then each tile's list (3 launches)
    "four_pass": (0, 512 << 10, 0),   # k_sweep_small: four 8-bit passes (8 launches)
    "full": (0, 0, 0),                # upsweep / row scan / downsweep per pass (12 launches)
    "prefix_whole": (0, 0, None),     # prefix sort, classes below the target kept whole
    "prefix_cut": (0, 0, 4096),       # prefix sort, lists cut (larger, mostly opaque splats)
    "prefix_partial": (0, 0, 64),     # prefix sort of 64-entry prefixes (misses re-rendered)
}


@pytest.mark.parametrize("form", list(SORT_FORMS))
@pytest.mark.parametrize("W,H,n", [(512, 512, 80_000), (1920, 1080, 80_000)])
def test_out_of_range_keys_every_sort_form(oracle, form, W, H, n):
    """ref-mode keys outside their tile's [t, t+1) (depth_range_scene: negative, below the tile,
    past t + 1) through every form of the frame sort, at 512x512 and 1080p: keys, values, bins
    and image of three consecutive frames (the first host-synchronous, the others enqueued without
    a round trip) bit-exact against the oracle.  The prefix forms run on frames of >= 64 x target
    entries; with the whole classes kept no frame may be rendered again."""
    bucket, small_sort, target = SORT_FORMS[form]
    ctx = g.Context(0)
    u = g.main_camera(W, H).uniforms()
    if form == "prefix_cut":  # larger, mostly opaque splats: the blends saturate within the prefix
        mm, cc, oo, ls, rr = depth_range_scene(u, n, log_scale=-4.5, opacity_bias=4.0)
    else:
        mm, cc, oo, ls, rr = depth_range_scene(u, n)
    sp = g.Splats.from_raw(mm, cc, oo, ls, rr, W, H, ctx=ctx)
    o = oracle.render(sp.means3D, sp.covarianceMatrices, sp.opacities, sp.colours, u, flags=0)
    if target is None:  # the deepest target the frame allows (E >= 64 x target): ~4x the mean
        target = o["E"] // 64  # class, so the sampled classes stay below it and are kept whole
    assert ctx.set_bucket_sort(bucket) == bucket
    ctx.set_small_limits(-1, small_sort)
    ctx.set_sort_prefix(target)
    keys = o["keys"].view(np.float32)
    assert (keys < 0).any(), "negative keys expected (splats in front of the near plane)"
    assert o["E"] >= 64 * max(target, 1)
    ctx.prefix_stats(reset=True)
    for frame in range(3):
        r = gpu_frame(sp, u, 0)
        assert [r["V"], r["D"], r["E"]] == [o["V"], o["D"], o["E"]], frame
        for k in ("keys", "vals", "bins"):
            assert_bits(r[k], o[k], f"{form} frame {frame}/{k}")
        assert_bits(r["image"].reshape(-1), o["image"].reshape(-1), f"{form} frame {frame}/image")
    ps = ctx.prefix_stats()
    print(form, W, H, "E", o["E"], "target", target, ps)
    if form.startswith("prefix"):
        assert ps["frames"] >= 2, ps
        if form == "prefix_whole":  # the prefix machinery sorted every entry, nothing redone
            assert ps["redone"] == 0 and ps["kept"] == o["E"], ps
        if form == "prefix_cut" and W == 512:  # lists cut, and the cut lists gave the exact images
            assert ps["redone"] == 0 and ps["kept"] < o["E"], ps
        # (at 1080p these splats are too small for any block to saturate: every cut frame misses
        # and is rendered again on the synchronous path -- the images above are still exact)
    else:
        assert ps["frames"] == 0, ps
    ctx.close()


@pytest.mark.parametrize("bucket", [1, 0])
def test_zero_entry_frames_then_bucket_sort(oracle, bucket):
    """a context's first frame has no entries (every splat off screen), then frames of
    out-of-range keys follow, alternating with empty ones, on rotating outputs: the small sort's
    tables after a sort of zero keys hold nothing stale -- every image equals the oracle's"""
    W, H = 512, 512
    ctx = g.Context(0)
    assert ctx.set_bucket_sort(bucket) == bucket
    u = g.main_camera(W, H).uniforms()
    mm, cc, oo, ls, rr = depth_range_scene(u, 20_000, seed=11)
    full = g.Splats.from_raw(mm, cc, oo, ls, rr, W, H, ctx=ctx)
    far = mm.copy()
    far[:, 0] += 1.0e5  # off screen: no entries
    empty = g.Splats.from_raw(far, cc, oo, ls, rr, W, H, ctx=ctx)
    of = oracle.render(full.means3D, full.covarianceMatrices, full.opacities, full.colours, u, flags=0)
    oe = oracle.render(empty.means3D, empty.covarianceMatrices, empty.opacities, empty.colours, u, flags=0)
    assert oe["E"] == 0 and of["E"] > 0
    seq = [empty, empty, full, empty, full, full, empty]
    outs = [g.DeviceBuffer(ctx, W * H * 4) for _ in seq]
    check_first = gpu_frame(empty, u, 0)  # host-synchronous (the context's first frame)
    assert check_first["E"] == 0 and np.array_equal(check_first["image"], oe["image"])
    for sp, out in zip(seq, outs):  # enqueued without a round trip
        N.check(N.lib().gs_render(ctx.handle, sp._scene, ctypes.byref(u), 0, out.ptr, 1, None), ctx.handle)
    ctx.sync()
    for k, (sp, out) in enumerate(zip(seq, outs)):
        ref = of if sp is full else oe
        got = out.download(np.uint8, W * H * 4)
        assert_bits(got, ref["image"].reshape(-1), f"frame {k} ({'full' if sp is full else 'empty'})")
    r = gpu_frame(full, u, 0)
    for k in ("keys", "vals", "bins"):
        assert_bits(r[k], of[k], f"after the sequence/{k}")
    ctx.close()


@pytest.mark.parametrize("bucket", [1, 0])
@pytest.mark.parametrize("flags", [0, g.GS_FLAG_CLEAN])
def test_small_sort_forms_match_oracle(oracle, bucket, flags):
    """frames below the small-sort limit sort by tile and then each tile's list (k_bucket_sort;
    a list over 4096 keys takes its global-memory passes) or in four 8-bit passes: keys, values,
    bins and image bit-exact against the oracle, for an ordinary scene and one whose splats all
    fall into a few tiles (30k-entry lists)"""
    from openglgaussiansplattingrenderer_amd.scenes import c2_scene
    ctx = g.Context(0)
    assert ctx.set_bucket_sort(bucket) == bucket
    means, rot, sc, op, col = c2_scene(30_000, seed=3)
    c = means.mean(0)
    scenes = [(means, col, np.log(op / (1 - op)), np.log(sc), rot),
              (c + (means - c) * 0.03, col, np.log(op / (1 - op)), np.log(sc * 0.05), rot)]
    for mm, cc, oo, ls, rr in scenes:
        sp = g.Splats.from_raw(mm.astype(np.float32), cc, oo, ls.astype(np.float32), rr, 512, 512, ctx=ctx)
        u = g.main_camera(512, 512).uniforms()
        o = oracle.render(sp.means3D, sp.covarianceMatrices, sp.opacities, sp.colours, u, flags=flags)
        for _ in range(2):  # the first frame of a context, then one whose predecessor's count is known
            r = gpu_frame(sp, u, flags)
            assert [r["V"], r["D"], r["E"]] == [o["V"], o["D"], o["E"]]
            for k in ("keys", "vals", "bins"):
                assert_bits(r[k], o[k], f"bucket {bucket}/{k}")
            assert_bits(r["image"].reshape(-1), o["image"].reshape(-1), f"bucket {bucket}/image")
    ctx.set_bucket_sort(1)


@pytest.mark.parametrize("flags", [0, g.GS_FLAG_CLEAN])
def test_non_finite_colours_match_oracle(ctx, oracle, flags, sub):
    """splats whose colour is +-inf or NaN (f_dc non-finite): the blend keeps a pixel by selects
    when an event does not blend (a batch with a non-finite colour; `rgb * 0` would be NaN), and
    the image still equals the oracle bit for bit"""
    from openglgaussiansplattingrenderer_amd.scenes import c2_scene
    means, rot, sc, op, col = c2_scene(6_000, seed=77)
    col = col.astype(np.float32).copy()
    rng = np.random.default_rng(5)
    bad = rng.choice(len(col), 300, replace=False)
    col[bad[:100], 0] = np.inf
    col[bad[100:200], 1] = -np.inf
    col[bad[200:], 2] = np.nan
    sp = g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, 640, 480, ctx=ctx)
    assert not np.isfinite(sp.colours).all()
    u = g.main_camera(640, 480).uniforms()
    r = gpu_frame(sp, u, flags)
    o = oracle.render(sp.means3D, sp.covarianceMatrices, sp.opacities, sp.colours, u, flags=flags)
    assert_bits(r["image"].reshape(-1), o["image"].reshape(-1), "non-finite colours/image")


def test_cull_is_exact_and_frames_deterministic(ctx, sub):
    """the per-block cull never changes a pixel; repeated frames are bit-identical"""
    from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw
    raw = bicycle_standin_raw(400_000, seed=3)
    sp = g.Splats.from_raw(*raw, 1920, 1080, ctx=ctx)
    u = g.main_camera(1920, 1080).uniforms()
    for flags in (0, g.GS_FLAG_CLEAN, g.GS_FLAG_FAST_EXP):
        a = gpu_frame(sp, u, flags)["image"]
        b = gpu_frame(sp, u, flags)["image"]
        c = gpu_frame(sp, u, flags | g.GS_FLAG_NO_CULL)["image"]
        assert np.array_equal(a, b)
        assert np.array_equal(a, c)


def test_full_size_properties(ctx, oracle):
    """BASELINE C3 size (6,131,954-splat synthetic stand-in, 1920x1080), the benchmark's own
    frame: preprocess, sort, bins and the RGBA8 image bit-exact against the oracle (the oracle
    blends the full frame on the host cores, ~2 s); fast-exp image within tolerance of the
    exact one."""
    from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw
    raw = bicycle_standin_raw()
    sp = g.Splats.from_raw(*raw, 1920, 1080, ctx=ctx)
    u = g.main_camera(1920, 1080).uniforms()
    for flags in (0, g.GS_FLAG_CLEAN):
        r = gpu_frame(sp, u, flags)
        o = oracle.render(sp.means3D, sp.covarianceMatrices, sp.opacities, sp.colours, u, flags=flags, draw=True)
        assert [r["V"], r["D"], r["E"]] == [o["V"], o["D"], o["E"]]
        for k in ("means2d", "conics", "keys", "vals", "bins"):
            assert_bits(r[k], o[k], f"C3 flags {flags}/{k}")
        assert_bits(r["image"].reshape(-1), o["image"].reshape(-1), f"C3 flags {flags}/image")
    r = gpu_frame(sp, u, 0)
    rf = gpu_frame(sp, u, g.GS_FLAG_FAST_EXP)
    assert_image_tol(rf["image"], r["image"], "C3 fast vs exact")


def test_stage_api_matches_gpuRender(ctx, golden_dir):
    """Splats.preprocess / sort / computeBins / draw == gpuRender (src/Splats.cpp:587-597),
    with the camera getters passed as main.cpp:62-64 passes them"""
    with tempfile.TemporaryDirectory() as td:
        sp = g.Splats(c2_path(td), 512, 512, ctx=ctx)
    cam = g.main_camera(512, 512)
    u = cam.uniforms()
    vp = np.array(u.vp[:], np.float32).reshape(4, 4)
    args = (cam.getViewMatrix(), 512, 512, cam.getFocalX(), cam.getFocalY(), cam.getTanFovy(), cam.getTanFovx(), vp)
    sp.flags = 0
    sp.gpuRender(*args)
    a = sp.texture()
    z = np.load(os.path.join(golden_dir, "golden_c2.npz"))
    assert np.array_equal(a, z["ref_image"])
    sp.preprocess(*args)
    sp.computeBins()  # the reference's order: bins, then sort (src/Splats.cpp:593-594)
    sp.sort()
    sp.draw(512, 512, 512 / 16.0, 512 / 16.0)
    assert np.array_equal(a, sp.texture())
    assert np.array_equal(np.flipud(a), sp.display())


def test_stage_order_errors():
    from openglgaussiansplattingrenderer_amd._native import GS_ERR_STATE
    c = g.Context(0)
    assert g.lib().gs_sort(c.handle) == GS_ERR_STATE
    assert g.lib().gs_compute_bins(c.handle) == GS_ERR_STATE
    c.close()


def test_scene_size_limit(ctx):
    """scenes hold at most 2^27 splats (32-bit byte offsets into the 32-B blend records): more is
    refused before any array is read"""
    import ctypes
    from openglgaussiansplattingrenderer_amd import _native as N
    a = np.zeros(16, np.float32)
    h = ctypes.c_void_p()
    rc = N.lib().gs_scene_create(ctx.handle, (1 << 27) + 1, N.ptr(a), N.ptr(a), N.ptr(a), N.ptr(a), ctypes.byref(h))
    assert rc < 0 and not h.value
    assert b"2^27" in N.lib().gs_last_error(ctx.handle)


def full_frame_vs_oracle(sp, oracle, W, H, view, flags=0, sub=0):
    sp.ctx.set_draw_sub(sub)
    cam = g.main_camera(W, H)
    cam.rotateRight(45.0 * view)
    u = cam.uniforms()
    r = gpu_frame(sp, u, flags)
    o = oracle.render(sp.means3D, sp.covarianceMatrices, sp.opacities, sp.colours, u, flags=flags, draw=True)
    assert [r["V"], r["D"], r["E"]] == [o["V"], o["D"], o["E"]]
    for k in ("keys", "vals", "bins"):
        assert_bits(r[k], o[k], f"{W}x{H} view {view}/{k}")
    assert_bits(r["image"].reshape(-1), o["image"].reshape(-1), f"{W}x{H} view {view}/image")
    if sub:
        assert sp.ctx.set_draw_sub() == sub
    sp.ctx.set_draw_sub(0)
    return r


def test_full_size_c4(ctx, oracle):
    """C4 (the bicycle-sized scene at 3840x2160), ref mode, bit-exact against the oracle"""
    from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw
    sp = g.Splats.from_raw(*bicycle_standin_raw(), 3840, 2160, ctx=ctx)
    full_frame_vs_oracle(sp, oracle, 3840, 2160, 0)


@pytest.fixture(scope="module")
def c5_scene(ctx):
    from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw
    return g.Splats.from_raw(*bicycle_standin_raw(), 1920, 1080, ctx=ctx)


@pytest.mark.parametrize("view", [1, 2, 3, 4, 5, 6, 7])
def test_c5_views(ctx, oracle, c5_scene, view):
    """every C5 pose at full size (pose k = main pose + rotateRight(45 deg * k), what rank k renders
    in the multi-GPU runs; view 0 is C3, test_full_size_properties), ref mode, bit-exact against
    the oracle.  Views 2-7 are the small-entry frames (0.16-0.96M entries), which blend in 8x8
    sub-blocks; view 4 also in the other form."""
    r = full_frame_vs_oracle(c5_scene, oracle, 1920, 1080, view)
    if view == 4:
        ctx.set_draw_sub(16)
        cam = g.main_camera(1920, 1080)
        cam.rotateRight(45.0 * view)
        r16 = gpu_frame(c5_scene, cam.uniforms(), 0)
        assert ctx.set_draw_sub(0) == 16
        assert np.array_equal(r16["image"], r["image"])


@pytest.mark.parametrize("staged", [False, True])
def test_culled_entries_drawn_as_splat_zero(oracle, staged):
    """ref mode: the reference's culled splats stay in the sorted range as splat 0 (key 1e6,
    preprocess.glsl:80-88) and a Q10 window reaches them (tests/culled_scene.py): bit-exact vs the
    oracle, through the frame path (bins from the sort) and the staged one (k_bins_*)"""
    from tests.culled_scene import culled_scene
    W, H = 512, 512
    ctx = g.Context(0)
    means, col, op, log_sc, rot, u = culled_scene(g, W, H)
    sp = g.Splats.from_raw(means, col, op, log_sc, rot, W, H, ctx=ctx)
    ref = oracle.render(sp.means3D, sp.covarianceMatrices, sp.opacities, sp.colours, u, flags=0)
    assert sp.numSplats - ref["V"] == 300
    if staged:
        sp._preprocess_u(u)
        sp.sort()
        sp.computeBins()
        sp.draw(W, H, W / 16.0, H / 16.0)
    else:
        sp.render_uniforms(u)
    assert np.array_equal(sp.texture(), ref["image"])
    # splat 0 culled: its culled record never blends (the block changes nothing)
    means2 = means.copy()
    means2[0] = means[-1]
    sp2 = g.Splats.from_raw(means2, col, op, log_sc, rot, W, H, ctx=ctx)
    ref2 = oracle.render(sp2.means3D, sp2.covarianceMatrices, sp2.opacities, sp2.colours, u, flags=0)
    sp2.render_uniforms(u)
    assert np.array_equal(sp2.texture(), ref2["image"])
    ctx.close()


@pytest.mark.parametrize("view", [0, 4])
def test_small_forms_forced_on_large_frames(ctx, oracle, c5_scene, view):
    """the small-frame forms on any frame: the 8-launch sort (k_sweep_small) and the 8x8 blend forced
    on the full C3 frame (10M entries) and the small view 4 -- and both turned off on view 4 -- all
    bit-exact against the oracle"""
    try:
        ctx.set_small_limits(1 << 40, 1 << 40)
        full_frame_vs_oracle(c5_scene, oracle, 1920, 1080, view, sub=8)
        ctx.set_small_limits(0, 0)
        full_frame_vs_oracle(c5_scene, oracle, 1920, 1080, view, sub=16)
    finally:
        ctx.set_small_limits(2 << 20, 512 << 10)
