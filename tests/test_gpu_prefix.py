"""Prefix sort of frames enqueued without a host round trip (gs_ctx_set_sort_prefix): each tile
list is sorted only to a depth that covers what the blend reads; a frame whose blend reaches an
unsorted position is rendered again with the full sort.  Images, bins and readbacks must equal
the full-sort path's bit for bit -- whether or not the prefix was deep enough."""
import ctypes

import numpy as np
import pytest

import openglgaussiansplattingrenderer_amd as g
from openglgaussiansplattingrenderer_amd import _native as N
from openglgaussiansplattingrenderer_amd._native import check, lib
from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw

pytestmark = pytest.mark.gpu


def render_sync(sp, u, out):
    st = N.gs_frame_stats()
    check(lib().gs_render(sp.ctx.handle, sp._scene, ctypes.byref(u), sp.flags, out.ptr, 1, ctypes.byref(st)),
          sp.ctx.handle)
    return st


def render_spec(sp, u, out):
    check(lib().gs_render(sp.ctx.handle, sp._scene, ctypes.byref(u), sp.flags, out.ptr, 1, None), sp.ctx.handle)


def pose(W, H, k):
    cam = g.main_camera(W, H)
    cam.rotateRight(6.0 * k)
    return cam.uniforms()


@pytest.fixture(scope="module")
def c3():
    ctx = g.Context(0)
    sp = g.Splats.from_raw(*bicycle_standin_raw(), 1920, 1080, ctx=ctx)
    yield ctx, sp
    ctx.close()


@pytest.mark.parametrize("flags", [0, g.GS_FLAG_CLEAN])
def test_prefix_c3_frames_equal_full_sort(c3, oracle, flags):
    """The benchmark's C3 frame, prefix-sorted at the default depth: no frame rendered again,
    far fewer entries sorted than emitted, and the image bit-exact against the oracle and the
    full-sort frame; the readbacks (values, keys) are the whole sorted lists."""
    ctx, sp = c3
    W, H = 1920, 1080
    sp.flags = flags
    u = g.main_camera(W, H).uniforms()
    ref = g.DeviceBuffer(ctx, W * H * 4)
    st = render_sync(sp, u, ref)  # full sort; the entry count is now known on the host
    img_full = ref.download(np.uint8, W * H * 4)
    assert ctx.set_sort_prefix() == 32768
    ctx.prefix_stats(reset=True)
    outs = [g.DeviceBuffer(ctx, W * H * 4) for _ in range(3)]
    for k in range(3):
        render_spec(sp, u, outs[k])
    ctx.sync()
    ps = ctx.prefix_stats()
    assert ps["frames"] == 3 and ps["redone"] == 0, ps
    assert ps["entries"] == st.entries and 0 < ps["kept"] < st.entries // 2, ps
    for k in range(3):
        assert np.array_equal(outs[k].download(np.uint8, W * H * 4), img_full), f"frame {k}"
    o = oracle.render(sp.means3D, sp.covarianceMatrices, sp.opacities, sp.colours, u, flags=flags, draw=True)
    assert np.array_equal(img_full.reshape(H, W, 4), o["image"])
    E = int(st.entries)
    assert np.array_equal(sp.read(g.GS_READ_VALS, E), o["vals"])
    assert np.array_equal(sp.read(g.GS_READ_KEYS, E), o["keys"])
    assert np.array_equal(sp.read(g.GS_READ_BINS, 256), o["bins"])


@pytest.mark.parametrize("kept", [0, 1])
def test_prefix_kept_frames_across_modes(c3, kept):
    """Phases of static prefix-sorted frames (ref mode, clean mode, ref mode again, each after a
    synchronous frame; each phase's bounds sized by the other mode's per-tile depths): no frame
    rendered again, every one bit-exact against the phase's synchronous frame -- with the full
    emission and with the kept emission (gs_ctx_set_kept_emission: each frame after a phase's
    first emits only the entries within the previous frame's bounds; a race on those bounds in
    LDS once gave wrong images here without a miss)."""
    ctx, sp = c3
    W, H = 1920, 1080
    u = g.main_camera(W, H).uniforms()
    ref = g.DeviceBuffer(ctx, W * H * 4)
    outs = [g.DeviceBuffer(ctx, W * H * 4) for _ in range(6)]
    assert ctx.set_sort_prefix() == 32768
    assert ctx.set_kept_emission(kept)[0] == kept
    k0 = ctx.set_kept_emission()[1]
    for flags in [0, g.GS_FLAG_CLEAN, 0, g.GS_FLAG_CLEAN]:
        sp.flags = flags
        render_sync(sp, u, ref)
        img = ref.download(np.uint8, W * H * 4)
        ctx.prefix_stats(reset=True)
        for o in outs:
            render_spec(sp, u, o)
        ctx.sync()
        ps = ctx.prefix_stats()
        assert ps["frames"] == len(outs) and ps["redone"] == 0, (flags, ps)
        for k, o in enumerate(outs):
            assert np.array_equal(o.download(np.uint8, W * H * 4), img), (flags, k)
    assert ctx.set_kept_emission(0)[1] - k0 == (4 * len(outs) if kept else 0)
    sp.flags = 0


def test_prefix_kept_emission_turning_camera():
    """The kept emission under a camera turning 3 degrees per frame and walking 0.1 per frame:
    turned frames emit every entry and select their own bounds, the frames after them keep by
    those; every image bit-exact against the host-synchronous full sort, at most one frame
    rendered again."""
    W, H = 1920, 1080
    ctx = g.Context(0)
    sp = g.Splats.from_raw(*bicycle_standin_raw(), W, H, ctx=ctx)
    ref = g.DeviceBuffer(ctx, W * H * 4)

    def cam(k):
        c = g.main_camera(W, H)
        c.rotateRight(3.0 * min(k, 4))  # turn for 4 frames, then walk
        c.moveForward(0.1 * max(0, k - 4))
        return c.uniforms()

    render_sync(sp, cam(0), ref)
    assert ctx.set_sort_prefix() == 32768
    assert ctx.set_kept_emission(1)[0] == 1
    ctx.prefix_stats(reset=True)
    outs = [g.DeviceBuffer(ctx, W * H * 4) for _ in range(3)]
    got = []
    for k in range(9):
        render_spec(sp, cam(k), outs[k % 3])
        if k % 3 == 2:
            ctx.sync()
            got += [o.download(np.uint8, W * H * 4) for o in outs]
    ps = ctx.prefix_stats()
    assert ps["frames"] == 9 and ps["redone"] <= 1, ps
    assert ctx.set_kept_emission()[1] >= 4  # the walking frames kept
    for k in range(9):
        render_sync(sp, cam(k), ref)
        assert np.array_equal(got[k], ref.download(np.uint8, W * H * 4)), f"frame {k}"
    ctx.close()


def test_prefix_misses_render_again():
    """A prefix far too shallow: the blend reaches unsorted positions, the frames are rendered
    again with the full sort (and the depth doubles) -- every image still equals the
    host-synchronous frame's, in order, over rotating outputs and changing poses."""
    W, H = 1280, 720
    ctx = g.Context(0)
    sp = g.Splats.from_raw(*bicycle_standin_raw(400_000, seed=3), W, H, ctx=ctx)
    ref = g.DeviceBuffer(ctx, W * H * 4)
    st = render_sync(sp, pose(W, H, 0), ref)
    assert st.entries >= 64 * 256
    ctx.set_sort_prefix(256)
    ctx.prefix_stats(reset=True)
    outs = [g.DeviceBuffer(ctx, W * H * 4) for _ in range(6)]
    for k in range(6):
        render_spec(sp, pose(W, H, k % 3), outs[k])
    ctx.sync()
    ps = ctx.prefix_stats()
    assert ps["redone"] >= 1, ps
    assert ctx.set_sort_prefix() > 256  # deepened after the miss
    got = [o.download(np.uint8, W * H * 4) for o in outs]
    for k in range(6):
        render_sync(sp, pose(W, H, k % 3), ref)
        assert np.array_equal(got[k], ref.download(np.uint8, W * H * 4)), f"frame {k}"
    ctx.close()


def test_prefix_sorted_boxes_draw_culled_entries_as_splat_zero(oracle):
    """VERDICT r5 / ADVICE r5 (medium): on a prefix-sorted frame the blend reads each entry's cull
    box in sorted order (GS_DRAW_SBOX).  The last tile's Q10 window runs past its list into the
    reference's culled entries, drawn as splat 0 (preprocess.glsl:80-88, draw.glsl:97-98); their
    box is splat 0's.  Scene (tests/culled_scene.py, n_bulk): millions of entries in the low tiles
    (the prefix sort engages), splat 0 visible in tile 255 with a list far shorter than the target
    and not a multiple of 1024, 300 culled splats, no key in [256, 1e6) -- so no prefix limit stops
    the window.  The prefix-sorted frames must equal the oracle and the full sort bit for bit."""
    from tests.culled_scene import culled_scene
    W, H = 1024, 512
    ctx = g.Context(0)
    means, col, op, log_sc, rot, u = culled_scene(g, W, H, n_bulk=30_000)
    sp = g.Splats.from_raw(means, col, op, log_sc, rot, W, H, ctx=ctx)
    o = oracle.render(sp.means3D, sp.covarianceMatrices, sp.opacities, sp.colours, u, flags=0, draw=True)
    assert sp.numSplats - o["V"] == 300
    keys = o["keys"].view(np.float32)
    assert not np.any((keys >= 256.0) & (keys < 1.0e6))
    bins = o["bins"].astype(np.int64)
    n255 = int(bins[255] - bins[254])
    assert 0 < n255 < 4096 and n255 % 1024 != 0, n255
    # the culled entries matter: the oracle's blend without them differs in the last row of tiles
    O = oracle
    img_no = np.zeros_like(o["image"])
    O.lib().ora_draw(W, H, 0, O._p(o["bins"]), O._p(o["vals"]), o["E"], O._p(o["means2d"]), O._p(o["conics"]),
                     O._p(np.ascontiguousarray(sp.colours, np.float32)), O._p(img_no))
    diff = np.any(img_no != o["image"], axis=2)
    assert diff[15 * H // 16:, 15 * W // 16:].sum() > 50 and not diff[: 15 * H // 16].any()
    ref = g.DeviceBuffer(ctx, W * H * 4)
    st = render_sync(sp, u, ref)
    assert st.entries >= 64 * 32768, st.entries
    img_full = ref.download(np.uint8, W * H * 4)
    assert np.array_equal(img_full.reshape(H, W, 4), o["image"])
    assert ctx.set_sort_prefix() == 32768
    ctx.prefix_stats(reset=True)
    outs = [g.DeviceBuffer(ctx, W * H * 4) for _ in range(3)]
    for k in range(3):
        render_spec(sp, u, outs[k])
    ctx.sync()
    ps = ctx.prefix_stats()
    assert ps["frames"] == 3 and ps["redone"] == 0, ps
    assert ps["kept"] < ps["entries"], ps
    for k in range(3):
        assert np.array_equal(outs[k].download(np.uint8, W * H * 4), img_full), f"frame {k}"
    ctx.close()


def test_prefix_off_and_stage_calls():
    """target 0 turns the prefix sort off; after a prefix-sorted frame the stage API (a draw of
    the frame's lists, a re-sort) sees the whole sorted lists."""
    W, H = 1280, 720
    ctx = g.Context(0)
    sp = g.Splats.from_raw(*bicycle_standin_raw(400_000, seed=5), W, H, ctx=ctx)
    u = pose(W, H, 1)
    ref = g.DeviceBuffer(ctx, W * H * 4)
    st = render_sync(sp, u, ref)
    img = ref.download(np.uint8, W * H * 4)
    E = int(st.entries)
    vals_full = sp.read(g.GS_READ_VALS, E)
    bins_full = sp.read(g.GS_READ_BINS, 256)
    ctx.set_sort_prefix(0)
    ctx.prefix_stats(reset=True)
    out = g.DeviceBuffer(ctx, W * H * 4)
    render_spec(sp, u, out)
    ctx.sync()
    assert ctx.prefix_stats()["frames"] == 0
    assert np.array_equal(out.download(np.uint8, W * H * 4), img)
    ctx.set_sort_prefix(1024)
    render_spec(sp, u, out)
    ctx.sync()
    assert ctx.prefix_stats()["frames"] == 1
    assert np.array_equal(out.download(np.uint8, W * H * 4), img)
    # gs_draw of the newest frame: its lists are sorted whole first
    out2 = g.DeviceBuffer(ctx, W * H * 4)
    check(lib().gs_draw(ctx.handle, sp._scene, W, H, ctypes.c_float(W / 16.0), ctypes.c_float(H / 16.0), 0,
                        out2.ptr, 1), ctx.handle)
    assert np.array_equal(out2.download(np.uint8, W * H * 4), img)
    assert np.array_equal(sp.read(g.GS_READ_VALS, E), vals_full)
    check(lib().gs_sort(ctx.handle), ctx.handle)
    assert np.array_equal(sp.read(g.GS_READ_VALS, E), vals_full)
    # gs_compute_bins right after a frame whose sort left the keys unsorted: the entries are sorted
    # again with their keys first
    render_spec(sp, u, out)
    check(lib().gs_compute_bins(ctx.handle), ctx.handle)
    assert np.array_equal(sp.read(g.GS_READ_BINS, 256), bins_full)
    ctx.set_sort_prefix(0)
    render_spec(sp, u, out)
    check(lib().gs_compute_bins(ctx.handle), ctx.handle)
    assert np.array_equal(sp.read(g.GS_READ_BINS, 256), bins_full)
    assert np.array_equal(sp.read(g.GS_READ_VALS, E), vals_full)
    ctx.close()


def sheet_and_cluster_scene(u, n_cluster, seed):
    """an opaque sheet of splats in front of the camera covering the whole image (every pixel
    saturates within the first entries of its tile's list), behind it a tight cluster of n_cluster
    splats around the world origin (a few tile lists of ~n_cluster entries): a frame that sorts
    only ~32k entries of each list deep and never misses, and keeps few entries in all"""
    rng = np.random.default_rng(seed)
    W, H = u.width, u.height
    VP = np.array(u.vp[:], np.float64).reshape(4, 4).T
    V = np.array(u.view[:], np.float64).reshape(4, 4).T
    gx, gy = np.meshgrid(np.arange(-60, W + 61, 24.0), np.arange(-60, H + 61, 24.0))
    ndc = np.stack([2 * gx.ravel() / W - 1, 2 * gy.ravel() / H - 1, np.full(gx.size, 0.9), np.ones(gx.size)], 1)
    wpt = (np.linalg.inv(VP) @ ndc.T).T
    sheet = wpt[:, :3] / wpt[:, 3:]
    depth = -(V @ np.c_[sheet, np.ones(len(sheet))].T)[2]  # view-space distance
    sig = 30.0 * depth / u.focal_y  # ~30 px
    n_s = len(sheet)
    cl = rng.normal(0.0, 0.05, (n_cluster, 3))
    means = np.r_[sheet, cl].astype(np.float32)
    q = rng.normal(size=(n_s + n_cluster, 4)).astype(np.float32)
    q[:n_s] = [1, 0, 0, 0]
    rot = q / np.linalg.norm(q, axis=1, keepdims=True)
    log_sc = np.r_[np.repeat(np.log(sig)[:, None], 3, 1), np.full((n_cluster, 3), -5.0)].astype(np.float32)
    op = np.r_[np.full(n_s, 10.0), rng.normal(0.0, 2.0, n_cluster)].astype(np.float32)  # logits
    col = rng.normal(0.0, 0.8, (n_s + n_cluster, 3)).astype(np.float32)
    return means, col, op, log_sc, rot


def test_prefix_kept_count_jump():
    """a prefix-sorted frame that keeps far more entries than the frame before it.  Scene
    A (an opaque sheet in front of a tight cluster: a few deep lists, every pixel saturating early)
    keeps ~0.2M entries, then scene B (the C3 stand-in) keeps ~2.2M in the same context.  B's first
    prefix frame may be rendered again -- its passes 1-3 were sized from A's kept count (the 4-pass
    form), or it selected with A's per-tile depths -- but at most once, and B's later frames are
    not; every image equals the host-synchronous frame's."""
    W, H = 1920, 1080
    ctx = g.Context(0)
    ctx.set_lanes(1)  # one lane: the entry buffers B's sync frame grows are the ones B's frame uses
    assert ctx.set_sort_prefix() == 32768
    u = g.main_camera(W, H).uniforms()
    spa = g.Splats.from_raw(*sheet_and_cluster_scene(u, 2_300_000, 8), W, H, ctx=ctx)
    spb = g.Splats.from_raw(*bicycle_standin_raw(), W, H, ctx=ctx)
    ref = g.DeviceBuffer(ctx, W * H * 4)
    render_sync(spb, u, ref)  # B's entries sized; the host now knows an entry count
    img_b = ref.download(np.uint8, W * H * 4)
    sta = render_sync(spa, u, ref)
    img_a = ref.download(np.uint8, W * H * 4)
    assert sta.entries >= 64 * 32768, sta.entries  # A's frames are prefix-sorted
    out = g.DeviceBuffer(ctx, W * H * 4)
    ctx.prefix_stats(reset=True)
    for _ in range(2):
        render_spec(spa, u, out)
    ctx.sync()
    psa = ctx.prefix_stats(reset=True)
    assert psa["frames"] == 2 and psa["redone"] == 0, psa
    assert np.array_equal(out.download(np.uint8, W * H * 4), img_a)
    kept_a = psa["kept"]
    render_spec(spb, u, out)
    ctx.sync()
    psb = ctx.prefix_stats()
    # (B's first frame selects with the per-tile depths A's blends recorded -- another scene's, far
    # shallower: it may miss, and is then rendered again; never for its kept count.  With the kept
    # emission B's first frame keeps every entry and forgets A's depths, so its bounds for the
    # second frame come from the target alone)
    assert psb["frames"] == 1 and psb["redone"] <= 1, psb
    assert np.array_equal(out.download(np.uint8, W * H * 4), img_b)
    for _ in range(2):
        render_spec(spb, u, out)
    ctx.sync()
    ps2 = ctx.prefix_stats()
    assert ps2["frames"] == 3 and ps2["redone"] == psb["redone"], ps2  # B's own depths now
    assert ps2["kept"] > kept_a * 5 // 4 + 65536, (kept_a, ps2)
    assert np.array_equal(out.download(np.uint8, W * H * 4), img_b)
    ctx.close()


def test_prefix_depth_decays_after_clean_frames():
    """misses double the depth; 64 frames in a row without a miss halve it again, never
    below the configured target -- misses do not deepen the sort (or turn it off: E < 64 * target)
    for good."""
    W, H = 1280, 720
    ctx = g.Context(0)
    sp = g.Splats.from_raw(*bicycle_standin_raw(400_000, seed=3), W, H, ctx=ctx)
    ref = g.DeviceBuffer(ctx, W * H * 4)
    u = pose(W, H, 0)
    render_sync(sp, u, ref)
    img = ref.download(np.uint8, W * H * 4)
    ctx.set_sort_prefix(256)
    out = g.DeviceBuffer(ctx, W * H * 4)
    targets = []
    for _ in range(200):
        render_spec(sp, u, out)
        ctx.sync()
        targets.append(ctx.set_sort_prefix())
    assert max(targets) > 256, targets[:20]  # 256 entries are too shallow here: misses deepened it
    drops = sum(1 for a, b in zip(targets, targets[1:]) if b < a)
    assert drops >= 1, targets  # ... and clean runs brought it down again
    assert min(targets) >= 256
    assert np.array_equal(out.download(np.uint8, W * H * 4), img)
    ctx.close()


def test_prefix_on_a_fused_frame():
    """A scene small enough for the fused preprocess + emission (k_pre_emit: at most 64 workgroups,
    the split entry layout) with entries enough for the prefix sort (>= 64 * target): the sampled
    histogram comes from the fused kernel, the sort's first pass reads the split layout -- every
    frame equals the host-synchronous one (rendered again or not)."""
    W, H = 1920, 1080
    ctx = g.Context(0)
    rng = np.random.default_rng(21)
    n = 60_000
    means = rng.normal(0.0, 1.5, (n, 3)).astype(np.float32)
    q = rng.normal(size=(n, 4)).astype(np.float32)
    rot = q / np.linalg.norm(q, axis=1, keepdims=True)
    log_sc = rng.uniform(np.log(0.3), np.log(1.2), (n, 3)).astype(np.float32)
    op = rng.normal(-1.0, 1.5, n).astype(np.float32)
    col = rng.normal(0.0, 0.8, (n, 3)).astype(np.float32)
    sp = g.Splats.from_raw(means, col, op, log_sc, rot, W, H, ctx=ctx)
    ref = g.DeviceBuffer(ctx, W * H * 4)
    outs = [g.DeviceBuffer(ctx, W * H * 4) for _ in range(3)]
    for k in range(3):
        st = render_sync(sp, pose(W, H, k), ref)
        assert st.entries >= 64 * 32768, st.entries
    ctx.prefix_stats(reset=True)
    for k in range(3):
        render_spec(sp, pose(W, H, k), outs[k])
    ctx.sync()
    ps = ctx.prefix_stats()
    assert ps["frames"] >= 1, ps
    for k in range(3):
        render_sync(sp, pose(W, H, k), ref)
        assert np.array_equal(outs[k].download(np.uint8, W * H * 4), ref.download(np.uint8, W * H * 4)), f"frame {k}"
    ctx.close()


def test_prefix_depth_follows_the_blend():
    """Per-tile depths: each blend records how deep its sub-blocks walked every tile list, and the
    next frames keep min(target, 2 x that + 4096) entries of each list.  At C3 static frames keep
    far fewer entries than the first (which knew no depths); a camera sweep (lists deepening and
    shallowing) still gives every image bit for bit as the host-synchronous full sort."""
    W, H = 1920, 1080
    ctx = g.Context(0)
    sp = g.Splats.from_raw(*bicycle_standin_raw(), W, H, ctx=ctx)
    ref = g.DeviceBuffer(ctx, W * H * 4)
    render_sync(sp, pose(W, H, 0), ref)
    assert ctx.set_sort_prefix() == 32768
    ctx.prefix_stats(reset=True)
    out = g.DeviceBuffer(ctx, W * H * 4)
    kept = []
    for _ in range(6):
        render_spec(sp, pose(W, H, 0), out)
        kept.append(ctx.prefix_stats()["kept"])
    assert kept[-1] < kept[0] * 3 // 4, kept
    img0 = out.download(np.uint8, W * H * 4)
    render_sync(sp, pose(W, H, 0), ref)
    assert np.array_equal(img0, ref.download(np.uint8, W * H * 4))
    outs = [g.DeviceBuffer(ctx, W * H * 4) for _ in range(3)]
    ks = [0, 2, 5, 9, 5, 1, 0, 7]
    got = []
    for i, k in enumerate(ks):
        render_spec(sp, pose(W, H, k), outs[i % 3])
        if i % 3 == 2 or i == len(ks) - 1:
            ctx.sync()
            got += [outs[j].download(np.uint8, W * H * 4) for j in range(i % 3 + 1)]
    for i, k in enumerate(ks):
        render_sync(sp, pose(W, H, k), ref)
        assert np.array_equal(got[i], ref.download(np.uint8, W * H * 4)), f"frame {i} (pose {k})"
    ctx.close()


@pytest.mark.parametrize("motion", ["turn", "walk"])
def test_prefix_moving_camera_ignores_stale_depths(motion):
    """A camera turning 3 degrees per frame: the per-tile depths recorded one pose earlier
    describe another view, so those frames select without them (the configured depth) -- no frame
    rendered again (selected with the depths, a 3-degree pan's first three frames missed and
    turned the prefix sort off).  A camera moving 0.1 per frame (the reference's key step,
    src/Camera.cpp:77-101) keeps the depths (they stay close as the content grows; at most one
    frame rendered again).  Every image bit-exact against the host-synchronous full sort."""
    W, H = 1920, 1080
    ctx = g.Context(0)
    sp = g.Splats.from_raw(*bicycle_standin_raw(), W, H, ctx=ctx)
    ref = g.DeviceBuffer(ctx, W * H * 4)

    def pan(k):
        cam = g.main_camera(W, H)
        if motion == "turn":
            cam.rotateRight(3.0 * k)
        else:
            cam.moveForward(0.1 * k)
        return cam.uniforms()

    render_sync(sp, pan(0), ref)
    assert ctx.set_sort_prefix() == 32768
    for _ in range(4):  # static frames first: the depths are recorded, and used
        render_spec(sp, pan(0), ref)
    ctx.sync()
    ctx.prefix_stats(reset=True)
    outs = [g.DeviceBuffer(ctx, W * H * 4) for _ in range(3)]
    got = []
    for k in range(1, 10):
        render_spec(sp, pan(k), outs[(k - 1) % 3])
        if k % 3 == 0:
            ctx.sync()
            got += [o.download(np.uint8, W * H * 4) for o in outs]
    ps = ctx.prefix_stats()
    assert ps["frames"] == 9 and ps["redone"] <= (0 if motion == "turn" else 1), ps
    for k in range(1, 10):
        render_sync(sp, pan(k), ref)
        assert np.array_equal(got[k - 1], ref.download(np.uint8, W * H * 4)), f"pose {k}"
    ctx.close()


def test_prefix_miss_keeps_the_newest_frame_readable():
    """a prefix miss is rendered again after later frames in flight completed.  The
    context's counts and readbacks must then still be the newest frame's (it is rendered again
    after the failed one), not the older re-rendered frame's: frame k (a large scene, 256 entries
    per list: misses), frame k+1 (a small scene, another output), then gs_last_stats and
    gs_frame_read give frame k+1's counts and values, and both images equal the synchronous ones."""
    W, H = 1280, 720
    ctx = g.Context(0)
    big = g.Splats.from_raw(*bicycle_standin_raw(400_000, seed=3), W, H, ctx=ctx)
    small = g.Splats.from_raw(*bicycle_standin_raw(3_000, seed=4), W, H, ctx=ctx)
    u = pose(W, H, 0)
    ref = g.DeviceBuffer(ctx, W * H * 4)
    st_s = render_sync(small, u, ref)
    img_s = ref.download(np.uint8, W * H * 4)
    E_s = int(st_s.entries)
    assert E_s > 0
    vals_s = small.read(g.GS_READ_VALS, E_s)
    st_b = render_sync(big, u, ref)  # the newest count seen: the large scene's (prefix-sorted frames next)
    img_b = ref.download(np.uint8, W * H * 4)
    assert st_b.entries >= 64 * 256 and st_b.entries != st_s.entries
    ctx.set_sort_prefix(256)
    ctx.prefix_stats(reset=True)
    outs = [g.DeviceBuffer(ctx, W * H * 4) for _ in range(2)]
    render_spec(big, u, outs[0])
    render_spec(small, u, outs[1])
    st = small.stats  # gs_last_stats: syncs, re-renders the miss
    assert ctx.prefix_stats()["redone"] >= 1
    assert (st.num_splats, st.visible, st.duplicates, st.entries) == \
        (st_s.num_splats, st_s.visible, st_s.duplicates, st_s.entries)
    assert np.array_equal(small.read(g.GS_READ_VALS, E_s), vals_s)
    assert np.array_equal(outs[0].download(np.uint8, W * H * 4), img_b)
    assert np.array_equal(outs[1].download(np.uint8, W * H * 4), img_s)
    ctx.close()
