"""Frames enqueued without a host round trip (gs_render with no stats and a device output):
the entry count stays on the device and the buffers are sized from the previous count.
These frames must give exactly the pixels of the host-synchronous path, including when
the entries outgrow the buffers (detected at gs_sync and rendered again)."""
import ctypes

import numpy as np
import pytest

import openglgaussiansplattingrenderer_amd as g
from openglgaussiansplattingrenderer_amd import _native as N
from openglgaussiansplattingrenderer_amd._native import check, lib
from openglgaussiansplattingrenderer_amd.scenes import c2_scene

pytestmark = pytest.mark.gpu


def make_splats(ctx, n, seed, W, H):
    rng = np.random.default_rng(seed)
    means = rng.uniform(-2, 2, (n, 3)).astype(np.float32)
    rot = rng.normal(size=(n, 4)).astype(np.float32)
    rot /= np.linalg.norm(rot, axis=1, keepdims=True)
    sc = np.exp(rng.uniform(np.log(0.01), np.log(0.2), (n, 3))).astype(np.float32)
    op = rng.uniform(0.05, 0.99, n).astype(np.float32)
    col = rng.normal(size=(n, 3)).astype(np.float32)
    return g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, W, H, ctx=ctx)


def render_sync(sp, u, out):
    """gs_render with a stats pointer: the host-synchronous path"""
    st = N.gs_frame_stats()
    check(lib().gs_render(sp.ctx.handle, sp._scene, ctypes.byref(u), sp.flags, out.ptr, 1, ctypes.byref(st)),
          sp.ctx.handle)
    return st


def render_spec(sp, u, out):
    check(lib().gs_render(sp.ctx.handle, sp._scene, ctypes.byref(u), sp.flags, out.ptr, 1, None), sp.ctx.handle)


def pose(W, H, k):
    cam = g.main_camera(W, H)
    cam.rotateRight(8.0 * k)  # every pose k < 7 still sees the scene
    return cam.uniforms()


@pytest.mark.parametrize("flags", [0, g.GS_FLAG_CLEAN])
def test_frames_in_flight_match_sync(flags):
    W, H = 512, 384
    ctx = g.Context(0)
    means, rot, sc, op, col = c2_scene()
    sp = g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, W, H, ctx=ctx, flags=flags)
    outs = [g.DeviceBuffer(ctx, W * H * 4) for _ in range(6)]
    render_sync(sp, pose(W, H, 0), outs[0])  # first frame on the ctx: counts seen once
    for k in range(6):  # six frames back to back, more than the 4 slots in flight
        render_spec(sp, pose(W, H, k), outs[k])
    ctx.sync()
    got = [o.download(np.uint8, W * H * 4) for o in outs]
    ref = g.DeviceBuffer(ctx, W * H * 4)
    for k in range(6):
        st = render_sync(sp, pose(W, H, k), ref)
        assert np.array_equal(got[k], ref.download(np.uint8, W * H * 4)), f"pose {k}"
        assert st.entries > 0
    ctx.close()


def test_overflow_renders_again():
    W, H = 640, 480
    ctx = g.Context(0)
    small = make_splats(ctx, 500, 1, W, H)
    big = make_splats(ctx, 200_000, 2, W, H)
    out_s = g.DeviceBuffer(ctx, W * H * 4)
    out_b = g.DeviceBuffer(ctx, W * H * 4)
    u = pose(W, H, 0)
    st_small = render_sync(small, u, out_s)  # sizes the buffers for ~500 splats
    render_spec(big, u, out_b)  # far more entries than that capacity
    ctx.sync()  # detects the overflow and renders the frame again
    got = out_b.download(np.uint8, W * H * 4)
    st = big.stats
    assert st.entries > 4 * (st_small.entries + st_small.entries // 4 + 65536), "the case must overflow"
    ref = g.DeviceBuffer(ctx, W * H * 4)
    st_ref = render_sync(big, u, ref)
    assert st.entries == st_ref.entries and st.visible == st_ref.visible
    assert np.array_equal(got, ref.download(np.uint8, W * H * 4))
    ctx.close()


def test_lookback_giveup_renders_again():
    """the fused preprocess + emission (k_pre_emit, scenes of <= 64k splats) bounds each
    look-back wait; a workgroup that gives up emits at partial offsets and flags the frame (ring
    word 2 = 2), which the host renders again on the synchronous path.  Spin limit 0 makes every
    workgroup after the first give up at once: every frame in flight is redone, and the images
    still equal the synchronous frames; with the limit back, none is"""
    W, H = 512, 384
    ctx = g.Context(0)
    means, rot, sc, op, col = c2_scene()
    sp = g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, W, H, ctx=ctx)
    outs = [g.DeviceBuffer(ctx, W * H * 4) for _ in range(5)]
    render_sync(sp, pose(W, H, 0), outs[0])  # counts seen once
    limit, red0 = ctx.set_lookback_spin(0)
    assert limit == 0
    for k in range(5):
        render_spec(sp, pose(W, H, k), outs[k])
    ctx.sync()
    got = [o.download(np.uint8, W * H * 4) for o in outs]
    _, red1 = ctx.set_lookback_spin(1 << 15)
    assert red1 - red0 >= 1, "the give-up path must have run"
    for k in range(5):
        render_spec(sp, pose(W, H, k), outs[k])
    ctx.sync()
    again = [o.download(np.uint8, W * H * 4) for o in outs]
    assert ctx.set_lookback_spin(-1)[1] == red1, "no frame redone with the default limit"
    ref = g.DeviceBuffer(ctx, W * H * 4)
    for k in range(5):
        render_sync(sp, pose(W, H, k), ref)
        r = ref.download(np.uint8, W * H * 4)
        assert np.array_equal(got[k], r), f"pose {k} (given up)"
        assert np.array_equal(again[k], r), f"pose {k}"
    ctx.close()


def test_staged_calls_after_inflight_frames():
    """the stage API validates frames in flight first (counts on the host, results intact)"""
    W, H = 256, 256
    ctx = g.Context(0)
    means, rot, sc, op, col = c2_scene()
    sp = g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, W, H, ctx=ctx)
    u = pose(W, H, 1)
    out = g.DeviceBuffer(ctx, W * H * 4)
    render_sync(sp, u, out)
    render_spec(sp, u, out)
    E = int(sp.stats.entries)
    keys = sp.read(g.GS_READ_KEYS, E)
    assert np.all(np.diff(keys.astype(np.int64)) >= 0)
    sp._preprocess_u(u)
    sp.computeBins()
    sp.draw(W, H, W / 16.0, H / 16.0)
    img = sp.texture().reshape(-1)
    assert np.array_equal(img, out.download(np.uint8, W * H * 4))
    ctx.close()


def near_camera_splats(ctx, W, H, n=20000, seed=5):
    """splats scattered around the main camera: some land in front of the near plane, giving
    negative keys (Q6) -- a key range far wider than 2^27 bit patterns"""
    u = g.main_camera(W, H).uniforms()
    V = np.array(u.view[:], np.float32).reshape(4, 4).T
    campos = -V[:3, :3].T @ V[:3, 3]
    rng = np.random.default_rng(seed)
    means = (campos + rng.normal(size=(n, 3)) * 1.5).astype(np.float32)
    rot = rng.normal(size=(n, 4)).astype(np.float32)
    log_sc = rng.uniform(np.log(0.01), np.log(0.1), (n, 3)).astype(np.float32)
    op = rng.normal(0, 2, n).astype(np.float32)
    col = rng.normal(size=(n, 3)).astype(np.float32)
    return g.Splats.from_raw(means, col, op, log_sc, rot, W, H, ctx=ctx)


def test_wide_key_range_sorts_all_bits(oracle):
    """a frame whose keys span more than 2^27 bit patterns (negative keys, all four digit
    passes carrying information) sorts bit-exact; the frame sort leaves only the values
    sorted, so reading the keys sorts the frame's entries again -- both must match the oracle"""
    W, H = 512, 384
    ctx = g.Context(0)
    sp = near_camera_splats(ctx, W, H)
    u = g.main_camera(W, H).uniforms()
    out = g.DeviceBuffer(ctx, W * H * 4)
    st = render_sync(sp, u, out)
    E = int(st.entries)
    ref = oracle.render(sp.means3D, sp.covarianceMatrices, sp.opacities, sp.colours, u, flags=0, draw=False)
    # the values as the frame's own sort left them (packed last passes, no keys) ...
    assert np.array_equal(sp.read(g.GS_READ_VALS, E), ref["vals"])
    # ... then the keys, which sorts the frame's entries again with keys, and the values again
    keys = sp.read(g.GS_READ_KEYS, E)
    vals = sp.read(g.GS_READ_VALS, E)
    assert int(keys.max()) - int(keys.min()) >= 1 << 27, "the case must be wide"
    assert np.array_equal(keys, ref["keys"]) and np.array_equal(vals, ref["vals"])
    ctx.close()


def test_wide_key_range_in_flight_renders_again():
    """a frame with a wide key range enqueued without a round trip right after narrow frames,
    and a narrow frame behind it: both images equal their host-synchronous renders"""
    W, H = 512, 384
    ctx = g.Context(0)
    means, rot, sc, op, col = c2_scene()
    narrow = g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, W, H, ctx=ctx)
    wide = near_camera_splats(ctx, W, H)
    u = g.main_camera(W, H).uniforms()
    out_n = g.DeviceBuffer(ctx, W * H * 4)
    out_w = g.DeviceBuffer(ctx, W * H * 4)
    render_sync(narrow, u, out_n)  # narrow key range observed: the next frame sorts in 3 passes
    render_spec(wide, u, out_w)
    render_spec(narrow, u, out_n)  # a frame behind it, rendered again too
    ctx.sync()
    got_w = out_w.download(np.uint8, W * H * 4)
    got_n = out_n.download(np.uint8, W * H * 4)
    ref = g.DeviceBuffer(ctx, W * H * 4)
    render_sync(wide, u, ref)
    assert np.array_equal(got_w, ref.download(np.uint8, W * H * 4))
    render_sync(narrow, u, ref)
    assert np.array_equal(got_n, ref.download(np.uint8, W * H * 4))
    ctx.close()


@pytest.mark.parametrize("lanes", [2, 3])
def test_lanes_keep_frame_order(lanes):
    """consecutive frames rotate over the lanes (streams); blends into one output land in frame
    order, and non-frame work between frames is ordered as on one stream"""
    W, H = 384, 256
    ctx = g.Context(0)
    ctx.set_lanes(lanes)
    means, rot, sc, op, col = c2_scene()
    sp = g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, W, H, ctx=ctx)
    out = g.DeviceBuffer(ctx, W * H * 4)
    ref = g.DeviceBuffer(ctx, W * H * 4)
    render_sync(sp, pose(W, H, 6), ref)
    want_last = ref.download(np.uint8, W * H * 4)
    render_sync(sp, pose(W, H, 0), out)
    for k in range(7):  # the last frame written must be pose 6's
        render_spec(sp, pose(W, H, k), out)
    ctx.sync()
    assert np.array_equal(out.download(np.uint8, W * H * 4), want_last)
    # a memset between frames: after frame A, before frame B (which writes elsewhere)
    other = g.DeviceBuffer(ctx, W * H * 4)
    render_spec(sp, pose(W, H, 1), out)
    check(lib().gs_memset(ctx.handle, out.ptr, 0, W * H * 4), ctx.handle)
    render_spec(sp, pose(W, H, 2), other)
    ctx.sync()
    assert not out.download(np.uint8, W * H * 4).any()
    # the memset's target written again by the next frame: that frame's image
    render_spec(sp, pose(W, H, 3), out)
    ctx.sync()
    render_sync(sp, pose(W, H, 3), ref)
    assert np.array_equal(out.download(np.uint8, W * H * 4), ref.download(np.uint8, W * H * 4))
    ctx.close()


def test_one_and_two_lanes_identical():
    W, H = 512, 384
    imgs = {}
    for lanes in (1, 2, 3):
        ctx = g.Context(0)
        ctx.set_lanes(lanes)
        means, rot, sc, op, col = c2_scene()
        sp = g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, W, H, ctx=ctx)
        outs = [g.DeviceBuffer(ctx, W * H * 4) for _ in range(5)]
        render_sync(sp, pose(W, H, 0), outs[0])
        for k in range(5):
            render_spec(sp, pose(W, H, k), outs[k])
        ctx.sync()
        imgs[lanes] = [o.download(np.uint8, W * H * 4) for o in outs]
        ctx.close()
    for lanes in (2, 3):
        for a, b in zip(imgs[1], imgs[lanes]):
            assert np.array_equal(a, b)
    with pytest.raises(g.GsError):
        ctx = g.Context(0)
        try:
            ctx.set_lanes(4)
        finally:
            ctx.close()


def test_rotating_outputs_keep_per_output_order():
    """blends wait only for frames in flight into the same output: with three outputs rotated
    over two lanes, frame k+3 (lane B) rewrites the output frame k (lane A) wrote -- each output
    must end up holding the newest frame written into it"""
    W, H = 384, 256
    ctx = g.Context(0)
    means, rot, sc, op, col = c2_scene()
    sp = g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, W, H, ctx=ctx)
    outs = [g.DeviceBuffer(ctx, W * H * 4) for _ in range(3)]
    render_sync(sp, pose(W, H, 0), outs[0])
    last = {}
    for k in range(7):
        render_spec(sp, pose(W, H, k), outs[k % 3])
        last[k % 3] = k
    ctx.sync()
    got = [o.download(np.uint8, W * H * 4) for o in outs]
    ref = g.DeviceBuffer(ctx, W * H * 4)
    for i, k in last.items():
        render_sync(sp, pose(W, H, k), ref)
        assert np.array_equal(got[i], ref.download(np.uint8, W * H * 4)), f"output {i} (pose {k})"
    ctx.close()


def test_double_buffered_texture_is_newest_frame():
    """Splats.render_uniforms renders into a back texture and swaps: texture() is the newest
    frame's image"""
    W, H = 384, 256
    ctx = g.Context(0)
    means, rot, sc, op, col = c2_scene()
    sp = g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, W, H, ctx=ctx)
    for k in range(5):
        sp.render_uniforms(pose(W, H, k))
    img = sp.texture().reshape(-1).copy()
    ref = g.DeviceBuffer(ctx, W * H * 4)
    render_sync(sp, pose(W, H, 4), ref)
    assert np.array_equal(img, ref.download(np.uint8, W * H * 4))
    ctx.close()


def test_memset_orders_before_every_lanes_next_frame():
    """three lanes: a memset enqueued after frame A must precede the next frame of EACH other
    lane -- here the second frame after it (on the third lane) rewrites the memset's target"""
    W, H = 384, 256
    ctx = g.Context(0)
    ctx.set_lanes(3)
    means, rot, sc, op, col = c2_scene()
    sp = g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, W, H, ctx=ctx)
    out, other = g.DeviceBuffer(ctx, W * H * 4), g.DeviceBuffer(ctx, W * H * 4)
    ref = g.DeviceBuffer(ctx, W * H * 4)
    render_sync(sp, pose(W, H, 2), ref)
    want = ref.download(np.uint8, W * H * 4)
    render_sync(sp, pose(W, H, 0), out)
    for _ in range(3):
        render_spec(sp, pose(W, H, 1), out)
        check(lib().gs_memset(ctx.handle, out.ptr, 0, W * H * 4), ctx.handle)
        render_spec(sp, pose(W, H, 1), other)  # next lane
        render_spec(sp, pose(W, H, 2), out)    # the lane after: must blend after the memset
        ctx.sync()
        assert np.array_equal(out.download(np.uint8, W * H * 4), want)
    ctx.close()


@pytest.mark.parametrize("seed,flags", [(1, 0), (2, 0), (3, g.GS_FLAG_CLEAN), (4, g.GS_FLAG_FAST_EXP)])
def test_random_frame_sequences_keep_per_output_order(seed, flags):
    """random mixes of frames without a round trip, host-synchronous frames, memsets and lane
    changes over four outputs: each output ends up holding the newest thing written into it
    (the image of the last frame into it, or zeros after a memset)"""
    W, H = 256, 192
    rng = np.random.default_rng(seed)
    ctx = g.Context(0)
    means, rot, sc, op, col = c2_scene()
    sp = g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, W, H, ctx=ctx, flags=flags)
    outs = [g.DeviceBuffer(ctx, W * H * 4) for _ in range(4)]
    render_sync(sp, pose(W, H, 0), outs[0])
    last = {}  # output -> pose, or None for zeros
    for _ in range(80):
        r = rng.random()
        o = int(rng.integers(0, 4))
        if r < 0.6:
            k = int(rng.integers(0, 7))
            render_spec(sp, pose(W, H, k), outs[o])
            last[o] = k
        elif r < 0.75:
            k = int(rng.integers(0, 7))
            render_sync(sp, pose(W, H, k), outs[o])
            last[o] = k
        elif r < 0.9:
            check(lib().gs_memset(ctx.handle, outs[o].ptr, 0, W * H * 4), ctx.handle)
            last[o] = None
        else:
            ctx.set_lanes(int(rng.integers(1, 4)))
    ctx.sync()
    got = [b.download(np.uint8, W * H * 4) for b in outs]
    ref = g.DeviceBuffer(ctx, W * H * 4)
    for o, k in last.items():
        if k is None:
            assert not got[o].any(), f"output {o}: memset expected"
        else:
            render_sync(sp, pose(W, H, k), ref)
            assert np.array_equal(got[o], ref.download(np.uint8, W * H * 4)), f"output {o}: pose {k}"
    ctx.close()


def test_overflow_retired_by_a_larger_scenes_frame():
    """a frame without a round trip that overflowed is retired (and rendered again,
    which moves the ctx to other lanes) by the begin of a later frame of a LARGER scene: that
    frame must size the buffers of the lane it finally runs on -- every image equals its
    host-synchronous render"""
    W, H = 640, 480
    ctx = g.Context(0)
    small = make_splats(ctx, 500, 1, W, H)
    big = make_splats(ctx, 200_000, 2, W, H)
    huge = make_splats(ctx, 400_000, 3, W, H)
    outs = [g.DeviceBuffer(ctx, W * H * 4) for _ in range(6)]
    u = pose(W, H, 0)
    render_sync(small, u, outs[0])              # capacity sized for ~500 splats
    seq = [(big, 1), (small, 2), (small, 3), (small, 4), (huge, 5)]
    for sp, o in seq:                           # big overflows; huge's frame retires it (ring of 4)
        render_spec(sp, u, outs[o])
    ctx.sync()
    got = [b.download(np.uint8, W * H * 4) for b in outs]
    ref = g.DeviceBuffer(ctx, W * H * 4)
    for sp, o in seq:
        render_sync(sp, u, ref)
        assert np.array_equal(got[o], ref.download(np.uint8, W * H * 4)), f"output {o}"
    ctx.close()


@pytest.mark.parametrize("write", ["memset", "upload"])
def test_overflow_then_write_keeps_the_write(write):
    """an overflowed frame is rendered again BEFORE a later memset / upload into its
    output, so the output holds what was written last"""
    W, H = 640, 480
    ctx = g.Context(0)
    small = make_splats(ctx, 500, 1, W, H)
    big = make_splats(ctx, 200_000, 2, W, H)
    out = g.DeviceBuffer(ctx, W * H * 4)
    u = pose(W, H, 0)
    render_sync(small, u, out)
    render_spec(big, u, out)                    # overflows (detected at the next validation)
    pattern = (np.arange(W * H * 4) % 251).astype(np.uint8)
    if write == "memset":
        check(lib().gs_memset(ctx.handle, out.ptr, 0, W * H * 4), ctx.handle)
        want = np.zeros(W * H * 4, np.uint8)
    else:
        out.upload(pattern)
        want = pattern
    ctx.sync()
    assert np.array_equal(out.download(np.uint8, W * H * 4), want)
    ctx.close()


@pytest.mark.parametrize("frames", [1, 2, 3, 4])
def test_set_lanes_keeps_newest_frame_readable(frames):
    """lowering the lane count after frames on three lanes leaves the newest frame's
    buffers addressed (reads return that frame's entries, not another lane's)"""
    W, H = 384, 256
    ctx = g.Context(0)
    ctx.set_lanes(3)
    means, rot, sc, op, col = c2_scene()
    sp = g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, W, H, ctx=ctx)
    out = g.DeviceBuffer(ctx, W * H * 4)
    for k in range(frames):
        st = render_sync(sp, pose(W, H, k), out)
    E = int(st.entries)
    vals = sp.read(g.GS_READ_VALS, E)
    keys = sp.read(g.GS_READ_KEYS, E)
    ctx.set_lanes(1)
    assert np.array_equal(sp.read(g.GS_READ_VALS, E), vals)
    assert np.array_equal(sp.read(g.GS_READ_KEYS, E), keys)
    # and the next frames run on the new lane count
    render_spec(sp, pose(W, H, 5), out)
    ctx.sync()
    ref = g.DeviceBuffer(ctx, W * H * 4)
    render_sync(sp, pose(W, H, 5), ref)
    assert np.array_equal(out.download(np.uint8, W * H * 4), ref.download(np.uint8, W * H * 4))
    ctx.close()


def test_emission_full_batch_of_out_of_rect_mains(oracle):
    """at a width not divisible by 16 (ref mode, Q5) a splat right of column 16*int(W/16)
    has its main tile outside its clamped rect, so ALL rect tiles are duplicates (256 for a
    splat covering the grid); 256 of them in one emission batch give 65536 duplicates -- the
    emission's packed block scan must not wrap"""
    W, H = 1000, 600
    ctx = g.Context(0)
    u = g.main_camera(W, H).uniforms()
    VP = np.array(u.vp[:], np.float64).reshape(4, 4).T
    n = 1024
    rng = np.random.default_rng(11)
    sx = rng.uniform(993.0, 999.0, n)                       # int(W/16) = 62: tileX = 16
    sy = rng.uniform(20.0, 580.0, n)
    ndc = np.stack([2 * sx / W - 1, 2 * sy / H - 1, np.full(n, 0.5), np.ones(n)], 1)
    wpt = (np.linalg.inv(VP) @ ndc.T).T
    means = (wpt[:, :3] / wpt[:, 3:]).astype(np.float32)
    rot = np.tile(np.array([1, 0, 0, 0], np.float32), (n, 1))
    log_sc = np.full((n, 3), np.log(3.0), np.float32)       # covers the whole grid
    op = np.full(n, -3.0, np.float32)                        # sigmoid: ~0.047 (slow saturation)
    col = rng.normal(size=(n, 3)).astype(np.float32)
    sp = g.Splats.from_raw(means, col, op, log_sc, rot, W, H, ctx=ctx)
    out = g.DeviceBuffer(ctx, W * H * 4)
    st = render_sync(sp, u, out)
    ref = oracle.render(sp.means3D, sp.covarianceMatrices, sp.opacities, sp.colours, u, flags=0)
    assert int(st.duplicates) >= 256 * 256, "the case must fill a batch with 256-duplicate splats"
    assert int(st.entries) == ref["E"]
    E = int(st.entries)
    assert np.array_equal(sp.read(g.GS_READ_VALS, E), ref["vals"])
    assert np.array_equal(sp.read(g.GS_READ_KEYS, E), ref["keys"])
    assert np.array_equal(out.download(np.uint8, W * H * 4), ref["image"].reshape(-1))
    ctx.close()
