#!/usr/bin/env python
"""bench.py -- frames/s at 1920x1080 on the bicycle-sized scene (+ radix-sort Gkeys/s), with
the HBM roofline of the dominant kernel and a bounded CPU-oracle baseline.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c4|c2] [--clean] [--fast-exp] [--lanes 1|2]

One frame = one step of the hot path (preprocess -> sort -> bins -> blend) over the
resident scene (BASELINE.json configs[2]: 6,131,954 splats at 1920x1080; the real bicycle
point_cloud.ply when $GS_BICYCLE_PLY names it, else the seeded synthetic stand-in).
Multi-GPU = replicas: rank k renders its own view (main.cpp pose + rotateRight(45 deg * k))
of its own copy of the scene; no collective on the data path.  Barrier +
device sync around exactly K timed frames; max time over ranks; rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
METRIC = "frames/s @1080p (bicycle ~6M splats) + radix-sort Gkeys/s; %HBM peak"
SORT_N = 32 * 16 * 10000 - 7  # tests/sortTests.cpp:181

CONFIGS = {
    "c3": dict(W=1920, H=1080, desc="C3: bicycle-sized scene, 1920x1080, 1 view per GPU"),
    "c4": dict(W=3840, H=2160, desc="C4: bicycle-sized scene, 3840x2160, 1 view per GPU"),
    "c2": dict(W=512, H=512, desc="C2: 10k synthetic splats, 512x512"),
}


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* in their environment, 127.0.0.1 rendezvous) and wait for them.  The
    parent never touches the GPU (no HIP call before the children exist); rank 0 prints the
    JSON line.  A failing rank ends the others (they would wait at a barrier)."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in live:  # the exact children we started
                    q.terminate()
        time.sleep(0.05)
    return rc


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    pg = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # timing / barrier plumbing only: gloo on the host (there is no data-path collective).
        # Gloo prints its connection lines on fd 1; they go to stderr so that stdout holds the
        # JSON line alone.
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world)
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
        pg = dist
    return world, rank, local, pg


def barrier(pg):
    if pg is not None:
        pg.barrier()


def max_over_ranks(pg, x: float) -> float:
    if pg is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(pg, x: float) -> float:
    if pg is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.SUM)
    return float(t.item())


def load_scene(cfg: str, W: int, H: int, ctx, flags: int):
    import openglgaussiansplattingrenderer_amd as g
    from openglgaussiansplattingrenderer_amd.scenes import BICYCLE_N, bicycle_standin_raw, c2_scene
    if cfg == "c2":
        means, rot, sc, op, col = c2_scene()
        sp = g.Splats.from_raw(means, col, np.log(op / (1 - op)), np.log(sc), rot, W, H, ctx=ctx, flags=flags)
        return sp, "synthetic (C2 generator, seed 20240101)"
    path = os.environ.get("GS_BICYCLE_PLY")
    if path and os.path.exists(path):
        return g.Splats(path, W, H, ctx=ctx, flags=flags), f"bicycle point_cloud.ply ({path})"
    raw = bicycle_standin_raw(BICYCLE_N)
    return g.Splats.from_raw(*raw, W, H, ctx=ctx, flags=flags), \
        f"synthetic stand-in for bicycle ({BICYCLE_N:,} splats, seeded; no checkpoint available)"


def camera_for_rank(W: int, H: int, rank: int):
    import openglgaussiansplattingrenderer_amd as g
    cam = g.main_camera(W, H)
    cam.rotateRight(45.0 * rank)  # C5: pose k = main pose + rotateRight(45 deg * k)
    return cam


def sort_bench(ctx, reps: int = 50, warm: int = 5):
    """radix-sort Gkeys/s on the sortTests input (5,119,993 srand(20) keys), GPURadixSort
    semantics (argsort of float keys); median of `reps` hipEvent-timed sorts."""
    import openglgaussiansplattingrenderer_amd as g
    from openglgaussiansplattingrenderer_amd.splats import createRandomNumbersFloat
    keys = createRandomNumbersFloat(SORT_N)
    iota = np.arange(SORT_N, dtype=np.int32)
    kb = g.DeviceBuffer.from_array(ctx, keys)
    ob = g.DeviceBuffer.from_array(ctx, iota)
    ms = []
    for i in range(warm + reps):
        ob.upload(iota)
        g.GPURadixSort(1, 3, 2, None, ob, None, SORT_N, 16, 32, kb)
        t = ctx.last_kernel_ms(g.GS_KERNEL_SORT)
        if i >= warm:
            ms.append(t)
    out = ob.download(np.int32, SORT_N)
    s = keys[out]
    ok = bool(np.all(s[1:] >= s[:-1]))
    # pair sort of the same keys (32-bit key + 32-bit payload): the renderer's sort
    kbits = keys.view(np.uint32)
    k2 = g.DeviceBuffer.from_array(ctx, kbits)
    v2 = g.DeviceBuffer.from_array(ctx, iota)
    ms_pairs = []
    for i in range(warm + reps):
        k2.upload(kbits)
        v2.upload(iota)
        g.sort_pairs(ctx, k2, v2, SORT_N)
        t = ctx.last_kernel_ms(g.GS_KERNEL_SORT)
        if i >= warm:
            ms_pairs.append(t)
    med = float(np.median(ms))
    medp = float(np.median(ms_pairs))
    out = dict(n=SORT_N, ms_argsort=med, gkeys_per_s=SORT_N / med / 1e6, ms_pairs=medp,
               gkeys_per_s_pairs=SORT_N / medp / 1e6,
               hbm_frac_pairs_cache_resident=68.0 * SORT_N / (medp * 1e-3) / 1e9 / HBM_PEAK_GBS,
               cache_resident_note="5.12M pairs = 41 MB (82 MB with the alternate buffers) sit inside the 256 MiB "
                                   "Infinity Cache: an L2/MALL figure, not an HBM one",
               sorted_ok=ok)
    del kb, ob, k2, v2
    out["beyond_cache"] = sort_bench_big(ctx)
    return out


SORT_BIG_N = 64 << 20  # 64M pairs: 512 MB of (key, value), 1.28 GB with the alternate buffers


def sort_bench_big(ctx, reps: int = 8, warm: int = 2):
    """The same pair sort beyond the caches: 64M uniform 32-bit keys (HBM-resident), median of
    `reps` hipEvent-timed sorts; algorithmic bytes 68 B/key; counter-based bytes from
    the newest committed rocprofv3 collection of this sort (profiles/rNN/sort_64M_pmc.json)."""
    import openglgaussiansplattingrenderer_amd as g
    n = SORT_BIG_N
    rng = np.random.default_rng(64)
    keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    vals = np.arange(n, dtype=np.uint32)
    kb = g.DeviceBuffer.from_array(ctx, keys)
    vb = g.DeviceBuffer.from_array(ctx, vals)
    ms = []
    for i in range(warm + reps):
        kb.upload(keys)
        vb.upload(vals)
        g.sort_pairs(ctx, kb, vb, n)
        t = ctx.last_kernel_ms(g.GS_KERNEL_SORT)
        if i >= warm:
            ms.append(t)
    k_out = kb.download(np.uint32, n)
    v_out = vb.download(np.uint32, n)
    # sorted, and the values a stable permutation carrying each key (vals were 0..n-1)
    ok = bool(np.all(k_out[1:] >= k_out[:-1]) and np.all(v_out < n)
              and np.array_equal(keys[np.minimum(v_out, n - 1)], k_out)
              and np.all((k_out[1:] != k_out[:-1]) | (v_out[1:] > v_out[:-1])))
    med = float(np.median(ms))
    out = dict(n=n, keys="uniform 32-bit, seeded", ms_pairs=round(med, 4), gkeys_per_s=round(n / med / 1e6, 2),
               hbm_frac_algorithmic=round(68.0 * n / (med * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), sorted_ok=ok,
               source="hipEvents around gs_sort_pairs_u32, median of %d; 68 B/key algorithmic" % reps)
    # counter bytes per key of this sort, from the newest committed PMC collection of it
    # (profiles/rNN/sort_64M_pmc.json: FETCH_SIZE x2 + WRITE_SIZE of one sort's kernels / n)
    p = newest_profile("sort_64M_pmc.json")
    if p:
        try:
            b = float(json.load(open(p))["counter_bytes_per_key"])
            out["counter_bytes_per_key"] = round(b, 2)
            out["hbm_frac_counters"] = round(b * n / (med * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            out["counter_source"] = os.path.relpath(p, ROOT)
        except Exception:
            pass
    return out


def sort_bench_c3(ctx, sp, u, reps: int = 20, warm: int = 3):
    """The reference's per-frame work on the C3 frame's own key set: every (key, value) pair the
    frame emits, sorted in full (GPURadixSort orders all entries each frame, src/sort.cpp:139-203)
    by the standalone pair sort (12 kernels, keys and values out).  The entries are the emission's
    (the staged preprocess, before gs_sort: splat-major order, keys tile + z01)."""
    import openglgaussiansplattingrenderer_amd as g
    sp._preprocess_u(u)
    E = int(sp.stats.entries)
    keys = sp.read(g.GS_READ_KEYS, E)
    vals = sp.read(g.GS_READ_VALS, E)
    kb = g.DeviceBuffer.from_array(ctx, keys)
    vb = g.DeviceBuffer.from_array(ctx, vals)
    ms = []
    for i in range(warm + reps):
        kb.upload(keys)
        vb.upload(vals)
        g.sort_pairs(ctx, kb, vb, E)
        t = ctx.last_kernel_ms(g.GS_KERNEL_SORT)
        if i >= warm:
            ms.append(t)
    k_out = kb.download(np.uint32, E)
    v_out = vb.download(np.uint32, E)
    perm = np.argsort(keys, kind="stable")
    ok = bool(np.array_equal(k_out, keys[perm]) and np.array_equal(v_out, vals[perm]))
    med = float(np.median(ms))
    del kb, vb
    return dict(n=E, keys="the C3 frame's emitted (tile + depth) keys, splat ids as values", ms_pairs=round(med, 4),
                gkeys_per_s=round(E / med / 1e6, 2),
                hbm_frac_algorithmic=round(68.0 * E / (med * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), sorted_ok=ok,
                note="80 MB of pairs (160 MB with the alternate buffers): inside the 256 MiB Infinity Cache, so "
                     "the rate is partly a cache figure",
                source="hipEvents around gs_sort_pairs_u32 (12 kernels), median of %d; 68 B/key algorithmic" % reps)


SWEEP_FRAMES = {"turn": 20, "walk": 40}  # fixed, whatever --steps is: every run measures the same poses


def camera_sweep(ctx, sp, W: int, H: int, view: int, lanes: int, static_fps: float,
                 motions=(("turn", 0.5), ("turn", 3.0), ("walk", 0.1))):
    """The reference's loop moves the camera every frame (main.cpp:52-89 calls getInput at :76,
    src/Camera.cpp:77-119).  Pose k = the static pose + rotateRight(delta * k): an interactive
    (0.5 deg / frame: a 9.5 deg pan) and a fast (3 deg / frame: 57 deg) pan, 20 frames each, and
    moveForward(0.1 * k) (the reference's key step), 40 frames -- the same poses whatever --steps
    is; on `lanes` frames in flight, with the prefix sort (the per-tile depths carried from frame
    to frame) and with every frame fully sorted; each run starts from a cold depth table, whose
    first frame is also timed alone (one lane)."""
    base = ctx.set_sort_prefix()
    out = {}
    for kind, d in motions:
        n = SWEEP_FRAMES[kind]
        poses = []
        for k in range(n):
            cam = camera_for_rank(W, H, view)
            if kind == "turn":
                cam.rotateRight(d * k)
            else:
                cam.moveForward(d * k)
            poses.append(cam.uniforms())
        if kind == "turn":
            row = {"deg_per_frame": d, "frames": n, "pan_deg": round(d * (n - 1), 2)}
        else:
            row = {"units_per_frame": d, "frames": n, "walk_units": round(d * (n - 1), 2)}
        for mode, tgt in (("prefix", base), ("full_sort", 0)):
            ctx.set_sort_prefix(0)
            ctx.set_lanes(1)
            sp.render_uniforms(poses[0])  # buffers sized for the first pose (the last run ended elsewhere)
            ctx.sync()
            ctx.set_sort_prefix(tgt)  # (clears the per-tile depths: a cold start)
            t0 = time.perf_counter()
            sp.render_uniforms(poses[0])
            ctx.sync()
            first_ms = (time.perf_counter() - t0) * 1e3
            ctx.set_lanes(lanes)
            ctx.prefix_stats(reset=True)
            ctx.sync()
            t0 = time.perf_counter()
            for uu in poses:
                sp.render_uniforms(uu)
            ctx.sync()
            dt = time.perf_counter() - t0
            ps = ctx.prefix_stats()
            row[mode] = {"frames_per_s": round(n / dt, 2), "vs_static": round(n / dt / static_fps, 4),
                         "cold_first_frame_ms": round(first_ms, 4),
                         "prefix_frames": ps["frames"], "rendered_again": ps["redone"],
                         "kept_frac_last": round(ps["kept"] / max(1, ps["entries"]), 4),
                         "E_last": int(sp.stats.entries)}
        # the same poses rendered static (warm depth table, 60 frames each at 5 poses along the pan):
        # the moving camera's frames/s against what those poses give without motion
        ctx.set_lanes(lanes)
        n_tot, t_tot, per_pose = 0, 0.0, {}
        for k in sorted({0, (n - 1) // 4, (n - 1) // 2, 3 * (n - 1) // 4, n - 1}):
            ctx.set_sort_prefix(base)
            for _ in range(10):
                sp.render_uniforms(poses[k])
            ctx.sync()
            t0 = time.perf_counter()
            for _ in range(60):
                sp.render_uniforms(poses[k])
            ctx.sync()
            dt = time.perf_counter() - t0
            per_pose[f"{d * k:g}{'deg' if kind == 'turn' else 'units'}"] = round(60 / dt, 1)
            t_tot += dt
            n_tot += 60
        st = n_tot / t_tot
        row["static_same_poses_fps"] = round(st, 2)
        row["static_per_pose_fps"] = per_pose
        for mode in ("prefix", "full_sort"):
            row[mode]["vs_static_same_poses"] = round(row[mode]["frames_per_s"] / st, 4)
        out[f"{d:g}deg" if kind == "turn" else f"walk{d:g}"] = row
    ctx.set_sort_prefix(base)
    out["source"] = ("host wall clock around the frames (gs_sync after the last); vs_static = frames/s over the "
                     "static headline's value from the same run; static_same_poses_fps: 60 frames each of 5 poses along the "
                     "pan rendered without motion (prefix sort, warm depth table), frames over total time, and "
                     "vs_static_same_poses the sweep against it; cold_first_frame_ms: the first pose alone, one "
                     "lane, host wall clock around gs_render + gs_sync")
    return out


def py_main_loop(ctx, sp, u, frames: int, warmup: int, serial: bool) -> float:
    """The C++ facade's loops (apps/gs_main_loop.cpp) through the Python package: warm-up frames,
    then `frames` frames of render_uniforms, gs_sync after each one (serial) or after the last
    (ahead); host wall clock, no timing events.  Frames per second."""
    for _ in range(warmup):
        sp.render_uniforms(u)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(frames):
        sp.render_uniforms(u)
        if serial:
            ctx.sync()
    ctx.sync()
    return frames / (time.perf_counter() - t0)


def cpp_facade(ctx, sp, u, W: int, H: int, frames: int, warmup: int, lanes: int, py_fps: float, E_py: int):
    """The kept C++ API (include/gsplat_splats.hpp) in the reference's own loop shape (main.cpp:40-89:
    Camera, Splats(path, W, H), then per frame the pose update, Splats::gpuRender, display), built as
    openglgaussiansplattingrenderer_amd/lib/gs_main_loop: the same scene written as a ply (raw fields,
    tests/plyFileGenerator.py layout, scenes.write_raw_ply; the facade's loader activates it as
    from_raw does) and loaded
    through the three-argument constructor; frames one at a time (finish() per frame, as main.cpp
    blocks on its timestamp query) and enqueued ahead on `lanes` lanes, host wall clock."""
    import shutil
    import subprocess
    import tempfile
    from openglgaussiansplattingrenderer_amd.scenes import BICYCLE_N, bicycle_standin_raw, write_raw_ply
    exe = os.path.join(ROOT, "openglgaussiansplattingrenderer_amd", "lib", "gs_main_loop")
    if not os.path.exists(exe) or sp.numSplats != BICYCLE_N or os.environ.get("GS_BICYCLE_PLY"):
        return None
    d = tempfile.mkdtemp(prefix="gs_facade_")
    # like for like: the same timing mode on both sides (GS_TIMING_FRAME: gs_main_loop sets it, as
    # main.cpp:52-58 queries one timestamp per frame) and the two sides alternated, Python / C++ /
    # Python / C++, so neither runs only first or only last
    ctx.timing_enable(0)  # GS_TIMING_FRAME
    runs, py_runs = [], []
    try:
        means, f_dc, logit, log_sc, rot = bicycle_standin_raw(BICYCLE_N)
        ply = os.path.join(d, "c3_standin.ply")
        write_raw_ply(ply, means, f_dc, logit, log_sc, rot)
        for _ in range(2):
            py_runs.append((py_main_loop(ctx, sp, u, frames, warmup, True),
                            py_main_loop(ctx, sp, u, frames, warmup, False)))
            r = subprocess.run([exe, ply, str(W), str(H), str(frames), str(warmup), str(lanes)], capture_output=True,
                               text=True, timeout=300)
            if r.returncode != 0:
                return {"error": (r.stdout + r.stderr)[-400:]}
            runs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    finally:
        shutil.rmtree(d, ignore_errors=True)
    out = dict(runs[-1])
    out["serial_fps"] = round(float(np.mean([x["serial_fps"] for x in runs])), 3)
    out["ahead_fps"] = round(float(np.mean([x["ahead_fps"] for x in runs])), 3)
    out["serial_ms_per_frame"] = round(1e3 / out["serial_fps"], 4)
    out["ahead_ms_per_frame"] = round(1e3 / out["ahead_fps"], 4)
    out["cpp_runs"] = [{"serial_fps": x["serial_fps"], "ahead_fps": x["ahead_fps"]} for x in runs]
    out["E_matches_python"] = all(x.get("E") == E_py for x in runs)
    py_serial = float(np.mean([a for a, _ in py_runs]))
    py_ahead = float(np.mean([b for _, b in py_runs]))
    out["python_runs"] = [{"serial_fps": round(a, 3), "ahead_fps": round(b, 3)} for a, b in py_runs]
    out["python_serial_fps"] = round(py_serial, 3)
    out["python_ahead_fps"] = round(py_ahead, 3)
    out["serial_vs_python"] = round(out["serial_fps"] / py_serial, 4)
    out["ahead_vs_python"] = round(out["ahead_fps"] / py_ahead, 4)
    out["ahead_vs_headline"] = round(out["ahead_fps"] / py_fps, 4)
    out["source"] = ("lib/gs_main_loop (apps/gs_main_loop.cpp): gs::Camera + gs::Splats(path, W, H) + gpuRender per "
                     "frame + present(); serial = finish() after every frame; ahead = frames enqueued on the lanes, "
                     "finish() after the last; host wall clock, timing mode GS_TIMING_FRAME.  python_*: the same "
                     "loops through the Python package (render_uniforms, gs_sync per frame / after the last), same "
                     "timing mode; the sides alternated Python, C++, Python, C++ and each averaged over its two runs; "
                     "ahead_vs_headline: against this run's headline value (its timed region carries draw events)")
    return out


def copy_peak(ctx, nbytes: int = 1 << 30, reps: int = 10):
    """stream-copy rate of this GPU in this run (gs_stream_copy_gbs: non-temporal float4 copy of
    1 GiB, one per lane, read + write bytes): the practical HBM ceiling beside the 8 TB/s spec"""
    import ctypes
    from openglgaussiansplattingrenderer_amd import _native as native
    med, best = ctypes.c_double(), ctypes.c_double()
    native.check(native.lib().gs_stream_copy_gbs(ctx.handle, nbytes, reps, ctypes.byref(med), ctypes.byref(best)),
                 ctx.handle)
    return dict(gbs_median=round(med.value, 1), gbs_best=round(best.value, 1), bytes=nbytes, reps=reps,
                source="gs_stream_copy_gbs: non-temporal float4 copy (one per lane) between two 1 GiB buffers, hipEvents, "
                       "(read + write bytes) / time, median of %d" % reps)


def cpu_baseline(sp, u, flags, budget_s: float = 20.0):
    """CPU oracle on the host cores, bounded: full preprocess + emit + sort + bins of the
    same frame, blend on every row_step-th pixel row (time scaled by row_step)."""
    from oracle import oracle as O
    O.build()
    probe = O.time_frame(sp.means3D, sp.covarianceMatrices, sp.opacities, sp.colours, u, flags=flags,
                         row_step=max(1, u.height // 4))
    fixed = probe["preprocess_s"] + probe["sort_s"] + probe["bins_s"]
    per_row = probe["draw_sample_s"] / max(1, len(range(0, u.height, probe["row_step"])))
    rows = int(max(1, min(u.height, (budget_s - fixed) / max(per_row, 1e-6))))
    step = max(1, u.height // rows)
    r = O.time_frame(sp.means3D, sp.covarianceMatrices, sp.opacities, sp.colours, u, flags=flags, row_step=step)
    return dict(value=1.0 / r["frame_est_s"], unit="frames/s", cores=int(r["threads"]), kind="port",
                sample=(f"oracle/gs_oracle.c (OpenMP, {r['threads']} threads) on the same frame: full preprocess+emit "
                        f"({r['preprocess_s']:.2f}s), stable sort ({r['sort_s']:.2f}s), bins; blend of every "
                        f"{step}th pixel row ({r['draw_sample_s']:.2f}s) scaled x{step} -> {r['frame_est_s']:.2f}s/frame"),
                detail=r)


def newest_profile(name: str):
    """the newest round's committed collection of `name` (profiles/rNN/name), or None"""
    import glob
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]", name)))
    return cands[-1] if cands else None


def load_pmc(kernel: str, field: str = "hbm_bytes_per_launch"):
    """From the newest round's committed rocprofv3 PMC summary (profiles/rNN/pmc_summary.json,
    `tools/gpu_run.sh profiles rNN`): HBM traffic per launch (FETCH_SIZE x2 for streams, x1 for
    the blend's calibrated gathers, + WRITE_SIZE), or another field ("sq": the SQ counters per
    dispatch); None if absent."""
    p = newest_profile("pmc_summary.json")
    if not p:
        return None
    try:
        d = json.load(open(p))
        return d.get(kernel, {}).get(field)
    except Exception:
        return None


def pmc_source() -> str | None:
    p = newest_profile("pmc_summary.json")
    return os.path.relpath(p, ROOT) if p else None


SIMDS = 1024            # 256 CUs x 4 SIMDs (MI355X_MICROARCH.md)
CLOCK_GHZ = 2.4         # peak engine clock
VALU_CYC = 2            # cycles per wave64 VALU instruction at full issue (v_fma_f32 row)
SHADER_ENGINES = 32     # SQ_BUSY_CYCLES is summed over them


def issue_ceiling(kernel: str, launch_ms: float):
    """The blend is bound by vector-instruction issue, not HBM.  Two views from the SQ pass
    (the newest profiles/rNN/pmc_summary.json, same collection as the traffic):
      * naive: SQ_INSTS_VALU at one wave64 VALU per SIMD every 2 cycles at 2.4 GHz -- a lower
        bound on the issue time, since most of the blend's instructions cost more than v_fma_f32
        (tools/micro/valu_cost.hip: v_readlane / v_cmp to an SGPR 1.7x, v_mbcnt / v_cndmask /
        v_med3 1.5x, packed fp32 1.8x, v_exp_f32 2.8x at 6 waves per SIMD);
      * vector-ALU occupancy: SQ_ACTIVE_INST_VALU (quad-cycles) x 4 over the SIMD-cycles of the
        dispatch (SQ_BUSY_CYCLES / 32 shader engines x 1024 SIMDs): the fraction of the kernel's
        time its VALU instructions occupy the SIMDs at one quad-cycle each."""
    sq = load_pmc(kernel, "sq")
    if not sq or not sq.get("SQ_INSTS_VALU"):
        return None
    v = float(sq["SQ_INSTS_VALU"])
    ceil_ms = v * VALU_CYC / (SIMDS * CLOCK_GHZ * 1e9) * 1e3
    out = {"valu_insts_per_launch": v, "salu_insts_per_launch": sq.get("SQ_INSTS_SALU"),
           "ceiling_ms": round(ceil_ms, 4), "frac": round(ceil_ms / launch_ms, 4),
           "source": "SQ_INSTS_VALU per launch (%s) x 2 cyc / (1024 SIMDs x 2.4 GHz)" % pmc_source()}
    act, busy = sq.get("SQ_ACTIVE_INST_VALU"), sq.get("SQ_BUSY_CYCLES")
    if act and busy:
        simd_cycles = float(busy) / SHADER_ENGINES * SIMDS
        out["valu_occupancy"] = round(4.0 * float(act) / simd_cycles, 4)
        out["valu_occupancy_source"] = ("SQ_ACTIVE_INST_VALU x 4 / (SQ_BUSY_CYCLES / 32 x 1024): SIMD time the "
                                        "blend's VALU instructions occupy, one quad-cycle each")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--clean", action="store_true", help="GS_FLAG_CLEAN: reference quirks fixed")
    ap.add_argument("--fast-exp", action="store_true", help="GS_FLAG_FAST_EXP: hardware exp in the blend")
    ap.add_argument("--sh", action="store_true", help="GS_FLAG_SH: degree-3 SH colours (SURVEY f3, beyond the "
                    "reference; seeded synthetic f_rest)")
    ap.add_argument("--lanes", type=int, default=3, choices=(1, 2, 3),
                    help="frames in flight per GPU (gs_ctx_set_lanes): 2 overlaps frame k+1's preprocess / "
                         "emission / sort with frame k's blend, 3 (default here) also the blends' tails")
    ap.add_argument("--view", type=int, default=None,
                    help="C5 pose index to render (default: this rank's, main pose + rotateRight(45 deg * k))")
    ap.add_argument("--draw-sub", type=int, default=0, choices=(0, 8, 16),
                    help="the blend's sub-block form (gs_ctx_set_draw_sub): 0 by entry count (default), 8, 16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sort-bench", action="store_true")
    ap.add_argument("--no-sweep", action="store_true", help="skip the moving-camera frames (frame.camera_sweep)")
    ap.add_argument("--no-facade", action="store_true", help="skip the C++ facade loop (frame.cpp_facade)")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--dry-run", action="store_true",
                    help="rank plumbing only (spawn / rendezvous / per-rank pose / barrier / gather), no GPU: "
                         "prints a dry-run line, not a measurement (tests/test_dist_cpu.py)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world, rank, local, pg = dist_setup()
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; reporting {world} rank(s)", file=sys.stderr)
    if args.dry_run:
        if os.environ.get("GS_BENCH_DRYRUN_FAIL_RANK") == str(rank):  # tests: a rank that dies
            sys.exit(3)
        view = rank if args.view is None else args.view
        cfg = CONFIGS[args.config]
        u = camera_for_rank(cfg["W"], cfg["H"], view).uniforms()
        barrier(pg)
        mine = {"rank": rank, "local_rank": local, "view": view, "view_matrix": [round(x, 6) for x in u.view]}
        ranks = [mine]
        if pg is not None:
            ranks = [None] * world
            pg.all_gather_object(ranks, mine)
        mx = max_over_ranks(pg, float(rank + 1))
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "max_over_ranks": mx, "ranks": ranks}), flush=True)
        if pg is not None:
            pg.destroy_process_group()
        return
    import openglgaussiansplattingrenderer_amd as g

    cfg = CONFIGS[args.config]
    W, H = cfg["W"], cfg["H"]
    flags = ((g.GS_FLAG_CLEAN if args.clean else 0) | (g.GS_FLAG_FAST_EXP if args.fast_exp else 0) |
             (g.GS_FLAG_SH if args.sh else 0))
    # one GPU per rank; ranks beyond the node's GPUs share them round-robin (labelled below)
    import ctypes
    from openglgaussiansplattingrenderer_amd import _native as native
    ndev = ctypes.c_int(0)
    native.lib().gs_device_count(ctypes.byref(ndev))
    ndev = max(1, ndev.value)
    ctx = g.Context(local % ndev)
    ctx.set_lanes(args.lanes)
    ctx.set_draw_sub(args.draw_sub)
    sp, data_desc = load_scene(args.config, W, H, ctx, flags)
    if args.sh:
        rng = np.random.default_rng(4242)
        f_dc = ((sp.colours[:, :3] / 255.0 - 0.5) / 0.28209479177387814).astype(np.float32)
        sp.set_sh(f_dc, rng.normal(0, 0.1, (sp.numSplats, 45)).astype(np.float32))
        data_desc += "; seeded synthetic f_rest N(0, 0.1^2)"
    view = rank if args.view is None else args.view
    u = camera_for_rank(W, H, view).uniforms()

    # one frame at a time (gs_ctx_set_lanes 1), measured before the timed region: the frame
    # latency, then the per-stage breakdown (the same frames with every stage boundary timed,
    # stages not sharing the GPU with the next frame's)
    nser = max(5, min(args.steps, 50))
    ctx.set_lanes(1)
    for _ in range(2):
        sp.render_uniforms(u)
    ctx.sync()
    ctx.timing_enable(g.GS_TIMING_DRAW)
    ctx.timing_reset()
    ts0 = time.perf_counter()
    for _ in range(nser):
        sp.render_uniforms(u)
    ctx.sync()
    serial_ms = (time.perf_counter() - ts0) / nser * 1e3
    tm_serial = ctx.timing_read()
    ctx.timing_enable(g.GS_TIMING_STAGES)
    ctx.timing_reset()
    for _ in range(nser):
        sp.render_uniforms(u)
    tm = ctx.timing_read()

    # the timed region: W warmup frames, then exactly K frames between barriers and device
    # syncs, on args.lanes frames in flight; every frame carries only its draw kernel's
    # start/stop events (each hipEvent idles the stream a few microseconds)
    ctx.set_lanes(args.lanes)
    ctx.timing_enable(g.GS_TIMING_DRAW)
    for _ in range(args.warmup):
        sp.render_uniforms(u)
    ctx.sync()
    barrier(pg)
    ctx.timing_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sp.render_uniforms(u)
    t_enq = time.perf_counter()
    ctx.sync()
    t1 = time.perf_counter()
    barrier(pg)
    local_s = t1 - t0
    elapsed = max_over_ranks(pg, local_s)
    tm_draw = ctx.timing_read()
    ps = ctx.prefix_stats()  # the prefix sort over the timed and untimed frames (gs_prefix_stats)
    prefix = {"target": ctx.set_sort_prefix(), "frames": ps["frames"], "rendered_again": ps["redone"],
              "kept_entries": ps["kept"], "entries": ps["entries"],
              "kept_frac": round(ps["kept"] / max(1, ps["entries"]), 4),
              "source": "gs_prefix_stats: each tile list sorted >= target entries deep; a frame whose blend "
                        "reaches an unsorted position is rendered again with the full sort"}
    host = {"enqueue_ms_per_frame": round((tm_draw["ms_host_render"] - tm_draw["ms_host_wait"]) /
                                          max(1, tm_draw["host_renders"]), 4),
            "blocked_ms_per_frame": round(tm_draw["ms_host_wait"] / max(1, tm_draw["host_renders"]), 4),
            "python_loop_ms_per_frame": round((t_enq - t0) / args.steps * 1e3, 4),
            "source": "host wall time inside gs_render (libgsplat_hip), minus its waits on frames in flight"}
    st = sp.stats
    N, V, D, E = int(st.num_splats), int(st.visible), int(st.duplicates), int(st.entries)
    frames_total = world * args.steps
    value = frames_total / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # per-stage average device time over the timed frames (hipEvents on the ctx stream)
    nf = max(1, tm["frames"])
    stage_ms = {k[3:]: tm[k] / nf for k in ("ms_preprocess", "ms_emit", "ms_sort", "ms_bins", "ms_draw")}
    # algorithmic bytes per launch, fp32 SoA, 4-B payload; a prefix-sorted frame's
    # sort: 4 B/entry (pass-0 key read for the histograms) + 16 B/entry (pass-0 pairs in and the
    # kept pairs out, charged at every entry) + 48 B per kept entry (passes 1-3), else 68 B/entry
    kept = int(ps["kept"]) if ps["frames"] and ps["entries"] == E else 0
    sort_bytes = 4 * E + 16 * E + 48 * kept if kept else 68 * E
    alg = {
        "preprocess": 40 * N + 24 * V,
        "emit": 8 * E,
        "sort": sort_bytes,
        "bins": 4 * E + 1024,
        "draw": 40 * E + 4 * W * H,
    }
    draw_ms_live = tm_draw["ms_draw"] / max(1, tm_draw["frames"])  # timed region, HIP events
    one_ms = tm_serial["ms_draw"] / max(1, tm_serial["frames"])    # frames one at a time
    # the dominant kernel: the longest stage of the one-lane stage pass (one rank per GPU); with
    # ranks sharing a GPU that pass overlaps other ranks' work, so the blend is taken as measured
    # on a GPU of its own in round 2 (profiles/r02: k_draw is the longest kernel at every config)
    if world <= ndev:
        dom = max(("preprocess", "emit", "sort", "draw"), key=lambda k: stage_ms[k])
        dom_source = "longest stage of the one-lane stage-timing pass"
    else:
        dom = "draw"
        dom_source = "fixed to the blend: ranks share a GPU, so the stage pass is not one kernel's time"
    kern_name = {"preprocess": "k_preprocess", "emit": "k_emit", "sort": "k_downsweep", "bins": "k_bins_count",
                 "draw": "k_draw"}[dom]
    # avg_launch_ms: the kernel with the GPU to itself (frames one at a time, hipEvents on its own
    # dispatch) -- what a rocprofv3 kernel trace of the one-lane pass reports for it
    # (profiles/r03/); the timed region's launches share the GPU with the other frames' kernels and
    # are reported beside it
    stage_ms_dom = one_ms if dom == "draw" else stage_ms[dom]
    achieved = alg[dom] / (stage_ms_dom * 1e-3) / 1e9
    roofline = {"bound": None, "kernel": kern_name, "stage": dom, "dominant_source": dom_source,
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "algorithmic_bytes_per_launch": int(alg[dom]), "avg_launch_ms": round(stage_ms_dom, 4),
                "avg_launch_ms_source": ("hipEvents on the draw dispatch, frames one at a time (1 lane): the kernel "
                                         "alone on the GPU" if dom == "draw" else
                                         "hipEvents of the one-lane stage-timing pass"),
                "traffic": load_pmc(kern_name), "traffic_source": pmc_source()}
    if dom == "draw":
        live = alg["draw"] / (draw_ms_live * 1e-3) / 1e9
        roofline["timed_region"] = {
            "avg_launch_ms": round(draw_ms_live, 4), "achieved": round(live, 2), "frac": round(live / HBM_PEAK_GBS, 4),
            "source": "hipEvents on the draw dispatch over the timed frames" +
                      (f" ({args.lanes} frames in flight: the blend shares the GPU with other frames' kernels, "
                       "so this span is longer than the kernel's own time)" if args.lanes > 1 else "")}
        roofline["issue"] = issue_ceiling(kern_name, one_ms)
    # what bounds the kernel, from the evidence: HBM unless its counters show it
    # moving well under its algorithmic bytes while its vector ALUs stay busy -- then instruction issue
    tr = roofline["traffic"]
    if tr:
        roofline["counter_achieved_gbs"] = round(tr / (stage_ms_dom * 1e-3) / 1e9, 2)
        roofline["counter_frac"] = round(roofline["counter_achieved_gbs"] / HBM_PEAK_GBS, 4)
        roofline["traffic_over_algorithmic"] = round(tr / alg[dom], 4)
    occ = (roofline.get("issue") or {}).get("valu_occupancy")
    if tr and occ and tr / alg[dom] < 0.5 and occ > 0.7:
        roofline["bound"] = "issue"
        roofline["bound_evidence"] = (f"counters: {tr / 1e6:.1f} MB per launch = {tr / alg[dom]:.2f}x the algorithmic "
                                      f"bytes, {roofline['counter_frac']:.3f} of HBM; VALU occupancy {occ:.2f}: "
                                      "vector-instruction issue, not HBM, bounds it (frac stays the algorithmic "
                                      "bytes over the launch time, SURVEY 8(d))")
    else:
        roofline["bound"] = "hbm"
        roofline["bound_evidence"] = ("no counter evidence against HBM" if not tr else
                                      f"counters: {tr / alg[dom]:.2f}x the algorithmic bytes")
    frame_bytes = alg["preprocess"] + alg["emit"] + alg["sort"] + alg["draw"]  # bins ride on the sort's first pass
    frame_frac = frame_bytes * (args.steps / local_s) / 1e9 / HBM_PEAK_GBS

    # per-rank (view, entries, time) to rank 0 (gloo, host side)
    mine = {"rank": rank, "device": local % ndev, "view": view, "E": E, "ms_per_frame": round(local_s / args.steps * 1e3, 4)}
    ranks = [mine]
    if pg is not None:
        ranks = [None] * world
        pg.all_gather_object(ranks, mine)

    sweep = None
    if not args.no_sweep and args.config != "c2":
        sweep = camera_sweep(ctx, sp, W, H, view, args.lanes, value / world)
    facade = None
    if not args.no_facade and rank == 0 and world == 1 and flags == 0 and args.config in ("c3", "c4"):
        facade = cpp_facade(ctx, sp, u, W, H, args.steps, args.warmup, args.lanes, value, E)
    copy = copy_peak(ctx) if rank == 0 else None
    if copy:
        roofline["copy_peak_gbs"] = copy["gbs_median"]
        roofline["frac_of_copy"] = round(roofline["achieved"] / copy["gbs_median"], 4)
        roofline["copy_source"] = copy["source"]
    sort = None
    if not args.no_sort_bench and rank == 0:
        sort = sort_bench(ctx)
        if args.config != "c2":
            sort["c3_full"] = sort_bench_c3(ctx, sp, u)
        if copy:
            for k in ("beyond_cache", "c3_full"):
                if k in sort:
                    b = sort[k]
                    b["frac_of_copy_algorithmic"] = round(68.0 * b["n"] / (b["ms_pairs"] * 1e-3) / 1e9 /
                                                          copy["gbs_median"], 4)
    cpu = None
    if not args.no_cpu_baseline and rank == 0 and world == 1:
        cpu = cpu_baseline(sp, u, flags, budget_s=args.cpu_budget)
        cpu.pop("detail", None)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": data_desc,
            "config": {"workload": cfg["desc"] + (" (clean mode)" if args.clean else " (ref mode)") +
                       (", fast exp" if args.fast_exp else ", defined exp") +
                       (", SH degree 3 (beyond the reference)" if args.sh else ""),
                       "splats": N, "width": W, "height": H, "views_per_gpu": 1,
                       "parallelism": f"replicas x{world} (independent views, no collective"
                                      + (f"; {world} ranks on {ndev} GPU(s)" if world > ndev else "") + "); "
                                      f"{args.lanes} frame(s) in flight per GPU"},
            "frame": {"V": V, "D": D, "E": E, "D_over_N": round(D / max(N, 1), 4),
                      "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
                      "stage_ms_source": f"{nser} frames one at a time (1 lane) with every stage boundary timed, before the timed region",
                      "frames_in_flight": args.lanes,
                      "draw_sub_block": ctx.set_draw_sub(),
                      "serial_ms_per_frame": round(serial_ms, 4),
                      "serial_draw_ms": round(tm_serial["ms_draw"] / max(1, tm_serial["frames"]), 4),
                      "prefix_sort": prefix,
                      "camera_sweep": sweep,
                      "cpp_facade": facade,
                      "frame_bytes_algorithmic": int(frame_bytes),
                      "frame_hbm_frac_algorithmic": round(frame_frac, 4),
                      "frame_bytes_source": "40N + 24V (preprocess) + 8E (emission) + sort (4E + 16E + 48 kept "
                                            "when prefix-sorted, else 68E) + 40E + 4WH (blend)"},
            "host": host,
            "ranks": ranks,
            "roofline": roofline,
            "sort": sort,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
