/*
 * gsplat.h -- C ABI of libgsplat_hip.so, the MI355X (gfx950) Gaussian-splat hot path.
 *
 * This is the drop-in boundary for the reference's GL dispatch
 * (thomas-chernaik/OpenGLGaussianSplattingRenderer; paths below are relative to it).
 * Every entry point names the reference interface it replaces.  Plain pointers and
 * sizes only; no torch / HIP types.  All functions return GS_OK (0) or a negative
 * GS_ERR_* code; gs_last_error() gives the message (the reference prints and
 * continues, src/sort.cpp:150-154, src/Splats.cpp:245-249 -- the C++ facade in
 * gsplat_splats.hpp prints the same messages).
 *
 * Threading: one gs_ctx per GPU; a ctx is not thread-safe; different ctxs may be
 * driven from different host threads.  Work is enqueued on the ctx's own HIP stream.
 * Ownership: the caller owns every host buffer it passes (copied on upload); a
 * gs_scene owns its device arrays; a gs_ctx owns its stream and frame scratch.
 */
#ifndef GSPLAT_H
#define GSPLAT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GS_OK 0
#define GS_ERR_INVALID (-1)  /* bad argument (null pointer, n < 0, ...) */
#define GS_ERR_HIP (-2)      /* HIP runtime error (no device, launch failure, ...) */
#define GS_ERR_IO (-3)       /* file could not be opened / parsed */
#define GS_ERR_NOMEM (-4)    /* device or host allocation failed */
#define GS_ERR_STATE (-5)    /* stage called out of order (e.g. gs_draw before gs_sort) */

/* render flags */
#define GS_FLAG_CLEAN 1u     /* fix the reference's deterministic quirks */
#define GS_FLAG_FAST_EXP 2u  /* blend uses the hardware v_exp_f32 (tolerance parity) instead of
                                the bit-exact polynomial exp shared with the oracle's definition */
#define GS_FLAG_TIMING 4u    /* record per-stage hipEvent timings into gs_frame_stats */
#define GS_FLAG_NO_CULL 8u   /* disable the (exactness-preserving) per-block entry cull */
#define GS_FLAG_DRAW_STATS 16u /* count blend work (see gs_draw_stats); slower, diagnostics only */
#define GS_FLAG_DRAW_TRACE 128u /* with GS_FLAG_DRAW_STATS: only per-block times, list steps, survivors
                                  * and batches (the full counters about double the blend's span) */
#define GS_FLAG_SH 64u       /* SURVEY f3, beyond the reference: view-dependent colour from degree-3
                              * spherical harmonics (scene needs gs_scene_set_sh); the reference
                              * reads f_rest and discards it (src/Splats.cpp:300-302) */

typedef struct gs_ctx gs_ctx;
typedef struct gs_scene gs_scene;

/* Uniforms of Splats::gpuRender (include/Splats.h:122, src/Splats.cpp:587-597):
 * glm::mat4 is column-major float[16]; tan_fov_x/y are passed exactly as main.cpp:62-64
 * passes them (x := Camera::getTanFovy(), y := getTanFovx()). */
typedef struct gs_uniforms {
    float view[16];
    float vp[16];
    int32_t width, height;
    float focal_x, focal_y;
    float tan_fov_x, tan_fov_y;
} gs_uniforms;

typedef struct gs_frame_stats {
    int64_t num_splats;   /* N */
    int64_t visible;      /* V: main entries (on-screen, det != 0) */
    int64_t duplicates;   /* D: extra (splat, tile) entries -- uncapped (Q12 resolved) */
    int64_t entries;      /* E = V + D: sorted entries */
    float ms_preprocess;  /* GS_FLAG_TIMING only (hipEvent, device time) */
    float ms_sort;
    float ms_bins;
    float ms_draw;
    float ms_total;
} gs_frame_stats;

/* Camera restatement (src/Camera.cpp:19-65,181-212, include/Camera.h:13-66) */
typedef struct gs_camera {
    float position[3];   /* Camera(x,y,z) */
    float rotation[3];   /* degrees, rotateUp adds to [0], rotateRight to [1] */
    float fovy;          /* 60 */
    float near_plane;    /* 0.1 */
    float far_plane;     /* 10000 */
    int32_t width, height;
} gs_camera;

/* ---------------------------------------------------------------- library */
const char *gs_version(void);
int gs_device_count(int *count);
/* last error message of this ctx (ctx == NULL: of the calling thread) */
const char *gs_last_error(const gs_ctx *ctx);

/* --------------------------------------------------------------- context
 * Replaces the GL context + program objects: Splats::loadShaders (src/Splats.cpp:156-172),
 * createAndLinkSortAndHistogramShaders (src/sort.cpp:15-124). */
int gs_ctx_create(int device, gs_ctx **out);
void gs_ctx_destroy(gs_ctx *ctx);
int gs_sync(gs_ctx *ctx);                    /* glFinish (src/Splats.cpp:595) */
void *gs_stream(gs_ctx *ctx);                /* the hipStream_t of the newest frame, for interop
                                                (after gs_sync no other ctx stream has work) */
/* Frames in flight on the device: 2 (default) or 3 -- consecutive frames rotate over that many
 * streams with their own frame buffers, so frame k+1's preprocess, emission and sort overlap
 * frame k's blend (blends into one output stay in frame order, blends into different outputs
 * may overlap; everything else behaves as one stream) -- or 1.
 * Beyond the reference, whose gpuRender blocks per frame (src/Splats.cpp:580,595). */
int gs_ctx_set_lanes(gs_ctx *ctx, int lanes);
/* Prefix sort of frames enqueued without a host round trip (beyond the reference, whose
 * GPURadixSort orders every entry, src/sort.cpp:139-203): each tile's list is sorted at least
 * `target` entries deep (default 32768; the blend reads ~2-20k of lists up to 0.8M long at
 * C3) and the rest of it is left unsorted.  Images are unchanged: a frame whose blend reaches
 * an unsorted position before saturating is rendered again with the full sort (alone, with any
 * later frame in flight that writes the same output), and the target doubles for the frames after
 * it; after 64 frames in a row without a miss it halves again, never below the configured target.
 * Three misses within 32 prefix-sorted frames turn the prefix sort off for the next 64 frames.
 * A frame whose camera turned more than 0.25 degrees since the frame before keeps each list twice
 * as deep as the deepest read of its 3 x 3 tile neighbourhood (plus slack), at most `target`: the
 * depths the blends recorded describe the other view, whose content moved by part of a tile.
 * target 0: always the full sort.  Frames with fewer than
 * 64 * target (the configured one) entries -- the previous frame's count -- use the full sort.  Setting a target
 * (>= 0) also clears the per-tile depths the blends recorded (a cold start).  Returns the
 * current target in *current when it is not NULL (with target < 0: only that). */
int gs_ctx_set_sort_prefix(gs_ctx *ctx, int target, int *current);
/* The blend's sub-block form (beyond the reference, whose draw.glsl runs 32x32 workgroups,
 * src/Splats.cpp:378): 16 = one wave per 16x16 pixels, each lane a 2x2 quad (throughput form:
 * large frames); 8 = one wave per 8x8 pixels, one pixel per lane (latency form: four times the
 * waves, for frames whose blend is bound by its longest sub-block); 0 (default) = 8 for frames
 * with fewer than 2^21 entries, else 16; -1 leaves it.  Images are identical in every form.
 * *current (when not NULL) receives the form the newest frame's blend used. */
int gs_ctx_set_draw_sub(gs_ctx *ctx, int sub, int *current);
/* The small-frame forms: frames whose entry count (the newest one seen) is below draw_entries
 * blend in 8x8 sub-blocks when gs_ctx_set_draw_sub is 0 (default 2^21), and below sort_entries
 * sort in 8 launches instead of 12 (default 2^19).  A negative value leaves a limit. */
int gs_ctx_set_small_limits(gs_ctx *ctx, int64_t draw_entries, int64_t sort_entries);
/* The small sort's form: 1 (default) = by tile, then each tile's list (3 launches: a stable
 * scatter by int(key), then LSD passes per tile in LDS); 0 = four 8-bit passes (8 launches);
 * -1 leaves it.  Returns the form now set (or a negative GS_ERR_*).  Same result either way. */
int gs_ctx_set_bucket_sort(gs_ctx *ctx, int on);
/* The kept emission of prefix-sorted frames (large scenes, frames enqueued without a round trip
 * whose camera did not turn since the frame before): the preprocess counts and the emission
 * writes only the entries at or below the key bounds the frame before selected, and the sort's
 * four passes run on those alone.  1 = on, 0 = off (default: measured slower),
 * -1 leaves it; *kept_frames (may be null) = frames emitted that way so far.  Returns the
 * setting (or a negative GS_ERR_*).  Images are the same either way. */
int gs_ctx_set_kept_emission(gs_ctx *ctx, int on, uint64_t *kept_frames);
/* The fused preprocess + emission of small scenes (<= 64k splats, frames enqueued without a host
 * round trip) places each workgroup's entries by a decoupled look-back over the workgroups before
 * it.  A wait for a predecessor is bounded (default 2^15 polls); a workgroup that gives up emits
 * at partial offsets and flags the frame, which the host renders again on the host-synchronous
 * path (same image).  limit 0 gives up at once (a test hook for that path); limit < 0 leaves it.
 * Returns the limit now set; *redone (when not NULL) receives the number of frames rendered
 * again for this reason. */
int gs_ctx_set_lookback_spin(gs_ctx *ctx, int limit, uint64_t *redone);
/* prefix-sort counters: [0] frames prefix-sorted, [1] of them rendered again (a blend reached
 * an unsorted position), [2] entries kept by the newest retired prefix-sorted frame, [3] its
 * entry count; reset != 0 clears [0] and [1] */
int gs_prefix_stats(gs_ctx *ctx, uint64_t out[4], int reset);

/* device memory helpers (callers without their own allocator, e.g. ctypes tests) */
int gs_malloc(gs_ctx *ctx, size_t bytes, void **dptr);
int gs_free(gs_ctx *ctx, void *dptr);
int gs_memcpy_h2d(gs_ctx *ctx, void *dst, const void *src, size_t bytes);
int gs_memcpy_d2h(gs_ctx *ctx, void *dst, const void *src, size_t bytes);
int gs_memset(gs_ctx *ctx, void *dst, int value, size_t bytes);

/* measurement helper (bench.py's roofline.frac_of_copy; not on the frame path): the stream-copy
 * rate of the ctx's GPU -- a non-temporal float4 copy (one per lane) of `bytes` between two fresh device buffers,
 * read + written bytes per second, median (and best) of `reps` hipEvent-timed copies */
int gs_stream_copy_gbs(gs_ctx *ctx, size_t bytes, int reps, double *gbs_median, double *gbs_best);

/* ------------------------------------------------------- host: loader etc. */
/* src/Splats.cpp:250-262: N from the header ("element vertex N" on line 3) */
int gs_ply_count(const char *path, int *n);
/* src/Splats.cpp:174-344 loadSplats: means4 (x,y,z,1), colours4 ((0.5+C0*f_dc)*255,..,1),
 * opacity sigmoid, scales3 exp, rots4 normalised (rot_0..rot_3).  Any output may be NULL. */
int gs_ply_load(const char *path, int n, float *means4, float *colours4, float *opacity,
                float *scales3, float *rots4);
/* the raw SH fields of the ply (f_dc_0..2 and f_rest_0..44, as stored: f_rest is channel-major,
 * 15 coefficients per channel) -- what loadSplats reads and drops (src/Splats.cpp:286-302) */
int gs_ply_load_sh(const char *path, int n, float *f_dc3, float *f_rest45);
/* tests/plyFileGenerator.py:155-249 save_ply byte layout (raw colours into f_dc, logit
 * opacity, log scale, zero normals / SH).  means3, rots4, scales3, opac, colours3 as given. */
int gs_ply_write(const char *path, int n, const float *means3, const float *rots4,
                 const float *scales3, const float *opacities, const float *colours3);
/* saveImage (src/Splats.cpp:516-540): RGBA8 PNG of a host image (W*H*4 bytes, row y = GL
 * row y).  flip_y = 0 writes row 0 first, as saveImage does (GL bottom row at the top of
 * the file); 1 writes the screen orientation. */
int gs_save_png(const char *path, int width, int height, const uint8_t *rgba8, int flip_y);
/* same activations as the loader, from raw (pre-activation) SoA records:
 * f_dc3, opacity logit, log-scale3, raw quaternion4 -> colours4, opacity, scales3, rots4 */
int gs_activate(int n, const float *f_dc3, const float *opacity_logit, const float *log_scale3,
                const float *rot_raw4, float *colours4, float *opacity, float *scales3,
                float *rots4);
/* src/Splats.cpp:414-479 computeCovarianceMatrices: [S00,S01,S02,S11,S12,S22] per splat */
int gs_covariance3d(int n, const float *scales3, const float *rots4, float *cov6);
/* Camera getters (src/Camera.cpp): view, projection, focal x/y, getTanFovx/y (degree-
 * argument quirk Q1 kept), and the uniforms as main.cpp:62-64 passes them (Q2 swap). */
int gs_camera_update(const gs_camera *cam, float view16[16], float proj16[16], float *focal_x,
                     float *focal_y, float *tan_fovx_getter, float *tan_fovy_getter);
int gs_camera_uniforms(const gs_camera *cam, gs_uniforms *out);

/* ---------------------------------------------------------------- scene
 * Splats::loadToGPU (src/Splats.cpp:61-154): host vectors copied to device SoA. */
int gs_scene_create(gs_ctx *ctx, int n, const float *means4, const float *cov6,
                    const float *opacity, const float *colours4, gs_scene **out);
void gs_scene_destroy(gs_scene *scene);
/* SURVEY f1 -- Splats(path) with the load-time work on the GPU: the ply body streams to the
 * device and one kernel applies the activations of src/Splats.cpp:289-331 and the covariance
 * of :414-479 with the same float operations (glibc's expf restated), so the scene equals
 * gs_ply_load + gs_covariance3d + gs_scene_create bit for bit.  Host arrays are not produced
 * (gs_scene_download fetches them).  Same errors and messages as gs_ply_load. */
int gs_scene_load_ply(gs_ctx *ctx, const char *path, gs_scene **out);
/* the scene's arrays in gs_scene_create's host layout (means4 w = 1); any may be NULL */
int gs_scene_download(const gs_scene *scene, float *means4, float *cov6, float *opacity, float *colours4);
/* attach degree-3 SH (raw f_dc3 + f_rest45 per splat, ply layout) to a scene;
 * GS_FLAG_SH frames then colour each splat by the standard 3DGS evaluation for the direction
 * from the camera: max(SH(dir) + 0.5, 0) * 255 (with f_rest = 0 this is the reference's
 * colour wherever that is non-negative) */
int gs_scene_set_sh(gs_scene *scene, const float *f_dc3, const float *f_rest45);
int gs_scene_count(const gs_scene *scene);

/* ---------------------------------------------------------------- frame
 * Splats::gpuRender (src/Splats.cpp:587-597) = preprocess -> sort -> bins -> draw.
 * out_rgba8: W*H*4 bytes, row y = GL row y (bottom-up as in the reference texture);
 * on the host (out_on_device = 0) or a device pointer (1).  stats may be NULL.
 * With stats == NULL, a device output and no GS_FLAG_TIMING, the frame is enqueued without
 * any host round trip (the entry count stays on the device; buffers are sized from the
 * previous frame's count with headroom).  Such a frame is complete and correct after
 * gs_sync (or any call that reads results back): a frame whose entries outgrew the buffers
 * is detected there and rendered again into the same output.  Keep the scene and the output
 * buffer alive until then. */
int gs_render(gs_ctx *ctx, const gs_scene *scene, const gs_uniforms *u, uint32_t flags,
              void *out_rgba8, int out_on_device, gs_frame_stats *stats);
/* counts (num_splats, visible, duplicates, entries) of the newest frame; waits for it */
int gs_last_stats(gs_ctx *ctx, gs_frame_stats *stats);
/* the same counts of the newest frame whose counts the host has already seen, without waiting:
 * behind gs_render's frames in flight by up to the number of lanes (the reference reads the count
 * back each frame, src/Splats.cpp:579-583, stalling its pipeline; the C++ facade's
 * Splats::numDuplicates reads it after a gs_sync, when it is read) */
int gs_seen_stats(gs_ctx *ctx, gs_frame_stats *stats);

/* stage-level entry points mirroring the reference's Splats methods */
/* Splats::preprocess (src/Splats.cpp:542-585) + the per-splat entry emission.
 * Replaces preprocess.glsl and the atomic-counter readback (:579-583). */
int gs_preprocess(gs_ctx *ctx, const gs_scene *scene, const gs_uniforms *u, uint32_t flags,
                  gs_frame_stats *stats);
/* Splats::sort (src/Splats.cpp:346-354): stable sort of the frame's entries by key bits */
int gs_sort(gs_ctx *ctx);
/* Splats::computeBins (src/Splats.cpp:481-512, countBins.glsl, prefixBins.glsl) */
int gs_compute_bins(gs_ctx *ctx);
/* Splats::draw (src/Splats.cpp:356-381, draw.glsl): tile_w/tile_h as gpuRender passes
 * them (float(W)/16.f, float(H)/16.f) */
int gs_draw(gs_ctx *ctx, const gs_scene *scene, int width, int height, float tile_w,
            float tile_h, uint32_t flags, void *out_rgba8, int out_on_device);

/* frame-state readback for parity tests (host buffers; counts in elements) */
#define GS_READ_KEYS 1      /* uint32[E] sorted (after gs_sort / gs_render) or emitted key bits;
                               gs_render's own sort carries no keys through its last passes,
                               so this read emits and sorts that frame's entries again */
#define GS_READ_VALS 2      /* uint32[E] splat index per entry */
#define GS_READ_BINS 3      /* uint32[256] inclusive tile ends (after gs_compute_bins) */
#define GS_READ_MEANS2D 4   /* float[2N] */
#define GS_READ_CONICS 5    /* float[4N] conic.xyz + opacity */
#define GS_READ_CULLBOX 6   /* float[4N] per-splat pixel box used by the block cull (whole pixels:
                               the device keeps floor/ceil 16-bit bounds) */
int gs_frame_read(gs_ctx *ctx, int what, void *host_dst, size_t count);

/* ------------------------------------------------------------- radix sort */
/* GPURadixSort (include/sort.h:18-20, src/sort.cpp:139-203): stable argsort of float
 * keys by floatBitsToUint; d_order (int32[n]) is read as the initial order and
 * overwritten with the sorted order; d_keys are not moved (read as keys[order[i]]). */
int gs_argsort_f32(gs_ctx *ctx, const float *d_keys, int32_t *d_order, int64_t n);
/* stable sort of (key, value) pairs in place by the 32-bit key */
int gs_sort_pairs_u32(gs_ctx *ctx, uint32_t *d_keys, uint32_t *d_vals, int64_t n);
/* PadBuffer (include/sort.h:23, src/sort.cpp:127-137) */
int gs_pad_buffer(int size, int unit_width);

/* device time (hipEvents on the ctx stream) of the last draw launch / last standalone sort */
#define GS_KERNEL_DRAW 1
#define GS_KERNEL_SORT 2
int gs_last_kernel_ms(gs_ctx *ctx, int kernel, float *ms);

/* per-stage device time summed over every frame since gs_timing_reset (events recorded on
 * the ctx stream around each stage; read back without adding syncs to the frame loop) */
typedef struct gs_timing {
    int64_t frames;
    double ms_preprocess;  /* preprocess kernel + block-sum scan */
    double ms_emit;        /* entry emission */
    double ms_sort;        /* 4-pass radix sort of the entries */
    double ms_bins;        /* tile bins */
    double ms_draw;        /* blend */
    double ms_frame;       /* first to last event of the frame (includes the E readback gap) */
    double ms_host_render; /* host wall time inside gs_render calls */
    double ms_host_wait;   /* ... of it blocked on frames in flight (slot reuse, readbacks):
                              ms_host_render - ms_host_wait is the host's enqueue cost */
    int64_t host_renders;  /* gs_render calls timed */
} gs_timing;
int gs_timing_reset(gs_ctx *ctx);
/* which hipEvents a frame records (each event idles the stream a few microseconds):
 * GS_TIMING_FRAME 0 the frame end only; GS_TIMING_DRAW 1 + the draw kernel (ms_draw);
 * GS_TIMING_STAGES 2 every stage (default; all gs_timing fields) */
#define GS_TIMING_FRAME 0
#define GS_TIMING_DRAW 1
#define GS_TIMING_STAGES 2
int gs_timing_enable(gs_ctx *ctx, int mode);

/* blend work counters accumulated by GS_FLAG_DRAW_STATS frames: [0] sub-blocks drawn,
 * [1] chunk iterations, [2] entries that survived the block cull, [3] list entries in range,
 * [4] max iterations of one block, [5] max survivors of one block, [6] max / [7] summed
 * block duration in s_memrealtime ticks (100 MHz), [8] (wave, survivor) steps, [9] steps where some pixel
 * of the wave needs the exp/blend path, [10] (pixel, survivor) pairs needing it */
int gs_draw_stats(gs_ctx *ctx, uint64_t out[16], int reset);
/* per-block trace of the last GS_FLAG_DRAW_STATS draw, 16 uint32 per block in launch order:
 * start, end (s_memrealtime ticks, 100 MHz, low 32 bits), iterations, survivors, (wave,
 * survivor) steps, steps with a needing pixel, (pixel, survivor) needs, list entries in range,
 * survivor steps while <= 64 / <= 128 pixels of the block were active, events while <= 64
 * were, done-mask refreshes (a survivor saturated a pixel), dense-phase survivor steps with
 * events, dense-phase extra event passes (more than 64 events), sparse-phase survivor steps with
 * events, survivor batches (gathered and culled exactly).
 * Returns the number of blocks copied (<= max_blocks, <= 65536). */
int gs_draw_block_trace(gs_ctx *ctx, uint32_t *out, int max_blocks);
int gs_timing_read(gs_ctx *ctx, gs_timing *out);

#ifdef __cplusplus
}
#endif
#endif
