// gs_internal.hpp -- declarations shared by the library's translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/gsplat.h"

namespace gs {

// error plumbing: every C entry point returns a status and records a message
int set_error(gs_ctx *ctx, int code, const std::string &msg);
// hipSetDevice(ctx's device), the first step of every entry point that allocates or launches
int ctx_use_device(gs_ctx *ctx);

// host side (gs_host.cpp)
int ply_count(const char *path, int *n);
int ply_open_body(const char *path, int *n, std::FILE **out);
int ply_load_sh(const char *path, int n, float *f_dc3, float *f_rest45);
int ply_load(const char *path, int n, float *means4, float *colours4, float *opacity, float *scales3,
             float *rots4);
int ply_write(const char *path, int n, const float *means3, const float *rots4, const float *scales3,
              const float *opacities, const float *colours3);
int activate(int n, const float *f_dc3, const float *opacity_logit, const float *log_scale3,
             const float *rot_raw4, float *colours4, float *opacity, float *scales3, float *rots4);
int covariance3d(int n, const float *scales3, const float *rots4, float *cov6);
int camera_update(const gs_camera *cam, float view16[16], float proj16[16], float *focal_x, float *focal_y,
                  float *tan_fovx_getter, float *tan_fovy_getter);
int camera_uniforms(const gs_camera *cam, gs_uniforms *u);
int save_png(const char *path, int width, int height, const uint8_t *rgba8, int flip_y);

// ---------------------------------------------------------------- device side
// splat ids address per-splat records through 32-bit byte offsets (32-B blend records: the
// blend's gathers), so a scene holds at most 2^27 splats (bicycle: 6.1M)
constexpr int kMaxSplats = 1 << 27;
constexpr int kTiles = 16;  // the reference's fixed 16x16 coarse grid (preprocess.glsl:143-153)
// preprocess.glsl:83 depth of a culled splat (1e6f), as key bits.  The reference leaves culled
// splats in the sorted range (as splat 0, splatKeys = 0): after every key whose bits are <= these
// (k_draw places them virtually; bins[512] = the number of entries with larger key bits)
constexpr uint32_t kKeyCulledBits = 0x49742400u;
constexpr int kValsPad = 16;         // zero words before a frame's sorted values (vals[-1] = splat 0)
// bins buffer: [256] tile ends, [256] draw order, [512] keys above 1e6, then (prefix-sorted
// frames) [kBinsLimit + t] the first list position of tile t's window that is not sorted
constexpr int kBinsLimit = 520;
constexpr int kBinsWords = kBinsLimit + 256;
constexpr int kBinCountWords = 260;  // counts of k_bins_count: [0, 256) tiles, [256] keys above 1e6

// ------------------------------------------------------------ prefix sort of a frame
// A frame's blend reads each tile's sorted list only up to where its sub-blocks saturate: at
// C3 (1080p, 6.1M splats) 8 % of the 10M entries (the longest lists, 0.3-0.8M entries, are
// read for their first 2-3k).  A frame enqueued without a host round trip therefore sorts a
// prefix of every list (gs_sort.hip, "prefix sort"):
//   * key classes: c = t for keys in [t, t+1) (t = 0..255, the tile lists of the bins), and
//     c = 256 for every other bit pattern (>= 256, inf, NaN, negative), always kept whole;
//   * k_emit adds one emitted key in kPrefixSample to a per-class histogram of the
//     distance d = bits(t + 1) - key (floating-point buckets: 5-bit exponent, 6-bit mantissa;
//     kPrefixHistCopies copies and consecutive buckets 1 KiB apart, so the hot buckets of a
//     deep list do not serialise on one cache line);
//   * k_prefix_select picks per class the largest key bound whose sampled count reaches
//     target / kPrefixSample (or keeps the class whole);
//   * the first sort pass keeps the keys at or below their class bound (stable), the other
//     passes sort that subset, and the last one writes each value at its position in the full
//     sorted order (class start in the full order - class start in the subset);
//   * the first pass's scan adds one workgroup for the class tables (kept count, placement),
//     the last pass's bins workgroup stores per tile the first position of its draw window
//     that was not sorted (bins[kBinsLimit + t]); a sub-block that reaches it unsaturated flags
//     the frame (pinned ring word 2 = 1), which is then rendered again with the full sort.
constexpr int kClasses = 257;
constexpr int kPrefixBuckets = 2048;
constexpr int kPrefixSample = 128;
constexpr int kPrefixHistCopies = 2;
// word of bucket b in its class's histogram: consecutive buckets on different cache lines
__host__ __device__ constexpr uint32_t prefix_slot(uint32_t b) { return (b & 7u) * (kPrefixBuckets / 8) + (b >> 3); }
constexpr int kPrefixCopies = 16;  // selected-count copies (spread same-address atomics)
// A turned frame's source tiles (PrefixDev::rects): for each tile t of the new view, the rectangle of
// tiles of the views the recorded depths came from that its content was in (the camera's rotation
// maps the tile's corners there; host-computed).  Tile t: 16 bits of word t / 2 (t odd: the high
// half): x0 | x1 << 4 | y0 << 8 | y1 << 12, or 0xffff -- the content came from outside those views
// (no depth describes it: the configured target).
struct TileRects {
    uint32_t w[128];
};
constexpr uint32_t kRectUnknown = 0xffffu;

struct PrefixDev {
    uint32_t *hist;    // [kPrefixHistCopies][256][kPrefixBuckets] sampled counts (zero between frames)
    uint32_t *theta;   // [kClasses] inclusive key bound of the kept keys
    uint32_t *counts;  // [kPrefixCopies][kClasses] kept per class, then [kPrefixCopies] keys < 1.0 (zero between frames)
    uint32_t *nsel;    // [2]: kept keys, 0 (the element count of passes 1-3)
    int32_t *delta;    // [kClasses]: full-order start - subset start of each class
    uint32_t *cls;     // [kClasses + 1] class starts in the full order (then E), [kClasses] ends of their kept keys
    uint32_t cap_sel;  // elements passes 1-3 are sized for (more kept: the host renders the frame again)
    const uint32_t *frame_count;  // the frame's device (V, D) (set by sort_pairs)
    uint32_t cap_all;             // the entry capacity, the bound of V + D (set by sort_pairs)
    uint32_t *h_slot;  // mapped pinned ring slot of the frame: [3] = kept keys (diagnostics), or null
    uint32_t target;   // entries per class to keep at least
    // [256] per tile: the deepest window position any recent blend of the context reached
    // (k_draw's atomicMax; decayed by 1/16 here each frame), or null.  A tile's target is then
    // min(target, 2 * depth + kPrefixDepthSlack): lists the blends read shallowly keep less.
    uint32_t *depth;
    int32_t use_depth;  // 0: the camera turned since the frame before (the depths describe another
                        // view): each class takes the deepest depth of the tiles its content came
                        // from (rects), or without rects of its 3 x 3 neighbourhood
                        // (GS_PREFIX_TURN_NB); its blend still records them
    const TileRects *rects;  // host memory, read at k_prefix_select's launch (by value), or null
    int32_t n;         // splats of the scene (the reference's culled entries: n - V)
    int32_t clean;     // GS_FLAG_CLEAN (no culled entries)
    // GS_DRAW_SBOX: the last pass also writes each placed value's cull box at its position
    // (box_out[pos] = cullbox[value]), so the blend reads boxes in list order; or null
    const uint2 *cullbox;
    uint2 *box_out;
};
// the blend reads a prefix-sorted frame's cull boxes in sorted order (PrefixDev::box_out) instead
// of gathering them by splat id: one gather per kept entry in the sort's last pass instead of one
// per entry and sub-block walk (same box, alternated: draw 0.289 -> 0.275 ms, sort 0.123 -> 0.143,
// three lanes +1.8 %, one frame at a time +1 %; profiles/r05/draw_sbox_ab.txt)
#ifndef GS_DRAW_SBOX
#define GS_DRAW_SBOX 1
#endif
#ifndef GS_PREFIX_SLACK
#define GS_PREFIX_SLACK 4096
#endif
constexpr uint32_t kPrefixDepthSlack = GS_PREFIX_SLACK;
// a turned frame (PrefixDev::use_depth 0) selects each class to twice the deepest depth of its 3 x 3
// tile neighbourhood plus twice the slack (1), or to the configured target (0)
#ifndef GS_PREFIX_TURN_NB
#define GS_PREFIX_TURN_NB 1
#endif
// a turned frame's class target: GS_PREFIX_TURN_MUL x the neighbourhood's depth + its slack x
// GS_PREFIX_TURN_SLACK_MUL
#ifndef GS_PREFIX_RECT_SLACK  // a turned frame's slack (x kPrefixDepthSlack) with source rectangles
#define GS_PREFIX_RECT_SLACK 2u
#endif
#ifndef GS_PREFIX_TURN_MUL
#define GS_PREFIX_TURN_MUL 2u
#endif
#ifndef GS_PREFIX_TURN_SLACK_MUL
#define GS_PREFIX_TURN_SLACK_MUL 1u
#endif
constexpr uint32_t kKey1Bits = 0x3f800000u;    // bits(1.0f)
constexpr uint32_t kKey256Bits = 0x43800000u;  // bits(256.0f)
// key class: t for the keys in [t, t+1), t < 256; 256 for every other bit pattern
__device__ __forceinline__ uint32_t key_class(uint32_t k) {
    return k < kKey256Bits ? (uint32_t)__uint_as_float(k) : 256u;  // (a float in [0, 256): truncation)
}
// bits of the upper bound t + 1 of tile class t
__host__ __device__ inline uint32_t class_hi(uint32_t t) {
    const float f = (float)(t + 1);
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    return u;
}
// histogram bucket of a distance d >= 1 below the class bound: monotone, 6 mantissa bits
// (d < 2^30: buckets < 30 * 64 = 1920)
__device__ __forceinline__ uint32_t prefix_bucket(uint32_t d) {
    const uint32_t e = 31u - (uint32_t)__builtin_clz(d);
    const uint32_t m = e >= 6 ? (d >> (e - 6)) & 63u : (d << (6 - e)) & 63u;
    return (e << 6) | m;
}
// the smallest d in bucket b
__host__ __device__ inline uint32_t prefix_bucket_dmin(uint32_t b) {
    const uint32_t e = b >> 6, m = 64u | (b & 63u);
    return e >= 6 ? m << (e - 6) : m >> (6 - e);
}
constexpr size_t kPrefixWords =
    (size_t)kPrefixHistCopies * 256 * kPrefixBuckets + kClasses + (size_t)kPrefixCopies * (kClasses + 1) + 2 + kClasses +
    (2 * kClasses + 1);

// Per-frame uniforms of the preprocess kernel (preprocess.glsl:18-37)
struct PreParams {
    float view[16];
    float vp[16];
    uint32_t W, H;
    float fx, fy, tan_fov_x, tan_fov_y;
    float tile_w, tile_h;  // int-derived (ref, Q4) or float (clean)
    int32_t clean;
    int32_t n;
    int32_t sh;            // GS_FLAG_SH: colours from degree-3 SH (SceneDev::sh) -> FrameDev::col
    float campos[3];       // camera position in world space (for the SH direction)
};

// Per-frame parameters of the blend kernel (draw.glsl:38-47)
struct DrawParams {
    int32_t W, H;
    int32_t E;                  // entries (or their capacity when count is set)
    const uint32_t *count;      // device (V, D): E = min(E, V + D), or null
    int32_t clean;
    int32_t no_cull;
    int32_t nbx, nby;           // max sub-blocks (16x16, or 8x8 in the small form) per coarse tile in x / y
    int32_t coverW, coverH;     // drawn coverage; pixels outside it are zeroed (Q9)
    int32_t n;                  // splats of the scene
    int32_t V;                  // splats with entries (when count is null; else count[0])
    int32_t prefix;             // prefix-sorted frame: windows end at bins[kBinsLimit + t] (a miss flags fr.h_totals[2])
    uint32_t *depth;            // [256] or null: each block atomicMax-es the window depth it reached (PrefixDev::depth)
    const uint2 *sbox;          // GS_DRAW_SBOX: the frame's cull boxes by position (sbox[-1]: splat 0's box), or null
    int32_t light_trace;        // GS_FLAG_DRAW_TRACE: the STATS form records per-block times and counts only
    int32_t xb[kTiles + 1];     // pixel x range of tile column t: [xb[t], xb[t+1])
    int32_t yb[kTiles + 1];
};

// radix sort scratch (gs_sort.hip)
struct SortScratch {
    uint32_t *keys_alt = nullptr;
    uint32_t *vals_alt = nullptr;
    size_t alt_cap = 0;            // elements
    uint32_t *hist = nullptr;      // [256][nb]
    size_t hist_cap = 0;           // elements
    uint32_t *row_total = nullptr; // [256], then [16][256] tile counts (zero between sorts)
    uint32_t *bkt = nullptr;       // [2][256]: the bucket form's bucket bases and counts
};

// Stable sort of (key, value) pairs: n elements, or -- when dev_count is given -- min(n,
// dev_count[0] + dev_count[1]) read on the device (n is then the capacity the grids are sized
// for).  With bins != null, also the reference's tile bins of the keys (countBins.glsl +
// prefix: bins[t] = #keys with int(key) <= t) and the longest-first tile order in bins[256..511]
// (what launch_bins computes), counted during the first pass's histogram read.
// keys_out false (values < 2^24 required): only the values come out sorted -- the last two
// passes move one packed word (top key byte | value) instead of the pair; keys is left holding
// an intermediate order.
// pre != null (with bins and dev_count): the frame's prefix sort (see PrefixDev): vals holds
// the sorted values at the positions bins[kBinsLimit + t] marks as sorted, keys are not output.
// dup_base >= 0 (with dev_count): the input is k_pre_emit's split layout, V = dev_count[0] mains
// at [0, V) and the dev_count[1] duplicates at [dup_base, dup_base + D); the first pass reads it
// as one array of V + D entries (n is then the capacity of that virtual array).
// kept != null (with pre), kept->count set: the input is a kept emission (k_emit_kept):
// kept->count[0] + [1] entries, already filtered by the class bounds and counted (tile counts,
// kept per class); the select writes the NEXT frame's bounds (pre->theta), and
// kept->after_select is recorded behind the first pass's scan (its last read of the bounds this
// frame kept by).  kept->count null: a full emission, after_select recorded behind the select
// (whose bounds a kept frame after this one reads)
struct KeptSort {
    const uint32_t *count;
    hipEvent_t after_select;
};
int sort_pairs(hipStream_t s, SortScratch &sc, uint32_t *keys, uint32_t *vals, int64_t n, std::string &err,
               const uint32_t *dev_count = nullptr, hipEvent_t start = nullptr, hipEvent_t stop = nullptr,
               uint32_t *bins = nullptr, bool keys_out = true, const PrefixDev *pre = nullptr,
               int64_t dup_base = -1, bool small = false, bool bucket = false, const KeptSort *kept = nullptr);
// small (not with pre): the form for few entries -- 8 launches instead of 12 (k_sweep_small);
// keys and values come out sorted.  Any n is sorted correctly; it pays off while n is small.
// bucket (with small): 3 launches -- a stable scatter by tile (bucket_of) and k_bucket_sort's
// per-bucket LSD passes in LDS (a bucket over 4096 keys through global memory, still exact).
int sort_ensure(SortScratch &sc, int64_t n, std::string &err, hipStream_t s, bool small = false);
void sort_free(SortScratch &sc);
// argsort helper: keys_out[i] = bits(keys[order[i]]), vals_out[i] = order[i]
void launch_gather_keys(hipStream_t s, const float *keys, const int32_t *order, uint32_t *kout, int64_t n,
                        hipEvent_t start = nullptr);

// render kernels (gs_render.hip)
// The scene on the device (gs_scene::soa): the means as three planes of n floats (the
// projection reads them for every splat), then from scene_shape_offset(n) floats on one 28-byte
// shape record per splat, (S00, S01, S02, S11, S12, S22, opacity): a 16-byte and a 12-byte load at
// 4-byte alignment, which lanes of NDC-culled splats can skip whole (k_preprocess_q, LAZY),
// instead of seven planes.  40 B per splat with the means, SURVEY 8(d)'s algorithmic bytes (round
// 6; a padded 32-byte record before: same box, alternated, preprocess 0.1142 / 0.1144 -> 0.1099 /
// 0.1102 ms, three lanes 2375 / 2384 -> 2398 / 2399 frames/s, profiles/r06/shape28_ab.txt)
constexpr int kShapeFloats = 7;  // floats per shape record
__host__ __device__ inline size_t scene_shape_offset(size_t n) { return (3 * n + 3) & ~(size_t)3; }
__host__ __device__ inline size_t scene_floats(size_t n) { return scene_shape_offset(n) + kShapeFloats * n + 1; }
typedef float f32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef float f32x3_a4 __attribute__((ext_vector_type(3), aligned(4)));
struct SceneDev {
    int n;
    const float *mx, *my, *mz;   // SoA means
    const float *shape;          // kShapeFloats per splat: S00, S01, S02, S11, S12, S22, opacity
    const float4 *colour;        // (r,g,b,1) 0..255 (reference colours vec4)
    const float *sh;             // degree-3 SH, 48 floats per splat, splat-major (gs_render.hip sh_quad), or null
};
// per-splat blend inputs, 24 bytes (the blend gathers it with the colour; the pre-exp skip
// threshold is derived from o where the blend needs it, draw_threshold)
struct alignas(8) SplatDraw {
    float mx, my;      // screen position (preprocess.glsl:91-94)
    float a, b, c, o;  // conic (:134-136) and opacity
};
static_assert(sizeof(SplatDraw) == 24, "24-byte blend records");
// the blend's pre-exp skip threshold: power < thr implies alpha < 1/255 (draw.glsl:123-126) for
// any exp within a few ulp; 255 o <= 0 gives +inf (never blends), NaN (opacity NaN) -inf (never
// skips).  v_log_f32 (margins far above its error); the box of the preprocess uses the same log.
__device__ __forceinline__ float draw_log255o(float o) { return __logf(255.0f * o); }
__device__ __forceinline__ float draw_threshold(float o) {
    const float thr = -draw_log255o(o) - 1.0e-3f;
    return thr != thr ? -__builtin_inff() : thr;
}
struct FrameDev {
    SplatDraw *sd;
    uint2 *cullbox;    // conservative pixel box of the alpha >= 1/255 region (int16 bounds, pack_box)
    int4 *rec;         // emission records: 8-byte packed (rec_packed) or (z01 bits, tileX, tileY (-1: no entries), rect)
    uint2 *blocksum;   // per-workgroup (main, dup) sums -> exclusive offsets
    uint32_t *totals;  // [0]=V [1]=D; kept emission: [2] kept mains, [3] kept duplicates
    uint32_t *h_totals;  // mapped pinned host copy of (V, D) for this frame, or null
    float4 *col;         // per-frame colours of GS_FLAG_SH frames (else null)
    // kept emission (a prefix-sorted frame with the class bounds of an earlier frame's select,
    // see KeptDev): the bounds this frame uses, per splat its kept duplicates, per workgroup
    // the (kept mains, kept duplicates) sums -> exclusive offsets
    const uint32_t *theta_in = nullptr;  // [kClasses], or null (kept emission off)
    uint16_t *kdup = nullptr;  // (up to 256: a 16 x 16 rect without the main tile)
    uint2 *blocksum_k = nullptr;
};
// The kept emission's counters (k_emit_kept): it emits only the entries at or below their class
// bound (PrefixDev::theta of the frame before: every class's kept keys a prefix of its sorted
// list, as in the first pass of the prefix sort), and counts what that pass's upsweep counted
// over every entry -- the tile counts of the bins, the keys above 1e6, the kept keys per class
// and the keys below 1.0 -- and samples the keys for this frame's select (the next frame's
// bounds).
constexpr int kTileCopyCount = 16;  // copies of the frame's tile counters (gs_sort.hip kTileCopies)
struct KeptDev {
    uint32_t *tile_counts;  // [kTileCopies = 16][256] tile counts, then [16] keys above 1e6 (SortScratch::row_total + 256)
    uint32_t *counts;       // PrefixDev::counts: [kPrefixCopies][kClasses] kept per class, then [kPrefixCopies] keys < 1.0
    uint32_t *phist;        // PrefixDev::hist (sampled distances to the class bounds)
};
int preprocess_blocks(int n);  // workgroups of k_preprocess / k_emit (= block sums)
int pre_emit_blocks(int n);    // workgroups of k_pre_emit (= its look-back status words)
// start / stop: optional hipEvents recorded on the dispatch packets (stage timing)
// lazy (most splats culled last frame): the queued form, k_preprocess_q -- the bulk of the
// preprocess, and the covariance / opacity loads, for the splats inside the NDC square only
void launch_preprocess(hipStream_t s, const PreParams &P, const SceneDev &sc, const FrameDev &fr, hipEvent_t start,
                       bool lazy = false);
void launch_scan_blocksums(hipStream_t s, const FrameDev &fr, int nblocks, hipEvent_t start, hipEvent_t stop);
// GS_FLAG_SH colours of a prefix-sorted frame after its sort (P.sh was cleared for its preprocess):
// the splats of ids[0, min(count[0], cap)) -- the kept entries -- and splat 0
void launch_sh_kept(hipStream_t s, const PreParams &P, const SceneDev &sc, const FrameDev &fr, const uint32_t *ids,
                    const uint32_t *count, uint32_t cap);
// GS_FLAG_SH colours of every splat with entries (k_sh_colour; after the frame's emission records)
void launch_sh_colour(hipStream_t s, const PreParams &P, const SceneDev &sc, const FrameDev &fr);
bool rec_packed(const PreParams &P);  // the 8-byte emission record (k_preprocess) fits this frame
// prefix_hist != null: also sample the emitted keys into the prefix sort's histogram
void launch_emit(hipStream_t s, int n, bool packed, const FrameDev &fr, uint32_t *keys, uint32_t *vals, uint32_t cap,
                 hipEvent_t start, hipEvent_t stop, uint32_t *prefix_hist = nullptr);
// the kept emission (k_emit_kept; fr.theta_in set, after a KEPT preprocess and block-sum scan)
void launch_emit_kept(hipStream_t s, int n, bool packed, const FrameDev &fr, uint32_t *keys, uint32_t *vals, uint32_t cap,
                      const KeptDev &kd, hipEvent_t start, hipEvent_t stop);
// The fused preprocess + emission of a frame enqueued without a host round trip (k_pre_emit):
// its decoupled look-back state, two halves per frame lane used by alternate frames (each frame
// clears the other half for the next one).
struct LookbackDev {
    uint64_t *st;          // [cap_blocks] this frame's per-workgroup status words (zero on entry)
    uint64_t *st_next;     // the other half, cleared by this frame
    uint32_t cap_blocks;
    // polls a workgroup spends waiting on a predecessor before it gives up, emits at the offsets
    // it has and flags the frame (ring word 4) for the host to render again; 0 gives up at
    // once (gs_ctx_set_lookback_spin: the test that drives the re-render)
    uint32_t spin_limit;
};
constexpr uint32_t kLbSpinLimit = 1u << 15;
// mains at [0, V), duplicates at [n, n + D) of keys / vals (the sort's first pass reads them as
// one array, sort_pairs' dup_base); (V, D) into fr.totals and the frame's pinned ring slot.
// lazy: the covariance / opacity loads only for the splats inside the NDC square.
void launch_pre_emit(hipStream_t s, const PreParams &P, const SceneDev &sc, const FrameDev &fr, const LookbackDev &lb,
                     bool lazy, uint32_t *keys, uint32_t *vals, uint32_t cap, uint32_t *prefix_hist, hipEvent_t start,
                     hipEvent_t stop);
// E entries, or min(E, dev_count[0] + dev_count[1]) when dev_count is given; counts must be
// zero on entry and are left zero
void launch_bins(hipStream_t s, const uint32_t *keys, int64_t E, const uint32_t *dev_count, uint32_t *counts,
                 uint32_t *bins, hipEvent_t stop);
// GPU load path (gs_load.hip): count raw 62-float ply records starting at splat `base` ->
// the scene's SoA planes (n floats each: mx my mz cov0..5 opacity) and colours
constexpr int kPlyFloats = 62;
void launch_ply_activate(hipStream_t s, const float *rec, int count, int base, int n, float *soa, float4 *colour);  // soa: SceneDev layout

// GS_FLAG_DRAW_STATS buffer: per block (launch order) kDrawTraceWords uint32: start, end
// (s_memrealtime, 100 MHz), steps, survivors, (wave, survivor) steps, steps with a needing
// pixel, (pixel, survivor) needs, list entries in range, survivor steps while <= 64 / <= 128
// pixels were active, events while <= 64 were, done-mask refreshes, dense-phase survivor
// steps with events, dense extra event passes, sparse steps with events, survivor batches; the host aggregates
// (gs_draw_stats)
constexpr int kDrawTraceBlocks = 65536;
constexpr int kDrawTraceWords = 16;
constexpr size_t kDrawStatsBytes = (size_t)kDrawTraceBlocks * kDrawTraceWords * 4;

// small: the 8x8 one-pixel-per-lane form (P.nbx / P.nby then count 8-pixel sub-blocks)
void launch_draw(hipStream_t s, const DrawParams &P, bool fast_exp, bool small, const uint32_t *bins,
                 const uint32_t *vals, const FrameDev &fr, const float4 *colour, uint32_t *out,
                 unsigned long long *stats, hipEvent_t start, hipEvent_t stop);

}  // namespace gs
