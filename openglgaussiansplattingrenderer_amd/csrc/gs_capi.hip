// gs_capi.hip -- the extern "C" boundary (include/gsplat.h) and the frame orchestration
// that replaces Splats::gpuRender's GL dispatch (src/Splats.cpp:542-597).
#include "gs_internal.hpp"

#include <hip/hip_runtime.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <thread>
#include <vector>

// frame events: 0 start, 1 preprocess+scan done, 2 emit start, 3 emit done,
// 4 sort start, 5 sort done, 6 bins done, 7 draw start, 8 draw done
constexpr int kEv = 9;
constexpr int kRing = 4;
// pinned ring words per frame slot: [0] V, [1] D (k_scan_blocksums / k_pre_emit), [2] k_draw's
// prefix-miss flag, [3] kept entries of a prefix-sorted frame, [4] k_pre_emit's look-back give-up
// flag (a word of its own: a miss store cannot overwrite it)
constexpr int kRingWords = 8;
constexpr int kPrefixDecay = 64;  // frames without a prefix-sort miss before the depth halves
// Frames with fewer entries than this, and at most kSmallDrawSubBlocks 16x16 sub-blocks, blend
// in 8x8 sub-blocks (gs_ctx_set_draw_sub): their blend is latency-bound (~one wave per SIMD, the
// longest sub-block running ~200 survivor steps), and four times the waves, each a quarter of
// the pixels, shorten it (C2: 0.134 -> 0.048 ms).  With more sub-blocks the 16x16 form wins even
// for few entries (1080p C5 views of 0.16-0.96M entries: 0.14-0.24 ms against 0.17-0.39).
constexpr int64_t kSmallDrawEntries = 2 << 20;
constexpr int64_t kSmallDrawSubBlocks = 2048;
// Scenes of at most this many preprocess workgroups (1024 splats each) run preprocess and
// emission fused (k_pre_emit, one launch instead of three).  Larger scenes keep the three
// kernels: the fused kernel's look-back chain (each co-resident workgroup walks back to the
// newest inclusive prefix, a cross-XCD round trip of ~2-3 us per 64 workgroups under the
// streaming load) cost more than the emission record round trip it saves (C3: 0.184 against
// 0.152 ms).
constexpr int kFusedMaxBlocks = 64;
// ... and sort in 8 launches instead of 12 (k_sweep_small: each sweep sums its histogram rows
// itself, which costs a round trip per 64 tiles of 4096 entries)
constexpr int64_t kSmallSortEntries = 512 << 10;
// per-tile prefix depths from the blends' reach (gs::PrefixDev::depth); 0: the configured target everywhere
constexpr uint64_t kPrefixMissWindow = 32;  // (three misses within it)
constexpr int kPrefixCooldown = 64;
#ifndef GS_PREFIX_DEPTH
#define GS_PREFIX_DEPTH 1
#endif
// a turn of more than GS_PREFIX_TURN_MDEG millidegrees between consecutive frames makes a frame's
// prefix selection ignore the per-tile depths
#ifndef GS_PREFIX_TURN_MDEG
#define GS_PREFIX_TURN_MDEG 250
#endif
const float kPrefixTurnCos = (float)std::cos(GS_PREFIX_TURN_MDEG * 1e-3 * 3.14159265358979323846 / 180.0);
// the default of gs_ctx_set_kept_emission: off.  Prefix-sorted frames of large scenes whose
// camera did not turn would emit only their kept entries (the bounds of the frame before:
// gs::KeptDev) -- bit-exact, but the work it moves into the preprocess and the emission (+21 and
// +16 us) costs what the sort saves (-36 us) one frame at a time, and more beside another lane's
// blend (2175-2196 vs 2344-2355 frames/s, profiles/r05/kept_emission_ab.txt)
// a turned frame selects each tile class by the depths of the tiles its content came from (the
// camera's rotation since the frames whose blends recorded them: turned_rects), not by its 3 x 3
// neighbourhood's
#ifndef GS_PREFIX_TURN_RECTS
#define GS_PREFIX_TURN_RECTS 1
#endif
#ifndef GS_PREFIX_TURN_VIEWS  // the views a turned frame maps its tiles into (0: one per lane)
#define GS_PREFIX_TURN_VIEWS 0
#endif
#ifndef GS_PREFIX_TURN_EDGE
#define GS_PREFIX_TURN_EDGE 1
#endif
#ifndef GS_KEPT_EMIT
#define GS_KEPT_EMIT 0
#endif
// cos of the rotation between two view matrices: (trace(R1^T R2) - 1) / 2 over their upper-left
// 3x3 blocks (the same index set in either storage order)
static float turn_cos(const float *a, const float *b) {
    float tr = 0.0f;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) tr += a[4 * c + r] * b[4 * c + r];
    return 0.5f * (tr - 1.0f);
}

// A turned frame's source tiles (gs::TileRects).  The draw's coarse tile t of the view u (float
// tile dims W/16, H/16, src/Splats.cpp:596) is mapped by the camera's rotation into each of the
// views[0, m) -- a pixel's ray in u's camera, the world direction, that view's camera, its pixel --
// and covers the union of the tile rectangles its corners land in there (the translation between
// the poses is left out: it moves content by a parallax, which the selection's slack absorbs).
// Content that lay outside a view entirely, or behind it, is unknown (kRectUnknown: the
// configured target); a footprint partly outside is clamped to the image and widened by a tile.
// P00, P11 of the projection from vp * view^-1 (glm::perspective: P02 = P12 = 0).
static void turned_rects(const gs_uniforms *u, const float (*views)[16], int m, gs::TileRects &tr) {
    auto at = [](const float *a, int r, int c) { return (double)a[4 * c + r]; };
    // view^-1 = [R^T | -R^T t] (a rigid view matrix); P = vp * view^-1: only P00 and P11 are needed
    double Rn[3][3], tn[3], inv[4][4] = {};
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) Rn[r][c] = at(u->view, r, c);
        tn[r] = at(u->view, r, 3);
    }
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) inv[r][c] = Rn[c][r];
        inv[r][3] = -(Rn[0][r] * tn[0] + Rn[1][r] * tn[1] + Rn[2][r] * tn[2]);
    }
    inv[3][3] = 1.0;
    double P00 = 0.0, P11 = 0.0;
    for (int k = 0; k < 4; ++k) {
        P00 += at(u->vp, 0, k) * inv[k][0];
        P11 += at(u->vp, 1, k) * inv[k][1];
    }
    const double W = u->width, H = u->height, tw = W / 16.0, th = H / 16.0;
    for (int t = 0; t < 256; ++t) {
        const int tx = t & 15, ty = t >> 4;
        double x0 = 1e30, x1 = -1e30, y0 = 1e30, y1 = -1e30;
        bool unknown = !(P00 != 0.0 && P11 != 0.0);
        for (int k = 0; k < m && !unknown; ++k) {
            for (int cn = 0; cn < 4; ++cn) {
                const double px = (tx + (cn & 1)) * tw, py = (ty + (cn >> 1)) * th;
                const double v[3] = {(2.0 * px / W - 1.0) / P00, (2.0 * py / H - 1.0) / P11, -1.0};
                double d[3], w[3];
                for (int r = 0; r < 3; ++r) d[r] = Rn[0][r] * v[0] + Rn[1][r] * v[1] + Rn[2][r] * v[2];  // R^T v
                for (int r = 0; r < 3; ++r) w[r] = at(views[k], r, 0) * d[0] + at(views[k], r, 1) * d[1] + at(views[k], r, 2) * d[2];
                if (!(w[2] < -1e-6)) {  // behind that camera
                    unknown = true;
                    break;
                }
                const double qx = (P00 * w[0] / -w[2] + 1.0) * 0.5 * W, qy = (P11 * w[1] / -w[2] + 1.0) * 0.5 * H;
                x0 = std::min(x0, qx);
                x1 = std::max(x1, qx);
                y0 = std::min(y0, qy);
                y1 = std::max(y1, qy);
            }
        }
        uint32_t code = gs::kRectUnknown;
        // (GS_PREFIX_TURN_EDGE: content that lay wholly outside the views takes the nearest edge
        // tiles', widened by a tile, as content partly outside does)
        if (!unknown && (GS_PREFIX_TURN_EDGE || (x1 >= 0.0 && x0 <= W && y1 >= 0.0 && y0 <= H))) {
            const bool part = x0 < 0.0 || x1 > W || y0 < 0.0 || y1 > H;
            int a0 = (int)std::floor(x0 / tw), a1 = (int)std::floor(x1 / tw);
            int b0 = (int)std::floor(y0 / th), b1 = (int)std::floor(y1 / th);
            if (part) a0 -= 1, a1 += 1, b0 -= 1, b1 += 1;
            a0 = std::clamp(a0, 0, 15), a1 = std::clamp(a1, 0, 15), b0 = std::clamp(b0, 0, 15), b1 = std::clamp(b1, 0, 15);
            code = (uint32_t)a0 | ((uint32_t)a1 << 4) | ((uint32_t)b0 << 8) | ((uint32_t)b1 << 12);
        }
        uint32_t &wd = tr.w[t >> 1];
        const int sh = 16 * (t & 1);
        wd = (wd & ~(0xffffu << sh)) | (code << sh);
    }
}

// A frame lane: a stream and the per-frame buffers of the frames it runs.  Consecutive frames
// alternate between the ctx's lanes (two by default), so frame k+1's preprocess, emission and
// sort run while frame k blends -- they fill the blend's tail and the gaps between kernels.
// Frame k+1's blend waits for frame k's (outputs and the draw-stats buffer are written in frame
// order); every other operation joins the lanes first (as if there were one stream).
struct Lane {
    hipStream_t stream = nullptr;
    // per-splat frame buffers (sized by the largest scene rendered so far)
    int n_cap = 0;
    gs::SplatDraw *sd = nullptr;
    float4 *col = nullptr;  // per-frame colours of GS_FLAG_SH frames
    int col_cap = 0;
    uint2 *cullbox = nullptr;
    int4 *rec = nullptr;
    uint2 *blocksum = nullptr;
    uint16_t *kdup = nullptr;        // kept emission: per splat its kept duplicates (<= 256)
    uint2 *blocksum_k = nullptr;     // ... per workgroup its (kept mains, kept duplicates)
    uint32_t *totals = nullptr;      // device [4]
    // entries
    int64_t e_cap = 0;
    uint32_t *keys = nullptr, *vals = nullptr;
    uint32_t *vals_base = nullptr;  // the allocation: kValsPad zero words, then vals (k_draw reads vals[-1] = 0)
    uint2 *sbox_base = nullptr;     // GS_DRAW_SBOX: splat 0's box, then the boxes by position
    int64_t sbox_cap = 0;           // ... positions it holds (allocated by the first prefix-sorted frame)
    bool keys_sorted = true;  // false: the frame sort left only the values sorted (gs_frame_read re-sorts)
    bool vals_partial = false;  // the frame was prefix-sorted: vals holds only each list's sorted prefix
    uint32_t *pre_buf = nullptr;  // prefix-sort state (gs::kPrefixWords words, see gs::PrefixDev)
    // k_pre_emit's look-back state: two halves of cap_blocks status words, alternate frames of
    // this lane use alternate halves (lb_par); zero on allocation
    uint64_t *lb = nullptr;
    uint32_t lb_cap = 0;  // status words per half
    int lb_par = 0;
    bool split = false;  // the newest frame's entries are in the split layout (k_pre_emit)
    // the newest frame (GS_FLAG_SH, prefix-sorted) coloured only its kept entries' splats
    // (k_sh_kept): a full re-sort for the stage calls colours every splat first (resort_full)
    bool sh_partial = false;
    // the newest frame's scene and preprocess parameters (a split frame's readbacks preprocess it
    // again on the staged path, which also writes the emission records)
    const gs_scene *pe_scene = nullptr;
    gs::PreParams pe_P{};
    gs::SortScratch sort;
    // bins
    uint32_t *bin_counts = nullptr;  // [256]
    uint32_t *bins = nullptr;        // [256] tile ranges + [256] draw dispatch order + keys above 1e6 (kBinsWords)
    // output staging (host-destination renders)
    uint32_t *img = nullptr;
    size_t img_cap = 0;
    // argsort key scratch
    uint32_t *ask = nullptr;
    size_t ask_cap = 0;
    // ordering between lanes (blends: per frame slot, see enqueue_draw)
    hipEvent_t aux_done = nullptr;   // after this lane's newest non-frame work
    uint32_t aux_waiters = 0;        // ... lanes (bits) whose next frame has yet to wait for it
    hipEvent_t tail = nullptr;       // scratch: "all work so far" on this lane
};
constexpr int kMaxLanes = 3;

struct gs_ctx {
    int device = 0;
    std::string err;
    Lane lane[kMaxLanes];
    int nlanes = 2;  // frames in flight on the device (gs_ctx_set_lanes)
    int cur_lane = 0;
    Lane *L = &lane[0];      // the lane of the newest frame (and of non-frame work)
    unsigned long long *draw_stats = nullptr;  // GS_FLAG_DRAW_STATS trace (shared: blends are ordered)
    // frame state
    int stage = 0;  // 0 none, 1 preprocessed, 2 sorted, 3 binned
    int n = 0;
    int64_t V = 0, D = 0, E = 0;  // of the newest frame whose counts the host has seen
    uint32_t flags = 0;
    bool rec_packed = true;  // the newest frame's emission records are 8-byte packed
    // Frames in flight.  Each frame takes the next of kRing slots: its hipEvent set, its
    // pinned (V, D) and -- for a frame enqueued without a host round trip ("speculative":
    // the entry count stays on the device, kernels are sized by the entry capacity) -- what is
    // needed to render it again if its entry count turns out to exceed that capacity.
    // Reusing a slot waits for the frame that held it, kRing frames back (flow control).
    struct Slot {
        bool used = false;  // events not yet folded into acc
        bool spec = false;  // speculative: totals not yet checked against cap
        uint64_t seq = 0;
        const gs_scene *scene = nullptr;
        gs_uniforms u{};
        uint32_t flags = 0;
        void *out = nullptr;
        int64_t cap = 0;
        // the frame's blend: lane, output and whether it writes the draw-stats buffer
        int lane = -1;
        const void *draw_out = nullptr;
        bool drawn = false, draw_stats = false;
        bool prefix = false;  // prefix-sorted: its blend may flag a miss (ring word 2)
        bool fused = false;   // k_pre_emit: split entry layout (needs n + D entries), no emission event
        int n = 0;
        uint32_t cap_sel = 0;  // prefix-sorted: the kept entries its sort passes 1-3 could hold
        int target = 0;        // prefix-sorted: its depth
        bool turned = false;   // prefix-sorted without the per-tile depths (PrefixDev::use_depth 0)
    };
    Slot slot[kRing];
    hipEvent_t ev[kRing][kEv] = {};
    hipEvent_t evs[2] = {};      // standalone sort calls
    uint32_t *h_ring = nullptr;      // pinned [kRing][4]: (V, D) of each slot's frame ...
    uint32_t *h_ring_dev = nullptr;  // ... as the device sees it (written by k_scan_blocksums)
    // which events a frame records (each costs the stream a few microseconds of idle):
    // 0 the frame end only, 1 + the draw kernel's start, 2 every stage boundary (default)
    int timing_mode = 2;
    uint64_t seq = 0;
    int cur = 0;                 // slot of the newest frame
    std::vector<gs_scene *> scenes;  // live scenes (detached when the ctx goes first)
    bool e_known = false;        // an entry count has been observed (sizes speculative frames)
    gs_timing acc = {};
    bool in_render = false;      // inside gs_render: host waits count as ms_host_wait
    // prefix sort (gs_ctx_set_sort_prefix)
    // the depth: prefix_base as configured; a miss doubles prefix_target, and every kPrefixDecay
    // frames in a row without one halve it again, down to prefix_base (one close-up or scene
    // swap does not deepen the sort -- or turn it off -- for good)
    int prefix_base = 32768;
    int prefix_target = 32768;
    int prefix_clean_run = 0;
    // a prefix miss was seen: the next prefix-sorted frame sizes its passes 1-3 for every entry (the
    // tiles that missed now keep whole windows, so the kept count can jump past the last one)
    bool prefix_after_miss = false;
    // misses close together (a fast camera: the per-tile depths lag the lists) cost more in
    // re-rendered frames than the prefix sort saves (a re-render ~1.2 ms, the saving ~0.12 ms per
    // frame at C3): kPrefixMissBurst misses within kPrefixMissWindow prefix-sorted frames turn the
    // prefix sort off for the next kPrefixCooldown frames (a cold depth table's first frames miss
    // once or twice while the depths settle; those do not)
    uint64_t prefix_seen = 0;                    // prefix-sorted frames retired
    uint64_t prefix_miss_at[2] = {~0ull, ~0ull}; // ... counts at the two misses before the newest
    int prefix_cooldown = 0;
    float prev_view[16] = {};  // the newest frame's view matrix (the prefix sort's turn test)
    // the view matrices of the newest frames, newest first (a turned frame's source tiles: the
    // depths it selects by were recorded by the blends of up to that many frames before it)
    float view_hist[kMaxLanes][16] = {};
    int view_hist_n = 0;
    gs::TileRects tile_rects{};  // the newest turned frame's (read at its k_prefix_select launch)
    bool prefix_kept_turned = false;  // prefix_kept came from a frame selected without the depths
    bool have_prev_view = false;
    uint64_t prefix_frames = 0, prefix_redo = 0, prefix_kept = 0, prefix_E = 0;
    int prefix_kept_target = 0;  // the depth the frame of prefix_kept was sorted to
    // the blend's sub-block form (gs_ctx_set_draw_sub): 0 by the frame's entry count, 8 or 16
    int draw_sub = 0;
    int last_draw_sub = 0;  // the newest frame's
    // the small-frame forms (gs_ctx_set_small_limits): frames with fewer entries (the newest count
    // seen) blend in 8x8 sub-blocks (draw_sub 0) and sort in 8 launches (k_sweep_small)
    int64_t small_draw_entries = kSmallDrawEntries;
    int64_t small_sort_entries = kSmallSortEntries;
    bool bucket_sort = true;
    // [256] per tile: the deepest window position recent blends reached (gs::PrefixDev::depth);
    // allocated with the first prefix-sorted frame, shared by the lanes
    uint32_t *prefix_depth = nullptr;
    // k_pre_emit's bounded look-back wait (gs_ctx_set_lookback_spin) and the fused frames
    // rendered again because a wait gave up
    uint32_t lb_spin = gs::kLbSpinLimit;
    uint64_t lb_redo = 0;
    // the kept emission (gs::KeptDev): a prefix-sorted frame emits only the entries at or below
    // the class bounds the frame before it selected.  Two bound buffers: frame k reads
    // theta_buf[theta_cur] (its preprocess counts, its emission writes) and its select writes the
    // other one for frame k + 1, whose preprocess waits (on the device) for theta_ev, recorded
    // behind that select.  Each buffer holds one bound set of kClasses words, selected with the
    // tiles' own depths or -- by a frame that turned since the one before (PrefixDev::use_depth
    // 0) -- with their 3x3 neighbourhoods' deepest; a turned frame emits every entry itself, and
    // the set it selects is the one the next unturned frame keeps by.  theta_valid: the read
    // buffer holds a select's bounds of this scene (else it is reset to "keep every entry", and
    // that frame sorts all of them).
    uint32_t *theta_buf[2] = {nullptr, nullptr};
    int theta_cur = 0;
    hipEvent_t theta_ev = nullptr;
    bool theta_valid = false, theta_ev_live = false;
    const gs_scene *theta_scene = nullptr;
    uint64_t kept_frames = 0;
    bool kept_emit = GS_KEPT_EMIT != 0;  // gs_ctx_set_kept_emission
};

struct gs_scene {
    gs_ctx *ctx = nullptr;
    int n = 0;
    float *soa = nullptr;       // mx | my | mz planes, then the 32-byte shape records (gs::SceneDev)
    float4 *colour = nullptr;   // (r,g,b,1)
    float *sh = nullptr;        // GS_FLAG_SH: 48 coefficients per splat, splat-major (sh_quad)
};

namespace gs {

static thread_local std::string t_err;

int set_error(gs_ctx *ctx, int code, const std::string &msg) {
    if (ctx) ctx->err = msg;
    t_err = msg;
    return code;
}

}  // namespace gs

using gs::set_error;

#define GS_HIP(ctx, call)                                                                                    \
    do {                                                                                                     \
        hipError_t e_ = (call);                                                                              \
        if (e_ != hipSuccess)                                                                                \
            return set_error((ctx), GS_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_));         \
    } while (0)

namespace {

int use_device(gs_ctx *ctx) {
    GS_HIP(ctx, hipSetDevice(ctx->device));
    return GS_OK;
}

}  // namespace

int gs::ctx_use_device(gs_ctx *ctx) { return use_device(ctx); }

namespace {

// wait on the host for every lane (all of them: after gs_ctx_set_lanes lowered the count, the
// newest frame and its non-frame work may sit on a lane beyond it)
int sync_lanes(gs_ctx *ctx) {
    for (Lane &ln : ctx->lane) GS_HIP(ctx, hipStreamSynchronize(ln.stream));
    return GS_OK;
}

// non-frame work about to be enqueued on the current lane: order it after everything enqueued
// so far on the other lanes (on the device), as a single stream would
int join_lanes(gs_ctx *ctx) {
    for (int i = 0; i < kMaxLanes; ++i) {
        Lane &o = ctx->lane[i];
        if (&o == ctx->L) continue;
        GS_HIP(ctx, hipEventRecord(o.tail, o.stream));
        GS_HIP(ctx, hipStreamWaitEvent(ctx->L->stream, o.tail, 0));
    }
    return GS_OK;
}

// ... and enqueued: each other lane's next frame waits for it
int mark_aux(gs_ctx *ctx) {
    GS_HIP(ctx, hipEventRecord(ctx->L->aux_done, ctx->L->stream));
    ctx->L->aux_waiters = ((1u << kMaxLanes) - 1) & ~(1u << ctx->cur_lane);
    return GS_OK;
}

// a new frame starts: move to the next lane; it waits (on the device) for non-frame work
// enqueued on the other lanes since their last frame
int next_lane(gs_ctx *ctx) {
    ctx->cur_lane = (ctx->cur_lane + 1) % ctx->nlanes;
    ctx->L = &ctx->lane[ctx->cur_lane];
    const uint32_t me = 1u << ctx->cur_lane;
    for (int i = 0; i < kMaxLanes; ++i) {
        Lane &o = ctx->lane[i];
        if (&o == ctx->L || !(o.aux_waiters & me)) continue;
        GS_HIP(ctx, hipStreamWaitEvent(ctx->L->stream, o.aux_done, 0));
        o.aux_waiters &= ~me;
    }
    return GS_OK;
}

template <typename T>
int grow(gs_ctx *ctx, T *&p, size_t count) {
    if (p) {  // frames in flight may still use the old buffer
        GS_HIP(ctx, hipStreamSynchronize(ctx->L->stream));
        (void)hipFree(p);
    }
    p = nullptr;
    GS_HIP(ctx, hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(T)));
    return GS_OK;
}

int ensure_splats(gs_ctx *ctx, int n) {
    if (n <= ctx->L->n_cap) return GS_OK;
    const int cap = n;
    const int nb = gs::preprocess_blocks(cap);
    int rc;
    if ((rc = grow(ctx, ctx->L->sd, cap)) || (rc = grow(ctx, ctx->L->cullbox, cap)) ||
        (rc = grow(ctx, ctx->L->rec, cap)) || (rc = grow(ctx, ctx->L->blocksum, nb)) ||
        (rc = grow(ctx, ctx->L->kdup, cap)) || (rc = grow(ctx, ctx->L->blocksum_k, nb)) ||
        (rc = grow(ctx, ctx->L->lb, 2 * (size_t)gs::pre_emit_blocks(cap))))
        return rc;
    // (ordered on the lane's stream with the kernels that use it)
    const size_t nbe = (size_t)gs::pre_emit_blocks(cap);
    GS_HIP(ctx, hipMemsetAsync(ctx->L->lb, 0, 2 * nbe * sizeof(uint64_t), ctx->L->stream));
    ctx->L->lb_cap = (uint32_t)nbe;
    ctx->L->lb_par = 0;
    ctx->L->n_cap = cap;
    return GS_OK;
}

int ensure_entries(gs_ctx *ctx, int64_t e) {
    if (e <= ctx->L->e_cap) return GS_OK;
    const int64_t cap = e + e / 4 + 4096;
    int rc;
    if ((rc = grow(ctx, ctx->L->keys, (size_t)cap)) || (rc = grow(ctx, ctx->L->vals_base, (size_t)cap + gs::kValsPad)))
        return rc;
    // the words before vals stay zero (nothing writes them): splat 0 for k_draw's culled entries;
    // the rest is zeroed too, so every word a kernel could read before it is written is a valid id
    GS_HIP(ctx, hipMemsetAsync(ctx->L->vals_base, 0, ((size_t)cap + gs::kValsPad) * 4, ctx->L->stream));
    GS_HIP(ctx, hipMemsetAsync(ctx->L->keys, 0, (size_t)cap * 4, ctx->L->stream));
    ctx->L->vals = ctx->L->vals_base + gs::kValsPad;
    ctx->L->e_cap = cap;
    return GS_OK;
}

gs::FrameDev frame_dev(gs_ctx *ctx) {
    gs::FrameDev f;
    f.sd = ctx->L->sd;
    f.cullbox = ctx->L->cullbox;
    f.rec = ctx->L->rec;
    f.blocksum = ctx->L->blocksum;
    f.totals = ctx->L->totals;
    f.h_totals = ctx->h_ring_dev + kRingWords * ctx->cur;
    f.col = ctx->L->col;
    f.kdup = ctx->L->kdup;
    f.blocksum_k = ctx->L->blocksum_k;
    return f;
}

gs::SceneDev scene_dev(const gs_scene *s) {
    gs::SceneDev d;
    const size_t n = (size_t)s->n;
    d.n = s->n;
    d.mx = s->soa;
    d.my = s->soa + n;
    d.mz = s->soa + 2 * n;
    d.shape = s->soa + gs::scene_shape_offset(n);
    d.colour = s->colour;
    d.sh = s->sh;
    return d;
}

float elapsed(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0.f;
    return ms;
}

// fold a completed frame's events into the accumulators
void accumulate(gs_ctx *ctx, int set) {
    hipEvent_t *e = ctx->ev[set];
    ctx->acc.frames += 1;
    if (ctx->timing_mode >= 1) ctx->acc.ms_draw += elapsed(e[7], e[8]);
    if (ctx->timing_mode < 2) return;
    ctx->acc.ms_preprocess += elapsed(e[0], e[1]);
    if (!ctx->slot[set].fused) ctx->acc.ms_emit += elapsed(e[2], e[3]);  // (fused: in the preprocess)
    ctx->acc.ms_sort += elapsed(e[4], e[5]);
    ctx->acc.ms_bins += elapsed(e[5], e[6]);
    ctx->acc.ms_frame += elapsed(e[0], e[8]);
}

// event i of the frame in flight, per the timing mode (GS_FLAG_TIMING: all); the frame-end
// event (kEv - 1, on the draw kernel) always: it retires the slot
hipEvent_t fev(gs_ctx *ctx, int i) {
    const int mode = (ctx->flags & GS_FLAG_TIMING) ? 2 : ctx->timing_mode;
    if (i == kEv - 1 || mode >= 2 || (mode == 1 && i == 7)) return ctx->ev[ctx->cur][i];
    return nullptr;
}

int render_sync(gs_ctx *ctx, const gs_scene *scene, const gs_uniforms *u, uint32_t flags, void *out,
                int out_on_device, gs_frame_stats *stats);
int resort_full(gs_ctx *ctx);

int oldest_used(const gs_ctx *ctx, uint64_t seq_limit) {
    int k = -1;
    for (int i = 0; i < kRing; ++i)
        if (ctx->slot[i].used && ctx->slot[i].seq <= seq_limit && (k < 0 || ctx->slot[i].seq < ctx->slot[k].seq))
            k = i;
    return k;
}

// A completed speculative frame (slot k): its counts from the pinned ring, the prefix sort's
// bookkeeping.  Returns true when the frame must be rendered again -- its entries exceeded the
// capacity (the emission dropped the excess), a prefix-sorted blend reached an unsorted position
// (miss) or the frame kept more entries than its sort passes could hold (full), or a fused
// frame's look-back gave up -- with *need = the entries it needs; else the frame's counts become
// the context's newest.
bool check_spec(gs_ctx *ctx, int k, int64_t *need) {
    const gs_ctx::Slot &sl = ctx->slot[k];
    const int64_t V = ctx->h_ring[kRingWords * k], D = ctx->h_ring[kRingWords * k + 1];
    // a prefix-sorted frame whose blend reached an unsorted position: render it again
    // (full sort) and sort deeper from now on
    const bool miss = sl.prefix && ctx->h_ring[kRingWords * k + 2] != 0u;
    // ... or a fused frame (k_pre_emit) whose look-back wait gave up: its entries were
    // placed from partial offsets (render it again; the depth stays)
    const bool lb_fail = sl.fused && ctx->h_ring[kRingWords * k + 4] != 0u;
    // ... or that kept more entries than its sort passes could hold (sized from earlier frames)
    const bool full = sl.prefix && ctx->h_ring[kRingWords * k + 3] > sl.cap_sel;
    if (sl.prefix) {
        ctx->prefix_kept = ctx->h_ring[kRingWords * k + 3];
        ctx->prefix_kept_target = sl.target;
        ctx->prefix_kept_turned = sl.turned;
        ctx->prefix_E = (uint64_t)(V + D);
    }
    if (miss) {
        ctx->prefix_target = (int)std::min<int64_t>((int64_t)ctx->prefix_target * 2, 1 << 30);
        ctx->prefix_clean_run = 0;
        ctx->prefix_after_miss = true;
        if (ctx->prefix_miss_at[0] != ~0ull && ctx->prefix_seen - ctx->prefix_miss_at[0] < kPrefixMissWindow) {
            ctx->prefix_cooldown = kPrefixCooldown;
            ctx->prefix_miss_at[0] = ctx->prefix_miss_at[1] = ~0ull;
        } else {
            ctx->prefix_miss_at[0] = ctx->prefix_miss_at[1];
            ctx->prefix_miss_at[1] = ctx->prefix_seen;
        }
    } else if (++ctx->prefix_clean_run >= kPrefixDecay) {  // (prefix-sorted or not: a depth that
        // a miss doubled comes down again)
        ctx->prefix_clean_run = 0;
        if (ctx->prefix_target > ctx->prefix_base)
            ctx->prefix_target = std::max(ctx->prefix_base, ctx->prefix_target / 2);
    }
    if (miss || full) ctx->prefix_redo += 1;
#ifdef GS_PREFIX_TRACE  // (diagnostic builds: tools/diag/prefix_sweep.py)
    if (sl.prefix)
        fprintf(stderr, "prefix seen %llu miss %d full %d kept %u cap_sel %u target %d cooldown %d E %lld\n",
                (unsigned long long)ctx->prefix_seen, (int)miss, (int)full, ctx->h_ring[kRingWords * k + 3], sl.cap_sel,
                ctx->prefix_target, ctx->prefix_cooldown, (long long)(V + D));
#endif
    if (sl.prefix) ctx->prefix_seen += 1;
    if (sl.prefix && !miss && !full && sl.cap_sel >= (uint32_t)sl.cap) ctx->prefix_after_miss = false;
    if (lb_fail) ctx->lb_redo += 1;
    // the split layout of a fused frame holds its duplicates from index n on
    *need = sl.fused ? (int64_t)sl.n + D : V + D;
    if (*need > sl.cap || miss || full || lb_fail) return true;
    ctx->V = V;
    ctx->D = D;
    ctx->E = V + D;
    ctx->e_known = true;
    return false;
}

// The frame in slot `bad` (checked, needing `need0` entries) must be rendered again.  After the
// sync every frame in flight is complete and the speculative ones are the newest (every
// host-synchronous operation validates first): each is checked, oldest first; the ones that
// failed are rendered again, in order, through the synchronous path with grown buffers, and so is
// every later frame that writes an output (or the draw-stats buffer) a re-rendered frame writes,
// since an output must be written in frame order.  The others stand as rendered: a prefix miss
// re-renders one frame (and the frame three later that shares its texture), not every frame in
// flight.
int handle_overflow(gs_ctx *ctx, int bad, int64_t need0) {
    if (int rc = sync_lanes(ctx)) return rc;
    gs_ctx::Slot redo[kRing + 1];
    const void *dirty[2 * kRing];
    int nredo = 0, ndirty = 0;
    int64_t need = need0;
    // the newest frame in flight: the context's readback state (counts, buffers, stage) must be
    // its own after the re-renders, so it is rendered again last if it stood (a
    // re-render of an older frame alone left gs_last_stats / gs_frame_read on that older frame)
    int newest = -1;
    for (int i = 0; i < kRing; ++i)
        if (ctx->slot[i].used && (newest < 0 || ctx->slot[i].seq > ctx->slot[newest].seq)) newest = i;
    const gs_ctx::Slot newest_sl = newest >= 0 ? ctx->slot[newest] : gs_ctx::Slot{};
    bool newest_redone = false;
    for (int k; (k = oldest_used(ctx, ~0ull)) >= 0;) {
        gs_ctx::Slot &sl = ctx->slot[k];
        int64_t nk = 0;
        bool again = k == bad;
        if (!again && sl.spec) {
            again = check_spec(ctx, k, &nk);
            for (int i = 0; i < ndirty && !again; ++i)
                again = dirty[i] == sl.out || (sl.draw_stats && dirty[i] == ctx->draw_stats);
            if (again) nk = std::max<int64_t>(nk, ctx->h_ring[kRingWords * k] + ctx->h_ring[kRingWords * k + 1]);
        }
        if (again) {
            redo[nredo++] = sl;
            need = std::max(need, nk);
            dirty[ndirty++] = sl.out;
            if (sl.draw_stats) dirty[ndirty++] = ctx->draw_stats;
            newest_redone = newest_redone || k == newest;
        } else {
            accumulate(ctx, k);
        }
        sl.used = false;  // (the re-rendered frames' timings are not accumulated)
    }
    // a standing newest frame: rendered again after the others (the same bits into its output,
    // which nothing later writes), so the context ends on its counts and buffers
    if (nredo > 0 && newest >= 0 && !newest_redone && newest_sl.spec) {
        redo[nredo++] = newest_sl;
        need = std::max<int64_t>(need, newest_sl.fused ? (int64_t)newest_sl.n + ctx->D : ctx->E);
    }
    if (int rc = ensure_entries(ctx, need)) return rc;
    for (int i = 0; i < nredo; ++i)
        if (int rc = render_sync(ctx, redo[i].scene, &redo[i].u, redo[i].flags, redo[i].out, 1, nullptr)) return rc;
    return GS_OK;
}

// wait for and retire the frames with seq <= seq_limit, oldest first: check speculative
// frames' entry counts against their capacity, fold their timings
int retire_upto(gs_ctx *ctx, uint64_t seq_limit) {
    for (int k; (k = oldest_used(ctx, seq_limit)) >= 0;) {
        gs_ctx::Slot &sl = ctx->slot[k];
        {
            const auto w0 = std::chrono::steady_clock::now();
            GS_HIP(ctx, hipEventSynchronize(ctx->ev[k][kEv - 1]));
            if (ctx->in_render)
                ctx->acc.ms_host_wait += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
        }
        int64_t need = 0;
        if (sl.spec && check_spec(ctx, k, &need)) return handle_overflow(ctx, k, need);
        accumulate(ctx, k);
        sl.used = false;
    }
    return GS_OK;
}

bool any_spec(const gs_ctx *ctx) {
    for (const auto &sl : ctx->slot)
        if (sl.used && sl.spec) return true;
    return false;
}

// every frame enqueued so far is complete and correct (and, if it was speculative, its counts
// are on the host)
int validate_all(gs_ctx *ctx) {
    if (!any_spec(ctx)) return GS_OK;
    if (int rc = sync_lanes(ctx)) return rc;
    return retire_upto(ctx, ~0ull);
}

// Before a new frame picks its lane and sizes that lane's buffers: retire the frame holding the
// slot it will take.  Retiring may find an overflowed speculative frame and render it again
// (handle_overflow -> render_sync), which moves ctx->L and ctx->cur; after this loop
// begin_frame retires nothing, so the lane and buffers chosen next stay the frame's own.
int prepare_frame(gs_ctx *ctx) {
    for (;;) {
        const gs_ctx::Slot &sl = ctx->slot[(ctx->cur + 1) % kRing];
        if (!sl.used) return GS_OK;
        if (int rc = retire_upto(ctx, sl.seq)) return rc;
    }
}

// take the next slot for a new frame (retiring the frame that held it)
int begin_frame(gs_ctx *ctx) {
    for (;;) {
        const int k = (ctx->cur + 1) % kRing;
        if (!ctx->slot[k].used) {
            ctx->cur = k;
            // the frame's flag words (word 2, k_draw: a prefix miss; word 4, k_pre_emit: a look-back
            // that gave up) start clear; the kernels only ever store nonzero flags to them.  (The
            // slot's previous frame is retired, so nothing on the device writes them now.)
            ctx->h_ring[kRingWords * k + 2] = 0;
            ctx->h_ring[kRingWords * k + 4] = 0;
            ctx->slot[k] = gs_ctx::Slot{};
            ctx->slot[k].used = true;
            ctx->slot[k].seq = ++ctx->seq;
            return GS_OK;
        }
        if (int rc = retire_upto(ctx, ctx->slot[k].seq)) return rc;
    }
}

}  // namespace

extern "C" {

const char *gs_version(void) { return "gsplat-mi355x 0.1 (gfx950)"; }

const char *gs_last_error(const gs_ctx *ctx) { return ctx ? ctx->err.c_str() : gs::t_err.c_str(); }

int gs_device_count(int *count) {
    if (!count) return set_error(nullptr, GS_ERR_INVALID, "count is null");
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *count = c;
    return GS_OK;
}

int gs_ctx_create(int device, gs_ctx **out) {
    if (!out) return set_error(nullptr, GS_ERR_INVALID, "out is null");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return set_error(nullptr, GS_ERR_HIP, "no HIP device available (libgsplat_hip needs an MI355X)");
    if (device < 0 || device >= count) return set_error(nullptr, GS_ERR_INVALID, "device index out of range");
    gs_ctx *ctx = new gs_ctx();
    ctx->device = device;
    int rc;
    auto fail = [&](int code) {
        gs_ctx_destroy(ctx);
        return code;
    };
    if ((rc = use_device(ctx))) return fail(rc);
    for (Lane &ln : ctx->lane) {
        if (hipStreamCreateWithFlags(&ln.stream, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&ln.aux_done, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ln.tail, hipEventDisableTiming) != hipSuccess)
            return fail(set_error(nullptr, GS_ERR_HIP, "hipStreamCreate / hipEventCreate failed"));
        if (hipMalloc(&ln.totals, 16) != hipSuccess || hipMalloc(&ln.bin_counts, gs::kBinCountWords * 4) != hipSuccess ||
            hipMalloc(&ln.bins, gs::kBinsWords * 4) != hipSuccess)
            return fail(set_error(nullptr, GS_ERR_NOMEM, "ctx allocation failed"));
        if (hipMemset(ln.bin_counts, 0, gs::kBinCountWords * 4) != hipSuccess)
            return fail(set_error(nullptr, GS_ERR_HIP, "ctx setup failed"));
    }
    if (hipHostMalloc(&ctx->h_ring, 4 * kRingWords * kRing, hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&ctx->draw_stats, gs::kDrawStatsBytes) != hipSuccess ||
        hipMemset(ctx->draw_stats, 0, gs::kDrawStatsBytes) != hipSuccess)
        return fail(set_error(nullptr, GS_ERR_NOMEM, "ctx allocation failed"));
    if (hipHostGetDevicePointer((void **)&ctx->h_ring_dev, ctx->h_ring, 0) != hipSuccess)
        return fail(set_error(nullptr, GS_ERR_HIP, "ctx setup failed"));
    // stage events are timing-only: no system-scope fence (its cache writeback / invalidate
    // idles the stream for microseconds); the frame-end event keeps it, since the host reads
    // the frame's pinned counts after it
    for (auto &set : ctx->ev)
        for (int i = 0; i < kEv; ++i)
            if (hipEventCreateWithFlags(&set[i], i == kEv - 1 ? hipEventDefault : hipEventDisableSystemFence) !=
                hipSuccess)
                return fail(set_error(nullptr, GS_ERR_HIP, "hipEventCreate failed"));
    for (auto &e : ctx->evs)
        if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess)
            return fail(set_error(nullptr, GS_ERR_HIP, "hipEventCreate failed"));
    *out = ctx;
    return GS_OK;
}

void gs_ctx_destroy(gs_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    for (Lane &ln : ctx->lane)
        if (ln.stream) (void)hipStreamSynchronize(ln.stream);
    for (gs_scene *sc : ctx->scenes) sc->ctx = nullptr;  // they stay valid for gs_scene_destroy
    for (Lane &ln : ctx->lane) {
        void *bufs[] = {ln.sd, ln.cullbox, ln.rec, ln.blocksum, ln.totals, ln.keys, ln.vals_base,
                        ln.bin_counts, ln.bins, ln.img, ln.ask, ln.col, ln.pre_buf, ln.lb, ln.kdup, ln.blocksum_k, ln.sbox_base};
        for (void *b : bufs)
            if (b) (void)hipFree(b);
        gs::sort_free(ln.sort);
        for (hipEvent_t e : {ln.aux_done, ln.tail})
            if (e) (void)hipEventDestroy(e);
        if (ln.stream) (void)hipStreamDestroy(ln.stream);
    }
    if (ctx->draw_stats) (void)hipFree(ctx->draw_stats);
    if (ctx->prefix_depth) (void)hipFree(ctx->prefix_depth);
    for (uint32_t *t : ctx->theta_buf)
        if (t) (void)hipFree(t);
    if (ctx->theta_ev) (void)hipEventDestroy(ctx->theta_ev);
    if (ctx->h_ring) (void)hipHostFree(ctx->h_ring);
    for (auto &set : ctx->ev)
        for (auto &e : set)
            if (e) (void)hipEventDestroy(e);
    for (auto &e : ctx->evs)
        if (e) (void)hipEventDestroy(e);
    delete ctx;
}

// frames in flight on the device: 2 (default: frame k+1's preprocess / emission / sort overlap
// frame k's blend) or 1 (frames run one after the other on one stream)
int gs_ctx_set_lanes(gs_ctx *ctx, int lanes) {
    if (!ctx) return set_error(nullptr, GS_ERR_INVALID, "ctx is null");
    if (lanes < 1 || lanes > kMaxLanes) return set_error(ctx, GS_ERR_INVALID, "gs_ctx_set_lanes: lanes must be 1, 2 or 3");
    if (int rc = gs_sync(ctx)) return rc;
    for (Lane &ln : ctx->lane) ln.aux_waiters = 0;  // everything enqueued so far is done
    // L stays on the newest frame's lane (gs_frame_read / gs_draw / gs_sort still address that
    // frame's buffers); next_lane takes the new count from the next frame on
    ctx->nlanes = lanes;
    return GS_OK;
}

int gs_sync(gs_ctx *ctx) {
    if (!ctx) return set_error(nullptr, GS_ERR_INVALID, "ctx is null");
    for (Lane &ln : ctx->lane) GS_HIP(ctx, hipStreamSynchronize(ln.stream));
    return validate_all(ctx);  // speculative frames checked (and rendered again if they overflowed)
}

void *gs_stream(gs_ctx *ctx) { return ctx ? (void *)ctx->L->stream : nullptr; }

int gs_malloc(gs_ctx *ctx, size_t bytes, void **dptr) {
    if (!ctx || !dptr) return set_error(ctx, GS_ERR_INVALID, "null argument");
    if (int rc = use_device(ctx)) return rc;
    GS_HIP(ctx, hipMalloc(dptr, std::max<size_t>(bytes, 1)));
    return GS_OK;
}
int gs_free(gs_ctx *ctx, void *dptr) {
    if (!ctx) return set_error(nullptr, GS_ERR_INVALID, "ctx is null");
    if (!dptr) return GS_OK;
    if (int rc = gs_sync(ctx)) return rc;  // frames in flight (or their re-renders) may use it
    GS_HIP(ctx, hipFree(dptr));
    return GS_OK;
}
int gs_memcpy_h2d(gs_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx) return set_error(nullptr, GS_ERR_INVALID, "ctx is null");
    // an overflowed speculative frame is rendered again before this write, not over it
    if (int rc = validate_all(ctx)) return rc;
    if (int rc = join_lanes(ctx)) return rc;  // frames in flight may read dst
    GS_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->L->stream));
    GS_HIP(ctx, hipStreamSynchronize(ctx->L->stream));
    return GS_OK;
}
int gs_memcpy_d2h(gs_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx) return set_error(nullptr, GS_ERR_INVALID, "ctx is null");
    if (int rc = gs_sync(ctx)) return rc;  // speculative frames complete and checked first
    GS_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->L->stream));
    GS_HIP(ctx, hipStreamSynchronize(ctx->L->stream));
    return GS_OK;
}
int gs_memset(gs_ctx *ctx, void *dst, int value, size_t bytes) {
    if (!ctx) return set_error(nullptr, GS_ERR_INVALID, "ctx is null");
    if (int rc = validate_all(ctx)) return rc;  // see gs_memcpy_h2d
    if (int rc = join_lanes(ctx)) return rc;
    GS_HIP(ctx, hipMemsetAsync(dst, value, bytes, ctx->L->stream));
    return mark_aux(ctx);
}

// ------------------------------------------------------------------ host side
int gs_ply_count(const char *path, int *n) {
    if (!path || !n) return set_error(nullptr, GS_ERR_INVALID, "null argument");
    return gs::ply_count(path, n);
}
int gs_ply_load(const char *path, int n, float *means4, float *colours4, float *opacity, float *scales3,
                float *rots4) {
    if (!path || n < 0) return set_error(nullptr, GS_ERR_INVALID, "bad argument");
    return gs::ply_load(path, n, means4, colours4, opacity, scales3, rots4);
}
int gs_ply_write(const char *path, int n, const float *means3, const float *rots4, const float *scales3,
                 const float *opacities, const float *colours3) {
    if (!path || n < 0 || (n > 0 && (!means3 || !rots4 || !scales3 || !opacities || !colours3)))
        return set_error(nullptr, GS_ERR_INVALID, "bad argument");
    return gs::ply_write(path, n, means3, rots4, scales3, opacities, colours3);
}
int gs_activate(int n, const float *f_dc3, const float *opacity_logit, const float *log_scale3, const float *rot_raw4,
                float *colours4, float *opacity, float *scales3, float *rots4) {
    if (n < 0 || (n > 0 && (!f_dc3 || !opacity_logit || !log_scale3 || !rot_raw4)))
        return set_error(nullptr, GS_ERR_INVALID, "bad argument");
    return gs::activate(n, f_dc3, opacity_logit, log_scale3, rot_raw4, colours4, opacity, scales3, rots4);
}
int gs_covariance3d(int n, const float *scales3, const float *rots4, float *cov6) {
    if (n < 0 || (n > 0 && (!scales3 || !rots4 || !cov6))) return set_error(nullptr, GS_ERR_INVALID, "bad argument");
    return gs::covariance3d(n, scales3, rots4, cov6);
}
int gs_camera_update(const gs_camera *cam, float view16[16], float proj16[16], float *focal_x, float *focal_y,
                     float *tan_fovx_getter, float *tan_fovy_getter) {
    if (!cam || cam->height == 0) return set_error(nullptr, GS_ERR_INVALID, "bad camera");
    return gs::camera_update(cam, view16, proj16, focal_x, focal_y, tan_fovx_getter, tan_fovy_getter);
}
int gs_camera_uniforms(const gs_camera *cam, gs_uniforms *out) {
    if (!cam || !out || cam->height == 0) return set_error(nullptr, GS_ERR_INVALID, "bad camera");
    return gs::camera_uniforms(cam, out);
}
int gs_ply_load_sh(const char *path, int n, float *f_dc3, float *f_rest45) {
    return gs::ply_load_sh(path, n, f_dc3, f_rest45);
}
int gs_save_png(const char *path, int width, int height, const uint8_t *rgba8, int flip_y) {
    return gs::save_png(path, width, height, rgba8, flip_y);
}
int gs_pad_buffer(int size, int unit_width) {
    // src/sort.cpp:127-137
    if (unit_width <= 0) return 0;
    if (size % unit_width == 0) return 0;
    return unit_width - (size % unit_width);
}

// ---------------------------------------------------------------------- scene
int gs_scene_create(gs_ctx *ctx, int n, const float *means4, const float *cov6, const float *opacity,
                    const float *colours4, gs_scene **out) {
    if (!ctx || !out || n < 0 || (n > 0 && (!means4 || !cov6 || !opacity || !colours4)))
        return set_error(ctx, GS_ERR_INVALID, "gs_scene_create: bad argument");
    if (n > gs::kMaxSplats) return set_error(ctx, GS_ERR_INVALID, "gs_scene_create: more than 2^27 splats");
    *out = nullptr;
    if (int rc = use_device(ctx)) return rc;
    // host AoS (reference layout) -> device SoA planes
    const size_t nn = (size_t)n;
    std::vector<float> soa(std::max<size_t>(gs::scene_floats(nn), 1), 0.0f);
    float *shape = soa.data() + gs::scene_shape_offset(nn);
    for (size_t i = 0; i < nn; ++i) {
        soa[i] = means4[4 * i + 0];
        soa[nn + i] = means4[4 * i + 1];
        soa[2 * nn + i] = means4[4 * i + 2];
        for (int c = 0; c < 6; ++c) shape[gs::kShapeFloats * i + c] = cov6[6 * i + c];
        shape[gs::kShapeFloats * i + 6] = opacity[i];
    }
    gs_scene *s = new gs_scene();
    s->ctx = ctx;
    s->n = n;
    if (hipMalloc(&s->soa, soa.size() * 4) != hipSuccess ||
        hipMalloc(&s->colour, std::max<size_t>(nn, 1) * sizeof(float4)) != hipSuccess) {
        gs_scene_destroy(s);
        return set_error(ctx, GS_ERR_NOMEM, "gs_scene_create: out of device memory");
    }
    GS_HIP(ctx, hipMemcpyAsync(s->soa, soa.data(), soa.size() * 4, hipMemcpyHostToDevice, ctx->L->stream));
    if (n > 0) GS_HIP(ctx, hipMemcpyAsync(s->colour, colours4, nn * sizeof(float4), hipMemcpyHostToDevice, ctx->L->stream));
    GS_HIP(ctx, hipStreamSynchronize(ctx->L->stream));
    ctx->scenes.push_back(s);
    *out = s;
    return GS_OK;
}

namespace {
// bytes of f at its current position into dst, by kReaders threads with pread (one fread
// stream tops out near 7 GB/s from the page cache); leaves f positioned after them
bool read_records(std::FILE *f, char *dst, size_t bytes) {
    constexpr int kReaders = 8;
    const int fd = fileno(f);
    const off_t at = (off_t)std::ftell(f);
    if (at < 0) return false;
    std::atomic<bool> ok{true};
    std::vector<std::thread> th;
    const size_t part = (bytes + kReaders - 1) / kReaders;
    for (int t = 0; t < kReaders; ++t) {
        const size_t b0 = std::min(bytes, (size_t)t * part), b1 = std::min(bytes, b0 + part);
        if (b0 == b1) continue;
        th.emplace_back([&, b0, b1] {
            for (size_t o = b0; o < b1;) {
                const ssize_t r = pread(fd, dst + o, b1 - o, at + (off_t)o);
                if (r <= 0) {
                    ok = false;
                    return;
                }
                o += (size_t)r;
            }
        });
    }
    for (auto &x : th) x.join();
    return ok && std::fseek(f, at + (off_t)bytes, SEEK_SET) == 0;
}
}  // namespace

// the load path on the GPU.  The ply body streams through two pinned chunk
// buffers (fread -> async H2D -> k_ply_activate), so reading, copying and the activations of
// consecutive chunks overlap; the scene equals gs_ply_load + gs_covariance3d +
// gs_scene_create bit for bit (gs_load.hip).  No host-side arrays are produced.
int gs_scene_load_ply(gs_ctx *ctx, const char *path, gs_scene **out) {
    if (!ctx || !path || !out) return set_error(ctx, GS_ERR_INVALID, "gs_scene_load_ply: null argument");
    *out = nullptr;
    if (int rc = use_device(ctx)) return rc;
    int n = 0;
    std::FILE *f = nullptr;
    if (int rc = gs::ply_open_body(path, &n, &f)) return set_error(ctx, rc, gs_last_error(nullptr));
    if (n > gs::kMaxSplats) {
        std::fclose(f);
        return set_error(ctx, GS_ERR_INVALID, "gs_scene_load_ply: more than 2^27 splats");
    }
    const size_t nn = (size_t)n, rec = gs::kPlyFloats * sizeof(float);
    gs_scene *s = new gs_scene();
    s->ctx = ctx;
    s->n = n;
    constexpr size_t kChunk = 1 << 18;  // splats per chunk (65 MB of records)
    float *h_buf[2] = {nullptr, nullptr}, *d_buf[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    auto cleanup = [&](int rc, const std::string &msg) {
        (void)hipStreamSynchronize(ctx->L->stream);
        for (int k = 0; k < 2; ++k) {
            if (h_buf[k]) (void)hipHostFree(h_buf[k]);
            if (d_buf[k]) (void)hipFree(d_buf[k]);
            if (done[k]) (void)hipEventDestroy(done[k]);
        }
        std::fclose(f);
        if (rc) {
            gs_scene_destroy(s);
            return set_error(ctx, rc, msg);
        }
        return GS_OK;
    };
    if (hipMalloc(&s->soa, std::max<size_t>(gs::scene_floats(nn), 1) * 4) != hipSuccess ||
        hipMalloc(&s->colour, std::max<size_t>(nn, 1) * sizeof(float4)) != hipSuccess)
        return cleanup(GS_ERR_NOMEM, "gs_scene_load_ply: out of device memory");
    const size_t chunk = std::min(kChunk, std::max<size_t>(nn, 1));
    for (int k = 0; k < 2; ++k)
        if (hipHostMalloc(&h_buf[k], chunk * rec, hipHostMallocDefault) != hipSuccess ||
            hipMalloc(&d_buf[k], chunk * rec) != hipSuccess || hipEventCreate(&done[k]) != hipSuccess)
            return cleanup(GS_ERR_NOMEM, "gs_scene_load_ply: staging allocation failed");
    for (size_t base = 0, it = 0; base < nn; base += chunk, ++it) {
        const int k = (int)(it & 1);
        const size_t cnt = std::min(chunk, nn - base);
        if (it >= 2 && hipEventSynchronize(done[k]) != hipSuccess)  // copy out of h_buf[k] finished
            return cleanup(GS_ERR_HIP, "gs_scene_load_ply: hipEventSynchronize failed");
        if (!read_records(f, (char *)h_buf[k], cnt * rec))  // src/Splats.cpp:333-340
            return cleanup(GS_ERR_IO, "Error: failed to read all splats from file");
        if (hipMemcpyAsync(d_buf[k], h_buf[k], cnt * rec, hipMemcpyHostToDevice, ctx->L->stream) != hipSuccess)
            return cleanup(GS_ERR_HIP, "gs_scene_load_ply: hipMemcpyAsync failed");
        gs::launch_ply_activate(ctx->L->stream, d_buf[k], (int)cnt, (int)base, n, s->soa, s->colour);
        if (hipEventRecord(done[k], ctx->L->stream) != hipSuccess)
            return cleanup(GS_ERR_HIP, "gs_scene_load_ply: hipEventRecord failed");
    }
    if (std::fgetc(f) != EOF) return cleanup(GS_ERR_IO, "Error: failed to read all splats from file");
    if (hipGetLastError() != hipSuccess) return cleanup(GS_ERR_HIP, "gs_scene_load_ply: kernel launch failed");
    if (int rc = cleanup(GS_OK, "")) return rc;
    ctx->scenes.push_back(s);
    *out = s;
    return GS_OK;
}

// the scene's arrays in the host layout of gs_scene_create (means4 w = 1); any may be NULL
int gs_scene_download(const gs_scene *scene, float *means4, float *cov6, float *opacity, float *colours4) {
    if (!scene || !scene->ctx) return set_error(nullptr, GS_ERR_INVALID, "gs_scene_download: bad scene");
    gs_ctx *ctx = scene->ctx;
    if (int rc = use_device(ctx)) return rc;
    const size_t nn = (size_t)scene->n;
    std::vector<float> soa(gs::scene_floats(nn));
    const float *shape = soa.data() + gs::scene_shape_offset(nn);
    if (nn) GS_HIP(ctx, hipMemcpyAsync(soa.data(), scene->soa, soa.size() * 4, hipMemcpyDeviceToHost, ctx->L->stream));
    if (nn && colours4)
        GS_HIP(ctx, hipMemcpyAsync(colours4, scene->colour, nn * sizeof(float4), hipMemcpyDeviceToHost, ctx->L->stream));
    GS_HIP(ctx, hipStreamSynchronize(ctx->L->stream));
    for (size_t i = 0; i < nn; ++i) {
        if (means4) {
            means4[4 * i + 0] = soa[i];
            means4[4 * i + 1] = soa[nn + i];
            means4[4 * i + 2] = soa[2 * nn + i];
            means4[4 * i + 3] = 1.f;
        }
        if (cov6)
            for (int c = 0; c < 6; ++c) cov6[6 * i + c] = shape[gs::kShapeFloats * i + c];
        if (opacity) opacity[i] = shape[gs::kShapeFloats * i + 6];
    }
    return GS_OK;
}

int gs_scene_set_sh(gs_scene *scene, const float *f_dc3, const float *f_rest45) {
    if (!scene || !scene->ctx || (scene->n > 0 && (!f_dc3 || !f_rest45)))
        return set_error(nullptr, GS_ERR_INVALID, "gs_scene_set_sh: bad argument");
    gs_ctx *ctx = scene->ctx;
    if (int rc = use_device(ctx)) return rc;
    if (int rc = gs_sync(ctx)) return rc;  // frames in flight may read the old planes
    const size_t n = (size_t)scene->n;
    // splat-major (gs_render.hip sh_quad): coefficient j = 16c + k of splat i at float 48 i + j
    std::vector<float> planes(48 * std::max<size_t>(n, 1), 0.0f);
    auto at = [](size_t i, int j) { return i * 48 + (size_t)j; };
    for (size_t i = 0; i < n; ++i)
        for (int c = 0; c < 3; ++c) {
            planes[at(i, 16 * c)] = f_dc3[3 * i + c];
            for (int k = 1; k < 16; ++k) planes[at(i, 16 * c + k)] = f_rest45[45 * i + 15 * c + (k - 1)];
        }
    if (!scene->sh && hipMalloc(&scene->sh, planes.size() * 4) != hipSuccess)
        return set_error(ctx, GS_ERR_NOMEM, "gs_scene_set_sh: out of device memory");
    GS_HIP(ctx, hipMemcpyAsync(scene->sh, planes.data(), planes.size() * 4, hipMemcpyHostToDevice, ctx->L->stream));
    GS_HIP(ctx, hipStreamSynchronize(ctx->L->stream));
    return GS_OK;
}

void gs_scene_destroy(gs_scene *scene) {
    if (!scene) return;
    if (gs_ctx *ctx = scene->ctx) {
        (void)hipSetDevice(ctx->device);
        (void)gs_sync(ctx);  // frames in flight (and their re-renders) may read the scene
        ctx->scenes.erase(std::remove(ctx->scenes.begin(), ctx->scenes.end(), scene), ctx->scenes.end());
        for (Lane &ln : ctx->lane)
            if (ln.pe_scene == scene) ln.pe_scene = nullptr;
    }
    if (scene->soa) (void)hipFree(scene->soa);
    if (scene->colour) (void)hipFree(scene->colour);
    if (scene->sh) (void)hipFree(scene->sh);
    delete scene;
}

int gs_scene_count(const gs_scene *scene) { return scene ? scene->n : -1; }

// ---------------------------------------------------------------------- frame
}  // extern "C"

namespace {

gs::PreParams pre_params(const gs_uniforms *u, uint32_t flags, int n) {
    gs::PreParams P;
    std::memcpy(P.view, u->view, sizeof(P.view));
    std::memcpy(P.vp, u->vp, sizeof(P.vp));
    P.W = (uint32_t)u->width;
    P.H = (uint32_t)u->height;
    P.fx = u->focal_x;
    P.fy = u->focal_y;
    P.tan_fov_x = u->tan_fov_x;
    P.tan_fov_y = u->tan_fov_y;
    P.clean = (flags & GS_FLAG_CLEAN) ? 1 : 0;
    if (!P.clean) {  // preprocess.glsl:143-144 integer screen/16 (Q4)
        P.tile_w = (float)(P.W / 16);
        P.tile_h = (float)(P.H / 16);
    } else {
        P.tile_w = (float)u->width / 16.f;
        P.tile_h = (float)u->height / 16.f;
    }
    P.n = n;
    return P;
}

int check_frame_args(gs_ctx *ctx, const gs_scene *scene, const gs_uniforms *u, const char *who) {
    if (!ctx || !scene || !u) return set_error(ctx, GS_ERR_INVALID, std::string(who) + ": null argument");
    if (scene->ctx != ctx) return set_error(ctx, GS_ERR_INVALID, std::string(who) + ": scene belongs to another ctx");
    if (u->width <= 0 || u->height <= 0) return set_error(ctx, GS_ERR_INVALID, std::string(who) + ": bad resolution");
    return use_device(ctx);
}

// covariance loads only for the splats inside the NDC square when the newest frame seen had most
// of the scene's splats culled (the small C5 views)
// GS_FLAG_SH frames prefix-sorted: SH colours for the kept entries' splats only (k_sh_kept)
#ifndef GS_SH_KEPT
#define GS_SH_KEPT 1
#endif
constexpr bool kShKept = GS_SH_KEPT != 0;


#ifndef GS_QUEUE_FRAC
#define GS_QUEUE_FRAC 2  // the queued preprocess when fewer than n / GS_QUEUE_FRAC splats were visible
#endif
bool lazy_loads(const gs_ctx *ctx, int n) { return ctx->n == n && ctx->e_known && ctx->V * GS_QUEUE_FRAC < (int64_t)n; }

// preprocess + block-sum scan of a new frame (events 0, 1); (V, D) land in ctx->L->totals.
// defer_sh (a prefix-sorted GS_FLAG_SH frame): no SH colours here -- k_sh_kept colours the kept
// entries' splats after the sort (enqueue_sh_kept)
int enqueue_preprocess(gs_ctx *ctx, const gs_scene *scene, const gs_uniforms *u, uint32_t flags,
                       bool defer_sh = false, const uint32_t *theta_in = nullptr) {
    const int n = scene->n;
    const bool sh = (flags & GS_FLAG_SH) != 0;
    if (sh && !scene->sh) return set_error(ctx, GS_ERR_INVALID, "GS_FLAG_SH: the scene has no SH (gs_scene_set_sh)");
    if (int rc = ensure_splats(ctx, n)) return rc;
    if (sh && ctx->L->col_cap < n) {
        if (int rc = grow(ctx, ctx->L->col, (size_t)n)) return rc;
        ctx->L->col_cap = n;
    }
    if (int rc = begin_frame(ctx)) return rc;
    ctx->flags = flags;
    gs::PreParams P = pre_params(u, flags, n);
    P.sh = sh ? 1 : 0;
    ctx->rec_packed = gs::rec_packed(P);
    // camera position = -R^T t of the view matrix (column-major, view[4c + r])
    for (int c = 0; c < 3; ++c)
        P.campos[c] = -(u->view[4 * c + 0] * u->view[12] + u->view[4 * c + 1] * u->view[13] +
                        u->view[4 * c + 2] * u->view[14]);
    gs::FrameDev fr = frame_dev(ctx);
    fr.theta_in = theta_in;  // (kept emission: the bounds this frame's preprocess counts with)
    const int nb = gs::preprocess_blocks(n);
    // k_scan_blocksums writes (V, D) to ctx->L->totals and to this slot's pinned host copy
    gs::PreParams Pl = P;
    if (defer_sh) Pl.sh = 0;
    gs::launch_preprocess(ctx->L->stream, Pl, scene_dev(scene), fr, fev(ctx, 0), !theta_in && lazy_loads(ctx, n));
    gs::launch_scan_blocksums(ctx->L->stream, fr, nb, nb > 0 ? nullptr : fev(ctx, 0), fev(ctx, 1));
    GS_HIP(ctx, hipGetLastError());
    ctx->n = n;
    ctx->L->split = false;
    ctx->L->sh_partial = defer_sh;
    ctx->L->pe_scene = scene;
    ctx->L->pe_P = P;
    return GS_OK;
}

// The fused preprocess + emission of a frame enqueued without a host round trip (k_pre_emit,
// events 0 and 1): entries in the split layout (duplicates from index n), (V, D) on the device
// and in the slot's pinned copy.  prefix_hist: the prefix sort's sampled histogram, or null.
int enqueue_pre_emit(gs_ctx *ctx, const gs_scene *scene, const gs_uniforms *u, uint32_t flags,
                     uint32_t *prefix_hist) {
    const int n = scene->n;
    const bool sh = (flags & GS_FLAG_SH) != 0;
    if (sh && !scene->sh) return set_error(ctx, GS_ERR_INVALID, "GS_FLAG_SH: the scene has no SH (gs_scene_set_sh)");
    if (int rc = ensure_splats(ctx, n)) return rc;
    if (sh && ctx->L->col_cap < n) {
        if (int rc = grow(ctx, ctx->L->col, (size_t)n)) return rc;
        ctx->L->col_cap = n;
    }
    if (int rc = begin_frame(ctx)) return rc;
    ctx->flags = flags;
    gs::PreParams P = pre_params(u, flags, n);
    P.sh = sh ? 1 : 0;
    ctx->rec_packed = gs::rec_packed(P);
    for (int c = 0; c < 3; ++c)
        P.campos[c] = -(u->view[4 * c + 0] * u->view[12] + u->view[4 * c + 1] * u->view[13] +
                        u->view[4 * c + 2] * u->view[14]);
    Lane &L = *ctx->L;
    uint64_t *cur = L.lb + (size_t)L.lb_par * L.lb_cap, *nxt = L.lb + (size_t)(L.lb_par ^ 1) * L.lb_cap;
    gs::LookbackDev lb{cur, nxt, L.lb_cap, ctx->lb_spin};
    L.lb_par ^= 1;
    gs::launch_pre_emit(L.stream, P, scene_dev(scene), frame_dev(ctx), lb, lazy_loads(ctx, n), L.keys, L.vals, (uint32_t)L.e_cap,
                        prefix_hist, fev(ctx, 0), fev(ctx, 1));
    GS_HIP(ctx, hipGetLastError());
    ctx->n = n;
    L.split = true;
    L.sh_partial = false;
    L.keys_sorted = true;
    L.vals_partial = false;
    L.pe_scene = scene;
    L.pe_P = P;
    return GS_OK;
}

int enqueue_emit(gs_ctx *ctx, uint32_t *prefix_hist = nullptr) {
    ctx->L->keys_sorted = true;  // emission order, as gs_frame_read shows it before gs_sort
    ctx->L->vals_partial = false;
    gs::launch_emit(ctx->L->stream, ctx->n, ctx->rec_packed, frame_dev(ctx), ctx->L->keys, ctx->L->vals, (uint32_t)ctx->L->e_cap, fev(ctx, 2),
                    fev(ctx, 3), prefix_hist);
    GS_HIP(ctx, hipGetLastError());
    return GS_OK;
}

// E entries, or (count != null) min(E, count[0] + count[1]) read on the device
// with_bins: the tile bins (gs_compute_bins' output) come from the sort's own histogram read;
// the bins stage is then empty (its timing event follows the sort's)
// A frame sort with bins leaves the keys unsorted (the blend reads the values and the bins
// only) when the splat ids fit 24 bits; gs_frame_read(GS_READ_KEYS) then sorts again.
// small: the small-frame form (with bins, no prefix; keys come out sorted)
int enqueue_sort(gs_ctx *ctx, int64_t E, const uint32_t *count, bool with_bins = false,
                 const gs::PrefixDev *pre = nullptr, int64_t dup_base = -1, bool small = false,
                 const gs::KeptSort *kept = nullptr) {
    small = small && with_bins && !pre;
    const bool keys_out = small || (!pre && (!with_bins || ctx->n > (1 << 24)));
    if (int rc = gs::sort_pairs(ctx->L->stream, ctx->L->sort, ctx->L->keys, ctx->L->vals, E, ctx->err, count, fev(ctx, 4),
                                fev(ctx, 5), with_bins ? ctx->L->bins : nullptr, keys_out, pre, dup_base, small,
                                small && ctx->bucket_sort, kept))
        return set_error(ctx, rc, ctx->err);
    ctx->L->keys_sorted = keys_out;
    ctx->L->vals_partial = pre != nullptr;
    if (with_bins)
        if (hipEvent_t e = fev(ctx, 6)) GS_HIP(ctx, hipEventRecord(e, ctx->L->stream));
    return GS_OK;
}

int enqueue_bins(gs_ctx *ctx, int64_t E, const uint32_t *count) {
    gs::launch_bins(ctx->L->stream, ctx->L->keys, E, count, ctx->L->bin_counts, ctx->L->bins, fev(ctx, 6));
    GS_HIP(ctx, hipGetLastError());
    return GS_OK;
}

int enqueue_draw(gs_ctx *ctx, const gs_scene *scene, int width, int height, float tile_w, float tile_h,
                 uint32_t flags, void *out_rgba8, int out_on_device, int64_t E, const uint32_t *count,
                 bool prefix = false) {
    const bool clean = (flags & GS_FLAG_CLEAN) != 0;
    gs::DrawParams P;
    P.W = width;
    P.H = height;
    P.E = (int32_t)E;
    P.count = count;
    P.clean = clean ? 1 : 0;
    P.no_cull = (flags & GS_FLAG_NO_CULL) ? 1 : 0;
    // Q9: the reference dispatches (W/32) x (H/32) workgroups of 32x32 pixels
    const int coverW = clean ? width : (width / 32) * 32;
    const int coverH = clean ? height : (height / 32) * 32;
    // tile pixel ranges with the kernel's own float formula: tileX = int(float(x) / tile_w)
    auto bounds = [](int cover, float tsz, int32_t *b) {
        for (int t = 0; t <= gs::kTiles; ++t) b[t] = cover;
        int prev = -1;
        for (int x = 0; x < cover; ++x) {
            int tt = (int)((float)x / tsz);
            tt = std::min(std::max(tt, 0), gs::kTiles);
            for (int q = prev + 1; q <= tt && q <= gs::kTiles; ++q) b[q] = x;
            prev = std::max(prev, tt);
        }
        b[0] = 0;
    };
    bounds(coverW, tile_w, P.xb);
    bounds(coverH, tile_h, P.yb);
    int mw = 0, mh = 0;
    for (int t = 0; t < gs::kTiles; ++t) {
        mw = std::max(mw, P.xb[t + 1] - P.xb[t]);
        mh = std::max(mh, P.yb[t + 1] - P.yb[t]);
    }
    // the sub-block form: the spec frame's count is the newest one seen (this frame's is on the device)
    const int64_t e_est = count ? ctx->E : E;
    const int64_t sub16 = (int64_t)gs::kTiles * gs::kTiles * ((mw + 15) / 16) * ((mh + 15) / 16);
    const bool small = ctx->draw_sub == 8 || (ctx->draw_sub == 0 && e_est < ctx->small_draw_entries &&
                                              sub16 <= kSmallDrawSubBlocks);
    const int sb = small ? 8 : 16;
    ctx->last_draw_sub = sb;
    P.nbx = (mw + sb - 1) / sb;
    P.nby = (mh + sb - 1) / sb;
    const size_t npx = (size_t)width * height;
    uint32_t *dst = (uint32_t *)out_rgba8;
    if (!out_on_device) {
        if (npx > ctx->L->img_cap) {
            if (int rc = grow(ctx, ctx->L->img, npx)) return rc;
            ctx->L->img_cap = npx;
        }
        dst = ctx->L->img;
    }
    P.coverW = coverW;
    P.coverH = coverH;
    P.n = scene->n;
    P.V = (int32_t)ctx->V;  // used when count is null (the frame's counts are on the host)
    P.prefix = prefix ? 1 : 0;
    P.depth = GS_PREFIX_DEPTH ? ctx->prefix_depth : nullptr;  // (every blend of the context refreshes the per-tile depths)
    P.sbox = (GS_DRAW_SBOX && prefix) ? ctx->L->sbox_base + 1 : nullptr;
    P.light_trace = (flags & GS_FLAG_DRAW_TRACE) ? 1 : 0;
    // GS_FLAG_SH frames blend the colours their preprocess evaluated
    const float4 *colour = (ctx->flags & GS_FLAG_SH) ? ctx->L->col : scene->colour;
    // Blends into one output land in frame order: wait for the frames in flight on other
    // lanes that blend into the same output (or, with GS_FLAG_DRAW_STATS, into the shared
    // stats buffer); frames into different outputs (a double-buffered texture) overlap.
    // Retired slots are complete; a slot's last event rides on its draw kernel.
    const bool with_stats = (flags & GS_FLAG_DRAW_STATS) != 0;
    for (int i = 0; i < kRing; ++i) {
        const gs_ctx::Slot &sl = ctx->slot[i];
        if (i == ctx->cur || !sl.used || !sl.drawn || sl.lane == ctx->cur_lane) continue;
        if (sl.draw_out == dst || (with_stats && sl.draw_stats))
            GS_HIP(ctx, hipStreamWaitEvent(ctx->L->stream, ctx->ev[i][kEv - 1], 0));
    }
    gs::launch_draw(ctx->L->stream, P, (flags & GS_FLAG_FAST_EXP) != 0, small, ctx->L->bins, ctx->L->vals, frame_dev(ctx), colour, dst, (flags & GS_FLAG_DRAW_STATS) ? ctx->draw_stats : nullptr, fev(ctx, 7),
                    fev(ctx, 8));
    GS_HIP(ctx, hipGetLastError());
    gs_ctx::Slot &me = ctx->slot[ctx->cur];
    me.lane = ctx->cur_lane;
    me.draw_out = dst;
    me.drawn = true;
    me.draw_stats = with_stats;
    if (!out_on_device) {
        GS_HIP(ctx, hipMemcpyAsync(out_rgba8, dst, npx * 4, hipMemcpyDeviceToHost, ctx->L->stream));
        GS_HIP(ctx, hipStreamSynchronize(ctx->L->stream));
    }
    return GS_OK;
}

// the host-synchronous frame: one 8-byte readback of (V, D) sizes the entry buffers
int render_sync(gs_ctx *ctx, const gs_scene *scene, const gs_uniforms *u, uint32_t flags, void *out,
                int out_on_device, gs_frame_stats *stats) {
    int rc;
    if ((rc = gs_preprocess(ctx, scene, u, flags, stats))) return rc;
    if ((rc = enqueue_sort(ctx, ctx->E, nullptr, true, nullptr, -1, ctx->E < ctx->small_sort_entries)))
        return rc;  // gs_sort + gs_compute_bins
    ctx->stage = 3;
    // src/Splats.cpp:596 draw(width, height, float(width) / 16.f, float(height) / 16.f)
    return gs_draw(ctx, scene, u->width, u->height, (float)u->width / 16.f, (float)u->height / 16.f, flags, out,
                   out_on_device);
}

// the speculative frame: no host round trip.  Kernels after the scan read the entry count on
// the device and are sized by the entry capacity (last observed count + 25 % + 64Ki); the
// slot keeps what is needed to render the frame again should the count exceed it.
int render_spec(gs_ctx *ctx, const gs_scene *scene, const gs_uniforms *u, uint32_t flags, void *out) {
    if (int rc = prepare_frame(ctx)) return rc;
    if (int rc = next_lane(ctx)) return rc;
    // (the split layout of the fused kernel, small scenes, holds the duplicates from index n on:
    // n + D entries)
    const int64_t n = scene->n;
    const int64_t want = std::max<int64_t>(ctx->E + ctx->E / 4 + 65536, n + ctx->D + ctx->D / 4 + 65536);
    if (ctx->L->e_cap < want)
        if (int rc = ensure_entries(ctx, want)) return rc;
    // prefix sort: frames of the size where the lists are long (the last observed count)
    // (enabled by the configured depth, not the doubled one: the per-tile depths keep what each
    // list needs, and a moving camera's occasional misses must not turn the prefix sort off)
    bool prefix = ctx->prefix_target > 0 && ctx->E >= (int64_t)64 * ctx->prefix_base;
    if (ctx->prefix_cooldown > 0) {  // (misses close together: the full sort for a while)
        ctx->prefix_cooldown -= 1;
        prefix = false;
    }
    gs::PrefixDev pd{};
    // passes 1-3 sized for the kept count of the newest retired prefix-sorted frame of the same
    // selection (with / without the depths) + 25 % (+ 64Ki); else every entry.  (Scaled by the
    // depth since: a miss doubles it, and the kept count roughly with it.)
    auto cap_for = [&](bool turned_sel) -> uint32_t {
        const int64_t cap_e = ctx->L->e_cap;
        const int64_t kept = ctx->prefix_kept_target > 0 && ctx->prefix_target > ctx->prefix_kept_target
                                 ? (int64_t)ctx->prefix_kept * ctx->prefix_target / ctx->prefix_kept_target
                                 : (int64_t)ctx->prefix_kept;
        const bool same_sel = ctx->prefix_kept_turned == turned_sel;
        return (uint32_t)(ctx->prefix_kept && same_sel && !ctx->prefix_after_miss
                              ? std::min<int64_t>(cap_e, kept * 5 / 4 + 65536)
                              : cap_e);
    };
    bool sel_turned = false;  // the selection this frame keeps by: the turned (neighbourhood) form
    if (prefix) {
        if (!ctx->L->pre_buf) {
            GS_HIP(ctx, hipMalloc(&ctx->L->pre_buf, gs::kPrefixWords * 4));
            GS_HIP(ctx, hipMemsetAsync(ctx->L->pre_buf, 0, gs::kPrefixWords * 4, ctx->L->stream));
        }
        uint32_t *b = ctx->L->pre_buf;  // (the lane's: enqueue_pre_emit keeps the lane)
        pd.hist = b;
        pd.theta = pd.hist + (size_t)gs::kPrefixHistCopies * 256 * gs::kPrefixBuckets;
        pd.counts = pd.theta + gs::kClasses;
        pd.nsel = pd.counts + (size_t)gs::kPrefixCopies * (gs::kClasses + 1);
        pd.delta = (int32_t *)(pd.nsel + 2);
        pd.cls = (uint32_t *)(pd.delta + gs::kClasses);
        pd.target = (uint32_t)ctx->prefix_target;
        if (!ctx->prefix_depth) {  // (zeroed before any frame can read it)
            GS_HIP(ctx, hipMalloc(&ctx->prefix_depth, 256 * 4));
            GS_HIP(ctx, hipMemset(ctx->prefix_depth, 0, 256 * 4));
        }
        pd.depth = GS_PREFIX_DEPTH ? ctx->prefix_depth : nullptr;
        // a camera that turned more than kPrefixTurnDeg since the frame before: the recorded
        // depths describe another view (their tiles' contents moved), so this frame's lists are
        // kept to the configured target instead (a fast pan missed on nearly every frame)
        pd.use_depth = ctx->have_prev_view && turn_cos(ctx->prev_view, u->view) < kPrefixTurnCos ? 0 : 1;
        sel_turned = pd.use_depth == 0;
        if (sel_turned && GS_PREFIX_TURN_RECTS && ctx->view_hist_n > 0) {
            // the depths come from the blends of up to nlanes frames back: each tile's sources in all
            // of those views
            turned_rects(u, ctx->view_hist,
                         std::min(ctx->view_hist_n, GS_PREFIX_TURN_VIEWS > 0 ? GS_PREFIX_TURN_VIEWS : ctx->nlanes),
                         ctx->tile_rects);
            pd.rects = &ctx->tile_rects;
        }
        pd.cap_sel = cap_for(sel_turned);
        pd.n = scene->n;
        pd.clean = (flags & GS_FLAG_CLEAN) ? 1 : 0;
        // GS_DRAW_SBOX: the cull boxes by sorted position, one per entry (only prefix-sorted frames
        // use them: allocated here, not with the entries; all ones = empty boxes until placed)
        if (GS_DRAW_SBOX && ctx->L->sbox_cap < ctx->L->e_cap) {
            if (int rc = grow(ctx, ctx->L->sbox_base, (size_t)ctx->L->e_cap + 1)) return rc;
            GS_HIP(ctx, hipMemsetAsync(ctx->L->sbox_base, 0xff, ((size_t)ctx->L->e_cap + 1) * 8, ctx->L->stream));
            ctx->L->sbox_cap = ctx->L->e_cap;
        }
    }
    const bool fused = gs::preprocess_blocks(scene->n) <= kFusedMaxBlocks;
    // GS_FLAG_SH with the prefix sort: colour only the kept entries' splats, after the sort
    const bool defer_sh = prefix && !fused && (flags & GS_FLAG_SH) && kShKept;
    // the kept emission (gs::KeptDev): a prefix-sorted frame of a large scene, not mostly culled,
    // whose camera did not turn since the frame before, emits only the entries at or below the
    // bounds the frame before it selected.  A turned frame emits every entry and selects its own
    // (its content moved: bounds selected at the other pose missed, tests/test_gpu_prefix.py);
    // either kind's select writes the bounds the next frame keeps by.
    const bool kept_base = prefix && !fused && ctx->kept_emit && !lazy_loads(ctx, scene->n);
    const bool kept_mode = kept_base && !sel_turned;
    const uint32_t *theta_in = nullptr;
    if (kept_base) {
        for (uint32_t *&t : ctx->theta_buf)
            if (!t) GS_HIP(ctx, hipMalloc(&t, gs::kClasses * 4));
        if (!ctx->theta_ev) GS_HIP(ctx, hipEventCreateWithFlags(&ctx->theta_ev, hipEventDisableTiming));
        const bool keep_all = kept_mode && (!ctx->theta_valid || ctx->theta_scene != scene);
        if (keep_all) {  // no bounds of this scene yet: keep everything
            static std::vector<uint32_t> all = [] {
                std::vector<uint32_t> a(gs::kClasses);
                for (int c = 0; c < 256; ++c) a[c] = gs::class_hi((uint32_t)c) - 1u;
                a[256] = 0xffffffffu;
                return a;
            }();
            if (ctx->theta_ev_live) GS_HIP(ctx, hipStreamWaitEvent(ctx->L->stream, ctx->theta_ev, 0));
            GS_HIP(ctx, hipMemcpyAsync(ctx->theta_buf[ctx->theta_cur], all.data(), gs::kClasses * 4,
                                       hipMemcpyHostToDevice, ctx->L->stream));
            // another scene's per-tile depths would size the bounds this frame selects for the
            // next one (which, unlike this frame, cannot hold more): forget them, as a new
            // context starts
            if (ctx->theta_scene && ctx->theta_scene != scene && ctx->prefix_depth)
                GS_HIP(ctx, hipMemsetAsync(ctx->prefix_depth, 0, 256 * 4, ctx->L->stream));
        } else if (kept_mode && ctx->theta_ev_live) {  // the frame before (another lane) wrote them
            GS_HIP(ctx, hipStreamWaitEvent(ctx->L->stream, ctx->theta_ev, 0));
        }
        // this frame's select: the bounds of the next frame (and a turned frame's own)
        pd.theta = ctx->theta_buf[ctx->theta_cur ^ 1];
        if (kept_mode) {
            theta_in = ctx->theta_buf[ctx->theta_cur];
            // the sort's four passes sized as passes 1-3 are (a frame keeping every entry: all)
            pd.cap_sel = keep_all ? (uint32_t)ctx->L->e_cap : cap_for(false);
        }
        ctx->theta_valid = true;
        ctx->theta_scene = scene;
    } else {
        ctx->theta_valid = false;  // (a frame between them: the bounds would be stale)
    }
    if (fused) {
        if (int rc = enqueue_pre_emit(ctx, scene, u, flags, prefix ? pd.hist : nullptr)) return rc;
    } else {
        if (int rc = enqueue_preprocess(ctx, scene, u, flags, defer_sh, theta_in)) return rc;
    }
    gs_ctx::Slot &sl = ctx->slot[ctx->cur];
    sl.spec = true;
    sl.scene = scene;
    sl.u = *u;
    sl.flags = flags;
    sl.out = out;
    sl.cap = ctx->L->e_cap;
    sl.fused = fused;
    sl.n = scene->n;
    const uint32_t *cnt = ctx->L->totals;
    if (prefix) {
        sl.cap_sel = pd.cap_sel;
        sl.target = ctx->prefix_target;
        sl.turned = sel_turned;
        pd.h_slot = ctx->h_ring_dev + kRingWords * ctx->cur;
        sl.prefix = true;
        ctx->prefix_frames += 1;
    }
    int rc;
    // the emission (the fused kernel's is done); the sort sized by the capacity (the entry count
    // stays on the device), reading the fused kernel's split layout as V + D entries
    gs::KeptSort ks{ctx->L->totals + 2, ctx->theta_ev};
    if (kept_mode) {
        gs::FrameDev fr = frame_dev(ctx);
        fr.theta_in = theta_in;
        // (the sort scratch holds the tile counters the emission adds to)
        if (int rc2 = gs::sort_ensure(ctx->L->sort, ctx->L->e_cap, ctx->err, ctx->L->stream)) return set_error(ctx, rc2, ctx->err);
        gs::KeptDev kd{ctx->L->sort.row_total + 256, pd.counts, pd.hist};
        ctx->L->keys_sorted = true;
        ctx->L->vals_partial = false;
        gs::launch_emit_kept(ctx->L->stream, ctx->n, ctx->rec_packed, fr, ctx->L->keys, ctx->L->vals, (uint32_t)ctx->L->e_cap,
                             kd, fev(ctx, 2), fev(ctx, 3));
        GS_HIP(ctx, hipGetLastError());
        ctx->kept_frames += 1;
    } else if (!fused && (rc = enqueue_emit(ctx, prefix ? pd.hist : nullptr))) {
        return rc;
    }
    if (kept_base && !kept_mode) {
        // a turned frame's select rewrites the bounds the frame before it kept by
        if (ctx->theta_ev_live) GS_HIP(ctx, hipStreamWaitEvent(ctx->L->stream, ctx->theta_ev, 0));
        ks.count = nullptr;
    }
    // (the lane's cull boxes exist once its preprocess was enqueued: a fresh lane allocates them there)
    pd.cullbox = ctx->L->cullbox;
    pd.box_out = GS_DRAW_SBOX && prefix ? ctx->L->sbox_base + 1 : nullptr;
    if ((rc = enqueue_sort(ctx, ctx->L->e_cap, cnt, true, prefix ? &pd : nullptr, fused ? scene->n : -1,
                           ctx->E < ctx->small_sort_entries, kept_base ? &ks : nullptr)))
        return rc;
    if (kept_base) {  // the next frame reads the bounds this frame's select writes
        ctx->theta_cur ^= 1;
        ctx->theta_ev_live = true;
    }
    if (defer_sh) {  // the kept entries' values: the sort's pass-2 output, left in the alternate buffer
        gs::launch_sh_kept(ctx->L->stream, ctx->L->pe_P, scene_dev(scene), frame_dev(ctx), ctx->L->sort.vals_alt,
                           pd.nsel, pd.cap_sel);
        GS_HIP(ctx, hipGetLastError());
    }
    if ((rc = enqueue_draw(ctx, scene, u->width, u->height, (float)u->width / 16.f, (float)u->height / 16.f, flags,
                           out, 1, ctx->L->e_cap, cnt, prefix)))
        return rc;
    ctx->stage = 3;
    return GS_OK;
}

}  // namespace

extern "C" {

int gs_preprocess(gs_ctx *ctx, const gs_scene *scene, const gs_uniforms *u, uint32_t flags, gs_frame_stats *stats) {
    if (int rc = check_frame_args(ctx, scene, u, "gs_preprocess")) return rc;
    if (int rc = validate_all(ctx)) return rc;
    if (int rc = prepare_frame(ctx)) return rc;
    if (int rc = next_lane(ctx)) return rc;  // a new frame
    if (int rc = enqueue_preprocess(ctx, scene, u, flags)) return rc;
    // E is needed on the host to size the sort (the reference maps its atomic counter back
    // every frame, src/Splats.cpp:579-583); one 8-byte readback, then emission.
    GS_HIP(ctx, hipStreamSynchronize(ctx->L->stream));  // (V, D) are in the slot's pinned copy
    ctx->V = ctx->h_ring[kRingWords * ctx->cur];
    ctx->D = ctx->h_ring[kRingWords * ctx->cur + 1];
    ctx->E = ctx->V + ctx->D;
    ctx->e_known = true;
    if (ctx->E >= ((int64_t)1 << 31)) return set_error(ctx, GS_ERR_INVALID, "gs_preprocess: more than 2^31 entries");
    if (int rc = ensure_entries(ctx, ctx->E)) return rc;
    if (int rc = enqueue_emit(ctx)) return rc;
    ctx->stage = 1;
    if (stats) {
        stats->num_splats = ctx->n;
        stats->visible = ctx->V;
        stats->duplicates = ctx->D;
        stats->entries = ctx->E;
    }
    return GS_OK;
}

int gs_sort(gs_ctx *ctx) {
    if (!ctx) return set_error(nullptr, GS_ERR_INVALID, "ctx is null");
    if (int rc = validate_all(ctx)) return rc;
    if (ctx->stage < 1) return set_error(ctx, GS_ERR_STATE, "gs_sort: call gs_preprocess first");
    if (int rc = use_device(ctx)) return rc;
    if (int rc = resort_full(ctx)) return rc;  // consistent (key, value) pairs after a frame sort
    if (int rc = enqueue_sort(ctx, ctx->E, nullptr)) return rc;
    ctx->stage = 2;
    return GS_OK;
}

int gs_compute_bins(gs_ctx *ctx) {
    if (!ctx) return set_error(nullptr, GS_ERR_INVALID, "ctx is null");
    if (int rc = validate_all(ctx)) return rc;
    if (ctx->stage < 2) return set_error(ctx, GS_ERR_STATE, "gs_compute_bins: call gs_sort first");
    if (int rc = use_device(ctx)) return rc;
    // the bins count the sorted keys: after a frame sort that left only the values sorted (or only
    // each list's prefix), the frame's entries are sorted again with their keys
    if (!ctx->L->keys_sorted || ctx->L->vals_partial)
        if (int rc = resort_full(ctx)) return rc;
    if (int rc = enqueue_bins(ctx, ctx->E, nullptr)) return rc;
    ctx->stage = 3;
    return GS_OK;
}

int gs_draw(gs_ctx *ctx, const gs_scene *scene, int width, int height, float tile_w, float tile_h, uint32_t flags,
            void *out_rgba8, int out_on_device) {
    if (!ctx || !scene || !out_rgba8) return set_error(ctx, GS_ERR_INVALID, "gs_draw: null argument");
    if (int rc = validate_all(ctx)) return rc;
    if (ctx->stage < 3) return set_error(ctx, GS_ERR_STATE, "gs_draw: call gs_compute_bins first");
    if (width <= 0 || height <= 0) return set_error(ctx, GS_ERR_INVALID, "gs_draw: bad resolution");
    if (scene->n != ctx->n) return set_error(ctx, GS_ERR_INVALID, "gs_draw: scene differs from the preprocessed one");
    if (int rc = use_device(ctx)) return rc;
    if (ctx->L->vals_partial)  // the whole sorted lists for a draw of them (the bins are exact)
        if (int rc = resort_full(ctx)) return rc;
    return enqueue_draw(ctx, scene, width, height, tile_w, tile_h, flags, out_rgba8, out_on_device, ctx->E, nullptr);
}

namespace {
int render_impl(gs_ctx *ctx, const gs_scene *scene, const gs_uniforms *u, uint32_t flags, void *out_rgba8,
                int out_on_device, gs_frame_stats *stats);
}

int gs_render(gs_ctx *ctx, const gs_scene *scene, const gs_uniforms *u, uint32_t flags, void *out_rgba8,
              int out_on_device, gs_frame_stats *stats) {
    if (!out_rgba8) return set_error(ctx, GS_ERR_INVALID, "gs_render: null argument");
    if (int rc = check_frame_args(ctx, scene, u, "gs_render")) return rc;
    // host cost of the call (enqueue vs blocked on frames in flight), gs_timing_read
    const auto t0 = std::chrono::steady_clock::now();
    ctx->in_render = true;
    const int rc = render_impl(ctx, scene, u, flags, out_rgba8, out_on_device, stats);
    ctx->in_render = false;
    ctx->acc.ms_host_render += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    ctx->acc.host_renders += 1;
    return rc;
}

}  // extern "C"

namespace {
int render_impl(gs_ctx *ctx, const gs_scene *scene, const gs_uniforms *u, uint32_t flags, void *out_rgba8,
                int out_on_device, gs_frame_stats *stats) {
    // no stats wanted, output on the device, an entry count seen before: enqueue the whole
    // frame without a host round trip (validated at gs_sync / the next readback)
    // (the prefix sort's turn test compares a frame's view with the frame before it)
    auto seen = [&](int rc) {
        if (rc == GS_OK) {
            std::memcpy(ctx->prev_view, u->view, sizeof(ctx->prev_view));
            ctx->have_prev_view = true;
            for (int i = kMaxLanes - 1; i > 0; --i) std::memcpy(ctx->view_hist[i], ctx->view_hist[i - 1], sizeof(ctx->view_hist[0]));
            std::memcpy(ctx->view_hist[0], u->view, sizeof(ctx->view_hist[0]));
            ctx->view_hist_n = std::min(ctx->view_hist_n + 1, kMaxLanes);
        }
        return rc;
    };
    if (!stats && out_on_device && ctx->e_known && !(flags & GS_FLAG_TIMING))
        return seen(render_spec(ctx, scene, u, flags, out_rgba8));
    ctx->theta_valid = false;  // (a kept emission after it starts from every entry)
    if (int rc = seen(render_sync(ctx, scene, u, flags, out_rgba8, out_on_device, stats))) return rc;
    if (flags & GS_FLAG_TIMING) {
        hipEvent_t *e = ctx->ev[ctx->cur];
        GS_HIP(ctx, hipEventSynchronize(e[8]));
        if (stats) {
            stats->ms_preprocess = elapsed(e[0], e[1]) + elapsed(e[2], e[3]);
            stats->ms_sort = elapsed(e[4], e[5]);
            stats->ms_bins = elapsed(e[5], e[6]);
            stats->ms_draw = elapsed(e[7], e[8]);
            stats->ms_total = elapsed(e[0], e[8]);
        }
    }
    return GS_OK;
}
}  // namespace

extern "C" {

int gs_last_stats(gs_ctx *ctx, gs_frame_stats *stats) {
    if (!ctx || !stats) return set_error(ctx, GS_ERR_INVALID, "gs_last_stats: null argument");
    if (int rc = gs_sync(ctx)) return rc;
    *stats = gs_frame_stats{};
    stats->num_splats = ctx->n;
    stats->visible = ctx->V;
    stats->duplicates = ctx->D;
    stats->entries = ctx->E;
    return GS_OK;
}

int gs_seen_stats(gs_ctx *ctx, gs_frame_stats *stats) {
    if (!ctx || !stats) return set_error(ctx, GS_ERR_INVALID, "gs_seen_stats: null argument");
    *stats = gs_frame_stats{};
    stats->num_splats = ctx->n;
    stats->visible = ctx->V;
    stats->duplicates = ctx->D;
    stats->entries = ctx->E;
    return GS_OK;
}

}  // extern "C"

namespace {
// The newest frame's entries again, emitted and sorted with their keys: after a frame sort
// that left the keys unsorted (keys_sorted false) or sorted only each list's prefix
// (vals_partial), for the stage calls and readbacks that need the whole sorted pairs.
int resort_full(gs_ctx *ctx) {
    if (ctx->stage < 2 || (ctx->L->keys_sorted && !ctx->L->vals_partial && !ctx->L->split)) return GS_OK;
    if (ctx->L->split) {  // a fused frame wrote no emission records: preprocess it again (staged path)
        if (!ctx->L->pe_scene) return set_error(ctx, GS_ERR_STATE, "the frame's scene was destroyed");
        const gs::FrameDev fr = frame_dev(ctx);
        gs::launch_preprocess(ctx->L->stream, ctx->L->pe_P, scene_dev(ctx->L->pe_scene), fr, nullptr);
        gs::launch_scan_blocksums(ctx->L->stream, fr, gs::preprocess_blocks(ctx->L->pe_P.n), nullptr, nullptr);
        GS_HIP(ctx, hipGetLastError());
        ctx->L->split = false;
    }
    if (ctx->L->sh_partial) {  // the SH colours of every splat with entries: the whole lists are drawn now
        if (!ctx->L->pe_scene) return set_error(ctx, GS_ERR_STATE, "the frame's scene was destroyed");
        gs::launch_sh_colour(ctx->L->stream, ctx->L->pe_P, scene_dev(ctx->L->pe_scene), frame_dev(ctx));
        GS_HIP(ctx, hipGetLastError());
        ctx->L->sh_partial = false;
    }
    gs::launch_emit(ctx->L->stream, ctx->n, ctx->rec_packed, frame_dev(ctx), ctx->L->keys, ctx->L->vals,
                    (uint32_t)ctx->L->e_cap, nullptr, nullptr);
    GS_HIP(ctx, hipGetLastError());
    if (int rc = gs::sort_pairs(ctx->L->stream, ctx->L->sort, ctx->L->keys, ctx->L->vals, ctx->E, ctx->err))
        return set_error(ctx, rc, ctx->err);
    ctx->L->keys_sorted = true;
    ctx->L->vals_partial = false;
    return GS_OK;
}
}  // namespace

extern "C" {

int gs_ctx_set_sort_prefix(gs_ctx *ctx, int target, int *current) {
    if (!ctx) return set_error(nullptr, GS_ERR_INVALID, "ctx is null");
    if (target >= 0) {
        ctx->prefix_base = ctx->prefix_target = target;
        ctx->prefix_clean_run = 0;
        ctx->prefix_cooldown = 0;
        ctx->prefix_miss_at[0] = ctx->prefix_miss_at[1] = ~0ull;
        ctx->prefix_after_miss = false;
        ctx->prefix_kept = 0;  // (passes 1-3 of the next prefix-sorted frame sized for every entry)
        ctx->theta_valid = false;  // (the next kept emission starts from every entry)
        if (ctx->prefix_depth) {  // a new target starts from a cold per-tile depth table (after the
            // frames in flight, whose blends write it)
            if (int rc = use_device(ctx)) return rc;
            if (int rc = validate_all(ctx)) return rc;
            if (int rc = sync_lanes(ctx)) return rc;
            GS_HIP(ctx, hipMemset(ctx->prefix_depth, 0, 256 * 4));
        }
    }
    if (current) *current = ctx->prefix_target;
    return GS_OK;
}

int gs_ctx_set_small_limits(gs_ctx *ctx, int64_t draw_entries, int64_t sort_entries) {
    if (!ctx) return set_error(nullptr, GS_ERR_INVALID, "ctx is null");
    if (draw_entries >= 0) ctx->small_draw_entries = draw_entries;
    if (sort_entries >= 0) ctx->small_sort_entries = sort_entries;
    return GS_OK;
}

int gs_ctx_set_bucket_sort(gs_ctx *ctx, int on) {
    if (!ctx) return set_error(nullptr, GS_ERR_INVALID, "ctx is null");
    if (on >= 0) ctx->bucket_sort = on != 0;
    return ctx->bucket_sort ? 1 : 0;
}

int gs_ctx_set_kept_emission(gs_ctx *ctx, int on, uint64_t *kept_frames) {
    if (!ctx) return set_error(nullptr, GS_ERR_INVALID, "ctx is null");
    if (on >= 0 && (on != 0) != ctx->kept_emit) {
        ctx->kept_emit = on != 0;
        ctx->theta_valid = false;  // (the next kept frame starts from every entry)
    }
    if (kept_frames) *kept_frames = ctx->kept_frames;
    return ctx->kept_emit ? 1 : 0;
}

int gs_ctx_set_lookback_spin(gs_ctx *ctx, int limit, uint64_t *redone) {
    if (!ctx) return set_error(nullptr, GS_ERR_INVALID, "ctx is null");
    if (limit >= 0) ctx->lb_spin = (uint32_t)limit;
    if (redone) *redone = ctx->lb_redo;
    return (int)std::min<uint32_t>(ctx->lb_spin, 0x7fffffffu);
}

int gs_ctx_set_draw_sub(gs_ctx *ctx, int sub, int *current) {
    if (!ctx) return set_error(nullptr, GS_ERR_INVALID, "ctx is null");
    if (sub != -1 && sub != 0 && sub != 8 && sub != 16)
        return set_error(ctx, GS_ERR_INVALID, "gs_ctx_set_draw_sub: sub must be 0 (by entry count), 8 or 16");
    if (sub >= 0) ctx->draw_sub = sub;
    if (current) *current = ctx->last_draw_sub;
    return GS_OK;
}

int gs_prefix_stats(gs_ctx *ctx, uint64_t out[4], int reset) {
    if (!ctx || !out) return set_error(ctx, GS_ERR_INVALID, "gs_prefix_stats: null argument");
    if (int rc = gs_sync(ctx)) return rc;
    out[0] = ctx->prefix_frames;
    out[1] = ctx->prefix_redo;
    out[2] = ctx->prefix_kept;
    out[3] = ctx->prefix_E;
    if (reset) ctx->prefix_frames = ctx->prefix_redo = 0;
    return GS_OK;
}

int gs_frame_read(gs_ctx *ctx, int what, void *host_dst, size_t count) {
    if (!ctx || (!host_dst && count)) return set_error(ctx, GS_ERR_INVALID, "gs_frame_read: null argument");
    if (int rc = gs_sync(ctx)) return rc;
    if (ctx->stage < 1) return set_error(ctx, GS_ERR_STATE, "gs_frame_read: no frame");
    if (int rc = use_device(ctx)) return rc;
    const void *src = nullptr;
    size_t avail = 0, esz = 4;
    // preprocess writes the blend records and boxes of splats with entries only; the rows of
    // the others read as the values a culled splat gets (zeros, the empty box)
    // culled(ty[r]): splat r has no entries (read after the stream sync)
    auto culled = [&](int32_t v) { return ctx->rec_packed ? v >= 0 : v < 0; };
    auto has_entries = [&](size_t rows, std::vector<int32_t> &ty) -> int {
        ty.resize(rows);
        if (ctx->rec_packed)  // word 1 of the 8-byte record, bit 31 set: has entries
            GS_HIP(ctx, hipMemcpy2DAsync(ty.data(), 4, (const char *)ctx->L->rec + 4, 8, 4, rows,
                                         hipMemcpyDeviceToHost, ctx->L->stream));
        else
            GS_HIP(ctx, hipMemcpy2DAsync(ty.data(), 4, (const char *)ctx->L->rec + 4, sizeof(int4), 4, rows,
                                         hipMemcpyDeviceToHost, ctx->L->stream));
        return GS_OK;
    };
    switch (what) {
    case GS_READ_KEYS:
        if (int rc = resort_full(ctx)) return rc;  // the frame's entries again, sorted with their keys
        src = ctx->L->keys; avail = (size_t)ctx->E; break;
    case GS_READ_VALS:
        if (ctx->L->vals_partial)
            if (int rc = resort_full(ctx)) return rc;
        src = ctx->L->vals; avail = (size_t)ctx->E; break;
    case GS_READ_BINS:
        if (ctx->stage < 3) return set_error(ctx, GS_ERR_STATE, "gs_frame_read: bins not computed");
        src = ctx->L->bins; avail = 256; break;
    case GS_READ_MEANS2D:
    case GS_READ_CONICS:
    case GS_READ_CULLBOX:
        // a fused frame (k_pre_emit) wrote no emission records, which mark the culled rows:
        // preprocess it again on the staged path (same records, and the emission records)
        if (ctx->L->split)
            if (int rc = resort_full(ctx)) return rc;
        break;
    default: break;
    }
    switch (what) {
    case GS_READ_MEANS2D:
    case GS_READ_CONICS: {  // fields of the 32-byte blend records
        const size_t comps = what == GS_READ_MEANS2D ? 2 : 4, off = what == GS_READ_MEANS2D ? 0 : 8;
        if (count > comps * (size_t)ctx->n) return set_error(ctx, GS_ERR_INVALID, "gs_frame_read: count exceeds the buffer");
        const size_t rows = (count + comps - 1) / comps;
        if (rows) {
            std::vector<float> tmp(rows * comps);
            std::vector<int32_t> ty;
            GS_HIP(ctx, hipMemcpy2DAsync(tmp.data(), comps * 4, (const char *)ctx->L->sd + off, sizeof(gs::SplatDraw),
                                         comps * 4, rows, hipMemcpyDeviceToHost, ctx->L->stream));
            if (int rc = has_entries(rows, ty)) return rc;
            GS_HIP(ctx, hipStreamSynchronize(ctx->L->stream));
            for (size_t r = 0; r < rows; ++r)
                if (culled(ty[r])) std::fill(tmp.begin() + r * comps, tmp.begin() + (r + 1) * comps, 0.0f);
            std::memcpy(host_dst, tmp.data(), count * 4);
        }
        return GS_OK;
    }
    case GS_READ_CULLBOX: {
        if (count > 4 * (size_t)ctx->n) return set_error(ctx, GS_ERR_INVALID, "gs_frame_read: count exceeds the buffer");
        const size_t rows = (count + 3) / 4;
        if (rows) {
            std::vector<float> tmp(rows * 4);
            std::vector<uint32_t> packed(rows * 2);
            std::vector<int32_t> ty;
            GS_HIP(ctx, hipMemcpyAsync(packed.data(), ctx->L->cullbox, rows * 8, hipMemcpyDeviceToHost, ctx->L->stream));
            if (int rc = has_entries(rows, ty)) return rc;
            GS_HIP(ctx, hipStreamSynchronize(ctx->L->stream));
            const float inf = std::numeric_limits<float>::infinity();
            for (size_t r = 0; r < rows; ++r) {  // biased 16-bit pixel bounds -> (x0, x1, y0, y1)
                for (int c = 0; c < 2; ++c) {
                    tmp[4 * r + 2 * c] = (float)((int)(packed[2 * r + c] & 0xffffu) - 32768);
                    tmp[4 * r + 2 * c + 1] = (float)((int)(packed[2 * r + c] >> 16) - 32768);
                }
                if (culled(ty[r])) {
                    tmp[4 * r] = inf;
                    tmp[4 * r + 1] = -inf;
                    tmp[4 * r + 2] = inf;
                    tmp[4 * r + 3] = -inf;
                }
            }
            std::memcpy(host_dst, tmp.data(), count * 4);
        }
        return GS_OK;
    }
    case GS_READ_KEYS:
    case GS_READ_VALS:
    case GS_READ_BINS: break;
    default: return set_error(ctx, GS_ERR_INVALID, "gs_frame_read: unknown buffer");
    }
    if (count > avail) return set_error(ctx, GS_ERR_INVALID, "gs_frame_read: count exceeds the buffer");
    if (count) {
        GS_HIP(ctx, hipMemcpyAsync(host_dst, src, count * esz, hipMemcpyDeviceToHost, ctx->L->stream));
        GS_HIP(ctx, hipStreamSynchronize(ctx->L->stream));
    }
    return GS_OK;
}

// ---------------------------------------------------------------- radix sort
int gs_argsort_f32(gs_ctx *ctx, const float *d_keys, int32_t *d_order, int64_t n) {
    if (!ctx || (n > 0 && (!d_keys || !d_order)) || n < 0) return set_error(ctx, GS_ERR_INVALID, "gs_argsort_f32: bad argument");
    if (n <= 1) return GS_OK;
    if (int rc = use_device(ctx)) return rc;
    if (int rc = validate_all(ctx)) return rc;  // see gs_memcpy_h2d (the outputs may alias a frame's)
    if ((size_t)n > ctx->L->ask_cap) {
        if (int rc = grow(ctx, ctx->L->ask, (size_t)n + (size_t)n / 4)) return rc;
        ctx->L->ask_cap = (size_t)n + (size_t)n / 4;
    }
    if (int rc = join_lanes(ctx)) return rc;
    gs::launch_gather_keys(ctx->L->stream, d_keys, d_order, ctx->L->ask, n, ctx->evs[0]);
    if (int rc = gs::sort_pairs(ctx->L->stream, ctx->L->sort, ctx->L->ask, (uint32_t *)d_order, n, ctx->err, nullptr, nullptr,
                                ctx->evs[1]))
        return set_error(ctx, rc, ctx->err);
    return mark_aux(ctx);
}

int gs_sort_pairs_u32(gs_ctx *ctx, uint32_t *d_keys, uint32_t *d_vals, int64_t n) {
    if (!ctx || (n > 0 && (!d_keys || !d_vals)) || n < 0) return set_error(ctx, GS_ERR_INVALID, "gs_sort_pairs_u32: bad argument");
    if (int rc = use_device(ctx)) return rc;
    if (int rc = validate_all(ctx)) return rc;  // see gs_memcpy_h2d
    if (int rc = join_lanes(ctx)) return rc;
    if (int rc = gs::sort_pairs(ctx->L->stream, ctx->L->sort, d_keys, d_vals, n, ctx->err, nullptr, ctx->evs[0], ctx->evs[1]))
        return set_error(ctx, rc, ctx->err);
    return mark_aux(ctx);
}

int gs_last_kernel_ms(gs_ctx *ctx, int kernel, float *ms) {
    if (!ctx || !ms) return set_error(ctx, GS_ERR_INVALID, "null argument");
    if (int rc = gs_sync(ctx)) return rc;
    if (kernel == GS_KERNEL_DRAW) *ms = elapsed(ctx->ev[ctx->cur][7], ctx->ev[ctx->cur][8]);
    else if (kernel == GS_KERNEL_SORT) *ms = elapsed(ctx->evs[0], ctx->evs[1]);
    else return set_error(ctx, GS_ERR_INVALID, "unknown kernel");
    return GS_OK;
}

int gs_draw_stats(gs_ctx *ctx, uint64_t out[16], int reset) {
    if (!ctx || !out) return set_error(ctx, GS_ERR_INVALID, "null argument");
    if (int rc = gs_sync(ctx)) return rc;
    std::vector<uint32_t> tr((size_t)gs::kDrawTraceBlocks * gs::kDrawTraceWords);
    GS_HIP(ctx, hipMemcpyAsync(tr.data(), ctx->draw_stats, tr.size() * 4, hipMemcpyDeviceToHost, ctx->L->stream));
    if (reset) GS_HIP(ctx, hipMemsetAsync(ctx->draw_stats, 0, gs::kDrawStatsBytes, ctx->L->stream));
    GS_HIP(ctx, hipStreamSynchronize(ctx->L->stream));
    std::memset(out, 0, 16 * sizeof(uint64_t));
    for (int b = 0; b < gs::kDrawTraceBlocks; ++b) {
        const uint32_t *r = tr.data() + (size_t)b * gs::kDrawTraceWords;
        if (r[1] == 0 && r[0] == 0) continue;  // block not drawn (or beyond its tile)
        const uint64_t cyc = (uint64_t)(uint32_t)(r[1] - r[0]);
        out[0] += 1;
        out[1] += r[2];
        out[2] += r[3];
        out[3] += r[7];
        out[4] = std::max<uint64_t>(out[4], r[2]);
        out[5] = std::max<uint64_t>(out[5], r[3]);
        out[6] = std::max<uint64_t>(out[6], cyc);
        out[7] += cyc;
        out[8] += r[4];
        out[9] += r[5];
        out[10] += r[6];
    }
    return GS_OK;
}

int gs_draw_block_trace(gs_ctx *ctx, uint32_t *out, int max_blocks) {
    if (!ctx || !out || max_blocks < 0) return set_error(ctx, GS_ERR_INVALID, "bad argument");
    if (int rc = gs_sync(ctx)) return rc;
    const int n = std::min(max_blocks, gs::kDrawTraceBlocks);
    std::vector<uint32_t> tr((size_t)n * gs::kDrawTraceWords);
    GS_HIP(ctx, hipMemcpyAsync(tr.data(), ctx->draw_stats, tr.size() * 4, hipMemcpyDeviceToHost, ctx->L->stream));
    GS_HIP(ctx, hipStreamSynchronize(ctx->L->stream));
    std::memcpy(out, tr.data(), tr.size() * 4);
    return n;
}

int gs_timing_enable(gs_ctx *ctx, int mode) {
    if (!ctx) return set_error(nullptr, GS_ERR_INVALID, "ctx is null");
    if (mode < 0 || mode > 2) return set_error(ctx, GS_ERR_INVALID, "gs_timing_enable: mode must be 0, 1 or 2");
    if (int rc = gs_sync(ctx)) return rc;
    if (int rc = retire_upto(ctx, ~0ull)) return rc;
    ctx->timing_mode = mode;
    return GS_OK;
}

int gs_timing_reset(gs_ctx *ctx) {
    if (!ctx) return set_error(nullptr, GS_ERR_INVALID, "ctx is null");
    if (int rc = gs_sync(ctx)) return rc;
    if (int rc = retire_upto(ctx, ~0ull)) return rc;
    ctx->acc = gs_timing{};
    return GS_OK;
}

int gs_timing_read(gs_ctx *ctx, gs_timing *out) {
    if (!ctx || !out) return set_error(ctx, GS_ERR_INVALID, "null argument");
    if (int rc = gs_sync(ctx)) return rc;
    if (int rc = retire_upto(ctx, ~0ull)) return rc;
    *out = ctx->acc;
    return GS_OK;
}

}  // extern "C"
