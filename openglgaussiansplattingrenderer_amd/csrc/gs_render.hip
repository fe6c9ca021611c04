// gs_render.hip -- gfx950 kernels of the frame: preprocess, entry emission, tile bins, blend.
//
// Reference semantics (paths relative to the reference checkout):
//   k_preprocess  shaders/preprocess.glsl:64-190   (one lane per splat, SoA coalesced loads)
//   k_emit        preprocess.glsl:153-188          (deterministic layout replacing the atomic
//                                                   counter: mains [0,V), duplicates [V,V+D))
//   k_bins_*      countBins.glsl + prefixBins.glsl
//   k_draw        draw.glsl:70-143                 (LDS-staged per-tile lists, block cull,
//                                                   block early exit)
// Float expressions are written in the same order as oracle/gs_oracle.c and compiled with
// contraction off, so means2D / conics / keys / bins match the CPU restatement bit for bit.
#pragma clang fp contract(off)

#include "gs_internal.hpp"

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <type_traits>

namespace gs {

namespace {

constexpr int kBlock = 256;

#ifndef GS_F2I_CVT
#define GS_F2I_CVT 1
#endif
__device__ __forceinline__ uint32_t f2u(float f) { return __float_as_uint(f); }
__device__ __forceinline__ float u2f(uint32_t u) { return __uint_as_float(u); }

// GLSL int(float) with v_cvt_i32_f32's out-of-range behaviour (saturate, NaN -> 0): the
// instruction itself (C++'s conversion is UB out of range, and the explicit checks compiled to
// three nested exec-mask branches per conversion; tools/micro/cvt_check.hip pins the two equal)
__device__ __forceinline__ int f2i(float f) {
#if GS_F2I_CVT
    int r;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(f));
    return r;
#else
    if (f != f) return 0;
    if (f >= 2147483648.0f) return 2147483647;
    if (f <= -2147483648.0f) return (-2147483647 - 1);
    return (int)f;
#endif
}

// the shape record of splat i (SceneDev::shape): covariance upper triangle c0..c5 and opacity
__device__ __forceinline__ void load_shape(const SceneDev &sc, size_t i, float &c0, float &c1, float &c2, float &c3,
                                           float &c4, float &c5, float &op) {
    const float *p = sc.shape + (size_t)kShapeFloats * i;
    const f32x4_a4 a = *reinterpret_cast<const f32x4_a4 *>(p);
    const f32x3_a4 b = *reinterpret_cast<const f32x3_a4 *>(p + 4);
    c0 = a.x, c1 = a.y, c2 = a.z, c3 = a.w, c4 = b.x, c5 = b.y, op = b.z;
}

// glm operator*(mat4, vec4): (m0*x + m1*y) + (m2*z + m3*w)
__device__ __forceinline__ float m4v_row(const float *m, int r, float x, float y, float z, float w) {
    return (m[0 * 4 + r] * x + m[1 * 4 + r] * y) + (m[2 * 4 + r] * z + m[3 * 4 + r] * w);
}

// glm operator*(mat3, mat3), column-major a[c][r]
struct M3 {
    float v[3][3];
};
__device__ __forceinline__ M3 mul3(const M3 &a, const M3 &b) {
    M3 o;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r) o.v[c][r] = a.v[0][r] * b.v[c][0] + a.v[1][r] * b.v[c][1] + a.v[2][r] * b.v[c][2];
    return o;
}
__device__ __forceinline__ M3 tr3(const M3 &a) {
    M3 o;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r) o.v[c][r] = a.v[r][c];
    return o;
}

// exp of draw.glsl:122 -- the definition the oracle states (ora_expf: Cody-Waite + degree-6
// Horner polynomial, each step one correctly rounded fma; 0 below -80, clamped at 80); every
// operation is IEEE-exact, so CPU == GPU bit for bit.  This is that function on the powers a
// blend event can carry (x <= 0 or NaN, see needs() in k_draw), where it is the same bits
// with the underflow branch as a select and the clamp inapplicable.
// UNDER false: for x known to lie in [-80, 0] (a blend batch whose events cannot reach the
// underflow cut, k_draw's evsafe): the same bits without the select
template <bool UNDER = true>
__device__ __forceinline__ float exp_defined_event(float x) {
    const float kf = rintf(x * 1.44269504088896341f);
    float r = __builtin_fmaf(-kf, 0.693359375f, x);
    r = __builtin_fmaf(-kf, -2.12194440e-4f, r);
    float t = __builtin_fmaf(0.00138888892f, r, 0.00833333377f);
    t = __builtin_fmaf(t, r, 0.0416666679f);
    t = __builtin_fmaf(t, r, 0.166666672f);
    t = __builtin_fmaf(t, r, 0.5f);
    t = __builtin_fmaf(t, r, 1.0f);
    const float p = __builtin_fmaf(t, r, 1.0f);
    // p * 2^k: for x in [-80, 0] k is in [-116, 0] and p in [0.7, 1.42], so 2^k and the product
    // are normal and exact: v_ldexp_f32 gives the oracle's p * u2f((k + 127) << 23) in one op
    const float v = __builtin_amdgcn_ldexpf(p, (int)kf);
    return (UNDER && !(x >= -80.0f)) ? 0.0f : v;
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// inclusive wave scan (wave64)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// exclusive block scan over 256 threads; returns prefix, *total = block sum
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t *s_wave, uint32_t *total) {
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan(v);
    if (lane == 63) s_wave[wid] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        const uint32_t c = s_wave[w];
        off += (w < wid) ? c : 0u;
        tot += c;
    }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

// ------------------------------------------------------------------ SH colour
// SURVEY f3 (beyond the reference, GS_FLAG_SH): degree-3 real spherical harmonics in the
// standard 3D Gaussian Splatting convention (coefficients SH_C0..SH_C3, the evaluation order of
// its computeColorFromSH), for the direction from the camera to the splat; colour =
// max(SH + 0.5, 0) * 255 so that with f_rest = 0 it is the reference's (0.5 + SH_C0 * f_dc) * 255
// wherever that is non-negative.  The oracle (ora_sh_colours) evaluates the same op sequence.
// one channel from its 16 coefficients k[j] (values in registers)
__device__ __forceinline__ float sh_channel_k(const float *k, float x, float y, float z) {
    const float SH_C0 = 0.28209479177387814f, SH_C1 = 0.4886025119029199f;
    const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f, -1.0925484305920792f,
                            0.5462742152960396f};
    const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f, 0.3731763325901154f,
                            -0.4570457994644658f, 1.445305721320277f, -0.5900435899266435f};
    float r = SH_C0 * k[0];
    r = r - SH_C1 * y * k[1] + SH_C1 * z * k[2] - SH_C1 * x * k[3];
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    r = r + SH_C2[0] * xy * k[4] + SH_C2[1] * yz * k[5] + SH_C2[2] * (2.0f * zz - xx - yy) * k[6] +
        SH_C2[3] * xz * k[7] + SH_C2[4] * (xx - yy) * k[8];
    r = r + SH_C3[0] * y * (3.0f * xx - yy) * k[9] + SH_C3[1] * xy * z * k[10] +
        SH_C3[2] * y * (4.0f * zz - xx - yy) * k[11] + SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * k[12] +
        SH_C3[4] * x * (4.0f * zz - xx - yy) * k[13] + SH_C3[5] * z * (xx - yy) * k[14] +
        SH_C3[6] * x * (xx - 3.0f * yy) * k[15];
    r = r + 0.5f;
    return fmaxf(r, 0.0f) * 255.0f;
}
// The scene's SH layout (gs_scene_set_sh): splat-major, 48 coefficients per splat
// (channel-major, 16c + j), 192 contiguous bytes read as 12 quads.  A wave's lanes of culled
// splats load nothing, so only the visible splats' bytes move (0.9 of 1.18 GB at C3): 232 us
// against 294 for per-coefficient planes or 64-splat quad-major groups, whose lines mix
// visible and culled splats.
__device__ __forceinline__ float4 sh_quad(const float *sh, size_t i, int q) {
    return reinterpret_cast<const float4 *>(sh)[i * 12 + (size_t)q];
}
__device__ __forceinline__ float sh_channel(const float *sh, size_t n, size_t i, int c, float x, float y, float z) {
    (void)n;
    float k[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float4 v = sh_quad(sh, i, 4 * c + q);
        k[4 * q] = v.x, k[4 * q + 1] = v.y, k[4 * q + 2] = v.z, k[4 * q + 3] = v.w;
    }
    return sh_channel_k(k, x, y, z);
}

// The SH colours of a frame's splats with entries (GS_FLAG_SH), after k_preprocess (its emission
// records say which): one splat per lane, all 48 coefficient loads issued before the arithmetic
// (12 coalesced 1-KB quad loads per wave, sh_quad) -- in the preprocess they came after its own
// loads and math, under its register budget, in several round trips per item.
#ifndef GS_SH_WAVES
#define GS_SH_WAVES 4
#endif
template <bool PACK>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(GS_SH_WAVES))) void k_sh_colour(PreParams P, SceneDev sc, FrameDev fr) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= P.n) return;
    const bool has = PACK ? (reinterpret_cast<const uint2 *>(fr.rec)[i].y >> 31) != 0 : fr.rec[i].y >= 0;
    if (!has) return;
    float k[48];
    float4 v[12];
#pragma unroll
    for (int q = 0; q < 12; ++q) v[q] = sh_quad(sc.sh, (size_t)i, q);
    float mx = sc.mx[i], my = sc.my[i], mz = sc.mz[i];
    // all fifteen loads in flight before any arithmetic (left alone, the compiler split them into
    // batches behind waits: three or four memory round trips per wave)
#pragma unroll
    for (int q = 0; q < 12; ++q) asm volatile("" : "+v"(v[q].x), "+v"(v[q].y), "+v"(v[q].z), "+v"(v[q].w));
    asm volatile("" : "+v"(mx), "+v"(my), "+v"(mz));
#pragma unroll
    for (int q = 0; q < 12; ++q) k[4 * q] = v[q].x, k[4 * q + 1] = v[q].y, k[4 * q + 2] = v[q].z, k[4 * q + 3] = v[q].w;
    float dx = mx - P.campos[0], dy = my - P.campos[1], dz = mz - P.campos[2];
    const float len = sqrtf(dx * dx + dy * dy + dz * dz);
    dx = dx / len;
    dy = dy / len;
    dz = dz / len;
    fr.col[i] = make_float4(sh_channel_k(k, dx, dy, dz), sh_channel_k(k + 16, dx, dy, dz), sh_channel_k(k + 32, dx, dy, dz),
                            1.0f);
}

// The SH colours of a prefix-sorted frame (GS_FLAG_SH), after its sort: only the splats of the
// kept entries -- the only ones its blend can read (a blend reaching past them flags the frame,
// which is rendered again on the synchronous path, k_sh_colour included) -- instead of every
// splat with entries: at C3 ~1.2M kept entries against 4.7M visible splats, a quarter of the
// coefficient bytes.  ids[0, min(count[0], cap)): the kept entries' splat ids (the sort's pass-2
// output, any order); thread `n` also colours splat 0, which the reference's culled entries
// draw.  A splat kept in several tiles is coloured by each of its entries (the same bits).
template <bool PACK>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(GS_SH_WAVES))) void k_sh_kept(
    PreParams P, SceneDev sc, FrameDev fr, const uint32_t *__restrict__ ids, const uint32_t *__restrict__ count,
    uint32_t cap) {
    const uint32_t n = min(count[0], cap);
    const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    if (j > n) return;
    const uint32_t i = j < n ? min(ids[j], (uint32_t)max(P.n - 1, 0)) : 0u;
    const bool has = PACK ? (reinterpret_cast<const uint2 *>(fr.rec)[i].y >> 31) != 0 : fr.rec[i].y >= 0;
    if (!has || P.n == 0) return;
    float k[48];
    float4 v[12];
#pragma unroll
    for (int q = 0; q < 12; ++q) v[q] = sh_quad(sc.sh, (size_t)i, q);
    float mx = sc.mx[i], my = sc.my[i], mz = sc.mz[i];
#pragma unroll
    for (int q = 0; q < 12; ++q) asm volatile("" : "+v"(v[q].x), "+v"(v[q].y), "+v"(v[q].z), "+v"(v[q].w));
    asm volatile("" : "+v"(mx), "+v"(my), "+v"(mz));
#pragma unroll
    for (int q = 0; q < 12; ++q) k[4 * q] = v[q].x, k[4 * q + 1] = v[q].y, k[4 * q + 2] = v[q].z, k[4 * q + 3] = v[q].w;
    float dx = mx - P.campos[0], dy = my - P.campos[1], dz = mz - P.campos[2];
    const float len = sqrtf(dx * dx + dy * dy + dz * dz);
    dx = dx / len;
    dy = dy / len;
    dz = dz / len;
    fr.col[i] = make_float4(sh_channel_k(k, dx, dy, dz), sh_channel_k(k + 16, dx, dy, dz), sh_channel_k(k + 32, dx, dy, dz),
                            1.0f);
}

// ------------------------------------------------------------------ preprocess
// kPer splats per lane, striped (splat = block*kSplatsPerBlock + k*256 + lane) so every load
// stays coalesced; one (main, dup) sum per workgroup feeds the emission scan.
constexpr int kPer = 4;
constexpr int kSplatsPerBlock = kPer * kBlock;  // 1024

// The emission record of splat i (rec): z01 bits, main tile, tile rect, "has entries".  PACK: 8
// bytes -- z01 bits, then tileX | tileY << 5 | minX << 10 | maxX << 15 | minY << 20 | maxY << 25 |
// has << 31 (every field fits 5 bits whenever the tile sizes are >= 1 px: tileX <= W / int(W/16)
// <= 31, min clamped to 16, max <= 15); else (reference mode below 16 px, tile size 0, where the
// main tile saturates) the 16-byte (z01 bits, tileX, tileY, rect bytes) form.
__device__ __forceinline__ uint32_t pack_rec(int tileX, int tileY, uint32_t rp) {
    return (uint32_t)tileX | ((uint32_t)tileY << 5) | ((rp & 0xffu) << 10) | (((rp >> 8) & 0xffu) << 15) |
           (((rp >> 16) & 0xffu) << 20) | ((rp >> 24) << 25) | 0x80000000u;
}
__device__ __forceinline__ int4 unpack_rec(uint2 r) {
    if (!(r.y >> 31)) return make_int4((int)r.x, -1, -1, 0);
    const uint32_t w = r.y;
    const uint32_t rp = ((w >> 10) & 31u) | (((w >> 15) & 31u) << 8) | (((w >> 20) & 31u) << 16) | (((w >> 25) & 31u) << 24);
    return make_int4((int)r.x, (int)(w & 31u), (int)((w >> 5) & 31u), (int)rp);
}

// The cull box as 16-bit pixel bounds biased by 32768 (unsigned), 8 bytes:
// (floor x0 | ceil x1 << 16, floor y0 | ceil y1 << 16), clamped to [-32768, 32767] -- never
// smaller than the float box, so the cull stays conservative (an empty box stays empty: +inf /
// -inf clamp to 32767 / -32768; NaN bounds open up).  The bias makes the blend's tests plain
// unsigned compares (kBoxBias).
constexpr int kBoxBias = 32768;
__device__ __forceinline__ uint2 pack_box(const float4 &b) {
    auto lo = [](float v) { return (uint32_t)((int)fminf(fmaxf(floorf(v), -32768.0f), 32767.0f) + kBoxBias); };  // NaN -> 0
    auto hi = [](float v) { return (uint32_t)((int)fmaxf(fminf(ceilf(v), 32767.0f), -32768.0f) + kBoxBias); };   // NaN -> 65535
    return make_uint2(lo(b.x) | (hi(b.y) << 16), lo(b.z) | (hi(b.w) << 16));
}

// One splat of preprocess.glsl:64-190: its blend record, cull box and (GS_FLAG_SH) colour
// written when it has entries, and its emission record returned: (z01 bits, tileX, tileY, rect)
// or (0, -1, -1, 0) without entries (culled, det == 0, or i out of range).
// CLEAN: clean mode (P.clean) as a template parameter -- a uniform flag's alternatives were
// if-converted into selects that every splat evaluated.
// LAZY: the covariance and opacity (28 of the 40 bytes) are loaded only for the lanes that pass
// the NDC cull, one round trip later -- for frames where most splats are culled (the small C5
// views: ~97 % culled, a 64-byte line of a plane then mostly holds culled splats only);
// otherwise all ten planes are loaded in one round trip.
// :77-89 the projection and the NDC cull: (p0, p1, p2) and whether x / y lie inside [-1, 1]
__device__ __forceinline__ bool project_ndc(const PreParams &P, float mx, float my, float mz, float &p0, float &p1,
                                            float &p2) {
    p0 = m4v_row(P.vp, 0, mx, my, mz, 1.0f);
    p1 = m4v_row(P.vp, 1, mx, my, mz, 1.0f);
    p2 = m4v_row(P.vp, 2, mx, my, mz, 1.0f);
    const float p3 = m4v_row(P.vp, 3, mx, my, mz, 1.0f);
    const float w = fmaxf(p3, 0.0001f);
    p0 = p0 / w;
    p1 = p1 / w;
    p2 = p2 / w;
    return !(p0 < -1.0f || p0 > 1.0f || p1 < -1.0f || p1 > 1.0f);
}

// splat 0 without entries: the record its culled entries draw (preprocess.glsl:80-88 splatKeys
// = 0, reached by a Q10 over-read; k_draw) -- means2D, conic and opacity 0 (never blends:
// threshold +inf, empty box)
__device__ __forceinline__ void write_culled_splat0(const FrameDev &fr) {
    const float inf = __builtin_inff();
    fr.sd[0] = SplatDraw{0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    fr.cullbox[0] = pack_box(make_float4(inf, -inf, inf, -inf));
}

template <bool CLEAN, bool SH = true>
__device__ __forceinline__ int4 preprocess_rest(const PreParams &P, const SceneDev &sc, const FrameDev &fr, int i,
                                                float mx, float my, float mz, float p0, float p1, float p2, bool vis,
                                                float c0, float c1, float c2, float c3, float c4, float c5, float opac);

// One splat of preprocess.glsl:64-190: its blend record, cull box and (GS_FLAG_SH) colour
// written when it has entries, and its emission record returned: (z01 bits, tileX, tileY, rect)
// or (0, -1, -1, 0) without entries (culled, det == 0, or i out of range).
// CLEAN: clean mode (P.clean) as a template parameter -- a uniform flag's alternatives were
// if-converted into selects that every splat evaluated.
// LAZY: the covariance and opacity (28 of the 40 bytes) are loaded only for the lanes that pass
// the NDC cull, one round trip later -- for frames where most splats are culled (the small C5
// views: ~97 % culled, a 64-byte line of a plane then mostly holds culled splats only);
// otherwise all ten planes are loaded in one round trip.
template <bool CLEAN, bool LAZY>
__device__ __forceinline__ int4 preprocess_one(const PreParams &P, const SceneDev &sc, const FrameDev &fr, int i,
                                               bool valid) {
    if (!valid) return make_int4(0, -1, -1, 0);
    const float mx = sc.mx[i], my = sc.my[i], mz = sc.mz[i];
    float c0, c1, c2, c3, c4, c5, opac;
    if (!LAZY) load_shape(sc, (size_t)i, c0, c1, c2, c3, c4, c5, opac);  // the means and the shape record in one round trip (see LAZY)
    // Straight-line body: every cull folds into `vis` and the outputs are selected at the
    // end (the NDC cull splits nearly every wave, so a branch saved no work; without branches
    // all ten plane loads issue up front and no exec-mask bookkeeping runs).  Culled lanes
    // compute garbage (inf / NaN) that is never used.
    float p0, p1, p2;
    const bool vis = project_ndc(P, mx, my, mz, p0, p1, p2);
    if (LAZY) {
        c0 = c1 = c2 = c3 = c4 = c5 = opac = 0.0f;
        if (vis) load_shape(sc, (size_t)i, c0, c1, c2, c3, c4, c5, opac);
    }
    return preprocess_rest<CLEAN>(P, sc, fr, i, mx, my, mz, p0, p1, p2, vis, c0, c1, c2, c3, c4, c5, opac);
}

// preprocess.glsl:91-190 after the NDC cull (vis: the splat passed it).  SH: the GS_FLAG_SH
// colour here (k_pre_emit); the other kernels leave it to k_sh_colour.
template <bool CLEAN, bool SH>
__device__ __forceinline__ int4 preprocess_rest(const PreParams &P, const SceneDev &sc, const FrameDev &fr, int i,
                                                float mx, float my, float mz, float p0, float p1, float p2, bool vis,
                                                float c0, float c1, float c2, float c3, float c4, float c5, float opac) {
    const size_t n = (size_t)P.n;
    // :91-94
    float sx = (p0 + 1.0f) * 0.5f, sy = (p1 + 1.0f) * 0.5f;
    const float sz = (p2 + 1.0f) * 0.5f;
    sx = sx * (float)P.W;
    sy = sy * (float)P.H;
    if (CLEAN) vis = vis && (sz >= 0.0f && sz <= 1.0f);  // clean: near/far cull (Q6)
    // :98-108 covariance (symmetric) and W3 (upper-left of the view matrix)
    const M3 Sig = {{{c0, c1, c2}, {c1, c3, c4}, {c2, c4, c5}}};
    const M3 W3 = {{{P.view[0], P.view[1], P.view[2]}, {P.view[4], P.view[5], P.view[6]},
                    {P.view[8], P.view[9], P.view[10]}}};
    // :110-116
    float tx = m4v_row(P.view, 0, mx, my, mz, 1.0f);
    float ty = m4v_row(P.view, 1, mx, my, mz, 1.0f);
    const float tz = m4v_row(P.view, 2, mx, my, mz, 1.0f);
    const float limx = -1.3f * P.tan_fov_x, limy = -1.3f * P.tan_fov_y;
    const float txtz = tx / tz, tytz = ty / tz;
    tx = fminf(limx, fmaxf(-limx, txtz)) * tz;
    ty = fminf(limy, fmaxf(-limy, tytz)) * tz;
    // :118-128
    const M3 J = {{{P.fx / tz, 0.0f, -(P.fx * tx) / (tz * tz)},
                   {0.0f, P.fy / tz, -(P.fy * ty) / (tz * tz)},
                   {0.0f, 0.0f, 0.0f}}};
    const M3 T = mul3(tr3(W3), J);
    M3 C = mul3(mul3(tr3(T), tr3(Sig)), T);
    C.v[0][0] += 0.3f;
    C.v[1][1] += 0.3f;
    // :129-136
    const float ca = C.v[0][0], cb = C.v[0][1], cc = C.v[1][1];
    const float det = ca * cc - cb * cb;
    vis = vis && det != 0;  // Q7: entry omitted
    if (CLEAN) vis = vis && det > 0.0f;
    const float inv = 1.0f / det;
    const float4 cov2 = make_float4(cc * inv, -cb * inv, ca * inv, opac);
    // :139-149
    const float middle = (cc + ca) * 0.5f;
    const float l1 = middle + sqrtf(fmaxf(0.1f, middle * middle - det));
    const float l2 = middle - sqrtf(fmaxf(0.1f, middle * middle - det));
    const float radius = ceilf(3.0f * sqrtf(fmaxf(l1, l2)));
    const int minX = max(0, f2i((sx - radius) / P.tile_w));
    const int maxX = min(15, f2i((sx + radius) / P.tile_w));
    const int minY = max(0, f2i((sy - radius) / P.tile_h));
    const int maxY = min(15, f2i((sy + radius) / P.tile_h));
    // :151-155 main tile (unclamped in ref mode, Q5)
    int tileX = f2i(sx / P.tile_w), tileY = f2i(sy / P.tile_h);
    if (CLEAN) {
        tileX = min(15, max(0, tileX));
        tileY = min(15, max(0, tileY));
    }
    const uint32_t rp = (uint32_t)min(minX, 16) | ((uint32_t)maxX << 8) | ((uint32_t)min(minY, 16) << 16) |
                        ((uint32_t)maxY << 24);

    // Conservative pixel box of the region where alpha >= 1/255 can hold
    // (draw.glsl:115-126): q = A dx^2 + 2B dx dy + C dy^2 <= 2 ln(255 o).  Margins
    // cover the rounding of power/exp (relative q error <= ~6 eps * cond), so
    // culling an entry outside the box never changes a pixel.
    // The box and the pre-exp threshold only cull (they never enter a pixel's
    // arithmetic) and carry margins far above hardware-instruction error (0.05 in ln,
    // 2 % in the half-widths, 1e-3 in the threshold), so they use v_log / v_rcp /
    // v_sqrt instead of the correctly rounded library sequences.
    const float A = cov2.x, B = cov2.y, Cq = cov2.z;
    const float lg = draw_log255o(opac);  // ln(255 o)
    const float tau = lg + 0.05f;
    const float detQ = A * Cq - B * B;
    const float trq = A + Cq;
    const bool wellc = A > 0.0f && Cq > 0.0f && detQ > 0.0f && trq * trq < 1.0e5f * detQ;
    const float rq = __builtin_amdgcn_rcpf(detQ);
    const float hx = __builtin_amdgcn_sqrtf(2.0f * tau * Cq * rq) * 1.02f + 1.0f;
    const float hy = __builtin_amdgcn_sqrtf(2.0f * tau * A * rq) * 1.02f + 1.0f;
    const float inf = __builtin_inff();
    // tau <= 0: never reaches 1/255 anywhere (empty box); ill-conditioned: unbounded box
    const float4 box = !(tau > 0.0f) ? make_float4(inf, -inf, inf, -inf)
                       : wellc       ? make_float4(sx - hx, sx + hx, sy - hy, sy + hy)
                                     : make_float4(-inf, inf, -inf, inf);
    const float2 m2 = make_float2(sx, sy);
    const float4 co = cov2;
    const int4 rc = vis ? make_int4((int)f2u(sz), tileX, tileY, (int)rp) : make_int4(0, -1, -1, 0);
    // pre-exp threshold of the blend: power < thr implies alpha < 1/255 (draw.glsl:123-126)
    // for any exp within a few ulp; 255*o <= 0 gives +inf (never blends); NaN (opacity NaN)
    // becomes -inf, which never skips
    // the blend record, box and (GS_FLAG_SH) colour are read only through entries: written
    // for the splats that have some (gs_frame_read shows the others as culled), and for
    // splat 0, which the reference's culled entries draw (preprocess.glsl:80-88 splatKeys = 0,
    // reached by a Q10 over-read; k_draw): without entries its record is the culled one --
    // means2D, conic and opacity 0 (never blends: threshold +inf, empty box)
    if (rc.y >= 0) {
        fr.sd[i] = SplatDraw{m2.x, m2.y, co.x, co.y, co.z, co.w};
        fr.cullbox[i] = pack_box(box);
        if (SH && P.sh) {  // GS_FLAG_SH: this frame's colour
            float dx = mx - P.campos[0], dy = my - P.campos[1], dz = mz - P.campos[2];
            const float len = sqrtf(dx * dx + dy * dy + dz * dz);
            dx = dx / len;
            dy = dy / len;
            dz = dz / len;
            fr.col[i] = make_float4(sh_channel(sc.sh, n, i, 0, dx, dy, dz), sh_channel(sc.sh, n, i, 1, dx, dy, dz),
                                    sh_channel(sc.sh, n, i, 2, dx, dy, dz), 1.0f);
        }
    } else if (i == 0) {  // splat 0 culled: the record its culled entries draw
        write_culled_splat0(fr);
    }
    return rc;
}

// duplicates of an emission record: the rect's tiles minus the main tile when it lies in the rect
__device__ __forceinline__ uint32_t rec_dups(const int4 &rc) {
    const int minX = rc.w & 0xff, maxX = (rc.w >> 8) & 0xff, minY = (rc.w >> 16) & 0xff, maxY = (rc.w >> 24) & 0xff;
    const int rectCount = (maxX >= minX && maxY >= minY) ? (maxX - minX + 1) * (maxY - minY + 1) : 0;
    const int mainInRect = (rc.y >= minX && rc.y <= maxX && rc.z >= minY && rc.z <= maxY) ? 1 : 0;
    return rc.y >= 0 ? (uint32_t)(rectCount - mainInRect) : 0u;
}

// The kept emission's count for one splat's entries (emission record rc, with entries): whether
// its main entry and how many of its duplicates have keys at or below their class bound -- the
// same keys k_emit_kept computes (tile + z01 as floats), the same test
__device__ __forceinline__ uint2 kept_of(const int4 &rc, const uint32_t *s_theta) {
    const float z = u2f((uint32_t)rc.x);
    const uint32_t mkey = f2u((float)((uint32_t)rc.z * 16u + (uint32_t)rc.y) + z);
    const uint32_t km = mkey <= s_theta[key_class(mkey)] ? 1u : 0u;
    const int minX = rc.w & 0xff, maxX = (rc.w >> 8) & 0xff, minY = (rc.w >> 16) & 0xff, maxY = (rc.w >> 24) & 0xff;
    uint32_t kd = 0;
    for (int ty = minY; ty <= maxY; ++ty)
        for (int tx = minX; tx <= maxX; ++tx) {
            if (tx == rc.y && ty == rc.z) continue;  // the main tile (preprocess.glsl:171-188)
            const uint32_t key = f2u((float)(ty * 16 + tx) + z);
            kd += key <= s_theta[key_class(key)] ? 1u : 0u;
        }
    return make_uint2(km, kd);
}

template <bool PACK, bool CLEAN, bool LAZY, bool KEPT = false>
__global__ __launch_bounds__(kBlock) void k_preprocess(PreParams P, SceneDev sc, FrameDev fr) {
    __shared__ uint32_t s_wave[kBlock / 64];
    __shared__ uint32_t s_theta[KEPT ? kClasses : 1];
    if (KEPT) {
        for (int c = threadIdx.x; c < kClasses; c += kBlock) s_theta[c] = fr.theta_in[c];
        __syncthreads();
    }
    uint32_t n_main = 0, n_dup = 0, n_km = 0, n_kd = 0;
#pragma unroll 1
    for (int it = 0; it < kPer; ++it) {
        const int i = blockIdx.x * kSplatsPerBlock + it * kBlock + threadIdx.x;
        const int4 rc = preprocess_one<CLEAN, LAZY>(P, sc, fr, i, i < P.n);
        n_main += rc.y >= 0 ? 1u : 0u;
        n_dup += rec_dups(rc);
        if (KEPT && rc.y >= 0) {  // (only splats with entries: i < P.n)
            const uint2 k = kept_of(rc, s_theta);
            n_km += k.x;
            n_kd += k.y;
            fr.kdup[i] = (uint16_t)k.y;
        }
        if (i < P.n) {
            if (PACK)
                reinterpret_cast<uint2 *>(fr.rec)[i] =
                    make_uint2((uint32_t)rc.x, rc.y >= 0 ? pack_rec(rc.y, rc.z, (uint32_t)rc.w) : 0u);
            else
                fr.rec[i] = rc;
        }
    }
    // block sums of (main, dup) for the emission offsets
    uint32_t tot_main, tot_dup;
    {  // one scan of both: mains in the low 11 bits (<= 1024 per block), duplicates above (<= 256
       // per splat, main tile outside the rect included: <= 262144 per block, 21 bits)
        uint32_t tot;
        block_excl_scan256(n_main | (n_dup << 11), s_wave, &tot);
        tot_main = tot & 0x7ffu;
        tot_dup = tot >> 11;
    }
    if (threadIdx.x == 0) fr.blocksum[blockIdx.x] = make_uint2(tot_main, tot_dup);
    if (KEPT) {  // the kept entries' block sums (the same packing)
        uint32_t tot;
        block_excl_scan256(n_km | (n_kd << 11), s_wave, &tot);
        if (threadIdx.x == 0) fr.blocksum_k[blockIdx.x] = make_uint2(tot & 0x7ffu, tot >> 11);
    }
}

// The same records with the NDC cull compacted out (QUEUE form).  kQWaves waves share a
// workgroup's kSplatsPerBlock splats (the block sums keep k_emit's granularity), each wave a
// contiguous run of kQItems * 64.  For each 64 of them a wave runs the projection (project_ndc),
// writes the culled splats' records at once and pushes the survivors -- (index, p0, p1, p2) --
// into a queue held in registers, one entry per lane, by a forward permute (ds_permute: the
// survivors to the next free queue lanes, the others to the remaining lanes, a permutation, so
// no two lanes collide).  Whenever 64 entries are queued they become the pending chunk: their
// ten plane loads are issued at once and every lane runs the rest of the preprocess
// (preprocess_rest) on one of them one projection step later, so the gathers are in flight
// behind that step's arithmetic (as the next projection's three loads are behind this one's);
// the remainder is flushed at the end.  The straight-line form (k_preprocess) computes the whole
// preprocess in every lane of a wave that has any survivor -- nearly every wave, so the culled
// splats' share of its arithmetic was spent for nothing (24 % at C3; ~97 % in the small C5
// views, where this also leaves their covariance and opacity unread).
#ifndef GS_QWAVES
#define GS_QWAVES 2
#endif
constexpr int kQWaves = GS_QWAVES;
constexpr int kQItems = kSplatsPerBlock / (64 * kQWaves);
template <bool PACK, bool CLEAN>
__global__ __launch_bounds__(64 * kQWaves) void k_preprocess_q(PreParams P, SceneDev sc, FrameDev fr) {
    __shared__ uint32_t s_sum[kQWaves];
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    const int base = blockIdx.x * kSplatsPerBlock + wid * (kQItems * 64);
    uint32_t n_main = 0, n_dup = 0;
    // queue: entries [0, qn) in lanes of qa (the first 64) and qb (the overflow)
    int qa_i = 0, qb_i = 0;
    float qa0 = 0.0f, qa1 = 0.0f, qa2 = 0.0f, qb0 = 0.0f, qb1 = 0.0f, qb2 = 0.0f;
    int qn = 0;
    // the pending chunk: lanes [0, pend_n) hold a survivor and its loaded planes
    int pend_n = 0, pi = 0;
    float pp0 = 0.0f, pp1 = 0.0f, pp2 = 0.0f, pmx = 0.0f, pmy = 0.0f, pmz = 0.0f;
    float pc0 = 0.0f, pc1 = 0.0f, pc2 = 0.0f, pc3 = 0.0f, pc4 = 0.0f, pc5 = 0.0f, pop = 0.0f;
    auto write_rec = [&](int i, const int4 &rc) {
        if (PACK)
            reinterpret_cast<uint2 *>(fr.rec)[i] = make_uint2((uint32_t)rc.x, rc.y >= 0 ? pack_rec(rc.y, rc.z, (uint32_t)rc.w) : 0u);
        else
            fr.rec[i] = rc;
    };
    // the next projection step's means, loaded one step ahead
    float nmx = 0.0f, nmy = 0.0f, nmz = 0.0f;
    if (base + lane < P.n) nmx = sc.mx[base + lane], nmy = sc.my[base + lane], nmz = sc.mz[base + lane];
#pragma unroll 1
    for (int it = 0; it <= kQItems + 1; ++it) {
        if (it < kQItems) {  // projection step
            const int i = base + it * 64 + lane;
            const bool valid = i < P.n;
            const float mx = nmx, my = nmy, mz = nmz;
            if (it + 1 < kQItems && i + 64 < P.n) nmx = sc.mx[i + 64], nmy = sc.my[i + 64], nmz = sc.mz[i + 64];
            float p0 = 0.0f, p1 = 0.0f, p2 = 0.0f;
            bool vis = false;
            if (valid) {
                vis = project_ndc(P, mx, my, mz, p0, p1, p2);
                if (!vis) {
                    write_rec(i, make_int4(0, -1, -1, 0));
                    if (i == 0) write_culled_splat0(fr);
                }
            }
            const uint64_t m = __ballot(vis);
            const int cnt = __popcll(m);
            if (cnt) {
                // survivors to queue lanes qn, qn+1, ... (mod 64), the others after them
                const int r_in = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                const int dst = (vis ? qn + r_in : qn + cnt + (lane - r_in)) & 63;
                const int addr = dst << 2;
                const int gi = __builtin_amdgcn_ds_permute(addr, i);
                const float g0 = __int_as_float(__builtin_amdgcn_ds_permute(addr, __float_as_int(p0)));
                const float g1 = __int_as_float(__builtin_amdgcn_ds_permute(addr, __float_as_int(p1)));
                const float g2 = __int_as_float(__builtin_amdgcn_ds_permute(addr, __float_as_int(p2)));
                const bool fresh = ((lane - qn) & 63) < cnt;
                if (fresh && lane >= qn) {
                    qa_i = gi, qa0 = g0, qa1 = g1, qa2 = g2;
                } else if (fresh) {
                    qb_i = gi, qb0 = g0, qb1 = g1, qb2 = g2;
                }
                qn += cnt;
            }
        }
        if (pend_n > 0) {  // the pending chunk, its planes loaded one step ago
            if (lane < pend_n) {
                const int4 rc = preprocess_rest<CLEAN, false>(P, sc, fr, pi, pmx, pmy, pmz, pp0, pp1, pp2, true, pc0, pc1, pc2, pc3,
                                                       pc4, pc5, pop);
                write_rec(pi, rc);
                n_main += rc.y >= 0 ? 1u : 0u;
                n_dup += rec_dups(rc);
            }
            pend_n = 0;
        }
        if (qn >= 64 || (it == kQItems && qn > 0)) {  // a full queue (or the rest) becomes pending
            pend_n = qn < 64 ? qn : 64;
            pi = qa_i, pp0 = qa0, pp1 = qa1, pp2 = qa2;
            if (lane < pend_n) {
                pmx = sc.mx[pi], pmy = sc.my[pi], pmz = sc.mz[pi];
                load_shape(sc, (size_t)pi, pc0, pc1, pc2, pc3, pc4, pc5, pop);
            }
            qa_i = qb_i, qa0 = qb0, qa1 = qb1, qa2 = qb2;
            qn -= pend_n;
        }
    }
    // block sums of (main, dup): mains in the low 11 bits (<= 1024), duplicates above (see k_preprocess)
    uint32_t v = n_main | (n_dup << 11);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) s_sum[wid] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int w = 0; w < kQWaves; ++w) t += s_sum[w];
        fr.blocksum[blockIdx.x] = make_uint2(t & 0x7ffu, t >> 11);
    }
}

// exclusive scan of the per-block (main, dup) sums; totals -> fr.totals[0..1].
// One workgroup of 256 (a small workgroup finds room on a CU beside the previous frame's blend,
// which occupies most wave slots while this runs; 1024 threads waited ~50 us for one CU to
// drain); each thread owns 24 consecutive sums per round (independent loads issued together):
// one round covers 6144 block sums = 6.3M splats.
constexpr int kScanThreads = 256, kScanPer = 24;
// one array of (a, b) block sums -> exclusive offsets; returns the totals (thread 0)
__device__ __forceinline__ uint2 scan_pairs(uint2 *bs, int nblocks, uint32_t *s_w0, uint32_t *s_w1, uint32_t *s_carry) {
    constexpr int W = kScanThreads / 64;
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_carry[0] = s_carry[1] = 0;
    __syncthreads();
    for (int base = 0; base < nblocks; base += kScanThreads * kScanPer) {
        const int i0 = base + threadIdx.x * kScanPer;
        uint2 v[kScanPer];
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) v[k] = (i0 + k < nblocks) ? bs[i0 + k] : make_uint2(0, 0);
        uint32_t a0 = 0, a1 = 0;
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            a0 += v[k].x;
            a1 += v[k].y;
        }
        const uint32_t c0 = wave_incl_scan(a0), c1 = wave_incl_scan(a1);
        if (lane == 63) {
            s_w0[wid] = c0;
            s_w1[wid] = c1;
        }
        __syncthreads();
        uint32_t o0 = s_carry[0], o1 = s_carry[1], t0 = 0, t1 = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            o0 += (w < wid) ? s_w0[w] : 0u;
            o1 += (w < wid) ? s_w1[w] : 0u;
            t0 += s_w0[w];
            t1 += s_w1[w];
        }
        o0 += c0 - a0;
        o1 += c1 - a1;
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            if (i0 + k < nblocks) bs[i0 + k] = make_uint2(o0, o1);
            o0 += v[k].x;
            o1 += v[k].y;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            s_carry[0] += t0;
            s_carry[1] += t1;
        }
        __syncthreads();
    }
    return make_uint2(s_carry[0], s_carry[1]);
}

// exclusive scan of the per-block (main, dup) sums; totals -> fr.totals[0..1] (KEPT: also the
// kept entries' sums, totals -> fr.totals[2..3]).
// One workgroup of 256 (a small workgroup finds room on a CU beside the previous frame's blend,
// which occupies most wave slots while this runs; 1024 threads waited ~50 us for one CU to
// drain); each thread owns 24 consecutive sums per round (independent loads issued together):
// one round covers 6144 block sums = 6.3M splats.
template <bool KEPT = false>
__global__ __launch_bounds__(kScanThreads) void k_scan_blocksums(FrameDev fr, int nblocks) {
    constexpr int W = kScanThreads / 64;
    __shared__ uint32_t s_w0[W], s_w1[W];
    __shared__ uint32_t s_carry[2];
    const uint2 t = scan_pairs(fr.blocksum, nblocks, s_w0, s_w1, s_carry);
    uint2 tk = make_uint2(0, 0);
    if (KEPT) tk = scan_pairs(fr.blocksum_k, nblocks, s_w0, s_w1, s_carry);
    if (threadIdx.x == 0) {
        fr.totals[0] = t.x;
        fr.totals[1] = t.y;
        if (KEPT) {
            fr.totals[2] = tk.x;
            fr.totals[3] = tk.y;
        }
        if (fr.h_totals) {  // mapped pinned host memory: the host reads it after the frame's event
            fr.h_totals[0] = t.x;
            fr.h_totals[1] = t.y;
            fr.h_totals[3] = 0;
        }
    }
}

// ---------------------------------------------------------------------- emit
// positions: mains [0,V) in splat order, duplicates [V, V+D) splat-major with the rect
// walked y-major / x-minor and the main tile skipped (preprocess.glsl:171-188).  Same
// striped kPer-per-lane layout as k_preprocess; item order (it, lane) == splat order.
// Duplicates are written cooperatively: a wave's duplicates are contiguous, lane l writes
// entries l, l+64, ... of that range (coalesced), finding the owning splat by a binary search
// over the wave's inclusive duplicate counts in LDS and decoding its place in the rect walk.
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Entries at positions >= cap are not written (a frame enqueued before its entry count is
// known on the host; the host detects the overflow from the totals and renders again).
template <bool PACK>
__global__ __launch_bounds__(kBlock) void k_emit(int n, FrameDev fr, uint32_t *__restrict__ keys,
                                                 uint32_t *__restrict__ vals, uint32_t cap,
                                                 uint32_t *__restrict__ phist) {
    // ~0.5 KB of LDS: the owners' records come by ds_bpermute and the counts are 16-bit (with
    // 5.6 KB it could not share a CU with seven waves of another frame's blend; measured
    // neutral either way, emit alone 0.0467 -> 0.0455 ms)
    __shared__ uint16_t s_incl[kBlock / 64][64];  // per wave: inclusive duplicate counts (<= 64 * 256)
    const uint2 off = fr.blocksum[blockIdx.x];
    const uint32_t V = fr.totals[0];
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    uint32_t carry_m = off.x, carry_d = off.y;
    // Wave-major: wave w emits the workgroup's splats [256 w, 256 w + 256) as four items of 64
    // consecutive splats, so one exchange of the waves' totals places every wave and each item
    // then runs on wave scans alone (no workgroup barrier per item).  Entry order is unchanged:
    // mains in splat order, duplicates splat-major.
    const int wbase = blockIdx.x * kSplatsPerBlock + wid * (kPer * 64);
    uint2 raws[kPer];
    int4 rcs[kPer];
    uint32_t ndup[kPer], incl_d[kPer];
    uint64_t hasm[kPer];
    uint32_t tot_m = 0, tot_d = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const int i = wbase + j * 64 + lane;
        raws[j] = make_uint2(0u, 0u);
        rcs[j] = make_int4(0, -1, -1, 0);
        if (PACK) {
            if (i < n) raws[j] = reinterpret_cast<const uint2 *>(fr.rec)[i];
        } else if (i < n) {
            rcs[j] = fr.rec[i];
        }
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        if (PACK) rcs[j] = unpack_rec(raws[j]);
        const int4 rc = rcs[j];
        const bool has = rc.y >= 0;
        const int minX = rc.w & 0xff, maxX = (rc.w >> 8) & 0xff, minY = (rc.w >> 16) & 0xff, maxY = (rc.w >> 24) & 0xff;
        const int rectCount = (maxX >= minX && maxY >= minY) ? (maxX - minX + 1) * (maxY - minY + 1) : 0;
        const int mainInRect = (rc.y >= minX && rc.y <= maxX && rc.z >= minY && rc.z <= maxY) ? 1 : 0;
        ndup[j] = has ? (uint32_t)(rectCount - mainInRect) : 0u;
        hasm[j] = __builtin_amdgcn_ballot_w64(has);
        incl_d[j] = wave_incl_scan(ndup[j]);
        tot_m += (uint32_t)__popcll(hasm[j]);
        tot_d += (uint32_t)__builtin_amdgcn_readlane((int)incl_d[j], 63);
    }
    // the waves' totals -> each wave's offsets within the workgroup (one exchange)
    __shared__ uint2 s_tot[kBlock / 64];
    if (lane == 0) s_tot[wid] = make_uint2(tot_m, tot_d);
    __syncthreads();
    uint32_t wm = 0, wd = 0, all_m = 0, all_d = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        const uint2 t = s_tot[w];
        wm += w < wid ? t.x : 0u;
        wd += w < wid ? t.y : 0u;
        all_m += t.x;
        all_d += t.y;
    }
    uint32_t run_m = off.x + wm, run_d = off.y + wd;
#pragma unroll 1
    for (int it = 0; it < kPer; ++it) {
        // (the item's registers selected from the arrays by the uniform counter: no scratch)
        int4 rc = rcs[0];
        uint2 raw = raws[0];
        uint32_t incl = incl_d[0];
        uint64_t hm = hasm[0];
#pragma unroll
        for (int j = 1; j < kPer; ++j)
            if (it == j) {
                rc = rcs[j];
                raw = raws[j];
                incl = incl_d[j];
                hm = hasm[j];
            }
        const int i = wbase + it * 64 + lane;
        const bool has = rc.y >= 0;
        if (has) {
            // :153-155 uint tileIndex = tileY*16 + tileX; key = tileIndex + projectedMean.z
            const uint32_t mpos = run_m + __builtin_amdgcn_mbcnt_hi((uint32_t)(hm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u));
            const uint32_t tileIndex = (uint32_t)rc.z * 16u + (uint32_t)rc.y;
            if (mpos < cap) {
                keys[mpos] = f2u((float)tileIndex + u2f((uint32_t)rc.x));
                vals[mpos] = (uint32_t)i;
            }
        }
        run_m += (uint32_t)__popcll(hm);
        const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        if (T) {  // uniform per wave: this item's duplicates [V + run_d, + T)
            s_incl[wid][lane] = (uint16_t)incl;
            wave_sync_lds();
            const uint32_t d0 = V + run_d;
            const uint32_t room = cap > d0 ? cap - d0 : 0u;  // entries of this range that fit
            uint32_t *kd = keys + d0;
            uint32_t *vd = vals + d0;
            const int ibase = wbase + it * 64;
            const uint32_t lim = min(T, room);  // entries to write
            // uniform trip count (lanes past the end compute a harmless owner, store nothing)
            for (uint32_t e0 = 0; e0 < T; e0 += 64) {
                const uint32_t e = e0 + (uint32_t)lane;
                int s = 0;  // owner: first lane with incl > e
#pragma unroll
                for (int step = 32; step > 0; step >>= 1)
                    if (s_incl[wid][s + step - 1] <= e) s += step;
                const uint32_t q = e - (s ? (uint32_t)s_incl[wid][s - 1] : 0u);  // index in the owner's walk
                // the owner's record from its lane (every lane runs this: uniform trip count)
                const int4 r = PACK ? unpack_rec(make_uint2((uint32_t)__shfl((int)raw.x, s, 64), (uint32_t)__shfl((int)raw.y, s, 64)))
                                    : make_int4(__shfl(rc.x, s, 64), __shfl(rc.y, s, 64), __shfl(rc.z, s, 64), __shfl(rc.w, s, 64));
                const int rx0 = r.w & 0xff, rx1 = (r.w >> 8) & 0xff, ry0 = (r.w >> 16) & 0xff, ry1 = (r.w >> 24) & 0xff;
                const int w = rx1 - rx0 + 1;
                // walk position, skipping the main tile if it lies in the rect
                const bool mainIn = r.y >= rx0 && r.y <= rx1 && r.z >= ry0 && r.z <= ry1;
                const uint32_t mpos_walk = (uint32_t)((r.z - ry0) * w + (r.y - rx0));
                const uint32_t k = q + ((mainIn && q >= mpos_walk) ? 1u : 0u);
                // k / w for k < 256, 1 <= w <= 16 (see below)
                const uint32_t dy = (uint32_t)(((float)k + 0.5f) * __builtin_amdgcn_rcpf((float)max(w, 1)));
                const uint32_t dx = k - dy * (uint32_t)w;
                const uint32_t tile = (uint32_t)(ry0 + (int)dy) * 16u + (uint32_t)(rx0 + (int)dx);
                if (e < lim) {
                    kd[e] = f2u((float)tile + u2f((uint32_t)r.x));
                    vd[e] = (uint32_t)(ibase + s);
                }
            }
            wave_sync_lds();  // s_incl is rewritten by the next item
        }
        run_d += T;
    }
    carry_m = off.x + all_m;
    carry_d = off.y + all_d;
    // prefix sort (gs_internal.hpp): the emitted keys at positions j * kPrefixSample of this
    // workgroup's two output ranges go to the sampled histogram (copy j % kPrefixHistCopies) --
    // after the loop, so no load of it waits behind these atomics
    if (phist) {
        __threadfence_block();
        __syncthreads();  // the workgroup's own key stores are visible to it
        const uint32_t r0[2] = {off.x, V + off.y}, r1[2] = {carry_m, V + carry_d};
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            // every sample position of the range (a workgroup's duplicate range can hold up to
            // 256 splats x 256 tiles = 65536 entries, more than one sample per thread covers)
            const uint32_t lim = min(r1[r], cap);
            for (uint32_t j = (r0[r] + kPrefixSample - 1) / kPrefixSample + threadIdx.x; j * kPrefixSample < lim;
                 j += kBlock) {
                const uint32_t p = j * kPrefixSample;
                const uint32_t key = keys[p];
                const uint32_t c = key_class(key);
                if (c < 256u)
                    atomicAdd(&phist[((size_t)(j % kPrefixHistCopies) * 256 + c) * kPrefixBuckets +
                                     prefix_slot(prefix_bucket(class_hi(c) - key))],
                              1u);
            }
        }
    }
}

// The kept emission of a prefix-sorted frame (KeptDev): k_emit's walk over every entry, in the
// same order and with the same keys, but only the entries at or below their class bound (the
// bounds an earlier frame's select chose, fr.theta_in) are written -- compacted, kept mains at
// [0, KV) in splat order, kept duplicates at [KV, KV + KD) splat-major (k_preprocess counted
// them: fr.kdup, fr.blocksum_k scanned), i.e. the emission order restricted to them, which a
// stable sort turns into the full sort restricted to them.  Over every entry it counts what the
// prefix sort's first pass counted (the tile counts, the keys above 1e6, the kept keys per
// class, the keys below 1.0) and samples one entry in kPrefixSample by full position for this
// frame's select.  The sort then runs its four passes over the kept entries alone.
template <bool PACK>
__global__ __launch_bounds__(kBlock) void k_emit_kept(int n, FrameDev fr, uint32_t *__restrict__ keys,
                                                      uint32_t *__restrict__ vals, uint32_t cap, KeptDev kd) {
    constexpr int kR = 4;  // counter replicas (lane % 4)
    __shared__ uint16_t s_incl[kBlock / 64][64];
    __shared__ uint32_t s_theta[kClasses];
    __shared__ uint32_t s_tiles[256 * kR];
    __shared__ uint32_t s_kept[kClasses * kR];
    __shared__ uint32_t s_above, s_low;
    __shared__ uint4 s_tot[kBlock / 64];
    for (int c = threadIdx.x; c < kClasses; c += kBlock) s_theta[c] = fr.theta_in[c];
    for (int c = threadIdx.x; c < 256 * kR; c += kBlock) s_tiles[c] = 0;
    for (int c = threadIdx.x; c < kClasses * kR; c += kBlock) s_kept[c] = 0;
    if (threadIdx.x == 0) s_above = s_low = 0;
    __syncthreads();  // s_theta (the kept ballots below read it) and the zeroed counters
    const uint2 off = fr.blocksum[blockIdx.x], koff = fr.blocksum_k[blockIdx.x];
    const uint32_t V = fr.totals[0], KV = fr.totals[2];
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    const uint32_t rep = (uint32_t)lane & (kR - 1);
    const int wbase = blockIdx.x * kSplatsPerBlock + wid * (kPer * 64);
    uint2 raws[kPer];
    int4 rcs[kPer];
    uint32_t incl_d[kPer];
    uint64_t hasm[kPer];
    uint32_t tot_m = 0, tot_d = 0, tot_kd = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const int i = wbase + j * 64 + lane;
        raws[j] = make_uint2(0u, 0u);
        rcs[j] = make_int4(0, -1, -1, 0);
        if (PACK) {
            if (i < n) raws[j] = reinterpret_cast<const uint2 *>(fr.rec)[i];
        } else if (i < n) {
            rcs[j] = fr.rec[i];
        }
    }
    uint32_t kdj[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const int i = wbase + j * 64 + lane;
        if (PACK) rcs[j] = unpack_rec(raws[j]);
        kdj[j] = (i < n && rcs[j].y >= 0) ? (uint32_t)fr.kdup[i] : 0u;
    }
    uint64_t kmm[kPer];  // kept mains
    uint32_t mkey[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const int4 rc = rcs[j];
        const bool has = rc.y >= 0;
        mkey[j] = f2u((float)((uint32_t)rc.z * 16u + (uint32_t)rc.y) + u2f((uint32_t)rc.x));
        hasm[j] = __builtin_amdgcn_ballot_w64(has);
        kmm[j] = __builtin_amdgcn_ballot_w64(has && mkey[j] <= s_theta[key_class(mkey[j])]);
        incl_d[j] = wave_incl_scan(rec_dups(rc));
        tot_m += (uint32_t)__popcll(hasm[j]);
        tot_d += (uint32_t)__builtin_amdgcn_readlane((int)incl_d[j], 63);
        tot_kd += wave_sum(kdj[j]);
    }
    uint32_t tot_km = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) tot_km += (uint32_t)__popcll(kmm[j]);
    if (lane == 0) s_tot[wid] = make_uint4(tot_m, tot_d, tot_km, tot_kd);
    __syncthreads();
    uint32_t wm = 0, wd = 0, wkm = 0, wkd = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        const uint4 t = s_tot[w];
        wm += w < wid ? t.x : 0u;
        wd += w < wid ? t.y : 0u;
        wkm += w < wid ? t.z : 0u;
        wkd += w < wid ? t.w : 0u;
    }
    uint32_t run_m = off.x + wm, run_d = off.y + wd, run_km = koff.x + wkm, run_kd = koff.y + wkd;
    uint32_t above = 0, low = 0;
    // one entry of the walk: its counts, its sample (full position p), its kept store (kpos)
    auto count = [&](uint32_t key, bool valid, bool kept) {
        if (!valid) return;
        const int t = f2i(u2f(key));
        if ((uint32_t)t < 256u) atomicAdd(&s_tiles[(uint32_t)t * kR + rep], 1u);  // countBins.glsl's int(key)
        above += key > kKeyCulledBits ? 1u : 0u;
        low += key < kKey1Bits ? 1u : 0u;
        if (kept) atomicAdd(&s_kept[key_class(key) * kR + rep], 1u);
    };
    auto sample = [&](uint32_t key, uint32_t p) {
        const uint32_t c = key_class(key);
        if ((p % kPrefixSample) == 0 && c < 256u && kd.phist)
            atomicAdd(&kd.phist[((size_t)((p / kPrefixSample) % kPrefixHistCopies) * 256 + c) * kPrefixBuckets +
                                prefix_slot(prefix_bucket(class_hi(c) - key))],
                      1u);
    };
#pragma unroll 1
    for (int it = 0; it < kPer; ++it) {
        int4 rc = rcs[0];
        uint2 raw = raws[0];
        uint32_t incl = incl_d[0], key = mkey[0];
        uint64_t hm = hasm[0], km = kmm[0];
#pragma unroll
        for (int j = 1; j < kPer; ++j)
            if (it == j) {
                rc = rcs[j];
                raw = raws[j];
                incl = incl_d[j];
                key = mkey[j];
                hm = hasm[j];
                km = kmm[j];
            }
        const int i = wbase + it * 64 + lane;
        const bool has = rc.y >= 0;
        {  // :153-155 the main entry
            const bool kept = ((km >> lane) & 1ull) != 0;
            count(key, has, kept);
            if (has) sample(key, run_m + __builtin_amdgcn_mbcnt_hi((uint32_t)(hm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u)));
            const uint32_t kpos = run_km + __builtin_amdgcn_mbcnt_hi((uint32_t)(km >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)km, 0u));
            if (kept && kpos < cap) {
                keys[kpos] = key;
                vals[kpos] = (uint32_t)i;
            }
        }
        run_m += (uint32_t)__popcll(hm);
        run_km += (uint32_t)__popcll(km);
        const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        if (T) {  // uniform per wave: this item's duplicates [V + run_d, + T)
            s_incl[wid][lane] = (uint16_t)incl;
            wave_sync_lds();
            const int ibase = wbase + it * 64;
            for (uint32_t e0 = 0; e0 < T; e0 += 64) {
                const uint32_t e = e0 + (uint32_t)lane;
                int s = 0;  // owner: first lane with incl > e
#pragma unroll
                for (int step = 32; step > 0; step >>= 1)
                    if (s_incl[wid][s + step - 1] <= e) s += step;
                const uint32_t q = e - (s ? (uint32_t)s_incl[wid][s - 1] : 0u);
                const int4 r = PACK ? unpack_rec(make_uint2((uint32_t)__shfl((int)raw.x, s, 64), (uint32_t)__shfl((int)raw.y, s, 64)))
                                    : make_int4(__shfl(rc.x, s, 64), __shfl(rc.y, s, 64), __shfl(rc.z, s, 64), __shfl(rc.w, s, 64));
                const int rx0 = r.w & 0xff, rx1 = (r.w >> 8) & 0xff, ry0 = (r.w >> 16) & 0xff, ry1 = (r.w >> 24) & 0xff;
                const int w = rx1 - rx0 + 1;
                const bool mainIn = r.y >= rx0 && r.y <= rx1 && r.z >= ry0 && r.z <= ry1;
                const uint32_t mpos_walk = (uint32_t)((r.z - ry0) * w + (r.y - rx0));
                const uint32_t k = q + ((mainIn && q >= mpos_walk) ? 1u : 0u);
                const uint32_t dy = (uint32_t)(((float)k + 0.5f) * __builtin_amdgcn_rcpf((float)max(w, 1)));
                const uint32_t dx = k - dy * (uint32_t)w;
                const uint32_t tile = (uint32_t)(ry0 + (int)dy) * 16u + (uint32_t)(rx0 + (int)dx);
                const uint32_t dkey = f2u((float)tile + u2f((uint32_t)r.x));
                const bool valid = e < T;
                const bool kept = valid && dkey <= s_theta[key_class(dkey)];
                const uint64_t kb = __builtin_amdgcn_ballot_w64(kept);
                count(dkey, valid, kept);
                if (valid) sample(dkey, V + run_d + e);
                const uint32_t kpos = KV + run_kd + __builtin_amdgcn_mbcnt_hi((uint32_t)(kb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)kb, 0u));
                if (kept && kpos < cap) {
                    keys[kpos] = dkey;
                    vals[kpos] = (uint32_t)(ibase + s);
                }
                run_kd += (uint32_t)__popcll(kb);
            }
            wave_sync_lds();  // s_incl is rewritten by the next item
        }
        run_d += T;
    }
    above = wave_sum(above);
    low = wave_sum(low);
    if (lane == 0) {
        if (above) atomicAdd(&s_above, above);
        if (low) atomicAdd(&s_low, low);
    }
    __syncthreads();
    // the workgroup's counts into the copies picked by its id (spread same-address atomics)
    const uint32_t cp = blockIdx.x % kTileCopyCount;
    for (int t = threadIdx.x; t < 256; t += kBlock) {
        const uint32_t c = s_tiles[t * kR] + s_tiles[t * kR + 1] + s_tiles[t * kR + 2] + s_tiles[t * kR + 3];
        if (c) atomicAdd(&kd.tile_counts[cp * 256 + t], c);
    }
    uint32_t *pc = kd.counts + (blockIdx.x % kPrefixCopies) * kClasses;
    for (int c = threadIdx.x; c < kClasses; c += kBlock) {
        const uint32_t v = s_kept[c * kR] + s_kept[c * kR + 1] + s_kept[c * kR + 2] + s_kept[c * kR + 3];
        if (v) atomicAdd(&pc[c], v);
    }
    if (threadIdx.x == 0) {
        if (s_above) atomicAdd(&kd.tile_counts[kTileCopyCount * 256 + cp], s_above);
        if (s_low) atomicAdd(&kd.counts[kPrefixCopies * kClasses + (blockIdx.x % kPrefixCopies)], s_low);
    }
}

// ------------------------------------------------ fused preprocess + emission (frame path)
// k_pre_emit: one pass over the splats for a frame enqueued without a host round trip.  Each
// workgroup preprocesses its 1024 splats (wave w: splats [256 w, 256 w + 256) as four items of
// 64), keeps their emission records in registers, learns its entry offsets by a decoupled
// look-back over the workgroups before it (single-pass scan: a workgroup publishes its (main,
// dup) counts, then their inclusive prefix), and emits its entries.  This removes the 8-byte
// emission record written and read back (98 MB per C3 frame), the block-sum scan launch and the
// separate emission pass of k_preprocess -> k_scan_blocksums -> k_emit.
// Entry layout ("split"): mains at [0, V) in splat order as before, duplicates at [dup_base,
// dup_base + D) splat-major -- a workgroup cannot know V (the mains of the workgroups after it)
// when it emits, so the duplicates start at dup_base = n >= V.  The sort's first pass reads the
// two ranges as one array of V + D entries (the same order as the contiguous layout), so the
// sorted result is unchanged.
// Forward progress: a workgroup waits only on workgroups with lower ids, which publish their
// counts right after their own preprocessing.  The hardware dispatches a grid in id order (per
// XCD, round-robin over them), so they are running or done; HIP does not promise that order
// (MI355X_MICROARCH.md, "Workgroup dispatch"), so a wait is bounded: after kLbSpinLimit polls
// (~tens of ms) it gives up, the workgroup goes on with what it has (every store stays inside the
// entry capacity) and flags the frame (ring word 4), which the host renders again on the
// host-synchronous path.  Nothing depends on the order for correctness.  (A ticket counter
// instead of the workgroup id serialised every workgroup's start on one address: ~33 ns each,
// 0.2 ms for the 6000 workgroups of C3.)
constexpr uint64_t kLbAgg = 1ull << 62, kLbInc = 2ull << 62;
__device__ __forceinline__ uint64_t lb_word(uint64_t flag, uint32_t m, uint32_t d) {
    return flag | ((uint64_t)(d & 0x7fffffffu) << 31) | (uint64_t)(m & 0x7fffffffu);
}
__device__ __forceinline__ uint64_t lb_load(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// KP items of 64 splats per wave (KP * 256 splats per workgroup): 1 for the small scenes it runs
// on (one memory round trip per splat, four times the workgroups of k_preprocess)
template <bool PACK, bool CLEAN, bool LAZY, int KP>
__global__ __launch_bounds__(kBlock) void k_pre_emit(PreParams P, SceneDev sc, FrameDev fr, LookbackDev lb,
                                                     uint32_t *__restrict__ keys, uint32_t *__restrict__ vals,
                                                     uint32_t cap, uint32_t dup_base, uint32_t *__restrict__ phist,
                                                     uint32_t nblocks) {
    // the workgroup's emission records and per-item inclusive duplicate counts stay in LDS between
    // the preprocessing and the emission (in registers they held the kernel to 5 waves per SIMD)
    using Rec = typename std::conditional<PACK, uint2, int4>::type;
    __shared__ Rec s_rec[KP * kBlock];
    __shared__ uint16_t s_incl[kBlock / 64][KP][64];  // (<= 64 * 256 per item)
    __shared__ uint2 s_tot[kBlock / 64];
    __shared__ uint2 s_off;
    const uint32_t blk = blockIdx.x;
    // the next frame of this lane uses the other half: clear it (its previous user, this lane's
    // frame before, is complete)
    for (uint32_t j = blk * kBlock + threadIdx.x; j < lb.cap_blocks; j += nblocks * kBlock) lb.st_next[j] = 0ull;
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    const int wbase = (int)blk * (KP * kBlock) + wid * (KP * 64);
    Rec *wrec = s_rec + wid * (KP * 64);
    uint32_t tot_m = 0, tot_d = 0;
#pragma unroll 1
    for (int j = 0; j < KP; ++j) {
        const int i = wbase + j * 64 + lane;
        const int4 rc = preprocess_one<CLEAN, LAZY>(P, sc, fr, i, i < P.n);
        if constexpr (PACK)
            wrec[j * 64 + lane] = make_uint2((uint32_t)rc.x, rc.y >= 0 ? pack_rec(rc.y, rc.z, (uint32_t)rc.w) : 0u);
        else
            wrec[j * 64 + lane] = rc;
        const uint32_t incl = wave_incl_scan(rec_dups(rc));
        s_incl[wid][j][lane] = (uint16_t)incl;
        tot_m += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(rc.y >= 0));
        tot_d += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    }
    if (lane == 0) s_tot[wid] = make_uint2(tot_m, tot_d);
    __syncthreads();
    uint32_t wm = 0, wd = 0, all_m = 0, all_d = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        const uint2 t = s_tot[w];
        wm += w < wid ? t.x : 0u;
        wd += w < wid ? t.y : 0u;
        all_m += t.x;
        all_d += t.y;
    }
    if (wid == 0) {  // the look-back (one wave): this workgroup's exclusive (mains, dups) offsets
        uint32_t exm = 0, exd = 0;
        bool fail = false;
        if (blk == 0) {
            if (lane == 0) lb_store(&lb.st[0], lb_word(kLbInc, all_m, all_d));
        } else {
            if (lane == 0) lb_store(&lb.st[blk], lb_word(kLbAgg, all_m, all_d));
            fail = lb.spin_limit == 0;  // (test hook: give up at once)
            int j = fail ? -1 : (int)blk - 1;  // the window's nearest predecessor
            uint32_t spins = 0;
            while (j >= 0) {  // uniform
                const int idx = j - lane;
                const uint64_t w = idx >= 0 ? lb_load(&lb.st[idx]) : kLbInc;  // before workgroup 0: zero
                const uint32_t flag = (uint32_t)(w >> 62);
                const uint64_t inc = __builtin_amdgcn_ballot_w64(flag == 2u);
                const uint64_t notready = __builtin_amdgcn_ballot_w64(flag == 0u);
                const int fp = inc ? __builtin_ctzll(inc) : 63;  // lanes 0..fp are needed
                const uint64_t need = fp == 63 ? ~0ull : ((2ull << fp) - 1ull);
                if (notready & need) {
                    if (++spins > lb.spin_limit) {
                        fail = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                exm += wave_sum(lane <= fp ? (uint32_t)w & 0x7fffffffu : 0u);
                exd += wave_sum(lane <= fp ? (uint32_t)(w >> 31) & 0x7fffffffu : 0u);
                if (inc) break;
                j -= 64;
            }
            if (lane == 0) lb_store(&lb.st[blk], lb_word(kLbInc, exm + all_m, exd + all_d));
        }
        if (lane == 0) {
            s_off = make_uint2(exm, exd);
            // (never expected) the frame is rendered again.  Word 2 is cleared by the host when the
            // slot is taken, and nothing on the device writes 0 to it during the frame: a plain
            // store of a nonzero flag (k_draw's prefix miss writes 1) cannot be lost
            if (fail && fr.h_totals) fr.h_totals[4] = 1u;
            if (blk == nblocks - 1) {  // the last workgroup: the frame's (V, D)
                // the device count holds the duplicates emitted (below cap: a frame that did not fit
                // is detected by the host from the pinned count, and rendered again), so every
                // entry the sort and the blend read was written
                fr.totals[0] = exm + all_m;
                fr.totals[1] = min(exd + all_d, cap > dup_base ? cap - dup_base : 0u);
                if (fr.h_totals) {  // mapped pinned host memory: the host reads it after the frame's event
                    fr.h_totals[0] = exm + all_m;
                    fr.h_totals[1] = exd + all_d;
                    fr.h_totals[3] = 0;
                }
            }
        }
    }
    __syncthreads();
    uint32_t run_m = s_off.x + wm, run_d = s_off.y + wd;
    // the emission (k_emit's, from the records in LDS; duplicates at dup_base)
#pragma unroll 1
    for (int it = 0; it < KP; ++it) {
        const Rec raw = wrec[it * 64 + lane];
        int4 rc;
        if constexpr (PACK) rc = unpack_rec(raw);
        else rc = raw;
        const uint64_t hm = __builtin_amdgcn_ballot_w64(rc.y >= 0);
        const int i = wbase + it * 64 + lane;
        if (rc.y >= 0) {
            // :153-155 uint tileIndex = tileY*16 + tileX; key = tileIndex + projectedMean.z
            const uint32_t mpos = run_m + __builtin_amdgcn_mbcnt_hi((uint32_t)(hm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u));
            const uint32_t key = f2u((float)((uint32_t)rc.z * 16u + (uint32_t)rc.y) + u2f((uint32_t)rc.x));
            if (mpos < cap) {
                keys[mpos] = key;
                vals[mpos] = (uint32_t)i;
            }
            // prefix sort: one main in kPrefixSample (by position) into the sampled histogram
            if (phist && (mpos % kPrefixSample) == 0 && key_class(key) < 256u) {
                const uint32_t c = key_class(key);
                atomicAdd(&phist[((size_t)((mpos / kPrefixSample) % kPrefixHistCopies) * 256 + c) * kPrefixBuckets +
                                 prefix_slot(prefix_bucket(class_hi(c) - key))],
                          1u);
            }
        }
        run_m += (uint32_t)__popcll(hm);
        const uint16_t *incl = s_incl[wid][it];
        const uint32_t T = incl[63];
        if (T) {  // uniform per wave: this item's duplicates [run_d, + T) of the duplicate range
            const int ibase = wbase + it * 64;
            for (uint32_t e0 = 0; e0 < T; e0 += 64) {
                const uint32_t e = e0 + (uint32_t)lane;
                int s = 0;  // owner: first lane with incl > e
#pragma unroll
                for (int step = 32; step > 0; step >>= 1)
                    if (incl[s + step - 1] <= e) s += step;
                const uint32_t q = e - (s ? (uint32_t)incl[s - 1] : 0u);  // index in the owner's walk
                int4 r;
                if constexpr (PACK) r = unpack_rec(wrec[it * 64 + s]);
                else r = wrec[it * 64 + s];
                const int rx0 = r.w & 0xff, rx1 = (r.w >> 8) & 0xff, ry0 = (r.w >> 16) & 0xff, ry1 = (r.w >> 24) & 0xff;
                const int w = rx1 - rx0 + 1;
                // walk position, skipping the main tile if it lies in the rect
                const bool mainIn = r.y >= rx0 && r.y <= rx1 && r.z >= ry0 && r.z <= ry1;
                const uint32_t mpos_walk = (uint32_t)((r.z - ry0) * w + (r.y - rx0));
                const uint32_t k = q + ((mainIn && q >= mpos_walk) ? 1u : 0u);
                // k / w for k < 256, 1 <= w <= 16 (k_emit)
                const uint32_t dy = (uint32_t)(((float)k + 0.5f) * __builtin_amdgcn_rcpf((float)max(w, 1)));
                const uint32_t dx = k - dy * (uint32_t)w;
                const uint32_t tile = (uint32_t)(ry0 + (int)dy) * 16u + (uint32_t)(rx0 + (int)dx);
                const uint32_t key = f2u((float)tile + u2f((uint32_t)r.x));
                const uint32_t dd = run_d + e;  // place in the duplicate range
                if (e < T && dup_base + dd < cap) {
                    keys[dup_base + dd] = key;
                    vals[dup_base + dd] = (uint32_t)(ibase + s);
                }
                if (phist && e < T && (dd % kPrefixSample) == 0 && key_class(key) < 256u) {
                    const uint32_t c = key_class(key);
                    atomicAdd(&phist[((size_t)((dd / kPrefixSample) % kPrefixHistCopies) * 256 + c) * kPrefixBuckets +
                                     prefix_slot(prefix_bucket(class_hi(c) - key))],
                              1u);
                }
            }
        }
        run_d += T;
    }
}

// ---------------------------------------------------------------------- bins
// countBins.glsl: bins[int(key)]++ for int(key) in [0,256).  Keys are already sorted, so
// each thread run-length counts 16 consecutive keys and flushes a run to LDS on change.
constexpr int kBinItems = 16;
__global__ __launch_bounds__(kBlock) void k_bins_count(const uint32_t *__restrict__ keys, int64_t E_max,
                                                       const uint32_t *__restrict__ cnt,
                                                       uint32_t *__restrict__ counts) {
    const int64_t E = cnt ? min(E_max, (int64_t)cnt[0] + (int64_t)cnt[1]) : E_max;
    __shared__ uint32_t s_cnt[256];
    __shared__ uint32_t s_above;
    s_cnt[threadIdx.x] = 0;
    if (threadIdx.x == 0) s_above = 0;
    __syncthreads();
    const int64_t base = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * kBinItems;
    int cur = -1;
    uint32_t run = 0, above = 0;
    if (base < E) {
        uint32_t kk[kBinItems];
        if (base + kBinItems <= E) {
            const uint4 *p = reinterpret_cast<const uint4 *>(keys + base);
#pragma unroll
            for (int q = 0; q < kBinItems / 4; ++q) {
                const uint4 v = p[q];
                kk[4 * q + 0] = v.x;
                kk[4 * q + 1] = v.y;
                kk[4 * q + 2] = v.z;
                kk[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int q = 0; q < kBinItems; ++q) kk[q] = (base + q < E) ? keys[base + q] : 0x7f800000u;  // +inf
        }
#pragma unroll
        for (int q = 0; q < kBinItems; ++q) {
            above += (kk[q] > kKeyCulledBits && base + q < E) ? 1u : 0u;
            const int v = f2i(u2f(kk[q]));
            if (v < 0 || v >= 256) continue;
            if (v == cur) {
                ++run;
            } else {
                if (run) atomicAdd(&s_cnt[cur], run);
                cur = v;
                run = 1;
            }
        }
        if (run) atomicAdd(&s_cnt[cur], run);
        if (above) atomicAdd(&s_above, above);
    }
    __syncthreads();
    const uint32_t c = s_cnt[threadIdx.x];
    if (c) atomicAdd(&counts[threadIdx.x], c);
    if (threadIdx.x == 0 && s_above) atomicAdd(&counts[256], s_above);
}

// prefixBins.glsl: inclusive scan of the 256 counts
// inclusive scan of the tile counts -> bins[0..255] (prefixBins.glsl), counts re-zeroed; also the draw's
// dispatch order bins[256..511]: tiles by list length, longest first (ties by index), so the
// longest-running sub-blocks start first and the blend's tail is short (speed only)
__global__ __launch_bounds__(kBlock) void k_bins_scan(uint32_t *__restrict__ counts, uint32_t *__restrict__ bins) {
    __shared__ uint32_t s_wave[kBlock / 64];
    __shared__ uint32_t s_cnt[256];
    const uint32_t v = counts[threadIdx.x];
    counts[threadIdx.x] = 0;  // ready for the next frame's k_bins_count (no memset launch)
    s_cnt[threadIdx.x] = v;
    if (threadIdx.x == 0) {  // keys above 1e6 (bits): where the reference's culled entries sit (k_draw)
        bins[512] = counts[256];
        counts[256] = 0;
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan256(v, s_wave, &tot);  // (contains __syncthreads)
    bins[threadIdx.x] = ex + v;
    uint32_t rank = 0;
#pragma unroll 32
    for (int u = 0; u < 256; ++u) {
        const uint32_t c = s_cnt[u];
        rank += (c > v || (c == v && u < (int)threadIdx.x)) ? 1u : 0u;
    }
    bins[256 + rank] = threadIdx.x;
}

// ---------------------------------------------------------------------- draw
// One wave (64-thread workgroup) per 16x16 pixel sub-block of a coarse tile; lane l owns
// the 2x2 pixel quad at (2*(l%8), 2*(l/8)).  Sub-blocks never straddle coarse tiles, so
// each pixel blends exactly its own tile's list (Q18 resolved).
//
// The tile's sorted list is consumed 64 entries per step through a three-stage register
// pipeline (index load, box gather, box test; see k_draw); the box survivors queue in LDS in
// list order, and batches of up to 64 are gathered one survivor per lane, culled exactly and
// blended while the next chunks' loads are in flight.  A batch's survivors stay in the
// registers of the lanes that gathered them and are broadcast with v_readlane while the wave
// walks the batch mask in ascending lane order -- exactly list order.  Per survivor, every lane
// evaluates power for its four pixels; the pixels that can blend become (pixel, power) events,
// compacted and processed one per lane on the pixel state kept in LDS (a pixel occurs at most
// once per survivor, so events never conflict, and each pixel still sees its survivors in list
// order).  Each pixel's arithmetic is the same sequence of IEEE ops as draw.glsl / the oracle,
// and the filters only drop work draw.glsl would `continue` past (draw.glsl:118-126):
//   * box cull: the entry's alpha >= 1/255 box misses the sub-block;
//   * exact cull: the alpha >= 1/255 ellipse misses the sub-block (ellipse_misses_rect);
//   * pre-exp skip: power < ln(1/(255*o)) - 1e-3 implies alpha < 1/255 for any exp
//     within a few ulp.
// Block placement (speed only; any placement gives the same pixels): workgroups are dealt
// round-robin over the 8 XCDs, so linear block id L runs on XCD L % 8.  Tiles are taken in
// k_bins_scan's longest-list-first order and the tile of rank r goes to XCD r % 8, its
// sub-blocks consecutively: each tile's list is gathered through one L2, and the longest
// sub-blocks start first.

__device__ __forceinline__ uint32_t pack_rgba8(const float4 &c) {
    // :141-142 imageStore(rgba8, col / 255): unorm, round to nearest
    const float vv[4] = {c.x / 255.0f, c.y / 255.0f, c.z / 255.0f, c.w / 255.0f};
    uint32_t packed = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float q = vv[k];
        q = (q != q) ? 0.0f : q;
        q = q < 0.0f ? 0.0f : (q > 1.0f ? 1.0f : q);
        packed |= ((uint32_t)floorf(q * 255.0f + 0.5f)) << (8 * k);
    }
    return packed;
}

// Exact block cull for a survivor of the box test.  Pixels of the sub-block need the splat
// only where the computed power >= thr, i.e. q = a dx^2 + 2b dx dy + c dy^2 <= -2*thr.  The
// minimum of the convex quadratic q over the continuous rectangle [x0,x1]x[y0,y1] (a lower
// bound over its integer pixels) is 0 if the centre is inside, else it lies on an edge:
// minimise the 1-D quadratic along each edge (clamped).  The splat is dropped only when that
// minimum exceeds the threshold by margins far above the rounding of power (relative error
// <= ~6 eps * cond; conics with cond >= 1e4 are never dropped here).
// Branch-free (every lane evaluates every term; the tests select): early returns here became
// nested exec-mask branches costing more scalar instructions than the arithmetic they skipped.
__device__ __forceinline__ bool ellipse_misses_rect(float mx, float my, float a, float b, float c, float thr,
                                                    float x0, float x1, float y0, float y1) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const float lim = -2.0f * thr;  // pixels with q <= lim may blend
    const float det = a * c - b * b, tr = a + c;
    // well conditioned (else never dropped)
    const bool ok = (a > 0.0f) & (c > 0.0f) & (det > 0.0f) & (tr * tr < 1.0e4f * det);
    const f2 X = f2{x0, x1} - f2{mx, mx}, Y = f2{y0, y1} - f2{my, my};
    const bool inside = (X.x <= 0.0f) & (X.y >= 0.0f) & (Y.x <= 0.0f) & (Y.y >= 0.0f);  // centre inside: keep
    // edge minimisers via v_rcp (1 ulp): a minimiser off by delta raises q by O(delta^2),
    // orders of magnitude inside the margins below; both edges of a pair in packed fp32
    const float ra = __builtin_amdgcn_rcpf(a), rc = __builtin_amdgcn_rcpf(c);
    const f2 A = f2{a, a}, B = f2{b, b}, C = f2{c, c}, two = f2{2.0f, 2.0f};
    // edges x = X0, X1: dy* = -b dx / c clamped to [Y0, Y1]
    f2 dy = -(B * X) * f2{rc, rc};
    dy = __builtin_elementwise_min(__builtin_elementwise_max(dy, f2{Y.x, Y.x}), f2{Y.y, Y.y});
    const f2 qx = A * X * X + two * B * X * dy + C * dy * dy;
    // edges y = Y0, Y1: dx* = -b dy / a clamped to [X0, X1]
    f2 dx = -(B * Y) * f2{ra, ra};
    dx = __builtin_elementwise_min(__builtin_elementwise_max(dx, f2{X.x, X.x}), f2{X.y, X.y});
    const f2 qy = A * dx * dx + two * B * dx * Y + C * Y * Y;
    const float qmin = fminf(fminf(qx.x, qx.y), fminf(qy.x, qy.y));
    const bool far = ok & !inside & (qmin > lim * 1.002f + 1.0e-3f);  // (NaN: kept)
    // lim <= 0 or NaN: thr > 0 means no power <= 0 reaches alpha 1/255 (dropped); NaN / 0: kept
    return (lim > 0.0f) ? far : (thr > 0.0f);
}

// order this wave's LDS writes before its later LDS reads (single-wave workgroup)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float rl(float x, int src) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), src));
}

__device__ __forceinline__ uint64_t ballot(bool b) { return __builtin_amdgcn_ballot_w64(b); }

typedef float f32x2 __attribute__((ext_vector_type(2)));

// the draw's lane-held copy of a SplatDraw record (without its pad)
// (read as whole 16-byte aligned records: 28 and 12 bytes, dwordx4 + dwordx3 / dwordx3)
struct alignas(16) SurvData {
    float mx, my, a, b, c, o, thr;
};
struct alignas(8) SurvLoad {  // SplatDraw as gathered (dwordx4 + dwordx2)
    float mx, my, a, b, c, o;
};
struct alignas(16) SurvRgb {
    float x, y, z;
};
static_assert(sizeof(SurvLoad) == sizeof(SplatDraw), "SurvLoad mirrors SplatDraw");

#ifndef GS_DRAW_POWPIX
#define GS_DRAW_POWPIX 1
#endif
// blend batches whose events all have powers in [-80, 0] (GS_EV_SAFE) skip the exp's underflow
// select: the same bits (see blend_batch)
#ifndef GS_EV_SAFE
#define GS_EV_SAFE 1
#endif
// the blend's pixel states lane-major in LDS (see k_draw's qbase)
#ifndef GS_DRAW_LANEMAJOR
#define GS_DRAW_LANEMAJOR 1
#endif
// a state slot's pixel in the sub-block: lane-major slot 64 k + l holds (2 (l % 8) + k % 2,
// 2 (l / 8) + k / 2); row-major slots and the SMALL form's pixel ids are 16 y + x
template <bool SMALL>
__device__ __forceinline__ int slot_x(uint32_t s) {
    return (SMALL || !GS_DRAW_LANEMAJOR) ? (int)(s & 15u) : (int)(2u * (s & 7u) + ((s >> 6) & 1u));
}
template <bool SMALL>
__device__ __forceinline__ int slot_y(uint32_t s) {
    return (SMALL || !GS_DRAW_LANEMAJOR) ? (int)(s >> 4) : (int)(2u * ((s >> 3) & 7u) + (s >> 7));
}
#ifndef GS_DRAW_BATCH
#define GS_DRAW_BATCH 32
#endif
// 7 waves per SIMD: the LDS (5760 B per wave, events compacted by exec-masked writes) allows it
// the exact cull of a batch runs from this many box survivors on (dense / sparse phase)
#ifndef GS_CULL_DENSE
#define GS_CULL_DENSE 3
#endif
#ifndef GS_CULL_SPARSE
#define GS_CULL_SPARSE 6
#endif
#ifndef GS_DRAW_WAVES
#define GS_DRAW_WAVES 7
#endif
// SMALL: the small-frame form -- 8x8 sub-blocks, one pixel per lane with its state in registers
// from the start (the sparse phase's survivor step throughout): four times the waves of the
// 16x16 form on the same image, each walking its tile's list for 64 pixels.  Frames whose blend
// is latency-bound (a few thousand short-lived sub-blocks, C2 / the small C5 views) take it; a
// pixel's arithmetic and its survivor order are the same, so the image is the same bit for bit.
template <bool FAST_EXP, bool STATS, bool SMALL, bool SBOX>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GS_DRAW_WAVES))) void k_draw(DrawParams P, const uint32_t *__restrict__ bins,
                                             const uint32_t *__restrict__ vals,
                                             const uint2 *__restrict__ cullbox,
                                             const SplatDraw *__restrict__ sd, const float4 *__restrict__ colour,
                                             uint32_t *__restrict__ out, unsigned long long *__restrict__ stats,
                                             uint32_t *fr_h_totals) {
    // pixel state, pixel id = 16*y + x in the sub-block; a pixel is done (:129-133) iff its
    // w >= 0.99 (pixels outside the image start at w = 1)
    constexpr int SB = SMALL ? 8 : 16;  // sub-block side
    // GS_FLAG_DRAW_TRACE (P.light_trace): the STATS form records only each block's times, list steps,
    // survivors and batches -- the per-survivor counters roughly double the kernel's span
    const bool STATS_FULL = STATS && !P.light_trace;
    __shared__ float4 s_col[SMALL ? 1 : 256];
    // one survivor's blend events: power and pixel id (split); 5760 B of LDS per wave in all
    // -> 7 waves/SIMD
    __shared__ __attribute__((aligned(16))) float s_epow[SMALL ? 1 : 256];
    __shared__ uint8_t s_epix[SMALL ? 1 : 256];
    // box survivors queued in list order until a batch is blended (at most kBatch - 1 + 64 queued)
    __shared__ uint32_t s_q[GS_DRAW_BATCH + 64];
    const int nsub = P.nbx * P.nby;
    const int L = blockIdx.x;
    if (L >= kTiles * kTiles * nsub) {  // uniform: a margin block -- zero pixels outside the
        // drawn coverage (Q9: the reference dispatches (W/32)x(H/32) groups of 32x32); done here
        // instead of a memset launch
        const int rw = P.W - P.coverW, right = rw * P.coverH;
        const int total = right + (P.H - P.coverH) * P.W;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int m = (L - kTiles * kTiles * nsub) * 256 + k * 64 + (int)threadIdx.x;
            if (m >= total) break;
            int x, y;
            if (m < right) {
                y = m / rw;
                x = P.coverW + (m - y * rw);
            } else {
                const int q = m - right;
                y = P.coverH + q / P.W;
                x = q - (y - P.coverH) * P.W;
            }
            out[(size_t)y * P.W + x] = 0u;
        }
        return;
    }
    const int xcd = L & 7, kk = L >> 3;
    // coarse tile: the (xcd + 8*(kk/nsub))-th longest (bins[256..]); its rank % 8 == xcd
    const int t = (int)bins[256 + xcd + 8 * (kk / nsub)];
    const int sub = kk - (kk / nsub) * nsub;
    const int tx = t & 15, ty = t >> 4;
    const int sby = sub / P.nbx, sbx = sub - sby * P.nbx;
    const int xe = P.xb[tx + 1], ye = P.yb[ty + 1];
    const int x0 = P.xb[tx] + sbx * SB, y0 = P.yb[ty] + sby * SB;
    if (x0 >= xe || y0 >= ye) return;  // uniform: sub-block beyond this tile
    const int x1 = min(x0 + SB, xe), y1 = min(y0 + SB, ye);
    const int lane = threadIdx.x;
    const int pxa = x0 + 2 * (lane & 7), pya = y0 + 2 * (lane >> 3);
    const bool in00 = pxa < x1 && pya < y1, in10 = pxa + 1 < x1 && pya < y1;
    const bool in01 = pxa < x1 && pya + 1 < y1, in11 = pxa + 1 < x1 && pya + 1 < y1;
    const f32x2 fxx = {(float)pxa, (float)(pxa + 1)}, fyy = {(float)pya, (float)(pya + 1)};
    const float bx0 = (float)x0, bx1 = (float)(x1 - 1), by0 = (float)y0, by1 = (float)(y1 - 1);

    const int start = (t == 0) ? 0 : (int)bins[t - 1];
    int end = (int)bins[t];
    // Positions are the reference's (ref mode): its sorted range also holds one entry per culled
    // splat, key 1e6, drawn as splat 0 (preprocess.glsl:80-88, draw.glsl:97-98), after every key
    // whose bits are <= 1e6's.  They are never binned, so only a Q10 window reaches them; here
    // they are virtual: positions [cpos, cpos + cn) read splat 0, later ones entry p - cn.
    // (uniform: pinned to scalar registers -- in VGPRs they were spilled, and the reload inside
    // the list loop waited for every gather in flight)
    const int E = __builtin_amdgcn_readfirstlane(P.count ? min(P.E, (int)(P.count[0] + P.count[1])) : P.E);
    const int cn = __builtin_amdgcn_readfirstlane(P.clean ? 0 : max(0, P.n - (P.count ? (int)P.count[0] : P.V)));
    const int cpos = __builtin_amdgcn_readfirstlane(min(max(E - (int)bins[2 * kTiles * kTiles], 0), E));
    if (!P.clean && end > start) {  // Q10: the last 1024-entry chunk is blended whole
        const int chunks = (end - start + 1023) / 1024;
        end = min(E + cn, start + chunks * 1024);
    }
    // prefix-sorted frame: positions from bins[kBinsLimit + t] on were not sorted; a block that
    // gets there before saturating flags the frame (rendered again with the full sort)
    const int wend = end;
    if (P.prefix) end = min(end, (int)min(bins[kBinsLimit + t], 0x7fffffffu));
    const int qmax = max(E - 1, 0);
    // pixels outside the image count as done
    bool d00 = !in00, d10 = !in10, d01 = !in01, d11 = !in11;
#if GS_DRAW_LANEMAJOR
    // the pixel states are lane-major: the state of the lane's value k (pixel (pxa + k % 2,
    // pya + k / 2)) is slot 64 k + lane -- a value's events, taken in lane order, read and write
    // states 16 B apart (fewer LDS bank conflicts than the row-major pixel order)
    const uint32_t qbase = (uint32_t)lane;
    constexpr uint32_t kQuad[4] = {0u, 64u, 128u, 192u};
#else
    // pixel ids are row-major in the sub-block (16 * y + x): the lane's quad is qbase + kQuad[k]
    const uint32_t qbase = 32u * ((uint32_t)lane >> 3) + 2u * ((uint32_t)lane & 7u);
    constexpr uint32_t kQuad[4] = {0u, 1u, 16u, 17u};
#endif
    if constexpr (!SMALL) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool dk = k == 0 ? d00 : k == 1 ? d10 : k == 2 ? d01 : d11;
            s_col[qbase + kQuad[k]] = make_float4(0.f, 0.f, 0.f, dk ? 1.0f : 0.0f);
        }
    }
    unsigned long long st_iter = 0, st_surv = 0, st_kit = 0, st_anyneed = 0, st_pxneed = 0;
    unsigned long long st_kit64 = 0, st_kit128 = 0, st_ev64 = 0, st_refresh = 0;
    // the VALU account's counts (tools/valu_account.py): dense steps with events, extra event passes
    // of dense steps (more than 64 events), sparse steps with events
    unsigned long long st_a192 = 0, st_a128 = 0, st_a64 = 0;
    unsigned long long st_batch = 0;  // survivor batches blended (gathered, culled exactly)
    const unsigned long long st_t0 = STATS ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const bool cull = !P.no_cull;
    const int jmax = max(end - 1, 0);
    // done pixels as uniform lane masks per slot (scalar loop state; refreshed from s_col only
    // after a survivor saturated a pixel)
    uint64_t D0 = ballot(d00), D1 = ballot(d10), D2 = ballot(d01), D3 = ballot(d11);
    bool all_done = (D0 & D1 & D2 & D3) == ~0ull;
    // does a pixel of power p need the exp / blend path?  :118-126 continue on p > 0, plus the
    // pre-exp skip p < thr: p in [thr, 0] or NaN, as med3(p, thr, 0) == p or unordered (one
    // compare).  For thr > 0 (opacity < ~1/255) it admits p in [0, thr] instead, where
    // exp(p) * o <= e^-0.001 / 255 < 1/255 (thr = -ln(255 o) - 1e-3, margins far above the
    // rounding): those events never blend, as draw.glsl skips them.
    auto needs = [](float p, float thr) {
        return !__builtin_islessgreater(__builtin_amdgcn_fmed3f(p, thr, 0.0f), p);
    };
    auto below = [](uint64_t m, uint32_t base0) {  // base0 + set bits of m below this lane
        return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, base0));
    };
    // the cull rectangle: the sub-block, then the bounding box of its active pixels (a done
    // pixel never blends, so a splat missing every active pixel is skipped exactly)
    float rx0 = bx0, rx1 = bx1, ry0 = by0, ry1 = by1;
    // the same, biased as the packed box bounds (pack_box)
    uint32_t irx0 = x0 + kBoxBias, irx1 = x1 - 1 + kBoxBias, iry0 = y0 + kBoxBias, iry1 = y1 - 1 + kBoxBias;

    // Sparse phase: once at most 64 pixels are active, each lane takes one of them (its state
    // in registers for the survivors of a chunk) and a survivor costs one power / exp / blend
    // per lane and no LDS traffic.  Lanes >= nact name lane nact-1's pixel and stay inactive.
    bool sparse = false;
    uint64_t SA = 0;   // lanes whose pixel is active
    uint32_t spix = 0, nact = 0;
    float4 pc = make_float4(0.f, 0.f, 0.f, 0.f);  // the lane's pixel state in the sparse phase
    auto go_sparse = [&]() {
        wave_lds_sync();
        const uint64_t A0 = ~D0, A1 = ~D1, A2 = ~D2, A3 = ~D3;
        const uint32_t a0 = (uint32_t)__popcll(A0), a1 = (uint32_t)__popcll(A1), a2 = (uint32_t)__popcll(A2);
        nact = a0 + a1 + a2 + (uint32_t)__popcll(A3);
        if (__builtin_amdgcn_inverse_ballot_w64(A0)) s_epix[below(A0, 0)] = (uint8_t)(qbase + kQuad[0]);
        if (__builtin_amdgcn_inverse_ballot_w64(A1)) s_epix[below(A1, a0)] = (uint8_t)(qbase + kQuad[1]);
        if (__builtin_amdgcn_inverse_ballot_w64(A2)) s_epix[below(A2, a0 + a1)] = (uint8_t)(qbase + kQuad[2]);
        if (__builtin_amdgcn_inverse_ballot_w64(A3)) s_epix[below(A3, a0 + a1 + a2)] = (uint8_t)(qbase + kQuad[3]);
        wave_lds_sync();
        spix = s_epix[min((uint32_t)lane, nact - 1)];
        SA = nact >= 64 ? ~0ull : ((1ull << nact) - 1);
        const float sfx = (float)(x0 + slot_x<SMALL>(spix));
        const float sfy = (float)(y0 + slot_y<SMALL>(spix));
        float mnx = sfx, mxx = sfx, mny = sfy, mxy = sfy;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            mnx = fminf(mnx, __shfl_xor(mnx, o, 64));
            mxx = fmaxf(mxx, __shfl_xor(mxx, o, 64));
            mny = fminf(mny, __shfl_xor(mny, o, 64));
            mxy = fmaxf(mxy, __shfl_xor(mxy, o, 64));
        }
        auto uni = [](float v) {  // uniform -> scalar register
            return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
        };
        rx0 = uni(mnx);
        rx1 = uni(mxx);
        ry0 = uni(mny);
        ry1 = uni(mxy);
        irx0 = (uint32_t)((int)rx0 + kBoxBias);
        irx1 = (uint32_t)((int)rx1 + kBoxBias);
        iry0 = (uint32_t)((int)ry0 + kBoxBias);
        iry1 = (uint32_t)((int)ry1 + kBoxBias);
        pc = s_col[spix];  // stays in registers to the end (written back once)
        sparse = true;
    };
    if constexpr (SMALL) {  // one pixel per lane, (x0 + lane % 8, y0 + lane / 8), from the start
        SA = ballot(x0 + (lane & 7) < x1 && y0 + (lane >> 3) < y1);
        nact = 64;
        spix = (uint32_t)(lane & 7) | ((uint32_t)(lane >> 3) << 4);  // (x, y) offsets as 16 * y + x
        sparse = true;
        all_done = SA == 0;
    } else {
        // blocks with few pixels in the image start sparse
        if (!all_done && 256 - __popcll(D0) - __popcll(D1) - __popcll(D2) - __popcll(D3) <= 64) go_sparse();
    }

    // The list streams through a three-stage pipeline, one 64-entry chunk per step; chunk c:
    //   step c-2: index load (coalesced)   step c-1: box gather   step c: box test
    // and the chunk's box survivors join a queue in LDS (list order).  Once kBatch are queued,
    // the first up to 64 become a batch: one survivor per lane gathers its splat data, and the
    // next step culls (exact ellipse test, all lanes busy) and blends the batch.  Each stage's
    // registers live one step, so two slots (ping-pong, unrolled) hold them.  Every global load
    // is issued with the full exec mask and no branch around it, and no register with a pending
    // load is ever copied: a load under a divergent branch or such a copy makes the compiler
    // wait for all outstanding loads (vmcnt is in-order) and the pipeline collapses to one
    // memory latency per step.
    constexpr uint32_t kBatch = GS_DRAW_BATCH;
    uint32_t Vi[2], Vb[2];      // indices: as loaded / riding with the box gather
    uint32_t Oi[2];             // GS_DRAW_SBOX: the index's word offset from vals - 1 (its box's too)
    uint2 Bx[2];                // boxes (int16 pixel bounds, pack_box)
    SurvData Dd;                // the batch's survivor data (lane j: survivor j)
    SurvRgb Dc;                 // ... colour
    uint64_t bk = 0;            // the batch's lanes (uniform)
    bool cfin = true;           // every colour of the batch is finite (uniform)
    uint32_t qn = 0;            // survivors queued (uniform)
    bool inflight = false;      // a batch's data gather is in flight (uniform)

    // Indices are loaded clamped to the list, so every loaded value is a valid splat id and
    // is used as loaded (a select on it right after the load would wait for the load);
    // whether an entry is in the list follows from its position (chunk base + lane < end).
    // gathers address through 32-bit byte offsets (global_load saddr form; splat ids < 2^27)
    auto at = [](const auto *base, uint32_t byte_off) {
        return reinterpret_cast<decltype(base)>(reinterpret_cast<const char *>(base) + byte_off);
    };
    // position p -> word of vals - 1 (the word before vals is 0: a culled entry, splat 0)
    const uint32_t *vals_m1 = vals - 1;
    auto load_idx = [&](int base, uint32_t &v, uint32_t &off) {
        const int p = min(base + lane, jmax);
        const int q = p < cpos ? p : p < cpos + cn ? -1 : p - cn;
        off = (uint32_t)(min(q, qmax) + 1);
        v = *at(vals_m1, off << 2);
    };
    // (ids clamped to the scene: the gathers stay inside the per-splat buffers whatever a frame's
    // values hold -- the clamp sits here, where the index load has arrived, not at the load)
    const uint32_t idmax = (uint32_t)max(P.n - 1, 0);
    // (GS_DRAW_SBOX, a prefix-sorted frame: the box at the entry's position, read in list order;
    // one load either way -- the base and offset are selected, not the load)
    // (SBOX: the launch's P.sbox is set -- a template parameter, so that the positional walk below
    // can issue a chunk's box load with its index load)
    constexpr bool sorted_box = SBOX;
    const uint2 *box_base = sorted_box ? P.sbox - 1 : cullbox;
    auto gather_box = [&](uint32_t v, uint32_t off, uint32_t &vb, uint2 &bx) {
        vb = min(v, idmax);
        bx = *at(box_base, (sorted_box ? off : vb) << 3);
    };
    // box test of a chunk; its survivors join the queue
    auto test_and_queue = [&](int cbase, uint32_t v, const uint2 &bx) __attribute__((always_inline)) {
        // bitwise, not short-circuit: no branch around the compares
        const bool in = (cbase + lane < end) &
                        (!cull | (((bx.x & 0xffffu) <= irx1) & ((bx.x >> 16) >= irx0) & ((bx.y & 0xffffu) <= iry1) &
                                  ((bx.y >> 16) >= iry0)));
        const uint64_t m = ballot(in);
        if (in) s_q[below(m, qn)] = v;
        qn += (uint32_t)__popcll(m);
    };
    // the first up to 64 queued survivors become the batch: lane j gathers survivor j's splat
    // (lanes past the batch re-read its last survivor: same lines); the rest of the queue moves up
    auto issue_batch = [&]() __attribute__((always_inline)) {
        wave_lds_sync();
        const uint32_t bn = min(qn, 64u);
        const uint32_t id = s_q[min((uint32_t)lane, bn - 1u)];
        // the 7 used floats of the SplatDraw record and rgb of the colour
        const SurvLoad ld = *at(reinterpret_cast<const SurvLoad *>(sd), id * (uint32_t)sizeof(SplatDraw));
        Dd = SurvData{ld.mx, ld.my, ld.a, ld.b, ld.c, ld.o, 0.0f};  // thr: once the data arrived (blend_batch)
        Dc = *at(reinterpret_cast<const SurvRgb *>(colour), id << 4);
        bk = bn >= 64u ? ~0ull : ((1ull << bn) - 1ull);
        if (qn > 64u) {  // uniform, rare
            const uint32_t r = s_q[64 + lane];
            wave_lds_sync();
            if ((uint32_t)lane < qn - 64u) s_q[lane] = r;
        }
        qn -= bn;
        inflight = true;
    };
    // dense phase: every survivor's power at all 256 pixels, its blend events compacted into
    // LDS and run one per lane.  Returns true when the block turns sparse (keep: the chunk's
    // survivors left for the sparse phase).
    auto blend_dense = [&](uint64_t &keep, const SurvData &d, const SurvRgb &c) {
        // exact cull of the survivors (uniform keep mask): it costs the wave the same for one
        // survivor as for 64 and drops about a third of them, so it runs from 3 survivors on
        // (same-box A/B: 1 -> 3 survivors, draw 0.335 -> 0.331 ms)
        if (cull && __popcll(keep) >= GS_CULL_DENSE)  // uniform
            keep &= ~ballot(ellipse_misses_rect(d.mx, d.my, d.a, d.b, d.c, d.thr, rx0, rx1, ry0, ry1));
        if (STATS) st_surv += __popcll(keep);
        // one exit (a uniform loop condition, no continue / return inside): fewer scalar
        // control-flow instructions per survivor
        bool turned = false, stop = all_done;  // stop = all_done | turned, set only on a refresh
        // single-exit loop on the survivors left (km): a few scalar instructions of loop control
        // per survivor; a refresh that stops the block hands the rest back in keep and ends it
        uint64_t km = all_done ? 0ull : keep;
        keep = 0;
        // a survivor saturated a pixel (rare): the done masks again from the pixel state; a stop
        // hands the survivors left back in keep and ends the loop
        auto refresh = [&]() {
            if (STATS_FULL) ++st_refresh;
            wave_lds_sync();
            D0 = ballot(s_col[qbase + kQuad[0]].w >= 0.99f);
            D1 = ballot(s_col[qbase + kQuad[1]].w >= 0.99f);
            D2 = ballot(s_col[qbase + kQuad[2]].w >= 0.99f);
            D3 = ballot(s_col[qbase + kQuad[3]].w >= 0.99f);
            all_done = (D0 & D1 & D2 & D3) == ~0ull;  // every pixel saturated
            turned = !all_done && 256 - __popcll(D0) - __popcll(D1) - __popcll(D2) - __popcll(D3) <= 64;
            stop = all_done | turned;
            if (stop) {
                keep = km;
                km = 0;
            }
        };
        if (km) do {
            const int src = __builtin_ctzll(km);
            km &= ~(1ull << src);
            const float mx = rl(d.mx, src), my = rl(d.my, src);
            const float ca = rl(d.a, src), cbv = rl(d.b, src), cc = rl(d.c, src);
            const float thr = rl(d.thr, src);
            // :111-116, per pixel: -0.5*((a*dx)*dx + (c*dy)*dy) - (b*dx)*dy
            // pairs (x0, x1) and (y0, y1) in packed fp32 (v_pk_*): each element is the same
            // IEEE op sequence as the scalar formula
            const f32x2 dx = fxx - f32x2{mx, mx}, dy = fyy - f32x2{my, my};
            const f32x2 ax = (f32x2{ca, ca} * dx) * dx;  // (a*dx)*dx
            const f32x2 cy = (f32x2{cc, cc} * dy) * dy;  // (c*dy)*dy
            const f32x2 bxd = f32x2{cbv, cbv} * dx;      // b*dx
            const f32x2 h = f32x2{-0.5f, -0.5f};
            const f32x2 r0 = h * (ax + f32x2{cy.x, cy.x}) - bxd * f32x2{dy.x, dy.x};  // (p00, p10)
            const f32x2 r1 = h * (ax + f32x2{cy.y, cy.y}) - bxd * f32x2{dy.y, dy.y};  // (p01, p11)
            const float p00 = r0.x, p10 = r0.y, p01 = r1.x, p11 = r1.y;
            // events: needing pixels that are not done
            const uint64_t b0 = ballot(needs(p00, thr)) & ~D0;
            const uint64_t b1 = ballot(needs(p10, thr)) & ~D1;
            const uint64_t b2 = ballot(needs(p01, thr)) & ~D2;
            const uint64_t b3 = ballot(needs(p11, thr)) & ~D3;
            const uint32_t e0 = (uint32_t)__popcll(b0), e1 = (uint32_t)__popcll(b1);
            const uint32_t e2 = (uint32_t)__popcll(b2), e3 = (uint32_t)__popcll(b3);
            const uint32_t nev = e0 + e1 + e2 + e3;
            if (STATS_FULL) {
                ++st_kit;
                const int active = 256 - __popcll(D0) - __popcll(D1) - __popcll(D2) - __popcll(D3);
                st_kit64 += active <= 64 ? 1 : 0;
                st_kit128 += active <= 128 ? 1 : 0;
                st_ev64 += active <= 64 ? nev : 0;
                st_anyneed += nev ? 1 : 0;
                st_pxneed += nev;
                st_a192 += nev ? 1 : 0;                                   // dense steps with events
                st_a128 += nev > 64 ? (unsigned long long)((nev - 1) / 64) : 0ull;  // extra event passes
            }
            if (nev != 0) {  // uniform
            // compact this survivor's blend events (slot k's after slots < k, lane order via
            // v_mbcnt); each pixel occurs at most once, so the events are independent.  The
            // writes are exec-masked by the uniform event masks themselves (inverse ballot).
#if GS_DRAW_POWPIX
            // the powers go to their pixels' slots (every lane, no address arithmetic); the
            // compaction lists only the event pixels
#if GS_DRAW_LANEMAJOR
            s_epow[qbase] = p00;
            s_epow[qbase + 64u] = p10;
            s_epow[qbase + 128u] = p01;
            s_epow[qbase + 192u] = p11;
#else
            *reinterpret_cast<float2 *>(&s_epow[qbase]) = make_float2(p00, p10);
            *reinterpret_cast<float2 *>(&s_epow[qbase + 16u]) = make_float2(p01, p11);
#endif
#endif
            if (__builtin_amdgcn_inverse_ballot_w64(b0)) {
                const uint32_t e = below(b0, 0);
#if !GS_DRAW_POWPIX
                s_epow[e] = p00;
#endif
                s_epix[e] = (uint8_t)(qbase + kQuad[0]);
            }
            if (__builtin_amdgcn_inverse_ballot_w64(b1)) {
                const uint32_t e = below(b1, e0);
#if !GS_DRAW_POWPIX
                s_epow[e] = p10;
#endif
                s_epix[e] = (uint8_t)(qbase + kQuad[1]);
            }
            if (__builtin_amdgcn_inverse_ballot_w64(b2)) {
                const uint32_t e = below(b2, e0 + e1);
#if !GS_DRAW_POWPIX
                s_epow[e] = p01;
#endif
                s_epix[e] = (uint8_t)(qbase + kQuad[2]);
            }
            if (__builtin_amdgcn_inverse_ballot_w64(b3)) {
                const uint32_t e = below(b3, e0 + e1 + e2);
#if !GS_DRAW_POWPIX
                s_epow[e] = p11;
#endif
                s_epix[e] = (uint8_t)(qbase + kQuad[3]);
            }
            wave_lds_sync();
            const float o = rl(d.o, src);
            const float r = rl(c.x, src), g = rl(c.y, src), bl = rl(c.z, src);
            uint32_t sat = 0;  // max bits of the w written (w >= 0: ordered as the floats)
            // one event's blend (draw.glsl:118-134 on the pixel's state)
            auto blend_ev = [&](float power, float4 col) __attribute__((always_inline)) {
                if (cfin) {  // uniform: finite colours -- adding rgb * 0 leaves the state as it is
                    // (and, GS_EV_SAFE, every event's power in [-80, 0]: no underflow select)
                    const float ex = FAST_EXP ? __expf(power) : exp_defined_event<!GS_EV_SAFE>(power);
                    const float alpha = fminf(0.99f, ex * o);
                    const bool take = !(alpha < 1.0f / 255.0f);
                    // alphaBlend :59-67
                    const float remaining = 1.0f - col.w;
                    const float aT = alpha * remaining;
                    const float aZ = take ? aT : 0.0f;
                    col.x = col.x + r * aZ;
                    col.y = col.y + g * aZ;
                    col.z = col.z + bl * aZ;
                    col.w = col.w + aZ;
                } else {
                    const float ex = FAST_EXP ? __expf(power) : exp_defined_event(power);
                    const float alpha = fminf(0.99f, ex * o);
                    const bool take = !(alpha < 1.0f / 255.0f);
                    const float remaining = 1.0f - col.w;
                    const float aT = alpha * remaining;
                    col.x = take ? col.x + r * aT : col.x;
                    col.y = take ? col.y + g * aT : col.y;
                    col.z = take ? col.z + bl * aT : col.z;
                    col.w = take ? col.w + aT : col.w;
                }
                return col;
            };
            auto event = [&](uint32_t e) {
                // straight line: the pixel's state is loaded with the event, before the exp
                const uint32_t pix = s_epix[e];
                const float power = s_epow[GS_DRAW_POWPIX ? pix : e];
                const float4 col = blend_ev(power, s_col[pix]);
                s_col[pix] = col;
                sat = max(sat, __float_as_uint(col.w));  // :129-133
            };
            // every lane runs an event (no exec mask around it): lanes >= nev repeat the last
            // one, reading the same old state and writing the same new state to one address
            event(min((uint32_t)lane, nev - 1u));
            // rare: more events than lanes -- uniform passes, lanes past the end repeat the
            // pass's last event (which no earlier pass held)
            for (uint32_t e0p = 64; e0p < nev; e0p += 64) event(min(e0p + (uint32_t)lane, nev - 1u));
            if (ballot(sat >= __float_as_uint(0.99f))) refresh();  // uniform, rare: a pixel saturated
            wave_lds_sync();  // the next survivor's compaction overwrites s_epow / s_epix
            }
        } while (km);
        return turned;
    };

    // sparse phase (see go_sparse): one pixel per lane, state in registers
    auto blend_sparse = [&](uint64_t keep, const SurvData &d, const SurvRgb &c) {
        if (cull && __popcll(keep) >= GS_CULL_SPARSE)  // uniform (a sparse step costs less: from 6 survivors on)
            keep &= ~ballot(ellipse_misses_rect(d.mx, d.my, d.a, d.b, d.c, d.thr, rx0, rx1, ry0, ry1));
        if (STATS) st_surv += __popcll(keep);
        if (!keep) return;  // uniform
        const float sfx = (float)(x0 + slot_x<SMALL>(spix));
        const float sfy = (float)(y0 + slot_y<SMALL>(spix));
        uint64_t km = all_done ? 0ull : keep;  // single-exit loop, as in blend_dense
        if (km) do {
            const int src = __builtin_ctzll(km);
            km &= ~(1ull << src);
            const float mx = rl(d.mx, src), my = rl(d.my, src);
            const float ca = rl(d.a, src), cbv = rl(d.b, src), cc = rl(d.c, src);
            const float thr = rl(d.thr, src);
            // :111-116, the same op sequence as the packed form below
            const float dx = sfx - mx, dy = sfy - my;
            const float p = -0.5f * ((ca * dx) * dx + (cc * dy) * dy) - (cbv * dx) * dy;
            const uint64_t nb = SA & ballot(needs(p, thr));
            if (STATS_FULL) {
                ++st_kit;
                ++st_kit64;
                ++st_kit128;
                st_anyneed += nb ? 1 : 0;
                st_pxneed += __popcll(nb);
                st_ev64 += __popcll(nb);
                st_a64 += nb ? 1 : 0;  // sparse steps with events
            }
            if (nb) {  // uniform (no continue: one loop exit)
                const float o = rl(d.o, src);
                const float r = rl(c.x, src), g = rl(c.y, src), bl = rl(c.z, src);
                if (cfin) {  // uniform (see the dense event)
                    const float ex = FAST_EXP ? __expf(p) : exp_defined_event<!GS_EV_SAFE>(p);
                    const float alpha = fminf(0.99f, ex * o);
                    const bool take = __builtin_amdgcn_inverse_ballot_w64(nb) & !(alpha < 1.0f / 255.0f);
                    // alphaBlend :59-67
                    const float aT = alpha * (1.0f - pc.w);
                    const float aZ = take ? aT : 0.0f;
                    pc.x = pc.x + r * aZ;
                    pc.y = pc.y + g * aZ;
                    pc.z = pc.z + bl * aZ;
                    pc.w = pc.w + aZ;
                } else {
                    const float ex = FAST_EXP ? __expf(p) : exp_defined_event(p);
                    const float alpha = fminf(0.99f, ex * o);
                    const bool take = __builtin_amdgcn_inverse_ballot_w64(nb) & !(alpha < 1.0f / 255.0f);
                    const float aT = alpha * (1.0f - pc.w);
                    pc.x = take ? pc.x + r * aT : pc.x;
                    pc.y = take ? pc.y + g * aT : pc.y;
                    pc.z = take ? pc.z + bl * aT : pc.z;
                    pc.w = take ? pc.w + aT : pc.w;
                }
                SA &= ~ballot(pc.w >= 0.99f);  // :129-133
                all_done = SA == 0;
                if (all_done) km = 0;
            }
        } while (km);
    };

    // the batch in flight: exact cull and blend (its data arrived; uniform branches)
    auto blend_batch = [&]() __attribute__((always_inline)) {
        if (STATS) ++st_batch;
        Dd.thr = draw_threshold(Dd.o);
        // A blend that does not take an event adds rgb * 0 (and 0 to w) instead of keeping the
        // state by selects: the same bits when every colour of the batch is finite (the state's
        // channels are never -0, and x + (+-0) == x otherwise); a non-finite colour (inf * 0 is
        // NaN) keeps the selects.
        bool ok = __builtin_isfinite(Dc.x) && __builtin_isfinite(Dc.y) && __builtin_isfinite(Dc.z);
        if (GS_EV_SAFE) {  // ... and every power an event can see is finite and >= -80: the need test
            // admits only p in [thr, 0] (NaN p only from non-finite or overflowing inputs, excluded
            // here: |conic| < 1e20 and |mean| < 1e6 keep every product below 1e33)
            ok = ok && (Dd.thr >= -80.0f) && (fabsf(Dd.mx) < 1.0e6f) && (fabsf(Dd.my) < 1.0e6f) &&
                 (fabsf(Dd.a) < 1.0e20f) && (fabsf(Dd.b) < 1.0e20f) && (fabsf(Dd.c) < 1.0e20f);
        }
        cfin = ballot(!ok) == 0;
        if constexpr (SMALL) {
            blend_sparse(bk, Dd, Dc);
        } else {
            if (!sparse && blend_dense(bk, Dd, Dc)) go_sparse();
            if (sparse) blend_sparse(bk, Dd, Dc);
        }
        inflight = false;
    };
    // prologue: chunk 0 index-loaded and box-gathered, chunk 1 index-loaded
    int base = start;
    if (base < end && !all_done) {  // uniform
        uint32_t v0, o0;
        load_idx(base, v0, o0);
        load_idx(base + 64, Vi[1], Oi[1]);
        gather_box(v0, o0, Vb[0], Bx[0]);
        // chunk c's stages use slot c & 1 for the box and (c + 1) & 1 for the next index; step c
        // (slot u = c & 1) issues the loads of chunks c+1..c+2, tests chunk c, then blends the
        // batch in flight and issues the next one
        auto step = [&](auto U) {
            constexpr int u = decltype(U)::value, w = u ^ 1;
            load_idx(base + 128, Vi[u], Oi[u]);        // chunk c+2
            gather_box(Vi[w], Oi[w], Vb[w], Bx[w]);    // chunk c+1
            test_and_queue(base, Vb[u], Bx[u]);  // chunk c
            if (STATS) ++st_iter;
            if (inflight) blend_batch();
            base += 64;
            // past the list's end the steps go on until the queue is drained (their loads re-read
            // the last entry, their tests take nothing)
            if (qn >= kBatch || (base >= end && qn)) issue_batch();  // uniform
            return (base < end || inflight) && !all_done;
        };
        for (;;) {
            if (!step(std::integral_constant<int, 0>{})) break;
            if (!step(std::integral_constant<int, 1>{})) break;
        }
    }
    const bool missed = P.prefix && end < wend && !all_done;  // (uniform) a prefix miss
    if (missed && fr_h_totals) fr_h_totals[2] = 1u;
    // the depth this block's walk reached (the next frames' per-tile prefix targets); a block that
    // missed stopped at the cut, short of what it needs, and records its whole window instead, so
    // the next frames keep that tile whole (up to the global target, which the miss doubles) --
    // recording the reach at the cut kept the tile at that depth: under a moving camera every
    // later frame missed again.  (The missed frame's re-render records the true depth too, but
    // on another lane, unordered with the next frame's class selection.)
    if (P.depth && lane == 0)
        atomicMax(&P.depth[t], (uint32_t)max(0, missed ? wend - start : min(base, end) - start));
    if constexpr (SMALL) {  // the lane's pixel (coordinates again from the lane id, see below)
        const int l2 = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        const int qx = x0 + (l2 & 7), qy = y0 + (l2 >> 3);
        if (qx < x1 && qy < y1) out[(size_t)qy * P.W + qx] = pack_rgba8(pc);
    } else {
    if (sparse && (uint32_t)lane < nact) s_col[spix] = pc;  // the sparse phase's state (distinct pixels)
    wave_lds_sync();
    {  // the quad's pixels again from the lane id (v_mbcnt, which the compiler does not merge with
       // the kernel's start): nothing of the pixel layout stays live across the list loop (it was
       // spilled there, a private segment in the dominant kernel)
        const int l2 = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        const int qx = x0 + 2 * (l2 & 7), qy = y0 + 2 * (l2 >> 3);
#if GS_DRAW_LANEMAJOR
        const int qb = l2, q1 = 64, q2 = 128, q3 = 192;
#else
        const int qb = 32 * (l2 >> 3) + 2 * (l2 & 7), q1 = 1, q2 = 16, q3 = 17;
#endif
        uint32_t *row0 = out + (size_t)qy * P.W + qx, *row1 = row0 + P.W;
        if (qx < x1 && qy < y1) row0[0] = pack_rgba8(s_col[qb + 0]);
        if (qx + 1 < x1 && qy < y1) row0[1] = pack_rgba8(s_col[qb + q1]);
        if (qx < x1 && qy + 1 < y1) row1[0] = pack_rgba8(s_col[qb + q2]);
        if (qx + 1 < x1 && qy + 1 < y1) row1[1] = pack_rgba8(s_col[qb + q3]);
    }
    }
    if (STATS && lane == 0) {  // one plain record per block (no contended atomics)
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        if (L < kDrawTraceBlocks) {
            uint32_t *tr = reinterpret_cast<uint32_t *>(stats) + kDrawTraceWords * L;
            tr[0] = (uint32_t)st_t0;
            tr[1] = (uint32_t)t1;
            tr[2] = (uint32_t)st_iter;
            tr[3] = (uint32_t)st_surv;
            tr[4] = (uint32_t)st_kit;
            tr[5] = (uint32_t)st_anyneed;
            tr[6] = (uint32_t)st_pxneed;
            tr[7] = (uint32_t)max(0, end - start);
            tr[8] = (uint32_t)st_kit64;
            tr[9] = (uint32_t)st_kit128;
            tr[10] = (uint32_t)st_ev64;
            tr[11] = (uint32_t)st_refresh;
            tr[12] = (uint32_t)st_a192;
            tr[13] = (uint32_t)st_a128;
            tr[14] = (uint32_t)st_a64;
            tr[15] = (uint32_t)st_batch;
        }
    }
}

}  // namespace

int preprocess_blocks(int n) { return (n + kSplatsPerBlock - 1) / kSplatsPerBlock; }
int pre_emit_blocks(int n) { return (n + kBlock - 1) / kBlock; }

// Stage timing rides on the dispatch packets (hipExtLaunchKernelGGL start / stop events): a
// separate hipEventRecord costs an idle gap of several microseconds on the stream.
bool rec_packed(const PreParams &P) { return P.clean || (P.W >= 16 && P.H >= 16); }

void launch_sh_kept(hipStream_t s, const PreParams &P, const SceneDev &sc, const FrameDev &fr, const uint32_t *ids,
                    const uint32_t *count, uint32_t cap) {
    const dim3 g((cap + 1 + kBlock - 1) / kBlock);
    if (rec_packed(P)) hipLaunchKernelGGL(k_sh_kept<true>, g, dim3(kBlock), 0, s, P, sc, fr, ids, count, cap);
    else hipLaunchKernelGGL(k_sh_kept<false>, g, dim3(kBlock), 0, s, P, sc, fr, ids, count, cap);
}

void launch_sh_colour(hipStream_t s, const PreParams &P, const SceneDev &sc, const FrameDev &fr) {
    if (P.n <= 0) return;
    const dim3 g((P.n + kBlock - 1) / kBlock);
    if (P.clean || rec_packed(P)) hipLaunchKernelGGL(k_sh_colour<true>, g, dim3(kBlock), 0, s, P, sc, fr);
    else hipLaunchKernelGGL(k_sh_colour<false>, g, dim3(kBlock), 0, s, P, sc, fr);
}

void launch_preprocess(hipStream_t s, const PreParams &P0, const SceneDev &sc, const FrameDev &fr, hipEvent_t start,
                       bool lazy) {
    const int nb = preprocess_blocks(P0.n);
    if (nb <= 0) return;
    PreParams P = P0;
    P.sh = 0;  // GS_FLAG_SH: the colours in a kernel of their own (k_sh_colour), after the records
    // most splats culled last frame (lazy): the queued form, which runs the bulk of the
    // preprocess on the NDC survivors only; else the straight-line form (at C3's 76 % survivors
    // the queue's bookkeeping and gathers cost more than the culled lanes' arithmetic it saves:
    // preprocess 0.110 -> 0.125 ms; view 4 (~3 % survivors) 0.075 -> 0.036 ms)
#define GS_PRE(PK, CL)                                                                                                      \
    if (lazy)                                                                                                               \
        hipExtLaunchKernelGGL((k_preprocess_q<PK, CL>), dim3(nb), dim3(64 * kQWaves), 0, s, start, nullptr, 0, P, sc, fr); \
    else if (fr.theta_in)                                                                                                   \
        hipExtLaunchKernelGGL((k_preprocess<PK, CL, false, true>), dim3(nb), dim3(kBlock), 0, s, start, nullptr, 0, P, sc, fr); \
    else                                                                                                                    \
        hipExtLaunchKernelGGL((k_preprocess<PK, CL, false>), dim3(nb), dim3(kBlock), 0, s, start, nullptr, 0, P, sc, fr)
    if (P.clean) {  // (clean mode always packs its records)
        GS_PRE(true, true);
    } else if (rec_packed(P)) {
        GS_PRE(true, false);
    } else {
        GS_PRE(false, false);
    }
#undef GS_PRE
    if (P0.sh) launch_sh_colour(s, P0, sc, fr);
}

void launch_scan_blocksums(hipStream_t s, const FrameDev &fr, int nblocks, hipEvent_t start, hipEvent_t stop) {
    if (fr.theta_in) hipExtLaunchKernelGGL(k_scan_blocksums<true>, dim3(1), dim3(kScanThreads), 0, s, start, stop, 0, fr, nblocks);
    else hipExtLaunchKernelGGL(k_scan_blocksums<false>, dim3(1), dim3(kScanThreads), 0, s, start, stop, 0, fr, nblocks);
}

void launch_emit(hipStream_t s, int n, bool packed, const FrameDev &fr, uint32_t *keys, uint32_t *vals, uint32_t cap,
                 hipEvent_t start, hipEvent_t stop, uint32_t *prefix_hist) {
    const dim3 grid(std::max(preprocess_blocks(n), 1));
    if (packed) hipExtLaunchKernelGGL(k_emit<true>, grid, dim3(kBlock), 0, s, start, stop, 0, n, fr, keys, vals, cap, prefix_hist);
    else hipExtLaunchKernelGGL(k_emit<false>, grid, dim3(kBlock), 0, s, start, stop, 0, n, fr, keys, vals, cap, prefix_hist);
}

void launch_emit_kept(hipStream_t s, int n, bool packed, const FrameDev &fr, uint32_t *keys, uint32_t *vals, uint32_t cap,
                      const KeptDev &kd, hipEvent_t start, hipEvent_t stop) {
    const dim3 grid(std::max(preprocess_blocks(n), 1));
    if (packed) hipExtLaunchKernelGGL(k_emit_kept<true>, grid, dim3(kBlock), 0, s, start, stop, 0, n, fr, keys, vals, cap, kd);
    else hipExtLaunchKernelGGL(k_emit_kept<false>, grid, dim3(kBlock), 0, s, start, stop, 0, n, fr, keys, vals, cap, kd);
}

void launch_pre_emit(hipStream_t s, const PreParams &P, const SceneDev &sc, const FrameDev &fr, const LookbackDev &lb,
                     bool lazy, uint32_t *keys, uint32_t *vals, uint32_t cap, uint32_t *prefix_hist, hipEvent_t start,
                     hipEvent_t stop) {
    constexpr int KP = 1;
    const uint32_t nb = (uint32_t)pre_emit_blocks(P.n);
    if (nb == 0) {  // no splats: no entries
        hipExtLaunchKernelGGL(k_scan_blocksums<false>, dim3(1), dim3(kScanThreads), 0, s, start, stop, 0, fr, 0);
        return;
    }
    const uint32_t dup_base = (uint32_t)P.n;
#define GS_PE(PK, CL, LZ)                                                                                          \
    hipExtLaunchKernelGGL((k_pre_emit<PK, CL, LZ, KP>), dim3(nb), dim3(kBlock), 0, s, start, stop, 0, P, sc, fr, lb, keys, \
                          vals, cap, dup_base, prefix_hist, nb)
    const bool packed = rec_packed(P);
    if (P.clean) {
        if (lazy) GS_PE(true, true, true);
        else GS_PE(true, true, false);
    } else if (packed) {
        if (lazy) GS_PE(true, false, true);
        else GS_PE(true, false, false);
    } else {
        if (lazy) GS_PE(false, false, true);
        else GS_PE(false, false, false);
    }
#undef GS_PE
}

void launch_bins(hipStream_t s, const uint32_t *keys, int64_t E, const uint32_t *dev_count, uint32_t *counts,
                 uint32_t *bins, hipEvent_t stop) {
    const int64_t per = (int64_t)kBlock * kBinItems;
    const int64_t nb = (E + per - 1) / per;
    if (nb > 0)
        hipLaunchKernelGGL(k_bins_count, dim3((unsigned)nb), dim3(kBlock), 0, s, keys, E, dev_count, counts);
    hipExtLaunchKernelGGL(k_bins_scan, dim3(1), dim3(kBlock), 0, s, nullptr, stop, 0, counts, bins);
}

void launch_draw(hipStream_t s, const DrawParams &P, bool fast_exp, bool small, const uint32_t *bins,
                 const uint32_t *vals, const FrameDev &fr, const float4 *colour, uint32_t *out,
                 unsigned long long *stats, hipEvent_t start, hipEvent_t stop) {
    // 1-D grid: 256 tiles x (nbx*nby) one-wave sub-blocks (16x16, or 8x8 when small), XCD-major
    // (see k_draw), then the margin blocks (256 uncovered pixels each); with no coverage only
    // margin blocks run
    const int margin = P.W * P.H - P.coverW * P.coverH;
    const dim3 grid(std::max(kTiles * kTiles * P.nbx * P.nby + (margin + 255) / 256, 1));
    // (GS_DRAW_SBOX off: the sorted boxes are never set, see the frame paths)
    auto go = [&](auto kern) {
        hipExtLaunchKernelGGL(kern, grid, dim3(64), 0, s, start, stop, 0, P, bins, vals, fr.cullbox, fr.sd, colour, out,
                              stats, fr.h_totals);
    };
#define GS_DRAW(F, S, M) (P.sbox ? go(k_draw<F, S, M, true>) : go(k_draw<F, S, M, false>))
#define GS_DRAW2(F, S) (small ? GS_DRAW(F, S, true) : GS_DRAW(F, S, false))
    if (stats) {
        if (fast_exp) GS_DRAW2(true, true);
        else GS_DRAW2(false, true);
    } else {
        if (fast_exp) GS_DRAW2(true, false);
        else GS_DRAW2(false, false);
    }
#undef GS_DRAW2
#undef GS_DRAW
}

}  // namespace gs
