/*
 * gs_oracle.h -- CPU oracle for the Gaussian-splat hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (openglgaussiansplattingrenderer_amd/)
 * links, loads or calls this code.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / the timed CPU baseline.
 *
 * It is a plain-C restatement of the reference's GPU semantics (reference = the
 * thomas-chernaik/OpenGLGaussianSplattingRenderer checkout, paths relative to it):
 *   loader        src/Splats.cpp:174-344          ora_ply_count / ora_ply_load
 *   covariance    src/Splats.cpp:414-479          ora_cov3d
 *   preprocess    shaders/preprocess.glsl:64-190  ora_preprocess
 *   entry layout  preprocess.glsl:153-188         ora_emit (deterministic)
 *   radix sort    src/sort.cpp:139-203 + generateHistograms/computePrefixSum/scan.glsl
 *                                                 ora_argsort_f32 / ora_sort_pairs
 *   bins          shaders/countBins.glsl:20-31 + prefixBins.glsl:13-54    ora_bins
 *   blend         shaders/draw.glsl:59-143        ora_draw
 *   test RNG      src/utils.cpp:49-63             ora_gen_sort_keys
 *
 * Parity pins: the sort is pinned by the reference's own known-answer test
 * (tests/sortTests.cpp:181-244; golden hashes in BASELINE.md section 4), the loader by
 * tests/plyParseTests.cpp:105-109 (testSingleItem.ply, N == 1).  Preprocess / bins /
 * blend: the reference ships no outputs for them (its GL output is undefined at every
 * configured size), so those stages are cross-checked against an independent
 * float64 numpy restatement in tests/ -- "parity pinned by restatement only".
 *
 * Floating point: compiled with -ffp-contract=off, every expression evaluated in the
 * order written below (glm's operator order for matrix products), so the HIP path can
 * reproduce keys / conics / means bit for bit.
 */
#ifndef GS_ORACLE_H
#define GS_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* flags (same bit meaning as the product's GS_FLAG_*) */
#define ORA_FLAG_CLEAN 1u  /* fix the deterministic quirks Q4/Q5/Q6/Q9/Q10 */

/* src/utils.cpp:49-63 createRandomNumbersFloat (srand(20), glibc rand) */
void ora_gen_sort_keys(int n, float *out);

/* FNV-1a-64, one 32-bit word per step (golden hashes in BASELINE.md section 4) */
uint64_t ora_fnv1a64_words(const uint32_t *words, uint64_t nwords);

/* src/sort.cpp:139-203 GPURadixSort(size=n, workGroupCount=16, workGroupSize=32):
 * stable LSD argsort, 8 passes x 4-bit digits of floatBitsToUint(keys[order[i]]),
 * 512 sections; `order` is permuted in place, keys are not moved. */
void ora_argsort_f32(const float *keys, int32_t *order, int n);

/* stable sort of (key, value) pairs by the key bits -- same algorithm, keys moved too */
void ora_sort_pairs(uint32_t *keys, uint32_t *vals, int64_t n);

/* src/Splats.cpp:252-267 header walk: returns N, or -1 on error */
int ora_ply_count(const char *path);
/* src/Splats.cpp:174-344: activations exactly as the loader applies them.
 * means4: (x,y,z,1)  colours4: ((0.5+C0*f_dc)*255, ..., 1)  opacity: sigmoid
 * scales3: exp(log-scale)  rots4: normalised (rot_0..rot_3).  returns 0 / -1 */
int ora_ply_load(const char *path, int n, float *means4, float *colours4, float *opacity,
                 float *scales3, float *rots4);

/* src/Splats.cpp:414-479: Sigma = (S*R)^T (S*R), upper triangle [00,01,02,11,12,22] */
void ora_cov3d(int n, const float *scales3, const float *rots4, float *cov6);

/* shaders/preprocess.glsl:64-190 for every splat.
 * outputs (per splat): means2d[2], conic4[4] (conic.xyz, opacity), z01, tilexy (main tile
 * x, y -- unclamped in ref mode), rect4 (minX,maxX,minY,maxY), counts2 (main entry 0/1, duplicates). */
void ora_preprocess(int n, const float *means4, const float *cov6, const float *opacity,
                    const float *view16, const float *vp16, int W, int H, float fx, float fy,
                    float tan_fov_x, float tan_fov_y, uint32_t flags,
                    float *means2d, float *conic4, float *z01, int32_t *tilexy, int32_t *rect4,
                    int32_t *counts2);

/* Deterministic entry layout: positions [0,V) hold the main entries in splat order,
 * [V, V+D) the duplicates splat-major (rect y-major, x-minor, main tile skipped).
 * key = floatBitsToUint(float(tileIndex) + z01), value = splat index.
 * Returns E = V + D (entries written only when E <= cap). */
int64_t ora_emit(int n, const float *z01, const int32_t *tilexy, const int32_t *rect4,
                 const int32_t *counts2, uint32_t *keys, uint32_t *vals, int64_t cap);

/* countBins.glsl + prefixBins.glsl: bins[t] = #entries with int(key) in [0,t] */
void ora_bins(const uint32_t *keys, int64_t n, uint32_t *bins256);

/* draw.glsl:70-143 -> RGBA8 (row y = gl y).  vals = sorted splat indices. */
void ora_draw(int W, int H, uint32_t flags, const uint32_t *bins256, const uint32_t *vals,
              int64_t E, const float *means2d, const float *conic4, const float *colours4,
              uint8_t *rgba);

/* same, only rows row_start, row_start + row_step, ... (bounded CPU-baseline samples) */
void ora_draw_rows(int W, int H, uint32_t flags, const uint32_t *bins256, const uint32_t *vals,
                   int64_t E, const float *means2d, const float *conic4, const float *colours4,
                   uint8_t *rgba, int row_start, int row_step);

/* the exp used by the blend (draw.glsl:122); exported for tests */
float ora_expf(float x);

/* SURVEY f3 (beyond the reference; GS_FLAG_SH): colours4[i] = (max(SH(dir)+0.5, 0)*255, 1) with
 * dir = normalize(mean - campos), campos = -R^T t of view16, degree-3 SH in the standard 3D
 * Gaussian Splatting convention (f_dc3 raw, f_rest45 channel-major as in the ply).  Only
 * splats with visible[i] != 0 are written.  Not pinned by the reference (it has no SH). */
void ora_sh_colours(int n, const float *means4, const float *f_dc3, const float *f_rest45, const float *view16,
                    const uint8_t *visible, float *colours4);

/* OpenMP threads the oracle uses (for the cpu_baseline "cores" field) */
int ora_num_threads(void);

#ifdef __cplusplus
}
#endif
#endif
