/*
 * gs_oracle.c -- CPU oracle (TEST INFRASTRUCTURE ONLY; see gs_oracle.h).
 * Build: oracle/Makefile  (gcc -O2 -fopenmp -ffp-contract=off)
 */
#include "gs_oracle.h"

#include <limits.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

int ora_num_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ------------------------------------------------------------------ helpers */

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* GLSL int(float): truncation.  Out-of-range / NaN resolved the way gfx950's
 * v_cvt_i32_f32 does it (saturate, NaN -> 0) so CPU and GPU agree. */
static inline int f2i(float f)
{
    if (f != f) return 0;
    if (f >= 2147483648.0f) return INT_MAX;
    if (f <= -2147483648.0f) return INT_MIN;
    return (int)f;
}
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int imin(int a, int b) { return a < b ? a : b; }

/* glm operator*(mat4, vec4) (type_mat4x4.inl): (m0*x + m1*y) + (m2*z + m3*w) */
static inline void mat4_vec4(const float *m, float x, float y, float z, float w, float o[4])
{
    for (int r = 0; r < 4; ++r)
        o[r] = (m[0 * 4 + r] * x + m[1 * 4 + r] * y) + (m[2 * 4 + r] * z + m[3 * 4 + r] * w);
}

/* glm operator*(mat3, mat3) (type_mat3x3.inl), column-major a[c][r]:
 * R[c][r] = A[0][r]*B[c][0] + A[1][r]*B[c][1] + A[2][r]*B[c][2] (left to right) */
static inline void mat3_mul(const float a[3][3], const float b[3][3], float o[3][3])
{
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r)
            o[c][r] = a[0][r] * b[c][0] + a[1][r] * b[c][1] + a[2][r] * b[c][2];
}
static inline void mat3_transpose(const float a[3][3], float o[3][3])
{
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) o[c][r] = a[r][c];
}

/* --------------------------------------------------------------- test RNG */

void ora_gen_sort_keys(int n, float *out)
{
    /* src/utils.cpp:49-63 */
    srand(20);
    for (int i = 0; i < n; i++) {
        int random = rand() % 255;
        out[i] = (float)rand() / RAND_MAX + random + 0.5f;
    }
}

uint64_t ora_fnv1a64_words(const uint32_t *words, uint64_t nwords)
{
    /* FNV-1a-64 with one 32-bit word per step (the convention of the golden hashes
     * in BASELINE.md section 4) */
    uint64_t h = 1469598103934665603ULL;
    for (uint64_t i = 0; i < nwords; ++i) {
        h ^= words[i];
        h *= 1099511628211ULL;
    }
    return h;
}

/* ------------------------------------------------------------- radix sort */

/*
 * src/sort.cpp:139-203.  numberOfSections = 16*32 = 512, sectionSize = ceil(n/512).
 * Per pass i (4-bit digit i):
 *   generateHistograms.glsl:30-68  per-section 16-bin histogram of
 *                                  (floatBitsToUint(key[order[j]]) >> 4i) & 15
 *   computePrefixSum.glsl:16-51    per digit exclusive scan over sections; digit bases =
 *                                  exclusive scan of the digit totals
 *   scan.glsl:36-81                per section in order: dst = base[d] + off[s][d]++
 *   then the order / intermediate buffers swap (8 passes -> result back in `order`).
 * Q15 (stale histograms of empty sections) and Q14 (in-place Hillis-Steele races) are
 * resolved to the intended semantics: empty sections contribute zero counts.
 */
static void lsd_sections(const uint32_t *key_of_pos, int32_t *order,
                         int32_t *tmp, int64_t n)
{
    const int64_t S = 16 * 32;
    const int64_t pad = (n % S == 0) ? 0 : S - n % S;   /* PadBuffer, src/sort.cpp:127-137 */
    const int64_t sectionSize = (n + pad) / S;
    int32_t *hist = (int32_t *)calloc((size_t)(S * 16 + 16), sizeof(int32_t));
    int32_t *src = order, *dst = tmp;
    for (int pass = 0; pass < 8; ++pass) {
        const int shift = pass * 4;
        /* generateHistograms */
        for (int64_t s = 0; s < S; ++s) {
            int32_t h[16] = {0};
            int64_t start = s * sectionSize;
            if (start < n) {
                int64_t end = start + sectionSize;
                if (end > n) end = n;
                for (int64_t j = start; j < end; ++j) {
                    uint32_t k = key_of_pos[src[j]];
                    h[(k >> shift) & 15u]++;
                }
            }
            memcpy(hist + s * 16, h, sizeof(h));
        }
        /* computePrefixSum */
        int32_t total[16];
        for (int d = 0; d < 16; ++d) {
            int32_t run = 0;
            for (int64_t s = 0; s < S; ++s) {
                int32_t v = hist[s * 16 + d];
                hist[s * 16 + d] = run;
                run += v;
            }
            total[d] = run;
        }
        int32_t base[16];
        base[0] = 0;
        for (int d = 1; d < 16; ++d) base[d] = base[d - 1] + total[d - 1];
        /* scan.glsl scatter */
        for (int64_t s = 0; s < S; ++s) {
            int64_t start = s * sectionSize;
            if (start >= n) continue;
            int64_t end = start + sectionSize;
            if (end > n) end = n;
            int32_t off[16];
            memcpy(off, hist + s * 16, sizeof(off));
            for (int64_t j = start; j < end; ++j) {
                uint32_t k = key_of_pos[src[j]];
                uint32_t d = (k >> shift) & 15u;
                dst[base[d] + off[d]++] = src[j];
            }
        }
        int32_t *t = src; src = dst; dst = t;
    }
    /* 8 passes (even): result is back in `order` */
    free(hist);
}

void ora_argsort_f32(const float *keys, int32_t *order, int n)
{
    if (n <= 0) return;
    int32_t *tmp = (int32_t *)malloc((size_t)n * sizeof(int32_t));
    lsd_sections((const uint32_t *)(const void *)keys, order, tmp, n);
    free(tmp);
}

void ora_sort_pairs(uint32_t *keys, uint32_t *vals, int64_t n)
{
    if (n <= 0) return;
    /* argsort by key bits (positions as the payload), then apply the permutation */
    int32_t *order = (int32_t *)malloc((size_t)n * sizeof(int32_t));
    int32_t *tmp = (int32_t *)malloc((size_t)n * sizeof(int32_t));
    for (int64_t i = 0; i < n; ++i) order[i] = (int32_t)i;
    lsd_sections(keys, order, tmp, n);
    uint32_t *k2 = (uint32_t *)malloc((size_t)n * 4), *v2 = (uint32_t *)malloc((size_t)n * 4);
    for (int64_t i = 0; i < n; ++i) { k2[i] = keys[order[i]]; v2[i] = vals[order[i]]; }
    memcpy(keys, k2, (size_t)n * 4);
    memcpy(vals, v2, (size_t)n * 4);
    free(k2); free(v2); free(order); free(tmp);
}

/* ------------------------------------------------------------------ loader */

static int read_line(FILE *f, char *buf, int cap)
{
    /* std::getline: read up to '\n', drop it */
    int len = 0, c;
    while ((c = fgetc(f)) != EOF && c != '\n')
        if (len < cap - 1) buf[len++] = (char)c;
    buf[len] = 0;
    return (c == EOF && len == 0) ? -1 : len;
}

int ora_ply_count(const char *path)
{
    /* src/Splats.cpp:250-262: skip 2 lines, third line "element vertex N" */
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    char line[512], a[64], b[64];
    int n = -1;
    for (int i = 0; i < 2; ++i) read_line(f, line, sizeof line);
    read_line(f, line, sizeof line);
    if (sscanf(line, "%63s %63s %d", a, b, &n) != 3) n = -1;
    fclose(f);
    return n;
}

int ora_ply_load(const char *path, int n, float *means4, float *colours4, float *opacity,
                 float *scales3, float *rots4)
{
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    char line[512];
    for (int i = 0; i < 3; ++i) read_line(f, line, sizeof line);
    /* src/Splats.cpp:264-267 loop until the exact line "end_header" */
    while (strcmp(line, "end_header") != 0)
        if (read_line(f, line, sizeof line) < 0) { fclose(f); return -1; }
    const float SH_C0 = 0.28209479177387814f;
    for (int i = 0; i < n; ++i) {
        float rec[62];
        if (fread(rec, 4, 62, f) != 62) { fclose(f); return -1; }
        /* mean :281-284 */
        means4[4 * i + 0] = rec[0]; means4[4 * i + 1] = rec[1];
        means4[4 * i + 2] = rec[2]; means4[4 * i + 3] = 1.f;
        /* normal rec[3..5] dropped :286-287; colour :291-299 */
        for (int c = 0; c < 3; ++c) colours4[4 * i + c] = (0.5f + (SH_C0 * rec[6 + c])) * 255.f;
        colours4[4 * i + 3] = 1.f;
        /* 45 f_rest rec[9..53] read and discarded :301-302; opacity :304-309 */
        float o = rec[54];
        opacity[i] = (1 / (1 + expf(-o)));
        /* scale :311-319 */
        for (int c = 0; c < 3; ++c) scales3[3 * i + c] = expf(rec[55 + c]);
        /* rotation :321-331 */
        float r0 = rec[58], r1 = rec[59], r2 = rec[60], r3 = rec[61];
        float length = sqrtf(r0 * r0 + r1 * r1 + r2 * r2 + r3 * r3);
        rots4[4 * i + 0] = r0 / length; rots4[4 * i + 1] = r1 / length;
        rots4[4 * i + 2] = r2 / length; rots4[4 * i + 3] = r3 / length;
    }
    /* :333-340 EOF check */
    int extra = fgetc(f);
    fclose(f);
    return extra == EOF ? 0 : -1;
}

/* -------------------------------------------------------------- covariance */

void ora_cov3d(int n, const float *scales3, const float *rots4, float *cov6)
{
    for (int i = 0; i < n; ++i) {
        /* src/Splats.cpp:440-479 */
        float S[3][3] = {{scales3[3 * i + 0], 0, 0}, {0, scales3[3 * i + 1], 0}, {0, 0, scales3[3 * i + 2]}};
        float r = rots4[4 * i + 0], x = rots4[4 * i + 1], y = rots4[4 * i + 2], z = rots4[4 * i + 3];
        float R[3][3] = {
            {1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y)},
            {2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x)},
            {2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y)}};
        float M[3][3], Mt[3][3], Sig[3][3];
        mat3_mul(S, R, M);             /* transformationMatrix = scaleMatrix * rotationMatrix */
        mat3_transpose(M, Mt);
        mat3_mul(Mt, M, Sig);          /* transpose(T) * T */
        cov6[6 * i + 0] = Sig[0][0]; cov6[6 * i + 1] = Sig[0][1]; cov6[6 * i + 2] = Sig[0][2];
        cov6[6 * i + 3] = Sig[1][1]; cov6[6 * i + 4] = Sig[1][2]; cov6[6 * i + 5] = Sig[2][2];
    }
}

/* -------------------------------------------------------------- preprocess */

void ora_preprocess(int n, const float *means4, const float *cov6, const float *opacity,
                    const float *view16, const float *vp16, int W, int H, float fx, float fy,
                    float tan_fov_x, float tan_fov_y, uint32_t flags,
                    float *means2d, float *conic4, float *z01, int32_t *tilexy, int32_t *rect4,
                    int32_t *counts2)
{
    const int clean = (flags & ORA_FLAG_CLEAN) != 0;
    const unsigned screenWidth = (unsigned)W, screenHeight = (unsigned)H;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        const float mx = means4[4 * i + 0], my = means4[4 * i + 1], mz = means4[4 * i + 2];
        means2d[2 * i + 0] = 0.f; means2d[2 * i + 1] = 0.f;
        conic4[4 * i + 0] = conic4[4 * i + 1] = conic4[4 * i + 2] = conic4[4 * i + 3] = 0.f;
        z01[i] = 0.f; tilexy[2 * i] = tilexy[2 * i + 1] = 0;
        rect4[4 * i + 0] = rect4[4 * i + 1] = rect4[4 * i + 2] = rect4[4 * i + 3] = 0;
        counts2[2 * i + 0] = counts2[2 * i + 1] = 0;

        /* :77-78 */
        float p[4];
        mat4_vec4(vp16, mx, my, mz, 1.0f, p);
        const float w = fmaxf(p[3], 0.0001f);
        p[0] = p[0] / w; p[1] = p[1] / w; p[2] = p[2] / w; p[3] = p[3] / w;
        /* :80-89 cull (NDC x/y only) */
        if (p[0] < -1.0f || p[0] > 1.0f || p[1] < -1.0f || p[1] > 1.0f) continue;
        /* :91-94 */
        float sx = (p[0] + 1.0f) * 0.5f, sy = (p[1] + 1.0f) * 0.5f, sz = (p[2] + 1.0f) * 0.5f;
        sx = sx * (float)screenWidth;
        sy = sy * (float)screenHeight;
        if (clean && !(sz >= 0.0f && sz <= 1.0f)) continue;   /* clean: near/far cull (Q6) */
        means2d[2 * i + 0] = sx; means2d[2 * i + 1] = sy;

        /* :98-108 */
        const float *c6 = cov6 + 6 * (size_t)i;
        float Sig[3][3] = {{c6[0], c6[1], c6[2]}, {c6[1], c6[3], c6[4]}, {c6[2], c6[4], c6[5]}};
        float W3[3][3] = {{view16[0], view16[1], view16[2]},
                          {view16[4], view16[5], view16[6]},
                          {view16[8], view16[9], view16[10]}};
        /* :110-116 */
        float t4[4];
        mat4_vec4(view16, mx, my, mz, 1.0f, t4);
        float tx = t4[0], ty = t4[1], tz = t4[2];
        const float limx = -1.3f * tan_fov_x, limy = -1.3f * tan_fov_y;
        const float txtz = tx / tz, tytz = ty / tz;
        tx = fminf(limx, fmaxf(-limx, txtz)) * tz;
        ty = fminf(limy, fmaxf(-limy, tytz)) * tz;
        /* :118-122 (column-major constructor) */
        float J[3][3] = {{fx / tz, 0.0f, -(fx * tx) / (tz * tz)},
                         {0.0f, fy / tz, -(fy * ty) / (tz * tz)},
                         {0.0f, 0.0f, 0.0f}};
        /* :124-128 */
        float W3t[3][3], T[3][3], Tt[3][3], Sigt[3][3], A[3][3], C[3][3];
        mat3_transpose(W3, W3t);
        mat3_mul(W3t, J, T);
        mat3_transpose(T, Tt);
        mat3_transpose(Sig, Sigt);
        mat3_mul(Tt, Sigt, A);
        mat3_mul(A, T, C);
        C[0][0] += 0.3f;
        C[1][1] += 0.3f;
        /* :129-136 */
        const float ca = C[0][0], cb = C[0][1], cc = C[1][1];
        const float det = ca * cc - cb * cb;
        if (det == 0) continue;                                  /* Q7: entry omitted */
        if (clean && !(det > 0.0f)) continue;
        const float inv = 1.0f / det;
        conic4[4 * i + 0] = cc * inv;
        conic4[4 * i + 1] = -cb * inv;
        conic4[4 * i + 2] = ca * inv;
        conic4[4 * i + 3] = opacity[i];
        /* :139-149 */
        const float middle = (cc + ca) * 0.5f;
        const float l1 = middle + sqrtf(fmaxf(0.1f, middle * middle - det));
        const float l2 = middle - sqrtf(fmaxf(0.1f, middle * middle - det));
        const float radius = ceilf(3.0f * sqrtf(fmaxf(l1, l2)));
        float tw, th;
        if (!clean) { tw = (float)(screenWidth / 16); th = (float)(screenHeight / 16); }  /* Q4 */
        else { tw = (float)W / 16.f; th = (float)H / 16.f; }
        int minX = imax(0, f2i((sx - radius) / tw));
        int maxX = imin(15, f2i((sx + radius) / tw));
        int minY = imax(0, f2i((sy - radius) / th));
        int maxY = imin(15, f2i((sy + radius) / th));
        /* :151-155 main tile (unclamped in the reference, Q5) */
        int tileX = f2i(sx / tw), tileY = f2i(sy / th);
        if (clean) { tileX = imin(15, imax(0, tileX)); tileY = imin(15, imax(0, tileY)); }
        z01[i] = sz;
        tilexy[2 * i + 0] = tileX;
        tilexy[2 * i + 1] = tileY;
        rect4[4 * i + 0] = minX; rect4[4 * i + 1] = maxX;
        rect4[4 * i + 2] = minY; rect4[4 * i + 3] = maxY;
        /* :157-189 duplicates: every rect tile except the main one (Q5/Q8/Q12 resolved) */
        int rectCount = (maxX >= minX && maxY >= minY) ? (maxX - minX + 1) * (maxY - minY + 1) : 0;
        int mainInRect = (tileX >= minX && tileX <= maxX && tileY >= minY && tileY <= maxY);
        counts2[2 * i + 0] = 1;
        counts2[2 * i + 1] = rectCount - mainInRect;
    }
}

int64_t ora_emit(int n, const float *z01, const int32_t *tilexy, const int32_t *rect4,
                 const int32_t *counts2, uint32_t *keys, uint32_t *vals, int64_t cap)
{
    int64_t V = 0, D = 0;
    for (int i = 0; i < n; ++i) { V += counts2[2 * i]; D += counts2[2 * i + 1]; }
    const int64_t E = V + D;
    if (E > cap || !keys || !vals) return E;
    int64_t m = 0, d = V;
    for (int i = 0; i < n; ++i) {
        if (!counts2[2 * i]) continue;
        const float z = z01[i];
        const int tileX = tilexy[2 * i], tileY = tilexy[2 * i + 1];
        /* :153-155 uint tileIndex = tileY*16 + tileX; key = tileIndex + projectedMean.z */
        const uint32_t tileIndex = (uint32_t)tileY * 16u + (uint32_t)tileX;
        keys[m] = f2u((float)tileIndex + z);
        vals[m] = (uint32_t)i;
        ++m;
        const int minX = rect4[4 * i], maxX = rect4[4 * i + 1], minY = rect4[4 * i + 2], maxY = rect4[4 * i + 3];
        /* :171-188 y-major, x-minor, main tile skipped */
        for (int y = minY; y <= maxY; ++y)
            for (int x = minX; x <= maxX; ++x) {
                if (x == tileX && y == tileY) continue;
                keys[d] = f2u((float)(uint32_t)(y * 16 + x) + z);
                vals[d] = (uint32_t)i;
                ++d;
            }
    }
    return E;
}

void ora_bins(const uint32_t *keys, int64_t n, uint32_t *bins256)
{
    /* countBins.glsl:20-31: bins[int(key)]++ for int(key) in [0,256) */
    uint32_t cnt[256] = {0};
    for (int64_t j = 0; j < n; ++j) {
        int v = f2i(u2f(keys[j]));
        if (v < 0 || v >= 256) continue;
        cnt[v]++;
    }
    /* prefixBins.glsl:13-54: inclusive scan */
    uint32_t run = 0;
    for (int t = 0; t < 256; ++t) { run += cnt[t]; bins256[t] = run; }
}

/* ---------------------------------------------------------------- blend */

float ora_expf(float x)
{
    /* exp for draw.glsl:122.  GLSL leaves exp's rounding to the implementation (3 + 2|x|
     * ulp allowed); this restatement fixes one: Cody-Waite reduction (cephes constants) and
     * a degree-6 Horner polynomial, every step one correctly rounded fmaf (~2 ulp).  The
     * GPU kernel evaluates the same fma sequence, so the two agree bit for bit.  Inputs
     * below -80 return 0 (exp(-80)*opacity is far below the 1/255 cut of draw.glsl:123). */
    if (!(x >= -80.0f)) return 0.0f;
    if (x > 80.0f) x = 80.0f;
    const float kf = rintf(x * 1.44269504088896341f);
    float r = fmaf(-kf, 0.693359375f, x);
    r = fmaf(-kf, -2.12194440e-4f, r);
    float t = fmaf(0.00138888892f, r, 0.00833333377f);
    t = fmaf(t, r, 0.0416666679f);
    t = fmaf(t, r, 0.166666672f);
    t = fmaf(t, r, 0.5f);
    t = fmaf(t, r, 1.0f);
    const float p = fmaf(t, r, 1.0f);
    const int k = (int)kf;
    return p * u2f((uint32_t)(k + 127) << 23);
}

void ora_draw(int W, int H, uint32_t flags, const uint32_t *bins256, const uint32_t *vals,
              int64_t E, const float *means2d, const float *conic4, const float *colours4,
              uint8_t *rgba)
{
    ora_draw_rows(W, H, flags, bins256, vals, E, means2d, conic4, colours4, rgba, 0, 1);
}

void ora_draw_rows(int W, int H, uint32_t flags, const uint32_t *bins256, const uint32_t *vals,
                   int64_t E, const float *means2d, const float *conic4, const float *colours4,
                   uint8_t *rgba, int row_start, int row_step)
{
    const int clean = (flags & ORA_FLAG_CLEAN) != 0;
    /* src/Splats.cpp:596 tile size passed as float(W)/16.f, float(H)/16.f */
    const float tileWidth = (float)W / 16.f, tileHeight = (float)H / 16.f;
    /* Q9: the dispatch is (W/32) x (H/32) groups of 32x32 */
    const int coverW = clean ? W : (W / 32) * 32, coverH = clean ? H : (H / 32) * 32;
    memset(rgba, 0, (size_t)W * H * 4);
    if (row_step < 1) row_step = 1;
#pragma omp parallel for schedule(dynamic, 1)
    for (int y = row_start; y < coverH; y += row_step) {
        for (int x = 0; x < coverW; ++x) {
            float cr = 0.f, cg = 0.f, cbl = 0.f, ca = 0.f;
            /* :78-89 */
            const int tileX = f2i((float)x / tileWidth), tileY = f2i((float)y / tileHeight);
            const int tileIndex = tileY * 16 + tileX;
            int64_t start = (tileIndex == 0) ? 0 : (int64_t)bins256[tileIndex - 1];
            int64_t end = bins256[tileIndex];
            if (!clean && end > start) {
                /* Q10: the last 1024-chunk is blended whole (draw.glsl:94-135) */
                int64_t chunks = (end - start + 1023) / 1024;
                end = start + chunks * 1024;
                if (end > E) end = E;
            }
            for (int64_t j = start; j < end; ++j) {
                const uint32_t s = vals[j];
                const float *m = means2d + 2 * (size_t)s;
                const float *co = conic4 + 4 * (size_t)s;
                /* :111-126 */
                const float dx = (float)x - m[0], dy = (float)y - m[1];
                const float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                if (power > 0.0f) continue;
                const float alpha = fminf(0.99f, ora_expf(power) * co[3]);
                if (alpha < 1.0f / 255.0f) continue;
                /* alphaBlend :59-67 */
                const float *rgb = colours4 + 4 * (size_t)s;
                const float remaining = 1.0f - ca;
                const float aT = alpha * remaining;
                cr = cr + rgb[0] * aT;
                cg = cg + rgb[1] * aT;
                cbl = cbl + rgb[2] * aT;
                ca = ca + aT;
                if (ca >= 0.99f) break;  /* :129-133 */
            }
            /* :141-142 col/255 stored to an rgba8 image: unorm round-to-nearest */
            const float v[4] = {cr / 255.0f, cg / 255.0f, cbl / 255.0f, ca / 255.0f};
            uint8_t *o = rgba + 4 * ((size_t)y * W + x);
            for (int c = 0; c < 4; ++c) {
                float t = v[c];
                t = t != t ? 0.0f : t;
                t = t < 0.0f ? 0.0f : (t > 1.0f ? 1.0f : t);
                o[c] = (uint8_t)floorf(t * 255.0f + 0.5f);
            }
        }
    }
}

/* ---------------------------------------------------------------- SH colour (f3) */

static float ora_sh_channel(const float *k16, float x, float y, float z)
{
    /* k16[0] = f_dc, k16[1..15] = f_rest of one channel; evaluation order of the standard 3DGS
     * computeColorFromSH (the kernel's sh_channel evaluates the same sequence) */
    const float SH_C0 = 0.28209479177387814f, SH_C1 = 0.4886025119029199f;
    const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f, -1.0925484305920792f,
                            0.5462742152960396f};
    const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f, 0.3731763325901154f,
                            -0.4570457994644658f, 1.445305721320277f, -0.5900435899266435f};
    float r = SH_C0 * k16[0];
    r = r - SH_C1 * y * k16[1] + SH_C1 * z * k16[2] - SH_C1 * x * k16[3];
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    r = r + SH_C2[0] * xy * k16[4] + SH_C2[1] * yz * k16[5] + SH_C2[2] * (2.0f * zz - xx - yy) * k16[6] +
        SH_C2[3] * xz * k16[7] + SH_C2[4] * (xx - yy) * k16[8];
    r = r + SH_C3[0] * y * (3.0f * xx - yy) * k16[9] + SH_C3[1] * xy * z * k16[10] +
        SH_C3[2] * y * (4.0f * zz - xx - yy) * k16[11] + SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * k16[12] +
        SH_C3[4] * x * (4.0f * zz - xx - yy) * k16[13] + SH_C3[5] * z * (xx - yy) * k16[14] +
        SH_C3[6] * x * (xx - 3.0f * yy) * k16[15];
    r = r + 0.5f;
    return fmaxf(r, 0.0f) * 255.0f;
}

void ora_sh_colours(int n, const float *means4, const float *f_dc3, const float *f_rest45, const float *view16,
                    const uint8_t *visible, float *colours4)
{
    float campos[3];
    for (int c = 0; c < 3; ++c)
        campos[c] = -(view16[4 * c + 0] * view16[12] + view16[4 * c + 1] * view16[13] + view16[4 * c + 2] * view16[14]);
    #pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        if (!visible[i]) continue;
        float dx = means4[4 * i] - campos[0], dy = means4[4 * i + 1] - campos[1], dz = means4[4 * i + 2] - campos[2];
        const float len = sqrtf(dx * dx + dy * dy + dz * dz);
        dx = dx / len;
        dy = dy / len;
        dz = dz / len;
        for (int c = 0; c < 3; ++c) {
            float k16[16];
            k16[0] = f_dc3[3 * (size_t)i + c];
            for (int k = 1; k < 16; ++k) k16[k] = f_rest45[45 * (size_t)i + 15 * c + (k - 1)];
            colours4[4 * (size_t)i + c] = ora_sh_channel(k16, dx, dy, dz);
        }
        colours4[4 * (size_t)i + 3] = 1.0f;
    }
}
