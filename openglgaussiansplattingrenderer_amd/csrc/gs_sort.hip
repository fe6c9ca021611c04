// gs_sort.hip -- stable LSD radix sort of (uint32 key, uint32 value) pairs on gfx950.
//
// Replaces GPURadixSort (src/sort.cpp:139-203) and its shaders generateHistograms.glsl,
// computePrefixSum.glsl, scan.glsl (8 passes x 4-bit digits, 512 serial threads with
// indirect key gathers).  Here: 4 passes x 8-bit digits, reduce-then-scan per pass with no
// inter-workgroup communication inside a launch:
//   k_upsweep    per 4096-key tile (8192 in pass 0), 256-bin digit histogram -> hist[digit][tile]
//   k_scan_rows  one workgroup per digit: exclusive scan of hist[digit][*], row totals
//   k_downsweep  wave64 ballot-match ranking (stable), LDS reorder, coalesced scatter
// A frame's tile bins (countBins.glsl: a count per int(key), then its prefix) ride along: the
// first upsweep also counts tiles, and one more workgroup of the last k_scan_rows launch
// scans them (replacing two launches and a read of the keys).
// Stability: inside a tile, wave w owns elements [w*1024, (w+1)*1024) in order and ranks them
// sequentially (item k, then lane), so equal digits keep their input order; tiles are
// ordered by the digit-major scan.  The result is therefore the unique stable sort -- the
// one the reference's test (tests/sortTests.cpp:240-243) and the oracle define.
#include "gs_internal.hpp"

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <type_traits>

namespace gs {

namespace {

constexpr int kItems = 16;                    // keys per lane
constexpr int kWaveTile = 64 * kItems;        // 1024 keys per wave
#ifndef GS_WAVE_SMALL
#define GS_WAVE_SMALL 4
#endif
#ifndef GS_WAVE_BIG
#define GS_WAVE_BIG 8
#endif
constexpr int kWaveSmall = GS_WAVE_SMALL, kWaveBig = GS_WAVE_BIG;   // waves per workgroup: passes 1-3 / pass 0
constexpr int kTileSmall = kWaveSmall * kWaveTile;  // 4096
// waves per workgroup of a frame's prefix-sort first pass (its downsweep's LDS holds a whole tile)
#ifndef GS_PREFIX_P0_WAVES
#define GS_PREFIX_P0_WAVES GS_WAVE_BIG
#endif
constexpr int kP0Waves = GS_PREFIX_P0_WAVES;
// keys per lane in a prefix sort's passes 1-3 (the ~1M kept keys of a frame: 8 -> 2048-key tiles, twice
// the workgroups of the 4096-key form; same box: sort stage 0.132 -> 0.123 ms, one frame -1 %)
#ifndef GS_SUB_ITEMS
#define GS_SUB_ITEMS 8
#endif
constexpr int kSubItems = GS_SUB_ITEMS;
constexpr int kRadix = 256;
constexpr int kRep = 8;  // upsweep counter replicas per digit (lane % 8)

__device__ __forceinline__ int lane_id() { return __lane_id(); }

constexpr int kTileCopies = kTileCopyCount;  // tile counters spread over copies (by workgroup): fewer same-address atomics

// GLSL int(float) (countBins.glsl's int(key)): v_cvt_i32_f32 itself (truncate, saturate, NaN -> 0)
__device__ __forceinline__ int f2i(float f) {
    int r;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(f));
    return r;
}

// mask of the active lanes whose 8-bit digit equals this lane's (8 ballots).  Per bit: s = the
// lane's bit sign-extended (v_bfe_i32), the ballot of it, and the lanes that differ accumulate
// as x |= ballot ^ s -- one v_bitop3 per mask half and bit, written out (left to itself the
// compiler pairs the xors into v_or3, three VALU per two bits and half instead of two);
// the match is ~x & active.  4 VALU per bit.
__device__ __forceinline__ uint32_t or_xor(uint32_t acc, uint32_t s, uint32_t ballot_half) {
    // acc | (s ^ ballot_half): the table is the expression evaluated on src0 = 0xf0, src1 = 0xcc,
    // src2 = 0xaa: 0xf0 | (0xcc ^ 0xaa) = 0xf6 (checked on the GPU: tools/micro/bitop3_check.hip).
    // The builtin, not inline asm: the compiler then also inserts the wait states a VALU read of
    // the just-written ballot SGPR needs (the inline-asm form missed them and mis-sorted)
    return __builtin_amdgcn_bitop3_b32(acc, s, ballot_half, 0xf6);
}
__device__ __forceinline__ uint64_t match_digit(uint32_t d, uint64_t active) {
    uint32_t xlo = 0, xhi = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        uint32_t sb = (uint32_t)__builtin_amdgcn_sbfe((int)d, b, 1);  // v_bfe_i32
        asm volatile("" : "+v"(sb));  // keep the compare on sb (no shift + compare rewrite)
        const uint64_t bb = __ballot(sb != 0u);
        xlo = or_xor(xlo, sb, (uint32_t)bb);
        xhi = or_xor(xhi, sb, (uint32_t)(bb >> 32));
    }
    return (((uint64_t)~xhi << 32) | ~xlo) & active;
}

// number of set bits of m below this lane (v_mbcnt)
__device__ __forceinline__ uint32_t count_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// exclusive scan over the W*64 threads of a block (one value each)
template <int W>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *s_wave) {
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan(v);
    if (lane == 63) s_wave[wid] = inc;
    __syncthreads();
    uint32_t off = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) off += (w < wid) ? s_wave[w] : 0u;
    __syncthreads();
    return off + inc - v;
}

// the same, also returning the block total
template <int W>
__device__ __forceinline__ uint32_t block_excl_scan_tot(uint32_t v, uint32_t *s_wave, uint32_t *total) {
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan(v);
    if (lane == 63) s_wave[wid] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        off += (w < wid) ? s_wave[w] : 0u;
        tot += s_wave[w];
    }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

// element count: n, or min(n, cnt[0] + cnt[1]) when the count lives on the device (a frame
// enqueued without a host round trip; the grid is sized for n, the capacity)
__device__ __forceinline__ uint32_t elem_count(uint32_t n, const uint32_t *cnt) {
    return cnt ? min(n, cnt[0] + cnt[1]) : n;
}

// Tile of a workgroup: workgroups are dealt round-robin over the 8 XCDs (block b runs on XCD
// b % 8), so XCD x is given the contiguous tiles [x * per, (x + 1) * per): neighbouring
// columns of hist[digit][tile] are then written and read through one L2 instead of eight
// (the upsweep's 4-byte column stores wrote back as partial lines from every XCD).  The grid
// is 8 * ceil(capacity tiles / 8) workgroups; the mapping uses the live tiles (the count read
// on the device), so every XCD gets work; workgroups mapped past them return.
__device__ __forceinline__ uint32_t xcd_tile(uint32_t live) {
    const uint32_t per = (live + 7) / 8, j = blockIdx.x >> 3;
    return j < per ? (blockIdx.x & 7u) * per + j : 0xffffffffu;  // (>= live: no tile)
}
// the same ranges walked from their ends: a pass's upsweep over a key array larger than the
// 256 MiB Infinity Cache, walked backwards, leaves the first tiles of each range -- where its
// downsweep starts -- the most recently read, so those key lines are still cached there
__device__ __forceinline__ uint32_t xcd_tile_rev(uint32_t live) {
    const uint32_t per = (live + 7) / 8, j = blockIdx.x >> 3;
    return j < per ? (blockIdx.x & 7u) * per + (per - 1 - j) : 0xffffffffu;
}
__host__ __device__ constexpr uint32_t xcd_grid(uint32_t nb) { return 8 * ((nb + 7) / 8); }

// W waves per workgroup, tile = W * 1024 keys (the pass-0 sort uses W = 8: its random low
// digits leave short runs per tile, so a larger tile doubles the scatter's write runs)
// tile_counts != null: also countBins.glsl:20-31 -- tile_counts[int(key)] += 1 for int(key) in
// [0, 256), LDS replicas, then one global atomic per nonzero tile and workgroup
// PREFIX (the first pass of a frame's prefix sort): only the keys at or below their class
// bound (PrefixDev::theta) are counted for the digits; the tile counts (TILES) stay over every
// key; the kept keys per class and the keys below 1.0 (class 0's total) go to pre.counts
// dup_base (the first pass of a frame sort after k_pre_emit, else kNoSplit): the input is the
// emission's split layout -- element i < V at i, element i >= V at i - V + dup_base (V = cnt[0])
constexpr uint32_t kNoSplit = 0xffffffffu;
__device__ __forceinline__ uint32_t split_at(uint32_t idx, uint32_t v0, uint32_t gap) {
    return idx >= v0 ? idx + gap : idx;
}

// The bucket sort's first digit (BKT): the key's tile, int(key) as a float, for keys below 255.0;
// 255 for every key from 255.0's bits on (tile 255's keys, 1e6, +inf, NaN and the negative
// floats, which sort after them as unsigned words).  Monotone in the unsigned key, so a stable
// scatter by it followed by a stable sort of each bucket is the stable sort of the keys.
constexpr uint32_t kBits255 = 0x437f0000u;  // 255.0f
__device__ __forceinline__ uint32_t bucket_of(uint32_t key) {
    return key >= kBits255 ? 255u : (uint32_t)f2i(__uint_as_float(key));
}
template <bool BKT>
__device__ __forceinline__ uint32_t digit_of(uint32_t key, int shift) {
    return BKT ? bucket_of(key) : (key >> shift) & 0xffu;
}

template <int W, bool TILES, bool PREFIX = false, bool BKT = false, int IT = kItems, bool REV = false>
__global__ __launch_bounds__(W * 64) void k_upsweep(const uint32_t *__restrict__ keys, uint32_t n_max,
                                                    const uint32_t *__restrict__ cnt, int shift,
                                                    uint32_t *__restrict__ hist, uint32_t nb,
                                                    uint32_t *__restrict__ tile_counts, PrefixDev pre,
                                                    uint32_t dup_base) {
    constexpr int kThreads = W * 64, kTile = kThreads * IT;
    static_assert(kThreads >= kRadix, "one thread per digit flushes the counts");
    const uint32_t n = elem_count(n_max, cnt);
    const uint32_t live = (n + kTile - 1) / kTile;
    const uint32_t tile = REV ? xcd_tile_rev(live) : xcd_tile(live);
    if (tile >= live) return;  // uniform: tile beyond the count (never scanned)
    // counts need no ranks: LDS atomics.  Each digit has kRep counters picked by lane % 8, so
    // a wave whose keys share one digit (the top-byte pass) serialises 8-way, not 64-way.
    __shared__ uint32_t s_cnt[kRadix * kRep];
    __shared__ uint32_t s_tiles[TILES ? kRadix * kRep : 1];
    __shared__ uint32_t s_above;
    __shared__ uint32_t s_theta[PREFIX ? kClasses : 1];
    __shared__ uint32_t s_sel[PREFIX ? kClasses * kRep : 1];
    __shared__ uint32_t s_low;
    for (int i = threadIdx.x; i < kRadix * kRep; i += kThreads) {
        s_cnt[i] = 0;
        if (TILES) s_tiles[i] = 0;
    }
    if (PREFIX) {
        for (int i = threadIdx.x; i < kClasses * kRep; i += kThreads) s_sel[i] = 0;
        for (int i = threadIdx.x; i < kClasses; i += kThreads) s_theta[i] = pre.theta[i];
        if (threadIdx.x == 0) s_low = 0;
    }
    if (TILES && threadIdx.x == 0) s_above = 0;
    __syncthreads();
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    const uint32_t base = tile * (uint32_t)kTile + wid * (uint32_t)(64 * IT) + lane;
    uint32_t kk[IT];
    if (dup_base != kNoSplit) {  // uniform: the split emission layout
        const uint32_t v0 = cnt[0], gap = dup_base - v0;
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const uint32_t idx = base + k * 64;
            kk[k] = (idx < n) ? keys[split_at(idx, v0, gap)] : 0u;
        }
    } else if (tile * (uint32_t)kTile + kTile <= n) {  // uniform: full tile, immediate offsets
        const uint32_t *p = keys + base;
#pragma unroll
        for (int k = 0; k < IT; ++k) kk[k] = p[k * 64];
    } else {
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const uint32_t idx = base + k * 64;
            kk[k] = (idx < n) ? keys[idx] : 0u;
        }
    }
    const uint32_t rep = (uint32_t)lane & (kRep - 1);
    uint32_t above = 0, low = 0;
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const uint32_t idx = base + k * 64;
        if (idx < n) {
            bool keep = true;
            if (PREFIX) {
                const uint32_t c = key_class(kk[k]);
                keep = kk[k] <= s_theta[c];
                if (keep) atomicAdd(&s_sel[c * kRep + rep], 1u);
                low += kk[k] < kKey1Bits ? 1u : 0u;
            }
            if (keep) atomicAdd(&s_cnt[digit_of<BKT>(kk[k], shift) * kRep + rep], 1u);
            if (TILES) {  // the frame's tile counts ride on the first pass
                const uint32_t t = (uint32_t)f2i(__uint_as_float(kk[k]));
                if (t < (uint32_t)kRadix) atomicAdd(&s_tiles[t * kRep + rep], 1u);
                above += kk[k] > kKeyCulledBits ? 1u : 0u;  // entries after the reference's culled ones
            }
        }
    }
    if (TILES) {
        above = wave_incl_scan(above);
        if (lane == 63 && above) atomicAdd(&s_above, above);
    }
    if (PREFIX) {
        low = wave_incl_scan(low);
        if (lane == 63 && low) atomicAdd(&s_low, low);
    }
    __syncthreads();
    if (TILES && threadIdx.x == 0 && s_above) atomicAdd(&tile_counts[kTileCopies * kRadix + (blockIdx.x % kTileCopies)], s_above);
    auto sum8 = [](const uint32_t *p) {
        const uint4 c0 = *reinterpret_cast<const uint4 *>(p);
        const uint4 c1 = *reinterpret_cast<const uint4 *>(p + 4);
        return (c0.x + c0.y + c0.z + c0.w) + (c1.x + c1.y + c1.z + c1.w);
    };
    if (PREFIX) {
        uint32_t *pc = pre.counts + (blockIdx.x % kPrefixCopies) * kClasses;
        for (int c = threadIdx.x; c < kClasses; c += kThreads) {
            const uint32_t v = sum8(&s_sel[c * kRep]);
            if (v) atomicAdd(&pc[c], v);
        }
        if (threadIdx.x == 0 && s_low) atomicAdd(&pre.counts[kPrefixCopies * kClasses + (blockIdx.x % kPrefixCopies)], s_low);
    }
    const int d = threadIdx.x;
    if (d >= kRadix) return;
    hist[(size_t)d * nb + tile] = sum8(&s_cnt[d * kRep]);
    if (TILES) {
        const uint32_t c = sum8(&s_tiles[d * kRep]);
        if (c) atomicAdd(&tile_counts[(blockIdx.x % kTileCopies) * kRadix + d], c);
    }
}

// tile bins from the tile counts (one workgroup of 256): bins[t] = inclusive prefix, and the
// draw's tile order bins[256 + r] = the tile with the r-th longest list (ties by index); the
// counts are cleared for the next frame
// (returns the tile's count and the exclusive prefix; *s_above gets the keys above 1e6)
// (s_c: kRadix words of LDS, 16-byte aligned, the caller's)
__device__ uint2 bins_scan(uint32_t *__restrict__ counts, uint32_t *__restrict__ bins, uint32_t *s_w,
                           uint32_t *s_above, uint32_t *s_c) {
    const int t = threadIdx.x;
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < kTileCopies; ++k) {
        v += counts[k * kRadix + t];
        counts[k * kRadix + t] = 0;
    }
    s_c[t] = v;
    if (t < kTileCopies) {  // entries with key bits above 1e6 (k_draw places the culled ones before them)
        const uint32_t a = counts[kTileCopies * kRadix + t];
        counts[kTileCopies * kRadix + t] = 0;
        uint32_t sa = a;
#pragma unroll
        for (int o = 1; o < kTileCopies; o <<= 1) sa += __shfl_xor(sa, o, 64);
        if (t == 0) {
            bins[2 * kRadix] = sa;
            *s_above = sa;
        }
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan_tot<4>(v, s_w, &tot);  // (its barriers also publish s_c)
    bins[t] = ex + v;
    // rank = #tiles ahead of t: longer, or as long with a smaller index.  With every count below
    // 2^24 (tot < 2^24; uniform) the order is that of one word, count << 8 | (255 - tile):
    // one compare per tile, four tiles per LDS read
    uint32_t r = 0;
    if (tot < (1u << 24)) {
        s_c[t] = (v << 8) | (uint32_t)(255 - t);  // (each thread rewrites its own word)
        __syncthreads();
        const uint32_t key = (v << 8) | (uint32_t)(255 - t);
        const uint4 *q = reinterpret_cast<const uint4 *>(s_c);
        // (unrolled by 4, not 16: 16 VGPRs of reads in flight, so the kernels holding this
        // workgroup stay within the 64 VGPRs a SIMD has free beside seven blend waves)
#pragma unroll 4
        for (int u = 0; u < kRadix / 4; ++u) {
            const uint4 c = q[u];
            r += (c.x > key ? 1u : 0u) + (c.y > key ? 1u : 0u) + (c.z > key ? 1u : 0u) + (c.w > key ? 1u : 0u);
        }
    } else {
#pragma unroll 32
        for (int u = 0; u < kRadix; ++u) {
            const uint32_t c = s_c[u];
            r += (c > v || (c == v && u < t)) ? 1u : 0u;
        }
    }
    bins[kRadix + r] = (uint32_t)t;
    return make_uint2(v, ex);
}

// The prefix sort's class tables (one workgroup of 256 in the first pass's scan, after its
// histogram read; t = tile = class): class starts in the full order P (class 0: the keys below
// 1.0; tiles 1..255: their counts; class 256: the rest) and in the kept subset, the placement
// delta, the kept count (the element count of passes 1-3; above their capacity the frame is
// flagged).  The kept counters are cleared for the next frame (the tile counts stay for the
// bins workgroup of the last pass).
__device__ void prefix_counts(const uint32_t *__restrict__ tile_counts, const PrefixDev &pre,
                              const uint32_t *__restrict__ cnt, uint32_t n_max, uint32_t *s_w) {
    __shared__ uint32_t s_low, s_k256;
    const int t = threadIdx.x;
    uint32_t kept = 0, v = 0;
#pragma unroll
    for (int k = 0; k < kPrefixCopies; ++k) {
        kept += pre.counts[k * kClasses + t];
        pre.counts[k * kClasses + t] = 0;
        v += tile_counts[k * kRadix + t];
    }
    if (t < kPrefixCopies) {  // class 256 and the keys below 1.0
        uint32_t a = pre.counts[t * kClasses + 256], b = pre.counts[kPrefixCopies * kClasses + t];
        pre.counts[t * kClasses + 256] = 0;
        pre.counts[kPrefixCopies * kClasses + t] = 0;
#pragma unroll
        for (int o = 1; o < kPrefixCopies; o <<= 1) {
            a += __shfl_xor(a, o, 64);
            b += __shfl_xor(b, o, 64);
        }
        if (t == 0) {
            s_k256 = a;
            s_low = b;
        }
    }
    __syncthreads();
    // (the frame's entry count: a kept emission's first pass counts only its kept entries)
    const uint32_t E = elem_count(pre.cap_all, pre.frame_count ? pre.frame_count : cnt);
    const uint32_t m = t == 0 ? s_low : v;  // keys of class t
    uint32_t tot_m, tot_k;
    const uint32_t P = block_excl_scan_tot<4>(m, s_w, &tot_m);
    const uint32_t off = block_excl_scan_tot<4>(kept, s_w, &tot_k);
    pre.delta[t] = (int32_t)(P - off);
    pre.cls[t] = P;
    pre.cls[kClasses + 1 + t] = P + kept;
    if (t == 0) {
        const uint32_t nsel = tot_k + s_k256;
        pre.delta[256] = (int32_t)(tot_m - tot_k);
        pre.cls[256] = tot_m;
        pre.cls[257] = E;
        pre.cls[kClasses + 1 + 256] = tot_m + s_k256;
        pre.nsel[0] = nsel;
        pre.nsel[1] = 0;
        if (pre.h_slot) pre.h_slot[3] = nsel;  // (above cap_sel: passes 1-3 cannot hold them, the host renders again)
    }
}

// The prefix sort's draw limits (the bins workgroup of the last pass): the bins, then per tile
// the first position of its draw window that was not sorted -- in the draw's positions, which
// hold the reference's culled entries (cn of them at cpos, k_draw) besides the sorted ones;
// 0xffffffff: none.
// LDS: s_PG holds bins_scan's scratch, then the class starts s_P and the gaps s_G (2 KB in all:
// with the row scans' 16 B this workgroup's kernel fits beside seven blend waves per SIMD); the
// kept ends are read from pre.cls where the search lands
__device__ void prefix_limits(uint32_t *__restrict__ counts, uint32_t *__restrict__ bins, const PrefixDev &pre,
                              const uint32_t *__restrict__ cnt, uint32_t *s_w, uint32_t *s_PG) {
    __shared__ uint32_t s_above;
    __shared__ uint32_t s_gw[4];
    uint32_t *s_P = s_PG, *s_G = s_PG + (kClasses + 1);
    const int t = threadIdx.x, lane = lane_id(), wid = t >> 6;
    const uint2 vb = bins_scan(counts, bins, s_w, &s_above, s_PG);  // (its barriers publish s_above)
    const uint32_t P = pre.cls[t], L = pre.cls[kClasses + 1 + t];
    const uint32_t P256 = pre.cls[256], E = pre.cls[257], L256 = pre.cls[kClasses + 1 + 256];
    const uint32_t Pn = t < 255 ? pre.cls[t + 1] : P256;  // the next class's start
    __syncthreads();  // every thread's bins_scan reads of s_PG are done
    s_P[t] = P;
    if (t == 0) {
        s_P[256] = P256;
        s_P[257] = E;
    }
    // G[c]: the first position not sorted at or after class c's start (E: none) -- a suffix min
    // of each class's gap (its kept end, when it kept less than all)
    const uint32_t gap256 = L256 < E ? L256 : E;
    uint32_t g = L < Pn ? L : E;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_down(g, o, 64);
        if (lane + o < 64) g = min(g, u);
    }
    if (lane == 0) s_gw[wid] = g;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < 4; ++w)
        if (w > wid) g = min(g, s_gw[w]);
    g = min(g, gap256);
    s_G[t] = g;
    if (t == 0) s_G[256] = gap256;
    __syncthreads();
    // tile t's draw window starts at its bins start (draw positions; culled entries at [cpos, cpos + cn))
    const int V = (int)cnt[0];
    const uint32_t cn = pre.clean ? 0u : (uint32_t)max(0, pre.n - V);
    const uint32_t cpos = (uint32_t)min(max((int)E - (int)s_above, 0), (int)E);
    const uint32_t p0 = vb.y;
    const uint32_t q0 = p0 < cpos ? p0 : (p0 < cpos + cn ? cpos : p0 - cn);
    uint32_t fi = 0xffffffffu;
    if (q0 < E) {
        int c = 0;  // the last class starting at or before q0
#pragma unroll
        for (int step = 256; step > 0; step >>= 1)
            if (c + step <= 256 && s_P[c + step] <= q0) c += step;
        const uint32_t fq = q0 >= pre.cls[kClasses + 1 + c] ? q0 : s_G[c];
        if (fq < E) fi = fq < cpos ? fq : fq + cn;
    }
    bins[kBinsLimit + t] = fi;
}

// One workgroup of 256 per digit (a small workgroup finds room on a CU beside the previous
// frame's blend; 1024-thread ones waited for a CU to drain): exclusive scan of that digit's
// per-tile counts (the tiles holding elements; rows are nb long), row total.  Each thread owns
// kPer consecutive counts per round, so a round (256 * kPer tiles) costs one memory round
// trip: kPer 16 (4096 tiles = 16.7M keys) for frames, 64 with 16-byte loads for sorts beyond
// that (64M keys: one round instead of four, 28 -> ? us per pass).  With bins != null, block
// kRadix computes the tile bins from tile_counts instead.
// BINS false (a pass without the bins workgroup): none of its LDS and a few VGPRs -- 16 bytes
// of LDS and kPer 4 fit beside seven blend waves per SIMD, so another frame's blend leaves room
template <int kPer = 16, bool BINS = true>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kPer <= 16 ? 8 : 1))) void k_scan_rows(uint32_t *__restrict__ hist, uint32_t nb_stride, uint32_t n_max,
                                                   const uint32_t *__restrict__ cnt, uint32_t tile,
                                                   uint32_t *__restrict__ row_total, uint32_t *__restrict__ tile_counts,
                                                   uint32_t *__restrict__ bins, PrefixDev pre, int prefix) {
    __shared__ uint32_t s_w[4];
    if (BINS && blockIdx.x == kRadix) {  // uniform: the bins workgroup
        __shared__ __attribute__((aligned(16))) uint32_t s_PG[2 * (kClasses + 1) + 1];
        if (prefix == 1) {
            prefix_counts(tile_counts, pre, cnt, n_max, s_w);
        } else if (prefix == 2) {
            prefix_limits(tile_counts, bins, pre, pre.frame_count, s_w, s_PG);
        } else {
            __shared__ uint32_t s_above;
            bins_scan(tile_counts, bins, s_w, &s_above, s_PG);
        }
        return;
    }
    const uint32_t nb = (elem_count(n_max, cnt) + tile - 1) / tile;
    uint32_t *row = hist + (size_t)blockIdx.x * nb_stride;
    uint32_t carry = 0;
    for (uint32_t b = 0; b < nb; b += 256 * kPer) {
        const uint32_t i0 = b + threadIdx.x * kPer;
        uint32_t v[kPer], a = 0;
        if (kPer > 16 && (nb_stride & 3u) == 0 && i0 + kPer <= nb) {  // whole 16-byte groups (row start aligned)
            const uint4 *r4 = reinterpret_cast<const uint4 *>(row + i0);
#pragma unroll
            for (int k = 0; k < kPer / 4; ++k) {
                const uint4 q = r4[k];
                v[4 * k] = q.x, v[4 * k + 1] = q.y, v[4 * k + 2] = q.z, v[4 * k + 3] = q.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < kPer; ++k) v[k] = (i0 + k < nb) ? row[i0 + k] : 0u;
        }
#pragma unroll
        for (int k = 0; k < kPer; ++k) a += v[k];
        uint32_t tot;
        uint32_t off = carry + block_excl_scan_tot<4>(a, s_w, &tot);
        if (kPer > 16 && (nb_stride & 3u) == 0 && i0 + kPer <= nb) {
            uint4 *r4 = reinterpret_cast<uint4 *>(row + i0);
#pragma unroll
            for (int k = 0; k < kPer / 4; ++k) {
                uint4 q;
                q.x = off;
                off += v[4 * k];
                q.y = off;
                off += v[4 * k + 1];
                q.z = off;
                off += v[4 * k + 2];
                q.w = off;
                off += v[4 * k + 3];
                r4[k] = q;
            }
        } else {
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                if (i0 + k < nb) row[i0 + k] = off;
                off += v[k];
            }
        }
        carry += tot;
    }
    if (threadIdx.x == 0) row_total[blockIdx.x] = carry;
}

// FMT: the pass's element format
//   kPairs   (key, value) in, (key, value) out
//   kPackOut (key, value) in, packed out: key's top byte | value (value < 2^24), into kout
//   kPackIn  packed in (kin), value out (vout): the last pass of a frame sort, whose keys
//            nobody reads (the draw needs the values and the bins only)
//   kPlace   (key, value) in, value out at its position in the full order: the last pass of a
//            frame's prefix sort (position in the subset + pre.delta[class of the key])
// PREFIX: the first pass of a prefix sort -- only the keys at or below their class bound move
constexpr int kPairs = 0, kPackOut = 1, kPackIn = 2, kPlace = 3;
template <int W, int FMT, bool PREFIX = false, int IT = kItems>
__global__ __launch_bounds__(W * 64) void k_downsweep(const uint32_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                      uint32_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                      uint32_t n_max, const uint32_t *__restrict__ cnt, int shift,
                                                      const uint32_t *__restrict__ hist, uint32_t nb,
                                                      const uint32_t *__restrict__ row_total, PrefixDev pre,
                                                      uint32_t dup_base) {
    constexpr int kThreads = W * 64, kTile = kThreads * IT, kWaves = W, kWT = 64 * IT;
    static_assert(kThreads >= kRadix, "one thread per digit scans the counts");
    const uint32_t n = elem_count(n_max, cnt);
    const uint32_t live = (n + kTile - 1) / kTile;
    const uint32_t tile = xcd_tile(live);
    // GS_DRAW_SBOX: the box before position 0 is what k_draw reads for the reference's culled
    // entries (a Q10 window past the last tile list; drawn as splat 0, preprocess.glsl:80-88,
    // draw.glsl:97-98): splat 0's box of this frame (its culled record when it has no entries)
    if (FMT == kPlace && GS_DRAW_SBOX && pre.box_out && blockIdx.x == 0 && threadIdx.x == 0)
        pre.box_out[-1] = pre.cullbox[0];
    if (tile >= live) return;  // uniform: tile beyond the count
    __shared__ uint32_t s_cnt[kWaves][kRadix];  // running per-wave counts -> per-wave exclusive offsets
    __shared__ uint32_t s_start[kRadix];        // block-local start of each digit
    __shared__ int32_t s_gbase[kRadix];         // global position of local slot 0 of each digit
    __shared__ uint32_t s_wave[kWaves];
    __shared__ uint32_t s_keys[kTile];
    __shared__ uint32_t s_vals[FMT == kPackIn ? 1 : kTile];
    __shared__ int32_t s_cls[(PREFIX || FMT == kPlace) ? kClasses : 1];  // class bounds / placement deltas
    __shared__ uint32_t s_tile_n;

    for (int i = threadIdx.x; i < kWaves * kRadix; i += kThreads) (&s_cnt[0][0])[i] = 0;
    if (PREFIX || FMT == kPlace)
        for (int i = threadIdx.x; i < kClasses; i += kThreads)
            s_cls[i] = PREFIX ? (int32_t)pre.theta[i] : pre.delta[i];
    __syncthreads();
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    const uint32_t tile0 = tile * (uint32_t)kTile;
    const uint32_t base = tile0 + wid * (uint32_t)kWT + lane;
    uint32_t kk[IT], vv[IT];
    if (dup_base != kNoSplit) {  // uniform: the split emission layout (see k_upsweep)
        const uint32_t v0 = cnt[0], gap = dup_base - v0;
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const uint32_t idx = base + k * 64;
            const uint32_t a = split_at(idx, v0, gap);
            kk[k] = (idx < n) ? kin[a] : 0u;
            vv[k] = (FMT != kPackIn && idx < n) ? vin[a] : 0u;
        }
    } else if (tile0 + kTile <= n) {  // uniform: full tile, immediate offsets
        const uint32_t *pk = kin + base, *pv = vin + base;
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            kk[k] = pk[k * 64];
            vv[k] = FMT == kPackIn ? 0u : pv[k * 64];
        }
    } else {
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const uint32_t idx = base + k * 64;
            kk[k] = (idx < n) ? kin[idx] : 0u;
            vv[k] = (FMT != kPackIn && idx < n) ? vin[idx] : 0u;
        }
    }
    // Stable rank of each key among this wave's keys of its digit, in (item, lane) order:
    //   1. per item, the match mask of equal digits (independent VALU work for all items);
    //   2. per item, its first lane adds the item's count to the wave's counter with a
    //      returning LDS atomic -- one wave's LDS operations execute in issue order, so the
    //      returned value is the count of that digit in the earlier items; all 16 atomics are
    //      issued back to back (one LDS round trip, not one per item);
    //   3. peers fetch their leader's returned value (ds_bpermute).
    uint32_t rank[IT], lead[IT], old[IT];
    uint32_t keepm = 0;  // PREFIX: bit k = item k is kept (after the compaction: k * 64 + lane < kept)
    uint32_t nit = IT;  // items holding elements (uniform)
    if (PREFIX) {
        // The kept keys of the wave (about a fifth) move to the front of its 1024 slots, in
        // (item, lane) order -- the order stability needs -- so only ceil(kept / 64) items are
        // ranked.  (s_keys / s_vals are free until the block-level reorder below.)
        uint32_t *ck = s_keys + wid * kWT, *cv = s_vals + wid * kWT;
        uint32_t nk = 0;
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const bool keep = base + k * 64 < n && kk[k] <= (uint32_t)s_cls[key_class(kk[k])];
            const uint64_t m = __ballot(keep);
            if (keep) {
                const uint32_t slot = nk + count_below(m);
                ck[slot] = kk[k];
                cv[slot] = vv[k];
            }
            nk += (uint32_t)__popcll(m);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        nit = (nk + 63) / 64;
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const uint32_t slot = (uint32_t)(k * 64 + lane);
            if ((uint32_t)k < nit && slot < nk) {
                kk[k] = ck[slot];
                vv[k] = cv[slot];
                keepm |= 1u << k;
            }
        }
    }
    // the ranking of the first NI items (the others hold no element)
#define GS_RANK_ITEMS(NI)                                                                             \
    do {                                                                                              \
        _Pragma("unroll") for (int k = 0; k < (NI); ++k) {                                            \
            const uint32_t idx = base + k * 64;                                                       \
            const bool valid = PREFIX ? ((keepm >> k) & 1u) != 0 : idx < n;                           \
            const uint32_t d = digit_of<false>(kk[k], shift);                                           \
            const uint64_t m = match_digit(d, __ballot(valid));                                       \
            rank[k] = count_below(m);                                                                 \
            lead[k] = valid ? (uint32_t)__builtin_ctzll(m) : (uint32_t)lane;                          \
            old[k] = valid ? (uint32_t)__popcll(m) : 0u; /* count, replaced by the atomic's result */ \
        }                                                                                             \
        _Pragma("unroll") for (int k = 0; k < (NI); ++k) {                                            \
            const uint32_t idx = base + k * 64;                                                       \
            const bool valid = PREFIX ? ((keepm >> k) & 1u) != 0 : idx < n;                           \
            if (valid && lead[k] == (uint32_t)lane)                                                   \
                old[k] = atomicAdd(&s_cnt[wid][digit_of<false>(kk[k], shift)], old[k]);                 \
        }                                                                                             \
        _Pragma("unroll") for (int k = 0; k < (NI); ++k) rank[k] +=                                   \
            (uint32_t)__builtin_amdgcn_ds_bpermute((int)(lead[k] << 2), (int)old[k]);                 \
    } while (0)
    if (!PREFIX) GS_RANK_ITEMS(IT);
    else if (nit <= IT / 4) GS_RANK_ITEMS(IT / 4);  // uniform
    else if (nit <= IT / 2) GS_RANK_ITEMS(IT / 2);
    else GS_RANK_ITEMS(IT);
#undef GS_RANK_ITEMS
    __syncthreads();
    {
        const int d = threadIdx.x;  // one thread per digit (threads >= 256 contribute zeros)
        const bool dig = d < kRadix;
        uint32_t tot = 0;
        if (dig) {
#pragma unroll
            for (int w = 0; w < kWaves; ++w) {
                const uint32_t c = s_cnt[w][d];
                s_cnt[w][d] = tot;
                tot += c;
            }
        }
        uint32_t tile_kept;
        const uint32_t start = block_excl_scan_tot<W>(tot, s_wave, &tile_kept);
        const uint32_t gdig = block_excl_scan<W>(dig ? row_total[d] : 0u, s_wave);  // digit base, whole array
        if (PREFIX && threadIdx.x == 0) s_tile_n = tile_kept;
        if (dig) {
            s_start[d] = start;
            s_gbase[d] = (int32_t)(gdig + hist[(size_t)d * nb + tile]) - (int32_t)start;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const uint32_t idx = base + k * 64;
        const bool valid = PREFIX ? ((keepm >> k) & 1u) != 0 : idx < n;
        if (valid) {
            const uint32_t d = digit_of<false>(kk[k], shift);
            const uint32_t pos = s_start[d] + s_cnt[wid][d] + rank[k];
            s_keys[pos] = kk[k];
            if (FMT != kPackIn) s_vals[pos] = vv[k];
        }
    }
    __syncthreads();
    const uint32_t tile_n = PREFIX ? s_tile_n : min((uint32_t)kTile, n - tile0);
    if (FMT == kPlace && GS_DRAW_SBOX && pre.box_out) {  // uniform
        // the placed values' cull boxes too (GS_DRAW_SBOX): every item's box gather in flight
        // before any is stored (a gather per loop trip waited one memory latency each)
        uint2 bx[IT];
        uint32_t at[IT];
        const uint32_t idmax = (uint32_t)max(pre.n - 1, 0);
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const uint32_t i = threadIdx.x + (uint32_t)(k * kThreads);
            const bool ok = i < tile_n;
            const uint32_t ii = ok ? i : 0u;
            const uint32_t key = s_keys[ii];
            const uint32_t o = (uint32_t)(s_gbase[digit_of<false>(key, shift)] + (int32_t)ii);
            const uint32_t id = s_vals[ii];
            at[k] = ok ? (uint32_t)((int32_t)o + s_cls[key_class(key)]) : 0xffffffffu;
            bx[k] = pre.cullbox[min(id, idmax)];
            if (ok) vout[at[k]] = id;
        }
#pragma unroll
        for (int k = 0; k < IT; ++k)
            if (at[k] != 0xffffffffu) pre.box_out[at[k]] = bx[k];
        return;
    }
    for (uint32_t i = threadIdx.x; i < tile_n; i += kThreads) {
        const uint32_t key = s_keys[i];
        const uint32_t d = digit_of<false>(key, shift);
        const uint32_t o = (uint32_t)(s_gbase[d] + (int32_t)i);
        if (FMT == kPairs) {
            kout[o] = key;
            vout[o] = s_vals[i];
        } else if (FMT == kPlace) {
            vout[(uint32_t)((int32_t)o + s_cls[key_class(key)])] = s_vals[i];
        } else if (FMT == kPackOut) {
            kout[o] = (key & 0xff000000u) | s_vals[i];
        } else {
            vout[o] = key & 0x00ffffffu;
        }
    }
}

// ------------------------------------------------------------ small sorts (few tiles)
// A frame with few entries (C2: 51k; the small C5 views: 0.2-1M) is latency-bound: each of the
// 12 launches of the reduce-then-scan sort costs ~4-10 us of dispatch and memory round trips
// for a handful of workgroups.  The small form runs 8: per pass the histogram (k_upsweep) and
// one k_sweep_small, which computes its tile's digit offsets itself from the pass's histogram
// rows (thread d sums row d: its total, and its tiles before this one; a block scan of the
// totals gives the digit bases) -- k_scan_rows' work, O(tiles) reads per thread, cheap for few
// tiles -- then ranks and scatters like k_downsweep.  (Counting the next pass's histogram in
// the sweep with global atomics instead of an upsweep launch was measured: the top-byte pass's
// few digits put ~800 cross-XCD atomics on each counter, 0.45 ms for the 51k-entry C2 sort.)
// Any entry count is sorted correctly; the host picks this form for frames whose previous count
// was small (kSmallSortEntries).  Tiles of 4096 keys (4 waves).
// BKT: the bucket sort's first pass (digit = bucket_of(key)); the workgroup of tile 0 also writes
// each bucket's (base, count) to bkt[d], bkt[256 + d] for k_bucket_sort.
template <bool BKT, int IT = kItems>
__global__ __launch_bounds__(kWaveSmall * 64) void k_sweep_small(const uint32_t *__restrict__ kin,
                                                               const uint32_t *__restrict__ vin,
                                                               uint32_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                               uint32_t n_max, const uint32_t *__restrict__ cnt,
                                                               int shift, const uint32_t *__restrict__ hist, uint32_t nb,
                                                               uint32_t dup_base, uint32_t *__restrict__ tile_counts,
                                                               uint32_t *__restrict__ bins, uint32_t *__restrict__ bkt) {
    constexpr int kThreads = kWaveSmall * 64, kTile = kThreads * IT, kWaves = kWaveSmall;
    static_assert(kThreads == kRadix, "one thread per digit");
    __shared__ uint32_t s_w[4];
    if (bins && blockIdx.x == gridDim.x - 1) {  // uniform: the bins workgroup (first pass)
        __shared__ uint32_t s_above;
        __shared__ __attribute__((aligned(16))) uint32_t s_c[kRadix];
        bins_scan(tile_counts, bins, s_w, &s_above, s_c);
        return;
    }
    const uint32_t n = elem_count(n_max, cnt);
    const uint32_t live = (n + kTile - 1) / kTile;
    const uint32_t tile = blockIdx.x;
    if (BKT && live == 0 && tile == 0) {  // no keys: every bucket empty (k_bucket_sort reads the table)
        bkt[threadIdx.x] = 0u;
        bkt[kRadix + threadIdx.x] = 0u;
    }
    if (tile >= live) return;  // uniform
    __shared__ uint32_t s_cnt[kWaves][kRadix];
    __shared__ uint32_t s_start[kRadix];
    __shared__ int32_t s_gbase[kRadix];
    __shared__ uint32_t s_wave[kWaves];
    __shared__ uint32_t s_keys[kTile];
    __shared__ uint32_t s_vals[kTile];
    for (int i = threadIdx.x; i < kWaves * kRadix; i += kThreads) (&s_cnt[0][0])[i] = 0;
    __syncthreads();
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    const uint32_t tile0 = tile * (uint32_t)kTile;
    const uint32_t base = tile0 + wid * (uint32_t)(64 * IT) + lane;
    uint32_t kk[IT], vv[IT];
    {
        const uint32_t v0 = dup_base != kNoSplit ? cnt[0] : 0xffffffffu, gap = dup_base - v0;
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const uint32_t idx = base + k * 64;
            const uint32_t a = split_at(idx, v0, gap);
            kk[k] = (idx < n) ? kin[a] : 0u;
            vv[k] = (idx < n) ? vin[a] : 0u;
        }
    }
    // the digit offsets, while the keys load: thread d sums hist row d (the tiles before this one,
    // and all of them)
    // (rows are nb words, nb a multiple of 4: 16-byte loads, 64 tiles per round trip)
    const int d = threadIdx.x;
    uint32_t before = 0, total = 0;
    {
        const uint4 *row = reinterpret_cast<const uint4 *>(hist + (size_t)d * nb);
        for (uint32_t j = 0; j < live; j += 64) {
            uint4 v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = (j + 4 * q < live) ? row[(j >> 2) + q] : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const uint32_t t0 = j + 4 * q;
                const uint32_t c[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t x = (t0 + r < live) ? c[r] : 0u;  // columns of tiles past the count are stale
                    total += x;
                    before += (t0 + r < tile) ? x : 0u;
                }
            }
        }
    }
    uint32_t rank[IT], lead[IT], old[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const bool valid = base + k * 64 < n;
        const uint32_t dg = digit_of<BKT>(kk[k], shift);
        const uint64_t m = match_digit(dg, __ballot(valid));
        rank[k] = count_below(m);
        lead[k] = valid ? (uint32_t)__builtin_ctzll(m) : (uint32_t)lane;
        old[k] = valid ? (uint32_t)__popcll(m) : 0u;
    }
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const bool valid = base + k * 64 < n;
        if (valid && lead[k] == (uint32_t)lane) old[k] = atomicAdd(&s_cnt[wid][digit_of<BKT>(kk[k], shift)], old[k]);
    }
#pragma unroll
    for (int k = 0; k < IT; ++k) rank[k] += (uint32_t)__builtin_amdgcn_ds_bpermute((int)(lead[k] << 2), (int)old[k]);
    __syncthreads();
    {
        uint32_t tot = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            const uint32_t c = s_cnt[w][d];
            s_cnt[w][d] = tot;
            tot += c;
        }
        const uint32_t start = block_excl_scan<kWaves>(tot, s_wave);
        const uint32_t gdig = block_excl_scan<kWaves>(total, s_wave);  // digit base, whole array
        s_start[d] = start;
        s_gbase[d] = (int32_t)(gdig + before) - (int32_t)start;
        if (BKT && tile == 0) {
            bkt[d] = gdig;
            bkt[kRadix + d] = total;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        if (base + k * 64 < n) {
            const uint32_t dg = digit_of<BKT>(kk[k], shift);
            const uint32_t pos = s_start[dg] + s_cnt[wid][dg] + rank[k];
            s_keys[pos] = kk[k];
            s_vals[pos] = vv[k];
        }
    }
    __syncthreads();
    const uint32_t tile_n = min((uint32_t)kTile, n - tile0);
    for (uint32_t i = threadIdx.x; i < tile_n; i += kThreads) {
        const uint32_t key = s_keys[i];
        const uint32_t o = (uint32_t)(s_gbase[digit_of<BKT>(key, shift)] + (int32_t)i);
        kout[o] = key;
        vout[o] = s_vals[i];
    }
}

// Stable ranks of one tile of up to 256 * IT keys held as k_sweep_small holds them (4 waves:
// wave w, item k, lane l is position w*64*IT + k*64 + l; valid below tn): ps[k] = the item's place in the
// tile's order by digit (key >> shift) & 0xff; s_tdig[d] = the tile's count of digit d, and
// s_start[d] its first place.  Starts and ends with a barrier.
template <int IT>
__device__ __forceinline__ void rank_tile(const uint32_t (&kk)[IT], uint32_t tn, int shift, uint32_t (&ps)[IT],
                                          uint32_t (*s_cnt)[kRadix], uint32_t *s_start, uint32_t *s_wave,
                                          uint32_t *s_tdig) {
    const int lane = lane_id(), wid = threadIdx.x >> 6, d = threadIdx.x;
    __syncthreads();  // the previous use of the scratch is done
#pragma unroll
    for (int w = 0; w < kWaveSmall; ++w) s_cnt[w][d] = 0;
    __syncthreads();
    const uint32_t base = wid * (uint32_t)(64 * IT) + lane;
    uint32_t rank[IT], lead[IT], old[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const bool valid = base + k * 64 < tn;
        const uint64_t m = match_digit((kk[k] >> shift) & 0xffu, __ballot(valid));
        rank[k] = count_below(m);
        lead[k] = valid ? (uint32_t)__builtin_ctzll(m) : (uint32_t)lane;
        old[k] = valid ? (uint32_t)__popcll(m) : 0u;
    }
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const bool valid = base + k * 64 < tn;
        if (valid && lead[k] == (uint32_t)lane) old[k] = atomicAdd(&s_cnt[wid][(kk[k] >> shift) & 0xffu], old[k]);
    }
#pragma unroll
    for (int k = 0; k < IT; ++k) rank[k] += (uint32_t)__builtin_amdgcn_ds_bpermute((int)(lead[k] << 2), (int)old[k]);
    __syncthreads();
    uint32_t tot = 0;
#pragma unroll
    for (int w = 0; w < kWaveSmall; ++w) {
        const uint32_t c = s_cnt[w][d];
        s_cnt[w][d] = tot;
        tot += c;
    }
    s_tdig[d] = tot;
    s_start[d] = block_excl_scan<kWaveSmall>(tot, s_wave);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const uint32_t dg = (kk[k] >> shift) & 0xffu;
        ps[k] = s_start[dg] + s_cnt[wid][dg] + rank[k];
    }
    __syncthreads();
}

// The bucket sort's second kernel: bucket b = [bkt[b], + bkt[256 + b]) of (kin, vin), in input
// order within the bucket (k_sweep_small<true>), stably sorted by key into the same positions
// of (kout, vout).  The keys of a bucket agree above the highest bit where its smallest and
// largest differ, so LSD passes over the bits below it (8 per pass: tile 0's depths up to 4,
// a tile >= 128's keys 2) order it completely.  Buckets of <= 4096 keys sort in registers and
// LDS; longer ones (rare: a tile list that long in a frame this small) take the same passes
// through global memory in 4096-key tiles, ping-ponging between the two arrays' bucket ranges.
// the bits of a bucket that vary (the smallest and largest key of it, over the workgroup; kk: each
// thread's keys, invalid ones neutral) -> the LSD passes needed
template <int IT>
__device__ __forceinline__ int bucket_passes(const uint32_t (&kmin)[IT], const uint32_t (&kmax)[IT], uint32_t (*s_mm)[kWaveSmall]) {
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    uint32_t mn = 0xffffffffu, mx = 0u;
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        mn = min(mn, kmin[k]);
        mx = max(mx, kmax[k]);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
    }
    if (lane == 0) {
        s_mm[0][wid] = mn;
        s_mm[1][wid] = mx;
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < kWaveSmall; ++w) {
        mn = min(mn, s_mm[0][w]);
        mx = max(mx, s_mm[1][w]);
    }
    const uint32_t diff = mn ^ mx;
    return diff ? (32 - __builtin_clz(diff) + 7) / 8 : 0;
}

// a bucket of m <= 256 * IT keys: registers and LDS (s_k, s_v hold 256 * IT)
template <int IT>
__device__ __forceinline__ void bucket_fast(const uint32_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                            uint32_t *__restrict__ kout, uint32_t *__restrict__ vout, uint32_t b0,
                                            uint32_t m, uint32_t *s_k, uint32_t *s_v, uint32_t (*s_cnt)[kRadix],
                                            uint32_t *s_start, uint32_t *s_wave, uint32_t *s_tdig,
                                            uint32_t (*s_mm)[kWaveSmall]) {
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    const uint32_t base = wid * (uint32_t)(64 * IT) + lane;
    uint32_t kk[IT], vv[IT], ps[IT], kmn[IT], kmx[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const uint32_t pos = base + k * 64;
        kk[k] = pos < m ? kin[b0 + pos] : 0u;
        vv[k] = pos < m ? vin[b0 + pos] : 0u;
    }
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const bool ok = base + k * 64 < m;
        kmn[k] = ok ? kk[k] : 0xffffffffu;
        kmx[k] = ok ? kk[k] : 0u;
    }
    const int passes = bucket_passes<IT>(kmn, kmx, s_mm);
    for (int p = 0; p < passes; ++p) {
        rank_tile<IT>(kk, m, 8 * p, ps, s_cnt, s_start, s_wave, s_tdig);
#pragma unroll
        for (int k = 0; k < IT; ++k)
            if (base + k * 64 < m) {
                s_k[ps[k]] = kk[k];
                s_v[ps[k]] = vv[k];
            }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const uint32_t pos = base + k * 64;
            kk[k] = pos < m ? s_k[pos] : 0u;
            vv[k] = pos < m ? s_v[pos] : 0u;
        }
    }
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const uint32_t pos = base + k * 64;
        if (pos < m) {
            kout[b0 + pos] = kk[k];
            vout[b0 + pos] = vv[k];
        }
    }
}

// (bins != null: one more workgroup, the last, scans the frame's tile counts into the bins --
// here rather than beside the scatter, whose duration it set at C2)
__global__ __launch_bounds__(kWaveSmall * 64) void k_bucket_sort(uint32_t *__restrict__ kin, uint32_t *__restrict__ vin,
                                                               uint32_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                               const uint32_t *__restrict__ bkt,
                                                               uint32_t *__restrict__ tile_counts,
                                                               uint32_t *__restrict__ bins, uint32_t cap) {
    static_assert(kWaveSmall * 64 == kRadix, "one thread per digit");
    constexpr uint32_t kTile = kTileSmall;
    if (bins && blockIdx.x == kRadix) {  // uniform: the bins workgroup
        __shared__ uint32_t s_w[4], s_above;
        __shared__ __attribute__((aligned(16))) uint32_t s_c[kRadix];
        bins_scan(tile_counts, bins, s_w, &s_above, s_c);
        return;
    }
    __shared__ uint32_t s_k[kTile], s_v[kTile];
    __shared__ uint32_t s_cnt[kWaveSmall][kRadix];
    __shared__ uint32_t s_start[kRadix], s_tdig[kRadix], s_run[kRadix];
    __shared__ uint32_t s_wave[kWaveSmall];
    __shared__ uint32_t s_mm[2][kWaveSmall];
    // (the table is the sweep's; a bucket is still held inside the arrays' n = cap entries, so a
    // table that is not this sort's can misorder a frame but never reach past its arrays)
    const uint32_t b0 = bkt[blockIdx.x], m = min(bkt[kRadix + blockIdx.x], cap - min(b0, cap));
    if (m == 0) return;  // uniform
    // (uniform) short buckets with 4 keys per lane, up to 4096 with 16
    if (m <= kTile / 4) return bucket_fast<kItems / 4>(kin, vin, kout, vout, b0, m, s_k, s_v, s_cnt, s_start, s_wave, s_tdig, s_mm);
    if (m <= kTile) return bucket_fast<kItems>(kin, vin, kout, vout, b0, m, s_k, s_v, s_cnt, s_start, s_wave, s_tdig, s_mm);
    const int lane = lane_id(), wid = threadIdx.x >> 6, d = threadIdx.x;
    int passes;
    {
        uint32_t mn[1] = {0xffffffffu}, mx[1] = {0u};
        for (uint32_t i = threadIdx.x; i < m; i += kRadix) {
            const uint32_t k = kin[b0 + i];
            mn[0] = min(mn[0], k);
            mx[0] = max(mx[0], k);
        }
        passes = bucket_passes<1>(mn, mx, s_mm);
    }
    const uint32_t base = wid * (uint32_t)kWaveTile + lane;
    uint32_t kk[kItems], vv[kItems], ps[kItems];
    // long bucket: LSD passes through global memory, 4096-key tiles in order
    uint32_t *sk = kin, *sv = vin, *dk = kout, *dv = vout;
    for (int p = 0; p < passes; ++p) {
        const int shift = 8 * p;
        s_run[d] = 0;
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < m; i += kRadix) atomicAdd(&s_run[(sk[b0 + i] >> shift) & 0xffu], 1u);
        __syncthreads();
        {
            const uint32_t c = s_run[d];
            const uint32_t ex = block_excl_scan<kWaveSmall>(c, s_wave);
            s_run[d] = ex;  // (each thread its own digit)
        }
        for (uint32_t t0 = 0; t0 < m; t0 += kTile) {
            const uint32_t tn = min(kTile, m - t0);
#pragma unroll
            for (int k = 0; k < kItems; ++k) {
                const uint32_t pos = base + k * 64;
                kk[k] = pos < tn ? sk[b0 + t0 + pos] : 0u;
                vv[k] = pos < tn ? sv[b0 + t0 + pos] : 0u;
            }
            rank_tile<kItems>(kk, tn, shift, ps, s_cnt, s_start, s_wave, s_tdig);
#pragma unroll
            for (int k = 0; k < kItems; ++k)
                if (base + k * 64 < tn) {
                    const uint32_t dg = (kk[k] >> shift) & 0xffu;
                    const uint32_t o = b0 + s_run[dg] + (ps[k] - s_start[dg]);
                    dk[o] = kk[k];
                    dv[o] = vv[k];
                }
            __syncthreads();
            s_run[d] += s_tdig[d];
        }
        // the pass's stores before the next pass's loads by the other waves (agent-scope
        // release / acquire: the acquire invalidates this CU's vector L1)
        __threadfence();
        __syncthreads();
        __threadfence();
        uint32_t *t = sk;
        sk = dk;
        dk = t;
        t = sv;
        sv = dv;
        dv = t;
    }
    if (sk != kout)  // uniform: an even number of passes left the bucket in (kin, vin)
        for (uint32_t i = threadIdx.x; i < m; i += kRadix) {
            kout[b0 + i] = kin[b0 + i];
            vout[b0 + i] = vin[b0 + i];
        }
}

// The prefix sort's class bounds (one workgroup of 256 per tile class; thread j owns buckets
// [8j, 8j + 8) of every copy): walking the sampled histogram from the largest distance (the
// front of the list) down, the bucket where the count reaches target / kPrefixSample sets
// theta = the class bound - that bucket's smallest distance; a class sampled less keeps every
// key.  The histogram is cleared for the next frame.
__global__ __launch_bounds__(256) void k_prefix_select(PrefixDev pre, TileRects tr, int use_rects) {
    constexpr int kB = kPrefixBuckets / 256;  // buckets per thread (8)
    __shared__ uint32_t s_w[4];
    __shared__ uint32_t s_dep;
    const uint32_t c = blockIdx.x, j = threadIdx.x;
    static_assert(kB == 8, "prefix_slot puts bucket 8j + k at word k * (kPrefixBuckets / 8) + j");
    uint32_t v[kB] = {};
    // a frame whose camera turned since the frame before (use_depth 0): the depths were recorded at
    // other poses, where this tile's content sat elsewhere -- class c takes the deepest depth of the
    // tiles it came from (tr: the camera's rotation maps the tile there, host side; content from
    // outside those views: the configured target), or without them of its 3 x 3 neighbourhood
    const uint32_t own = pre.depth ? pre.depth[c] : 0u;
    uint32_t dep_nb = 0;
    if (pre.depth && !pre.use_depth && use_rects) {  // uniform
        const uint32_t r = (tr.w[c >> 1] >> (16u * (c & 1u))) & 0xffffu;
        if (j == 0) s_dep = 0;
        __syncthreads();
        const uint32_t x = j & 15u, y = j >> 4;
        if (r != kRectUnknown && x >= (r & 15u) && x <= ((r >> 4) & 15u) && y >= ((r >> 8) & 15u) && y <= (r >> 12))
            atomicMax(&s_dep, pre.depth[j]);
        __syncthreads();
        dep_nb = r == kRectUnknown ? 0u : s_dep;  // (0: the target)
    } else if (pre.depth && GS_PREFIX_TURN_NB && !pre.use_depth) {
        const int tx = (int)(c & 15u), ty = (int)(c >> 4);
        constexpr int ry = GS_PREFIX_TURN_NB == 3 ? 0 : 1;  // (3: the row neighbours only)
#pragma unroll
        for (int dy = -ry; dy <= ry; ++dy)
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx) {
                const int x = tx + dx, y = ty + dy;
                if (x >= 0 && x < 16 && y >= 0 && y < 16) dep_nb = max(dep_nb, pre.depth[y * 16 + x]);
            }
    }
    // (the source rectangles: GS_PREFIX_RECT_SLACK x the slack; the 3 x 3 neighbourhood: twice it)
    const uint32_t slack_nb = use_rects ? GS_PREFIX_RECT_SLACK * kPrefixDepthSlack
                                        : (GS_PREFIX_TURN_NB == 1 ? 2 * kPrefixDepthSlack : kPrefixDepthSlack) * GS_PREFIX_TURN_SLACK_MUL;
#pragma unroll
    for (int cp = 0; cp < kPrefixHistCopies; ++cp) {
        uint32_t *h = pre.hist + ((size_t)cp * 256 + c) * kPrefixBuckets;
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            v[k] += h[prefix_slot(kB * j + k)];
            h[prefix_slot(kB * j + k)] = 0;
        }
    }
    uint32_t a = 0;
#pragma unroll
    for (int k = 0; k < kB; ++k) a += v[k];
    uint32_t tot;
    const uint32_t ex = block_excl_scan_tot<4>(a, s_w, &tot);
    const uint32_t above = tot - ex - a;  // samples in the buckets of the higher threads
    // the class's target: the configured one, or less where recent blends read the list
    // shallowly (the depth words were read before the scan's barriers; the decay written after)
    auto target_of = [&](uint32_t dep, uint32_t slack, uint32_t mul) { return dep ? min(pre.target, mul * dep + slack) : pre.target; };
    // (decayed by a CAS loop on the current word, not a store of own - own / 16: with frames in
    // flight another lane's blend may have raised it since it was read, and a plain store would
    // drop that maximum)
    if (pre.depth && j == 0 && own) {  // (every prefix-sorted frame decays its class's own depth)
        uint32_t cur = own;
        for (int tries = 0; tries < 16; ++tries) {
            const uint32_t seen = atomicCAS(&pre.depth[c], cur, cur - (cur >> 4));
            if (seen == cur) break;
            cur = seen;
        }
    }
    const uint32_t hi = class_hi(c);
    auto select = [&](uint32_t *theta, uint32_t target) {
        const uint32_t tgt = (target + kPrefixSample - 1) / kPrefixSample;
        if (c == 0 && j == 0) theta[256] = 0xffffffffu;  // class 256 is kept whole
        if (target == 0 || tot < tgt) {
            if (j == 0) theta[c] = hi - 1u;  // the whole class
            return;
        }
        if (above < tgt && above + a >= tgt) {
            uint32_t cum = above, b = 0;
            bool found = false;
#pragma unroll
            for (int k = kB - 1; k >= 0; --k) {
                cum += v[k];
                if (!found && cum >= tgt) {
                    b = kB * j + (uint32_t)k;
                    found = true;
                }
            }
            theta[c] = hi - prefix_bucket_dmin(b);
        }
    };
    if (pre.use_depth)
        select(pre.theta, target_of(own, kPrefixDepthSlack, 2u));
    else
        select(pre.theta, target_of(dep_nb, slack_nb, GS_PREFIX_TURN_MUL));
}

__global__ __launch_bounds__(256) void k_gather_keys(const float *__restrict__ keys, const int32_t *__restrict__ order,
                                                     uint32_t *__restrict__ kout, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) kout[i] = __float_as_uint(keys[order[i]]);
}

}  // namespace

int sort_ensure(SortScratch &sc, int64_t n, std::string &err, hipStream_t s, bool small) {
    // the most tiles of any pass (the small form keeps all four passes' histograms)
    // (small: the bucket pass's 1024-key tiles)
    // (and a prefix sort's passes 1-3: kSubItems keys per lane)
    const size_t tsz = small ? kTileSmall / 4 : std::min(kTileSmall, kWaveSmall * 64 * kSubItems);
    const size_t nb = (size_t)((n + tsz - 1) / tsz) + 3;  // (+3: the small form's 16-byte rows)
    const bool grow_alt = (size_t)n > sc.alt_cap, grow_hist = nb * kRadix > sc.hist_cap;
    if ((grow_alt && sc.keys_alt) || (grow_hist && sc.hist)) (void)hipStreamSynchronize(s);  // in-flight users
    if (grow_alt) {
        if (sc.keys_alt) (void)hipFree(sc.keys_alt);
        if (sc.vals_alt) (void)hipFree(sc.vals_alt);
        sc.keys_alt = sc.vals_alt = nullptr;
        sc.alt_cap = 0;
        const size_t cap = (size_t)n + (size_t)n / 4 + 4096;
        if (hipMalloc(&sc.keys_alt, cap * 4) != hipSuccess || hipMalloc(&sc.vals_alt, cap * 4) != hipSuccess) {
            err = "radix sort: out of device memory";
            return GS_ERR_NOMEM;
        }
        sc.alt_cap = cap;
    }
    if (grow_hist) {
        if (sc.hist) (void)hipFree(sc.hist);
        sc.hist = nullptr;
        const size_t cap = (nb + nb / 4 + 16) * kRadix;
        if (hipMalloc(&sc.hist, cap * 4) != hipSuccess) {
            err = "radix sort: out of device memory";
            return GS_ERR_NOMEM;
        }
        sc.hist_cap = cap;
    }
    if (!sc.bkt) {  // the bucket form's (base, count) table, zeroed: a sort of no keys reads it as empty
        if (hipMalloc(&sc.bkt, 2 * kRadix * 4) != hipSuccess || hipMemsetAsync(sc.bkt, 0, 2 * kRadix * 4, s) != hipSuccess) {
            err = "radix sort: out of device memory";
            return GS_ERR_NOMEM;
        }
    }
    if (!sc.row_total) {  // row totals [256] + tile counts [16][256] + above-1e6 counts [16] (zero between sorts)
        const size_t bytes = ((size_t)(1 + kTileCopies) * kRadix + kTileCopies) * 4;
        if (hipMalloc(&sc.row_total, bytes) != hipSuccess || hipMemsetAsync(sc.row_total, 0, bytes, s) != hipSuccess) {
            err = "radix sort: out of device memory";
            return GS_ERR_NOMEM;
        }
    }
    return GS_OK;
}

void sort_free(SortScratch &sc) {
    if (sc.keys_alt) (void)hipFree(sc.keys_alt);
    if (sc.vals_alt) (void)hipFree(sc.vals_alt);
    if (sc.hist) (void)hipFree(sc.hist);
    if (sc.row_total) (void)hipFree(sc.row_total);
    if (sc.bkt) (void)hipFree(sc.bkt);
    sc = SortScratch{};
}

int sort_pairs(hipStream_t s, SortScratch &sc, uint32_t *keys, uint32_t *vals, int64_t n, std::string &err,
               const uint32_t *dev_count, hipEvent_t start, hipEvent_t stop, uint32_t *bins, bool keys_out,
               const PrefixDev *pre, int64_t dup_base, bool small, bool bucket, const KeptSort *kept) {
    if (kept && (!pre || dup_base >= 0)) {
        err = "radix sort: a kept emission needs the prefix sort and the contiguous layout";
        return GS_ERR_INVALID;
    }
    if (dup_base >= 0 && !dev_count) {
        err = "radix sort: the split layout needs a device count";
        return GS_ERR_INVALID;
    }
    small = small && !pre && n >= 1;
    bucket = bucket && small;
    if (pre && (!bins || !dev_count)) {
        err = "radix sort: a prefix sort needs bins and a device count";
        return GS_ERR_INVALID;
    }
    if (((n <= 1 && !dev_count) || n < 1) && !bins) {  // nothing to sort; the events still mark the call
        if (start) (void)hipEventRecord(start, s);
        if (stop) (void)hipEventRecord(stop, s);
        return GS_OK;
    }
    if (n >= (int64_t)1 << 31) {
        err = "radix sort: n must be < 2^31";
        return GS_ERR_INVALID;
    }
    int rc = sort_ensure(sc, std::max<int64_t>(n, 1), err, s, small);
    if (rc) return rc;
    uint32_t *tile_counts = sc.row_total + kRadix;
    if (n < 1 && !dev_count) {  // no keys: the (zero) bins only
        if (start) (void)hipEventRecord(start, s);
        hipLaunchKernelGGL(k_scan_rows<>, dim3(kRadix + 1), dim3(256), 0, s, sc.hist, 0u, 0u, nullptr, 1u, sc.row_total,
                           tile_counts, bins, PrefixDev{}, 0);
        if (stop) (void)hipEventRecord(stop, s);
        return hipGetLastError() == hipSuccess ? GS_OK : GS_ERR_HIP;
    }
    if (small) {  // the small form (k_sweep_small): 8 launches, keys and values out
        // (the bucket pass of up to 192k keys -- n is the capacity for a frame counted on the
        // device -- in 1024-key tiles: 4x the workgroups, each a quarter of the serial work; above
        // that the per-workgroup reads of the histogram rows, O(tiles), outweigh it: C5 view 2,
        // 383k keys, sort 0.043 -> 0.056 ms)
        const bool t1k = bucket && n <= (192 << 10);
        const uint32_t tsz = t1k ? kTileSmall / 4 : kTileSmall;
        const uint32_t nb = (uint32_t)((n + tsz - 1) / tsz + 3) & ~3u;  // row stride: 16-byte rows
        const uint32_t split = dup_base >= 0 ? (uint32_t)dup_base : kNoSplit;
        uint32_t *kin = keys, *vin = vals, *kout = sc.keys_alt, *vout = sc.vals_alt;
        for (int pass = 0; pass < 4; ++pass) {
            const uint32_t sp = pass == 0 ? split : kNoSplit;
            hipEvent_t e0 = pass == 0 ? start : nullptr, e1 = pass == 3 ? stop : nullptr;
            // the bucket form: pass 0 scatters by bucket (tile), then one k_bucket_sort finishes
            // every bucket (3 launches in all)
            const bool bk = bucket && pass == 0;
            auto up = pass == 0 && bins
                          ? (bk ? (t1k ? k_upsweep<kWaveSmall, true, false, true, kItems / 4> : k_upsweep<kWaveSmall, true, false, true>)
                                : k_upsweep<kWaveSmall, true>)
                          : (bk ? (t1k ? k_upsweep<kWaveSmall, false, false, true, kItems / 4> : k_upsweep<kWaveSmall, false, false, true>)
                                : k_upsweep<kWaveSmall, false>);
            hipExtLaunchKernelGGL(up, dim3(xcd_grid(nb)), dim3(kWaveSmall * 64), 0, s, e0, nullptr, 0, kin, (uint32_t)n,
                                  dev_count, 8 * pass, sc.hist, nb, pass == 0 && bins ? tile_counts : nullptr, PrefixDev{}, sp);
            const dim3 grid(nb + ((pass == 0 && bins && !bk) ? 1 : 0));
            auto sw = bk ? (t1k ? k_sweep_small<true, kItems / 4> : k_sweep_small<true>) : k_sweep_small<false>;
            hipExtLaunchKernelGGL(sw, grid, dim3(kWaveSmall * 64), 0, s, nullptr, bk ? nullptr : e1, 0, kin, vin, kout, vout,
                                  (uint32_t)n, dev_count, 8 * pass, sc.hist, nb, sp, tile_counts,
                                  pass == 0 && !bk ? bins : nullptr, sc.bkt);
            if (bk) {  // (alt -> keys: the result is where the 4-pass form leaves it)
                hipExtLaunchKernelGGL(k_bucket_sort, dim3(kRadix + (bins ? 1 : 0)), dim3(kWaveSmall * 64), 0, s, nullptr, stop, 0,
                                      kout, vout, kin, vin, sc.bkt, tile_counts, bins, (uint32_t)n);
                break;
            }
            std::swap(kin, kout);
            std::swap(vin, vout);
        }
        if (hipGetLastError() != hipSuccess) {
            err = "radix sort: kernel launch failed";
            return GS_ERR_HIP;
        }
        return GS_OK;
    }
    uint32_t *kin = keys, *vin = vals, *kout = sc.keys_alt, *vout = sc.vals_alt;
    PrefixDev pd = pre ? *pre : PrefixDev{};
    pd.frame_count = dev_count;
    pd.cap_all = (uint32_t)n;
    const int64_t n_sub = pre ? std::min<int64_t>(n, pre->cap_sel) : n;  // passes 1-3 of a prefix sort
    // a kept emission's input (kept->count set); else kept->after_select alone (see KeptSort)
    const bool kept_in = kept && kept->count;
    if (pre) {  // the class bounds from the keys the emission sampled (kept: the next frame's)
        hipExtLaunchKernelGGL(k_prefix_select, dim3(256), dim3(256), 0, s, start, nullptr, 0, pd,
                              pd.rects ? *pd.rects : TileRects{}, pd.rects ? 1 : 0);
        start = nullptr;
    }
    // passes 1-3 in the pass-0 form (8 waves, 8192-key tiles) too for sorts of 16M keys or more:
    // 64M pairs, downsweep 272 -> 232 us and upsweep 75 -> 54 us per pass (a frame's kept keys,
    // ~2M, ran 3 % slower that way; 12- and 16-wave tiles spill: 2.8 / 3.5 ms against 1.20)
    // (standalone pair sorts: no bins, pairs out in every pass)
    const bool all_big = !pre && !bins && keys_out && n >= (int64_t)1 << 24;
#ifndef GS_UPSWEEP_REV
#define GS_UPSWEEP_REV 1
#endif
    for (int pass = 0; pass < 4; ++pass) {
        const int shift = 8 * pass;
        // (a kept emission's first pass reads only the kept keys: the passes-1-3 form and sizes)
        const bool big = (pass == 0 && !kept_in) || all_big;
        // (a prefix sort's first pass keeps ~1 key in 8: its tiles of kP0Waves waves)
        const bool p0 = big && pre && !kept_in;
        // (a prefix sort's passes on the kept keys: kSubItems keys per lane)
        const bool sub = pre && !big;
        const uint32_t tile = p0 ? kP0Waves * kWaveTile : big ? kWaveBig * kWaveTile : sub ? kWaveSmall * 64 * kSubItems : kTileSmall;
        // a prefix sort's passes 1-3 run on the kept keys (their count on the device, at most n_sub)
        const uint32_t *cnt = pre && pass > 0 ? pre->nsel : kept_in ? kept->count : dev_count;
        const int64_t np = pass > 0 || kept_in ? n_sub : n;
        const uint32_t nb = (uint32_t)((np + tile - 1) / tile);  // tiles of this pass = hist row stride
        // timing events on the first and last dispatch (see launch_preprocess)
        hipEvent_t e0 = pass == 0 ? start : nullptr, e1 = pass == 3 ? stop : nullptr;
        // the first pass reads the split emission layout (dup_base >= 0), the others their own output
        const uint32_t split = (pass == 0 && dup_base >= 0) ? (uint32_t)dup_base : kNoSplit;
        if (p0)
            hipExtLaunchKernelGGL((k_upsweep<kP0Waves, true, true>), dim3(xcd_grid(nb)), dim3(kP0Waves * 64), 0, s, e0, nullptr,
                                  0, kin, (uint32_t)np, cnt, shift, sc.hist, nb, tile_counts, pd, split);
        else if (big && bins && !kept_in)  // (a kept emission counted the tiles itself)
            hipExtLaunchKernelGGL((k_upsweep<kWaveBig, true>), dim3(xcd_grid(nb)), dim3(kWaveBig * 64), 0, s, e0, nullptr, 0,
                                  kin, (uint32_t)np, cnt, shift, sc.hist, nb, tile_counts, pd, split);
        else if (big && all_big && GS_UPSWEEP_REV)  // (standalone sorts of >= 16M keys)
            hipExtLaunchKernelGGL((k_upsweep<kWaveBig, false, false, false, kItems, true>), dim3(xcd_grid(nb)), dim3(kWaveBig * 64),
                                  0, s, e0, nullptr, 0, kin, (uint32_t)np, cnt, shift, sc.hist, nb, nullptr, pd, split);
        else if (big)
            hipExtLaunchKernelGGL((k_upsweep<kWaveBig, false>), dim3(xcd_grid(nb)), dim3(kWaveBig * 64), 0, s, e0, nullptr, 0,
                                  kin, (uint32_t)np, cnt, shift, sc.hist, nb, nullptr, pd, split);
        else if (sub)
            hipExtLaunchKernelGGL((k_upsweep<kWaveSmall, false, false, false, kSubItems>), dim3(xcd_grid(nb)), dim3(kWaveSmall * 64),
                                  0, s, e0, nullptr, 0, kin, (uint32_t)np, cnt, shift, sc.hist, nb, nullptr, pd, kNoSplit);
        else
            hipExtLaunchKernelGGL((k_upsweep<kWaveSmall, false>), dim3(xcd_grid(nb)), dim3(kWaveSmall * 64), 0, s, e0, nullptr,
                                  0, kin, (uint32_t)np, cnt, shift, sc.hist, nb, nullptr, pd, kNoSplit);
        // one more workgroup scans the tile counts in the last pass (a prefix sort: with the draw
        // limits; and one in the first pass makes the class tables passes 1-3 need)
        const bool with_bins = bins && (pass == 3 || (pre && pass == 0));
        const int pmode = !pre ? 0 : pass == 0 ? 1 : 2;
#ifndef GS_SCAN_LIGHT
#define GS_SCAN_LIGHT 1
#endif
#ifndef GS_SCAN_LIGHT_BINS
#define GS_SCAN_LIGHT_BINS 1
#endif
        // (the passes with the bins workgroup in the light form too: 4 counts per thread, and the
        // bins workgroup's LDS shared between its phases -- ~2 KB in all)
        auto scan = with_bins ? (nb > 4096 ? k_scan_rows<64> : GS_SCAN_LIGHT_BINS ? k_scan_rows<4> : k_scan_rows<16>)
                    : nb > 4096  ? k_scan_rows<64, false>
                    : (GS_SCAN_LIGHT && nb <= 1024) ? k_scan_rows<4, false>
                                                    : k_scan_rows<16, false>;
        hipLaunchKernelGGL(scan, dim3(kRadix + (with_bins ? 1 : 0)), dim3(256), 0, s, sc.hist, nb, (uint32_t)np, cnt, tile,
                           sc.row_total, tile_counts, with_bins ? bins : nullptr, pd, pmode);
        // (a kept emission's next frame waits for its bounds, and for this pass's reads of them)
        if (kept_in && pass == 0 && kept->after_select) (void)hipEventRecord(kept->after_select, s);
        // keys_out false: pass 2 packs (top key byte, value), pass 3 unpacks the values only;
        // a prefix sort moves pairs and places the values in its last pass
        const int fmt = pre ? (pass == 3 ? kPlace : kPairs) : keys_out || pass < 2 ? kPairs : pass == 2 ? kPackOut : kPackIn;
        if (p0)
            hipExtLaunchKernelGGL((k_downsweep<kP0Waves, kPairs, true>), dim3(xcd_grid(nb)), dim3(kP0Waves * 64), 0, s, nullptr,
                                  e1, 0, kin, vin, kout, vout, (uint32_t)np, cnt, shift, sc.hist, nb, sc.row_total, pd, split);
        else if (big)
            hipExtLaunchKernelGGL((k_downsweep<kWaveBig, kPairs>), dim3(xcd_grid(nb)), dim3(kWaveBig * 64), 0, s, nullptr, e1, 0,
                                  kin, vin, kout, vout, (uint32_t)np, cnt, shift, sc.hist, nb, sc.row_total, pd, split);
        else if (sub && fmt == kPairs)
            hipExtLaunchKernelGGL((k_downsweep<kWaveSmall, kPairs, false, kSubItems>), dim3(xcd_grid(nb)), dim3(kWaveSmall * 64), 0,
                                  s, nullptr, e1, 0, kin, vin, kout, vout, (uint32_t)np, cnt, shift, sc.hist, nb, sc.row_total, pd, split);
        else if (sub && fmt == kPlace)
            hipExtLaunchKernelGGL((k_downsweep<kWaveSmall, kPlace, false, kSubItems>), dim3(xcd_grid(nb)), dim3(kWaveSmall * 64), 0,
                                  s, nullptr, e1, 0, kin, vin, kout, vout, (uint32_t)np, cnt, shift, sc.hist, nb, sc.row_total, pd, split);
        else if (fmt == kPairs)
            hipExtLaunchKernelGGL((k_downsweep<kWaveSmall, kPairs>), dim3(xcd_grid(nb)), dim3(kWaveSmall * 64), 0, s, nullptr, e1,
                                  0, kin, vin, kout, vout, (uint32_t)np, cnt, shift, sc.hist, nb, sc.row_total, pd, split);
        else if (fmt == kPlace)
            hipExtLaunchKernelGGL((k_downsweep<kWaveSmall, kPlace>), dim3(xcd_grid(nb)), dim3(kWaveSmall * 64), 0, s, nullptr, e1,
                                  0, kin, vin, kout, vout, (uint32_t)np, cnt, shift, sc.hist, nb, sc.row_total, pd, split);
        else if (fmt == kPackOut)
            hipExtLaunchKernelGGL((k_downsweep<kWaveSmall, kPackOut>), dim3(xcd_grid(nb)), dim3(kWaveSmall * 64), 0, s, nullptr,
                                  e1, 0, kin, vin, kout, vout, (uint32_t)np, cnt, shift, sc.hist, nb, sc.row_total, pd, split);
        else
            hipExtLaunchKernelGGL((k_downsweep<kWaveSmall, kPackIn>), dim3(xcd_grid(nb)), dim3(kWaveSmall * 64), 0, s, nullptr,
                                  e1, 0, kin, vin, kout, vout, (uint32_t)np, cnt, shift, sc.hist, nb, sc.row_total, pd, split);
        // (a full emission's first pass kept its keys by the bounds its select wrote: the frame
        // after it, which keeps by the same bounds and then rewrites the other buffer, waits)
        if (kept && !kept_in && pass == 0 && kept->after_select) (void)hipEventRecord(kept->after_select, s);
        std::swap(kin, kout);
        std::swap(vin, vout);
    }
    // 4 (even) passes: the result is back in (keys, vals); without keys_out, keys holds the
    // pass-1 order
    if (hipGetLastError() != hipSuccess) {
        err = "radix sort: kernel launch failed";
        return GS_ERR_HIP;
    }
    return GS_OK;
}

void launch_gather_keys(hipStream_t s, const float *keys, const int32_t *order, uint32_t *kout, int64_t n,
                        hipEvent_t start) {
    const int64_t nb = (n + 255) / 256;
    if (nb > 0)
        hipExtLaunchKernelGGL(k_gather_keys, dim3((unsigned)nb), dim3(256), 0, s, start, nullptr, 0, keys, order, kout,
                              n);
    else if (start)
        (void)hipEventRecord(start, s);
}

}  // namespace gs
