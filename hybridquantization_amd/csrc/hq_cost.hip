// hq_cost.hip -- the S-CIELAB stencil cost of a population (CL:234-306,
// vertical pass first), Opp->Lab (CL:124-145) and dE (CL:201-226) against the
// precomputed LabRef, one fp64 partial per (tile, palette); plus the generic
// two-pass path (any half-width) that cross-checks it.
#include "hq_device.h"
#include "hq_launch.h"

#include <algorithm>
#include <cmath>
#include <type_traits>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>

#ifndef HQ_CHW
#define HQ_CHW 8  // horizontal taps per chunk at HB = 15, 24
#endif
#ifndef HQ_CH19
#define HQ_CH19 6  // horizontal taps per chunk at HB = 19 (6, 8, 13: equal since the pair layout; with the
                   // 32-row layout 8 spilled 40 B per lane at 3 waves/SIMD, 6 spilled 12)
#endif

namespace hq {

// ----------------------------------------------------------------------------
// Fast path (HALF = 10, the 21-tap filters of the default viewing set): a 1-D
// grid of (output tile, palette) work items.  One workgroup = one TW x TH output
// tile; its region = (TH + 2*HALF) rows x RW columns of palette indices.
// Vertical pass first on all RW region columns (separable filters commute),
// then the horizontal pass on the TW output columns, Opp->Lab, dE, fp64 partial.
// ----------------------------------------------------------------------------
// Tile geometry of the fast path: 8 x 108 output tiles of a 28 x 128 region
// (cost_mfma_kernel) or 16 x 128 tiles of a 36 x 148 region (cost16w_kernel).
constexpr int kFastHalf = 10, kFastRW = 128;
constexpr int kFastTW = kFastRW - 2 * kFastHalf;

template <int HALF>
struct CostTaps {
    float v[kNumFilt][2 * HALF + 1];
    float h[kNumFilt][2 * HALF + 1];
};

// Taps are read through a constant-address-space pointer into device memory
// (uniform s_load per filter; build_fast_taps holds both scalings).
template <int HALF>
using TapsPtr = const __attribute__((address_space(4))) CostTaps<HALF>*;

// TRIM: the narrow k1.x / k1.y / k1.z filters (f = 0, 3, 5) run over their
// significant-tap windows kTrimLo..kTrimHi only (|taps| outside are below 1e-9
// of the filter's peak for the default filter set; see trim_window_ok()).
// Per-filter loops keep one filter's 21 taps live in SGPRs (interleaving a
// channel's filters needs 63 and spills to VGPR lanes).
constexpr int kTrimLo[3] = {7, 6, 5}, kTrimHi[3] = {13, 14, 15};

// ---- vertical pass on the matrix cores --------------------------------------
// The vertical pass of a filter over a 16-column block is a banded-Toeplitz
// product with the block's TH + 2*HALF gathered input rows: one
// v_mfma_f32_16x16x32_f16 K step (rows past the region zero-weighted).  fp32
// accuracy from f16 operands: x = hi + lo (both f16, x scaled by 2^14 so lo
// stays normal down to |x| ~ 1e-5) and the products hi.hi + hi.lo + lo.hi (each
// exact in the f32 accumulator; the dropped lo.lo is ~2^-22 relative).  Taps
// are split the same way on the host, scaled by 2^16
// (build_vpass_f16_stack_fragments); the 2^30 total scale is folded into the
// horizontal taps, exactly (a power of two).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr float kVTapScale = 65536.0f;                    // 2^16
constexpr float kVOutScale = 1.0f / (16384.0f * 65536.0f);  // 2^-30

// Region row of K slot (g = lane >> 4, j) of the vertical pass's B operand.
// Half 0 (output rows 0-7): rows 4j + g (lane group g holds every 4th row).
// Half 1 (output rows 8-15 of a 16-row tile, rows 8-39): slots 2-7 are half
// 0's slots 2-7 (rows 8-31), slots 0 and 1 are rows 32 + g and 36 + g (rows
// 36-39 carry zero taps, so slot 1 needs no gather: 0).  Every lane gathers one
// new value for half 1, and
// half 1's B operand is half 0's with only its first dword replaced (same
// registers, no moves: pack_b_halves).  The A fragments permute K to match.
__host__ __device__ __forceinline__ constexpr int kv_row(int half, int g, int j) {
    return half == 0 || j >= 2 ? 4 * j + g : (j == 0 ? 32 + g : 36 + g);
}


// One work item of the cost pass: palette p over output tile `tile`.
struct TileItem {
    int p, tile, x0, y0;
};

template <int TW, int TH>
__device__ __forceinline__ TileItem tile_item(const CostArgs& a, int w, int P) {
    TileItem t;
    t.p = w % P;
    t.tile = w / P;
    t.x0 = (t.tile % a.tiles_x) * TW;
    t.y0 = a.g.r0 + (t.tile / a.tiles_x) * TH;
    return t;
}

// The global loads that fill one item's LDS (index rows of its region, its
// palette's opponent entry), held in registers between issue and commit.
// Every load is issued before the first wait: vmcnt retires in order, so a
// load -> wait -> store loop pays one memory round trip per trip (4 for the
// interior index rows, 14 for the byte gathers of edge tiles).
// Interior rows are read as DW = RW / 4 dword pairs: the first DM = NTH / 8
// dword columns by a (row, column) = (tid / DM + 8q, tid % DM) map (shifts and
// masks, row offsets one multiply-add), the DW - DM tail columns (cost16w's
// 148-byte rows: 5 of 37; the 276-byte rows of 256-column tiles: 5 of 69) by a
// second, short pass.  NTH = threads of the workgroup.
template <int HALF, int RW, int TH, int NTH = 256>
struct TileFill {
    static constexpr int TW = RW - 2 * HALF, RH = TH + 2 * HALF, DW = RW / 4, DM = NTH / 8;
    static constexpr int DWT = DW - DM;                                   // tail dword columns
    static constexpr int DWTD = DWT > 0 ? DWT : 1;                        // its divisor (no tail: unused)
    static constexpr int NM = (RH * DM + NTH - 1) / NTH, NT = (RH * DWT + NTH - 1) / NTH;
    static constexpr int NFD = NM + NT, NFB = (RH * RW + NTH - 1) / NTH;
    static_assert(RW % 4 == 0 && DW >= DM && DWT < DM, "whole dwords per region row, DM <= DW < 2 DM");
    uint32_t lo[NFD], hi[NFD];  // interior tiles: aligned dword pairs of the index rows
    uint32_t roff[NFD];         // their rows' byte offsets (alignment for commit)
    uint4 ov;  // the palette's split opponent entry tid (zeros past K)
    TileItem t;
    bool interior;

    // Byte offset of region row i in the palette's index image (reflection at the
    // image edges, clamped to the rows held on this device).
    __device__ __forceinline__ static int row_base(const Geom& g, const TileItem& t, int i) {
        int gy = reflect_clamp(t.y0 - HALF + i, g.H);
        gy = min(max(gy, g.e0), g.e1 - 1);
        return (gy - g.e0) * g.W + (t.x0 - HALF);
    }

    // Issue the loads; interior tiles only (edge tiles -- the image's first and
    // last tile columns -- gather bytes with reflection at commit time).  Tiles
    // whose halo rows need neither reflection nor clamping (all but the image's
    // and the shard's first and last tile rows) take row offsets from one
    // multiply-add.  Loads are unconditional (rows clamped into the region) and
    // use 32-bit unsigned offsets from the palette's base (saddr form); the host
    // keeps a shard's index image below 2^31 bytes.
    __device__ __forceinline__ void issue(const CostArgs& a, const TileItem& ti, int tid) {
        static_assert(kMaxK <= NTH, "one opponent-table entry per thread");
        const Geom& g = a.g;
        t = ti;
        const uint8_t* idx = a.idx + (int64_t)t.p * g.idx_pitch;
#ifdef HQ_ABL_NOFILL  // timing ablation (wrong results): no global loads for the fill
        ov = make_uint4(tid, tid + 1, tid + 2, 0u);
        interior = true;
#pragma unroll
        for (int q = 0; q < NFD; ++q) lo[q] = hi[q] = roff[q] = (uint32_t)(tid * 7 + q);
        return;
#endif
        ov = tid < a.K ? a.opp16[(int64_t)t.p * kMaxK + tid] : make_uint4(0u, 0u, 0u, 0u);
        interior = t.x0 - HALF >= 0 && t.x0 + TW + HALF <= g.W;
        if (interior) {
            const int ytop = t.y0 - HALF;
            const bool vfast = ytop >= 0 && ytop >= g.e0 && ytop + RH <= g.H && ytop + RH <= g.e1;
            const int ubase = (ytop - g.e0) * g.W + (t.x0 - HALF);
            auto load = [&](int q, int i, int c) {
                roff[q] = (uint32_t)(vfast ? ubase + i * g.W : row_base(g, t, i));
                const uint32_t* src =
                    reinterpret_cast<const uint32_t*>(idx + ((roff[q] & ~3u) + 4u * (uint32_t)c));
                lo[q] = src[0];
                hi[q] = src[1];
            };
#pragma unroll
            for (int q = 0; q < NM; ++q) load(q, min(tid / DM + 8 * q, RH - 1), tid % DM);
#pragma unroll
            for (int q = 0; q < NT; ++q) {
                const int e = min(tid + NTH * q, RH * DWT - 1);
                load(NM + q, e / DWTD, DM + e % DWTD);
            }
        }
    }

    // index rows into s_idx (row pitch IDXP bytes); the first write waits for the loads
    template <int IDXP>
    __device__ __forceinline__ void commit_idx(const CostArgs& a, uint8_t* s_idx, int tid) const {
        const Geom& g = a.g;
        if (interior) {
            uint32_t* s32 = reinterpret_cast<uint32_t*>(s_idx);
#pragma unroll
            for (int q = 0; q < NM; ++q) {
                const int i = tid / DM + 8 * q;
                if (i < RH)
                    s32[i * (IDXP / 4) + tid % DM] = __builtin_amdgcn_alignbyte(hi[q], lo[q], roff[q] & 3u);
            }
#pragma unroll
            for (int q = 0; q < NT; ++q) {
                const int e = tid + NTH * q;
                if (e < RH * DWT)
                    s32[(e / DWTD) * (IDXP / 4) + DM + e % DWTD] =
                        __builtin_amdgcn_alignbyte(hi[NM + q], lo[NM + q], roff[NM + q] & 3u);
            }
        } else {
            const uint8_t* idx = a.idx + (int64_t)t.p * g.idx_pitch;
            uint32_t b[NFB];
#pragma unroll
            for (int q = 0; q < NFB; ++q) {  // all loads first: one round trip
                const int e = min(tid + NTH * q, RH * RW - 1);
                const int i = e / RW, j = e % RW;
                int gy = reflect_clamp(t.y0 - HALF + i, g.H);
                gy = min(max(gy, g.e0), g.e1 - 1);
                const int gx = reflect_clamp(t.x0 - HALF + j, g.W);
                b[q] = idx[(uint32_t)((gy - g.e0) * g.W + gx)];
            }
#pragma unroll
            for (int q = 0; q < NFB; ++q) {
                const int e = tid + NTH * q;
                if (e < RH * RW) s_idx[(e / RW) * IDXP + e % RW] = (uint8_t)b[q];
            }
        }
    }
};

// The 16-bit index rows of a chunked palette's tile (256 < K <= 4096): region
// row i = RWL indices from column x0 - HALF into s_idx row i (pitch RW
// elements; columns RWL .. RW - 1, read by the vertical pass's last block but
// never used, are zeroed so they index the table).  Tiles whose rows all start
// on a dword (interior tiles of an even-width image at an even HALF) load
// dwords of two indices; the others gather element by element with reflection.
template <int HALF, int RWL, int RW, int TH, int NTH = 256>
struct TileFill16 {
    static constexpr int RH = TH + 2 * HALF, DW = RWL / 2, NL = (RH * DW + NTH - 1) / NTH;
    static constexpr int NE = (RH * RW + NTH - 1) / NTH, NZ = RH * (RW - RWL) / 2;
    static_assert(RWL % 2 == 0 && RW % 2 == 0, "whole dwords");
    uint32_t v[NL];
    TileItem t;
    bool fast;

    __device__ __forceinline__ void issue(const CostArgs& a, const TileItem& ti, int tid) {
        const Geom& g = a.g;
        t = ti;
        const uint16_t* idx = reinterpret_cast<const uint16_t*>(a.idx) + (int64_t)t.p * g.idx_pitch;
        fast = t.x0 - HALF >= 0 && t.x0 + RWL - HALF <= g.W && (g.W & 1) == 0 && ((t.x0 - HALF) & 1) == 0;
        if (fast) {
#pragma unroll
            for (int q = 0; q < NL; ++q) {
                const int e = min(tid + NTH * q, RH * DW - 1), i = e / DW, c = e - i * DW;
                const int roff = TileFill<HALF, RWL, TH, NTH>::row_base(g, t, i);  // even: dword aligned
                v[q] = *reinterpret_cast<const uint32_t*>(idx + roff + 2 * c);
            }
        }
    }

    __device__ __forceinline__ void commit(const CostArgs& a, uint16_t* s_idx, int tid) const {
        const Geom& g = a.g;
        uint32_t* s32 = reinterpret_cast<uint32_t*>(s_idx);
        if (fast) {
#pragma unroll
            for (int q = 0; q < NL; ++q) {
                const int e = tid + NTH * q, i = e / DW, c = e - i * DW;
                if (e < RH * DW) s32[i * (RW / 2) + c] = v[q];
            }
            for (int e = tid; e < NZ; e += NTH) {
                const int i = e / ((RW - RWL) / 2), c = e - i * ((RW - RWL) / 2);
                s32[i * (RW / 2) + RWL / 2 + c] = 0u;
            }
        } else {
            const uint16_t* idx = reinterpret_cast<const uint16_t*>(a.idx) + (int64_t)t.p * g.idx_pitch;
            uint32_t b[NE];
#pragma unroll
            for (int q = 0; q < NE; ++q) {  // all loads first: one round trip
                const int e = min(tid + NTH * q, RH * RW - 1), i = e / RW, j = e - i * RW;
                int gy = reflect_clamp(t.y0 - HALF + i, g.H);
                gy = min(max(gy, g.e0), g.e1 - 1);
                const int gx = reflect_clamp(t.x0 - HALF + min(j, RWL - 1), g.W);
                b[q] = idx[(uint32_t)((gy - g.e0) * g.W + gx)];
            }
#pragma unroll
            for (int q = 0; q < NE; ++q) {
                const int e = tid + NTH * q, i = e / RW, j = e - i * RW;
                if (e < RH * RW) s_idx[i * RW + j] = j < RWL ? (uint16_t)b[q] : (uint16_t)0;
            }
        }
    }
};

// Horizontal pass on row pairs: s_v holds float2 (row 2m, row 2m+1) per column,
// so v_pk_fma_f32 runs across a row pair and every tap reads a naturally
// aligned register pair (a row layout's odd taps needed register-pair shuffles,
// ~29% of the pass's VALU instructions).  HR output columns per item.
template <int HALF, int TH, int RW, int HR, int TLO = 0, int THI = 2 * HALF>
__device__ __forceinline__ void hpass_pair_filters(const f32x4* src, TapsPtr<HALF> taps, int f0,
                                                   int f1, f32x2 (&acc)[HR], int fslot = 0) {
    constexpr int NIN = HR + 2 * HALF;  // window columns (float2 each)
    constexpr int NQ = (NIN + 1) / 2;   // ds_read_b128, two columns each
#pragma unroll 1
    for (int f = f0; f < f1; ++f) {
        const f32x4* row = src + (f - fslot) * (TH / 2) * RW / 2;
        f32x4 v[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) v[q] = row[q];
        f32x2 in[2 * NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            in[2 * q] = v[q].xy;
            in[2 * q + 1] = v[q].zw;
        }
#pragma unroll
        for (int t = TLO; t <= THI; ++t) {
            const float k = taps->h[f][t];
            const f32x2 kk = {k, k};
#pragma unroll
            for (int xo = 0; xo < HR; ++xo) acc[xo] = __builtin_elementwise_fma(in[xo + t], kk, acc[xo]);
        }
    }
}

// ----------------------------------------------------------------------------
// cost_mfma: 8-row tiles in two channel groups -- channel 0's three filters (V
// then H), then channels 1-2's four -- so s_v holds at most four filter planes
// (23 KiB of LDS, 6 workgroups per CU).  Both vertical passes on the matrix
// cores in split f16: per 16-column block and pair of filters
// of one channel, one v_mfma_f32_16x16x32_f16 K-step covers the 28 region rows
// (+4 zero-weight rows) as hi.hi + hi.lo + lo.hi (each product exact in the
// fp32 accumulator; lo.lo ~2^-22 relative is dropped).  A = the stacked
// Toeplitz taps (rows = filter pair x 8 output rows, x 2^16, split on the host:
// build_vpass_f16_stack_fragments), B = the gathered opponent values (x 2^14),
// read from per-channel (hi, lo) f16 dword tables (split once per palette by
// the prep, PaletteArgs::opp16), so the gathers need no conversion (one LDS
// read per value).  D (x 2^30, folded exactly into the
// horizontal taps) holds 4 consecutive output rows of one filter and column per
// lane: two row-pair stores.  Stacks (f0, f1), (f2, -), (f3, f4), (f5, f6); wave
// w takes region columns 32w .. +31: 12 MFMAs per group and wave.
// (An exact-fp32 version on v_mfma_f32_16x16x4_f32, 56 MFMAs per wave, was 9%
// slower than the VALU pass: fp32 MFMA runs at the fp32 vector rate.)
// ----------------------------------------------------------------------------
typedef float f32x4v __attribute__((ext_vector_type(4)));

// D of one 16x16 stack block -> s_v row pairs: lane (c = l & 15, q = l >> 4)
// holds rows 4(q & 1) .. +3 of the stack's filter q >> 1 at column c.
__device__ __forceinline__ void store_vstack(float* s_v, const f32x4v& d, int plane_a, int plane_b,
                                             int lk, int col) {
    constexpr int RW = 128, PAIRS = 4;
    const int plane = lk < 2 ? plane_a : plane_b;
    if (plane < 0) return;
    const int p0 = 2 * (lk & 1);
    f32x2* v = reinterpret_cast<f32x2*>(s_v);
    v[(plane * PAIRS + p0) * RW + col] = f32x2{d[0], d[1]};
    v[(plane * PAIRS + p0 + 1) * RW + col] = f32x2{d[2], d[3]};
}

// B fragments of one 16-column block: region rows 8q .. 8q+7 (q = lane >> 4) of
// column `col`.  Table entries hold (hi, lo) f16 of a channel in one dword
// (split_f16), so one LDS read per value; v_perm packs the halves.
__device__ __forceinline__ void pack_b(const uint32_t (&w)[8], f16x8& bh, f16x8& bl) {
    u32x4 h, l;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        h[m] = __builtin_amdgcn_perm(w[2 * m + 1], w[2 * m], 0x05040100u);  // hi halves
        l[m] = __builtin_amdgcn_perm(w[2 * m + 1], w[2 * m], 0x07060302u);  // lo halves
    }
    bh = __builtin_bit_cast(f16x8, h);
    bl = __builtin_bit_cast(f16x8, l);
}

// Both halves' B operands of a 16-row tile's block: w[0..7] = half 0's slots,
// w[8], w[9] = half 1's slots 0 and 1 (kv_row).  Half 1's operand is half 0's
// with dword 0 replaced: the caller issues half 0's MFMAs, then writes nh / nl
// into dword 0 (the registers are reused in place).
__device__ __forceinline__ void pack_b_halves(const uint32_t (&w)[10], u32x4& h, u32x4& l,
                                              uint32_t& nh, uint32_t& nl) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        h[m] = __builtin_amdgcn_perm(w[2 * m + 1], w[2 * m], 0x05040100u);  // hi halves
        l[m] = __builtin_amdgcn_perm(w[2 * m + 1], w[2 * m], 0x07060302u);  // lo halves
    }
    nh = __builtin_amdgcn_perm(w[9], w[8], 0x05040100u);
    nl = __builtin_amdgcn_perm(w[9], w[8], 0x07060302u);
}

__device__ __forceinline__ f32x4v mfma3(const f16x8& ah, const f16x8& al, const f16x8& bh,
                                        const f16x8& bl) {
    f32x4v d = {0.f, 0.f, 0.f, 0.f};
#ifndef HQ_ABL_MFMA1  // (timing ablation, wrong results: the hi.hi product only)
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, d, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, d, 0, 0, 0);
#endif
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, d, 0, 0, 0);
    return d;
}

template <int DE, bool TRIM>
__global__ __launch_bounds__(256, 6) void cost_mfma_kernel(CostArgs a, int P_) {
    constexpr int HALF = 10, RW = 128, TH = 8, HR = 2, T2 = 2 * HALF;
    constexpr int TW = RW - 2 * HALF, RH = TH + 2 * HALF;
    constexpr int NRUN = TW / HR, SLOTS = 64, NITEM = (TH / 2) * SLOTS;
    constexpr int PLANE = (TH / 2) * RW / 2;  // f32x4 per filter plane (row pairs)
    static_assert(NRUN <= SLOTS && NITEM <= 256 && RH <= 32, "tile");
    __shared__ f32x4 s_vq[4 * PLANE];
    __shared__ uint32_t s_ox[kMaxK];  // opponent x 2^14 as (hi, lo) f16 pairs: channel 0
    __shared__ uint2 s_oyz[kMaxK];     // channels 1, 2
    // 32 rows: the K = 32 step reads rows 28-31 too (zero taps; any finite index)
    __shared__ __attribute__((aligned(16))) uint8_t s_idx[32 * RW];
    __shared__ double s_red[4];
    float* s_v = reinterpret_cast<float*>(s_vq);
    const int tid = threadIdx.x;
    const Geom& g = a.g;
    const TileItem cur = tile_item<TW, TH>(a, xcd_remap(blockIdx.x, a.ntiles * P_), P_);
    const TapsPtr<HALF> taps = (TapsPtr<HALF>)(uintptr_t)a.taps;  // H taps x 2^-30
    const int lane = tid & 63, wv = tid >> 6, lc = lane & 15, lk = lane >> 4;
    const uint4* frag = a.vfrag16 + (TRIM ? 2 * 4 * 2 * 64 : 0) + lane;  // [trim][half 0][stack][hi,lo][lane]

    TileFill<HALF, RW, TH> fill;
    fill.issue(a, cur, tid);
    uint4 F0h = frag[(0 * 2 + 0) * 64], F0l = frag[(0 * 2 + 1) * 64];  // group 0 stacks
    uint4 F1h = frag[(1 * 2 + 0) * 64], F1l = frag[(1 * 2 + 1) * 64];
    // every entry (zeros for tid >= K): the zero-weight rows 28-31 gather arbitrary
    // indices, and 0 x NaN would be NaN
    s_ox[tid] = fill.ov.x;
    s_oyz[tid] = make_uint2(fill.ov.y, fill.ov.z);
    fill.template commit_idx<RW>(a, s_idx, tid);
    const int m = tid / SLOTS, jr = tid % SLOTS;
    const bool has_item = tid < NITEM && jr < NRUN;
    const int gy0 = cur.y0 + 2 * m, gx0 = cur.x0 + HR * jr;
    __syncthreads();

    const int col0 = 32 * wv + lc;
    const f32x4* hsrc = &s_vq[(m * RW + HR * jr) / 2];
    f32x2 acc0[HR], acc1[HR], acc2[HR];
#pragma unroll
    for (int xo = 0; xo < HR; ++xo) acc0[xo] = acc1[xo] = acc2[xo] = f32x2{0.f, 0.f};

    // ---- group 0: channel 0 -> planes 0-2 ----
    {
        const f16x8 a0h = __builtin_bit_cast(f16x8, F0h), a0l = __builtin_bit_cast(f16x8, F0l);
        const f16x8 a1h = __builtin_bit_cast(f16x8, F1h), a1l = __builtin_bit_cast(f16x8, F1l);
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            uint32_t w[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) w[j] = s_ox[s_idx[kv_row(0, lk, j) * RW + col0 + 16 * bb]];
            f16x8 bh, bl;
            pack_b(w, bh, bl);
            store_vstack(s_v, mfma3(a0h, a0l, bh, bl), 0, 1, lk, col0 + 16 * bb);
            store_vstack(s_v, mfma3(a1h, a1l, bh, bl), 2, -1, lk, col0 + 16 * bb);
        }
    }
    const uint4 F2h = frag[(2 * 2 + 0) * 64], F2l = frag[(2 * 2 + 1) * 64];  // group 1 stacks,
    const uint4 F3h = frag[(3 * 2 + 0) * 64], F3l = frag[(3 * 2 + 1) * 64];  // in flight during H
    __syncthreads();
    if (has_item) {
        if constexpr (TRIM) {
            hpass_pair_filters<HALF, TH, RW, HR, kTrimLo[0], kTrimHi[0]>(hsrc, taps, 0, 1, acc0);
            hpass_pair_filters<HALF, TH, RW, HR, 0, T2>(hsrc, taps, 1, 3, acc0);
        } else {
            hpass_pair_filters<HALF, TH, RW, HR, 0, T2>(hsrc, taps, 0, 3, acc0);
        }
    }
    __syncthreads();

    // ---- group 1: channels 1, 2 -> planes 0-3 ----
    {
        const f16x8 a2h = __builtin_bit_cast(f16x8, F2h), a2l = __builtin_bit_cast(f16x8, F2l);
        const f16x8 a3h = __builtin_bit_cast(f16x8, F3h), a3l = __builtin_bit_cast(f16x8, F3l);
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            uint32_t wy[8], wz[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint2 e = s_oyz[s_idx[kv_row(0, lk, j) * RW + col0 + 16 * bb]];
                wy[j] = e.x; wz[j] = e.y;
            }
            f16x8 bh, bl;
            pack_b(wy, bh, bl);
            store_vstack(s_v, mfma3(a2h, a2l, bh, bl), 0, 1, lk, col0 + 16 * bb);
            pack_b(wz, bh, bl);
            store_vstack(s_v, mfma3(a3h, a3l, bh, bl), 2, 3, lk, col0 + 16 * bb);
        }
    }
    float labv[2][3][HR];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const bool ok = has_item && gy0 + r < g.r1 && gx0 < g.W;
        const uint32_t off = ok ? (uint32_t)((gy0 + r - g.r0) * g.lab_pitch + gx0) : 0u;
        const float* src3[3] = {a.labL, a.labA, a.labB};
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            const float2 v = *reinterpret_cast<const float2*>(
                reinterpret_cast<const char*>(src3[ch]) + (off << 2));  // 32-bit byte offset
            labv[r][ch][0] = v.x; labv[r][ch][1] = v.y;
        }
    }
    __syncthreads();

    double sum = 0.0;
    if (has_item) {
        if constexpr (TRIM) {
            hpass_pair_filters<HALF, TH, RW, HR, kTrimLo[1], kTrimHi[1]>(hsrc, taps, 3, 4, acc1, 3);
            hpass_pair_filters<HALF, TH, RW, HR, 0, T2>(hsrc, taps, 4, 5, acc1, 3);
            hpass_pair_filters<HALF, TH, RW, HR, kTrimLo[2], kTrimHi[2]>(hsrc, taps, 5, 6, acc2, 3);
            hpass_pair_filters<HALF, TH, RW, HR, 0, T2>(hsrc, taps, 6, 7, acc2, 3);
        } else {
            hpass_pair_filters<HALF, TH, RW, HR, 0, T2>(hsrc, taps, 3, 5, acc1, 3);
            hpass_pair_filters<HALF, TH, RW, HR, 0, T2>(hsrc, taps, 5, 7, acc2, 3);
        }
        float part = 0.f;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
#pragma unroll
            for (int xo = 0; xo < HR; ++xo) {
                const float3 lf = opp2f_fast(acc0[xo][r], acc1[xo][r], acc2[xo][r], a.m_lab);
                const float e = delta_e_f<DE>(labv[r][0][xo], labv[r][1][xo], labv[r][2][xo], lf);
                const bool in = gy0 + r < g.r1 && gx0 + xo < g.W;
                part += in ? e : 0.f;
                if (a.pix_err && in)  // test option: the per-pixel dE (CL:201-209's error image)
                    a.pix_err[(int64_t)cur.p * a.pix_pitch + (int64_t)(gy0 + r - g.r0) * g.W + gx0 + xo] = e;
            }
        }
        sum = (double)part;
    }
    sum = wave_sum_to_lane63(sum);
    if ((tid & 63) == 63) s_red[tid >> 6] = sum;
    __syncthreads();
    if (tid == 0)
        acc_add(a.acc, a.acc_P, a.acc_p0 + cur.p, cur.tile, (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]));
}

// ----------------------------------------------------------------------------
// cost16w<HB>: 16 x 128 output tiles of a (16 + 2 HB) x (128 + 2 HB) region,
// HB = the tap bucket's half-width: the filters' own half-width H <= HB sits
// centred in 2 HB + 1 taps (zero-padded; Tile16, fast_bucket), so every viewing
// geometry of the plugin (dpi, distance: HQ:229-231, SP:80-102, IM:408) up to
// H = 24 runs this kernel.  HB = 10 is the default 21-tap set.  The random
// opponent-table gathers of the vertical pass and the horizontal windows are
// the kernel's LDS traffic; FP32 VALU issue (horizontal taps, Lab/dE) bounds it.
// - vertical pass on the matrix cores: output rows 0-7 take region rows
//   0 .. 32 S - 1 (S K steps of 32 rows), rows 8-15 take rows 8 .. 32 S + 7.
//   Lane group g holds every 4th row (kv_row: K slot (g, j) of step s = row
//   32 s + 4 j + g), so half 1's operand of step s is half 0's with dword 0
//   replaced by the next step's dword 0: each lane gathers 8 S + 2 rows (the
//   ones past the region are zero, not gathered) for 2 x 8 output rows, no
//   divergence.  At HB = 10 (S = 1): 36 gathered rows per 16 output rows.
//   Above HB = 10 the (hi, lo) pair layout instead (vblock_pair): steps of 16
//   rows, the gathered dwords used as B operands as they are, 4 S + 2 rows per
//   lane.
//   RW / 16 blocks of 16 columns (ranges of 32) cover the region columns
//   (+ unread ones): each block is the 16 columns of one parity half of a range
//   (lane n -> column 4(n >> 1) + 2 (b & 1) + (n & 1)), so its stores fill 16
//   contiguous float2 of one half: conflict free without padding.  Block sets
//   {s, s+4, s+8} go to the waves, rotated per workgroup.
// - horizontal pass: items of 4 output columns x a row pair (256 items, one per
//   thread: 8 row pairs x 32), a (4 + 2 HB)-column window = 2 + HB ds_read_b128
//   per filter for 8 outputs.  Row-pair rows store their column pairs split by
//   parity (pair p -> half p & 1, slot p >> 1), so read q of item j lands at
//   half q & 1, slot j + q / 2: lanes 16 B apart, conflict free.  (The
//   108-column tile of a 128-column region gave 27 items to 32 threads: 16% of
//   the lanes idle through the horizontal pass and Lab/dE; 0.398 vs 0.383 ms.)
// - the row-pair planes fit 4 workgroups per CU (3 for HB > 10) three filters
//   at a time, so the channels run in three phases: channel 0 (f0, f1, f2),
//   channel 1 (f3, f4), channel 2 (f5, f6).  Channels 1 and 2 share one gather
//   per region row; channel 2's vertical results wait in registers through
//   channel 1's horizontal pass.  HB = 10: 39,584 B of LDS.
// ----------------------------------------------------------------------------
constexpr int kTH16 = 16;
#ifndef HQ_LAB_SKIPLIN
#define HQ_LAB_SKIPLIN 1  // cost16w: skip the linear Lab segment when no pixel of the wave is in it
#endif
#ifndef HQ_LAB_NT
#define HQ_LAB_NT 0  // 1: LabRef read with non-temporal loads (streamed past the caches)
#endif

template <int HB, int NW = 4>
struct Tile16 {
    static constexpr int TH = kTH16, TW = 32 * NW, HR = 4;  // NW waves: 4 (16 x 128) or 8 (16 x 256)
    static constexpr int RWL = (TW + 2 * HB + 3) / 4 * 4;  // region columns read (whole dwords)
    static constexpr int RW = (RWL + 31) / 32 * 32;    // LDS pitch: whole 32-column ranges
    static constexpr int RH = TH + 2 * HB;             // region rows
    static constexpr int NBLK = RW / 16;               // vertical-pass column blocks
    static constexpr int NSET = (NBLK + NW - 1) / NW;  // blocks per wave (at most)
    static constexpr int WH = RW / 2;                  // float2 per half of a permuted row-pair row
    // vertical pass: the (hi, lo) pair layout (vblock_pair) above the 21-tap
    // bucket, the 32-row layout (vblock) at HB = 10 (same-box A/B: pair layout
    // -3% cost at HB = 19, -1.5% at 15, +4% at 10, where it needs 4 MFMAs per
    // half and stack instead of 3 and its overlapping B windows cost copies)
    static constexpr bool PAIR = HB > 10;
    static constexpr int S = PAIR ? (8 + 2 * HB + 15) / 16 : (8 + 2 * HB + 31) / 32;  // MFMA K steps per half
    static constexpr int NJ = PAIR ? 4 * S + 2 : 8 * S + 2;  // rows 4 n + g a lane gathers
    static constexpr int AH = PAIR ? 1 : 2;  // fragment sets per stack and step (the pair layout's halves share)
    static constexpr int PLANE4 = (TH / 2) * RW / 2;   // f32x4 per filter plane
    static constexpr int NQ = (HR + 2 * HB) / 2;       // horizontal window reads per filter
    static_assert(RWL % 4 == 0 && RWL / 4 >= 8 * NW && RWL / 4 < 16 * NW, "TileFill: 8 NW <= dwords per row < 16 NW");
    static_assert(NSET <= 3, "three blocks per wave at most");
};

// Significant half-windows of the narrow k1.x / k1.y / k1.z filters per bucket:
// the largest over every geometry whose H falls in the bucket (checked per
// filter set at hq_set_filters: trim_window_ok; the windows of 18 dpi x 13
// distance settings were swept with the oracle's filter design, SP:66-254).
__host__ __device__ constexpr int trim_w(int HB, int ch) {
    return HB == 10 ? (ch == 0 ? 3 : ch == 1 ? 4 : 5)
         : HB == 15 ? (ch == 0 ? 4 : ch == 1 ? 5 : 7)
         : HB == 19 ? (ch == 0 ? 5 : ch == 1 ? 7 : 9)
                    : (ch == 0 ? 6 : ch == 1 ? 9 : 12);
}

// Region row of K slot (g, j) of step s for output-row half `half` (see above).
__host__ __device__ __forceinline__ constexpr int kv_row_s(int half, int s, int g, int j) {
    return half == 0 || j >= 2 ? 32 * s + 4 * j + g : 32 * (s + 1) + 4 * j + g;
}

// float2 position of column `col` in a permuted row-pair row: half = bit 1 of
// col, 16-B slot col >> 2, float2 col & 1.
template <int WH>
__device__ __forceinline__ int wide_pos(int col) {
    return ((col >> 1) & 1) * WH + ((col >> 2) << 1) + (col & 1);
}

// Horizontal pass of filter f for item j (output columns 4j .. 4j+3) of a row
// pair: src = the row-pair row in plane 0; pstride = f32x4 per plane; taps
// [TLO, THI].  Item j's read q (columns 4j + 2q, +1) sits at half q & 1,
// slot j + q / 2.  Windows longer than 24 columns run in chunks of 12 taps
// (each chunk's reads issued together) to bound the live registers.
template <int HB, int TLO = 0, int THI = 2 * HB, int WH = 80>
__device__ __forceinline__ void hpass_wide(const f32x4* src, int j, TapsPtr<HB> taps, int f,
                                           int plane, int pstride, f32x2 (&acc)[4]) {
    constexpr int HR = 4;
    constexpr int CH = HB <= 10 ? 2 * HB + 1 : HB == 19 ? HQ_CH19 : HQ_CHW;  // taps per chunk
    const f32x4* row = src + plane * pstride + j;
#ifdef HQ_ABL_NOHPASS  // timing ablation (wrong results): one window read, no taps
    {
        const f32x4 v = row[0];
        acc[0] += v.xy;
        acc[1] += v.zw;
        return;
    }
#endif
#pragma unroll
    for (int t0 = TLO; t0 <= THI; t0 += CH) {
        const int t1 = t0 + CH - 1 < THI ? t0 + CH - 1 : THI;
        const int q0 = t0 / 2, q1 = (t1 + HR - 1) / 2;  // reads covering columns t0 .. t1 + 3
        f32x2 in[2 * (CH / 2 + 3)];
#pragma unroll
        for (int q = q0; q <= q1; ++q) {
            const f32x4 v = row[(q & 1) * (WH / 2) + (q >> 1)];
            in[2 * (q - q0)] = v.xy;
            in[2 * (q - q0) + 1] = v.zw;
        }
#pragma unroll
        for (int t = t0; t <= t1; ++t) {
            const float k = taps->h[f][t];
            const f32x2 kk = {k, k};
#pragma unroll
            for (int xo = 0; xo < HR; ++xo)
                acc[xo] = __builtin_elementwise_fma(in[xo + t - 2 * q0], kk, acc[xo]);
        }
    }
}

// D of one 16x16 stack block of output-row half `half` -> permuted row pairs:
// lane (c = l & 15, q = l >> 4) holds rows 8 half + 4(q & 1) .. +3 of the
// stack's filter q >> 1 at its column.  Addresses hoisted: `base` = the
// lane's float2 slot of block set i = 0, half 0 in its plane (vstack_base);
// block i and half add compile-time offsets (block b + 4 moves 64 columns =
// 32 float2 of the permuted row).
template <int WH>
__device__ __forceinline__ f32x2* vstack_base(float* s_v, int plane, int lk, int col0) {
    constexpr int PAIRS = kTH16 / 2, ROW = 2 * WH;
    return reinterpret_cast<f32x2*>(s_v) + (plane * PAIRS + 2 * (lk & 1)) * ROW + wide_pos<WH>(col0);
}
template <int WH, int NW = 4>
__device__ __forceinline__ void store_vstack_at(f32x2* base, const f32x4v& d, int i, int half) {
    constexpr int ROW = 2 * WH;
#ifdef HQ_ABL_NOVSTORE  // timing ablation (wrong results): vertical results not stored
    if (d[0] != 12345.f) return;
#endif
    f32x2* v = base + 4 * half * ROW + 8 * NW * i;  // block set i + 1: 16 NW columns on
    v[0] = f32x2{d[0], d[1]};
    v[ROW] = f32x2{d[2], d[3]};
}

__device__ __forceinline__ f32x4v mfma3_acc(const f16x8& ah, const f16x8& al, const f16x8& bh,
                                            const f16x8& bl, f32x4v d) {
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, d, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, d, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, d, 0, 0, 0);
    return d;
}

// One column block's vertical products for up to two stacks: w[NJ] = the
// gathered (hi, lo) dwords of rows 4 n + g; A[stack][half][step][hi, lo] the
// split-f16 tap fragments.  d[stack][half] = both halves' 16 x 16 blocks.
template <int S, int NST>
__device__ __forceinline__ void vblock(const uint32_t (&w)[8 * S + 2], const uint4 (&A)[NST][2][S][2],
                                       f32x4v (&d)[NST][2]) {
    auto H = [](const uint4& u) { return __builtin_bit_cast(f16x8, u); };
    auto B = [](const u32x4& u) { return __builtin_bit_cast(f16x8, u); };
#pragma unroll
    for (int st = 0; st < NST; ++st) d[st][0] = d[st][1] = f32x4v{0.f, 0.f, 0.f, 0.f};
#ifdef HQ_ABL_NOMFMA  // timing ablation (wrong results): no operand packing, no MFMA
#pragma unroll
    for (int st = 0; st < NST; ++st) {
        d[st][0] = f32x4v{__uint_as_float(w[0]), __uint_as_float(w[1]), __uint_as_float(A[st][0][0][0].x), 0.f};
        d[st][1] = f32x4v{__uint_as_float(w[2]), __uint_as_float(w[3]), __uint_as_float(A[st][1][0][1].y), 0.f};
    }
    return;
#endif
#pragma unroll
    for (int s = 0; s < S; ++s) {
        u32x4 bh, bl;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            bh[m] = __builtin_amdgcn_perm(w[8 * s + 2 * m + 1], w[8 * s + 2 * m], 0x05040100u);  // hi halves
            bl[m] = __builtin_amdgcn_perm(w[8 * s + 2 * m + 1], w[8 * s + 2 * m], 0x07060302u);  // lo halves
        }
        const uint32_t nh = __builtin_amdgcn_perm(w[8 * s + 9], w[8 * s + 8], 0x05040100u);
        const uint32_t nl = __builtin_amdgcn_perm(w[8 * s + 9], w[8 * s + 8], 0x07060302u);
#pragma unroll
        for (int st = 0; st < NST; ++st)
            d[st][0] = mfma3_acc(H(A[st][0][s][0]), H(A[st][0][s][1]), B(bh), B(bl), d[st][0]);
        bh[0] = nh;  // half 1 of step s: half 0's operand with dword 0 of step s + 1
        bl[0] = nl;
#pragma unroll
        for (int st = 0; st < NST; ++st)
            d[st][1] = mfma3_acc(H(A[st][1][s][0]), H(A[st][1][s][1]), B(bh), B(bl), d[st][1]);
    }
}

// One column block's vertical products in the (hi, lo) pair layout: w[n] =
// the gathered dword of region row 4 n + g, its (hi, lo) f16 pair, used as
// two K slots of the B operand as is (no repacking).  Step u of half 0 reads
// w[4 u .. 4 u + 3] (rows 16 u .. 16 u + 15 over the four lane groups), half 1
// the rows 8 further on, w[4 u + 2 .. 4 u + 5], with the same A fragments
// A[stack][u][hi, lo] (each K-slot pair holds one tap part twice): hi taps x
// (hi + lo) data, then lo taps x (hi + lo) data, fp32 accumulate -- the full
// split product (the lo.lo term included), two MFMAs per 16 rows and no
// v_perm (the 32-row layout needed ten per step to split hi and lo halves).
template <int N>
using u32xn = uint32_t __attribute__((ext_vector_type(N)));

// dwords O .. O + 3 of the gathered rows as one B operand: a sub-register of
// the rows' single wide register, so the overlapping windows of the two
// halves need no copies
template <int O, int N>
__device__ __forceinline__ f16x8 pair_window(const u32xn<N>& v) {
    return __builtin_bit_cast(f16x8, __builtin_shufflevector(v, v, O, O + 1, O + 2, O + 3));
}

template <int U, int S, int NST>
__device__ __forceinline__ void vblock_pair_step(const u32xn<4 * S + 2>& v, const uint4 (&A)[NST][S][2],
                                                 f32x4v (&d)[NST][2]) {
    if constexpr (U < S) {
        auto H = [](const uint4& u) { return __builtin_bit_cast(f16x8, u); };
        const f16x8 b0 = pair_window<4 * U, 4 * S + 2>(v);
        const f16x8 b1 = pair_window<4 * U + 2, 4 * S + 2>(v);
#pragma unroll
        for (int st = 0; st < NST; ++st) {
            d[st][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(H(A[st][U][0]), b0, d[st][0], 0, 0, 0);
            d[st][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(H(A[st][U][1]), b0, d[st][0], 0, 0, 0);
            d[st][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(H(A[st][U][0]), b1, d[st][1], 0, 0, 0);
            d[st][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(H(A[st][U][1]), b1, d[st][1], 0, 0, 0);
        }
        vblock_pair_step<U + 1, S, NST>(v, A, d);
    }
}

template <int S, int NST>
__device__ __forceinline__ void vblock_pair(const uint32_t (&w)[4 * S + 2], const uint4 (&A)[NST][S][2],
                                            f32x4v (&d)[NST][2]) {
    u32xn<4 * S + 2> v;
#pragma unroll
    for (int n = 0; n < 4 * S + 2; ++n) v[n] = w[n];
#pragma unroll
    for (int st = 0; st < NST; ++st) d[st][0] = d[st][1] = f32x4v{0.f, 0.f, 0.f, 0.f};
    vblock_pair_step<0, S, NST>(v, A, d);
}

// cost16w's vertical products in its bucket's layout (Tile16::PAIR)
template <bool PAIR, int S, int NST, int AH, int NJ>
__device__ __forceinline__ void vblock_any(const uint32_t (&w)[NJ], const uint4 (&A)[NST][AH][S][2],
                                           f32x4v (&d)[NST][2]) {
    if constexpr (PAIR) vblock_pair<S, NST>(w, *reinterpret_cast<const uint4(*)[NST][S][2]>(&A), d);
    else vblock<S, NST>(w, A, d);
}

#ifndef HQ_LB15
#define HQ_LB15 3  // waves per SIMD of the 15-tap bucket (4, with its (y, z) table moved into plane 2 to
                   // fit 4 workgroups' LDS: no faster, 0.476 against 0.477 ms at 150/30)
#endif
#ifndef HQ_LB24
#define HQ_LB24 2  // waves per SIMD of the 24-tap bucket (3: 92 B of spill, 0.823-0.826 against 0.820 ms)
#endif
#ifndef HQ_LB19
#define HQ_LB19 3  // waves per SIMD of the 19-tap bucket
#endif
// occupancy per bucket: LDS allows 4 workgroups per CU at HB = 10, 3 above;
// chunked palettes (NCH > 1: 16-bit indices, a table of 256 NCH entries): 3 up
// to 1,024 colours, 2 up to 4,096, 1 above (the 64 KiB table at 8,192)
template <int HB, int NCH = 1>
constexpr int cost16w_waves() {
    return NCH > 16 ? 1 : NCH > 4 ? 2 : NCH > 1 ? 3 : HB == 10 ? 4 : HB == 15 ? HQ_LB15 : HB == 19 ? HQ_LB19 : HQ_LB24;
}

// NCH > 1 (chunked palettes, 256 < K <= 256 NCH; HB = 10): the index image is
// 16-bit and the split opponent table has KT = 256 NCH entries, in dynamic LDS
// (8 KT bytes): channel 0's x words first, then -- loaded from global memory
// during channel 0's horizontal pass, once its gathers are done -- the (y, z)
// pairs in the same bytes.
template <int HB, int DE, bool TRIM, int NW, int NCH = 1>
__global__ __launch_bounds__(64 * NW, (cost16w_waves<HB, NCH>())) void cost16w_kernel(CostArgs a, int P_) {
    using Gm = Tile16<HB, NW>;
    constexpr int NTH = 64 * NW, IPR = 8 * NW;  // threads; horizontal items per row pair
    constexpr int TH = kTH16, HR = 4, T2 = 2 * HB, TW = Gm::TW, RWL = Gm::RWL, RW = Gm::RW;
    constexpr int RH = Gm::RH, WH = Gm::WH, NBLK = Gm::NBLK, NSET = Gm::NSET, S = Gm::S, NJ = Gm::NJ;
    constexpr bool PAIR = Gm::PAIR;
    constexpr int AH = Gm::AH;
    constexpr int ROW = 2 * WH, PLANE4 = Gm::PLANE4;
    constexpr int L0 = HB - trim_w(HB, 0), L1 = HB - trim_w(HB, 1), L2 = HB - trim_w(HB, 2);
    static_assert(TW / HR == IPR && 8 * IPR == NTH, "one horizontal item per thread");
    constexpr bool W16 = NCH > 1;
    constexpr int KT = kMaxK * NCH, NTE = KT / NTH;  // table entries (per thread)
    using IT = std::conditional_t<W16, uint16_t, uint8_t>;
    __shared__ f32x4 s_vq[3 * PLANE4];
    __shared__ uint32_t s_ox8[W16 ? 1 : kMaxK];  // opponent x 2^14 as (hi, lo) f16 pairs: channel 0
    __shared__ uint2 s_oyz8[W16 ? 1 : kMaxK];    // channels 1, 2
    __shared__ __attribute__((aligned(16))) IT s_idx[RH * RW];
    extern __shared__ __attribute__((aligned(16))) uint32_t s_tab[];  // W16: 8 KT bytes
    uint32_t* const s_ox = W16 ? s_tab : s_ox8;
    uint2* const s_oyz = W16 ? reinterpret_cast<uint2*>(s_tab) : s_oyz8;
    float* s_v = reinterpret_cast<float*>(s_vq);
    const int tid = threadIdx.x;
    const Geom& g = a.g;
    const TileItem cur = tile_item<TW, TH>(a, xcd_remap(blockIdx.x, a.ntiles * P_), P_);
    const TapsPtr<HB> taps = (TapsPtr<HB>)(uintptr_t)a.taps;  // H taps x 2^-30
    const int lane = tid & 63, wv = tid >> 6, lc = lane & 15, lk = lane >> 4;
    // pair layout: [trim][step][stack][hi, lo][lane] (build_vpass_f16_pair_fragments);
    // else [trim][half][step][stack][hi, lo][lane] (build_vpass_f16_stack_fragments)
    const uint4* frag = (PAIR ? a.vfrag16p : a.vfrag16) + (TRIM ? AH * S * 4 * 2 * 64 : 0) + lane;
    auto F = [&](int half, int s, int st, int hl) { return frag[(((half * S + s) * 4 + st) * 2 + hl) * 64]; };

    std::conditional_t<W16, TileFill16<HB, RWL, RW, TH, NTH>, TileFill<HB, RWL, TH, NTH>> fill;
    fill.issue(a, cur, tid);
    uint32_t tx[W16 ? NTE : 1];  // W16: this thread's x words of the table (entries tid + NTH j)
    if constexpr (W16) {
#pragma unroll
        for (int j = 0; j < NTE; ++j) tx[j] = a.opp16[(int64_t)cur.p * KT + tid + NTH * j].x;
    }
    uint4 A[2][AH][S][2];  // channel 0's stacks (f0, f1), (f2, -); then channels 1-2's
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int h = 0; h < AH; ++h)
#pragma unroll
            for (int s = 0; s < S; ++s) {
                A[st][h][s][0] = F(h, s, st, 0);
                A[st][h][s][1] = F(h, s, st, 1);
            }
    // every entry (zeros for tid >= K): zero-weight rows and the columns past
    // the region gather arbitrary indices, and 0 x NaN would be NaN
    if constexpr (W16) {
#pragma unroll
        for (int j = 0; j < NTE; ++j) s_ox[tid + NTH * j] = tx[j];
        fill.commit(a, s_idx, tid);
    } else {
        if (NTH == kMaxK || tid < kMaxK) {
            s_ox[tid] = fill.ov.x;
            s_oyz[tid] = make_uint2(fill.ov.y, fill.ov.z);
        }
        fill.template commit_idx<RW>(a, s_idx, tid);
    }
    // H item: row pair m, output columns 4j .. 4j+3 (every thread has one)
    const int m = tid / IPR, jr = tid % IPR;
    const int gy0 = cur.y0 + 2 * m, gx0 = cur.x0 + HR * jr;
    const f32x4* hsrc = &s_vq[(m * ROW) / 2];
    f32x2 acc0[HR], acc1[HR], acc2[HR];
#pragma unroll
    for (int xo = 0; xo < HR; ++xo) acc0[xo] = acc1[xo] = acc2[xo] = f32x2{0.f, 0.f};
    __syncthreads();

    // Block b = wset + NW i covers the 16 columns of parity half b & 1 of range
    // b >> 1.  With 10 blocks over 4 waves, sets 0 and 1 hold 3 blocks and sets
    // 2 and 3 hold 2 (18 over 8: sets 0, 1 hold 3): the sets rotate with the
    // workgroup, so the extra blocks do not land on the same SIMDs in every
    // workgroup.
    const int wset = (wv + (int)blockIdx.x) & (NW - 1);
    const int col0 = 32 * (wset >> 1) + 4 * (lc >> 1) + (lc & 1) + 2 * (wset & 1);
    f32x2* const st01 = vstack_base<WH>(s_v, lk < 2 ? 0 : 1, lk, col0);  // stacks -> planes 0, 1
    f32x2* const st2 = vstack_base<WH>(s_v, 2, lk, col0);                // (f2, -) -> plane 2
    // gather of K slot n (rows 4 n + lk) of column col from a table; slots past
    // the region are zero (zero taps), a partly covered slot reads a clamped row
    auto gather_row = [&](int n, int col) {
        const int row = 4 * n + lk;
        return (4 * n + 3 < RH ? row : min(row, RH - 1)) * RW + col;
    };
    // index of a gathered element (timing ablations, wrong results: HQ_ABL_NOIDX
    // skips the index read, HQ_ABL_NOTAB the table read below)
    auto gidx = [&](int n, int col) -> uint32_t {
#ifdef HQ_ABL_NOIDX
        return (uint32_t)(gather_row(n, col) & 255);
#else
        return s_idx[gather_row(n, col)];
#endif
    };

    // ---- channel 0: stacks (f0, f1) -> planes 0, 1 and (f2, -) -> plane 2 ----
#pragma unroll
    for (int i = 0; i < NSET; ++i) {
        const int b = wset + NW * i;
        if (b >= NBLK) break;
        const int col = col0 + 16 * NW * i;
        uint32_t w[NJ];
#pragma unroll
#ifdef HQ_ABL_NOTAB
        for (int n = 0; n < NJ; ++n) w[n] = 4 * n < RH ? gidx(n, col) * 0x00010001u : 0u;
#else
        for (int n = 0; n < NJ; ++n) w[n] = 4 * n < RH ? s_ox[gidx(n, col)] : 0u;
#endif
        f32x4v d[2][2];
        vblock_any<PAIR>(w, A, d);
        store_vstack_at<WH, NW>(st01, d[0][0], i, 0);
        store_vstack_at<WH, NW>(st01, d[0][1], i, 1);
        if (lk < 2) {  // the (f2, -) stack's second filter slot is empty
            store_vstack_at<WH, NW>(st2, d[1][0], i, 0);
            store_vstack_at<WH, NW>(st2, d[1][1], i, 1);
        }
    }
    // channel 1-2 stacks: in flight during channel 0's horizontal pass with one
    // K step (32 VGPRs); with two, loaded after it (64 VGPRs would spill)
    auto load_a12 = [&]() {
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
            for (int h = 0; h < AH; ++h)
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    A[st][h][s][0] = F(h, s, 2 + st, 0);
                    A[st][h][s][1] = F(h, s, 2 + st, 1);
                }
    };
    // (32 fragment VGPRs in flight at most)
    constexpr bool A12_EARLY = AH * S <= 2;
    if constexpr (A12_EARLY) load_a12();
    __syncthreads();
    uint2 tyz[W16 ? NTE : 1];  // W16: the (y, z) words, in flight through channel 0's horizontal pass
    if constexpr (W16) {
#pragma unroll
        for (int j = 0; j < NTE; ++j) {
            const uint4 e = a.opp16[(int64_t)cur.p * KT + tid + NTH * j];
            tyz[j] = make_uint2(e.y, e.z);
        }
    }
    if constexpr (TRIM) hpass_wide<HB, L0, T2 - L0, WH>(hsrc, jr, taps, 0, 0, PLANE4, acc0);
    else hpass_wide<HB, 0, T2, WH>(hsrc, jr, taps, 0, 0, PLANE4, acc0);
    hpass_wide<HB, 0, T2, WH>(hsrc, jr, taps, 1, 1, PLANE4, acc0);
    hpass_wide<HB, 0, T2, WH>(hsrc, jr, taps, 2, 2, PLANE4, acc0);
    if constexpr (W16) {  // (the x words' last reads were the gathers before the barrier)
#pragma unroll
        for (int j = 0; j < NTE; ++j) s_oyz[tid + NTH * j] = tyz[j];
    }
    __syncthreads();

    {
        // ---- channels 1, 2: one gather of (y, z) per region row; stack (f3, f4)
        // -> planes 0, 1 now, stack (f5, f6)'s results held in registers until
        // channel 1's horizontal pass has read the planes ----
        if constexpr (!A12_EARLY) load_a12();
        f32x4v d5[NSET][2];
#pragma unroll
        for (int i = 0; i < NSET; ++i) {
            const int b = wset + NW * i;
            if (b >= NBLK) break;
            const int col = col0 + 16 * NW * i;
            uint32_t wy[NJ], wz[NJ];
#pragma unroll
            for (int n = 0; n < NJ; ++n) {
                if (4 * n < RH) {
#ifdef HQ_ABL_NOTAB
                    const uint32_t ix = gidx(n, col);
                    const uint2 e = make_uint2(ix * 0x00010001u, ix * 0x00020002u);
#else
                    const uint2 e = s_oyz[gidx(n, col)];
#endif
                    wy[n] = e.x; wz[n] = e.y;
                } else {
                    wy[n] = wz[n] = 0u;
                }
            }
            {
                const uint4(&Ay)[1][AH][S][2] = *reinterpret_cast<const uint4(*)[1][AH][S][2]>(&A[0]);
                f32x4v d[1][2];
                vblock_any<PAIR>(wy, Ay, d);
                store_vstack_at<WH, NW>(st01, d[0][0], i, 0);
                store_vstack_at<WH, NW>(st01, d[0][1], i, 1);
            }
            {
                const uint4(&Az)[1][AH][S][2] = *reinterpret_cast<const uint4(*)[1][AH][S][2]>(&A[1]);
                f32x4v d[1][2];
                vblock_any<PAIR>(wz, Az, d);
                d5[i][0] = d[0][0];
                d5[i][1] = d[0][1];
            }
        }
        __syncthreads();
        if constexpr (TRIM) hpass_wide<HB, L1, T2 - L1, WH>(hsrc, jr, taps, 3, 0, PLANE4, acc1);
        else hpass_wide<HB, 0, T2, WH>(hsrc, jr, taps, 3, 0, PLANE4, acc1);
        hpass_wide<HB, 0, T2, WH>(hsrc, jr, taps, 4, 1, PLANE4, acc1);
        __syncthreads();

        // ---- channel 2: stack (f5, f6) -> planes 0, 1 ----
#pragma unroll
        for (int i = 0; i < NSET; ++i) {
            const int b = wset + NW * i;
            if (b >= NBLK) break;
            store_vstack_at<WH, NW>(st01, d5[i][0], i, 0);
            store_vstack_at<WH, NW>(st01, d5[i][1], i, 1);
        }
    }
    // LabRef of the item's 2 x 4 pixels, in flight across the barrier
    float4 lab[2][3];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const bool ok = gy0 + r < g.r1 && gx0 < g.W;
        const uint32_t off = ok ? (uint32_t)((gy0 + r - g.r0) * g.lab_pitch + gx0) : 0u;
#ifdef HQ_ABL_NOLABLD  // timing ablation (wrong results): no LabRef loads
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) lab[r][ch] = make_float4(off, off + 1, off + ch, r);
#else
        const float* src3[3] = {a.labL, a.labA, a.labB};
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            const float4* lp =
                reinterpret_cast<const float4*>(reinterpret_cast<const char*>(src3[ch]) + (off << 2));  // 32-bit byte offset
#if HQ_LAB_NT
            const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(lp));
            lab[r][ch] = make_float4(v.x, v.y, v.z, v.w);
#else
            lab[r][ch] = *lp;
#endif
        }
#endif
    }
    __syncthreads();
    if constexpr (TRIM) hpass_wide<HB, L2, T2 - L2, WH>(hsrc, jr, taps, 5, 0, PLANE4, acc2);
    else hpass_wide<HB, 0, T2, WH>(hsrc, jr, taps, 5, 0, PLANE4, acc2);
    hpass_wide<HB, 0, T2, WH>(hsrc, jr, taps, 6, 1, PLANE4, acc2);

    float e[2][HR];
#if HQ_LAB_SKIPLIN
    // t = X/Xn, Y/Yn, Z/Zn of the item's 8 pixels; when no t of the wave is in
    // the linear Lab segment (t <= delta^3: near-black filtered colours, rare),
    // the cube roots alone (lab_f_root), else lab_f_fast's select (same values)
    float3 tf[2][HR];
    float tmin = INFINITY;
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int xo = 0; xo < HR; ++xo) {
            const float o0 = acc0[xo][r], o1 = acc1[xo][r], o2 = acc2[xo][r];
            tf[r][xo] = make_float3(dot3(o0, o1, o2, a.m_lab + 0), dot3(o0, o1, o2, a.m_lab + 3),
                                    dot3(o0, o1, o2, a.m_lab + 6));
            tmin = fminf(tmin, fminf(tf[r][xo].x, fminf(tf[r][xo].y, tf[r][xo].z)));  // (v_min3; a NaN t drops out)
        }
    if (__builtin_amdgcn_ballot_w64(!(tmin > LAB_DELTA3)) == 0) {
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int xo = 0; xo < HR; ++xo)
                tf[r][xo] = make_float3(lab_f_root(tf[r][xo].x), lab_f_root(tf[r][xo].y), lab_f_root(tf[r][xo].z));
    } else {
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int xo = 0; xo < HR; ++xo)
                tf[r][xo] = make_float3(lab_f_fast(tf[r][xo].x), lab_f_fast(tf[r][xo].y), lab_f_fast(tf[r][xo].z));
    }
#endif
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const float Ls[4] = {lab[r][0].x, lab[r][0].y, lab[r][0].z, lab[r][0].w};
        const float As[4] = {lab[r][1].x, lab[r][1].y, lab[r][1].z, lab[r][1].w};
        const float Bs[4] = {lab[r][2].x, lab[r][2].y, lab[r][2].z, lab[r][2].w};
#pragma unroll
        for (int xo = 0; xo < HR; ++xo) {
#ifdef HQ_ABL_NOLAB  // timing ablation (wrong results): no Opp->Lab / dE
            e[r][xo] = (acc0[xo][r] + acc1[xo][r]) + (acc2[xo][r] + (Ls[xo] + As[xo] + Bs[xo]));
#elif HQ_LAB_SKIPLIN
            e[r][xo] = delta_e_f<DE>(Ls[xo], As[xo], Bs[xo], tf[r][xo]);
#else
            const float3 lf = opp2f_fast(acc0[xo][r], acc1[xo][r], acc2[xo][r], a.m_lab);
            e[r][xo] = delta_e_f<DE>(Ls[xo], As[xo], Bs[xo], lf);
#endif
        }
    }
    if (a.pix_err) {  // test option: the per-pixel dE (CL:201-209's error image)
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int xo = 0; xo < HR; ++xo)
                if (gy0 + r < g.r1 && gx0 + xo < g.W)
                    a.pix_err[(int64_t)cur.p * a.pix_pitch + (int64_t)(gy0 + r - g.r0) * g.W + gx0 + xo] =
                        e[r][xo];
    }
    // tiles inside the image and shard (all but the last tile column and row)
    // sum without per-pixel masks
    float part = 0.f;
    if (cur.x0 + TW <= g.W && cur.y0 + TH <= g.r1) {
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int xo = 0; xo < HR; ++xo) part += e[r][xo];
    } else {
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int xo = 0; xo < HR; ++xo) part += (gy0 + r < g.r1 && gx0 + xo < g.W) ? e[r][xo] : 0.f;
    }
#ifdef HQ_ABL_NORED  // timing ablation (wrong results): no reduction / accumulation
    if (part == 12345.f) a.acc[tid] = 1;
#else
    // each wave adds its own partial: the fixed-point sum is order-free, so no
    // end-of-tile barrier and LDS fold (that form: cost 0.3522 against 0.3499 ms)
    const double sum = wave_sum_to_lane63((double)part);
    if (lane == 63) acc_add(a.acc, a.acc_P, a.acc_p0 + cur.p, cur.tile * NW + wv, sum);
#endif
}

// ----------------------------------------------------------------------------
// Generic two-pass path (any half-width; option cost_variant 1): the reference's
// computeScielabKernelsTemp (CL:234-272) and computeScielabKernelsEnd
// (CL:274-306) restated per pixel through a [7][n_ext] fp32 scratch, one
// palette per launch pair.  It cross-checks the fast path in the tests.
// ----------------------------------------------------------------------------
template <typename IT>
__global__ __launch_bounds__(256) void gen_hpass_kernel(GenArgs a) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= a.g.n_ext) return;
    const int ly = (int)(q / a.g.W), x = (int)(q % a.g.W);
    const IT* row = static_cast<const IT*>(a.idx) + (int64_t)ly * a.g.W;
    float t1x = 0, t1y = 0, t1z = 0, t2x = 0, t2y = 0, t2z = 0, t3 = 0;
    for (int i = -a.half, t = 0; i <= a.half; ++i, ++t) {  // CL:254-267
        const float4 in = a.opp[row[reflect_only(x + i, a.g.W)]];
        t1x = fmaf(in.x, a.k1[4 * t + 0], t1x);
        t1y = fmaf(in.y, a.k1[4 * t + 1], t1y);
        t1z = fmaf(in.z, a.k1[4 * t + 2], t1z);
        t2x = fmaf(in.x, a.k2[4 * t + 0], t2x);
        t2y = fmaf(in.y, a.k2[4 * t + 1], t2y);
        t2z = fmaf(in.z, a.k2[4 * t + 2], t2z);
        t3 = fmaf(in.x, a.k3[t], t3);
    }
    const int64_t n = a.g.n_ext;
    a.t[q] = t1x; a.t[n + q] = t1y; a.t[2 * n + q] = t1z;
    a.t[3 * n + q] = t2x; a.t[4 * n + q] = t2y; a.t[5 * n + q] = t2z;
    a.t[6 * n + q] = t3;
}

template <int DE>
__global__ __launch_bounds__(256) void gen_vpass_kernel(GenArgs a) {
    __shared__ double s_red[4];
    const int own_w = a.g.W;
    const int64_t n_own = (int64_t)own_w * (a.g.r1 - a.g.r0);
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    double e = 0.0;
    if (q < n_own) {
        const int y = a.g.r0 + (int)(q / own_w), x = (int)(q % own_w);
        const int64_t n = a.g.n_ext;
        float ox = 0, oy = 0, oz = 0;
        for (int i = -a.half, t = 0; i <= a.half; ++i, ++t) {  // CL:292-304
            const int64_t s = (int64_t)(reflect_only(y + i, a.g.H) - a.g.e0) * a.g.W + x;
            ox = fmaf(a.t[s], a.k1[4 * t + 0], fmaf(a.t[3 * n + s], a.k2[4 * t + 0], ox));
            oy = fmaf(a.t[n + s], a.k1[4 * t + 1], fmaf(a.t[4 * n + s], a.k2[4 * t + 1], oy));
            oz = fmaf(a.t[2 * n + s], a.k1[4 * t + 2], fmaf(a.t[5 * n + s], a.k2[4 * t + 2], oz));
            ox = fmaf(a.t[6 * n + s], a.absk3[t], ox);
        }
        const float3 lf = opp2f_fast(ox, oy, oz, a.m_lab);
        const int64_t off = (int64_t)(y - a.g.r0) * a.g.lab_pitch + x;
        const float ef = delta_e_f<DE>(a.labL[off], a.labA[off], a.labB[off], lf);
        if (a.pix_err) a.pix_err[q] = ef;  // test option: the per-pixel dE
        e = (double)ef;
    }
    e = wave_sum(e);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = e;
    __syncthreads();
    if (threadIdx.x == 0) acc_add(a.acc, a.P, a.p, blockIdx.x, (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]));
}

// ----------------------------------------------------------------------------
// Tiled generic path (any half-width; the default generic path since round 4,
// and the one half > 24 -- e.g. 300 dpi at 50 cm, half 51 -- takes).  The same
// two passes and the same [7][n_ext] scratch as gen_hpass / gen_vpass, staged
// through LDS so each input feeds many outputs from LDS instead of L1/L2:
// - gen_hrow: grid (ceil(W / 256), extended rows), block 256.  The opponent
//   colours of the row segment x0 - half .. x0 + 255 + half (reflected,
//   CL:256-263) land in LDS once (a float4 each); output x then reads one
//   float4 per tap for its 7 FMAs, in the reference's tap order (CL:254-267).
//   (gen_hpass gathered index and table entry per tap: 2 (2 half + 1) L1 reads.)
// - gen_vtile: grid (64 x 64 output tiles of the owned rows), block 256.  For
//   each filter (plane t1.xyz, t2.xyz, t3 with vertical taps k1.xyz, k2.xyz,
//   |k3|), rows y0 - half .. y0 + 63 + half of the tile's 64 columns land in LDS;
//   thread (column c, row block rb) owns output rows 16 rb .. 16 rb + 15 and runs
//   the taps in chunks of 16: 32 window values from LDS and 16 taps (scalar
//   loads, zero-padded to a multiple of 16) make 256 FMAs.  The filters are
//   summed one after another (the reference interleaves them per tap): the
//   fp32 rounding differs, as in the fast path (1e-6 relative on costs).  Then
//   Opp->Lab, dE and the tile's fixed-point partial.  (gen_vpass read 7 (2 half
//   + 1) floats per output from L2: 2.9 KB at half 51.)
// ----------------------------------------------------------------------------
template <typename IT>
__global__ __launch_bounds__(256) void gen_hrow_kernel(GenArgs a) {
    extern __shared__ float4 s_opp[];  // [256 + 2 half]
    const int tid = threadIdx.x, half = a.half, W = a.g.W;
    const int x0 = blockIdx.x * 256, ly = blockIdx.y;
    const IT* row = static_cast<const IT*>(a.idx) + (int64_t)ly * W;
    for (int e = tid; e < 256 + 2 * half; e += 256) {
        const int x = min(x0 - half + e, W - 1 + half);  // (past the row end: reflected, unused)
        s_opp[e] = a.opp[row[reflect_only(x, W)]];
    }
    __syncthreads();
    const int x = x0 + tid;
    if (x >= W) return;
    float t1x = 0, t1y = 0, t1z = 0, t2x = 0, t2y = 0, t2z = 0, t3 = 0;
    for (int t = 0; t <= 2 * half; ++t) {  // CL:254-267
        const float4 in = s_opp[tid + t];
        t1x = fmaf(in.x, a.k1[4 * t + 0], t1x);
        t1y = fmaf(in.y, a.k1[4 * t + 1], t1y);
        t1z = fmaf(in.z, a.k1[4 * t + 2], t1z);
        t2x = fmaf(in.x, a.k2[4 * t + 0], t2x);
        t2y = fmaf(in.y, a.k2[4 * t + 1], t2y);
        t2z = fmaf(in.z, a.k2[4 * t + 2], t2z);
        t3 = fmaf(in.x, a.k3[t], t3);
    }
    const int64_t n = a.g.n_ext, q = (int64_t)ly * W + x;
    a.t[q] = t1x; a.t[n + q] = t1y; a.t[2 * n + q] = t1z;
    a.t[3 * n + q] = t2x; a.t[4 * n + q] = t2y; a.t[5 * n + q] = t2z;
    a.t[6 * n + q] = t3;
}

// gen_hrow4: the same horizontal pass with 4 adjacent outputs per thread
// (grid (ceil(W / 1024), rows), block 256): a thread slides a window of 7
// colours over its taps in chunks of 4 -- 4 new ds_read_b128 per 4 taps and
// 112 FMAs, against 4 reads per 28 FMAs above, which left gen_hrow bound by
// the LDS reads at large half-widths.  The row segment sits in LDS permuted
// (element e at slot (e & 3) Q + e / 4), so the 64 lanes of a read hit
// consecutive slots.  Each output sums its taps in ascending order (CL:254-
// 267), so the planes equal gen_hrow's bit for bit.
// NO adjacent outputs per thread (4 or 8: option gen_hrow_outputs), a row
// segment of 256 NO outputs per workgroup; element e of the segment sits at
// slot (e % NO) Q + e / NO, so a read's 64 lanes hit consecutive slots.
template <typename IT, bool SPLIT, int NO>
__global__ __launch_bounds__(256) void gen_hrow4_kernel(GenArgs a) {
    extern __shared__ float4 s_opp[];  // [NO][Q] permuted
    constexpr int SEG = 256 * NO, NW = NO + 3;  // window: NO outputs x a chunk of 4 taps
    const int tid = threadIdx.x, half = a.half, W = a.g.W, T = 2 * half + 1;
    const int x0 = blockIdx.x * SEG, ly = blockIdx.y;
    const int Q = (SEG + 2 * half + 3 + NO - 1) / NO;
    const IT* row = static_cast<const IT*>(a.idx) + (int64_t)ly * W;
    // the segment's colours, 8 per thread and batch: every index load of a batch
    // first, then every table load, then the stores (one dependent pair of round
    // trips per batch; a load -> load -> store loop paid two per element)
    for (int e0 = 0; e0 < NO * Q; e0 += 8 * 256) {
        uint32_t ix[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int e = min(e0 + tid + 256 * u, NO * Q - 1);
            const int x = min(x0 - half + e, W - 1 + half);  // (past the row end: reflected, unused)
            ix[u] = (uint32_t)row[reflect_only(x, W)];
        }
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = a.opp[ix[u]];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int e = e0 + tid + 256 * u;
            if (e < NO * Q) s_opp[(e % NO) * Q + e / NO] = v[u];
        }
    }
    __syncthreads();
    float acc[7][NO];
#pragma unroll
    for (int f = 0; f < 7; ++f)
#pragma unroll
        for (int xo = 0; xo < NO; ++xo) acc[f][xo] = 0.f;
    // window w[i] = element NO tid + t0 + i of the segment, i = 0 .. NO + 2
    auto rd = [&](int e) { return s_opp[(e % NO) * Q + e / NO]; };
    float4 w[NW];
#pragma unroll
    for (int i = 0; i < NO - 1; ++i) w[i] = rd(NO * tid + i);
    // taps t: ka = (k1.xyz, k3), kb = (k2.xyz, 0) (a.htaps, packed on the host: a
    // chunk's 4 taps are 2 wide scalar loads, not 7 per tap)
    auto taps_fma = [&](int d, float4 ka, float4 kb) {
#pragma unroll
        for (int xo = 0; xo < NO; ++xo) {
            const float4 in = w[d + xo];
            acc[0][xo] = fmaf(in.x, ka.x, acc[0][xo]);
            acc[1][xo] = fmaf(in.y, ka.y, acc[1][xo]);
            acc[2][xo] = fmaf(in.z, ka.z, acc[2][xo]);
            acc[3][xo] = fmaf(in.x, kb.x, acc[3][xo]);
            acc[4][xo] = fmaf(in.y, kb.y, acc[4][xo]);
            acc[5][xo] = fmaf(in.z, kb.z, acc[5][xo]);
            acc[6][xo] = fmaf(in.x, ka.w, acc[6][xo]);
        }
    };
    const float4* tp = a.htaps;
    int t0 = 0;
    for (; t0 + 4 <= T; t0 += 4) {  // whole chunks
#pragma unroll
        for (int i = NO - 1; i < NW; ++i) w[i] = rd(NO * tid + t0 + i);
#pragma unroll
        for (int d = 0; d < 4; ++d) taps_fma(d, tp[2 * (t0 + d)], tp[2 * (t0 + d) + 1]);
#pragma unroll
        for (int i = 0; i < NO - 1; ++i) w[i] = w[i + 4];
    }
    if (t0 < T) {  // the last taps: guarded (a tap past T is not a zero product on a non-finite colour)
#pragma unroll
        for (int i = NO - 1; i < NW; ++i) w[i] = rd(NO * tid + t0 + i);
#pragma unroll
        for (int d = 0; d < 3; ++d)
            if (t0 + d < T) taps_fma(d, tp[2 * (t0 + d)], tp[2 * (t0 + d) + 1]);
    }
    const int64_t n = a.g.n_ext, q0 = (int64_t)ly * W + x0 + NO * tid;
    const bool whole = (W & 3) == 0 && x0 + NO * tid + NO - 1 < W;  // (planes of n_ext = W rows: 16-B aligned)
    if constexpr (SPLIT) {  // planes of (hi, lo) f16 pairs of x 2^14 for the matrix-core vertical pass
        uint32_t* t = reinterpret_cast<uint32_t*>(a.t);
        if (whole) {
#pragma unroll
            for (int f = 0; f < 7; ++f)
#pragma unroll
                for (int v = 0; v < NO; v += 4)
                    *reinterpret_cast<uint4*>(t + f * n + q0 + v) =
                        make_uint4(split_f16(acc[f][v]), split_f16(acc[f][v + 1]), split_f16(acc[f][v + 2]),
                                   split_f16(acc[f][v + 3]));
        } else {
#pragma unroll
            for (int xo = 0; xo < NO; ++xo)
                if (x0 + NO * tid + xo < W)
#pragma unroll
                    for (int f = 0; f < 7; ++f) t[f * n + q0 + xo] = split_f16(acc[f][xo]);
        }
        return;
    }
    if (whole) {
#pragma unroll
        for (int f = 0; f < 7; ++f)
#pragma unroll
            for (int v = 0; v < NO; v += 4)
                *reinterpret_cast<float4*>(a.t + f * n + q0 + v) =
                    make_float4(acc[f][v], acc[f][v + 1], acc[f][v + 2], acc[f][v + 3]);
    } else {
#pragma unroll
        for (int xo = 0; xo < NO; ++xo)
            if (x0 + NO * tid + xo < W)
#pragma unroll
                for (int f = 0; f < 7; ++f) a.t[f * n + q0 + xo] = acc[f][xo];
    }
}

constexpr int kVtTile = 64, kVtRows = 16;  // gen_vtile: 64 x 64 tiles, 16 output rows per thread
template <int DE>
__global__ __launch_bounds__(256) void gen_vtile_kernel(GenArgs a, int tiles_x) {
    extern __shared__ float s_win[];  // [64 + 2 half][64]
    constexpr int TW = kVtTile, RB = kVtRows;
    __shared__ double s_red[4];
    const int tid = threadIdx.x, c = tid & (TW - 1), rb = tid >> 6;
    const Geom& g = a.g;
    const int x0 = (blockIdx.x % tiles_x) * TW, y0 = g.r0 + (blockIdx.x / tiles_x) * TW;
    const int half = a.half, RH = TW + 2 * half, T = 2 * half + 1;
    const int64_t n = g.n_ext;
    float acc[3][RB];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch)
#pragma unroll
        for (int j = 0; j < RB; ++j) acc[ch][j] = 0.f;
    for (int f = 0; f < kNumFilt; ++f) {
        const float* plane = a.t + (int64_t)f * n;
        const float* vt = a.vtaps + f * a.vtap_pitch;  // zero-padded to a multiple of 16
        __syncthreads();  // (the previous filter's window reads)
        // the window rows, 16 loads per thread in flight per batch (a load ->
        // store loop paid one memory round trip per element: ~42 per filter at
        // half 51, most of the kernel's time)
        const int jx = min(x0 + (tid & (TW - 1)), g.W - 1);
        for (int e0 = 0; e0 < RH * TW; e0 += 16 * 256) {
            float v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int i = min(e0 + tid + 256 * u, RH * TW - 1) / TW;  // (clamped: loaded, not stored)
                int gy = reflect_clamp(y0 - half + i, g.H);
                gy = min(max(gy, g.e0), g.e1 - 1);
                v[u] = plane[(int64_t)(gy - g.e0) * g.W + jx];
            }
#pragma unroll
            for (int u = 0; u < 16; ++u)
                if (e0 + tid + 256 * u < RH * TW) s_win[e0 + tid + 256 * u] = v[u];
        }
        __syncthreads();
        float o[RB];
#pragma unroll
        for (int j = 0; j < RB; ++j) o[j] = 0.f;
        for (int k0 = 0; k0 < T; k0 += 16) {
            float v[RB + 16];
#pragma unroll
            for (int i = 0; i < RB + 16; ++i) v[i] = s_win[min(RB * rb + k0 + i, RH - 1) * TW + c];
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) {
                const float w = vt[k0 + kk];
#pragma unroll
                for (int j = 0; j < RB; ++j) o[j] = fmaf(v[j + kk], w, o[j]);
            }
        }
        // planes: 0 t1.x, 1 t1.y, 2 t1.z, 3 t2.x, 4 t2.y, 5 t2.z, 6 t3 -> channels x y z x y z x
        const int chp = f == 6 ? 0 : f % 3;
#pragma unroll
        for (int j = 0; j < RB; ++j) {
            if (chp == 0) acc[0][j] += o[j];
            else if (chp == 1) acc[1][j] += o[j];
            else acc[2][j] += o[j];
        }
    }
    double part = 0.0;
    const int gx = x0 + c;
#pragma unroll
    for (int j = 0; j < RB; ++j) {
        const int y = y0 + RB * rb + j;
        if (gx < g.W && y < g.r1) {
            const float3 lf = opp2f_fast(acc[0][j], acc[1][j], acc[2][j], a.m_lab);
            const int64_t off = (int64_t)(y - g.r0) * g.lab_pitch + gx;
            const float ef = delta_e_f<DE>(a.labL[off], a.labA[off], a.labB[off], lf);
            if (a.pix_err) a.pix_err[(int64_t)(y - g.r0) * g.W + gx] = ef;  // test option: the per-pixel dE
            part += (double)ef;
        }
    }
    part = wave_sum_to_lane63(part);
    if ((tid & 63) == 63) s_red[tid >> 6] = part;
    __syncthreads();
    if (tid == 0) acc_add(a.acc, a.P, a.p, blockIdx.x, (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]));
}

// gen_vtile2: the vertical pass on 32 x 64 output tiles (half <= kVt2MaxHalf)
// with the filters' windows double-buffered in LDS and filled by LDS DMA
// (global_load_lds_dword: no registers held): filter f + 1's window streams in
// while filter f's taps run, so the fill's memory round trips hide behind the
// FMAs (gen_vtile waits for each window between two barriers).  Thread
// (column c = tid % 32, row block rb = tid / 32) owns output rows 8 rb .. 8 rb
// + 7.  Element e of a window is row e / 32, column e % 32 -- a wave's DMA
// instruction writes 64 consecutive LDS dwords, two window rows.  Same sums
// in the same order as gen_vtile (filters one after another, each filter's
// taps in chunks of 16), so every pixel's dE is bit-identical (the fixed-point
// sums round per tile, and the tiles differ: 2^-20 per partial).
// One filter's window (rows y0 - half .. of the tile's 32 columns, NE = RH x 32
// dwords) from a [n_ext] plane into LDS by DMA.  An image width that is a
// multiple of 4 makes every row segment 16-B aligned: global_load_lds_dwordx4,
// 1 KiB per wave instruction (a lane's 4 dwords: row e4 / 8, columns 4 (e4 % 8)
// .. + 3; the last tile column reads up to 31 elements past its row, which stay
// inside the planes' 256-B tail pad and feed only masked output columns);
// otherwise one dword per lane, columns clamped.  (Dword DMA is 4x the
// instructions, and their issue held the vertical pass.)
template <typename T>
__device__ __forceinline__ void dma_window(const T* plane, T* dst, int NE, int tid, int wv, const Geom& g, int x0,
                                           int y0, int half, bool rows_inside, bool wide) {
    auto row_off = [&](int i) -> uint32_t {
        int gy = y0 - half + i;
        if (!rows_inside) {
            gy = reflect_clamp(gy, g.H);
            gy = min(max(gy, g.e0), g.e1 - 1);
        }
        return (uint32_t)((gy - g.e0) * g.W);
    };
    if (wide) {
        const int NE4 = NE >> 2;
        for (int e0 = 0; e0 < NE4; e0 += 256) {
            const int e = e0 + tid;
            if (e < NE4) {
                const T* src = plane + row_off(e >> 3) + (uint32_t)(x0 + 4 * (e & 7));
                __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(dst + 4 * (e0 + 64 * wv)),
                                                 16, 0, 0);
            }
        }
    } else {
        const int jx = min(x0 + (tid & 31), g.W - 1);
        for (int e0 = 0; e0 < NE; e0 += 256) {
            const int e = e0 + tid;
            if (e < NE) {
                const T* src = plane + row_off(e >> 5) + (uint32_t)jx;
                __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(dst + e0 + 64 * wv), 4, 0, 0);
            }
        }
    }
}

constexpr int kVt2W = 32, kVt2MaxHalf = 64;
#ifndef HQ_VT2_RB
#define HQ_VT2_RB 8  // gen_vtile2: output rows per thread, tiles of 32 x 8 RB (16: 3.677 vs 3.619 ms at 300/50)
#endif
template <int DE, int RB>
__global__ __launch_bounds__(256) void gen_vtile2_kernel(GenArgs a, int tiles_x) {
    extern __shared__ float s_w2[];  // [2][8 RB + 2 half][32]
    constexpr int TW = kVt2W, kVt2H = 8 * RB;
    __shared__ double s_red[4];
    const int tid = threadIdx.x, c = tid & (TW - 1), rb = tid >> 5;
    const Geom& g = a.g;
    const int x0 = (blockIdx.x % tiles_x) * TW, y0 = g.r0 + (blockIdx.x / tiles_x) * kVt2H;
    const int half = a.half, RH = kVt2H + 2 * half, T = 2 * half + 1, NE = RH * TW;
    const int64_t n = g.n_ext;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool rows_inside = y0 - half >= g.e0 && y0 - half >= 0 && y0 + kVt2H + half <= g.e1 && y0 + kVt2H + half <= g.H;
    const bool wide = (g.W & 3) == 0;
    auto issue = [&](int f, int b) {
        dma_window(a.t + (int64_t)f * n, s_w2 + b * NE, NE, tid, wv, g, x0, y0, half, rows_inside, wide);
    };
    float acc[3][RB];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch)
#pragma unroll
        for (int j = 0; j < RB; ++j) acc[ch][j] = 0.f;
    issue(0, 0);
    for (int f = 0; f < kNumFilt; ++f) {
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's rows of window f have landed
        __syncthreads();                     // every wave's rows; window f - 1's readers are done
        if (f + 1 < kNumFilt) issue(f + 1, (f + 1) & 1);
        const float* win = s_w2 + (f & 1) * NE;
        const float* vt = a.vtaps + f * a.vtap_pitch;  // zero-padded to a multiple of 16
        float o[RB];
#pragma unroll
        for (int j = 0; j < RB; ++j) o[j] = 0.f;
        for (int k0 = 0; k0 < T; k0 += 16) {
            float v[RB + 16];
#pragma unroll
            for (int i = 0; i < RB + 16; ++i) v[i] = win[min(RB * rb + k0 + i, RH - 1) * TW + c];
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) {
                const float w = vt[k0 + kk];
#pragma unroll
                for (int j = 0; j < RB; ++j) o[j] = fmaf(v[j + kk], w, o[j]);
            }
        }
        const int chp = f == 6 ? 0 : f % 3;  // planes t1.xyz, t2.xyz, t3 -> channels x y z x y z x
#pragma unroll
        for (int j = 0; j < RB; ++j) {
            if (chp == 0) acc[0][j] += o[j];
            else if (chp == 1) acc[1][j] += o[j];
            else acc[2][j] += o[j];
        }
    }
    double part = 0.0;
    const int gx = x0 + c;
#pragma unroll
    for (int j = 0; j < RB; ++j) {
        const int y = y0 + RB * rb + j;
        if (gx < g.W && y < g.r1) {
            const float3 lf = opp2f_fast(acc[0][j], acc[1][j], acc[2][j], a.m_lab);
            const int64_t off = (int64_t)(y - g.r0) * g.lab_pitch + gx;
            const float ef = delta_e_f<DE>(a.labL[off], a.labA[off], a.labB[off], lf);
            if (a.pix_err) a.pix_err[(int64_t)(y - g.r0) * g.W + gx] = ef;  // test option: the per-pixel dE
            part += (double)ef;
        }
    }
    part = wave_sum_to_lane63(part);
    if ((tid & 63) == 63) s_red[tid >> 6] = part;
    __syncthreads();
    if (tid == 0) acc_add(a.acc, a.P, a.p, blockIdx.x, (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]));
}

// gen_vmfma: the tiled generic path's vertical pass on the matrix cores
// (half <= kVt2MaxHalf), the split-f16 (hi, lo) pair scheme of cost16w's wide
// buckets: gen_hrow4<SPLIT> writes each plane value x as the dword (hi, lo) of
// x 2^14 (split_f16), which is two K slots of the B operand as it stands; A
// holds the vertical taps x 2^16 split on the host, each tap part in both
// slots of a row (build_vtile_dup_taps, read from LDS), the hi parts in one MFMA and
// the lo parts in the next: (t_hi + t_lo)(x_hi + x_lo), every product exact in
// the fp32 accumulator.  A 16 x 16 output block takes K steps of 16 window rows
// (S = ceil((16 + 2 half) / 16)); K slot (g, 2 j + h) of step s is window row
// 16 s + 4 g + j of the block, part h.  The windows are the 32 x (64 + 2 half)
// dword planes of gen_vtile2, double-buffered by LDS DMA.  Wave w owns output
// rows 16 w .. 16 w + 15 of the 64 x 32 tile, both 16-column blocks; a
// channel's filters accumulate into its two D blocks (x 2^30, folded into the
// Lab matrix).
// NRB = 2: wave w owns output rows 32 w .. 32 w + 31 of a 128 x 32 tile.  Block
// 1's B operand of step s is block 0's of step s + 1 (the rows 16 further
// down), so one window read feeds both blocks: D0 += A_b B_b, D1 += A_(b-1) B_b
// over b = 0 .. S; and the (128 + 2 half)-row window re-reads 1.8x the tile's
// rows at half 51 instead of 2.6x.
template <int DE, int NRB>
__global__ __launch_bounds__(256) void gen_vmfma_kernel(GenArgs a, int tiles_x) {
    // [2][TH + 2 half][32] windows, then the duplicated split taps [7][hi, lo][TP]
    extern __shared__ uint32_t s_wm[];
    constexpr int TW = kVt2W, TH = 64 * NRB;
    __shared__ double s_red[4];
    const int tid = threadIdx.x, lane = tid & 63, n = lane & 15, g = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const Geom& gm = a.g;
    const int x0 = (blockIdx.x % tiles_x) * TW, y0 = gm.r0 + (blockIdx.x / tiles_x) * TH;
    const int half = a.half, RH = TH + 2 * half, NE = RH * TW, S = (16 + 2 * half + 15) / 16;
    const int BUF = NE, TP = 16 * S + 16;
    uint32_t* s_tap = s_wm + 2 * BUF;
    // the taps, once per workgroup (their first reads are after the first barrier)
    for (int i = tid; i < kNumFilt * 2 * TP; i += 256) s_tap[i] = a.vtapd[i];
    const int64_t np = gm.n_ext;
    const bool rows_inside = y0 - half >= gm.e0 && y0 - half >= 0 && y0 + TH + half <= gm.e1 && y0 + TH + half <= gm.H;
    const bool wide = (gm.W & 3) == 0;
    auto issue = [&](int f, int b) {
        dma_window(reinterpret_cast<const uint32_t*>(a.t) + (int64_t)f * np, s_wm + b * BUF, NE, tid, wv, gm, x0, y0,
                   half, rows_inside, wide);
    };
    f32x4v D[3][NRB][2];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch)
#pragma unroll
        for (int rb = 0; rb < NRB; ++rb) D[ch][rb][0] = D[ch][rb][1] = f32x4v{0.f, 0.f, 0.f, 0.f};
    issue(0, 0);
    for (int f = 0; f < kNumFilt; ++f) {
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's rows of window f have landed
        __syncthreads();                     // every wave's rows; window f - 1's readers are done
        if (f + 1 < kNumFilt) issue(f + 1, (f + 1) & 1);
        const uint32_t* win = s_wm + (f & 1) * BUF;
        // A of step s: dwords 16 s + 4 g + j - m + 15 (j = 0 .. 3) of the filter's
        // duplicated hi and lo tap rows -- a window sliding over the taps
        // (fragments read from global memory left each filter waiting on L2)
        const uint32_t* th = s_tap + f * 2 * TP + 4 * g - (lane & 15) + 15;
        f32x4v e[NRB][2];
#pragma unroll
        for (int rb = 0; rb < NRB; ++rb) e[rb][0] = e[rb][1] = f32x4v{0.f, 0.f, 0.f, 0.f};
        f16x8 PH = {}, PL = {};  // A of the previous step (block 1)
        for (int bs = 0; bs < S + NRB - 1; ++bs) {
            const int r = TH / 4 * wv + 16 * bs + 4 * g;
            u32x4 b0, b1;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int row = min(r + j, RH - 1);  // (rows past the window: zero taps, finite data)
                b0[j] = win[row * TW + n];
                b1[j] = win[row * TW + 16 + n];
            }
            const f16x8 B0 = __builtin_bit_cast(f16x8, b0), B1 = __builtin_bit_cast(f16x8, b1);
            f16x8 AH = {}, AL = {};
            if (bs < S) {
                uint4 ch, cl;
                ch.x = th[16 * bs]; ch.y = th[16 * bs + 1]; ch.z = th[16 * bs + 2]; ch.w = th[16 * bs + 3];
                cl.x = th[TP + 16 * bs]; cl.y = th[TP + 16 * bs + 1]; cl.z = th[TP + 16 * bs + 2]; cl.w = th[TP + 16 * bs + 3];
                AH = __builtin_bit_cast(f16x8, ch);
                AL = __builtin_bit_cast(f16x8, cl);
                e[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(AH, B0, e[0][0], 0, 0, 0);
                e[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(AH, B1, e[0][1], 0, 0, 0);
                e[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(AL, B0, e[0][0], 0, 0, 0);
                e[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(AL, B1, e[0][1], 0, 0, 0);
            }
            if constexpr (NRB == 2) {
                if (bs >= 1) {
                    e[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(PH, B0, e[1][0], 0, 0, 0);
                    e[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(PH, B1, e[1][1], 0, 0, 0);
                    e[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(PL, B0, e[1][0], 0, 0, 0);
                    e[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(PL, B1, e[1][1], 0, 0, 0);
                }
                PH = AH;
                PL = AL;
            }
        }
        const int chp = f == 6 ? 0 : f % 3;  // planes t1.xyz, t2.xyz, t3 -> channels x y z x y z x
#pragma unroll
        for (int rb = 0; rb < NRB; ++rb) {
            if (chp == 0) { D[0][rb][0] += e[rb][0]; D[0][rb][1] += e[rb][1]; }
            else if (chp == 1) { D[1][rb][0] += e[rb][0]; D[1][rb][1] += e[rb][1]; }
            else { D[2][rb][0] += e[rb][0]; D[2][rb][1] += e[rb][1]; }
        }
    }
    double part = 0.0;
#pragma unroll
    for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int y = y0 + TH / 4 * wv + 16 * rb + 4 * g + i, gx = x0 + 16 * cb + n;
                if (gx < gm.W && y < gm.r1) {
                    // (x 2^-30: the data and tap scales, exactly)
                    const float3 lf = opp2f_fast(D[0][rb][cb][i] * kVOutScale, D[1][rb][cb][i] * kVOutScale,
                                                 D[2][rb][cb][i] * kVOutScale, a.m_lab);
                    const int64_t off = (int64_t)(y - gm.r0) * gm.lab_pitch + gx;
                    const float ef = delta_e_f<DE>(a.labL[off], a.labA[off], a.labB[off], lf);
                    if (a.pix_err) a.pix_err[(int64_t)(y - gm.r0) * gm.W + gx] = ef;  // test option: the per-pixel dE
                    part += (double)ef;
                }
            }
    part = wave_sum_to_lane63(part);
    if ((tid & 63) == 63) s_red[tid >> 6] = part;
    __syncthreads();
    if (tid == 0) acc_add(a.acc, a.P, a.p, blockIdx.x, (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]));
}

// gen_hmfma: the horizontal pass on the matrix cores as well (with gen_vmfma;
// palettes in the fast range): gen_vmfma's pair scheme on its side.  D[m][n] =
// sum_k A[m][k] B[k][n] with m an output column of a 16-column block, n a row
// and k an input column: B of step s for lane (n, g) is columns 16 s + 4 g ..
// + 3 of row n's segment (one ds_read_b128 of split dwords), A the
// horizontal taps' duplicated rows (build_vtile_dup_taps with k3 signed: the
// t3 plane's horizontal taps, CL:254-267).  D's lane holds 4 adjacent output
// columns of one row: one 16-B store of split dwords per plane, which is
// gen_vmfma's input as it stands.  A workgroup: 16 rows x 128 columns (4 waves
// x 2 blocks of 16), rpt such tiles down the image per workgroup; its
// segment the 3 channels' split opponent colours, [3][16][pitch] dwords,
// pitch = 8 mod 64 (ds_read_b128's lane groups then hit 64 distinct banks).
constexpr int kHmCB = 2, kHmCols = 64 * kHmCB;
static int hmfma_seg_cols(int H) { return kHmCols - 16 + 16 * ((16 + 2 * H + 15) / 16); }
static int hmfma_pitch(int H) { return (hmfma_seg_cols(H) - 8 + 63) / 64 * 64 + 8; }
template <typename IT>
__global__ __launch_bounds__(256, 2) void gen_hmfma_kernel(GenArgs a, int pitch, int rpt) {  // (2 waves per SIMD: LDS allows 2 workgroups)
    extern __shared__ uint32_t s_hm[];  // [3][16][pitch] segment, then the taps [7][hi, lo][TP]
    const int tid = threadIdx.x, lane = tid & 63, n = lane & 15, g = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int half = a.half, W = a.g.W, rows = a.g.e1 - a.g.e0;
    const int S = (16 + 2 * half + 15) / 16, TP = 16 * S + 16, SW = kHmCols - 16 + 16 * S;
    const int x0 = blockIdx.x * kHmCols, yb = blockIdx.y * 16 * rpt;
    const int nt = min(rpt, (rows - yb + 15) / 16);  // this workgroup's tiles
    uint32_t* s_tap = s_hm + 3 * 16 * pitch;
    for (int i = tid; i < kNumFilt * 2 * TP; i += 256) s_tap[i] = a.htapd[i];
    // the segment of a tile: column tid of its 16 rows (SW <= 256 for half <= 64).
    // Software pipeline over the tiles: tile t + 1's colours and tile t + 2's
    // indices are in flight while tile t's MFMAs run (the fill's two dependent
    // memory round trips were exposed once per 16 rows)
    const bool act = tid < SW;
    const IT* col = static_cast<const IT*>(a.idx) + reflect_clamp(x0 - half + tid, W);  // (past the row end: masked)
    uint32_t ix[16];
    float vx[16], vy[16], vz[16];  // (12 bytes each: the registers of two waves per SIMD)
    auto load_ix = [&](int t) {
#pragma unroll
        for (int u = 0; u < 16; ++u) ix[u] = act ? (uint32_t)col[(int64_t)min(yb + 16 * t + u, rows - 1) * W] : 0u;
    };
    auto gather = [&]() {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const float* o = reinterpret_cast<const float*>(a.opp + ix[u]);
            vx[u] = o[0];
            vy[u] = o[1];
            vz[u] = o[2];
        }
    };
    load_ix(0);
    gather();
    if (nt > 1) load_ix(1);
    const uint32_t* sb = s_hm + n * pitch + 16 * kHmCB * wv + 4 * g;
    const uint32_t* th = s_tap + 4 * g - n + 15;  // (m = lane & 15 = n)
    uint32_t* tpl = reinterpret_cast<uint32_t*>(a.t);
    const int64_t np = a.g.n_ext;
    for (int t = 0; t < nt; ++t) {
        if (t) __syncthreads();  // tile t - 1's operand reads are done
        if (act) {
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                uint32_t* d = s_hm + u * pitch + tid;
                d[0] = split_f16(vx[u]);
                d[16 * pitch] = split_f16(vy[u]);
                d[32 * pitch] = split_f16(vz[u]);
            }
        }
        __syncthreads();
        if (t + 1 < nt) {
            gather();
            if (t + 2 < nt) load_ix(t + 2);
        }
        f32x4v D[kNumFilt][kHmCB];
#pragma unroll
        for (int f = 0; f < kNumFilt; ++f)
#pragma unroll
            for (int cb = 0; cb < kHmCB; ++cb) D[f][cb] = f32x4v{0.f, 0.f, 0.f, 0.f};
        for (int st = 0; st < S; ++st) {
            f16x8 B[3][kHmCB];
#pragma unroll
            for (int ch = 0; ch < 3; ++ch)
#pragma unroll
                for (int cb = 0; cb < kHmCB; ++cb)
                    B[ch][cb] =
                        __builtin_bit_cast(f16x8, *reinterpret_cast<const u32x4*>(sb + ch * 16 * pitch + 16 * cb + 16 * st));
#pragma unroll
            for (int f = 0; f < kNumFilt; ++f) {
                const int ch = f == 6 ? 0 : f % 3;  // planes t1.xyz, t2.xyz, t3 -> channels x y z x y z x
                const uint32_t* tf = th + f * 2 * TP + 16 * st;
                uint4 ah, al;
                ah.x = tf[0]; ah.y = tf[1]; ah.z = tf[2]; ah.w = tf[3];
                al.x = tf[TP]; al.y = tf[TP + 1]; al.z = tf[TP + 2]; al.w = tf[TP + 3];
                const f16x8 AH = __builtin_bit_cast(f16x8, ah), AL = __builtin_bit_cast(f16x8, al);
#pragma unroll
                for (int cb = 0; cb < kHmCB; ++cb)
                    D[f][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(AH, B[ch][cb], D[f][cb], 0, 0, 0);
#pragma unroll
                for (int cb = 0; cb < kHmCB; ++cb)
                    D[f][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(AL, B[ch][cb], D[f][cb], 0, 0, 0);
            }
        }
        // lane (n, g): plane row y0 + n, columns 4 g .. 4 g + 3 of each block, x 2^-30
        const int y = yb + 16 * t + n;
        if (y < rows) {
#pragma unroll
            for (int cb = 0; cb < kHmCB; ++cb) {
                const int x = x0 + 16 * (kHmCB * wv + cb) + 4 * g;
                const int64_t q = (int64_t)y * W + x;
                if ((W & 3) == 0 && x + 3 < W) {
#pragma unroll
                    for (int f = 0; f < kNumFilt; ++f)
                        *reinterpret_cast<uint4*>(tpl + f * np + q) =
                            make_uint4(split_f16(D[f][cb][0] * kVOutScale), split_f16(D[f][cb][1] * kVOutScale),
                                       split_f16(D[f][cb][2] * kVOutScale), split_f16(D[f][cb][3] * kVOutScale));
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (x + i < W)
#pragma unroll
                            for (int f = 0; f < kNumFilt; ++f) tpl[f * np + q + i] = split_f16(D[f][cb][i] * kVOutScale);
                }
            }
        }
    }
}
template __global__ void gen_hmfma_kernel<uint8_t>(GenArgs, int, int);
template __global__ void gen_hmfma_kernel<uint16_t>(GenArgs, int, int);
template __global__ void gen_hmfma_kernel<uint32_t>(GenArgs, int, int);

// (explicit instantiations: taken only through a generic lambda, the dE94
// kernels' host handles were left undefined by the host compile)
template __global__ void gen_vmfma_kernel<0, 1>(GenArgs, int);
template __global__ void gen_vmfma_kernel<1, 1>(GenArgs, int);
template __global__ void gen_vmfma_kernel<0, 2>(GenArgs, int);
template __global__ void gen_vmfma_kernel<1, 2>(GenArgs, int);
template __global__ void gen_vtile2_kernel<0, HQ_VT2_RB>(GenArgs, int);
template __global__ void gen_vtile2_kernel<1, HQ_VT2_RB>(GenArgs, int);
template __global__ void gen_vtile_kernel<0>(GenArgs, int);
template __global__ void gen_vtile_kernel<1>(GenArgs, int);

// ----------------------------------------------------------------------------
// Host side: tap tables, MFMA fragments, launchers
// ----------------------------------------------------------------------------
// Opp->XYZ (CL:118) with row r divided by the illuminant's component r
// (lab_f_fast works on t = X/Xn, Y/Yn, Z/Zn).
void opp2xyz_over_illum(const float inv_illum[3], float m[9]) {
    static const float opp2xyz[9] = HQ_OPP2XYZ;
    for (int i = 0; i < 9; ++i) m[i] = (float)((double)opp2xyz[i] * inv_illum[i / 3]);
}

// The fast path's tap bucket for a filter half-width H (halfSize, IM:408): the
// smallest of 10, 15, 19, 24 that holds it; 0 = none (H > 24: the generic path).
// 72 dpi / 45 cm (the default) is H = 10, 150 dpi / 30 cm H = 15, 96 dpi /
// 60 cm H = 19: those run without zero taps.
int fast_bucket(int half) {
    return half <= 10 ? 10 : half <= 15 ? 15 : half <= 19 ? 19 : half <= 24 ? 24 : 0;
}

static int bucket_steps(int HB) { return (8 + 2 * HB + 31) / 32; }
// MFMA K steps of 16 region rows per output-row half in the pair layout (cost16w)
static int pair_steps(int HB) { return (8 + 2 * HB + 15) / 16; }

// The 7 filters (f: 0 k1.x, 1 k2.x, 2 k3 (|k3| vertical), 3 k1.y, 4 k2.y,
// 5 k1.z, 6 k2.z) of half-width H centred in 2 HB + 1 taps (zeros around):
// v[f][d], h[f][d], d = 0 .. 2 HB, row-major [7][2 HB + 1].
static void bucket_taps(const float* k1, const float* k2, const float* k3, const float* absk3, int H,
                        int HB, std::vector<float>& v, std::vector<float>& h) {
    const int T = 2 * HB + 1, off = HB - H;
    v.assign(kNumFilt * T, 0.f);
    h.assign(kNumFilt * T, 0.f);
    for (int i = 0; i < 2 * H + 1; ++i) {
        const int d = i + off;
        const float vv[7] = {k1[4 * i], k2[4 * i], absk3[i], k1[4 * i + 1], k2[4 * i + 1], k1[4 * i + 2], k2[4 * i + 2]};
        const float hh[7] = {k1[4 * i], k2[4 * i], k3[i], k1[4 * i + 1], k2[4 * i + 1], k1[4 * i + 2], k2[4 * i + 2]};
        for (int f = 0; f < kNumFilt; ++f) {
            v[f * T + d] = vv[f];
            h[f * T + d] = hh[f];
        }
    }
}

// f32 -> f16 bits, round to nearest even (host; finite inputs well inside the
// f16 range after scaling, subnormal results included).
static uint16_t host_f16(float x) {
    uint32_t u;
    std::memcpy(&u, &x, 4);
    const uint32_t sign = (u >> 16) & 0x8000u;
    const float ax = std::fabs(x);
    if (ax < 5.9604645e-08f * 0.5f) return (uint16_t)sign;          // below half the smallest subnormal
    if (ax < 6.1035156e-05f) {                                        // f16 subnormal: multiples of 2^-24
        const float q = std::nearbyint(ax * 16777216.0f);             // round-half-even (default mode)
        return (uint16_t)(sign | (uint32_t)q);
    }
    uint32_t a = u & 0x7fffffffu;
    const uint32_t mant = a & 0x7fffffu;
    int32_t e = (int32_t)(a >> 23) - 127 + 15;
    uint32_t m = mant >> 13, rem = mant & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (m & 1u))) {
        if (++m == 0x400u) { m = 0; ++e; }
    }
    return (uint16_t)(sign | ((uint32_t)e << 10) | m);
}

static float host_f16_to_f32(uint16_t h) {
    const uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
    const float v = e == 0 ? std::ldexp((float)m, -24) : std::ldexp((float)(m | 0x400u), (int)e - 25);
    return (h & 0x8000u) ? -v : v;
}

// Split-f16 A fragments of v_mfma_f32_16x16x32_f16 for the vertical pass,
// [trim][half][step][stack][hi, lo][lane] x 8 halves (trim 0 = all taps, 1 =
// the narrow filters' significant windows).  Lane l holds A[i = l & 15][k = 8g
// + j], g = l >> 4: the tap (x 2^16) of filter stack[i >> 3] that multiplies
// the region row held in K slot k of step s into output row 8 half + (i & 7),
// i.e. bucket tap d = row - 8 half - (i & 7), zero outside [0, 2 HB] (and
// outside the trimmed window).  The region row of K slot (g, j) is
// kv_row_s(half, s, g, j): half 1 (output rows 8-15 of a 16-row tile) reuses
// six of half 0's slots per lane, so its B operand costs two gathered values
// per lane per step instead of eight.  At HB = 10 (one step) this is also the
// layout cost_mfma_kernel reads (half 0 only).
size_t vpass_f16_stack_fragment_halves(int HB) { return (size_t)2 * 2 * bucket_steps(HB) * 4 * 2 * 64 * 8; }

void build_vpass_f16_stack_fragments(int HB, int H, const float* k1, const float* k2, const float* k3,
                                     const float* absk3, uint16_t* out) {
    std::vector<float> tv, th;
    bucket_taps(k1, k2, k3, absk3, H, HB, tv, th);
    const int T = 2 * HB + 1, S = bucket_steps(HB);
    const int stack[4][2] = {{0, 1}, {2, -1}, {3, 4}, {5, 6}};
    for (int trim = 0; trim < 2; ++trim)
        for (int half = 0; half < 2; ++half)
            for (int s = 0; s < S; ++s)
                for (int st = 0; st < 4; ++st)
                    for (int l = 0; l < 64; ++l)
                        for (int j = 0; j < 8; ++j) {
                            const int i = l & 15, g = l >> 4, r = i & 7, f = stack[st][i >> 3];
                            const int row = kv_row_s(half, s, g, j);
                            const int d = row - 8 * half - r;
                            float w = 0.f;
                            if (f >= 0 && d >= 0 && d < T) {
                                w = tv[f * T + d];
                                const int ch = f == 0 ? 0 : (f == 3 ? 1 : (f == 5 ? 2 : -1));
                                if (trim && ch >= 0 && std::abs(d - HB) > trim_w(HB, ch)) w = 0.f;
                            }
                            w *= kVTapScale;
                            const uint16_t hi = host_f16(w);
                            const uint16_t lo = host_f16(w - host_f16_to_f32(hi));
                            const size_t base = (((((size_t)trim * 2 + half) * S + s) * 4 + st) * 2) * 64;
                            out[((base + 0 * 64) + l) * 8 + j] = hi;
                            out[((base + 1 * 64) + l) * 8 + j] = lo;
                        }
}

// cost16w's A fragments in the (hi, lo) pair layout (see vblock_pair):
// [trim][u][stack][hi, lo][lane] x 8 halves.  Lane l holds A[i = l & 15][k =
// 8 g + 2 j + e], g = l >> 4: K slots 2 j and 2 j + 1 both stand for region row
// 4 (4 u + j) + g (the gathered dword of that row is its (hi, lo) f16 pair), so
// both hold the same tap part -- the tap's hi half in fragment hl = 0, its lo
// half in hl = 1 -- of filter stack[i >> 3] for output row i & 7: bucket tap d =
// row - (i & 7), zero outside [0, 2 HB] (and outside the trimmed window).  Half
// 1 (output rows 8-15) reads the rows 8 further on with the same fragments.
size_t vpass_f16_pair_fragment_halves(int HB) { return (size_t)2 * pair_steps(HB) * 4 * 2 * 64 * 8; }

void build_vpass_f16_pair_fragments(int HB, int H, const float* k1, const float* k2, const float* k3,
                                    const float* absk3, uint16_t* out) {
    std::vector<float> tv, th;
    bucket_taps(k1, k2, k3, absk3, H, HB, tv, th);
    const int T = 2 * HB + 1, U = pair_steps(HB);
    const int stack[4][2] = {{0, 1}, {2, -1}, {3, 4}, {5, 6}};
    for (int trim = 0; trim < 2; ++trim)
        for (int u = 0; u < U; ++u)
            for (int st = 0; st < 4; ++st)
                for (int l = 0; l < 64; ++l)
                    for (int kk = 0; kk < 8; ++kk) {
                        const int i = l & 15, g = l >> 4, r = i & 7, f = stack[st][i >> 3];
                        const int row = 4 * (4 * u + (kk >> 1)) + g;
                        const int d = row - r;
                        float w = 0.f;
                        if (f >= 0 && d >= 0 && d < T) {
                            w = tv[f * T + d];
                            const int ch = f == 0 ? 0 : (f == 3 ? 1 : (f == 5 ? 2 : -1));
                            if (trim && ch >= 0 && std::abs(d - HB) > trim_w(HB, ch)) w = 0.f;
                        }
                        w *= kVTapScale;
                        const uint16_t hi = host_f16(w);
                        const uint16_t lo = host_f16(w - host_f16_to_f32(hi));
                        const size_t base = ((((size_t)trim * U + u) * 4 + st) * 2) * 64;
                        out[((base + 0 * 64) + l) * 8 + kk] = hi;
                        out[((base + 1 * 64) + l) * 8 + kk] = lo;
                    }
}

// gen_vmfma's A operands come from duplicated tap rows (below): in the pair
// layout lane l = (m = l & 15, g = l >> 4) needs, in K slots 2 j + h of step s,
// part h of tap t = 16 s + 4 g + j - m -- a window sliding over the taps.
int vtile_pair_steps(int H) { return (16 + 2 * H + 15) / 16; }
// gen_vmfma's tap rows: [7][hi, lo][TP = 16 S + 16] dwords, entry i the part of
// tap i - 15 x 2^16 in both halves (zero outside 0 .. 2 H): A of step s for
// lane (m, g) is entries 16 s + 4 g - m + 15 .. + 3 of the filter's rows.
size_t vtile_dup_tap_words(int H) { return (size_t)kNumFilt * 2 * (16 * vtile_pair_steps(H) + 16); }
void build_vtile_dup_taps(int H, const float* k1, const float* k2, const float* absk3, uint32_t* out) {
    const int TP = 16 * vtile_pair_steps(H) + 16, T = 2 * H + 1;
    for (int f = 0; f < kNumFilt; ++f)
        for (int i = 0; i < TP; ++i) {
            const int t = i - 15;
            float w = 0.f;
            if (t >= 0 && t < T) w = f < 3 ? k1[4 * t + f] : f < 6 ? k2[4 * t + f - 3] : absk3[t];
            w *= kVTapScale;
            const uint32_t hi = host_f16(w), lo = host_f16(w - host_f16_to_f32((uint16_t)hi));
            out[((size_t)f * 2 + 0) * TP + i] = hi | (hi << 16);
            out[((size_t)f * 2 + 1) * TP + i] = lo | (lo << 16);
        }
}

// The narrow k1 filters' taps outside the bucket's trimmed windows are below
// 1e-9 of their peak (then the fast path may skip them; else it runs all taps).
bool trim_window_ok(const float* k1, int H, int HB) {
    for (int ch = 0; ch < 3; ++ch) {
        float peak = 0.f;
        for (int t = 0; t < 2 * H + 1; ++t) peak = std::max(peak, std::fabs(k1[4 * t + ch]));
        for (int t = 0; t < 2 * H + 1; ++t)
            if (std::abs(t - H) > trim_w(HB, ch) && std::fabs(k1[4 * t + ch]) > 1e-9f * peak) return false;
    }
    return true;
}

template <int HB>
static size_t taps_bytes() { return 2 * sizeof(CostTaps<HB>); }

size_t fast_taps_bytes(int HB) {
    switch (HB) {
    case 10: return taps_bytes<10>();
    case 15: return taps_bytes<15>();
    case 19: return taps_bytes<19>();
    default: return taps_bytes<24>();
    }
}

// [0] the bucket's taps as designed, [1] the same with the horizontal taps
// scaled by 2^-30 (exact) for the matrix-core vertical pass, whose outputs
// carry 2^30.  Layout: two CostTaps<HB>.
void build_fast_taps(int HB, int H, const float* k1, const float* k2, const float* k3, const float* absk3,
                     void* out) {
    std::vector<float> tv, th;
    bucket_taps(k1, k2, k3, absk3, H, HB, tv, th);
    const size_t n = tv.size();  // == sizeof(CostTaps<HB>) / 8
    float* o = static_cast<float*>(out);
    for (int copy = 0; copy < 2; ++copy, o += 2 * n) {
        std::memcpy(o, tv.data(), n * sizeof(float));
        for (size_t i = 0; i < n; ++i) o[n + i] = copy ? th[i] * kVOutScale : th[i];
    }
}

// tile_rows: 8 (cost_mfma_kernel, 8 x 108 tiles) or 16 (cost16w_kernel, 16 x
// tile_w tiles, tile_w = 128 or 256)
void fast_tile_dims(int W, int own_rows, int tile_rows, int tile_w, int* tiles_x, int* ntiles) {
    const int tw = tile_rows == kTH16 ? tile_w : kFastTW;
    *tiles_x = (W + tw - 1) / tw;
    *ntiles = *tiles_x * ((own_rows + tile_rows - 1) / tile_rows);
}

// a.taps = the two CostTaps<HB> of build_fast_taps; [1] carries the vertical
// pass's 2^30 scale in its horizontal taps.  8-row tiles: HB = 10 only.
template <int HB, int NW>
static void launch_cost16w(const CostArgs& a0, int P, int de, bool trim, hipStream_t s) {
    CostArgs a = a0;
    a.taps = static_cast<const char*>(a0.taps) + sizeof(CostTaps<HB>);
    const dim3 grid((unsigned)(a.ntiles * P)), block(64 * NW);
    if (de == 0) {
        if (trim) HQ_LAUNCH((cost16w_kernel<HB, 0, true, NW>), grid, block, 0, s, a, P);
        else HQ_LAUNCH((cost16w_kernel<HB, 0, false, NW>), grid, block, 0, s, a, P);
    } else {
        if (trim) HQ_LAUNCH((cost16w_kernel<HB, 1, true, NW>), grid, block, 0, s, a, P);
        else HQ_LAUNCH((cost16w_kernel<HB, 1, false, NW>), grid, block, 0, s, a, P);
    }
}

// Chunked palettes (nch = 2 .. 16 chunks of 256 colours, 16-bit indices): HB =
// 10, 16 x 128 tiles; the table takes 8 * 256 nch bytes of dynamic LDS.
template <int NCH>
static void launch_cost16w_chunked(const CostArgs& a0, int P, int de, bool trim, hipStream_t s) {
    CostArgs a = a0;
    a.taps = static_cast<const char*>(a0.taps) + sizeof(CostTaps<10>);
    const dim3 grid((unsigned)(a.ntiles * P)), block(256);
    const size_t dyn = 8 * (size_t)kMaxK * NCH;
    auto go = [&](auto kern) {
        // LDS above 64 KB in all (NCH 16: 74 KB)
        if (!allow_dyn_lds(reinterpret_cast<const void*>(kern), dyn)) return;  // (the caller's hipGetLastError)
        HQ_LAUNCH(kern, grid, block, dyn, s, a, P);
    };
    if (de == 0) {
        if (trim) go(cost16w_kernel<10, 0, true, 4, NCH>);
        else go(cost16w_kernel<10, 0, false, 4, NCH>);
    } else {
        if (trim) go(cost16w_kernel<10, 1, true, 4, NCH>);
        else go(cost16w_kernel<10, 1, false, 4, NCH>);
    }
}

hipError_t launch_cost_chunked(const CostArgs& a, int P, int nch, int de, bool trim, hipStream_t s) {
    switch (nch) {
    case 2: launch_cost16w_chunked<2>(a, P, de, trim, s); break;
    case 4: launch_cost16w_chunked<4>(a, P, de, trim, s); break;
    case 8: launch_cost16w_chunked<8>(a, P, de, trim, s); break;
    case 16: launch_cost16w_chunked<16>(a, P, de, trim, s); break;
    case 32: launch_cost16w_chunked<32>(a, P, de, trim, s); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// 256-column tiles (8 waves, 69 KB of LDS at HB = 10): HB = 10 only.
hipError_t launch_cost_fast(const CostArgs& a0, int P, int de, bool trim, int tile_rows, int tile_w, int HB,
                            hipStream_t s) {
    if (tile_rows == kTH16) {
        if (tile_w == 256) {
            if (HB != 10) return hipErrorInvalidValue;
            launch_cost16w<10, 8>(a0, P, de, trim, s);
            return hipGetLastError();
        }
        switch (HB) {
        case 10: launch_cost16w<10, 4>(a0, P, de, trim, s); break;
        case 15: launch_cost16w<15, 4>(a0, P, de, trim, s); break;
        case 19: launch_cost16w<19, 4>(a0, P, de, trim, s); break;
        case 24: launch_cost16w<24, 4>(a0, P, de, trim, s); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    if (HB != 10) return hipErrorInvalidValue;
    CostArgs a = a0;
    a.taps = static_cast<const char*>(a0.taps) + sizeof(CostTaps<10>);
    const dim3 grid((unsigned)(a.ntiles * P));
#define HQ_COST(KN, DEV, TR) HQ_LAUNCH((KN<DEV, TR>), grid, dim3(256), 0, s, a, P)
    if (de == 0) { if (trim) HQ_COST(cost_mfma_kernel, 0, true); else HQ_COST(cost_mfma_kernel, 0, false); }
    else { if (trim) HQ_COST(cost_mfma_kernel, 1, true); else HQ_COST(cost_mfma_kernel, 1, false); }
#undef HQ_COST
    return hipGetLastError();
}

// gen_hrow4 with a.hrow_no outputs per thread (4 or 8)
template <bool SPLIT, int NO>
static void launch_hrow4_no(const GenArgs& a, int idx_bytes, hipStream_t s) {
    constexpr int SEG = 256 * NO;
    const dim3 hg((unsigned)((a.g.W + SEG - 1) / SEG), (unsigned)(a.g.e1 - a.g.e0));
    const size_t hl = sizeof(float4) * NO * (size_t)((SEG + 2 * a.half + 3 + NO - 1) / NO);
    auto go = [&](auto kern) {
        if (!allow_dyn_lds(reinterpret_cast<const void*>(kern), hl)) return;  // (the caller's hipGetLastError)
        HQ_LAUNCH(kern, hg, dim3(256), hl, s, a);
    };
    if (idx_bytes == 4) go(gen_hrow4_kernel<uint32_t, SPLIT, NO>);
    else if (idx_bytes == 2) go(gen_hrow4_kernel<uint16_t, SPLIT, NO>);
    else go(gen_hrow4_kernel<uint8_t, SPLIT, NO>);
}
template <bool SPLIT>
static void launch_hrow4(const GenArgs& a, int idx_bytes, hipStream_t s) {
    if (a.hrow_no == 8) launch_hrow4_no<SPLIT, 8>(a, idx_bytes, s);
    else launch_hrow4_no<SPLIT, 4>(a, idx_bytes, s);
}

// The tiled generic pair (gen_hrow + gen_vtile).  idx_bytes: 1, 2 (chunked
// palettes) or 4 (K > 4096).
hipError_t launch_cost_tiled_generic(const GenArgs& a, int de, int idx_bytes, hipStream_t s) {
    const hipEvent_t ev0 = t_ev_start, ev1 = t_ev_stop;
    t_ev_stop = nullptr;
    const bool vm = a.vmfma && a.vtapd && a.half <= kVt2MaxHalf;  // the matrix-core vertical pass
    if (vm) {
        // workgroup shapes by grid size: the taller forms only when they still
        // give every CU two rounds of work (1024^2: 128-row tiles left 256
        // workgroups, one per CU)
        static const int cus = [] {
            int d = 0, n = 0;
            return hipGetDevice(&d) == hipSuccess &&
                           hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && n > 0
                       ? n
                       : 256;
        }();
        const int rows = a.g.e1 - a.g.e0;
        if (a.hmfma && a.htapd) {  // both passes on the matrix cores
            const int pitch = hmfma_pitch(a.half), S = (16 + 2 * a.half + 15) / 16;
            const size_t hl = sizeof(uint32_t) * (3 * 16 * (size_t)pitch + (size_t)kNumFilt * 2 * (16 * S + 16));
            const int hx = (a.g.W + kHmCols - 1) / kHmCols, tiles = hx * ((rows + 15) / 16);
            // 16-row tiles per workgroup (pipelined fills): 4 on large images
            const int rpt = a.shape == 2 ? 4 : a.shape == 1 ? 1 : tiles >= 16 * cus ? 4 : tiles >= 8 * cus ? 2 : 1;
            const dim3 hg((unsigned)hx, (unsigned)((rows + 16 * rpt - 1) / (16 * rpt)));
            auto goh = [&](auto kern) {
                if (!allow_dyn_lds(reinterpret_cast<const void*>(kern), hl)) return;
                HQ_LAUNCH(kern, hg, dim3(256), hl, s, a, pitch, rpt);
            };
            if (idx_bytes == 4) goh(gen_hmfma_kernel<uint32_t>);
            else if (idx_bytes == 2) goh(gen_hmfma_kernel<uint16_t>);
            else goh(gen_hmfma_kernel<uint8_t>);
        } else {
            launch_hrow4<true>(a, idx_bytes, s);
        }
        t_ev_start = nullptr;
        t_ev_stop = ev1;
        const int tx = (a.g.W + kVt2W - 1) / kVt2W, S = (16 + 2 * a.half + 15) / 16;
        const bool two = a.shape == 2 || (a.shape == 0 && tx * ((a.g.r1 - a.g.r0 + 127) / 128) >= 4 * cus);  // 128-row tiles
        const int vth = two ? 128 : 64, ty = (a.g.r1 - a.g.r0 + vth - 1) / vth;
        const size_t l2 = sizeof(uint32_t) * (2 * kVt2W * (vth + 2 * (size_t)a.half) + (size_t)kNumFilt * 2 * (16 * S + 16));
        auto gov = [&](auto kern) {
            if (!allow_dyn_lds(reinterpret_cast<const void*>(kern), l2)) return;
            HQ_LAUNCH(kern, dim3((unsigned)(tx * ty)), dim3(256), l2, s, a, tx);
        };
        if (two) {
            if (de == 0) gov(gen_vmfma_kernel<0, 2>);
            else gov(gen_vmfma_kernel<1, 2>);
        } else {
            if (de == 0) gov(gen_vmfma_kernel<0, 1>);
            else gov(gen_vmfma_kernel<1, 1>);
        }
        t_ev_start = ev0;
        return hipGetLastError();
    }
    if (a.hrow4) {  // (option gen_hrow4, default on; gen_hrow stays as its bitwise cross-check)
        launch_hrow4<false>(a, idx_bytes, s);
    } else {
        const dim3 hg((unsigned)((a.g.W + 255) / 256), (unsigned)(a.g.e1 - a.g.e0));
        const size_t hl = sizeof(float4) * (256 + 2 * (size_t)a.half);
        if (idx_bytes == 4) HQ_LAUNCH(gen_hrow_kernel<uint32_t>, hg, dim3(256), hl, s, a);
        else if (idx_bytes == 2) HQ_LAUNCH(gen_hrow_kernel<uint16_t>, hg, dim3(256), hl, s, a);
        else HQ_LAUNCH(gen_hrow_kernel<uint8_t>, hg, dim3(256), hl, s, a);
    }
    t_ev_start = nullptr;
    t_ev_stop = ev1;
    if (a.half <= kVt2MaxHalf && a.vtile2) {  // the double-buffered DMA form (option gen_vtile2)
        constexpr int kVt2H = 8 * HQ_VT2_RB;
        const int tx = (a.g.W + kVt2W - 1) / kVt2W, ty = (a.g.r1 - a.g.r0 + kVt2H - 1) / kVt2H;
        const size_t l2 = sizeof(float) * 2 * kVt2W * (kVt2H + 2 * (size_t)a.half);
        auto go2 = [&](auto kern) {
            if (!allow_dyn_lds(reinterpret_cast<const void*>(kern), l2)) return;  // (the caller's hipGetLastError)
            HQ_LAUNCH(kern, dim3((unsigned)(tx * ty)), dim3(256), l2, s, a, tx);
        };
        if (de == 0) go2(gen_vtile2_kernel<0, HQ_VT2_RB>);
        else go2(gen_vtile2_kernel<1, HQ_VT2_RB>);
        t_ev_start = ev0;
        return hipGetLastError();
    }
    const int tiles_x = (a.g.W + kVtTile - 1) / kVtTile, tiles_y = (a.g.r1 - a.g.r0 + kVtTile - 1) / kVtTile;
    const size_t vl = sizeof(float) * kVtTile * (kVtTile + 2 * (size_t)a.half);
    auto go = [&](auto kern) {
        // window rows above 64 KB (half > 95): raise the limit
        if (!allow_dyn_lds(reinterpret_cast<const void*>(kern), vl)) return;  // (the caller's hipGetLastError)
        HQ_LAUNCH(kern, dim3((unsigned)(tiles_x * tiles_y)), dim3(256), vl, s, a, tiles_x);
    };
    if (de == 0) go(gen_vtile_kernel<0>);
    else go(gen_vtile_kernel<1>);
    t_ev_start = ev0;
    return hipGetLastError();
}

// idx_bytes: 1, 2 (chunked palettes) or 4 (K > 4096)
hipError_t launch_cost_generic(const GenArgs& a, int de, int idx_bytes, hipStream_t s) {
    // profiling events (when set) bracket both launches: start on the first, stop on the second
    const hipEvent_t ev0 = t_ev_start, ev1 = t_ev_stop;
    t_ev_stop = nullptr;
    if (idx_bytes == 4) HQ_LAUNCH(gen_hpass_kernel<uint32_t>, dim3(blocks_for(a.g.n_ext)), dim3(256), 0, s, a);
    else if (idx_bytes == 2) HQ_LAUNCH(gen_hpass_kernel<uint16_t>, dim3(blocks_for(a.g.n_ext)), dim3(256), 0, s, a);
    else HQ_LAUNCH(gen_hpass_kernel<uint8_t>, dim3(blocks_for(a.g.n_ext)), dim3(256), 0, s, a);
    t_ev_start = nullptr;
    t_ev_stop = ev1;
    const int64_t n_own = (int64_t)a.g.W * (a.g.r1 - a.g.r0);
    if (de == 0)
        HQ_LAUNCH(gen_vpass_kernel<0>, dim3(blocks_for(n_own)), dim3(256), 0, s, a);
    else
        HQ_LAUNCH(gen_vpass_kernel<1>, dim3(blocks_for(n_own)), dim3(256), 0, s, a);
    t_ev_start = ev0;
    return hipGetLastError();
}

}  // namespace hq
