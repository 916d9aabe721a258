// hq_device.h -- device helpers shared by the gfx950 kernels of libhq:
// colour constants and conversions (CL:77-145), the argmin distance as the
// reference computes it on gfx950 (CL:179-193), dE (CL:201-226), wave
// reductions and the XCD-aware grid relabelling.  Included by every .hip translation unit of the library.
#pragma once

// HQ_ABL_* switches are timing ablations: they drop work and give wrong
// results.  A build that sets one must say so with HQ_ABLATION_BUILD, so a
// stray -D can never produce a library that silently returns wrong costs
// (such a library says so on stderr at every hq_create; tests/test_capi.py
// checks that every HQ_ABL_ name in the sources is listed here).
#if !defined(HQ_ABLATION_BUILD) &&                                                                    \
    (defined(HQ_ABL_NOLOOP) || defined(HQ_ABL_NOSLOW) || defined(HQ_ABL_HASHLOOKUP) ||                \
     defined(HQ_ABL_COHERENT) || defined(HQ_ABL_NOLOOKUP) || defined(HQ_ABL_NOUSED) ||                \
     defined(HQ_ABL_GRID_L1ONLY) || defined(HQ_ABL_TRUNC) || defined(HQ_ABL_NOFILL) ||                \
     defined(HQ_ABL_MFMA1) || defined(HQ_ABL_NOHPASS) || defined(HQ_ABL_NOVSTORE) ||                  \
     defined(HQ_ABL_NOMFMA) || defined(HQ_ABL_NOIDX) || defined(HQ_ABL_NOTAB) ||                      \
     defined(HQ_ABL_NOLABLD) || defined(HQ_ABL_NOLAB) || defined(HQ_ABL_NORED) ||                      \
     defined(HQ_ABL_N16NOL2))
#error "HQ_ABL_* ablations give wrong results: define HQ_ABLATION_BUILD as well to build one"
#endif

#include "hq_internal.h"

#include <hip/hip_ext.h>

#include <math.h>

namespace hq {

// ----------------------------------------------------------------------------
// Colour constants (CL:77, CL:110, CL:118, CL:171; CL:120-123)
// ----------------------------------------------------------------------------
__constant__ float c_RGB2XYZ[9] = {0.4124564f, 0.3575761f, 0.1804375f, 0.2126729f, 0.7151522f,
                                   0.0721750f, 0.0193339f, 0.1191920f, 0.9503041f};
__constant__ float c_XYZ2Opp[9] = {0.2787336f,  0.7218031f, -0.1065520f, -0.4487736f, 0.2898056f,
                                   -0.0771569f, 0.0859513f, -0.5899859f, 0.5011089f};
#define HQ_OPP2XYZ {0.624045f, -1.87044f, -0.155304f, 1.36606f, 0.931563f, \
                   0.433903f, 1.5013f,   1.41761f,  2.53307f}
__constant__ float c_Opp2XYZ[9] = HQ_OPP2XYZ;
__constant__ float c_RGB2Opp[9] = {0.266413f,  0.603167f, 0.00113333f, -0.124957f, 0.0375879f,
                                   -0.133381f, -0.0803345f, -0.331467f, 0.449132f};

#define LAB_DELTA3 (216.0f / 24389.0f)
#define LAB_KAPPA (24389.0f / 27.0f)

__device__ __forceinline__ float dot3(float x, float y, float z, const float* m) {
    return (x * m[0] + y * m[1]) + z * m[2];
}

__device__ __forceinline__ float srgb_lin(float x) {  // CL:85-87, CL:194-196
    return x <= 0.04045f ? x / 12.92f : powf((x + 0.055f) / 1.055f, 2.4f);
}

__device__ __forceinline__ float lab_f(float t) {  // CL:137
    return t > LAB_DELTA3 ? cbrtf(t) : fmaf(LAB_KAPPA, t, 16.0f) * (1.0f / 116.0f);
}

// The hot path's Opp->Lab (CL:124-145): m = Opp->XYZ with row r divided by the
// illuminant's component r (opp2xyz_over_illum), so t = X/Xn etc. is one dot
// product; cube root as exp2(log2(t)/3) (v_log_f32 / v_exp_f32; ~1 ulp over
// t in (delta^3, ~1.1]: log2 t stays small, so its fp32 rounding moves the
// root by ~2e-8 relative on average -- round 3 worked on t' = 116^3 t, whose
// log2 near 20 carried 6x that), the linear segment fma(kappa / 116, t,
// 16 / 116), selected branch-free.
__device__ __forceinline__ float lab_f_fast(float t) {
    // y is only selected for t > delta^3 > 0 (for t <= 0 it is 0 or NaN, discarded)
    const float y = __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(t) * (1.0f / 3.0f));
    const float lin = fmaf(LAB_KAPPA / 116.0f, t, 16.0f / 116.0f);
    return t > LAB_DELTA3 ? y : lin;
}

// lab_f_fast's cube-root branch alone: for a wave whose every t is above
// delta^3 (the caller's ballot), the linear segment and the select are dead.
// (A NaN t gives NaN either way.)
__device__ __forceinline__ float lab_f_root(float t) {
    return __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(t) * (1.0f / 3.0f));
}

// (f(X/Xn), f(Y/Yn), f(Z/Zn)) of an opponent colour: L = 116 f.y - 16,
// a = 500 (f.x - f.y), b = 200 (f.y - f.z).
__device__ __forceinline__ float3 opp2f_fast(float o0, float o1, float o2, const float* m) {
    return make_float3(lab_f_fast(dot3(o0, o1, o2, m + 0)), lab_f_fast(dot3(o0, o1, o2, m + 3)),
                       lab_f_fast(dot3(o0, o1, o2, m + 6)));
}

// CL:124-145 with true division (setup paths: LabRef, quantize/error image).
__device__ __forceinline__ float3 opp2lab_ref(float o0, float o1, float o2, const float* illum) {
    const float X = dot3(o0, o1, o2, c_Opp2XYZ + 0);
    const float Y = dot3(o0, o1, o2, c_Opp2XYZ + 3);
    const float Z = dot3(o0, o1, o2, c_Opp2XYZ + 6);
    const float fx = lab_f(X / illum[0]), fy = lab_f(Y / illum[1]), fz = lab_f(Z / illum[2]);
    return make_float3(116.0f * fy - 16.0f, 500.0f * (fx - fy), 200.0f * (fy - fz));
}

// CL:201-231: dE76 (distance) or dE94.  Hardware square root (v_sqrt_f32, <= 1 ulp):
// HIP's sqrtf is a correctly rounded ~10-instruction sequence, and the
// reference's OpenCL distance()/sqrt on gfx950 is v_sqrt_f32 itself (ref_len
// below); the cost is compared at 1e-6 relative.
__device__ __forceinline__ float hw_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }

template <int DE>
__device__ __forceinline__ float delta_e(float L1, float a1, float b1, float L2, float a2,
                                         float b2) {
    if constexpr (DE == 0) {
        const float dl = L1 - L2, da = a1 - a2, db = b1 - b2;
        return hw_sqrt((dl * dl + da * da) + db * db);
    } else {
        const float dL = L1 - L2;
        const float c1 = hw_sqrt(fmaf(a1, a1, b1 * b1));
        const float dC = c1 - hw_sqrt(fmaf(a2, a2, b2 * b2));
        const float da = a1 - a2, db = b1 - b2;
        const float dH = hw_sqrt(fmaf(da, da, db * db) - dC * dC);
        // CL:223-224: double literals, so 1 + 0.045 c1 in double (not fused), stored as float
        const double c1d = (double)c1;
        const float sc = (float)__dadd_rn(1.0, __dmul_rn(0.045, c1d));
        const float sh = (float)__dadd_rn(1.0, __dmul_rn(0.015, c1d));
        return hw_sqrt(fmaf(dL, dL, fmaf(dC / sc, dC / sc, (dH / sh) * (dH / sh))));
    }
}

// dE (CL:201-226) between a reference Lab and the Lab of f = opp2f_fast(...):
// for dE76 each channel's difference is one fma.
template <int DE>
__device__ __forceinline__ float delta_e_f(float Lr, float Ar, float Br, float3 f) {
    if constexpr (DE == 0) {
        const float dl = fmaf(-116.0f, f.y, Lr + 16.0f);
        const float da = fmaf(-500.0f, f.x - f.y, Ar);
        const float db = fmaf(-200.0f, f.y - f.z, Br);
        return hw_sqrt((dl * dl + da * da) + db * db);
    } else {
        return delta_e<DE>(Lr, Ar, Br, fmaf(116.0f, f.y, -16.0f), 500.0f * (f.x - f.y), 200.0f * (f.y - f.z));
    }
}

// (hi, lo) f16 split of x * 2^14 in one dword, hi in bits 0-15: the vertical
// stencil's MFMA data operand (hq_cost.hip), made once per palette by the prep.
constexpr float kVDataScale = 16384.0f;  // 2^14
__device__ __forceinline__ uint32_t split_f16(float x) {
    const float xs = x * kVDataScale;
    const _Float16 hi = (_Float16)xs;
    const _Float16 lo = (_Float16)(xs - (float)hi);
    return (uint32_t)__builtin_bit_cast(uint16_t, hi) |
           ((uint32_t)__builtin_bit_cast(uint16_t, lo) << 16);
}

// CL:256-263 reflection; clamped so garbage coordinates of partial tiles stay
// in bounds (their results are masked).
__device__ __forceinline__ int reflect_clamp(int j, int n) {
    if (j < 0) j = -j - 1;
    if (j >= n) j = 2 * n - j - 1;
    return min(max(j, 0), n - 1);
}

__device__ __forceinline__ int reflect_only(int j, int n) {
    if (j < 0) return -j - 1;
    if (j >= n) return 2 * n - j - 1;
    return j;
}

// The argmin's distance, CL:179-192 `distance(pixel, colour)`, as the
// reference's own OpenCL build computes it on gfx950 (disassembly of its
// quantize / quantizeAndConvertToOpp kernels, compiled unmodified into
// oracle/_ref by oracle/Makefile):
//   d^2 = fma(dw, dw, fma(dz, dz, fma(dy, dy, dx * dx))),  d = p - c,
//   d = v_sqrt_f32(d^2) for FLT_MIN <= d^2 < inf (or NaN),
// and below FLT_MIN (or at +inf) the library's rescaled form: the components
// times 2^86 (2^-66), the same chain, v_sqrt_f32 with its own ldexp 32 / -16
// step for a subnormal sum, and back by 2^-86 (2^66).  v_sqrt_f32 is monotone
// and within 1 ulp, but not correctly rounded (15.1% of the normal floats are 1
// ulp off: scripts/mb/sqrt_probe.hip, profiles/r06_sqrt_probe.json), so two
// different d^2 can share one distance, and then the lower index wins (strict
// <).  The kernels rank by d^2 (dist2_rank: the same chain, so the same
// value) and re-resolve by ref_len any pixel whose runner-up lies within 1e-6
// relative of its best d^2 or below 2^-125 (near_d2).
__device__ __forceinline__ float ref_len_scaled(float dx, float dy, float dz, float dw, bool small) {
    const float s = small ? 0x1p86f : 0x1p-66f;
    const float x = dx * s, y = dy * s, z = dz * s, w = dw * s;
    float e = __builtin_fmaf(w, w, __builtin_fmaf(z, z, __builtin_fmaf(y, y, x * x)));
    const bool den = e < 0x1p-126f;
    e = __builtin_amdgcn_ldexpf(e, den ? 32 : 0);
    float r = __builtin_amdgcn_sqrtf(e);
    r = __builtin_amdgcn_ldexpf(r, den ? -16 : 0);
    return r * (small ? 0x1p-86f : 0x1p66f);
}
__device__ __forceinline__ float ref_len(float dx, float dy, float dz, float dw) {
    const float d2 = __builtin_fmaf(dw, dw, __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx)));
    if (__builtin_expect(!(d2 < 0x1p-126f) && d2 != INFINITY, 1)) return __builtin_amdgcn_sqrtf(d2);
    return ref_len_scaled(dx, dy, dz, dw, d2 < 0x1p-126f);
}
// pixel (r, g, b, 0) against colour c (whose .w is 0 on every argmin path:
// prep_palette / prep_wide clear it, SW:49)
__device__ __forceinline__ float ref_dist(float r, float g, float b, float4 c) {
    return ref_len(r - c.x, g - c.y, b - c.z, -c.w);
}
// pixel and colour as the reference's float4s (the final quantize, CL:147-170)
__device__ __forceinline__ float ref_dist4(float4 p, float4 c) {
    return ref_len(p.x - c.x, p.y - c.y, p.z - c.z, p.w - c.w);
}

// Ranking distance of the pruned argmin: the reference's d^2 (w = 0).
__device__ __forceinline__ float dist2_rank(float r, float g, float b, float4 c) {
    const float dx = r - c.x, dy = g - c.y, dz = b - c.z;
    return __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
}

// A pixel whose ranking by d^2 may differ from the reference's by distance:
// the runner-up within 1e-6 relative of the best d^2 (v_sqrt_f32 can merge d^2
// up to ~4 ulp apart), or itself below 2^-125 (the rescaled form's distance
// is not a function of the underflowed d^2).
__device__ __forceinline__ bool near_d2(float best2, float second2) {
    return second2 <= __builtin_fmaf(best2, 1.0f + 1e-6f, 0x1p-125f);  // (one v_fma, as the plain bound's v_mul)
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// (byte j of w) << 4 in one instruction (SDWA operand select): a list entry's
// candidate index straight to its 16-byte LDS offset.
__device__ __forceinline__ uint32_t byte_x16(uint32_t w, int j) {
    uint32_t r;
    switch (j) {
    case 0: asm("v_lshlrev_b32_sdwa %0, 4, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(w)); break;
    case 1: asm("v_lshlrev_b32_sdwa %0, 4, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(w)); break;
    case 2: asm("v_lshlrev_b32_sdwa %0, 4, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(w)); break;
    default: asm("v_lshlrev_b32_sdwa %0, 4, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(w)); break;
    }
    return r;
}

// dist2_rank with the x/y differences in one v_pk_add_f32 ({c.x, c.y} sit in
// consecutive registers after the ds_read_b128; rg = {r, g}).  c - p is the
// exact negation of p - c, so the squares and the result are bit-identical.
__device__ __forceinline__ float dist2_rank_pk(f32x2 rg, float b, float4 c) {
    const f32x2 d = f32x2{c.x, c.y} - rg;
    const float dz = c.z - b;
    return __builtin_fmaf(dz, dz, __builtin_fmaf(d.y, d.y, d.x * d.x));
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <typename V>
__device__ __forceinline__ V wave_sum(V v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    return v;
}

// Sum of a double over the wave with DPP moves only (no LDS round trips: the
// __shfl_down tree above is 12 dependent ds_bpermute for an f64).  Fixed order:
// row_shr 1, 2, 4, 8 leave each 16-lane row's sum in its lane 15; row_bcast 15
// and 31 fold the rows into lane 63, which alone holds the total.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_f64(double v) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, ROW_MASK, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, ROW_MASK, 0xf, true);
    return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

__device__ __forceinline__ double wave_sum_to_lane63(double v) {
    v += dpp_f64<0x111, 0xf>(v);  // row_shr:1
    v += dpp_f64<0x112, 0xf>(v);  // row_shr:2
    v += dpp_f64<0x114, 0xf>(v);  // row_shr:4
    v += dpp_f64<0x118, 0xf>(v);  // row_shr:8
    v += dpp_f64<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
    v += dpp_f64<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3
    return v;
}

// k/255 exactly as the host's float division makes it, from byte j of v: the
// product with RN(1/255) is off by one ulp for 126 of the 256 values; one FMA
// residual step corrects all 256 (checked exhaustively, tests/test_assign_u8.py).
__device__ __forceinline__ float u8_unit(uint32_t v, int j) {
    const float k = (float)((v >> (8 * j)) & 0xffu);
    const float c = 1.0f / 255.0f;
    const float q = k * c;
    const float r = __builtin_fmaf(-q, 255.0f, k);
    return __builtin_fmaf(r, c, q);
}

// ----------------------------------------------------------------------------
// The dE sum of a palette (IM:736-768) as a fixed-point integer sum: each
// fp64 partial x (a wave's part of a cost16w tile, a tile of the other tiled
// kernels, or 256 pixels of the generic path) adds
// v = RN(x 2^20) to kAccSlots slot counters of 64 bits (slot = its index mod
// kAccSlots, which spreads the atomics), split as v mod 2^32 into `lo` and
// v >> 32 into `hi` so neither can overflow (2^32 partials of < 2^43).
// Integer addition is associative: the total is the same bits whatever order
// the workgroups finish in, so no partial array and no ordered fold are needed
// (round 3 stored [P][tiles] partials and summed them in a fixed order in
// finalize or the SA step).  Resolution 2^-20 per partial: < 1e-10 relative at
// 4096^2.  A partial that is not a finite number in [0, 2^43) (a NaN pixel,
// an absurd palette) counts in `bad` and makes the sum NaN.
// Layout: [kAccSlots][acc_pitch(P)][4] u64: lo, hi, bad, (pad).
// ----------------------------------------------------------------------------
constexpr double kAccScale = 1048576.0;  // 2^20
__device__ __forceinline__ void acc_add(uint64_t* acc, int P, int p, int slot, double x) {
    uint64_t* a = acc + ((int64_t)(slot & (kAccSlots - 1)) * acc_pitch(P) + p) * 4;
    if (x >= 0.0 && x < 8796093022208.0) {  // 2^43 (NaN fails the test)
        const uint64_t v = (uint64_t)__double2ull_rn(x * kAccScale);
        atomicAdd((unsigned long long*)(a + 0), (unsigned long long)(v & 0xffffffffull));
        if (v >> 32) atomicAdd((unsigned long long*)(a + 1), (unsigned long long)(v >> 32));
    } else {
        atomicAdd((unsigned long long*)(a + 2), 1ull);
    }
}
// The total of palette p (any thread; kAccSlots x 3 loads, issued together).
__device__ __forceinline__ double acc_total(const uint64_t* acc, int P, int p) {
    uint64_t lo = 0, hi = 0, bad = 0;
#pragma unroll
    for (int sl = 0; sl < kAccSlots; ++sl) {
        const uint64_t* a = acc + ((int64_t)sl * acc_pitch(P) + p) * 4;
        lo += a[0];
        hi += a[1];
        bad += a[2];
    }
    // hi 2^12 and lo 2^-20 are exact doubles (hi < 2^41, lo < 2^53): one rounding
    return bad ? __builtin_nan("") : (double)hi * 4096.0 + (double)lo * (1.0 / kAccScale);
}

// Candidate-grid box bounds (build_grid, hq_search.hip; the 16-bit lists,
// hq_lists16.hip).
// Box bounds in fp32.  Box edges are multiples of 1/G (G a power of two):
// exact.  Valid colours are finite (prep_palette routes non-finite palettes to
// the exhaustive path), so every term is a correctly rounded difference,
// squared and summed with non-negative terms: each bound is within 3 ulp
// (2e-7 relative) of its exact value, and the 1e-5 margin covers that on
// both sides of the test on top of the reference's own 1.1e-6.  An fp32
// overflow (|colour| > 1e19) gives inf bounds: T = inf makes every colour a
// candidate, which overflows the list into the exhaustive loop.  (fp64 was
// ~570 VALU instructions per wave at half the fp32 rate.)
__device__ __forceinline__ float ax_min2(float c, float lo, float hi) {
    const float d = fmaxf(fmaxf(lo - c, c - hi), 0.f);
    return d * d;
}
__device__ __forceinline__ float ax_max2(float c, float lo, float hi) {
    const float d = fmaxf(c - lo, hi - c);
    return d * d;
}

#define HQ_CAND_MARGIN (1.0f + 1e-5f)

// ----------------------------------------------------------------------------
// XCD-aware relabelling of a 1-D grid of N workgroups.  Workgroups are placed
// round-robin over the 8 XCDs (b % 8), so XCD x is given the contiguous work
// range starting at x*(N/8) + min(x, N%8): neighbouring work items (the P
// palettes of one tile or pixel block, adjacent tiles) then meet in one L2 and
// LabRef / RGB reach HBM once instead of once per palette.  Bijective for any N;
// placement only affects speed, never results.
__device__ __forceinline__ int xcd_remap(int b, int N) {
    const int q = N >> 3, r = N & 7, x = b & 7, s = b >> 3;
    return x * q + min(x, r) + s;
}

}  // namespace hq
