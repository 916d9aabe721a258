// hq_kernels.hip -- gfx950 kernels of the SWASA dE cost evaluator.
//
// Hot path for one population of P candidate palettes (IM:620-727 restated):
//   prep_palette   : opponent colour per palette entry (CL:194-198), exact
//                    duplicate flags, non-finite guard.
//   build_grid     : exact two-level candidate lists for the argmin (grid over
//                    the RGB cube, bounds in fp64), per palette.
//   assign         : per-pixel palette index (CL:179-193 argmin, bit-exact) +
//                    used-colour bitmask (CL:193); u8 index image in HBM.
//   cost_tile      : S-CIELAB stencil of the quantized image (CL:234-306,
//                    vertical pass first), Opp->Lab (CL:124-145), dE76 vs the
//                    precomputed LabRef (CL:201-209), fp64 per-tile partials.
//   finalize       : deterministic fixed-order fp64 reduction (IM:736-768) and
//                    used-flag OR (-> penalty SW:74-82 on the host).
// Setup / once-per-search kernels: LabRef (CL:79-116, CL:2-74, CL:124-145),
// final quantize (CL:147-170), CIEDE error image (CL:201-231).
//
// Numerical contract of the argmin (frozen, see oracle/oracle.py header):
// d2 = ((dx*dx + dy*dy) + dz*dz) in fp32 with no contraction, ranking by
// sqrtf(d2) (correctly rounded), strict '<' in ascending palette order.
#include "hq_internal.h"

#include <hip/hip_ext.h>

#include <math.h>

#include <algorithm>
#include <cmath>
#include <cstring>

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

// Branch-free f(t) of CL:137 for the hot path: cube root as exp2(log2(t)/3)
// (v_log_f32 / v_exp_f32, about 3 ulp; no Newton step -- the cost tolerance is
// 1e-4 relative and this moves the mean dE by ~1e-7), linear segment selected.
__device__ __forceinline__ float lab_f_fast(float t) {
    const float tc = fmaxf(t, LAB_DELTA3);  // cbrt branch only used for t > delta^3 > 0
    const float y = __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(tc) * (1.0f / 3.0f));
    const float lin = fmaf(LAB_KAPPA, t, 16.0f) * (1.0f / 116.0f);
    return t > LAB_DELTA3 ? y : lin;
}

// CL:124-145 Opp2LAB for the hot path: m = Opp->XYZ with row r divided by the
// illuminant's component r (opp2xyz_over_illum), so X/Xn etc. come out of the
// 3x3 product directly.
__device__ __forceinline__ float3 opp2lab_fast(float o0, float o1, float o2, const float* m) {
    const float fx = lab_f_fast(dot3(o0, o1, o2, m + 0));
    const float fy = lab_f_fast(dot3(o0, o1, o2, m + 3));
    const float fz = lab_f_fast(dot3(o0, o1, o2, m + 6));
    return make_float3(116.0f * fy - 16.0f, 500.0f * (fx - fy), 200.0f * (fy - fz));
}

// CL:124-145 with true division (setup paths: LabRef, quantize/error image).
__device__ __forceinline__ float3 opp2lab_ref(float o0, float o1, float o2, const float* illum) {
    const float X = dot3(o0, o1, o2, c_Opp2XYZ + 0);
    const float Y = dot3(o0, o1, o2, c_Opp2XYZ + 3);
    const float Z = dot3(o0, o1, o2, c_Opp2XYZ + 6);
    const float fx = lab_f(X / illum[0]), fy = lab_f(Y / illum[1]), fz = lab_f(Z / illum[2]);
    return make_float3(116.0f * fy - 16.0f, 500.0f * (fx - fy), 200.0f * (fy - fz));
}

// CL:201-231: dE76 (distance) or dE94.  Hardware square root (v_sqrt_f32, ~1 ulp):
// HIP's sqrtf is a correctly rounded ~10-instruction sequence, and the
// reference's OpenCL distance()/sqrt is itself only ulp-accurate; the cost is
// compared at 1e-4 relative.  (The argmin keeps sqrtf: its ties are exact.)
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
        const float sc = 1.0f + 0.045f * c1, sh = 1.0f + 0.015f * c1;
        return hw_sqrt(fmaf(dL, dL, fmaf(dC / sc, dC / sc, (dH / sh) * (dH / sh))));
    }
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

// Exact argmin distance ((dx*dx + dy*dy) + dz*dz), never fused: hipcc's default
// -ffp-contract=fast would otherwise turn it into FMAs (and differently at
// different call sites), breaking bit-exactness against the oracle.
__device__ __forceinline__ float dist2(float r, float g, float b, float4 c) {
#pragma clang fp contract(off)
    const float dx = r - c.x, dy = g - c.y, dz = b - c.z;
    return (dx * dx + dy * dy) + dz * dz;
}

// Ranking distance of the pruned argmin: the same sum with two FMAs.  All three
// terms are non-negative, so it is within 3 ulp (< 2e-7 relative) of dist2;
// argmin_from_entry re-resolves with dist2 + sqrtf whenever a runner-up lies
// within 1e-6 relative, so the winner it returns is the reference's.
__device__ __forceinline__ float dist2_rank(float r, float g, float b, float4 c) {
    const float dx = r - c.x, dy = g - c.y, dz = b - c.z;
    return __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
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

// ----------------------------------------------------------------------------
// prep_palette: grid (P), block 1024.
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

// Palette prep of palette p by a 1024-thread workgroup; `c` is colour k = tid & 255
// (threads with tid >= 256 pass the same colour as their k).
// Duplicate flags (colour k is a duplicate when an equal colour -- float
// equality per channel -- sits at a lower index; the strict < of the argmin,
// CL:179-193, never picks it, so build_grid leaves it out of lists) by an LDS
// hash table of first occurrences: each colour claims or finds its key's slot
// (open addressing, CAS on a representative index, equality checked against
// the representative's colour), then atomicMin of its index on that slot; k is
// a duplicate when the slot's minimum is below k.  +0/-0 hash alike (they
// compare equal); a NaN channel equals nothing, so such a colour always takes
// a fresh slot of its own.  (An all-pairs scan was O(K^2) VALU on one CU:
// ~5 us per step at K = 256.)
constexpr int kDupSlots = 2 * kMaxK;
__device__ __forceinline__ uint32_t dup_hash(float4 c) {
    const uint32_t x = __float_as_uint(c.x == 0.f ? 0.f : c.x);
    const uint32_t y = __float_as_uint(c.y == 0.f ? 0.f : c.y);
    const uint32_t z = __float_as_uint(c.z == 0.f ? 0.f : c.z);
    const uint32_t h = x * 0x9E3779B1u ^ (y * 0x85EBCA77u + 0x27D4EB2Fu) ^ (z * 0xC2B2AE3Du + 0x165667B1u);
    return (h ^ (h >> 15)) & (kDupSlots - 1);
}

__device__ __forceinline__ void prep_palette_body(const PaletteArgs& a, int p, float4 c) {
    // threads 0..K-1 handle colour k = tid; any block size >= K.
    const int tid = threadIdx.x, k = tid;
    __shared__ float4 s[kMaxK];
    __shared__ uint32_t s_tab[kDupSlots], s_min[kDupSlots];
    __shared__ int s_nonfinite;
    for (int i = tid; i < kDupSlots; i += blockDim.x) { s_tab[i] = ~0u; s_min[i] = ~0u; }
    if (tid == 0) s_nonfinite = 0;
    const bool own = k < a.K;
    if (own) c.w = 0.f;  // SW:49: palettes carry .w = 0
    else c = make_float4(0.f, 0.f, 0.f, 0.f);
    if (own) s[k] = c;
    __syncthreads();
    uint32_t slot = 0;
    if (own) {
        if (!(isfinite(c.x) && isfinite(c.y) && isfinite(c.z))) atomicOr(&s_nonfinite, 1);
        slot = dup_hash(c);
        for (;;) {
            const uint32_t r = atomicCAS(&s_tab[slot], ~0u, (uint32_t)k);
            if (r == ~0u) break;
            const float4 o = s[r];
            if (o.x == c.x && o.y == c.y && o.z == c.z) break;
            slot = (slot + 1) & (kDupSlots - 1);
        }
        atomicMin(&s_min[slot], (uint32_t)k);
    }
    __syncthreads();
    if (own) {
        const float lr = srgb_lin(c.x), lg = srgb_lin(c.y), lb = srgb_lin(c.z);
        const float4 opp = make_float4(dot3(lr, lg, lb, c_RGB2Opp + 0),
                                       dot3(lr, lg, lb, c_RGB2Opp + 3),
                                       dot3(lr, lg, lb, c_RGB2Opp + 6), 0.f);
        a.pal[(int64_t)p * kMaxK + k] = c;
        a.opp[(int64_t)p * kMaxK + k] = opp;
        a.dup[(int64_t)p * kMaxK + k] = s_min[slot] < (uint32_t)k ? 1u : 0u;
    }
    if (tid == 0) a.pflags[p] = s_nonfinite;
}

__global__ __launch_bounds__(1024) void prep_palette_kernel(PaletteArgs a) {
    const int p = blockIdx.x, k = threadIdx.x;
    const float4 c = k < a.K ? a.pal_in[(int64_t)p * a.K + k] : make_float4(0.f, 0.f, 0.f, 0.f);
    prep_palette_body(a, p, c);
}

// ----------------------------------------------------------------------------
// sa_step: one step of the device-resident SWASA search (IM:497-568 with
// SW:54-101), so an iteration needs no host round trip.  Grid (P), block 1024.
//  - accept: the costs of the population just evaluated (finalize's
//    [P][1+K] sums and used flags, all-reduced), C = sum/N + delta * #unused
//    (IM:712; the repeated double additions of a float delta are exact, so the
//    count times delta equals the host's loop), then the acceptance loop
//    (SW:54-57, one next_double per positive delta), best tracking and the
//    convergence loop (SW:59-62, IM:538-545) -- sequential on thread 0 of every
//    workgroup, identically, so no workgroup waits for another;
//  - generate: candidate palette p (SW:91-101 neighbours, or SW:40-52 random at
//    the start), one java.util.Random draw per thread via a jump table
//    (LCG^n = A_n s + C_n mod 2^48), then prep_palette_body.
// State is ping-ponged (in -> out) so no workgroup overwrites what another reads.
// Host-side values that depend only on the iteration (temperature, the
// convergence threshold, the step width) arrive as arguments.
// ----------------------------------------------------------------------------
constexpr uint64_t kLcgMask = (1ull << 48) - 1;
constexpr uint64_t kLcgMult = 0x5DEECE66Dull;

__device__ __forceinline__ int32_t lcg_next(uint64_t& s, int bits) {
    s = (s * kLcgMult + 0xBull) & kLcgMask;
    return (int32_t)(int64_t)(s >> (48 - bits));
}
__device__ __forceinline__ double lcg_next_double(uint64_t& s) {
    const int64_t hi = lcg_next(s, 26), lo = lcg_next(s, 27);
    return (double)((hi << 27) + lo) * (1.0 / (double)(1LL << 53));
}
__device__ __forceinline__ uint64_t lcg_jump(uint64_t s, uint64_t A, uint64_t C) {
    return (A * s + C) & kLcgMask;
}

// Block-shared SA state of one step (thread 0 runs the sequential logic).
struct SaShared {
    int unused[kSaMaxP];
    int src[kSaMaxP];  // >= 0: member p continues from candidate src; -1: keeps its palette
    double cur[kSaMaxP], err[kSaMaxP], ex[kSaMaxP];  // ex: exp(-(err - cur) / T), lanes in parallel
    double sum[kSaMaxP], err_in[kSaMaxP];  // prefetched inputs of the sequential part
    uint64_t seed;     // java.util.Random state (prefetched, then after the acceptance draws)
    double best_in;
    int best;          // candidate that set a new best (-1: none)
};

// Accept step (all threads of the block; returns after a barrier).  `writer`:
// this block writes the shared outputs (errors, best error, next seed).  Every
// global input is loaded before the first barrier, in parallel, so the
// sequential part on thread 0 works from LDS (a chain of dependent global
// loads on one thread was most of this kernel's ~13 us).
__device__ __forceinline__ void sa_accept(const SaArgs& a, bool writer, SaShared& s) {
#pragma clang fp contract(off)
    const int tid = threadIdx.x, nt = blockDim.x, P = a.P, K = a.K;
    constexpr int MAXF = 16;  // used flags per thread held in registers
    const int nf = (P * K + nt - 1) / nt;
    double fv[MAXF];
    if (a.accept) {
        if (tid < P) {
            s.sum[tid] = a.out[(int64_t)tid * (1 + K)];
            s.err_in[tid] = a.err_in[tid];
        }
        if (nf <= MAXF) {
#pragma unroll
            for (int j = 0; j < MAXF; ++j) {
                const int e = tid + j * nt;
                fv[j] = 1.0;
                if (j < nf && e < P * K) {
                    const int i = e / K, k = e - i * K;
                    fv[j] = a.out[(int64_t)i * (1 + K) + 1 + k];
                }
            }
        }
    }
    uint64_t jA = 0, jC = 0;  // the writer's jump past this step's draws
    if (tid == 0) {
        s.seed = *a.seed_in;
        s.best_in = a.accept && !a.init ? *a.best_err : 0.0;
        if (writer && a.generate) { jA = a.jump_A[K * 3 * P]; jC = a.jump_C[K * 3 * P]; }
    }
    if (tid < P) s.unused[tid] = 0;
    __syncthreads();
    if (a.accept) {
        if (nf <= MAXF) {
#pragma unroll
            for (int j = 0; j < MAXF; ++j) {
                const int e = tid + j * nt;
                if (j < nf && e < P * K && fv[j] == 0.0) atomicAdd(&s.unused[e / K], 1);
            }
        } else {
            for (int e = tid; e < P * K; e += nt)
                if (a.out[(int64_t)(e / K) * (1 + K) + 1 + e % K] == 0.0) atomicAdd(&s.unused[e / K], 1);
        }
        __syncthreads();
        if (tid < P) {  // per member, in parallel: error, current, acceptance probability
            const double e = s.sum[tid] / a.n_total + (double)s.unused[tid] * (double)a.delta;
            const double c = a.init ? e : s.err_in[tid];
            s.err[tid] = e;
            s.cur[tid] = c;
            s.ex[tid] = exp(-(e - c) / (double)a.temperature);
            s.src[tid] = a.init ? tid : -1;
        }
        __syncthreads();
        if (tid == 0) {
            uint64_t seed = s.seed;
            double* cur = s.cur;
            const double* err = s.err;
            double best = a.init ? err[0] : s.best_in;
            int best_src = a.init ? 0 : -1;
            if (a.init) {  // IM:490-493: argmin_first
                for (int i = 1; i < P; ++i)
                    if (best > err[i]) { best = err[i]; best_src = i; }
            } else {
                double minerror = 1.7976931348623157e308;
                int minidx = 0;
                for (int i = 0; i < P; ++i) {  // IM:518-537
                    if (P > 1 && err[i] < minerror) { minerror = err[i]; minidx = i; }
                    const double d = err[i] - cur[i];
                    const bool acc = d <= 0 || s.ex[i] > lcg_next_double(seed);
                    if (acc) {
                        cur[i] = err[i];
                        s.src[i] = i;
                        if (cur[i] < best) { best = cur[i]; best_src = i; }
                    }
                }
                for (int i = 0; a.convergence && P > 1 && i < P; ++i) {  // IM:538-545
                    if (!(a.keep_threshold > lcg_next_double(seed))) {
                        cur[i] = minerror;
                        s.src[i] = minidx;
                    }
                }
            }
            s.seed = seed;
            s.best = best_src;
            if (writer) {
                for (int i = 0; i < P; ++i) a.err_out[i] = cur[i];
                *a.best_err = best;
                *a.seed_out = a.generate ? lcg_jump(seed, jA, jC) : seed;
            }
        }
    } else if (tid == 0) {
        s.best = -1;
        for (int i = 0; i < P; ++i) s.src[i] = -1;
        if (writer) {
            for (int i = 0; i < P; ++i) a.err_out[i] = a.err_in[i];
            *a.seed_out = a.generate ? lcg_jump(s.seed, a.jump_A[K * 3 * P], a.jump_C[K * 3 * P]) : s.seed;
        }
    }
    __syncthreads();
}

// Member p's accepted palette into s_from (LDS, 4K floats); `lead` also copies
// it to colors_out (and, for p = 0, a new best to best_colors).  The two likely
// sources -- member p's candidate and its kept palette -- are read before the
// acceptance (pf_cand, pf_col: element tid); only a convergence copy from
// another member's candidate reads after it.
__device__ __forceinline__ void sa_keep(const SaArgs& a, int p, bool lead, const SaShared& s,
                                        float pf_cand, float pf_col, float* s_from) {
    const int n4 = 4 * a.K, tid = threadIdx.x, nt = blockDim.x;
    const int src = s.src[p];
    for (int e = tid; e < n4; e += nt) {
        float v;
        if (e == tid && src == p) v = pf_cand;
        else if (e == tid && src < 0) v = pf_col;
        else v = src >= 0 ? a.cand_in[(int64_t)src * n4 + e] : a.colors_in[(int64_t)p * n4 + e];
        s_from[e] = v;
        if (lead) a.colors_out[(int64_t)p * n4 + e] = v;
    }
    if (lead && p == 0 && s.best >= 0)  // IM:533-536: the best palette so far
        for (int e = tid; e < n4; e += nt) a.best_colors[e] = a.cand_in[(int64_t)s.best * n4 + e];
    __syncthreads();
}

// Candidate p into s_cand (.w = 0; cand_out too when `lead`): draw t = 3i + c of
// this palette's block (SW:91-101 neighbours of s_from, or SW:40-52 random).
// jA/jC: this thread's prefetched jump to its first draw (t = tid).
__device__ __forceinline__ void sa_generate(const SaArgs& a, int p, const float* s_from, uint64_t seed,
                                            float4* s_cand, bool lead, uint64_t jA, uint64_t jC,
                                            uint64_t bA, uint64_t bC) {
#pragma clang fp contract(off)
    const int K = a.K, n4 = 4 * K, tid = threadIdx.x, nt = blockDim.x;
    const uint64_t base = lcg_jump(seed, bA, bC);  // bA, bC: jump_A/C[3Kp], prefetched
    for (int t = tid; t < 3 * K; t += nt) {
        const int i = t / 3, c = t - 3 * i;
        const uint64_t st = t == tid ? lcg_jump(base, jA, jC) : lcg_jump(base, a.jump_A[t + 1], a.jump_C[t + 1]);
        const float u = (float)(int32_t)(st >> 24) / (float)(1 << 24);
        float v;
        if (a.random) {
            v = u;
        } else {
            const float step = (u * 2 - 1) * a.amax;
            const float x = s_from[4 * i + c] + step;
            v = x > 0.f ? (x > 1.f ? 1.f : x) : 0.f;  // clampf_java (SW:103-106)
        }
        reinterpret_cast<float*>(s_cand)[4 * i + c] = v;
        if (lead) a.cand_out[(int64_t)p * n4 + 4 * i + c] = v;
    }
    for (int k = tid; k < K; k += nt) {
        reinterpret_cast<float*>(s_cand)[4 * k + 3] = 0.f;
        if (lead) a.cand_out[(int64_t)p * n4 + 4 * k + 3] = 0.f;
    }
    __syncthreads();
}

// Prefetches of a step, issued before the acceptance: member p's candidate and
// kept palette (element tid) and this thread's jump to draw tid.
struct SaPf {
    float cand = 0.f, col = 0.f;
    uint64_t jA = 0, jC = 0, bA = 0, bC = 0;
    __device__ __forceinline__ void load(const SaArgs& a, int p) {
        const int n4 = 4 * a.K, tid = threadIdx.x;
        if (tid < n4) {
            if (a.accept) cand = a.cand_in[(int64_t)p * n4 + tid];
            col = a.colors_in[(int64_t)p * n4 + tid];
        }
        if (a.generate && tid < 3 * a.K) {
            jA = a.jump_A[tid + 1];
            jC = a.jump_C[tid + 1];
            bA = a.jump_A[3 * a.K * p];
            bC = a.jump_C[3 * a.K * p];
        }
    }
};

// Build with -DHQ_SA_TIMING to print block 0's phase times (accept, keep,
// generate, prep; wall_clock64 ticks of 10 ns) per launch.
__global__ __launch_bounds__(1024) void sa_step_kernel(SaArgs a) {
    const int p = blockIdx.x, K = a.K;
    __shared__ SaShared s;
    __shared__ float s_from[4 * kMaxK];
    __shared__ float4 s_cand[kMaxK];
#ifdef HQ_SA_TIMING
    const uint64_t t0 = wall_clock64();
#endif
    SaPf pf;
    pf.load(a, p);
    sa_accept(a, p == 0, s);
#ifdef HQ_SA_TIMING
    const uint64_t t1 = wall_clock64();
#endif
    sa_keep(a, p, true, s, pf.cand, pf.col, s_from);
#ifdef HQ_SA_TIMING
    const uint64_t t2 = wall_clock64();
#endif
    if (!a.generate) return;
    sa_generate(a, p, s_from, s.seed, s_cand, true, pf.jA, pf.jC, pf.bA, pf.bC);
#ifdef HQ_SA_TIMING
    const uint64_t t3 = wall_clock64();
#endif
    const int k = threadIdx.x;
    prep_palette_body(a.prep, p, k < K ? s_cand[k] : make_float4(0.f, 0.f, 0.f, 0.f));
#ifdef HQ_SA_TIMING
    __syncthreads();
    if (threadIdx.x == 0 && p == 0)
        printf("SA_T %d %d %d %d %d\n", a.accept, (int)(t1 - t0), (int)(t2 - t1), (int)(t3 - t2),
               (int)(wall_clock64() - t3));
#endif
}


// ----------------------------------------------------------------------------
// build_grid: grid (G1^3, P), block 256.  One workgroup per level-1 cell; it
// also writes the 64 level-2 children (G2 = 4*G1).
//
// Exactness: for a closed box B and any pixel p in B, the reference winner k*
// satisfies dmin2(B,k*) <= T(B)*(1+~1.1e-6) with T(B) = min_j dmax2(B,j) (fp32
// rounding of d2 and the sqrt collapse bounded by ~18 ulp); candidates keep
// dmin2 <= T*(1+1e-5).  Children lists are subsets of the parent list, and
// the child's T is attained inside it, so level 2 needs only the parent list.
// Entries: byte0 = count (255 = overflow), then ascending indices.
// ----------------------------------------------------------------------------
__device__ __forceinline__ double ax_min2(double c, double lo, double hi) {
    const double d = fmax(fmax(lo - c, c - hi), 0.0);
    return d * d;
}
__device__ __forceinline__ double ax_max2(double c, double lo, double hi) {
    const double d = fmax(c - lo, hi - c);
    return d * d;
}

#define HQ_CAND_MARGIN (1.0 + 1e-5)

// Level-2 entries are interleaved by groups of 4 palettes: the 4 entries of one
// cell share a 64-byte line, so a pixel evaluated under the 4 palettes of a
// group fetches one line instead of 4 (random 16-B lookups are bound by the
// line fetches they cause, not by their bytes).
__host__ __device__ __forceinline__ int64_t lvl2_offset(int64_t gstride, int p, int64_t cell) {
    return (int64_t)(p >> 2) * gstride + cell * 64 + (p & 3) * 16;
}

// The grid work of level-1 cell `cell` of palette p; thread tid holds colour
// tid (zeros past K) and whether it may be a candidate.  dedup: exact
// duplicates are dropped from the cell's list itself (a colour equal to an
// earlier one has the same bounds, so it is in the list exactly when that one
// is): the lists of the palette-wide dup flags without their O(K^2) scan.
__device__ __forceinline__ void grid_cell_body(const GridArgs& a, int p, int cell, float4 c,
                                               bool valid, bool exh, bool dedup) {
    const int tid = threadIdx.x;
    const int G1 = a.G1, G2 = 4 * G1;
    const int ci = cell / (G1 * G1), cj = (cell / G1) % G1, ck = cell % G1;
    __shared__ float4 s_col[kMaxK];
    __shared__ uint8_t s_list[kMaxK];
    __shared__ double s_min[4];
    __shared__ int s_wcount[4];

    s_col[tid] = c;
    const double inv1 = 1.0 / G1;
    const double lo0 = ci * inv1, hi0 = (ci + 1) * inv1;
    const double lo1 = cj * inv1, hi1 = (cj + 1) * inv1;
    const double lo2 = ck * inv1, hi2 = (ck + 1) * inv1;
    double dmin2 = INFINITY, dmax2 = INFINITY;
    if (valid) {
        dmin2 = ax_min2(c.x, lo0, hi0) + ax_min2(c.y, lo1, hi1) + ax_min2(c.z, lo2, hi2);
        dmax2 = ax_max2(c.x, lo0, hi0) + ax_max2(c.y, lo1, hi1) + ax_max2(c.z, lo2, hi2);
    }
    double m = dmax2;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmin(m, __shfl_xor(m, off, 64));
    const int wave = tid >> 6, lane = tid & 63;
    if (lane == 0) s_min[wave] = m;
    __syncthreads();
    const double T1 = fmin(fmin(s_min[0], s_min[1]), fmin(s_min[2], s_min[3]));
    const bool cand = valid && dmin2 <= T1 * HQ_CAND_MARGIN;
    const uint64_t bal = __ballot(cand);
    if (lane == 0) s_wcount[wave] = __popcll(bal);
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wave; ++w) base += s_wcount[w];
    int total = s_wcount[0] + s_wcount[1] + s_wcount[2] + s_wcount[3];
    if (cand) s_list[base + __popcll(bal & ((1ull << lane) - 1ull))] = (uint8_t)tid;
    __syncthreads();
    if (dedup) {
        bool keep = false;
        int kk = 0;
        if (tid < total) {
            kk = s_list[tid];
            const float4 me = s_col[kk];
            keep = true;
            for (int j = 0; j < tid; ++j) {
                const float4 o = s_col[s_list[j]];
                if (o.x == me.x && o.y == me.y && o.z == me.z) { keep = false; break; }
            }
        }
        __syncthreads();
        const uint64_t bk = __ballot(keep);
        if (lane == 0) s_wcount[wave] = __popcll(bk);
        __syncthreads();
        int b2 = 0;
        for (int w = 0; w < wave; ++w) b2 += s_wcount[w];
        total = s_wcount[0] + s_wcount[1] + s_wcount[2] + s_wcount[3];
        if (keep) s_list[b2 + __popcll(bk & ((1ull << lane) - 1ull))] = (uint8_t)kk;
        __syncthreads();
    }

    uint8_t* l1 = a.lvl1 + (int64_t)p * a.lvl1_pitch + (int64_t)cell * 32;
    const bool ovf1 = exh || total > kL1Cap;
    if (tid < 32) {
        uint8_t v;
        if (tid == 0) v = ovf1 ? kOverflow : (uint8_t)total;
        else v = (!ovf1 && tid - 1 < total) ? s_list[tid - 1] : 0;
        l1[tid] = v;
    }
    // Level 2: child c = tid >> 2 of this cell, its parent-list positions shared
    // by the 4 threads of a quad (q = tid & 3 takes positions q, q+4, ...): T2 and
    // the candidate mask are combined across the quad by shuffles, and each
    // candidate's byte lands at its rank in ascending list order.  (One thread
    // per child walking the list twice, on one wave of the four, made this
    // kernel ~15 us per population.)
    {
        const int ch = tid >> 2, q = tid & 3;
        const int ci2 = ci * 4 + (ch >> 4), cj2 = cj * 4 + ((ch >> 2) & 3), ck2 = ck * 4 + (ch & 3);
        const double inv2 = 1.0 / G2;
        const double l0 = ci2 * inv2, h0 = (ci2 + 1) * inv2;
        const double l1b = cj2 * inv2, h1 = (cj2 + 1) * inv2;
        const double l2 = ck2 * inv2, h2 = (ck2 + 1) * inv2;
        // pass 1: T2 over the whole parent list (which can exceed 31 entries: the
        // level-1 entry then overflows, the children still get lists)
        double t2 = INFINITY;
        for (int i = q; !exh && i < total; i += 4) {
            const float4 cc = s_col[s_list[i]];
            t2 = fmin(t2, ax_max2(cc.x, l0, h0) + ax_max2(cc.y, l1b, h1) + ax_max2(cc.z, l2, h2));
        }
        t2 = fmin(t2, __shfl_xor(t2, 1, 64));
        t2 = fmin(t2, __shfl_xor(t2, 2, 64));
        const double thr = t2 * HQ_CAND_MARGIN;
        // pass 2, 32 positions at a time: candidate mask, ranks in list order
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        int n = 0;  // candidates so far (quad-uniform)
        for (int b0 = 0; !exh && b0 < total && n <= kL2Cap; b0 += 32) {
            uint32_t mine = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int i = b0 + q + 4 * j;
                if (i < total) {
                    const float4 cc = s_col[s_list[i]];
                    const double d = ax_min2(cc.x, l0, h0) + ax_min2(cc.y, l1b, h1) + ax_min2(cc.z, l2, h2);
                    if (d <= thr) mine |= 1u << (q + 4 * j);
                }
            }
            uint32_t M = mine | (uint32_t)__shfl_xor((int)mine, 1, 64);
            M |= (uint32_t)__shfl_xor((int)M, 2, 64);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int r = q + 4 * j;
                if ((mine >> r) & 1u) {
                    const int pos = n + __popc(M & ((1u << r) - 1u)) + 1;  // byte in the entry
                    if (pos <= kL2Cap) w[pos >> 2] |= (uint32_t)s_list[b0 + r] << (8 * (pos & 3));
                }
            }
            n += __popc(M);
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            w[m] |= (uint32_t)__shfl_xor((int)w[m], 1, 64);
            w[m] |= (uint32_t)__shfl_xor((int)w[m], 2, 64);
        }
        if (q == 0) {
            if (exh || n > kL2Cap) { w[0] = kOverflow; w[1] = w[2] = w[3] = 0; }
            else w[0] |= (uint32_t)n;
            uint8_t* l2e = a.lvl2 + lvl2_offset(a.lvl2_gstride, p, (int64_t)(ci2 * G2 + cj2) * G2 + ck2);
            *reinterpret_cast<uint4*>(l2e) = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
}

__global__ __launch_bounds__(256) void build_grid_kernel(GridArgs a) {
    const int p = blockIdx.y, tid = threadIdx.x;
    const bool exh = a.pflags[p] != 0;
    bool valid = false;
    float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tid < a.K) {
        c = a.pal[(int64_t)p * kMaxK + tid];
        valid = !exh && a.dup[(int64_t)p * kMaxK + tid] == 0;
    }
    grid_cell_body(a, p, blockIdx.x, c, valid, exh, false);
}

// sa_step fused with build_grid: grid (G1^3, P), block 256.  Every workgroup
// repeats the (cheap, sequential) acceptance and generates candidate p itself,
// then builds its grid cell from it; cell 0 writes palette p's outputs (the
// state, the candidate, its sanitised colours, opponent table and non-finite
// flag).  Exact duplicates are dropped per cell list (grid_cell_body's dedup),
// so the palette-wide O(K^2) duplicate scan is not needed.  One launch and one
// dependent kernel boundary fewer per SA iteration.
__global__ __launch_bounds__(256) void sa_grid_kernel(SaArgs a, GridArgs ga) {
    const int p = blockIdx.y, cell = blockIdx.x, tid = threadIdx.x, K = a.K;
    const bool lead = cell == 0;
    __shared__ SaShared s;
    __shared__ float s_from[4 * kMaxK];
    __shared__ float4 s_cand[kMaxK];
    SaPf pf;
    pf.load(a, p);
    sa_accept(a, lead && p == 0, s);
    sa_keep(a, p, lead, s, pf.cand, pf.col, s_from);
    sa_generate(a, p, s_from, s.seed, s_cand, lead, pf.jA, pf.jC, pf.bA, pf.bC);
    const float4 c = tid < K ? s_cand[tid] : make_float4(0.f, 0.f, 0.f, 0.f);
    const bool bad = tid < K && !(isfinite(c.x) && isfinite(c.y) && isfinite(c.z));
    const bool nonfinite = __syncthreads_or(bad);
    if (lead && tid < K) {
        const float lr = srgb_lin(c.x), lg = srgb_lin(c.y), lb = srgb_lin(c.z);
        a.prep.pal[(int64_t)p * kMaxK + tid] = c;
        a.prep.opp[(int64_t)p * kMaxK + tid] = make_float4(dot3(lr, lg, lb, c_RGB2Opp + 0),
                                                           dot3(lr, lg, lb, c_RGB2Opp + 3),
                                                           dot3(lr, lg, lb, c_RGB2Opp + 6), 0.f);
        a.prep.dup[(int64_t)p * kMaxK + tid] = 0;
    }
    if (lead && tid == 0) a.prep.pflags[p] = nonfinite;
    grid_cell_body(ga, p, cell, c, tid < K && !nonfinite, nonfinite, true);
}

// ----------------------------------------------------------------------------
// assign: grid (nblocks, P), block 256, dynamic LDS = K*REP*16 bytes.
// Palette replicated REP times in LDS; lane l reads copy (l % REP) so that a
// ds_read_b128 16-lane group never hits one bank position twice (REP = 16).
// ----------------------------------------------------------------------------
// Level-2 entry lookup: returns false (exhaustive) for pixels outside [0,1]^3
// or NaN, and for palettes flagged non-finite.
__device__ __forceinline__ bool lvl2_lookup(float r, float g, float b, const uint8_t* lvl2,
                                            int64_t gstride, int p, int G2, bool exh_pal, uint4& e) {
    const bool inside = r >= 0.f && r <= 1.f && g >= 0.f && g <= 1.f && b >= 0.f && b <= 1.f;
    e = make_uint4(0, 0, 0, 0);
    if (exh_pal || !inside) return false;
    const int ir = min((int)(r * (float)G2), G2 - 1);
    const int ig = min((int)(g * (float)G2), G2 - 1);
    const int ib = min((int)(b * (float)G2), G2 - 1);
    e = *reinterpret_cast<const uint4*>(lvl2 + lvl2_offset(gstride, p, (int64_t)(ir * G2 + ig) * G2 + ib));
    return true;
}

// Reference loop verbatim (CL:179-192) over a candidate list or all K colours.
template <int REP>
__device__ __noinline__ int argmin_exact_slow(float r, float g, float b, uint4 L0, uint4 L1,
                                              int cnt, bool all, const float4* s_pal, int copy,
                                              int K) {
    const uint32_t words[8] = {L0.x, L0.y, L0.z, L0.w, L1.x, L1.y, L1.z, L1.w};
    const int n = all ? K : cnt;
    int bi = all ? 0 : (int)((words[0] >> 8) & 0xff);
    float best = sqrtf(dist2(r, g, b, s_pal[bi * REP + copy]));
    for (int i = 1; i < n; ++i) {
        const int k = all ? i : (int)((words[(i + 1) >> 2] >> (8 * ((i + 1) & 3))) & 0xff);
        const float d = sqrtf(dist2(r, g, b, s_pal[k * REP + copy]));
        if (d < best) { best = d; bi = k; }
    }
    return bi;
}

// Exact argmin (CL:179-193 semantics) over the pixel's candidate list.
// Candidates are ranked by d2; the reference ranks by sqrtf(d2), which can map
// two different d2 onto one distance, and then keeps the lower index.  Equal
// sqrtf values imply |d2a - d2b| < 2^-22 * d2, so lanes whose runner-up d2 lies
// within 1e-6 relative of the best are re-resolved with the reference loop
// (rare).
template <int REP>
__device__ __forceinline__ int argmin_from_entry(float r, float g, float b, uint4 L0, bool listed,
                                                 const float4* s_pal, int copy,
                                                 const uint8_t* lvl1p, int G2, int K) {
    uint4 L1 = make_uint4(0, 0, 0, 0);
    int cnt = listed ? (int)(L0.x & 0xff) : 0;
    bool exh = !listed;
    if (cnt == kOverflow) {  // level-2 overflow: the parent's level-1 list (rare)
        const int G1 = G2 >> 2;
        const int ir = min((int)(r * (float)G2), G2 - 1) >> 2;
        const int ig = min((int)(g * (float)G2), G2 - 1) >> 2;
        const int ib = min((int)(b * (float)G2), G2 - 1) >> 2;
        const uint4* e = reinterpret_cast<const uint4*>(
            lvl1p + ((int64_t)(ir * G1 + ig) * G1 + ib) * 32);
        L0 = e[0];
        L1 = e[1];
        cnt = L0.x & 0xff;
        if (cnt == kOverflow) { exh = true; cnt = 0; }
    }
    int bi = (L0.x >> 8) & 0xff;  // first candidate (lowest index)
    bool near = false;
    if (__any(cnt > 1)) {
        const uint32_t words[8] = {L0.x, L0.y, L0.z, L0.w, L1.x, L1.y, L1.z, L1.w};
        auto cand = [&](int i) { return (int)((words[(i + 1) >> 2] >> (8 * ((i + 1) & 3))) & 0xff); };
        // Ranked by dist2_rank.  best2 <= second2 always, so the runner-up after a
        // new value is the median of the three (v_med3_f32): 4 VALU per candidate
        // to track best, runner-up and index (the compare-and-select form took 7).
        // Slots past a lane's list (build_grid writes index 0 there) rank as +inf.
        const f32x2 rg = {r, g};
        float best2 = dist2_rank(r, g, b, s_pal[bi * REP + copy]);
        float second2 = INFINITY;
        // the next candidate's colour is read while this one is evaluated (the
        // loop is unrolled, so the hand-over is register renaming, not a copy)
        if constexpr (REP == 1) {
            // Candidates tracked by LDS byte offset (index x 16): one SDWA shift
            // takes list byte j straight to the ds_read_b128 address.
            const char* base = reinterpret_cast<const char*>(s_pal);
            auto at = [&](uint32_t off) { return *reinterpret_cast<const float4*>(base + off); };
            auto cand16 = [&](int i) { return byte_x16(words[(i + 1) >> 2], (i + 1) & 3); };
            uint32_t ba = (uint32_t)bi << 4;
            uint32_t an = cand16(1);
            float4 cn = at(an);
#pragma unroll
            for (int i = 1; i < kL1Cap; ++i) {
                if (!__any(i < cnt)) break;
                const uint32_t ak = an;
                const float4 c = cn;
                if (i + 1 < kL1Cap) {
                    an = cand16(i + 1);
                    cn = at(an);
                }
                asm volatile("" ::"v"(c.w));  // keep .w: one ds_read_b128 (16-lane groups), not b96
                const float d2 = i < cnt ? dist2_rank_pk(rg, b, c) : INFINITY;
                const bool lt = d2 < best2;
                ba = lt ? ak : ba;
                second2 = __builtin_amdgcn_fmed3f(best2, second2, d2);
                best2 = lt ? d2 : best2;
            }
            bi = (int)(ba >> 4);
        } else {
        int kn = cand(1);
        float4 cn = s_pal[kn * REP + copy];
#pragma unroll
        for (int i = 1; i < kL1Cap; ++i) {
            if (!__any(i < cnt)) break;
            const int k = kn;
            const float4 c = cn;
            if (i + 1 < kL1Cap) {
                kn = cand(i + 1);
                cn = s_pal[kn * REP + copy];
            }
            asm volatile("" ::"v"(c.w));  // keep .w: one ds_read_b128 (16-lane groups), not b96
            const float d2 = i < cnt ? dist2_rank_pk(rg, b, c) : INFINITY;
            const bool lt = d2 < best2;  // a select, not fminf (which canonicalises its inputs)
            bi = lt ? k : bi;
            second2 = __builtin_amdgcn_fmed3f(best2, second2, d2);
            best2 = lt ? d2 : best2;
        }
        }
        near = second2 <= best2 * (1.0f + 1e-6f);
    }
    if (__any(exh || near)) {
        if (exh || near) bi = argmin_exact_slow<REP>(r, g, b, L0, L1, cnt, exh, s_pal, copy, K);
    }
    return bi;
}

// assign: grid (nblocks * P), block 256, dynamic LDS = K*REP*16 B.  Thread t of
// a chunk handles pixels q0 + (t/64)*64*PPT + (t%64) + 64*j, j < PPT, so every
// pixel load and index store is coalesced across the wave; the next pixel's
// RGB and level-2 entry are loaded while the current one is resolved.
template <int REP>
__global__ __launch_bounds__(256) void assign_kernel(AssignArgs a, int P) {
    constexpr int PPT = 8;
    extern __shared__ __attribute__((aligned(16))) float4 s_pal[];
    __shared__ uint32_t s_used[8];
    // 1-D grid of nblocks * P: work item w = blk * P + p, so the P palettes of
    // one pixel block run side by side on one XCD and share its RGB reads in L2.
    const int w = xcd_remap(blockIdx.x, a.nblocks * P);
    const int p = w % P, blk = w / P, tid = threadIdx.x;
    const float4* pal = a.pal + (int64_t)p * kMaxK;
    for (int e = tid; e < a.K * REP; e += 256) s_pal[e] = pal[e / REP];
    if (tid < 8) s_used[tid] = 0;
    __syncthreads();
    const bool exh_pal = a.pflags[p] != 0 || a.G2 == 0;
    const int copy = tid & (REP - 1);
    const uint8_t* lvl1p = a.lvl1 + (int64_t)p * a.lvl1_pitch;
    uint8_t* idx = a.idx + (int64_t)p * a.idx_pitch;
    const int64_t chunk = 256 * PPT;
    const int64_t lane_off = (int64_t)(tid >> 6) * 64 * PPT + (tid & 63);
    for (int64_t q0 = (int64_t)blk * chunk; q0 < a.n_ext; q0 += (int64_t)a.nblocks * chunk) {
        int64_t q = q0 + lane_off;
        bool in = q < a.n_ext;
        float r = in ? a.R[q] : 0.f, gv = in ? a.G[q] : 0.f, b = in ? a.B[q] : 0.f;
        uint4 e;
        bool li = lvl2_lookup(r, gv, b, a.lvl2, a.lvl2_gstride, p, a.G2, exh_pal, e);
#pragma unroll 1
        for (int j = 0; j < PPT; ++j) {
            // prefetch pixel j+1
            const int64_t qn = q + 64;
            const bool inn = j + 1 < PPT && qn < a.n_ext;
            const float rn = inn ? a.R[qn] : 0.f, gn = inn ? a.G[qn] : 0.f,
                        bn = inn ? a.B[qn] : 0.f;
            uint4 en;
            const bool lin = lvl2_lookup(rn, gn, bn, a.lvl2, a.lvl2_gstride, p, a.G2, exh_pal || !inn, en);
            const int k = argmin_from_entry<REP>(r, gv, b, e, li, s_pal, copy, lvl1p, a.G2, a.K);
            if (in) {
                idx[q] = (uint8_t)k;
                const uint32_t bit = 1u << (k & 31);
                if (!(s_used[k >> 5] & bit)) atomicOr(&s_used[k >> 5], bit);
            }
            q = qn; in = inn; r = rn; gv = gn; b = bn; e = en; li = lin;
        }
    }
    __syncthreads();
    if (tid < 8) a.used_mask[((int64_t)p * a.mask_blocks + a.mask_off + blk) * 8 + tid] = s_used[tid];
}

// assign_batch: the assign kernel with the memory round trips batched.  Per
// chunk, each thread issues the RGB loads of all its PPT pixels, then the
// level-2 entry loads of all of them (they need the RGB), then resolves the PPT
// pixels from LDS: two round trips per PPT pixels.  (assign_kernel prefetches one
// pixel ahead, but the next pixel's level-2 lookup waits for its RGB at once,
// so each pixel there pays an HBM round trip of its own.)
template <int REP, int PPT>
__global__ __launch_bounds__(256) void assign_batch_kernel(AssignArgs a, int P) {
    extern __shared__ __attribute__((aligned(16))) float4 s_pal[];
    __shared__ uint32_t s_used[8];
    // 1-D grid of nblocks * P: work item w = blk * P + p, so the P palettes of
    // one pixel block run side by side on one XCD and share its RGB reads in L2.
    const int w = xcd_remap(blockIdx.x, a.nblocks * P);
    const int p = w % P, blk = w / P, tid = threadIdx.x;
    const float4* pal = a.pal + (int64_t)p * kMaxK;
    for (int e = tid; e < a.K * REP; e += 256) s_pal[e] = pal[e / REP];
    if (tid < 8) s_used[tid] = 0;
    __syncthreads();
    const bool exh_pal = a.pflags[p] != 0 || a.G2 == 0;
    const int copy = tid & (REP - 1);
    const uint8_t* lvl1p = a.lvl1 + (int64_t)p * a.lvl1_pitch;
    uint8_t* idx = a.idx + (int64_t)p * a.idx_pitch;
    const int64_t chunk = 256 * PPT;
    const int64_t lane_off = (int64_t)(tid >> 6) * 64 * PPT + (tid & 63);
    for (int64_t q0 = (int64_t)blk * chunk; q0 < a.n_ext; q0 += (int64_t)a.nblocks * chunk) {
        const int64_t qb = q0 + lane_off;
        float r[PPT], gv[PPT], b[PPT];
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const int64_t q = qb + 64 * j;
            const bool in = q < a.n_ext;
            r[j] = in ? a.R[q] : 0.f;
            gv[j] = in ? a.G[q] : 0.f;
            b[j] = in ? a.B[q] : 0.f;
        }
        uint4 e[PPT];
        bool li[PPT];
#pragma unroll
        for (int j = 0; j < PPT; ++j)
            li[j] = lvl2_lookup(r[j], gv[j], b[j], a.lvl2, a.lvl2_gstride, p, a.G2,
                                exh_pal || qb + 64 * j >= a.n_ext, e[j]);
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const int64_t q = qb + 64 * j;
            const int k = argmin_from_entry<REP>(r[j], gv[j], b[j], e[j], li[j], s_pal, copy, lvl1p,
                                                 a.G2, a.K);
            if (q < a.n_ext) {
                idx[q] = (uint8_t)k;
                const uint32_t bit = 1u << (k & 31);
                if (!(s_used[k >> 5] & bit)) atomicOr(&s_used[k >> 5], bit);
            }
        }
    }
    __syncthreads();
    if (tid < 8) a.used_mask[((int64_t)p * a.mask_blocks + a.mask_off + blk) * 8 + tid] = s_used[tid];
}

// assign_quad: the batched assign for a group of up to 4 palettes.  One pixel
// pass serves the group: the pixel's RGB is read once, its cell index computed
// once, and the group's 4 level-2 entries -- one 64-byte line of the
// interleaved table -- arrive in one line fetch.  (Per palette, the random
// 16-B lookups of assign_batch_kernel each pull a line from L2, and those
// fetches, not the candidate loop, bound it: a fixed-cell ablation ran 40%
// faster, a loop-free one 4%.)  Grid: nblocks * ceil(P/4), XCD-relabelled;
// dynamic LDS = 4 * K * 16 B.
template <int PPT>
__global__ __launch_bounds__(256) void assign_quad_kernel(AssignArgs a, int P) {
    extern __shared__ __attribute__((aligned(16))) float4 s_pal[];  // [4][K]
    __shared__ uint32_t s_used[4][8];
    const int ngroups = (P + 3) / 4;
    const int w = xcd_remap(blockIdx.x, a.nblocks * ngroups);
    const int grp = w % ngroups, blk = w / ngroups, tid = threadIdx.x;
    const int p0 = 4 * grp, ng = min(4, P - p0);
    for (int e = tid; e < ng * a.K; e += 256) {
        const int pp = e / a.K, k = e - pp * a.K;
        s_pal[e] = a.pal[(int64_t)(p0 + pp) * kMaxK + k];
    }
    if (tid < 32) s_used[tid >> 3][tid & 7] = 0;
    __syncthreads();
    bool exh_pal[4];
#pragma unroll
    for (int pp = 0; pp < 4; ++pp) exh_pal[pp] = pp >= ng || a.pflags[p0 + min(pp, ng - 1)] != 0 || a.G2 == 0;
    const uint8_t* lines = a.lvl2 + (int64_t)grp * a.lvl2_gstride;
    const int G2 = a.G2 > 0 ? a.G2 : 4;
    const int64_t chunk = 256 * PPT;
    const int64_t lane_off = (int64_t)(tid >> 6) * 64 * PPT + (tid & 63);
    for (int64_t q0 = (int64_t)blk * chunk; q0 < a.n_ext; q0 += (int64_t)a.nblocks * chunk) {
        const int64_t qb = q0 + lane_off;
        float r[PPT], gv[PPT], b[PPT];
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const int64_t q = qb + 64 * j;
            const bool in = q < a.n_ext;
            r[j] = in ? a.R[q] : 0.f;
            gv[j] = in ? a.G[q] : 0.f;
            b[j] = in ? a.B[q] : 0.f;
        }
        uint4 e[PPT][4];
        bool inside[PPT];
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            inside[j] = qb + 64 * j < a.n_ext && r[j] >= 0.f && r[j] <= 1.f && gv[j] >= 0.f &&
                        gv[j] <= 1.f && b[j] >= 0.f && b[j] <= 1.f;
            const int64_t cell = (int64_t)(min((int)(r[j] * (float)G2), G2 - 1) * G2 +
                                           min((int)(gv[j] * (float)G2), G2 - 1)) * G2 +
                                 min((int)(b[j] * (float)G2), G2 - 1);
            const uint4* line = reinterpret_cast<const uint4*>(lines + (inside[j] ? cell : 0) * 64);
#pragma unroll
            for (int pp = 0; pp < 4; ++pp)
                e[j][pp] = (inside[j] && !exh_pal[pp]) ? line[pp] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const int64_t q = qb + 64 * j;
#pragma unroll
            for (int pp = 0; pp < 4; ++pp) {
                if (pp >= ng) break;
                const int pq = p0 + pp;
                const int k = argmin_from_entry<1>(r[j], gv[j], b[j], e[j][pp],
                                                   inside[j] && !exh_pal[pp], s_pal + pp * a.K, 0,
                                                   a.lvl1 + (int64_t)pq * a.lvl1_pitch, G2, a.K);
                if (q < a.n_ext) {
                    a.idx[(int64_t)pq * a.idx_pitch + q] = (uint8_t)k;
                    const uint32_t bit = 1u << (k & 31);
                    if (!(s_used[pp][k >> 5] & bit)) atomicOr(&s_used[pp][k >> 5], bit);
                }
            }
        }
    }
    __syncthreads();
    if (tid < 8 * ng)
        a.used_mask[((int64_t)(p0 + (tid >> 3)) * a.mask_blocks + a.mask_off + blk) * 8 + (tid & 7)] =
            s_used[tid >> 3][tid & 7];
}

// assign_pipe: assign_quad as a three-stage software pipeline over a thread's
// pixels.  The level-2 lookup depends on the pixel's RGB, so a batch that loads
// RGB, then looks up, then resolves pays two dependent memory round trips per
// batch (a lookup made independent of the RGB ran 40% faster).  Here, while
// pixel i is resolved, pixel i+1's line lookup and pixel i+2's RGB are in flight.
__device__ __forceinline__ int64_t quad_cell(float r, float g, float b, int G2) {
    return (int64_t)(min((int)(r * (float)G2), G2 - 1) * G2 + min((int)(g * (float)G2), G2 - 1)) * G2 +
           min((int)(b * (float)G2), G2 - 1);
}

// NG = min(P, 4): the palettes a pixel pass can serve.  A population below 4
// loads only its NG 16-B entries of each 64-B level-2 line (P = 1 issued four
// dwordx4 lookups per pixel for one useful one) and keeps NG palette tables.
template <int NG>
__global__ __launch_bounds__(256) void assign_pipe_kernel(AssignArgs a, int P) {
    constexpr int PPT = 8;  // pixels per thread per chunk (the pipeline runs across chunks)
    // [NG][kMaxK]: a fixed palette stride, so each palette's base folds into the
    // ds_read_b128 offset field and a candidate's address is its byte << 4
    __shared__ __attribute__((aligned(16))) float4 s_pal[NG * kMaxK];
    __shared__ uint32_t s_used[NG][8];
    const int ngroups = (P + 3) / 4;
    const int w = xcd_remap(blockIdx.x, a.nblocks * ngroups);
    const int grp = w % ngroups, blk = w / ngroups, tid = threadIdx.x;
    const int p0 = 4 * grp, ng = min(NG, P - p0);
    const uint8_t* lines = a.lvl2 + (int64_t)grp * a.lvl2_gstride;
    const int G2 = a.G2 > 0 ? a.G2 : 4;
    // pixel sequence of this thread: chunk c (stride nblocks), slot j < PPT
    const int64_t chunk = 256 * PPT, cstride = (int64_t)a.nblocks * chunk;
    const int64_t lane_off = (int64_t)(tid >> 6) * 64 * PPT + (tid & 63);
    auto qpos = [&](int64_t i) {  // i-th pixel of this thread
        return (int64_t)blk * chunk + (i / PPT) * cstride + lane_off + 64 * (i % PPT);
    };
    // Loads are unconditional (clamped addresses, results selected afterwards):
    // predicated loads sit behind branches, and the compiler's wait counting
    // then keeps at most one load in flight.
    const int64_t qlast = a.n_ext - 1;
    auto load_rgb = [&](int64_t q, float& r, float& g, float& b) {
        const int64_t qc = min(q, qlast);
        r = a.R[qc];
        g = a.G[qc];
        b = a.B[qc];
    };
    auto lookup = [&](int64_t q, float r, float g, float b, bool& inside, uint4 (&e)[NG]) {
        inside = q < a.n_ext && r >= 0.f && r <= 1.f && g >= 0.f && g <= 1.f && b >= 0.f && b <= 1.f;
        const uint4* line = reinterpret_cast<const uint4*>(lines + (inside ? quad_cell(r, g, b, G2) : 0) * 64);
#pragma unroll
        for (int pp = 0; pp < NG; ++pp) e[pp] = line[pp];  // selected by the `listed` flag at use
    };
    // Pipeline, unrolled by two so every buffer has a fixed register set (a
    // register copy of an in-flight load waits for it: rotating buffers at the
    // loop end serialised the whole pipeline behind an s_waitcnt vmcnt(0)).
    // Step i (parity h = i & 1): RGB(i+1) has landed -> its cell lookup goes out
    // into E[h^1] and its RGB moves to X[h^1]; RGB(i+3) goes out into the freed
    // buffer; pixel i is resolved from E[h], X[h] while those loads fly.
    float rb[2], gb[2], bb[2];        // RGB loads in flight: pixel i+1 / i+2 by parity
    float xr[2], xg[2], xb[2];        // RGB of pixels being looked up / resolved
    uint4 E[2][NG];
    bool in_[2];
    int64_t qq[2];
    load_rgb(qpos(0), xr[0], xg[0], xb[0]);
    qq[0] = qpos(0);
    lookup(qq[0], xr[0], xg[0], xb[0], in_[0], E[0]);
    load_rgb(qpos(1), rb[1], gb[1], bb[1]);
    load_rgb(qpos(2), rb[0], gb[0], bb[0]);
    // The palette table is filled while the first pixels' loads are in flight
    // (the fill used to come first: one more memory round trip per workgroup).
    for (int e = tid; e < ng * a.K; e += 256) {
        const int pp = e / a.K, k = e - pp * a.K;
        s_pal[pp * kMaxK + k] = a.pal[(int64_t)(p0 + pp) * kMaxK + k];
    }
    if (tid < 8 * NG) s_used[tid >> 3][tid & 7] = 0;
    __syncthreads();
    bool exh_pal[NG];
#pragma unroll
    for (int pp = 0; pp < NG; ++pp) exh_pal[pp] = pp >= ng || a.pflags[p0 + min(pp, ng - 1)] != 0 || a.G2 == 0;
    auto resolve = [&](int h) {
        const int64_t q = qq[h];
#pragma unroll
        for (int pp = 0; pp < NG; ++pp) {
            if (pp >= ng) break;
            const int pq = p0 + pp;
            const int k = argmin_from_entry<1>(xr[h], xg[h], xb[h], E[h][pp], in_[h] && !exh_pal[pp],
                                               s_pal + pp * kMaxK, 0,
                                               a.lvl1 + (int64_t)pq * a.lvl1_pitch, G2, a.K);
            // non-temporal: streamed out during the kernel rather than left dirty
            // in L2 for the kernel boundary to write back (67 MB per population;
            // ~0.5-1% per evaluation)
            __builtin_nontemporal_store((uint8_t)k, &a.idx[(int64_t)pq * a.idx_pitch + q]);
            const uint32_t bit = 1u << (k & 31);
            if (!(s_used[pp][k >> 5] & bit)) atomicOr(&s_used[pp][k >> 5], bit);
        }
    };
    auto step = [&](int64_t i, int h) {  // h == i & 1, a compile-time constant at each call
        const int n = h ^ 1;
        qq[n] = qpos(i + 1);
        xr[n] = rb[n]; xg[n] = gb[n]; xb[n] = bb[n];  // RGB(i+1): landed, needed now anyway
        lookup(qq[n], xr[n], xg[n], xb[n], in_[n], E[n]);
        load_rgb(qpos(i + 3), rb[n], gb[n], bb[n]);
        resolve(h);
    };
    for (int64_t i = 0;; i += 2) {
        if (qpos(i) >= a.n_ext) break;
        step(i, 0);
        if (qpos(i + 1) >= a.n_ext) break;
        step(i + 1, 1);
    }
    __syncthreads();
    if (tid < 8 * ng)
        a.used_mask[((int64_t)(p0 + (tid >> 3)) * a.mask_blocks + a.mask_off + blk) * 8 + (tid & 7)] =
            s_used[tid >> 3][tid & 7];
}

// assign_lane: assign_pipe with one (pixel, palette) pair per lane.  Lane l of
// a wave takes palette l % ng of pixel l / ng (ng = the group's palettes, 64 / ng
// pixels per wave instruction), so a pixel's level-2 line -- its 4 palettes'
// 16-B entries -- is read by 4 neighbouring lanes in ONE global_load_dwordx4
// that touches 16 cache lines, instead of 4 loads touching 64 lines each
// (assign_pipe: every lane reads the whole line for its pixel).  Same three-stage
// pipeline: while pair i is resolved, pair i+1's entry and pair i+2's RGB are in
// flight.  Grid: nblocks * ceil(P/4), XCD-relabelled; dynamic LDS = 4 * K * 16 B.
__global__ __launch_bounds__(256) void assign_lane_kernel(AssignArgs a, int P) {
    constexpr int PPT = 8;  // wave instructions per thread per chunk
    extern __shared__ __attribute__((aligned(16))) float4 s_pal[];  // [4][K]
    __shared__ uint32_t s_used[4][8];
    const int ngroups = (P + 3) / 4;
    const int w = xcd_remap(blockIdx.x, a.nblocks * ngroups);
    const int grp = w % ngroups, blk = w / ngroups, tid = threadIdx.x;
    const int p0 = 4 * grp, ng = min(4, P - p0);
    for (int e = tid; e < ng * a.K; e += 256) {
        const int pp = e / a.K, k = e - pp * a.K;
        s_pal[e] = a.pal[(int64_t)(p0 + pp) * kMaxK + k];
    }
    if (tid < 32) s_used[tid >> 3][tid & 7] = 0;
    __syncthreads();
    const int lane = tid & 63, wave = tid >> 6;
    const int ppw = 64 / ng;                 // pixels per wave instruction
    const int pp = lane % ng, pix = lane / ng;
    const bool lane_ok = pix < ppw;          // ng = 3: lane 63 idles
    const int pq = p0 + pp;
    const bool exh = a.pflags[pq] != 0 || a.G2 == 0;
    const float4* pal = s_pal + pp * a.K;
    const uint8_t* lvl1p = a.lvl1 + (int64_t)pq * a.lvl1_pitch;
    uint8_t* idx = a.idx + (int64_t)pq * a.idx_pitch;
    const uint8_t* lines = a.lvl2 + (int64_t)grp * a.lvl2_gstride + 16 * pp;
    const int G2 = a.G2 > 0 ? a.G2 : 4;
    const int64_t chunk = 4 * PPT * ppw, cstride = (int64_t)a.nblocks * chunk;
    const int64_t lane_off = (int64_t)wave * PPT * ppw + pix;
    const int64_t qend = lane_ok ? a.n_ext : 0;
    auto qpos = [&](int64_t i) {  // i-th pixel of this lane
        return (int64_t)blk * chunk + (i / PPT) * cstride + lane_off + ppw * (i % PPT);
    };
    const int64_t qlast = a.n_ext - 1;
    auto load_rgb = [&](int64_t q, float& r, float& g, float& b) {
        const int64_t qc = min(q, qlast);
        r = a.R[qc];
        g = a.G[qc];
        b = a.B[qc];
    };
    auto lookup = [&](int64_t q, float r, float g, float b, bool& inside, uint4& e) {
        inside = q < qend && r >= 0.f && r <= 1.f && g >= 0.f && g <= 1.f && b >= 0.f && b <= 1.f;
        e = *reinterpret_cast<const uint4*>(lines + (inside ? quad_cell(r, g, b, G2) : 0) * 64);
    };
    float rb[2], gb[2], bb[2];  // RGB loads in flight: pair i+1 / i+2 by parity
    float xr[2], xg[2], xb[2];  // RGB of the pairs being looked up / resolved
    uint4 E[2];
    bool in_[2];
    int64_t qq[2];
    qq[0] = qpos(0);
    load_rgb(qq[0], xr[0], xg[0], xb[0]);
    lookup(qq[0], xr[0], xg[0], xb[0], in_[0], E[0]);
    load_rgb(qpos(1), rb[1], gb[1], bb[1]);
    load_rgb(qpos(2), rb[0], gb[0], bb[0]);
    auto resolve = [&](int h) {
        const int k = argmin_from_entry<1>(xr[h], xg[h], xb[h], E[h], in_[h] && !exh, pal, 0, lvl1p,
                                           G2, a.K);
        idx[qq[h]] = (uint8_t)k;
        const uint32_t bit = 1u << (k & 31);
        if (!(s_used[pp][k >> 5] & bit)) atomicOr(&s_used[pp][k >> 5], bit);
    };
    auto step = [&](int64_t i, int h) {  // h == i & 1, a compile-time constant at each call
        const int n = h ^ 1;
        qq[n] = qpos(i + 1);
        xr[n] = rb[n]; xg[n] = gb[n]; xb[n] = bb[n];
        lookup(qq[n], xr[n], xg[n], xb[n], in_[n], E[n]);
        load_rgb(qpos(i + 3), rb[n], gb[n], bb[n]);
        resolve(h);
    };
    for (int64_t i = 0;; i += 2) {
        if (qpos(i) >= qend) break;
        step(i, 0);
        if (qpos(i + 1) >= qend) break;
        step(i + 1, 1);
    }
    __syncthreads();
    if (tid < 8 * ng)
        a.used_mask[((int64_t)(p0 + (tid >> 3)) * a.mask_blocks + a.mask_off + blk) * 8 + (tid & 7)] =
            s_used[tid >> 3][tid & 7];
}

// assign_multi: grid (nblocks, ceil(P/PG)), dynamic LDS = PG*K*REP*16 B.  One
// pass over the pixels serves PG palettes: each pixel's RGB is read once, its
// cell index computed once, and the PG level-2 entries loaded together
// (512 KiB tables at G2 = 32 stay L2-resident), then resolved palette by palette.
template <int REP, int PG>
__global__ __launch_bounds__(256) void assign_multi_kernel(AssignArgs a, int P) {
    constexpr int PPT = 8;
    extern __shared__ __attribute__((aligned(16))) float4 s_pal[];
    __shared__ uint32_t s_used[PG][8];
    const int tid = threadIdx.x;
    const int p0 = blockIdx.y * PG;
    const int ng = min(PG, P - p0);
    for (int e = tid; e < ng * a.K * REP; e += 256) {
        const int pp = e / (a.K * REP), r = e - pp * a.K * REP;
        s_pal[e] = a.pal[(int64_t)(p0 + pp) * kMaxK + r / REP];
    }
    if (tid < 8 * PG) s_used[tid >> 3][tid & 7] = 0;
    __syncthreads();
    const int copy = tid & (REP - 1);
    bool exh_pal[PG];
#pragma unroll
    for (int pp = 0; pp < PG; ++pp) {
        const int pq = min(p0 + pp, P - 1);
        exh_pal[pp] = a.pflags[pq] != 0 || a.G2 == 0;
    }
    const int64_t chunk = 256 * PPT;
    const int64_t lane_off = (int64_t)(tid >> 6) * 64 * PPT + (tid & 63);
    const int G2 = a.G2 > 0 ? a.G2 : 4;
    for (int64_t q0 = (int64_t)blockIdx.x * chunk; q0 < a.n_ext; q0 += (int64_t)a.nblocks * chunk) {
        int64_t q = q0 + lane_off;
        bool in = q < a.n_ext;
        float r = in ? a.R[q] : 0.f, gv = in ? a.G[q] : 0.f, b = in ? a.B[q] : 0.f;
#pragma unroll 1
        for (int j = 0; j < PPT; ++j) {
            const int64_t qn = q + 64;
            const bool inn = j + 1 < PPT && qn < a.n_ext;
            const float rn = inn ? a.R[qn] : 0.f, gn = inn ? a.G[qn] : 0.f,
                        bn = inn ? a.B[qn] : 0.f;
            // one cell index, PG table loads in flight
            const bool inside = r >= 0.f && r <= 1.f && gv >= 0.f && gv <= 1.f && b >= 0.f && b <= 1.f;
            const int64_t cell = (int64_t)(min((int)(r * (float)G2), G2 - 1) * G2 +
                                           min((int)(gv * (float)G2), G2 - 1)) * G2 +
                                 min((int)(b * (float)G2), G2 - 1);
            uint4 e[PG];
            bool li[PG];
#pragma unroll
            for (int pp = 0; pp < PG; ++pp) {
                li[pp] = inside && !exh_pal[pp] && pp < ng;
                e[pp] = li[pp] ? *reinterpret_cast<const uint4*>(
                                     a.lvl2 + lvl2_offset(a.lvl2_gstride, min(p0 + pp, P - 1), cell))
                               : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int pp = 0; pp < PG; ++pp) {
                if (pp >= ng) break;
                const int pq = p0 + pp;
                const int k = argmin_from_entry<REP>(r, gv, b, e[pp], li[pp],
                                                     s_pal + pp * a.K * REP, copy,
                                                     a.lvl1 + (int64_t)pq * a.lvl1_pitch, G2,
                                                     a.K);
                if (in) {
                    a.idx[(int64_t)pq * a.idx_pitch + q] = (uint8_t)k;
                    const uint32_t bit = 1u << (k & 31);
                    if (!(s_used[pp][k >> 5] & bit)) atomicOr(&s_used[pp][k >> 5], bit);
                }
            }
            q = qn; in = inn; r = rn; gv = gn; b = bn;
        }
    }
    __syncthreads();
    if (tid < 8 * ng)
        a.used_mask[((int64_t)(p0 + (tid >> 3)) * a.mask_blocks + a.mask_off + blockIdx.x) * 8 + (tid & 7)] =
            s_used[tid >> 3][tid & 7];
}

// ----------------------------------------------------------------------------
// cost_tile: grid (ntiles * P), block 256.  One workgroup = one TW x TH output
// tile; region = (TH + 2*HALF) rows x RW cols of indices (RW = TW + 2*HALF).
// Vertical pass first on all RW region columns (separable filters commute),
// then horizontal pass on the TW output columns, Opp->Lab, dE, fp64 partial.
// ----------------------------------------------------------------------------
template <int HALF>
struct CostTaps {
    float v[kNumFilt][2 * HALF + 1];
    float h[kNumFilt][2 * HALF + 1];
};

// Taps are read through a constant-address-space pointer into device memory
// (uniform s_load per filter; build_fast_taps holds both scalings).
template <int HALF>
using TapsPtr = const __attribute__((address_space(4))) CostTaps<HALF>*;

// Vertical pass of filters [f0, f1) of one opponent channel: RV outputs per
// thread from RV + 2*HALF gathered inputs; results to s_v[f][row][col].
// Taps [TLO, THI] only (the default filter set's narrow k1 filters have |taps|
// below 1e-9 of their peak outside a short window; see trim_window()).
// PAIR: s_v holds row pairs, float2 (row 2m, row 2m+1) per column (cost_pair_kernel).
template <int HALF, int RV, int TH, int RW, int TLO = 0, int THI = 2 * HALF, bool PAIR = false>
__device__ __forceinline__ void vpass_filters(const float (&o)[RV + 2 * HALF],
                                              TapsPtr<HALF> taps, int f0, int f1,
                                              float* out, int fslot = 0) {
#pragma unroll 1
    for (int f = f0; f < f1; ++f) {
        float acc[RV];
#pragma unroll
        for (int y = 0; y < RV; ++y) acc[y] = 0.f;
#pragma unroll
        for (int t = TLO; t <= THI; ++t) {
            const float k = taps->v[f][t];
#pragma unroll
            for (int y = 0; y < RV; ++y) acc[y] = fmaf(o[y + t], k, acc[y]);
        }
        if constexpr (PAIR) {
            static_assert(RV % 2 == 0, "whole row pairs per item");
#pragma unroll
            for (int y = 0; y < RV; y += 2)
                *reinterpret_cast<float2*>(out + ((f - fslot) * (TH / 2) + y / 2) * RW * 2) =
                    make_float2(acc[y], acc[y + 1]);
        } else {
#pragma unroll
            for (int y = 0; y < RV; ++y) out[(f * TH + y) * RW] = acc[y];
        }
    }
}

// Horizontal pass of filters [f0, f1) of one channel for a 4-column run:
// 4 + 2*HALF inputs per filter read as ds_read_b128 from s_v.
// Accumulates filters [f0, f1) into acc (caller zeroes it); taps [TLO, THI].
template <int HALF, int TH, int RW, int TLO = 0, int THI = 2 * HALF>
__device__ __forceinline__ void hpass_filters(const float4* src, TapsPtr<HALF> taps,
                                              int f0, int f1, float (&acc)[4]) {
    constexpr int NQ = (4 + 2 * HALF + 3) / 4;
    static_assert(NQ == 6, "the asm barrier below names six vectors");
#pragma unroll 1
    for (int f = f0; f < f1; ++f) {
        float in[4 * NQ];
        const f32x4* row = reinterpret_cast<const f32x4*>(src + (f * TH * RW) / 4);
        f32x4 v0 = row[0], v1 = row[1], v2 = row[2], v3 = row[3], v4 = row[4], v5 = row[5];
        // One opaque barrier over all six loads: keeps them whole ds_read_b128
        // (scalar reads re-paired at odd offsets were 4-way conflicted) and lets
        // all six be in flight before a single wait.
        asm volatile("" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5));
        const f32x4 vv[NQ] = {v0, v1, v2, v3, v4, v5};
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            in[4 * q] = vv[q].x; in[4 * q + 1] = vv[q].y; in[4 * q + 2] = vv[q].z;
            in[4 * q + 3] = vv[q].w;
        }
#pragma unroll
        for (int t = TLO; t <= THI; ++t) {
            const float k = taps->h[f][t];
#pragma unroll
            for (int xo = 0; xo < 4; ++xo) acc[xo] = fmaf(in[xo + t], k, acc[xo]);
        }
    }
}

// The seven filters of both passes.  TRIM: the narrow k1.x / k1.y / k1.z filters
// (f = 0, 3, 5) run over their significant-tap windows kTrimLo/Hi only
// (|taps| outside are below 1e-9 of the filter's peak for the default filter
// set; see trim_window_ok()).  Per-filter loops keep one filter's 21 taps live
// in SGPRs (interleaving a channel's filters needs 63 and spills to VGPR lanes).
constexpr int kTrimLo[3] = {7, 6, 5}, kTrimHi[3] = {13, 14, 15};

template <int HALF, int RV, int TH, int RW, bool TRIM, bool PAIR = false>
__device__ __forceinline__ void vpass_all(const float (&o0)[RV + 2 * HALF],
                                          const float (&o1)[RV + 2 * HALF],
                                          const float (&o2)[RV + 2 * HALF],
                                          TapsPtr<HALF> taps, float* out) {
    constexpr int T2 = 2 * HALF;
    if constexpr (TRIM) {
        vpass_filters<HALF, RV, TH, RW, kTrimLo[0], kTrimHi[0], PAIR>(o0, taps, 0, 1, out);
        vpass_filters<HALF, RV, TH, RW, 0, T2, PAIR>(o0, taps, 1, 3, out);
        vpass_filters<HALF, RV, TH, RW, kTrimLo[1], kTrimHi[1], PAIR>(o1, taps, 3, 4, out);
        vpass_filters<HALF, RV, TH, RW, 0, T2, PAIR>(o1, taps, 4, 5, out);
        vpass_filters<HALF, RV, TH, RW, kTrimLo[2], kTrimHi[2], PAIR>(o2, taps, 5, 6, out);
        vpass_filters<HALF, RV, TH, RW, 0, T2, PAIR>(o2, taps, 6, 7, out);
    } else {
        vpass_filters<HALF, RV, TH, RW, 0, T2, PAIR>(o0, taps, 0, 3, out);
        vpass_filters<HALF, RV, TH, RW, 0, T2, PAIR>(o1, taps, 3, 5, out);
        vpass_filters<HALF, RV, TH, RW, 0, T2, PAIR>(o2, taps, 5, 7, out);
    }
}

template <int HALF, int TH, int RW, bool TRIM>
__device__ __forceinline__ void hpass_all(const float4* src, TapsPtr<HALF> taps,
                                          float (&acc0)[4], float (&acc1)[4], float (&acc2)[4]) {
#pragma unroll
    for (int xo = 0; xo < 4; ++xo) acc0[xo] = acc1[xo] = acc2[xo] = 0.f;
    if constexpr (TRIM) {
        hpass_filters<HALF, TH, RW, kTrimLo[0], kTrimHi[0]>(src, taps, 0, 1, acc0);
        hpass_filters<HALF, TH, RW>(src, taps, 1, 3, acc0);
        hpass_filters<HALF, TH, RW, kTrimLo[1], kTrimHi[1]>(src, taps, 3, 4, acc1);
        hpass_filters<HALF, TH, RW>(src, taps, 4, 5, acc1);
        hpass_filters<HALF, TH, RW, kTrimLo[2], kTrimHi[2]>(src, taps, 5, 6, acc2);
        hpass_filters<HALF, TH, RW>(src, taps, 6, 7, acc2);
    } else {
        hpass_filters<HALF, TH, RW>(src, taps, 0, 3, acc0);
        hpass_filters<HALF, TH, RW>(src, taps, 3, 5, acc1);
        hpass_filters<HALF, TH, RW>(src, taps, 5, 7, acc2);
    }
}

// V pass split by channel group (VSPLIT): threads [0, RW) own channel 0
// (filters 0-2) of region column c, threads [RW, 2*RW) channels 1 and 2
// (filters 3-6), each over all TH rows.  The gathers are then ds_read_b32 /
// ds_read_b64 from per-group tables (2 LDS cycles per wave-instruction against
// 4 for the float4 table) and every gathered row feeds TH outputs instead of RV.
template <int HALF, int TH, int RW, bool TRIM>
__device__ __forceinline__ void vpass_split(const uint8_t* s_idx, const float* s_oppA,
                                            const float2* s_oppB, TapsPtr<HALF> taps,
                                            float* s_v, int tid) {
    constexpr int NIN = TH + 2 * HALF;
    const int c = tid % RW;
    float* out = s_v + c;
    if (tid < RW) {
        float o0[NIN];
#pragma unroll
        for (int r = 0; r < NIN; ++r) o0[r] = s_oppA[s_idx[r * RW + c]];
        if constexpr (TRIM) {
            vpass_filters<HALF, TH, TH, RW, kTrimLo[0], kTrimHi[0]>(o0, taps, 0, 1, out);
            vpass_filters<HALF, TH, TH, RW>(o0, taps, 1, 3, out);
        } else {
            vpass_filters<HALF, TH, TH, RW>(o0, taps, 0, 3, out);
        }
    } else {
        float o1[NIN], o2[NIN];
#pragma unroll
        for (int r = 0; r < NIN; ++r) {
            const float2 v = s_oppB[s_idx[r * RW + c]];
            o1[r] = v.x; o2[r] = v.y;
        }
        if constexpr (TRIM) {
            vpass_filters<HALF, TH, TH, RW, kTrimLo[1], kTrimHi[1]>(o1, taps, 3, 4, out);
            vpass_filters<HALF, TH, TH, RW>(o1, taps, 4, 5, out);
            vpass_filters<HALF, TH, TH, RW, kTrimLo[2], kTrimHi[2]>(o2, taps, 5, 6, out);
            vpass_filters<HALF, TH, TH, RW>(o2, taps, 6, 7, out);
        } else {
            vpass_filters<HALF, TH, TH, RW>(o1, taps, 3, 5, out);
            vpass_filters<HALF, TH, TH, RW>(o2, taps, 5, 7, out);
        }
    }
}

// ---- vertical pass on the matrix cores (cost_tile 3) -------------------------
// The vertical pass of one filter over a 16-column block is a banded-Toeplitz
// product V^T = X^T . T^T with X the block's TH + 2*HALF gathered input rows:
// v_mfma_f32_16x16x32_f16 with A = X^T (16 columns x 32 input rows, rows past
// the region zero-weighted), B = T^T (32 input rows x 16 output rows, the TH
// valid ones carrying the taps) -- one K step.  fp32 accuracy from f16 operands:
// x = hi + lo (both f16, x scaled by 2^14 so lo stays normal down to |x| ~ 1e-5)
// and the products hi.hi + hi.lo + lo.hi (each exact in the f32 accumulator;
// the dropped lo.lo is ~2^-22 relative).  Taps are split the same way on the
// host, scaled by 2^16 (build_vpass_fragments); the 2^30 total scale is folded
// into the horizontal taps, exactly (a power of two).
// Lane l of the 16x16 result holds output row (l & 15) of four consecutive
// columns 4(l >> 4) .. +3 -- one float4 into s_v[f][row][col], the layout the
// horizontal pass already reads.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr float kVDataScale = 16384.0f;                   // 2^14
constexpr float kVTapScale = 65536.0f;                    // 2^16
constexpr float kVOutScale = 1.0f / (16384.0f * 65536.0f);  // 2^-30

// (hi, lo) f16 split of x * 2^14 in one dword, hi in bits 0-15.
__device__ __forceinline__ uint32_t split_f16(float x) {
    const float xs = x * kVDataScale;
    const _Float16 hi = (_Float16)xs;
    const _Float16 lo = (_Float16)(xs - (float)hi);
    return (uint32_t)__builtin_bit_cast(uint16_t, hi) |
           ((uint32_t)__builtin_bit_cast(uint16_t, lo) << 16);
}

__device__ __forceinline__ uint32_t chan(const uint4& v, int c) {
    return c == 0 ? v.x : (c == 1 ? v.y : v.z);
}

template <int HALF, int TH, int RW, int IDXP, int SVP>
__device__ __forceinline__ void vpass_mfma(const uint8_t* s_idx, const uint4* s_opph,
                                           const uint4* vfrag, float* s_v, int tid) {
    static_assert(TH + 2 * HALF <= 32 && TH <= 16, "one K = 32 step per output block");
    static_assert(RW % 64 == 0, "whole 16-column blocks, the same number per wave");
    constexpr int BPW = RW / 64;  // column blocks per wave
    const int lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, n = lane & 15;
    uint4 bf[2 * kNumFilt];  // Toeplitz B fragments (L2-resident), live only in this pass
#pragma unroll
    for (int i = 0; i < 2 * kNumFilt; ++i) bf[i] = vfrag[i * 64 + lane];
#pragma unroll
    for (int bi = 0; bi < BPW; ++bi) {
        const int cb = wave * BPW + bi;
        // A fragment rows: input rows 8g .. 8g+7 of column cb*16 + n
        uint4 e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) e[j] = s_opph[s_idx[(8 * g + j) * IDXP + cb * 16 + n]];
        u32x4 ah[3], al[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const uint32_t w0 = chan(e[2 * m], c), w1 = chan(e[2 * m + 1], c);
                ah[c][m] = __builtin_amdgcn_perm(w1, w0, 0x05040100u);  // hi halves
                al[c][m] = __builtin_amdgcn_perm(w1, w0, 0x07060302u);  // lo halves
            }
        }
#pragma unroll
        for (int f = 0; f < kNumFilt; ++f) {
            const int c = filt_chan(f);
            const f16x8 a_hi = __builtin_bit_cast(f16x8, ah[c]);
            const f16x8 a_lo = __builtin_bit_cast(f16x8, al[c]);
            const f16x8 b_hi = __builtin_bit_cast(f16x8, bf[2 * f]);
            const f16x8 b_lo = __builtin_bit_cast(f16x8, bf[2 * f + 1]);
            f32x4 d = {0.f, 0.f, 0.f, 0.f};
            d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_lo, b_hi, d, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_hi, b_lo, d, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_hi, b_hi, d, 0, 0, 0);
            if (n < TH) *reinterpret_cast<f32x4*>(s_v + (f * TH + n) * SVP + cb * 16 + 4 * g) = d;
        }
    }
}

// One work item of the cost pass: palette p over output tile `tile`.
struct TileItem {
    int p, tile, x0, y0;
};

template <int TW, int TH>
__device__ __forceinline__ TileItem tile_item(const CostArgs& a, int w, int P) {
    TileItem t;
    t.p = w % P;
    t.tile = a.tile0 + w / P;
    t.x0 = (t.tile % a.tiles_x) * TW;
    t.y0 = a.g.r0 + (t.tile / a.tiles_x) * TH;
    return t;
}

// The global loads that fill one item's LDS (index rows of its region, its
// palette's opponent entry), held in registers between issue and commit.
// Every load is issued before the first wait: vmcnt retires in order, so a
// load -> wait -> store loop pays one memory round trip per trip (4 for the
// interior index rows, 14 for the byte gathers of edge tiles).
template <int HALF, int RW, int TH>
struct TileFill {
    static constexpr int TW = RW - 2 * HALF, RH = TH + 2 * HALF, DW = RW / 4;
    static constexpr int NFD = (RH * DW + 255) / 256, NFB = (RH * RW + 255) / 256;
    static_assert((DW & (DW - 1)) == 0, "dword columns per row: a power of two");
    uint32_t lo[NFD], hi[NFD];  // interior tiles: aligned dword pairs of the index rows
    uint32_t roff[NFD];         // their rows' byte offsets (alignment for commit)
    float4 ov;
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
        static_assert(kMaxK == 256, "one opponent-table entry per thread");
        const Geom& g = a.g;
        t = ti;
        const uint8_t* idx = a.idx + (int64_t)t.p * g.idx_pitch;
        ov = tid < a.K ? a.opp[(int64_t)t.p * kMaxK + tid] : make_float4(0.f, 0.f, 0.f, 0.f);
        interior = t.x0 - HALF >= 0 && t.x0 + TW + HALF <= g.W;
        if (interior) {
            const int ytop = t.y0 - HALF;
            const bool vfast = ytop >= 0 && ytop >= g.e0 && ytop + RH <= g.H && ytop + RH <= g.e1;
            const int ubase = (ytop - g.e0) * g.W + (t.x0 - HALF);
#pragma unroll
            for (int q = 0; q < NFD; ++q) {
                const int e = min(tid + 256 * q, RH * DW - 1);
                const int i = e / DW;
                roff[q] = (uint32_t)(vfast ? ubase + i * g.W : row_base(g, t, i));
                const uint32_t* src = reinterpret_cast<const uint32_t*>(
                    idx + ((roff[q] & ~3u) + 4u * (uint32_t)(e % DW)));
                lo[q] = src[0];
                hi[q] = src[1];
            }
        }
    }

    // index rows into s_idx (row pitch IDXP bytes); the first write waits for the loads
    template <int IDXP>
    __device__ __forceinline__ void commit_idx(const CostArgs& a, uint8_t* s_idx, int tid) const {
        const Geom& g = a.g;
        if (interior) {
#pragma unroll
            for (int q = 0; q < NFD; ++q) {
                const int e = tid + 256 * q;
                if (e < RH * DW)
                    reinterpret_cast<uint32_t*>(s_idx)[(e / DW) * (IDXP / 4) + e % DW] =
                        __builtin_amdgcn_alignbyte(hi[q], lo[q], roff[q] & 3u);
            }
        } else {
            const uint8_t* idx = a.idx + (int64_t)t.p * g.idx_pitch;
            uint32_t b[NFB];
#pragma unroll
            for (int q = 0; q < NFB; ++q) {  // all loads first: one round trip
                const int e = min(tid + 256 * q, RH * RW - 1);
                const int i = e / RW, j = e % RW;
                int gy = reflect_clamp(t.y0 - HALF + i, g.H);
                gy = min(max(gy, g.e0), g.e1 - 1);
                const int gx = reflect_clamp(t.x0 - HALF + j, g.W);
                b[q] = idx[(uint32_t)((gy - g.e0) * g.W + gx)];
            }
#pragma unroll
            for (int q = 0; q < NFB; ++q) {
                const int e = tid + 256 * q;
                if (e < RH * RW) s_idx[(e / RW) * IDXP + e % RW] = (uint8_t)b[q];
            }
        }
    }
};

// LabRef of a thread's H items (NH = TH * 32 / 256 of them).
template <int TW, int TH>
struct TileLab {
    static constexpr int NH = TH * 32 / 256, NRUN = TW / 4;
    float4 L[NH], A[NH], B[NH];
    __device__ __forceinline__ void issue(const CostArgs& a, const TileItem& t, int tid) {
        const Geom& g = a.g;
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            const int item = tid + 256 * h, y = item >> 5, j = item & 31;
            const int gy = t.y0 + y, gx0 = t.x0 + 4 * j;
            L[h] = A[h] = B[h] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (j < NRUN && gy < g.r1 && gx0 < g.W) {
                const int off = (gy - g.r0) * (int)g.lab_pitch + gx0;
                L[h] = *reinterpret_cast<const float4*>(a.labL + off);
                A[h] = *reinterpret_cast<const float4*>(a.labA + off);
                B[h] = *reinterpret_cast<const float4*>(a.labB + off);
            }
        }
    }
};

// cost_tile: one workgroup = one TW x TH output tile of one palette; region =
// (TH + 2*HALF) rows x RW columns of indices.  Vertical pass first on all RW
// region columns (separable filters commute), then horizontal pass on the TW
// output columns, Opp->Lab, dE, one fp64 partial per (tile, palette).
// VMODE: 0 = V items of RV rows on VALU, 1 = V split by channel group (VALU),
// 2 = V pass on the matrix cores (vpass_mfma).
// 1-D grid of ntiles * P: work item w = tile * P + p, XCD-relabelled so the P
// palettes of a tile run side by side on one XCD and read its LabRef from L2
// after the first.  (Persistent variants -- a workgroup walking a run of tiles
// with the next tile's loads in flight in registers, or DMA'd into a second LDS
// buffer -- measured 20-40% slower than this grid with 4 workgroups per CU.)
template <int HALF, int RW, int TH, int RV, int DE, int OCC, bool TRIM, int VMODE>
__global__ __launch_bounds__(256, OCC) void cost_tile_kernel(CostArgs a, int P_) {
    constexpr bool VSPLIT = VMODE == 1, VMFMA = VMODE == 2;
    constexpr int TW = RW - 2 * HALF;
    constexpr int RH = TH + 2 * HALF;
    constexpr int NIN = RV + 2 * HALF;
    constexpr int NRUN = TW / 4;
    constexpr int NH = TH * 32 / 256;
    static_assert(VMFMA || (VSPLIT ? (RV == TH && 2 * RW == 256) : RW * (TH / RV) == 256),
                  "one V item per thread");
    static_assert(TW % 4 == 0, "4-wide H runs");
    static_assert(TH * 32 % 256 == 0 && TH * 32 <= 512, "one or two H items per thread");
    // s_v is float4-typed so the H-pass reads stay ds_read_b128 (a float-typed
    // array let the compiler split them into 4-way-conflicted ds_read2_b32).
    // Row pitches of s_v (floats) and s_idx (bytes).  VMFMA pads both by 16 B:
    // its float4 stores of 8 rows at once (and its index reads of 4 rows) would
    // otherwise land on one bank set (8-way conflicts at a 512-B pitch).
    constexpr int SVP = VMFMA ? RW + 4 : RW, IDXP = VMFMA ? RW + 4 : RW;
    __shared__ float4 s_v4[kNumFilt * TH * SVP / 4];
    // opponent table, one copy: replicating it to spread the random gathers over
    // more banks (2 or 4 copies) measured slower -- the LDS it costs is worth
    // more as a fourth workgroup per CU (36 KiB per workgroup at TH = 8).
    __shared__ float4 s_opp[VMODE == 0 ? kMaxK : 1];
    __shared__ float s_oppA[VSPLIT ? kMaxK : 1];    // VSPLIT: opponent channel 0
    __shared__ float2 s_oppB[VSPLIT ? kMaxK : 1];   // VSPLIT: opponent channels 1, 2
    __shared__ uint4 s_opph[VMFMA ? kMaxK : 1];     // VMFMA: split_f16 of channels 0-2
    constexpr int IDX_ROWS = VMFMA ? 32 : RH;       // VMFMA reads a whole K = 32 step
    __shared__ __attribute__((aligned(16))) uint8_t s_idx[IDX_ROWS * IDXP];
    __shared__ double s_red[4];
    float* s_v = reinterpret_cast<float*>(s_v4);
    const int tid = threadIdx.x;
    const Geom& g = a.g;
    const TileItem cur = tile_item<TW, TH>(a, xcd_remap(blockIdx.x, a.band_tiles * P_), P_);
    const TapsPtr<HALF> taps = (TapsPtr<HALF>)(uintptr_t)a.taps;  // flat -> constant: same address

    // ---- prologue: every fill load issued before the first wait (TileFill),
    // LabRef after the LDS writes, in flight during the V pass
    TileFill<HALF, RW, TH> fill;
    fill.issue(a, cur, tid);
    if constexpr (VMFMA) {
        // every entry finite: the padding rows of the K = 32 step gather too
        s_opph[tid] = tid < a.K ? make_uint4(split_f16(fill.ov.x), split_f16(fill.ov.y),
                                             split_f16(fill.ov.z), 0u)
                                : make_uint4(0u, 0u, 0u, 0u);
        for (int e = tid; e < (IDX_ROWS - RH) * IDXP / 4; e += 256)
            reinterpret_cast<uint32_t*>(s_idx + RH * IDXP)[e] = 0u;
    } else if constexpr (VSPLIT) {
        if (tid < a.K) {
            s_oppA[tid] = fill.ov.x;
            s_oppB[tid] = make_float2(fill.ov.y, fill.ov.z);
        }
    } else {
        if (tid < a.K) s_opp[tid] = fill.ov;
    }
    fill.template commit_idx<IDXP>(a, s_idx, tid);
    TileLab<TW, TH> lab;
    lab.issue(a, cur, tid);
    __syncthreads();

    // ---- vertical pass ----
    // The filter loops are not unrolled so only one filter's 21 taps are live in
    // SGPRs at a time (all 294 taps at once spill into VGPR lanes).
    if constexpr (VMFMA) {
        vpass_mfma<HALF, TH, RW, IDXP, SVP>(s_idx, s_opph, a.vfrag, s_v, tid);
    } else if constexpr (VSPLIT) {
        vpass_split<HALF, TH, RW, TRIM>(s_idx, s_oppA, s_oppB, taps, s_v, tid);
    } else {
        // thread = (region column c, rows [RV*gr, RV*gr+RV))
        const int c = tid % RW, gr = tid / RW;
        float o0[NIN], o1[NIN], o2[NIN];
        float wsum = 0.f;  // .w (= 0) is consumed so the gather stays one ds_read_b128
#pragma unroll
        for (int r = 0; r < NIN; ++r) {
            const float4 v = s_opp[s_idx[(gr * RV + r) * IDXP + c]];
            o0[r] = v.x; o1[r] = v.y; o2[r] = v.z;
            wsum += v.w;
        }
        o0[0] += wsum;  // wsum == 0 exactly (prep_palette writes .w = 0)
        vpass_all<HALF, RV, TH, RW, TRIM>(o0, o1, o2, taps, s_v + (gr * RV) * SVP + c);
    }
    __syncthreads();

    // ---- horizontal pass + Lab + dE: item = (row y, 4-column run j) ----
    double sum = 0.0;
    // 32 run slots per row (NRUN used): a ds_read_b128 16-lane group then
    // covers 16 distinct bank positions of one row (27 runs per row wrapped
    // lanes into the next row's bank 0).
    static_assert(NRUN <= 32, "runs per row");
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        const int item = tid + 256 * h, y = item >> 5, j = item & 31;
        if (j >= NRUN) continue;
        float acc0[4], acc1[4], acc2[4];
        hpass_all<HALF, TH, SVP, TRIM>(&s_v4[(y * SVP) / 4 + j], taps, acc0, acc1, acc2);
        const int gy = cur.y0 + y, gx0 = cur.x0 + 4 * j;
        if (gy < g.r1 && gx0 < g.W) {
            const float4 L4 = lab.L[h], A4 = lab.A[h], B4 = lab.B[h];
            const float Ls[4] = {L4.x, L4.y, L4.z, L4.w};
            const float As[4] = {A4.x, A4.y, A4.z, A4.w};
            const float Bs[4] = {B4.x, B4.y, B4.z, B4.w};
            float part = 0.f;
#pragma unroll
            for (int xo = 0; xo < 4; ++xo) {
                const float3 l3 = opp2lab_fast(acc0[xo], acc1[xo], acc2[xo], a.m_lab);
                const float e = delta_e<DE>(Ls[xo], As[xo], Bs[xo], l3.x, l3.y, l3.z);
                part += (gx0 + xo < g.W) ? e : 0.f;
            }
            sum += (double)part;
        }
    }
    sum = wave_sum_to_lane63(sum);
    if ((tid & 63) == 63) s_red[tid >> 6] = sum;
    __syncthreads();
    if (tid == 0)
        a.partial[(int64_t)cur.p * a.ntiles + cur.tile] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
}

// ----------------------------------------------------------------------------


__global__ __launch_bounds__(256) void gen_hpass_kernel(GenArgs a) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= a.g.n_ext) return;
    const int ly = (int)(q / a.g.W), x = (int)(q % a.g.W);
    const uint8_t* row = a.idx + (int64_t)ly * a.g.W;
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
        const float3 lab = opp2lab_fast(ox, oy, oz, a.m_lab);
        const int64_t off = (int64_t)(y - a.g.r0) * a.g.lab_pitch + x;
        e = (double)delta_e<DE>(a.labL[off], a.labA[off], a.labB[off], lab.x, lab.y, lab.z);
    }
    e = wave_sum(e);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = e;
    __syncthreads();
    if (threadIdx.x == 0) a.partial[blockIdx.x] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
}

// ----------------------------------------------------------------------------
// finalize: grid (P), block 256.  Fixed-order fp64 sum of the tile partials
// and OR of the per-block used masks -> out[p] = {sum, used[0..K-1]}.
// ----------------------------------------------------------------------------
// finalize: one 1024-thread workgroup per palette.  Thread t sums partials
// t, t + 1024, ... with all of its loads issued before the first add (one memory
// round trip; 256 threads summing 8 at a time took ~10 dependent rounds), then
// a fixed-order wave and workgroup reduction: bitwise reproducible.
__global__ __launch_bounds__(1024) void finalize_kernel(FinalizeArgs a) {
    constexpr int NT = 1024, NL = 24;  // loads in flight per thread per round
    const int p = blockIdx.x, tid = threadIdx.x;
    __shared__ double s_red[NT / 64];
    __shared__ uint32_t s_mask[NT];
    const double* part = a.partial + (int64_t)p * a.ntiles;
    double s = 0.0;
    for (int t0 = 0; t0 < a.ntiles; t0 += NT * NL) {
        double v[NL];
#pragma unroll
        for (int u = 0; u < NL; ++u) {
            const int t = t0 + u * NT + tid;
            v[u] = t < a.ntiles ? part[t] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < NL; ++u) s += v[u];
    }
    s = wave_sum_to_lane63(s);
    if ((tid & 63) == 63) s_red[tid >> 6] = s;
    // used: thread = (word w = tid & 7, block slice tid >> 3)
    uint32_t m = 0;
    const int w = tid & 7;
    const uint32_t* um = a.used_mask + (int64_t)p * a.nblocks * 8;
    for (int b0 = tid >> 3; b0 < a.nblocks; b0 += (NT / 8) * 8) {
        uint32_t mv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int b = b0 + (NT / 8) * u;
            mv[u] = b < a.nblocks ? um[b * 8 + w] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) m |= mv[u];
    }
    s_mask[tid] = m;
    __syncthreads();
    double* out = a.out + (int64_t)p * (1 + a.K);
    if (tid == 0) {
        double tot = 0.0;
        for (int i = 0; i < NT / 64; ++i) tot += s_red[i];
        out[0] = tot;
    }
    if (tid < 8) {
        uint32_t acc = 0;
        for (int i = tid; i < NT; i += 8) acc |= s_mask[i];
        s_mask[tid] = acc;  // slots 0..7 are only read after the barrier below
    }
    __syncthreads();
    for (int k = tid; k < a.K; k += NT) out[1 + k] = (s_mask[k >> 5] >> (k & 31)) & 1u ? 1.0 : 0.0;
}

// ----------------------------------------------------------------------------
// LabRef (setup, once per search): IM:100-153 + IM:285-370 on the device.
// ----------------------------------------------------------------------------
// planar R,G,B -> Opp float4 (CL:79-90 then CL:111-116)
__global__ __launch_bounds__(256) void labref_opp_kernel(const float* R, const float* G,
                                                         const float* B, float4* opp, int64_t n) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= n) return;
    const float lr = srgb_lin(R[q]), lg = srgb_lin(G[q]), lb = srgb_lin(B[q]);
    const float X = dot3(lr, lg, lb, c_RGB2XYZ + 0);
    const float Y = dot3(lr, lg, lb, c_RGB2XYZ + 3);
    const float Z = dot3(lr, lg, lb, c_RGB2XYZ + 6);
    opp[q] = make_float4(dot3(X, Y, Z, c_XYZ2Opp + 0), dot3(X, Y, Z, c_XYZ2Opp + 3),
                         dot3(X, Y, Z, c_XYZ2Opp + 6), 0.f);
}

// inline XYZ float4 -> Opp float4 (CL:111-116), for hq_xyz_to_scielab
__global__ __launch_bounds__(256) void xyz_to_opp_kernel(const float4* xyz, float4* opp, int64_t n) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= n) return;
    const float4 v = xyz[q];
    opp[q] = make_float4(dot3(v.x, v.y, v.z, c_XYZ2Opp + 0), dot3(v.x, v.y, v.z, c_XYZ2Opp + 3),
                         dot3(v.x, v.y, v.z, c_XYZ2Opp + 6), 0.f);
}

// planar R,G,B -> inline XYZ float4 (CL:79-90), for hq_rgb_to_xyz
__global__ __launch_bounds__(256) void rgb_to_xyz_kernel(const float* R, const float* G,
                                                         const float* B, float4* xyz, int64_t n) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= n) return;
    const float lr = srgb_lin(R[q]), lg = srgb_lin(G[q]), lb = srgb_lin(B[q]);
    xyz[q] = make_float4(dot3(lr, lg, lb, c_RGB2XYZ + 0), dot3(lr, lg, lb, c_RGB2XYZ + 3),
                         dot3(lr, lg, lb, c_RGB2XYZ + 6), 0.f);
}

// Horizontal 1-D pass of convolve4Channels / convolve1Channel (CL:2-74) on the
// extended rows: out = sum_t fma(in[refl], k[t], acc), chans 3 (.xyz) or 1 (.x).
__global__ __launch_bounds__(256) void labref_hconv_kernel(const float4* in, float4* out,
                                                           const float* k, int half, int chans,
                                                           int W, int64_t n) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= n) return;
    const int ly = (int)(q / W), x = (int)(q % W);
    const float4* row = in + (int64_t)ly * W;
    float ax = 0.f, ay = 0.f, az = 0.f;
    for (int i = -half, t = 0; i <= half; ++i, ++t) {
        const float4 v = row[reflect_only(x + i, W)];
        ax = fmaf(v.x, k[4 * t + 0], ax);
        if (chans == 3) {
            ay = fmaf(v.y, k[4 * t + 1], ay);
            az = fmaf(v.z, k[4 * t + 2], az);
        }
    }
    out[q] = make_float4(ax, ay, az, 0.f);
}

// Vertical pass over the owned rows reading the extended rows; update = 1
// accumulates into conv like the `update` flag of CL:30-36 / CL:67-73.
__global__ __launch_bounds__(256) void labref_vconv_kernel(const float4* in, float4* conv,
                                                           const float* k, int half, int chans,
                                                           int update, Geom g) {
    const int64_t n_own = (int64_t)g.W * (g.r1 - g.r0);
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= n_own) return;
    const int y = g.r0 + (int)(q / g.W), x = (int)(q % g.W);
    float ax = 0.f, ay = 0.f, az = 0.f;
    for (int i = -half, t = 0; i <= half; ++i, ++t) {
        const float4 v = in[(int64_t)(reflect_only(y + i, g.H) - g.e0) * g.W + x];
        ax = fmaf(v.x, k[4 * t + 0], ax);
        if (chans == 3) {
            ay = fmaf(v.y, k[4 * t + 1], ay);
            az = fmaf(v.z, k[4 * t + 2], az);
        }
    }
    float4 o = conv[q];
    if (update) {
        o.x += ax;
        if (chans == 3) { o.y += ay; o.z += az; }
    } else {
        o.x = ax;
        if (chans == 3) { o.y = ay; o.z = az; }
    }
    conv[q] = o;
}

// conv (Opp) -> Lab (CL:124-145, true division) -> planar L,A,B (pitch) and
// optional inline float4 copy.
__global__ __launch_bounds__(256) void labref_lab_kernel(const float4* conv, float* L, float* A,
                                                         float* B, float4* inline4, int W,
                                                         int64_t n, int pitch, float ilx,
                                                         float ily, float ilz) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= n) return;
    const float4 o = conv[q];
    const float il[3] = {ilx, ily, ilz};
    const float3 lab = opp2lab_ref(o.x, o.y, o.z, il);
    if (L) {
        const int64_t off = (q / W) * pitch + (q % W);
        L[off] = lab.x; A[off] = lab.y; B[off] = lab.z;
    }
    if (inline4) inline4[q] = make_float4(lab.x, lab.y, lab.z, 0.f);
}

// inline float4 Lab (owned rows) -> planar with pitch
__global__ __launch_bounds__(256) void lab_to_planar_kernel(const float4* lab4, float* L, float* A,
                                                            float* B, int W, int64_t n, int pitch) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= n) return;
    const float4 v = lab4[q];
    const int64_t off = (q / W) * pitch + (q % W);
    L[off] = v.x; A[off] = v.y; B[off] = v.z;
}

// ----------------------------------------------------------------------------
// Final quantize (CL:147-170): exhaustive argmin, any K, chosen colour out.
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void quantize_kernel(const float4* in, const float4* colors,
                                                       int K, int* used, float4* out, int64_t n) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= n) return;
    const float4 px = in[q];
    float4 bc = colors[0];
    float best = sqrtf(dist2(px.x, px.y, px.z, bc));
    int bi = 0;
    for (int i = 1; i < K; ++i) {
        const float4 c = colors[i];
        const float d = sqrtf(dist2(px.x, px.y, px.z, c));
        if (d < best) { best = d; bc = c; bi = i; }
    }
    out[q] = bc;
    if (used[bi] == 0) atomicOr(&used[bi], 1);
}

// CIEDE (CL:201-231) + error image of IM:886-893, fp64 block partials.
template <int DE>
__global__ __launch_bounds__(256) void error_image_kernel(const float4* orig, const float4* quant,
                                                          float4* err_img, double* partial,
                                                          int64_t n) {
    __shared__ double s_red[4];
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    double v = 0.0;
    if (q < n) {
        const float4 a = orig[q], b = quant[q];
        const float e = delta_e<DE>(a.x, a.y, a.z, b.x, b.y, b.z);
        const float im = ((255.f - e) * (255.f - e)) / (255.f * 255.f);
        if (err_img) err_img[q] = make_float4(im, im, im, 0.f);
        v = e;
    }
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) partial[blockIdx.x] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
}

// ----------------------------------------------------------------------------
// cost_pair (cost_tile 4 / 5): the 8-row tile with s_v stored as row pairs,
// float2 (row 2m, row 2m+1) per column.  The horizontal pass then runs
// v_pk_fma_f32 across a row pair, so every tap reads a naturally aligned
// register pair: the row layout's odd taps needed register-pair shuffles (17
// moves per filter and item, ~29% of the pass's VALU instructions).  HR output
// columns per item: HR = 2 gives 216 items per tile (balanced over 256 threads)
// at 1.8x the LDS reads per output; HR = 4 keeps the reads but fills 108 threads.
// ----------------------------------------------------------------------------

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

template <int HALF, int TH, int RW, int HR, bool TRIM>
__device__ __forceinline__ void hpass_pair_all(const f32x4* src, TapsPtr<HALF> taps,
                                               f32x2 (&acc0)[HR], f32x2 (&acc1)[HR],
                                               f32x2 (&acc2)[HR]) {
    constexpr int T2 = 2 * HALF;
#pragma unroll
    for (int xo = 0; xo < HR; ++xo) acc0[xo] = acc1[xo] = acc2[xo] = f32x2{0.f, 0.f};
    if constexpr (TRIM) {
        hpass_pair_filters<HALF, TH, RW, HR, kTrimLo[0], kTrimHi[0]>(src, taps, 0, 1, acc0);
        hpass_pair_filters<HALF, TH, RW, HR, 0, T2>(src, taps, 1, 3, acc0);
        hpass_pair_filters<HALF, TH, RW, HR, kTrimLo[1], kTrimHi[1]>(src, taps, 3, 4, acc1);
        hpass_pair_filters<HALF, TH, RW, HR, 0, T2>(src, taps, 4, 5, acc1);
        hpass_pair_filters<HALF, TH, RW, HR, kTrimLo[2], kTrimHi[2]>(src, taps, 5, 6, acc2);
        hpass_pair_filters<HALF, TH, RW, HR, 0, T2>(src, taps, 6, 7, acc2);
    } else {
        hpass_pair_filters<HALF, TH, RW, HR, 0, T2>(src, taps, 0, 3, acc0);
        hpass_pair_filters<HALF, TH, RW, HR, 0, T2>(src, taps, 3, 5, acc1);
        hpass_pair_filters<HALF, TH, RW, HR, 0, T2>(src, taps, 5, 7, acc2);
    }
}

template <int DE, bool TRIM, int HR>
__global__ __launch_bounds__(256, 4) void cost_pair_kernel(CostArgs a, int P_) {
    constexpr int HALF = 10, RW = 128, TH = 8, RV = 4;
    constexpr int TW = RW - 2 * HALF, RH = TH + 2 * HALF, NIN = RV + 2 * HALF;
    constexpr int NRUN = TW / HR;
    constexpr int SLOTS = HR == 2 ? 64 : 32;  // run slots per row pair: 16-lane b128 groups
    constexpr int NITEM = (TH / 2) * SLOTS;  // read consecutive 16-B columns pairs
    static_assert(TW % HR == 0 && NRUN <= SLOTS && NITEM <= 256, "H items");
    __shared__ f32x4 s_vq[kNumFilt * (TH / 2) * RW / 2];  // float2 per (filter, pair, column)
    __shared__ float4 s_opp[kMaxK];
    __shared__ __attribute__((aligned(16))) uint8_t s_idx[RH * RW];
    __shared__ double s_red[4];
    float* s_v = reinterpret_cast<float*>(s_vq);
    const int tid = threadIdx.x;
    const Geom& g = a.g;
    const TileItem cur = tile_item<TW, TH>(a, xcd_remap(blockIdx.x, a.band_tiles * P_), P_);
    const TapsPtr<HALF> taps = (TapsPtr<HALF>)(uintptr_t)a.taps;

    TileFill<HALF, RW, TH> fill;
    fill.issue(a, cur, tid);
    if (tid < a.K) s_opp[tid] = fill.ov;
    fill.template commit_idx<RW>(a, s_idx, tid);
    // this thread's H item: row pair m, columns HR*jr .. +HR-1; its LabRef now
    const int m = tid / SLOTS, jr = tid % SLOTS;
    const bool has_item = tid < NITEM && jr < NRUN;
    const int gy0 = cur.y0 + 2 * m, gx0 = cur.x0 + HR * jr;
    float labv[2][3][HR];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const bool ok = has_item && gy0 + r < g.r1 && gx0 < g.W;
        const uint32_t off = ok ? (uint32_t)((gy0 + r - g.r0) * g.lab_pitch + gx0) : 0u;
        const float* src3[3] = {a.labL, a.labA, a.labB};
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            const char* base = reinterpret_cast<const char*>(src3[ch]) + (off << 2);  // 32-bit bytes
            if constexpr (HR == 4) {
                const float4 v = *reinterpret_cast<const float4*>(base);
                labv[r][ch][0] = v.x; labv[r][ch][1] = v.y; labv[r][ch][2] = v.z; labv[r][ch][3] = v.w;
            } else {
                const float2 v = *reinterpret_cast<const float2*>(base);
                labv[r][ch][0] = v.x; labv[r][ch][1] = v.y;
            }
        }
    }
    __syncthreads();

    // ---- vertical pass (row-pair output layout): thread = (column c, rows RV*gr..) ----
    {
        const int c = tid % RW, gr = tid / RW;
        float o0[NIN], o1[NIN], o2[NIN];
        float wsum = 0.f;  // .w (= 0) is consumed so the gather stays one ds_read_b128
#pragma unroll
        for (int r = 0; r < NIN; ++r) {
            const float4 v = s_opp[s_idx[(gr * RV + r) * RW + c]];
            o0[r] = v.x; o1[r] = v.y; o2[r] = v.z;
            wsum += v.w;
        }
        o0[0] += wsum;  // wsum == 0 exactly (prep_palette writes .w = 0)
        vpass_all<HALF, RV, TH, RW, TRIM, true>(o0, o1, o2, taps, s_v + ((gr * RV / 2) * RW + c) * 2);
    }
    __syncthreads();

    // ---- horizontal pass over the row pair + Lab + dE ----
    double sum = 0.0;
    if (has_item) {
        f32x2 acc0[HR], acc1[HR], acc2[HR];
        hpass_pair_all<HALF, TH, RW, HR, TRIM>(&s_vq[(m * RW + HR * jr) / 2], taps, acc0, acc1, acc2);
        float part = 0.f;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
#pragma unroll
            for (int xo = 0; xo < HR; ++xo) {
                const float3 l3 = opp2lab_fast(acc0[xo][r], acc1[xo][r], acc2[xo][r], a.m_lab);
                const float e = delta_e<DE>(labv[r][0][xo], labv[r][1][xo], labv[r][2][xo], l3.x,
                                            l3.y, l3.z);
                part += (gy0 + r < g.r1 && gx0 + xo < g.W) ? e : 0.f;
            }
        }
        sum = (double)part;
    }
    sum = wave_sum_to_lane63(sum);
    if ((tid & 63) == 63) s_red[tid >> 6] = sum;
    __syncthreads();
    if (tid == 0)
        a.partial[(int64_t)cur.p * a.ntiles + cur.tile] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
}


// ----------------------------------------------------------------------------
// cost_chan (cost_tile 6): cost_pair's tile and passes, run in two channel
// groups -- channel 0's three filters (V then H), then channels 1-2's four --
// so s_v holds at most four filter planes (16 KiB instead of 28) and each V
// pass gathers only its group's channels from planar opponent tables (24 or 48
// values live instead of 72).  23 KiB of LDS and <= 80 VGPRs: 6 workgroups per
// CU instead of 4, more waves to cover the prologue's memory latency, for two
// more barriers and the index bytes read twice.  LabRef is loaded after the
// last vertical pass (loaded up front it spilled at 80 VGPRs).
// ----------------------------------------------------------------------------
template <int DE, bool TRIM>
__global__ __launch_bounds__(256, 6) void cost_chan_kernel(CostArgs a, int P_) {
    constexpr int HALF = 10, RW = 128, TH = 8, RV = 4, HR = 2, T2 = 2 * HALF;
    constexpr int TW = RW - 2 * HALF, RH = TH + 2 * HALF, NIN = RV + 2 * HALF;
    constexpr int NRUN = TW / HR, SLOTS = 64, NITEM = (TH / 2) * SLOTS;
    constexpr int PLANE = (TH / 2) * RW / 2;  // f32x4 per filter plane (row pairs)
    static_assert(NRUN <= SLOTS && NITEM <= 256, "H items");
    __shared__ f32x4 s_vq[4 * PLANE];
    __shared__ float s_ox[kMaxK];
    __shared__ float2 s_oyz[kMaxK];
    __shared__ __attribute__((aligned(16))) uint8_t s_idx[RH * RW];
    __shared__ double s_red[4];
    float* s_v = reinterpret_cast<float*>(s_vq);
    const int tid = threadIdx.x;
    const Geom& g = a.g;
    const TileItem cur = tile_item<TW, TH>(a, xcd_remap(blockIdx.x, a.band_tiles * P_), P_);
    const TapsPtr<HALF> taps = (TapsPtr<HALF>)(uintptr_t)a.taps;

    TileFill<HALF, RW, TH> fill;
    fill.issue(a, cur, tid);
    if (tid < a.K) {
        s_ox[tid] = fill.ov.x;
        s_oyz[tid] = make_float2(fill.ov.y, fill.ov.z);
    }
    fill.template commit_idx<RW>(a, s_idx, tid);
    const int m = tid / SLOTS, jr = tid % SLOTS;
    const bool has_item = tid < NITEM && jr < NRUN;
    const int gy0 = cur.y0 + 2 * m, gx0 = cur.x0 + HR * jr;
    __syncthreads();

    const int c = tid % RW, gr = tid / RW;
    float* vout = s_v + ((gr * RV / 2) * RW + c) * 2;
    const f32x4* hsrc = &s_vq[(m * RW + HR * jr) / 2];
    f32x2 acc0[HR], acc1[HR], acc2[HR];
#pragma unroll
    for (int xo = 0; xo < HR; ++xo) acc0[xo] = acc1[xo] = acc2[xo] = f32x2{0.f, 0.f};

    // ---- group 0: channel 0 (filters 0-2 -> planes 0-2) ----
    {
        float o[NIN];
#pragma unroll
        for (int r = 0; r < NIN; ++r) o[r] = s_ox[s_idx[(gr * RV + r) * RW + c]];
        if constexpr (TRIM) {
            vpass_filters<HALF, RV, TH, RW, kTrimLo[0], kTrimHi[0], true>(o, taps, 0, 1, vout);
            vpass_filters<HALF, RV, TH, RW, 0, T2, true>(o, taps, 1, 3, vout);
        } else {
            vpass_filters<HALF, RV, TH, RW, 0, T2, true>(o, taps, 0, 3, vout);
        }
    }
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

    // ---- group 1: channels 1 and 2 (filters 3-6 -> planes 0-3) ----
    {
        float o1[NIN], o2[NIN];
#pragma unroll
        for (int r = 0; r < NIN; ++r) {
            const float2 v = s_oyz[s_idx[(gr * RV + r) * RW + c]];
            o1[r] = v.x; o2[r] = v.y;
        }
        if constexpr (TRIM) {
            vpass_filters<HALF, RV, TH, RW, kTrimLo[1], kTrimHi[1], true>(o1, taps, 3, 4, vout, 3);
            vpass_filters<HALF, RV, TH, RW, 0, T2, true>(o1, taps, 4, 5, vout, 3);
            vpass_filters<HALF, RV, TH, RW, kTrimLo[2], kTrimHi[2], true>(o2, taps, 5, 6, vout, 3);
            vpass_filters<HALF, RV, TH, RW, 0, T2, true>(o2, taps, 6, 7, vout, 3);
        } else {
            vpass_filters<HALF, RV, TH, RW, 0, T2, true>(o1, taps, 3, 5, vout, 3);
            vpass_filters<HALF, RV, TH, RW, 0, T2, true>(o2, taps, 5, 7, vout, 3);
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
                const float3 l3 = opp2lab_fast(acc0[xo][r], acc1[xo][r], acc2[xo][r], a.m_lab);
                const float e = delta_e<DE>(labv[r][0][xo], labv[r][1][xo], labv[r][2][xo], l3.x,
                                            l3.y, l3.z);
                part += (gy0 + r < g.r1 && gx0 + xo < g.W) ? e : 0.f;
            }
        }
        sum = (double)part;
    }
    sum = wave_sum_to_lane63(sum);
    if ((tid & 63) == 63) s_red[tid >> 6] = sum;
    __syncthreads();
    if (tid == 0)
        a.partial[(int64_t)cur.p * a.ntiles + cur.tile] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
}


// ----------------------------------------------------------------------------
// cost_mfma (cost_tile 7): cost_chan with both vertical passes on the matrix
// cores in split f16 (cf. vpass_mfma): per 16-column block and pair of filters
// of one channel, one v_mfma_f32_16x16x32_f16 K-step covers the 28 region rows
// (+4 zero-weight rows) as hi.hi + hi.lo + lo.hi (each product exact in the
// fp32 accumulator; lo.lo ~2^-22 relative is dropped).  A = the stacked
// Toeplitz taps (rows = filter pair x 8 output rows, x 2^16, split on the host:
// build_vpass_f16_stack_fragments), B = the gathered opponent values (x 2^14),
// read from per-channel (hi, lo) f16 dword tables that the prologue splits once
// per tile, so the gathers need no conversion (one LDS read per value).  D (x 2^30, folded exactly into the
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

__device__ __forceinline__ f32x4v mfma3(const f16x8& ah, const f16x8& al, const f16x8& bh,
                                        const f16x8& bl) {
    f32x4v d = {0.f, 0.f, 0.f, 0.f};
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, d, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, d, 0, 0, 0);
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
    const TileItem cur = tile_item<TW, TH>(a, xcd_remap(blockIdx.x, a.band_tiles * P_), P_);
    const TapsPtr<HALF> taps = (TapsPtr<HALF>)(uintptr_t)a.taps;  // H taps x 2^-30
    const int lane = tid & 63, wv = tid >> 6, lc = lane & 15, lk = lane >> 4;
    const uint4* frag = a.vfrag16 + (TRIM ? 4 * 2 * 64 : 0) + lane;  // [trim][stack][hi,lo][lane]

    TileFill<HALF, RW, TH> fill;
    fill.issue(a, cur, tid);
    uint4 F0h = frag[(0 * 2 + 0) * 64], F0l = frag[(0 * 2 + 1) * 64];  // group 0 stacks
    uint4 F1h = frag[(1 * 2 + 0) * 64], F1l = frag[(1 * 2 + 1) * 64];
    // every entry (zeros for tid >= K): the zero-weight rows 28-31 gather arbitrary
    // indices, and 0 x NaN would be NaN
    s_ox[tid] = split_f16(fill.ov.x);
    s_oyz[tid] = make_uint2(split_f16(fill.ov.y), split_f16(fill.ov.z));
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
            for (int j = 0; j < 8; ++j) w[j] = s_ox[s_idx[(8 * lk + j) * RW + col0 + 16 * bb]];
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
                const uint2 e = s_oyz[s_idx[(8 * lk + j) * RW + col0 + 16 * bb]];
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
                const float3 l3 = opp2lab_fast(acc0[xo][r], acc1[xo][r], acc2[xo][r], a.m_lab);
                const float e = delta_e<DE>(labv[r][0][xo], labv[r][1][xo], labv[r][2][xo], l3.x,
                                            l3.y, l3.z);
                part += (gy0 + r < g.r1 && gx0 + xo < g.W) ? e : 0.f;
            }
        }
        sum = (double)part;
    }
    sum = wave_sum_to_lane63(sum);
    if ((tid & 63) == 63) s_red[tid >> 6] = sum;
    __syncthreads();
    if (tid == 0)
        a.partial[(int64_t)cur.p * a.ntiles + cur.tile] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
}


// ----------------------------------------------------------------------------
// cost_wide (cost_tile 11): cost_mfma with horizontal items of 4 output columns
// of a row pair (108 items on waves 0-1): each filter's window is 24 row-pair
// columns = 12 ds_read_b128 for 8 outputs, against 11 for cost_mfma's 4.  The
// horizontal windows were ~45% of cost_mfma's LDS cycles, and LDS is what bounds
// it.  A plain row-pair layout would put item j's reads 32 B apart, two lanes of
// every 16-lane b128 group in one bank (why cost_tile 5 never paid); here each
// row-pair row stores its column pairs split by parity: pair p = col / 2 goes to
// half p & 1, position p >> 1, so read q of item j lands at half q & 1, position
// j + q / 2 -- 16 B apart across the lanes, conflict-free.  The halves are 72
// float2 apart (8 mod 16), so the V pass's 16-column float2 stores stay
// conflict-free too.
// ----------------------------------------------------------------------------
constexpr int kWideHalf = 72;  // float2 per half of a permuted row-pair row (64 + 8 pad)

// float2 position of column `col` in a permuted row-pair row
__device__ __forceinline__ int wide_pos(int col) {
    return ((col >> 1) & 1) * kWideHalf + ((col >> 2) << 1) + (col & 1);
}

template <int HALF, int TLO = 0, int THI = 2 * HALF>
__device__ __forceinline__ void hpass_wide_filters(const f32x4* src, TapsPtr<HALF> taps, int f0,
                                                   int f1, f32x2 (&acc)[4], int fslot, int pstride) {
    constexpr int HR = 4, NIN = HR + 2 * HALF, NQ = NIN / 2;  // 12 reads of 2 columns
#pragma unroll 1
    for (int f = f0; f < f1; ++f) {
        const f32x4* row = src + (f - fslot) * pstride;
        f32x4 v[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) v[q] = row[(q & 1) * (kWideHalf / 2) + (q >> 1)];
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

// D of one 16x16 stack block -> permuted row pairs (cf. store_vstack)
__device__ __forceinline__ void store_vstack_wide(float* s_v, const f32x4v& d, int plane_a,
                                                  int plane_b, int lk, int col) {
    constexpr int PAIRS = 4, ROW = 2 * kWideHalf;  // float2 per row-pair row
    const int plane = lk < 2 ? plane_a : plane_b;
    if (plane < 0) return;
    const int p0 = 2 * (lk & 1);
    f32x2* v = reinterpret_cast<f32x2*>(s_v);
    const int pos = wide_pos(col);
    v[(plane * PAIRS + p0) * ROW + pos] = f32x2{d[0], d[1]};
    v[(plane * PAIRS + p0 + 1) * ROW + pos] = f32x2{d[2], d[3]};
}

template <int DE, bool TRIM>
__global__ __launch_bounds__(256, 6) void cost_wide_kernel(CostArgs a, int P_) {
    constexpr int HALF = 10, RW = 128, TH = 8, HR = 4, T2 = 2 * HALF;
    constexpr int TW = RW - 2 * HALF, RH = TH + 2 * HALF;
    constexpr int NRUN = TW / HR;                 // 27 items per row pair, 32 slots
    constexpr int ROW = 2 * kWideHalf;            // float2 per row-pair row
    constexpr int PLANE4 = (TH / 2) * ROW / 2;    // f32x4 per filter plane
    static_assert(NRUN <= 32 && RH <= 32 && 4 * PLANE4 >= 512, "tile");
    __shared__ f32x4 s_vq[4 * PLANE4];
    __shared__ uint32_t s_ox[kMaxK];  // opponent x 2^14 as (hi, lo) f16 pairs: channel 0
    __shared__ uint2 s_oyz[kMaxK];     // channels 1, 2
    __shared__ __attribute__((aligned(16))) uint8_t s_idx[32 * RW];
    __shared__ double s_red[4];
    float* s_v = reinterpret_cast<float*>(s_vq);
    const int tid = threadIdx.x;
    const Geom& g = a.g;
    const TileItem cur = tile_item<TW, TH>(a, xcd_remap(blockIdx.x, a.band_tiles * P_), P_);
    const TapsPtr<HALF> taps = (TapsPtr<HALF>)(uintptr_t)a.taps;  // H taps x 2^-30
    const int lane = tid & 63, wv = tid >> 6, lc = lane & 15, lk = lane >> 4;
    const uint4* frag = a.vfrag16 + (TRIM ? 4 * 2 * 64 : 0) + lane;  // [trim][stack][hi,lo][lane]

    TileFill<HALF, RW, TH> fill;
    fill.issue(a, cur, tid);
    uint4 F0h = frag[(0 * 2 + 0) * 64], F0l = frag[(0 * 2 + 1) * 64];
    uint4 F1h = frag[(1 * 2 + 0) * 64], F1l = frag[(1 * 2 + 1) * 64];
    s_ox[tid] = split_f16(fill.ov.x);
    s_oyz[tid] = make_uint2(split_f16(fill.ov.y), split_f16(fill.ov.z));
    fill.template commit_idx<RW>(a, s_idx, tid);
    // H item: row pair m, output columns 4j .. 4j+3, shared by thread t (half 0,
    // waves 0-1) and t + 128 (half 1): each applies about half of every channel
    // group's taps -- half 0 filters 0, 1 (ch 0) and 3, 4 (ch 1), half 1 filter 2
    // (ch 0) and 5, 6 (ch 2) -- and finishes one row of the pair after an exchange
    // of partial sums, so all four waves carry the same horizontal work.
    const int hh = tid >> 7, it = tid & 127, m = it >> 5, jr = it & 31;
    const bool has_item = jr < NRUN;
    const int gy = cur.y0 + 2 * m + hh, gx0 = cur.x0 + HR * jr;  // the row this thread finishes
    __syncthreads();

    const int col0 = 32 * wv + lc;
    const f32x4* hsrc = &s_vq[(m * ROW) / 2 + jr];
    f32x2 accA[HR], accB[HR];  // half 0: ch 0 part, ch 1; half 1: ch 0 part, ch 2
#pragma unroll
    for (int xo = 0; xo < HR; ++xo) accA[xo] = accB[xo] = f32x2{0.f, 0.f};

    // ---- group 0: channel 0 -> planes 0-2 ----
    {
        const f16x8 a0h = __builtin_bit_cast(f16x8, F0h), a0l = __builtin_bit_cast(f16x8, F0l);
        const f16x8 a1h = __builtin_bit_cast(f16x8, F1h), a1l = __builtin_bit_cast(f16x8, F1l);
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            uint32_t w[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) w[j] = s_ox[s_idx[(8 * lk + j) * RW + col0 + 16 * bb]];
            f16x8 bh, bl;
            pack_b(w, bh, bl);
            store_vstack_wide(s_v, mfma3(a0h, a0l, bh, bl), 0, 1, lk, col0 + 16 * bb);
            store_vstack_wide(s_v, mfma3(a1h, a1l, bh, bl), 2, -1, lk, col0 + 16 * bb);
        }
    }
    const uint4 F2h = frag[(2 * 2 + 0) * 64], F2l = frag[(2 * 2 + 1) * 64];
    const uint4 F3h = frag[(3 * 2 + 0) * 64], F3l = frag[(3 * 2 + 1) * 64];
    __syncthreads();
    if (has_item) {
        if (hh == 0) {
            if constexpr (TRIM) hpass_wide_filters<HALF, kTrimLo[0], kTrimHi[0]>(hsrc, taps, 0, 1, accA, 0, PLANE4);
            else hpass_wide_filters<HALF, 0, T2>(hsrc, taps, 0, 1, accA, 0, PLANE4);
            hpass_wide_filters<HALF, 0, T2>(hsrc, taps, 1, 2, accA, 0, PLANE4);
        } else {
            hpass_wide_filters<HALF, 0, T2>(hsrc, taps, 2, 3, accA, 0, PLANE4);
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
                const uint2 e = s_oyz[s_idx[(8 * lk + j) * RW + col0 + 16 * bb]];
                wy[j] = e.x; wz[j] = e.y;
            }
            f16x8 bh, bl;
            pack_b(wy, bh, bl);
            store_vstack_wide(s_v, mfma3(a2h, a2l, bh, bl), 0, 1, lk, col0 + 16 * bb);
            pack_b(wz, bh, bl);
            store_vstack_wide(s_v, mfma3(a3h, a3l, bh, bl), 2, 3, lk, col0 + 16 * bb);
        }
    }
    __syncthreads();
    if (has_item) {
        const int fa = hh == 0 ? 3 : 5;  // trimmed filter of the channel
        if constexpr (TRIM) {
            if (hh == 0) hpass_wide_filters<HALF, kTrimLo[1], kTrimHi[1]>(hsrc, taps, 3, 4, accB, 3, PLANE4);
            else hpass_wide_filters<HALF, kTrimLo[2], kTrimHi[2]>(hsrc, taps, 5, 6, accB, 3, PLANE4);
        } else {
            hpass_wide_filters<HALF, 0, T2>(hsrc, taps, fa, fa + 1, accB, 3, PLANE4);
        }
        hpass_wide_filters<HALF, 0, T2>(hsrc, taps, fa + 1, fa + 2, accB, 3, PLANE4);
    }
    // LabRef of the finished row, in flight across the exchange
    float4 L4 = make_float4(0.f, 0.f, 0.f, 0.f), A4 = L4, B4 = L4;
    {
        const bool ok = has_item && gy < g.r1 && gx0 < g.W;
        const uint32_t off = ok ? (uint32_t)((gy - g.r0) * g.lab_pitch + gx0) : 0u;
        L4 = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(a.labL) + (off << 2));
        A4 = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(a.labA) + (off << 2));
        B4 = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(a.labB) + (off << 2));
    }
    __syncthreads();
    // exchange: each thread passes on the row the other half finishes (row 1 - hh)
    {
        const int o = 1 - hh;
        s_vq[tid] = f32x4{accA[0][o], accA[1][o], accA[2][o], accA[3][o]};
        s_vq[256 + tid] = f32x4{accB[0][o], accB[1][o], accB[2][o], accB[3][o]};
    }
    __syncthreads();
    double sum = 0.0;
    if (has_item) {
        const f32x4 pA = s_vq[tid ^ 128], pB = s_vq[256 + (tid ^ 128)];
        const float Ls[4] = {L4.x, L4.y, L4.z, L4.w}, As[4] = {A4.x, A4.y, A4.z, A4.w},
                    Bs[4] = {B4.x, B4.y, B4.z, B4.w};
        float part = 0.f;
#pragma unroll
        for (int xo = 0; xo < HR; ++xo) {
            const float c0 = accA[xo][hh] + pA[xo];           // channel 0: both halves' filters
            const float c1 = hh == 0 ? accB[xo][0] : pB[xo];  // channel 1: half 0's
            const float c2 = hh == 0 ? pB[xo] : accB[xo][1];  // channel 2: half 1's
            const float3 l3 = opp2lab_fast(c0, c1, c2, a.m_lab);
            const float e = delta_e<DE>(Ls[xo], As[xo], Bs[xo], l3.x, l3.y, l3.z);
            part += (gy < g.r1 && gx0 + xo < g.W) ? e : 0.f;
        }
        sum = (double)part;
    }
    sum = wave_sum_to_lane63(sum);
    if ((tid & 63) == 63) s_red[tid >> 6] = sum;
    __syncthreads();
    if (tid == 0)
        a.partial[(int64_t)cur.p * a.ntiles + cur.tile] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
}


// ----------------------------------------------------------------------------
// cost_vt (cost_tile 9): cost_mfma with the vertical pass's operand roles
// swapped, V^T = X^T . T^T, so each lane's D is 4 consecutive columns of one
// output row (one ds_write_b128 per stack block), the horizontal pass on
// 1-row x 4-column items (a 24-float window: 6 ds_read_b128 per filter for 4
// outputs, against 11 for the row-pair items' 4 outputs), and the index region
// stored column-major (CP bytes per column, rows contiguous), so a lane reads
// the 8 region rows of its column with one ds_read_b64 instead of 8 ds_read_u8.
// What bounds cost_mfma is LDS issue (PMC: ~78% of cycles LDS-active), and the
// horizontal windows and the byte-wise index reads were ~half of it.
// ----------------------------------------------------------------------------
template <int HALF, int TH, int VP, int TLO = 0, int THI = 2 * HALF>
__device__ __forceinline__ void hpass_row_filters(const f32x4* src, TapsPtr<HALF> taps, int f0,
                                                  int f1, float (&acc)[4], int fslot) {
    constexpr int NQ = (4 + 2 * HALF + 3) / 4;
    static_assert(NQ == 6, "the asm barrier below names six vectors");
#pragma unroll 1
    for (int f = f0; f < f1; ++f) {
        const f32x4* row = src + (f - fslot) * TH * VP / 4;
        f32x4 v0 = row[0], v1 = row[1], v2 = row[2], v3 = row[3], v4 = row[4], v5 = row[5];
        asm volatile("" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5));
        const f32x4 vv[NQ] = {v0, v1, v2, v3, v4, v5};
        float in[4 * NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            in[4 * q] = vv[q].x; in[4 * q + 1] = vv[q].y; in[4 * q + 2] = vv[q].z; in[4 * q + 3] = vv[q].w;
        }
#pragma unroll
        for (int t = TLO; t <= THI; ++t) {
            const float k = taps->h[f][t];
#pragma unroll
            for (int xo = 0; xo < 4; ++xo) acc[xo] = fmaf(in[xo + t], k, acc[xo]);
        }
    }
}

// 4 x 4 byte transpose: v[i] byte c -> w[c] byte i.
__device__ __forceinline__ void transpose4x4_u8(const uint32_t (&v)[4], uint32_t (&w)[4]) {
    const uint32_t lo01 = __builtin_amdgcn_perm(v[1], v[0], 0x05010400u);  // v0b0 v1b0 v0b1 v1b1
    const uint32_t hi01 = __builtin_amdgcn_perm(v[1], v[0], 0x07030602u);  // v0b2 v1b2 v0b3 v1b3
    const uint32_t lo23 = __builtin_amdgcn_perm(v[3], v[2], 0x05010400u);
    const uint32_t hi23 = __builtin_amdgcn_perm(v[3], v[2], 0x07030602u);
    w[0] = __builtin_amdgcn_perm(lo23, lo01, 0x05040100u);
    w[1] = __builtin_amdgcn_perm(lo23, lo01, 0x07060302u);
    w[2] = __builtin_amdgcn_perm(hi23, hi01, 0x05040100u);
    w[3] = __builtin_amdgcn_perm(hi23, hi01, 0x07060302u);
}

// Column-major fill of the 28 (+4 zero) x 128 index region: thread (cb = tid >> 3,
// rb = tid & 7) loads rows 4rb .. 4rb+3 of region columns 4cb .. 4cb+3 (aligned
// dword pairs + alignbyte, all loads before the first wait) and stores their
// transpose as 4 dwords (4 rows of one column each).  Edge tiles gather bytes
// with reflection at commit time.
template <int HALF, int CP>
struct TileFillT {
    static constexpr int RW = 128, TH = 8, TW = RW - 2 * HALF, RH = TH + 2 * HALF;
    static_assert(RH == 28 && CP % 8 == 0 && CP >= 32, "7 row blocks of 4 + one zero block");
    uint32_t lo[4], hi[4], sh[4];
    float4 ov;
    TileItem t;
    bool interior;

    __device__ __forceinline__ static int row_base(const Geom& g, const TileItem& t, int i) {
        int gy = reflect_clamp(t.y0 - HALF + i, g.H);
        gy = min(max(gy, g.e0), g.e1 - 1);
        return (gy - g.e0) * g.W + (t.x0 - HALF);
    }

    __device__ __forceinline__ void issue(const CostArgs& a, const TileItem& ti, int tid) {
        const Geom& g = a.g;
        t = ti;
        const uint8_t* idx = a.idx + (int64_t)t.p * g.idx_pitch;
        ov = tid < a.K ? a.opp[(int64_t)t.p * kMaxK + tid] : make_float4(0.f, 0.f, 0.f, 0.f);
        interior = t.x0 - HALF >= 0 && t.x0 + TW + HALF <= g.W;
        if (interior) {
            const int cb = tid >> 3, rb = min(tid & 7, 6);  // rb 7: the zero rows (loads discarded)
            const int ytop = t.y0 - HALF;
            const bool vfast = ytop >= 0 && ytop >= g.e0 && ytop + RH <= g.H && ytop + RH <= g.e1;
            const int ubase = (ytop - g.e0) * g.W + (t.x0 - HALF);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = 4 * rb + i;
                const uint32_t off = (uint32_t)(vfast ? ubase + row * g.W : row_base(g, t, row));
                sh[i] = off & 3u;
                const uint32_t* src = reinterpret_cast<const uint32_t*>(idx + ((off & ~3u) + 4u * (uint32_t)cb));
                lo[i] = src[0];
                hi[i] = src[1];
            }
        }
    }

    __device__ __forceinline__ void commit_idx(const CostArgs& a, uint8_t* s_idx, int tid) const {
        const Geom& g = a.g;
        if (interior) {
            const int cb = tid >> 3, rb = tid & 7;
            uint32_t v[4], w[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = rb < 7 ? __builtin_amdgcn_alignbyte(hi[i], lo[i], sh[i]) : 0u;
            transpose4x4_u8(v, w);
#pragma unroll
            for (int c = 0; c < 4; ++c)
                *reinterpret_cast<uint32_t*>(s_idx + (4 * cb + c) * CP + 4 * rb) = w[c];
        } else {
            constexpr int NFB = (RH * RW + 255) / 256;
            const uint8_t* idx = a.idx + (int64_t)t.p * g.idx_pitch;
            uint32_t b[NFB];
#pragma unroll
            for (int q = 0; q < NFB; ++q) {  // all loads first: one round trip
                const int e = min(tid + 256 * q, RH * RW - 1);
                const int i = e / RW, j = e % RW;
                int gy = reflect_clamp(t.y0 - HALF + i, g.H);
                gy = min(max(gy, g.e0), g.e1 - 1);
                const int gx = reflect_clamp(t.x0 - HALF + j, g.W);
                b[q] = idx[(uint32_t)((gy - g.e0) * g.W + gx)];
            }
#pragma unroll
            for (int q = 0; q < NFB; ++q) {
                const int e = tid + 256 * q;
                if (e < RH * RW) s_idx[(e % RW) * CP + e / RW] = (uint8_t)b[q];
            }
            if (tid < RW) *reinterpret_cast<uint32_t*>(s_idx + tid * CP + RH) = 0u;  // rows 28-31
        }
    }
};

// D of one V^T stack block -> s_v rows: lane (c4 = l >> 4, n = l & 15) holds
// columns 4 c4 .. +3 of output row n & 7 of the stack's filter n >> 3.
template <int TH, int VP>
__device__ __forceinline__ void store_vt(float* s_v, const f32x4v& d, int plane_a, int plane_b,
                                         int n, int col) {
    const int plane = n < 8 ? plane_a : plane_b;
    if (plane < 0) return;
    *reinterpret_cast<f32x4v*>(s_v + (plane * TH + (n & 7)) * VP + col) = d;
}

template <int DE, bool TRIM>
__global__ __launch_bounds__(256, 6) void cost_vt_kernel(CostArgs a, int P_) {
    constexpr int HALF = 10, RW = 128, TH = 8, T2 = 2 * HALF;
    constexpr int TW = RW - 2 * HALF;
    constexpr int NRUN = TW / 4;  // 27 runs of 4 output columns per row, 32 slots
    constexpr int CP = 48;        // bytes per region column (32 rows + pad: conflict-free b64 reads)
    constexpr int VP = RW + 4;    // floats per s_v row (528 B = 16 mod 128: conflict-free b128 stores)
    __shared__ f32x4 s_v4[4 * TH * VP / 4];
    __shared__ uint32_t s_ox[kMaxK];  // opponent x 2^14 as (hi, lo) f16 pairs: channel 0
    __shared__ uint2 s_oyz[kMaxK];     // channels 1, 2
    __shared__ __attribute__((aligned(16))) uint8_t s_idx[RW * CP];
    __shared__ double s_red[4];
    float* s_v = reinterpret_cast<float*>(s_v4);
    const int tid = threadIdx.x;
    const Geom& g = a.g;
    const TileItem cur = tile_item<TW, TH>(a, xcd_remap(blockIdx.x, a.band_tiles * P_), P_);
    const TapsPtr<HALF> taps = (TapsPtr<HALF>)(uintptr_t)a.taps;  // H taps x 2^-30
    const int lane = tid & 63, wv = tid >> 6, lc = lane & 15, lk = lane >> 4;
    const uint4* frag = a.vfrag16 + (TRIM ? 4 * 2 * 64 : 0) + lane;  // [trim][stack][hi,lo][lane]

    TileFillT<HALF, CP> fill;
    fill.issue(a, cur, tid);
    uint4 F0h = frag[(0 * 2 + 0) * 64], F0l = frag[(0 * 2 + 1) * 64];  // group 0 stacks
    uint4 F1h = frag[(1 * 2 + 0) * 64], F1l = frag[(1 * 2 + 1) * 64];
    // every entry (zeros for tid >= K): the zero-weight rows 28-31 gather index 0
    s_ox[tid] = split_f16(fill.ov.x);
    s_oyz[tid] = make_uint2(split_f16(fill.ov.y), split_f16(fill.ov.z));
    fill.commit_idx(a, s_idx, tid);
    // H item: row y, output columns 4j .. 4j+3
    const int y = tid >> 5, j = tid & 31;
    const bool has_item = j < NRUN;
    const int gy = cur.y0 + y, gx0 = cur.x0 + 4 * j;
    __syncthreads();

    // V pass: lane (c = lc, q = lk) gathers region rows 8q .. 8q+7 of column
    // 32 wv + 16 bb + c (A = X^T fragment), D = 4 columns of one (filter, row)
    const int colA = 32 * wv + lc;
    const int colD = 32 * wv + 4 * lk;
    const f32x4* hsrc = &s_v4[(y * VP) / 4 + j];
    float acc0[4] = {0.f, 0.f, 0.f, 0.f}, acc1[4] = {0.f, 0.f, 0.f, 0.f}, acc2[4] = {0.f, 0.f, 0.f, 0.f};

    // ---- group 0: channel 0 -> planes 0-2 ----
    {
        const f16x8 t0h = __builtin_bit_cast(f16x8, F0h), t0l = __builtin_bit_cast(f16x8, F0l);
        const f16x8 t1h = __builtin_bit_cast(f16x8, F1h), t1l = __builtin_bit_cast(f16x8, F1l);
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            const uint2 ix = *reinterpret_cast<const uint2*>(s_idx + (colA + 16 * bb) * CP + 8 * lk);
            uint32_t w[8];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                w[jj] = s_ox[(ix.x >> (8 * jj)) & 0xffu];
                w[4 + jj] = s_ox[(ix.y >> (8 * jj)) & 0xffu];
            }
            f16x8 xh, xl;
            pack_b(w, xh, xl);
            store_vt<TH, VP>(s_v, mfma3(xh, xl, t0h, t0l), 0, 1, lc, colD + 16 * bb);
            store_vt<TH, VP>(s_v, mfma3(xh, xl, t1h, t1l), 2, -1, lc, colD + 16 * bb);
        }
    }
    const uint4 F2h = frag[(2 * 2 + 0) * 64], F2l = frag[(2 * 2 + 1) * 64];  // group 1 stacks,
    const uint4 F3h = frag[(3 * 2 + 0) * 64], F3l = frag[(3 * 2 + 1) * 64];  // in flight during H
    __syncthreads();
    if (has_item) {
        if constexpr (TRIM) {
            hpass_row_filters<HALF, TH, VP, kTrimLo[0], kTrimHi[0]>(hsrc, taps, 0, 1, acc0, 0);
            hpass_row_filters<HALF, TH, VP, 0, T2>(hsrc, taps, 1, 3, acc0, 0);
        } else {
            hpass_row_filters<HALF, TH, VP, 0, T2>(hsrc, taps, 0, 3, acc0, 0);
        }
    }
    __syncthreads();

    // ---- group 1: channels 1, 2 -> planes 0-3 ----
    {
        const f16x8 t2h = __builtin_bit_cast(f16x8, F2h), t2l = __builtin_bit_cast(f16x8, F2l);
        const f16x8 t3h = __builtin_bit_cast(f16x8, F3h), t3l = __builtin_bit_cast(f16x8, F3l);
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            const uint2 ix = *reinterpret_cast<const uint2*>(s_idx + (colA + 16 * bb) * CP + 8 * lk);
            uint32_t wy[8], wz[8];
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
                const uint2 e = s_oyz[((jj < 4 ? ix.x : ix.y) >> (8 * (jj & 3))) & 0xffu];
                wy[jj] = e.x; wz[jj] = e.y;
            }
            f16x8 xh, xl;
            pack_b(wy, xh, xl);
            store_vt<TH, VP>(s_v, mfma3(xh, xl, t2h, t2l), 0, 1, lc, colD + 16 * bb);
            pack_b(wz, xh, xl);
            store_vt<TH, VP>(s_v, mfma3(xh, xl, t3h, t3l), 2, 3, lc, colD + 16 * bb);
        }
    }
    float4 Lr = make_float4(0.f, 0.f, 0.f, 0.f), Ar = Lr, Br = Lr;
    {
        const bool ok = has_item && gy < g.r1 && gx0 < g.W;
        const uint32_t off = ok ? (uint32_t)((gy - g.r0) * g.lab_pitch + gx0) : 0u;
        Lr = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(a.labL) + (off << 2));
        Ar = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(a.labA) + (off << 2));
        Br = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(a.labB) + (off << 2));
    }
    __syncthreads();

    double sum = 0.0;
    if (has_item) {
        if constexpr (TRIM) {
            hpass_row_filters<HALF, TH, VP, kTrimLo[1], kTrimHi[1]>(hsrc, taps, 3, 4, acc1, 3);
            hpass_row_filters<HALF, TH, VP, 0, T2>(hsrc, taps, 4, 5, acc1, 3);
            hpass_row_filters<HALF, TH, VP, kTrimLo[2], kTrimHi[2]>(hsrc, taps, 5, 6, acc2, 3);
            hpass_row_filters<HALF, TH, VP, 0, T2>(hsrc, taps, 6, 7, acc2, 3);
        } else {
            hpass_row_filters<HALF, TH, VP, 0, T2>(hsrc, taps, 3, 5, acc1, 3);
            hpass_row_filters<HALF, TH, VP, 0, T2>(hsrc, taps, 5, 7, acc2, 3);
        }
        const float Ls[4] = {Lr.x, Lr.y, Lr.z, Lr.w}, As[4] = {Ar.x, Ar.y, Ar.z, Ar.w},
                    Bs[4] = {Br.x, Br.y, Br.z, Br.w};
        float part = 0.f;
#pragma unroll
        for (int xo = 0; xo < 4; ++xo) {
            const float3 l3 = opp2lab_fast(acc0[xo], acc1[xo], acc2[xo], a.m_lab);
            const float e = delta_e<DE>(Ls[xo], As[xo], Bs[xo], l3.x, l3.y, l3.z);
            part += (gy < g.r1 && gx0 + xo < g.W) ? e : 0.f;
        }
        sum = (double)part;
    }
    sum = wave_sum_to_lane63(sum);
    if ((tid & 63) == 63) s_red[tid >> 6] = sum;
    __syncthreads();
    if (tid == 0)
        a.partial[(int64_t)cur.p * a.ntiles + cur.tile] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
}


// ----------------------------------------------------------------------------
// cost_mm (cost_tile 8): both stencil passes on the matrix cores in split f16,
// Lab / dE on VALU.  Tile = 8 rows x 96 output columns (8 blocks of 12), region
// 28 (+4 zero-weight) rows x 128 columns, two opponent-channel groups as in
// cost_mfma.
//  - vertical pass: as cost_mfma (stacked filter pairs, one K = 32 step per
//    16-column block), but D (x 2^30) is rescaled to x 2^12 and stored as f16
//    hi / lo (hi = f16(v), lo = f16(v - hi)) in row-major planes;
//  - horizontal pass: per 12-column output block, the 32 input columns of its
//    window are one K = 32 step: D[x][n] += Htap[x][k] * V[row][12b + k] with
//    n = (block of the wave's pair, row), hi.hi + hi.lo + lo.hi per filter, the
//    filters of one channel accumulated in one D (x 2^28, folded into the
//    Opp -> XYZ rows by the host, exactly);
//  - Lab / dE: lane (n, q) holds output columns 12b + 4q .. +3 of one row
//    (q = 3 is padding), LabRef as float4 loads.
// LDS per tile: the H-pass B fragments are 2 x 16 B per lane and filter
// (cost_pair's horizontal windows were 1.2 KB per item), the V-pass stores one
// f16 per value and half.
// ----------------------------------------------------------------------------
constexpr int kMMTW = 96;                          // output columns per tile
constexpr float kVToH = 1.0f / 262144.0f;          // 2^-18: V-pass D (x 2^30) -> x 2^12
constexpr float kHTapScale = 65536.0f;             // 2^16
constexpr float kHOutScale = 1.0f / 268435456.0f;  // 2^-28 (into m_lab)

typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

// D of one V stack block -> f16 hi / lo rows of the planes: lane (c = l & 15,
// q = l >> 4) holds rows 4(q & 1) .. +3 of filter q >> 1 at column `col`.
template <int RS>
__device__ __forceinline__ void store_vstack_f16(_Float16* s_vh, const f32x4v& d, int plane_a,
                                                 int plane_b, int lk, int col) {
    constexpr int RW = 128;
    const int plane = lk < 2 ? plane_a : plane_b;
    if (plane < 0) return;
    _Float16* base = s_vh + (plane * 8 + 4 * (lk & 1)) * RS + col;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        const float x = d[v] * kVToH;
        const _Float16 hi = (_Float16)x;
        base[v * RS] = hi;
        base[v * RS + RW] = (_Float16)(x - (float)hi);
    }
}

template <int DE, bool TRIM>
__global__ __launch_bounds__(256, 6) void cost_mm_kernel(CostArgs a, int P_) {
    constexpr int HALF = 10, RW = 128, TH = 8, TW = kMMTW, RH = TH + 2 * HALF;
    constexpr int RS = 2 * RW + 16;  // halves per plane row: hi row, lo row, 32 B pad
    static_assert(RH <= 32 && TW == 8 * 12 && 12 * 7 + 32 <= RW, "tile");
    __shared__ __attribute__((aligned(16))) _Float16 s_vh[4 * TH * RS];
    __shared__ uint32_t s_ox[kMaxK];
    __shared__ uint2 s_oyz[kMaxK];
    __shared__ __attribute__((aligned(16))) uint8_t s_idx[32 * RW];
    __shared__ double s_red[4];
    const int tid = threadIdx.x;
    const Geom& g = a.g;
    const TileItem cur = tile_item<TW, TH>(a, xcd_remap(blockIdx.x, a.band_tiles * P_), P_);
    const int lane = tid & 63, wv = tid >> 6, lc = lane & 15, lk = lane >> 4;
    const uint4* vfrag = a.vfrag16 + (TRIM ? 4 * 2 * 64 : 0) + lane;  // [trim][stack][hi,lo][lane]
    const uint4* hfrag = a.hfrag16 + (TRIM ? 7 * 2 * 64 : 0) + lane;  // [trim][filter][hi,lo][lane]

    TileFill<HALF, RW, TH> fill;  // region x0 - 10 .. x0 + 117 (stride 96)
    fill.issue(a, cur, tid);
    const uint4 F0h = vfrag[0 * 64], F0l = vfrag[1 * 64], F1h = vfrag[2 * 64], F1l = vfrag[3 * 64];
    s_ox[tid] = split_f16(fill.ov.x);  // every entry (zeros past K): rows 28-31 gather any index
    s_oyz[tid] = make_uint2(split_f16(fill.ov.y), split_f16(fill.ov.z));
    fill.template commit_idx<RW>(a, s_idx, tid);
    __syncthreads();

    const int col0 = 32 * wv + lc;  // V pass: region columns of this wave's two 16-blocks
    // H pass: lane (n = lc, q = lk): output block ob = 2 wv + (n >> 3), row hr = n & 7,
    // B = input columns 12 ob + 8q .. +7 of row hr
    const int ob = 2 * wv + (lc >> 3), hr = lc & 7;
    const _Float16* hb = s_vh + hr * RS + 12 * ob + 8 * lk;
    f32x4v D0 = {0.f, 0.f, 0.f, 0.f}, D1 = D0, D2 = D0;

    auto hpass = [&](int f, int plane, f32x4v& D) {
        const f16x8 ah = __builtin_bit_cast(f16x8, hfrag[(2 * f) * 64]);
        const f16x8 al = __builtin_bit_cast(f16x8, hfrag[(2 * f + 1) * 64]);
        const _Float16* p = hb + plane * 8 * RS;
        const f16x4 h0 = *reinterpret_cast<const f16x4*>(p), h1 = *reinterpret_cast<const f16x4*>(p + 4);
        const f16x4 l0 = *reinterpret_cast<const f16x4*>(p + RW),
                    l1 = *reinterpret_cast<const f16x4*>(p + RW + 4);
        const f16x8 bh = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
        const f16x8 bl = __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7);
        D = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, D, 0, 0, 0);
        D = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, D, 0, 0, 0);
        D = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, D, 0, 0, 0);
    };

    // ---- group 0: channel 0 ----
    {
        const f16x8 a0h = __builtin_bit_cast(f16x8, F0h), a0l = __builtin_bit_cast(f16x8, F0l);
        const f16x8 a1h = __builtin_bit_cast(f16x8, F1h), a1l = __builtin_bit_cast(f16x8, F1l);
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            uint32_t w[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) w[j] = s_ox[s_idx[(8 * lk + j) * RW + col0 + 16 * bb]];
            f16x8 bh, bl;
            pack_b(w, bh, bl);
            store_vstack_f16<RS>(s_vh, mfma3(a0h, a0l, bh, bl), 0, 1, lk, col0 + 16 * bb);
            store_vstack_f16<RS>(s_vh, mfma3(a1h, a1l, bh, bl), 2, -1, lk, col0 + 16 * bb);
        }
    }
    const uint4 F2h = vfrag[4 * 64], F2l = vfrag[5 * 64], F3h = vfrag[6 * 64], F3l = vfrag[7 * 64];
    __syncthreads();
    hpass(0, 0, D0);
    hpass(1, 1, D0);
    hpass(2, 2, D0);
    __syncthreads();

    // ---- group 1: channels 1, 2 ----
    {
        const f16x8 a2h = __builtin_bit_cast(f16x8, F2h), a2l = __builtin_bit_cast(f16x8, F2l);
        const f16x8 a3h = __builtin_bit_cast(f16x8, F3h), a3l = __builtin_bit_cast(f16x8, F3l);
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            uint32_t wy[8], wz[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint2 e = s_oyz[s_idx[(8 * lk + j) * RW + col0 + 16 * bb]];
                wy[j] = e.x; wz[j] = e.y;
            }
            f16x8 bh, bl;
            pack_b(wy, bh, bl);
            store_vstack_f16<RS>(s_vh, mfma3(a2h, a2l, bh, bl), 0, 1, lk, col0 + 16 * bb);
            pack_b(wz, bh, bl);
            store_vstack_f16<RS>(s_vh, mfma3(a3h, a3l, bh, bl), 2, 3, lk, col0 + 16 * bb);
        }
    }
    // LabRef of this lane's 4 outputs (row hr, columns 12 ob + 4 lk .. +3), in flight
    const int gy = cur.y0 + hr, gx = cur.x0 + 12 * ob + 4 * lk;
    const bool lab_ok = lk < 3 && gy < g.r1 && gx < g.W;
    const uint32_t loff = lab_ok ? (uint32_t)((gy - g.r0) * g.lab_pitch + gx) : 0u;
    const float4 Lr = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(a.labL) + (loff << 2));
    const float4 Ar = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(a.labA) + (loff << 2));
    const float4 Br = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(a.labB) + (loff << 2));
    __syncthreads();
    hpass(3, 0, D1);
    hpass(4, 1, D1);
    hpass(5, 2, D2);
    hpass(6, 3, D2);

    float part = 0.f;
    if (lk < 3) {
        const float lr[4] = {Lr.x, Lr.y, Lr.z, Lr.w}, ar[4] = {Ar.x, Ar.y, Ar.z, Ar.w},
                    br[4] = {Br.x, Br.y, Br.z, Br.w};
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const float3 l3 = opp2lab_fast(D0[v], D1[v], D2[v], a.m_lab);
            const float e = delta_e<DE>(lr[v], ar[v], br[v], l3.x, l3.y, l3.z);
            part += (gy < g.r1 && gx + v < g.W) ? e : 0.f;
        }
    }
    double sum = wave_sum_to_lane63((double)part);
    if ((tid & 63) == 63) s_red[tid >> 6] = sum;
    __syncthreads();
    if (tid == 0)
        a.partial[(int64_t)cur.p * a.ntiles + cur.tile] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
}

// ----------------------------------------------------------------------------
// cost_mh (cost_tile 10): both stencil passes on the matrix cores, built on
// cost_vt's layout.  Tile = 8 rows x 96 output columns (8 blocks of 12), region
// 28 (+4 zero) rows x 128 columns, column-major indices, two channel groups.
//  - vertical pass: V^T = X^T . T^T as in cost_vt; each lane's D (4 columns of
//    one filter row, x 2^30) is rescaled to x 2^12 and split into f16 hi / lo,
//    one ds_write_b64 each into row-major planes (cost_mm wrote 8 ds_write_b16);
//  - horizontal pass: per 12-column output block the 32 window columns are one
//    K = 32 step, D[x][n] += Htap[x][k] . V[row][12 ob + k], n = (block of the
//    wave's pair, row); the B fragment is 2 ds_read_b64 per half, the filters of
//    a channel accumulate in one D (x 2^28, folded into the Opp -> XYZ rows);
//  - no horizontal FMAs on the VALU and no horizontal windows in LDS (cost_vt's
//    6 ds_read_b128 per filter and item).
// s_vh: per (plane, row) a 544-B block = hi row (256 B), lo row (256 B), 32 B pad:
// the B reads (rows r, 8 B at column offsets {0, 16, 24, 40} B) are conflict-free
// at a stride of 32 (mod 256) B; planes are 16 B apart mod 128 for the stores.
// ----------------------------------------------------------------------------
template <int DE, bool TRIM>
__global__ __launch_bounds__(256, 6) void cost_mh_kernel(CostArgs a, int P_) {
    constexpr int HALF = 10, RW = 128, TH = 8, TW = kMMTW;
    constexpr int CP = 48;                    // bytes per region column (column-major indices)
    constexpr int RB = 544;                   // bytes per (plane, row) block: hi, lo, pad
    constexpr int PB = TH * RB + 16;          // bytes per plane
    static_assert(TW == 8 * 12 && 12 * 7 + 32 <= RW, "tile");
    __shared__ __attribute__((aligned(16))) uint8_t s_vh[4 * PB];
    __shared__ uint32_t s_ox[kMaxK];
    __shared__ uint2 s_oyz[kMaxK];
    __shared__ __attribute__((aligned(16))) uint8_t s_idx[RW * CP];
    __shared__ double s_red[4];
    const int tid = threadIdx.x;
    const Geom& g = a.g;
    const TileItem cur = tile_item<TW, TH>(a, xcd_remap(blockIdx.x, a.band_tiles * P_), P_);
    const int lane = tid & 63, wv = tid >> 6, lc = lane & 15, lk = lane >> 4;
    const uint4* vfrag = a.vfrag16 + (TRIM ? 4 * 2 * 64 : 0) + lane;  // [trim][stack][hi,lo][lane]
    const uint4* hfrag = a.hfrag16 + (TRIM ? 7 * 2 * 64 : 0) + lane;  // [trim][filter][hi,lo][lane]
    TileFillT<HALF, CP> fill;  // region x0 - 10 .. x0 + 117
    fill.issue(a, cur, tid);
    const uint4 F0h = vfrag[0 * 64], F0l = vfrag[1 * 64], F1h = vfrag[2 * 64], F1l = vfrag[3 * 64];
    s_ox[tid] = split_f16(fill.ov.x);  // every entry (zeros past K): rows 28-31 gather index 0
    s_oyz[tid] = make_uint2(split_f16(fill.ov.y), split_f16(fill.ov.z));
    fill.commit_idx(a, s_idx, tid);
    __syncthreads();

    // V pass: lane (c = lc, q = lk) gathers region rows 8q .. +7 of column 32 wv + 16 bb + c
    const int colA = 32 * wv + lc;
    const int colD = 32 * wv + 4 * lk;  // + 16 bb: this lane's 4 D columns
    auto store_v = [&](const f32x4v& d, int plane_a, int plane_b, int col) {
        const int plane = lc < 8 ? plane_a : plane_b;
        if (plane < 0) return;
        uint8_t* base = s_vh + plane * PB + (lc & 7) * RB + col * 2;
        f16x4 h, l;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const float x = d[v] * kVToH;
            h[v] = (_Float16)x;
            l[v] = (_Float16)(x - (float)h[v]);
        }
        *reinterpret_cast<f16x4*>(base) = h;
        *reinterpret_cast<f16x4*>(base + 256) = l;
    };
    // H pass: lane (n = lc, q = lk): output block ob = 2 wv + (n >> 3), row hr = n & 7,
    // B = window columns 12 ob + 8q .. +7 of row hr
    const int ob = 2 * wv + (lc >> 3), hr = lc & 7;
    const uint8_t* hb = s_vh + hr * RB + (12 * ob + 8 * lk) * 2;
    f32x4v D0 = {0.f, 0.f, 0.f, 0.f}, D1 = D0, D2 = D0;
    // The two 8-B halves of a B fragment are separate ds_read_b64 (32-lane groups over
    // 64 banks: conflict-free at this row stride); an opaque offset keeps the compiler
    // from merging them into one ds_read2_b64 (16-lane groups over 32 banks: 2-way).
    uint32_t o8 = 8, o256 = 256, o264 = 264;
    asm volatile("" : "+v"(o8), "+v"(o256), "+v"(o264));
    auto hpass = [&](int f, int plane, f32x4v& D) {
        const uint4 fh = hfrag[(2 * f) * 64], fl = hfrag[(2 * f + 1) * 64];
        const f16x8 ah = __builtin_bit_cast(f16x8, fh), al = __builtin_bit_cast(f16x8, fl);
        const uint8_t* p = hb + plane * PB;
        const f16x4 h0 = *reinterpret_cast<const f16x4*>(p), h1 = *reinterpret_cast<const f16x4*>(p + o8);
        const f16x4 l0 = *reinterpret_cast<const f16x4*>(p + o256),
                    l1 = *reinterpret_cast<const f16x4*>(p + o264);
        const f16x8 bh = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
        const f16x8 bl = __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7);
        D = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, D, 0, 0, 0);
        D = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, D, 0, 0, 0);
        D = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, D, 0, 0, 0);
    };

    // ---- group 0: channel 0 ----
    {
        const f16x8 t0h = __builtin_bit_cast(f16x8, F0h), t0l = __builtin_bit_cast(f16x8, F0l);
        const f16x8 t1h = __builtin_bit_cast(f16x8, F1h), t1l = __builtin_bit_cast(f16x8, F1l);
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            const uint2 ix = *reinterpret_cast<const uint2*>(s_idx + (colA + 16 * bb) * CP + 8 * lk);
            uint32_t w[8];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                w[jj] = s_ox[(ix.x >> (8 * jj)) & 0xffu];
                w[4 + jj] = s_ox[(ix.y >> (8 * jj)) & 0xffu];
            }
            f16x8 xh, xl;
            pack_b(w, xh, xl);
            store_v(mfma3(xh, xl, t0h, t0l), 0, 1, colD + 16 * bb);
            store_v(mfma3(xh, xl, t1h, t1l), 2, -1, colD + 16 * bb);
        }
    }
    const uint4 F2h = vfrag[4 * 64], F2l = vfrag[5 * 64], F3h = vfrag[6 * 64], F3l = vfrag[7 * 64];
    __syncthreads();
    hpass(0, 0, D0);
    hpass(1, 1, D0);
    hpass(2, 2, D0);
    __syncthreads();

    // ---- group 1: channels 1, 2 ----
    {
        const f16x8 t2h = __builtin_bit_cast(f16x8, F2h), t2l = __builtin_bit_cast(f16x8, F2l);
        const f16x8 t3h = __builtin_bit_cast(f16x8, F3h), t3l = __builtin_bit_cast(f16x8, F3l);
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            const uint2 ix = *reinterpret_cast<const uint2*>(s_idx + (colA + 16 * bb) * CP + 8 * lk);
            uint32_t wy[8], wz[8];
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
                const uint2 e = s_oyz[((jj < 4 ? ix.x : ix.y) >> (8 * (jj & 3))) & 0xffu];
                wy[jj] = e.x; wz[jj] = e.y;
            }
            f16x8 xh, xl;
            pack_b(wy, xh, xl);
            store_v(mfma3(xh, xl, t2h, t2l), 0, 1, colD + 16 * bb);
            pack_b(wz, xh, xl);
            store_v(mfma3(xh, xl, t3h, t3l), 2, 3, colD + 16 * bb);
        }
    }
    // LabRef of this lane's 4 outputs (row hr, columns 12 ob + 4 lk .. +3), in flight
    const int gy = cur.y0 + hr, gx = cur.x0 + 12 * ob + 4 * lk;
    const bool lab_ok = lk < 3 && gy < g.r1 && gx < g.W;
    const uint32_t loff = lab_ok ? (uint32_t)((gy - g.r0) * g.lab_pitch + gx) : 0u;
    const float4 Lr = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(a.labL) + (loff << 2));
    const float4 Ar = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(a.labA) + (loff << 2));
    const float4 Br = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(a.labB) + (loff << 2));
    __syncthreads();
    hpass(3, 0, D1);
    hpass(4, 1, D1);
    hpass(5, 2, D2);
    hpass(6, 3, D2);

    float part = 0.f;
    if (lk < 3) {
        const float lr[4] = {Lr.x, Lr.y, Lr.z, Lr.w}, ar[4] = {Ar.x, Ar.y, Ar.z, Ar.w},
                    br[4] = {Br.x, Br.y, Br.z, Br.w};
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const float3 l3 = opp2lab_fast(D0[v], D1[v], D2[v], a.m_lab);
            const float e = delta_e<DE>(lr[v], ar[v], br[v], l3.x, l3.y, l3.z);
            part += (gy < g.r1 && gx + v < g.W) ? e : 0.f;
        }
    }
    double sum = wave_sum_to_lane63((double)part);
    if ((tid & 63) == 63) s_red[tid >> 6] = sum;
    __syncthreads();
    if (tid == 0)
        a.partial[(int64_t)cur.p * a.ntiles + cur.tile] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
}

// ----------------------------------------------------------------------------
// Launchers (host side of this translation unit)
// ----------------------------------------------------------------------------
static inline unsigned blocks_for(int64_t n) { return (unsigned)((n + 255) / 256); }

void opp2xyz_over_illum(const float inv_illum[3], float m[9]) {
    static const float opp2xyz[9] = HQ_OPP2XYZ;
    for (int i = 0; i < 9; ++i) m[i] = opp2xyz[i] * inv_illum[i / 3];
}

// Profiling: the next launches carry start/stop events in their dispatch packet
// (hipExtLaunchKernel), so timing a kernel adds no marker packet between kernels
// (each hipEventRecord between two kernels left the GPU idle ~5 us).
static thread_local hipEvent_t t_ev_start = nullptr, t_ev_stop = nullptr;
void set_launch_events(hipEvent_t start, hipEvent_t stop) {
    t_ev_start = start;
    t_ev_stop = stop;
}
#define HQ_LAUNCH(K, G, B, S, STREAM, ...)                                                   \
    do {                                                                                     \
        if (t_ev_start || t_ev_stop)                                                         \
            hipExtLaunchKernelGGL(K, G, B, S, STREAM, t_ev_start, t_ev_stop, 0, __VA_ARGS__); \
        else                                                                                 \
            hipLaunchKernelGGL(K, G, B, S, STREAM, __VA_ARGS__);                             \
    } while (0)

hipError_t launch_prep_palette(const PaletteArgs& a, int P, hipStream_t s) {
    HQ_LAUNCH(prep_palette_kernel, dim3(P), dim3(1024), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_sa_step(const SaArgs& a, hipStream_t s) {
    HQ_LAUNCH(sa_step_kernel, dim3(a.P), dim3(1024), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_sa_grid(const SaArgs& a, const GridArgs& ga, hipStream_t s) {
    HQ_LAUNCH(sa_grid_kernel, dim3(ga.G1 * ga.G1 * ga.G1, a.P), dim3(256), 0, s, a, ga);
    return hipGetLastError();
}

hipError_t launch_build_grid(const GridArgs& a, int P, hipStream_t s) {
    HQ_LAUNCH(build_grid_kernel, dim3(a.G1 * a.G1 * a.G1, P), dim3(256), 0, s, a);
    return hipGetLastError();
}

template <int REP>
static hipError_t launch_assign_rep(const AssignArgs& a, int P, hipStream_t s) {
    const size_t lds = (size_t)a.K * REP * sizeof(float4);
    static bool attr_set = false;  // allow > 64 KiB of dynamic LDS (160 KiB per CU on gfx950)
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)assign_kernel<REP>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)(kMaxK * REP * sizeof(float4)));
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    HQ_LAUNCH(assign_kernel<REP>, dim3(a.nblocks * P), dim3(256), lds, s, a, P);
    return hipGetLastError();
}

template <int REP, int PG>
static hipError_t launch_assign_multi(const AssignArgs& a, int P, hipStream_t s) {
    const size_t lds = (size_t)PG * a.K * REP * sizeof(float4);
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)assign_multi_kernel<REP, PG>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)(PG * kMaxK * REP * sizeof(float4)));
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    HQ_LAUNCH((assign_multi_kernel<REP, PG>), dim3(a.nblocks, (P + PG - 1) / PG),
                       dim3(256), lds, s, a, P);
    return hipGetLastError();
}

template <int PPT>
static hipError_t launch_assign_batch(const AssignArgs& a, int P, hipStream_t s) {
    const size_t lds = (size_t)a.K * sizeof(float4);
    HQ_LAUNCH((assign_batch_kernel<1, PPT>), dim3(a.nblocks * P), dim3(256), lds, s, a, P);
    return hipGetLastError();
}

// rep: LDS replication of the palette (1, 4 or 16); lane l reads copy l % rep.
// group > 1: one pixel pass serves `group` palettes (assign_multi_kernel).
// batch: 4 or 8 = assign_batch_kernel with that many pixels per round trip
// (single palette copy), 0 = assign_kernel; with group 4, batch 1 or 2 =
// assign_quad_kernel (4 palettes per pixel pass, PPT = batch).
template <int PPT>
static hipError_t launch_assign_quad(const AssignArgs& a, int P, hipStream_t s) {
    const size_t lds = (size_t)4 * a.K * sizeof(float4);
    const unsigned grid = (unsigned)(a.nblocks * ((P + 3) / 4));
    HQ_LAUNCH((assign_quad_kernel<PPT>), dim3(grid), dim3(256), lds, s, a, P);
    return hipGetLastError();
}

static hipError_t launch_assign_pipe(const AssignArgs& a, int P, hipStream_t s) {
    const size_t lds = 0;  // static [NG][kMaxK] palette table
    const unsigned grid = (unsigned)(a.nblocks * ((P + 3) / 4));
    switch (P) {
    case 1: HQ_LAUNCH(assign_pipe_kernel<1>, dim3(grid), dim3(256), lds, s, a, P); break;
    case 2: HQ_LAUNCH(assign_pipe_kernel<2>, dim3(grid), dim3(256), lds, s, a, P); break;
    case 3: HQ_LAUNCH(assign_pipe_kernel<3>, dim3(grid), dim3(256), lds, s, a, P); break;
    default: HQ_LAUNCH(assign_pipe_kernel<4>, dim3(grid), dim3(256), lds, s, a, P); break;
    }
    return hipGetLastError();
}

static hipError_t launch_assign_lane(const AssignArgs& a, int P, hipStream_t s) {
    const size_t lds = (size_t)4 * a.K * sizeof(float4);
    const unsigned grid = (unsigned)(a.nblocks * ((P + 3) / 4));
    HQ_LAUNCH(assign_lane_kernel, dim3(grid), dim3(256), lds, s, a, P);
    return hipGetLastError();
}

hipError_t launch_assign(const AssignArgs& a, int P, int rep, int group, int batch, hipStream_t s) {
    if (group == 4 && batch == 5) return launch_assign_lane(a, P, s);
    if (group == 4 && batch == 3) return launch_assign_pipe(a, P, s);
    if (group == 4 && batch == 1) return launch_assign_quad<1>(a, P, s);
    if (group == 4 && batch == 2) return launch_assign_quad<2>(a, P, s);
    if (batch == 4) return launch_assign_batch<4>(a, P, s);
    if (batch == 8) return launch_assign_batch<8>(a, P, s);
    if (group == 4) {
        if (rep == 1) return launch_assign_multi<1, 4>(a, P, s);
        if (rep == 2) return launch_assign_multi<2, 4>(a, P, s);
        return launch_assign_multi<4, 4>(a, P, s);
    }
    if (group == 2) return launch_assign_multi<4, 2>(a, P, s);
    if (rep == 16) return launch_assign_rep<16>(a, P, s);
    if (rep == 1) return launch_assign_rep<1>(a, P, s);
    return launch_assign_rep<4>(a, P, s);
}

static void make_taps10(const float* k1, const float* k2, const float* k3, const float* absk3,
                        CostTaps<10>& t) {
    for (int i = 0; i < 21; ++i) {
        // f: 0 k1.x, 1 k2.x, 2 k3 (|k3| vertical), 3 k1.y, 4 k2.y, 5 k1.z, 6 k2.z
        t.v[0][i] = k1[4 * i + 0]; t.h[0][i] = k1[4 * i + 0];
        t.v[1][i] = k2[4 * i + 0]; t.h[1][i] = k2[4 * i + 0];
        t.v[2][i] = absk3[i];      t.h[2][i] = k3[i];
        t.v[3][i] = k1[4 * i + 1]; t.h[3][i] = k1[4 * i + 1];
        t.v[4][i] = k2[4 * i + 1]; t.h[4][i] = k2[4 * i + 1];
        t.v[5][i] = k1[4 * i + 2]; t.h[5][i] = k1[4 * i + 2];
        t.v[6][i] = k2[4 * i + 2]; t.h[6][i] = k2[4 * i + 2];
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

// B fragments of v_mfma_f32_16x16x32_f16 for the matrix-core vertical pass
// (vpass_mfma): lane l holds B[k = 8(l >> 4) + j][n = l & 15], j = 0..7, with
// B[i][r] = v-tap (i - r) of the filter for output rows r < 8 and 0 <= i - r <= 20,
// scaled by 2^16 and split into hi / lo f16.  out: [7][2][64][8] f16 bits.
void build_vpass_fragments(const float* k1, const float* k2, const float* k3,
                           const float* absk3, uint16_t* out) {
    CostTaps<10> t;
    make_taps10(k1, k2, k3, absk3, t);
    for (int f = 0; f < kNumFilt; ++f)
        for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 8; ++j) {
                const int i = 8 * (l >> 4) + j, r = l & 15, d = i - r;
                const float w = (r < 8 && d >= 0 && d <= 20) ? t.v[f][d] * kVTapScale : 0.f;
                const uint16_t hi = host_f16(w);
                const uint16_t lo = host_f16(w - host_f16_to_f32(hi));
                out[((f * 2 + 0) * 64 + l) * 8 + j] = hi;
                out[((f * 2 + 1) * 64 + l) * 8 + j] = lo;
            }
}

// cost_tile 7: split-f16 A fragments of v_mfma_f32_16x16x32_f16 for the vertical
// pass, [trim][stack][hi, lo][lane] x 8 halves (trim 0 = all 21 taps, 1 = the
// narrow filters' significant windows).  Lane l holds A[i = l & 15][k = 8(l >> 4)
// + j]: the tap (x 2^16) of filter stack[i >> 3] that multiplies region row k
// into output row i & 7, i.e. tap d = k - (i & 7), zero outside [0, 20] (and
// outside the window).
size_t vpass_f16_stack_fragment_halves() { return 2 * 4 * 2 * 64 * 8; }

void build_vpass_f16_stack_fragments(const float* k1, const float* k2, const float* k3,
                                     const float* absk3, uint16_t* out) {
    CostTaps<10> t;
    make_taps10(k1, k2, k3, absk3, t);
    const int stack[4][2] = {{0, 1}, {2, -1}, {3, 4}, {5, 6}};
    for (int trim = 0; trim < 2; ++trim)
        for (int st = 0; st < 4; ++st)
            for (int l = 0; l < 64; ++l)
                for (int j = 0; j < 8; ++j) {
                    const int i = l & 15, k = 8 * (l >> 4) + j, r = i & 7, f = stack[st][i >> 3];
                    const int d = k - r;
                    float w = 0.f;
                    if (f >= 0 && d >= 0 && d <= 20) {
                        w = t.v[f][d];
                        const int ch = f == 0 ? 0 : (f == 3 ? 1 : (f == 5 ? 2 : -1));
                        if (trim && ch >= 0 && (d < kTrimLo[ch] || d > kTrimHi[ch])) w = 0.f;
                    }
                    w *= kVTapScale;
                    const uint16_t hi = host_f16(w);
                    const uint16_t lo = host_f16(w - host_f16_to_f32(hi));
                    out[(((trim * 4 + st) * 2 + 0) * 64 + l) * 8 + j] = hi;
                    out[(((trim * 4 + st) * 2 + 1) * 64 + l) * 8 + j] = lo;
                }
}

// cost_tile 8: split-f16 A fragments of the horizontal taps, [trim][filter][hi, lo]
// [lane] x 8 halves.  Lane l holds A[x = l & 15][k = 8(l >> 4) + j]: the tap (x 2^16)
// that multiplies window column k into output column x of a 12-column block, i.e.
// tap d = k - x, zero outside [0, 20], for x >= 12 (padding rows) and outside the
// narrow filters' windows when trimmed.
size_t hpass_f16_fragment_halves() { return 2 * 7 * 2 * 64 * 8; }

void build_hpass_f16_fragments(const float* k1, const float* k2, const float* k3,
                               const float* absk3, uint16_t* out) {
    CostTaps<10> t;
    make_taps10(k1, k2, k3, absk3, t);
    for (int trim = 0; trim < 2; ++trim)
        for (int f = 0; f < kNumFilt; ++f)
            for (int l = 0; l < 64; ++l)
                for (int j = 0; j < 8; ++j) {
                    const int x = l & 15, k = 8 * (l >> 4) + j, d = k - x;
                    float w = 0.f;
                    if (x < 12 && d >= 0 && d <= 20) {
                        w = t.h[f][d];
                        const int ch = f == 0 ? 0 : (f == 3 ? 1 : (f == 5 ? 2 : -1));
                        if (trim && ch >= 0 && (d < kTrimLo[ch] || d > kTrimHi[ch])) w = 0.f;
                    }
                    w *= kHTapScale;
                    const uint16_t hi = host_f16(w);
                    const uint16_t lo = host_f16(w - host_f16_to_f32(hi));
                    out[(((trim * 7 + f) * 2 + 0) * 64 + l) * 8 + j] = hi;
                    out[(((trim * 7 + f) * 2 + 1) * 64 + l) * 8 + j] = lo;
                }
}

// Tile geometry of the fast path (HALF = 10): RW = 128 region columns,
// TW = 108 output columns, TH = 16 output rows, RV = 8 rows per V item.
constexpr int kFastHalf = 10, kFastRW = 128, kFastTH = 16, kFastRV = 8;
constexpr int kFastTW = kFastRW - 2 * kFastHalf;

// tile rows of the fast path: cfg 0 = 16 (RV 8, 2 WG/CU); cfg 1 = 8 with the V
// pass split by channel group (4 WG/CU); cfg 2 = 8 (RV 4, 4 WG/CU); cfg 3 = 8
// with the V pass on the matrix cores
int fast_tile_rows(int tile_cfg) { return tile_cfg == 0 ? kFastTH : 8; }  // cfg 1-11: 8 rows

void fast_tile_dims(int W, int own_rows, int tile_cfg, int* tiles_x, int* ntiles) {
    const int th = fast_tile_rows(tile_cfg);
    const int tw = (tile_cfg == 8 || tile_cfg == 10) ? kMMTW : kFastTW;
    *tiles_x = (W + tw - 1) / tw;
    *ntiles = *tiles_x * ((own_rows + th - 1) / th);
}

template <int TH, int RV, int OCC, bool TRIM, int VMODE>
static void launch_tile_cfg(const CostArgs& a, int P, int de, hipStream_t s) {
    const dim3 grid((unsigned)(a.band_tiles * P));
    if (de == 0)
        HQ_LAUNCH((cost_tile_kernel<kFastHalf, kFastRW, TH, RV, 0, OCC, TRIM, VMODE>), grid,
                           dim3(256), 0, s, a, P);
    else
        HQ_LAUNCH((cost_tile_kernel<kFastHalf, kFastRW, TH, RV, 1, OCC, TRIM, VMODE>), grid,
                           dim3(256), 0, s, a, P);
}

// True when every tap of the narrow filters outside the trim window is below
// 1e-9 of that filter's peak (products that far under fp32 rounding).
bool trim_window_ok(const float* k1) {
    const int ch[3] = {0, 1, 2};
    for (int i = 0; i < 3; ++i) {
        float peak = 0.f;
        for (int t = 0; t < 21; ++t) peak = std::max(peak, std::fabs(k1[4 * t + ch[i]]));
        for (int t = 0; t < 21; ++t)
            if ((t < kTrimLo[i] || t > kTrimHi[i]) && std::fabs(k1[4 * t + ch[i]]) > 1e-9f * peak)
                return false;
    }
    return true;
}

size_t fast_taps_bytes() { return 2 * sizeof(CostTaps<10>); }

// [0] the taps as designed, [1] the same with the horizontal taps scaled by
// 2^-30 (exact) for the matrix-core vertical pass, whose outputs carry 2^30.
void build_fast_taps(const float* k1, const float* k2, const float* k3, const float* absk3,
                     void* out) {
    CostTaps<10> t[2];
    make_taps10(k1, k2, k3, absk3, t[0]);
    t[1] = t[0];
    for (int f = 0; f < kNumFilt; ++f)
        for (int i = 0; i < 2 * kFastHalf + 1; ++i) t[1].h[f][i] *= kVOutScale;
    std::memcpy(out, t, sizeof t);
}

// a.taps = the two CostTaps<10> of build_fast_taps
hipError_t launch_cost_fast(const CostArgs& a0, int P, int de, int tile_cfg, bool trim,
                            hipStream_t s) {
    CostArgs a = a0;
    if (tile_cfg == 3 || tile_cfg == 7 || tile_cfg == 9 || tile_cfg == 11)  // matrix-core V passes: x 2^30
        a.taps = static_cast<const char*>(a0.taps) + sizeof(CostTaps<10>);
    if (tile_cfg == 4 || tile_cfg == 5) {
        const dim3 grid((unsigned)(a.band_tiles * P));
#define HQ_PAIR(DEV, TR, HRV) HQ_LAUNCH((cost_pair_kernel<DEV, TR, HRV>), grid, dim3(256), 0, s, a, P)
        if (tile_cfg == 4) {
            if (de == 0) { if (trim) HQ_PAIR(0, true, 2); else HQ_PAIR(0, false, 2); }
            else { if (trim) HQ_PAIR(1, true, 2); else HQ_PAIR(1, false, 2); }
        } else {
            if (de == 0) { if (trim) HQ_PAIR(0, true, 4); else HQ_PAIR(0, false, 4); }
            else { if (trim) HQ_PAIR(1, true, 4); else HQ_PAIR(1, false, 4); }
        }
#undef HQ_PAIR
    } else if (tile_cfg == 6) {
        const dim3 grid((unsigned)(a.band_tiles * P));
#define HQ_CHAN(DEV, TR) HQ_LAUNCH((cost_chan_kernel<DEV, TR>), grid, dim3(256), 0, s, a, P)
        if (de == 0) { if (trim) HQ_CHAN(0, true); else HQ_CHAN(0, false); }
        else { if (trim) HQ_CHAN(1, true); else HQ_CHAN(1, false); }
#undef HQ_CHAN
    } else if (tile_cfg == 7) {
        const dim3 grid((unsigned)(a.band_tiles * P));
#define HQ_MFMA(DEV, TR) HQ_LAUNCH((cost_mfma_kernel<DEV, TR>), grid, dim3(256), 0, s, a, P)
        if (de == 0) { if (trim) HQ_MFMA(0, true); else HQ_MFMA(0, false); }
        else { if (trim) HQ_MFMA(1, true); else HQ_MFMA(1, false); }
#undef HQ_MFMA
    } else if (tile_cfg == 11) {
        const dim3 grid((unsigned)(a.band_tiles * P));
#define HQ_WIDE(DEV, TR) HQ_LAUNCH((cost_wide_kernel<DEV, TR>), grid, dim3(256), 0, s, a, P)
        if (de == 0) { if (trim) HQ_WIDE(0, true); else HQ_WIDE(0, false); }
        else { if (trim) HQ_WIDE(1, true); else HQ_WIDE(1, false); }
#undef HQ_WIDE
    } else if (tile_cfg == 9) {
        const dim3 grid((unsigned)(a.band_tiles * P));
#define HQ_VT(DEV, TR) HQ_LAUNCH((cost_vt_kernel<DEV, TR>), grid, dim3(256), 0, s, a, P)
        if (de == 0) { if (trim) HQ_VT(0, true); else HQ_VT(0, false); }
        else { if (trim) HQ_VT(1, true); else HQ_VT(1, false); }
#undef HQ_VT
    } else if (tile_cfg == 10) {
        for (int i = 0; i < 9; ++i) a.m_lab[i] *= kHOutScale;  // H outputs carry 2^28 (exact)
        const dim3 grid((unsigned)(a.band_tiles * P));
#define HQ_MH(DEV, TR) HQ_LAUNCH((cost_mh_kernel<DEV, TR>), grid, dim3(256), 0, s, a, P)
        if (de == 0) { if (trim) HQ_MH(0, true); else HQ_MH(0, false); }
        else { if (trim) HQ_MH(1, true); else HQ_MH(1, false); }
#undef HQ_MH
    } else if (tile_cfg == 8) {
        for (int i = 0; i < 9; ++i) a.m_lab[i] *= kHOutScale;  // H outputs carry 2^28 (exact)
        const dim3 grid((unsigned)(a.band_tiles * P));
#define HQ_MM(DEV, TR) HQ_LAUNCH((cost_mm_kernel<DEV, TR>), grid, dim3(256), 0, s, a, P)
        if (de == 0) { if (trim) HQ_MM(0, true); else HQ_MM(0, false); }
        else { if (trim) HQ_MM(1, true); else HQ_MM(1, false); }
#undef HQ_MM
    } else if (tile_cfg == 3) {
        if (trim) launch_tile_cfg<8, 8, 4, true, 2>(a, P, de, s);
        else launch_tile_cfg<8, 8, 4, false, 2>(a, P, de, s);
    } else if (tile_cfg == 1) {
        if (trim) launch_tile_cfg<8, 8, 4, true, 1>(a, P, de, s);
        else launch_tile_cfg<8, 8, 4, false, 1>(a, P, de, s);
    } else if (tile_cfg == 2) {
        if (trim) launch_tile_cfg<8, 4, 4, true, 0>(a, P, de, s);
        else launch_tile_cfg<8, 4, 4, false, 0>(a, P, de, s);
    } else {
        if (trim) launch_tile_cfg<kFastTH, kFastRV, 2, true, 0>(a, P, de, s);
        else launch_tile_cfg<kFastTH, kFastRV, 2, false, 0>(a, P, de, s);
    }
    return hipGetLastError();
}

hipError_t launch_cost_generic(const GenArgs& a, int de, hipStream_t s) {
    HQ_LAUNCH(gen_hpass_kernel, dim3(blocks_for(a.g.n_ext)), dim3(256), 0, s, a);
    const int64_t n_own = (int64_t)a.g.W * (a.g.r1 - a.g.r0);
    if (de == 0)
        HQ_LAUNCH(gen_vpass_kernel<0>, dim3(blocks_for(n_own)), dim3(256), 0, s, a);
    else
        HQ_LAUNCH(gen_vpass_kernel<1>, dim3(blocks_for(n_own)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_finalize(const FinalizeArgs& a, int P, hipStream_t s) {
    HQ_LAUNCH(finalize_kernel, dim3(P), dim3(1024), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_labref_opp(const float* R, const float* G, const float* B, float4* opp,
                             int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(labref_opp_kernel, dim3(blocks_for(n)), dim3(256), 0, s, R, G, B, opp, n);
    return hipGetLastError();
}

hipError_t launch_xyz_to_opp(const float4* xyz, float4* opp, int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(xyz_to_opp_kernel, dim3(blocks_for(n)), dim3(256), 0, s, xyz, opp, n);
    return hipGetLastError();
}

hipError_t launch_rgb_to_xyz(const float* R, const float* G, const float* B, float4* xyz,
                             int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(rgb_to_xyz_kernel, dim3(blocks_for(n)), dim3(256), 0, s, R, G, B, xyz, n);
    return hipGetLastError();
}

hipError_t launch_labref_hconv(const float4* in, float4* out, const float* k, int half,
                               int chans, int W, int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(labref_hconv_kernel, dim3(blocks_for(n)), dim3(256), 0, s, in, out, k,
                       half, chans, W, n);
    return hipGetLastError();
}

hipError_t launch_labref_vconv(const float4* in, float4* conv, const float* k, int half,
                               int chans, int update, const Geom& g, hipStream_t s) {
    const int64_t n_own = (int64_t)g.W * (g.r1 - g.r0);
    hipLaunchKernelGGL(labref_vconv_kernel, dim3(blocks_for(n_own)), dim3(256), 0, s, in, conv,
                       k, half, chans, update, g);
    return hipGetLastError();
}

hipError_t launch_labref_lab(const float4* conv, float* L, float* A, float* B, float4* inline4,
                             int W, int64_t n, int pitch, const float* illum, hipStream_t s) {
    hipLaunchKernelGGL(labref_lab_kernel, dim3(blocks_for(n)), dim3(256), 0, s, conv, L, A, B,
                       inline4, W, n, pitch, illum[0], illum[1], illum[2]);
    return hipGetLastError();
}

hipError_t launch_lab_to_planar(const float4* lab4, float* L, float* A, float* B, int W,
                                int64_t n, int pitch, hipStream_t s) {
    hipLaunchKernelGGL(lab_to_planar_kernel, dim3(blocks_for(n)), dim3(256), 0, s, lab4, L, A, B,
                       W, n, pitch);
    return hipGetLastError();
}

hipError_t launch_quantize(const float4* in, const float4* colors, int K, int* used, float4* out,
                           int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(quantize_kernel, dim3(blocks_for(n)), dim3(256), 0, s, in, colors, K,
                       used, out, n);
    return hipGetLastError();
}

hipError_t launch_error_image(const float4* orig, const float4* quant, float4* err_img,
                              double* partial, int64_t n, int de, hipStream_t s) {
    if (de == 0)
        hipLaunchKernelGGL(error_image_kernel<0>, dim3(blocks_for(n)), dim3(256), 0, s, orig,
                           quant, err_img, partial, n);
    else
        hipLaunchKernelGGL(error_image_kernel<1>, dim3(blocks_for(n)), dim3(256), 0, s, orig,
                           quant, err_img, partial, n);
    return hipGetLastError();
}

}  // namespace hq
