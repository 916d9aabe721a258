// hq_wide.hip -- palettes of K > 256 colours (the plugin accepts K up to
// 2^24, HybridQuantization.java:192): 32-bit palette indices, the exhaustive
// argmin of CL:179-193 over LDS-staged colour chunks, and used flags as the
// reference keeps them (int usedColors[K], CL:193).  The stencil cost of these
// populations runs the generic two-pass path on the 32-bit index image
// (hq_cost.hip, gen_*_kernel<uint32_t>).
#include "hq_device.h"
#include "hq_launch.h"

namespace hq {

// ----------------------------------------------------------------------------
// prep_wide: grid (ceil(K / 256), P), block 256.  Colour k of palette p:
// .w = 0 (SW:49), its opponent colour (CL:194-198), and pflags[p] bit 0 when a
// channel is not finite (those palettes take the reference loop verbatim).
// pflags must be zero on entry.
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void prep_wide_kernel(WideArgs a) {
    const int p = blockIdx.y, k = blockIdx.x * 256 + threadIdx.x;
    if (k >= a.K) return;
    float4 c = a.pal_in[(int64_t)p * a.K + k];
    c.w = 0.f;
    const float lr = srgb_lin(c.x), lg = srgb_lin(c.y), lb = srgb_lin(c.z);
    a.pal[(int64_t)p * a.K + k] = c;
    a.opp[(int64_t)p * a.K + k] = make_float4(dot3(lr, lg, lb, c_RGB2Opp + 0), dot3(lr, lg, lb, c_RGB2Opp + 3),
                                              dot3(lr, lg, lb, c_RGB2Opp + 6), 0.f);
    if (!(isfinite(c.x) && isfinite(c.y) && isfinite(c.z))) atomicOr(&a.pflags[p], 1);
}

// The reference loop verbatim (CL:179-192): ref_dist (hq_device.h), first
// minimum in ascending index.
__device__ __noinline__ uint32_t argmin_wide_slow(float r, float g, float b, const float4* pal, int K) {
    float best = ref_dist(r, g, b, pal[0]);
    uint32_t bi = 0;
    for (int k = 1; k < K; ++k) {
        const float d = ref_dist(r, g, b, pal[k]);
        if (d < best) { best = d; bi = (uint32_t)k; }
    }
    return bi;
}

// ----------------------------------------------------------------------------
// assign_wide: grid (ceil(n_ext / (256 * kWidePPT)), P), block 256.
// Each thread ranks kWidePPT pixels against every colour of palette p, chunk by
// chunk from LDS (a chunk entry is read by all lanes at once: a broadcast).
// Ranking is by the reference's d^2 (dist2_rank) with the runner-up tracked
// by v_med3; a pixel whose runner-up lies within 1e-6 relative of its best (or
// below 2^-125) -- where its distance could merge the two and the lower index
// would win (CL:186) -- or that is not finite, or whose palette
// has a non-finite colour, is re-resolved by the reference loop (the argument
// of argmin_from_entry, hq_assign.hip).  Used flags: the reference's idempotent
// store (CL:193), skipped when the flag is already set.
// ----------------------------------------------------------------------------
constexpr int kWidePPT = 4, kWideChunk = 1024;

__global__ __launch_bounds__(256) void assign_wide_kernel(WideArgs a) {
    __shared__ float4 s_pal[kWideChunk];
    const int p = blockIdx.y, tid = threadIdx.x;
    const float4* pal = a.pal + (int64_t)p * a.K;
    const int64_t q0 = (int64_t)blockIdx.x * 256 * kWidePPT + tid;
    float r[kWidePPT], g[kWidePPT], b[kWidePPT], best[kWidePPT], second[kWidePPT];
    uint32_t bi[kWidePPT];
#pragma unroll
    for (int u = 0; u < kWidePPT; ++u) {
        const int64_t q = min(q0 + 256 * u, a.n_ext - 1);
        r[u] = a.R[q];
        g[u] = a.G[q];
        b[u] = a.B[q];
        best[u] = second[u] = INFINITY;
        bi[u] = 0;
    }
    for (int k0 = 0; k0 < a.K; k0 += kWideChunk) {
        const int n = min(kWideChunk, a.K - k0);
        __syncthreads();
        for (int i = tid; i < n; i += 256) s_pal[i] = pal[k0 + i];
        __syncthreads();
        for (int i = 0; i < n; ++i) {
            const float4 c = s_pal[i];
#pragma unroll
            for (int u = 0; u < kWidePPT; ++u) {
                const float d2 = dist2_rank(r[u], g[u], b[u], c);
                const bool lt = d2 < best[u];
                bi[u] = lt ? (uint32_t)(k0 + i) : bi[u];
                second[u] = __builtin_amdgcn_fmed3f(best[u], second[u], d2);
                best[u] = lt ? d2 : best[u];
            }
        }
    }
    const bool exh = a.pflags[p] != 0;
    uint32_t* idx = a.idx32 + (int64_t)p * a.idx_pitch;
    uint32_t* used = a.used32 + (int64_t)p * a.K;
#pragma unroll
    for (int u = 0; u < kWidePPT; ++u) {
        const int64_t q = q0 + 256 * u;
        if (q >= a.n_ext) continue;
        const bool finite = isfinite(r[u]) && isfinite(g[u]) && isfinite(b[u]);
        uint32_t k = bi[u];
        if (exh || !finite || !(second[u] > __builtin_fmaf(best[u], 1.0f + 1e-6f, 0x1p-125f))) k = argmin_wide_slow(r[u], g[u], b[u], pal, a.K);
        idx[q] = k;
        if (used[k] == 0u) used[k] = 1u;
    }
}

hipError_t launch_prep_wide(const WideArgs& a, int P, hipStream_t s) {
    HQ_LAUNCH(prep_wide_kernel, dim3((unsigned)((a.K + 255) / 256), (unsigned)P), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_assign_wide(const WideArgs& a, int P, hipStream_t s) {
    const unsigned gx = (unsigned)((a.n_ext + 256 * kWidePPT - 1) / (256 * kWidePPT));
    HQ_LAUNCH(assign_wide_kernel, dim3(gx, (unsigned)P), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace hq
