// hq_assign.hip -- per-pixel palette index (CL:179-193 argmin, bit-exact)
// and used-colour bitmask (CL:193) for a population of palettes, through the
// exact candidate lists of build_grid (hq_search.hip).
#include "hq_device.h"
#include "hq_launch.h"

namespace hq {

// Reference loop verbatim (CL:179-192) over a candidate list or all K colours.
__device__ __noinline__ int argmin_exact_slow(float r, float g, float b, uint4 L0, uint4 L1,
                                              int cnt, bool all, const float4* s_pal, int K) {
    const uint32_t words[8] = {L0.x, L0.y, L0.z, L0.w, L1.x, L1.y, L1.z, L1.w};
    const int n = all ? K : cnt;
    int bi = all ? 0 : (int)((words[0] >> 8) & 0xff);
    float best = sqrtf(dist2(r, g, b, s_pal[bi]));
    for (int i = 1; i < n; ++i) {
        const int k = all ? i : (int)((words[(i + 1) >> 2] >> (8 * ((i + 1) & 3))) & 0xff);
        const float d = sqrtf(dist2(r, g, b, s_pal[k]));
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
__device__ __forceinline__ int argmin_from_entry(float r, float g, float b, uint4 L0, bool listed,
                                                 const float4* s_pal, const uint8_t* lvl1p, int G2,
                                                 int K) {
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
        // Ranked by dist2_rank.  best2 <= second2 always, so the runner-up after a
        // new value is the median of the three (v_med3_f32): 4 VALU per candidate
        // to track best, runner-up and index (the compare-and-select form took 7).
        // Slots past a lane's list (build_grid writes index 0 there) rank as +inf.
        const f32x2 rg = {r, g};
        float best2 = dist2_rank(r, g, b, s_pal[bi]);
        float second2 = INFINITY;
        // The next candidate's colour is read while this one is evaluated (the
        // loop is unrolled, so the hand-over is register renaming, not a copy).
        // Candidates are tracked by LDS byte offset (index x 16): one SDWA shift
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
            const bool lt = d2 < best2;  // a select, not fminf (which canonicalises its inputs)
            ba = lt ? ak : ba;
            second2 = __builtin_amdgcn_fmed3f(best2, second2, d2);
            best2 = lt ? d2 : best2;
        }
        bi = (int)(ba >> 4);
        near = second2 <= best2 * (1.0f + 1e-6f);
    }
    if (__any(exh || near)) {
        if (exh || near) bi = argmin_exact_slow(r, g, b, L0, L1, cnt, exh, s_pal, K);
    }
    return bi;
}

// ----------------------------------------------------------------------------
// assign: grid (nblocks * ceil(P/4)), block 256, XCD-relabelled.
// ----------------------------------------------------------------------------
// One pixel pass serves a group of up to 4 palettes: the pixel's RGB is read
// once, its cell index computed once, and the group's 4 level-2 entries -- one
// 64-byte line of the interleaved table -- arrive in one line fetch (random 16-B
// lookups per palette are bound by the line fetches they cause).  The passes
// run as a three-stage software pipeline over a thread's pixels: the level-2
// lookup depends on the pixel's RGB, so a batch that loads RGB, then looks up,
// then resolves pays two dependent memory round trips per batch (a lookup made
// independent of the RGB ran 40% faster).  Here, while pixel i is resolved,
// pixel i+1's line lookup and pixel i+2's RGB are in flight.
__device__ __forceinline__ int64_t quad_cell(float r, float g, float b, int G2) {
    return (int64_t)(min((int)(r * (float)G2), G2 - 1) * G2 + min((int)(g * (float)G2), G2 - 1)) * G2 +
           min((int)(b * (float)G2), G2 - 1);
}

// NG = min(P, 4): the palettes a pixel pass can serve.  A population below 4
// loads only its NG 16-B entries of each 64-B level-2 line (P = 1 issued four
// dwordx4 lookups per pixel for one useful one) and keeps NG palette tables.
template <int NG>
#ifndef HQ_ASSIGN_WAVES
#define HQ_ASSIGN_WAVES 1
#endif
__global__ __launch_bounds__(256, HQ_ASSIGN_WAVES) void assign_pipe_kernel(AssignArgs a, int P) {
    constexpr int PPT = kAssignPPT;  // pixels per thread per chunk (the pipeline runs across chunks)
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
    // pixel sequence of this thread: chunk c (stride nblocks), slot j < PPT.
    // Positions and byte offsets are 32-bit (the host keeps a shard's extended
    // rows below 2^30 pixels), so loads and stores take the scalar-base form.
    const uint32_t chunk = 256 * PPT, cstride = (uint32_t)a.nblocks * chunk;
    const uint32_t qbase = (uint32_t)blk * chunk + (uint32_t)(tid >> 6) * 64 * PPT + (tid & 63);
    auto qpos = [&](int i) {  // i-th pixel of this thread
        return qbase + (uint32_t)(i / PPT) * cstride + 64u * (uint32_t)(i % PPT);
    };
    // Loads are unconditional (clamped addresses, results selected afterwards):
    // predicated loads sit behind branches, and the compiler's wait counting
    // then keeps at most one load in flight.
    const uint32_t n_ext = (uint32_t)a.n_ext, qlast = n_ext - 1;
    auto at = [](const float* base, uint32_t q) {
        return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + (q << 2));
    };
    auto load_rgb = [&](uint32_t q, float& r, float& g, float& b) {
        const uint32_t qc = min(q, qlast);
        r = at(a.R, qc);
        g = at(a.G, qc);
        b = at(a.B, qc);
    };
    auto lookup = [&](uint32_t q, float r, float g, float b, bool& inside, uint4 (&e)[NG]) {
        inside = q < n_ext && r >= 0.f && r <= 1.f && g >= 0.f && g <= 1.f && b >= 0.f && b <= 1.f;
        const uint4* line =
            reinterpret_cast<const uint4*>(lines + (inside ? (uint32_t)quad_cell(r, g, b, G2) : 0u) * 64u);
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
    uint32_t qq[2];
    load_rgb(qpos(0), xr[0], xg[0], xb[0]);
    qq[0] = qpos(0);
    lookup(qq[0], xr[0], xg[0], xb[0], in_[0], E[0]);
    load_rgb(qpos(1), rb[1], gb[1], bb[1]);
    load_rgb(qpos(2), rb[0], gb[0], bb[0]);
    // The palette table is filled while the first pixels' loads are in flight
    // (the fill used to come first: one more memory round trip per workgroup).
    static_assert(kMaxK == 256, "one table entry per thread and palette");
    for (int pp = 0; pp < ng; ++pp)
        if (tid < a.K) s_pal[pp * kMaxK + tid] = a.pal[(int64_t)(p0 + pp) * kMaxK + tid];
    if (tid < 8 * NG) s_used[tid >> 3][tid & 7] = 0;
    __syncthreads();
    uint8_t* idx_base[NG];  // each palette's index image
#pragma unroll
    for (int pp = 0; pp < NG; ++pp) idx_base[pp] = a.idx + (int64_t)(p0 + min(pp, ng - 1)) * a.idx_pitch;
    bool exh_pal[NG];
#pragma unroll
    for (int pp = 0; pp < NG; ++pp) exh_pal[pp] = pp >= ng || a.pflags[p0 + min(pp, ng - 1)] != 0 || a.G2 == 0;
    auto resolve = [&](int h) {
        const uint32_t q = qq[h];
#pragma unroll
        for (int pp = 0; pp < NG; ++pp) {
            if (pp >= ng) break;
            const int pq = p0 + pp;
            const int k = argmin_from_entry(xr[h], xg[h], xb[h], E[h][pp], in_[h] && !exh_pal[pp],
                                            s_pal + pp * kMaxK, a.lvl1 + (int64_t)pq * a.lvl1_pitch,
                                            G2, a.K);
            // non-temporal: streamed out during the kernel rather than left dirty
            // in L2 for the kernel boundary to write back (67 MB per population;
            // ~0.5-1% per evaluation)
            __builtin_nontemporal_store((uint8_t)k, idx_base[pp] + q);
            const uint32_t bit = 1u << (k & 31);
            if (!(s_used[pp][k >> 5] & bit)) atomicOr(&s_used[pp][k >> 5], bit);
        }
    };
    auto step = [&](int i, int h) {  // h == i & 1, a compile-time constant at each call
        const int n = h ^ 1;
        qq[n] = qpos(i + 1);
        xr[n] = rb[n]; xg[n] = gb[n]; xb[n] = bb[n];  // RGB(i+1): landed, needed now anyway
        lookup(qq[n], xr[n], xg[n], xb[n], in_[n], E[n]);
        load_rgb(qpos(i + 3), rb[n], gb[n], bb[n]);
        resolve(h);
    };
    for (int i = 0;; i += 2) {
        if (qpos(i) >= n_ext) break;
        step(i, 0);
        if (qpos(i + 1) >= n_ext) break;
        step(i + 1, 1);
    }
    __syncthreads();
    // the workgroup's used bits into the palette's 8 words (OR is order-free:
    // the result does not depend on which workgroup gets there first).  A
    // device-scope load first, so only bits nobody has set yet cost an atomic:
    // after the first workgroups every colour of a 256-colour palette is
    // usually in, and 2,000-4,000 workgroups' atomics on the same 32 words
    // serialised at the end of a short (row-block shard) launch.
    if (tid < 8 * ng) {
        const uint32_t m = s_used[tid >> 3][tid & 7];
        uint32_t* gw = &a.used_glob[(p0 + (tid >> 3)) * 8 + (tid & 7)];
        const uint32_t seen = __hip_atomic_load(gw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (m & ~seen) atomicOr(gw, m);
    }
}

// ----------------------------------------------------------------------------
// Launcher
// ----------------------------------------------------------------------------
hipError_t launch_assign(const AssignArgs& a, int P, hipStream_t s) {
    const unsigned grid = (unsigned)(a.nblocks * ((P + 3) / 4));
    switch (P) {
    case 1: HQ_LAUNCH(assign_pipe_kernel<1>, dim3(grid), dim3(256), 0, s, a, P); break;
    case 2: HQ_LAUNCH(assign_pipe_kernel<2>, dim3(grid), dim3(256), 0, s, a, P); break;
    case 3: HQ_LAUNCH(assign_pipe_kernel<3>, dim3(grid), dim3(256), 0, s, a, P); break;
    default: HQ_LAUNCH(assign_pipe_kernel<4>, dim3(grid), dim3(256), 0, s, a, P); break;
    }
    return hipGetLastError();
}

}  // namespace hq
