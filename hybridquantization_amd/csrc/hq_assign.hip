// hq_assign.hip -- per-pixel palette index (CL:179-193 argmin, bit-exact)
// and used-colour bitmask (CL:193) for a population of palettes, through the
// exact candidate lists of build_grid (hq_search.hip).
#include <type_traits>

#include "hq_device.h"
#include "hq_launch.h"

#ifndef HQ_ASSIGN_PF
#define HQ_ASSIGN_PF 1
#endif
#ifndef HQ_ASSIGN_PRED
#define HQ_ASSIGN_PRED 2
#endif
#ifndef HQ_ASSIGN_DEPTH
#define HQ_ASSIGN_DEPTH 1  // pixels the level-2 lookups run ahead of the resolve (1 or 2)
#endif
// wave-uniform "any lane": the compare's lane mask itself (HIP's __any
// materialised the predicate in a VGPR and compared it again)
#define HQ_ANY(c) (__builtin_amdgcn_ballot_w64(c) != 0)
#ifndef HQ_ASSIGN_JOINT
#define HQ_ASSIGN_JOINT 0  // 1: argmin_group over the whole group in lockstep (measured slower:
                           // 0.218 vs 0.199 ms at C3 P=4, fewer waves and longer walks)
#endif

namespace hq {

// A level-2 entry in registers: count + kL2Cap indices (hq_internal.h).
using L2E = std::conditional_t<kL2Bytes == 16, uint4, uint2>;
__device__ __forceinline__ uint32_t l2_word(const uint2& e, int k) { return k == 0 ? e.x : e.y; }
__device__ __forceinline__ uint32_t l2_word(const uint4& e, int k) {
    return k == 0 ? e.x : k == 1 ? e.y : k == 2 ? e.z : e.w;
}
__device__ __forceinline__ uint4 l2_u4(const uint2& e) { return make_uint4(e.x, e.y, 0u, 0u); }
__device__ __forceinline__ uint4 l2_u4(const uint4& e) { return e; }
__device__ __forceinline__ void l2_set(uint2& e, uint32_t x, uint32_t y) { e = make_uint2(x, y); }
__device__ __forceinline__ void l2_set(uint4& e, uint32_t x, uint32_t y) { e = make_uint4(x, y, 0u, 0u); }

#ifdef HQ_ASSIGN_TIMING
__device__ unsigned int g_asg_slow[2];
constexpr int kAsgStamps = 16384;
// per workgroup: start, fill barrier, end, then each wave's loop end
__device__ unsigned long long g_asg_t[kAsgStamps][8];
#endif

// Reference loop verbatim (CL:179-192) over a candidate list or all K colours.
__device__ __noinline__ int argmin_exact_slow(float r, float g, float b, uint4 L0, uint4 L1,
                                              int cnt, bool all, const float4* s_pal, int K) {
    const uint32_t words[8] = {L0.x, L0.y, L0.z, L0.w, L1.x, L1.y, L1.z, L1.w};
    const int n = all ? K : cnt;
    int bi = all ? 0 : (int)((words[0] >> 8) & 0xff);
    float best = ref_dist(r, g, b, s_pal[bi]);
    for (int i = 1; i < n; ++i) {
        const int k = all ? i : (int)((words[(i + 1) >> 2] >> (8 * ((i + 1) & 3))) & 0xff);
        const float d = ref_dist(r, g, b, s_pal[k]);
        if (d < best) { best = d; bi = k; }
    }
    return bi;
}

// Re-resolution of one palette's pixel by the reference loop: the level-1 list
// when the level-2 list overflowed (or all K colours when that overflowed too),
// else the level-2 list itself (a near tie) or all K (no list: pixel outside
// the unit cube, or a palette outside it).
__device__ __noinline__ int argmin_resolve_slow(float r, float g, float b, uint4 L0, bool listed,
                                                const float4* s_pal, const uint8_t* lvl1p, int G2,
                                                int K) {
    uint4 L1 = make_uint4(0, 0, 0, 0);
    int cnt = listed ? (int)(L0.x & 0xff) : 0;
    bool all = !listed;
    if (cnt == kOverflow) {
        const int G1 = G2 >> 2;
        const int ir = min((int)(r * (float)G2), G2 - 1) >> 2;
        const int ig = min((int)(g * (float)G2), G2 - 1) >> 2;
        const int ib = min((int)(b * (float)G2), G2 - 1) >> 2;
        const uint4* e = reinterpret_cast<const uint4*>(
            lvl1p + ((int64_t)(ir * G1 + ig) * G1 + ib) * 32);
        L0 = e[0];
        L1 = e[1];
        cnt = L0.x & 0xff;
        if (cnt == kOverflow) all = true;
    }
    return argmin_exact_slow(r, g, b, L0, L1, cnt, all, s_pal, K);
}

// The reference loop (CL:179-192) for the few lanes of a wave that need it
// (mask sm), the whole wave working on one lane's pixel at a time: lane l
// takes colours l, l + 64, ... in ascending order (strict <, so the first
// minimum within the lane), then a butterfly picks the least (distance,
// index) -- the reference's first minimum.  A NaN distance never wins unless
// colour 0's is NaN, which the reference keeps (nothing compares below NaN).
// One rare near tie or list overflow used to cost its wave a 256-colour loop
// on one lane (3-4 times the wave's other work): the launch waited for those
// waves (assign_timing.py: the slowest waves 67 us against 20 at the median
// on a 512-row shard).  Call with every lane active.
constexpr int kCoopMax = 16;
__device__ __forceinline__ int argmin_fix(float r, float g, float b, bool s, int cur, L2E L0, bool listed,
                                       const float4* s_pal, const uint8_t* lvl1p, int G2, int K) {
    uint64_t sm = __ballot(s);
    if (__popcll(sm) > kCoopMax)  // many (a palette with a non-finite colour): each lane its own loop
        return s ? argmin_resolve_slow(r, g, b, l2_u4(L0), listed, s_pal, lvl1p, G2, K) : cur;
    const int lane = (int)__lane_id();
    int result = cur;
    while (sm) {
        const int L = __builtin_ctzll(sm);
        sm &= sm - 1;
        const float pr = __shfl(r, L, 64), pg = __shfl(g, L, 64), pb = __shfl(b, L, 64);
        // (distance, key): a NaN distance counts as +inf with key bit 16 set, so a
        // number (+inf included) beats it; equal distances: the lower index
        float bd = INFINITY;
        uint32_t bkey = 0xffffffffu;  // no colour yet
        for (int k = lane; k < K; k += 64) {
            const float d = ref_dist(pr, pg, pb, s_pal[k]);
            const bool nan = d != d;
            const float dv = nan ? INFINITY : d;
            const uint32_t key = (nan ? 0x10000u : 0u) | (uint32_t)k;
            if (dv < bd || (dv == bd && key < bkey)) {
                bd = dv;
                bkey = key;
            }
        }
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) {
            const float od = __shfl_xor(bd, m, 64);
            const uint32_t ok = (uint32_t)__shfl_xor((int)bkey, m, 64);
            if (od < bd || (od == bd && ok < bkey)) {
                bd = od;
                bkey = ok;
            }
        }
        const int bk = (int)(bkey & 0xffffu);
        const float d0 = ref_dist(pr, pg, pb, s_pal[0]);
        if (lane == L) result = d0 != d0 ? 0 : bk;
    }
    return result;
}

// Exact argmin (CL:179-193 semantics) of one pixel against the NG palettes of
// its group over their level-2 candidate lists.  Candidates are ranked by d2
// (the reference's); the reference ranks by ref_dist (v_sqrt_f32 of d2), which
// can map two different d2 onto one distance, and then keeps the lower index.
// Equal distances imply |d2a - d2b| < 2^-21 * d2 (v_sqrt_f32 is monotone and
// within 1 ulp), so lanes whose runner-up d2 lies within 1e-6 relative of the
// best (or below 2^-125: near_d2) are re-resolved with the reference loop
// (rare), as are
// lanes whose list overflowed the level-2 entry or that have no list.
// NG > 1 walks the lists in lockstep (HQ_ASSIGN_JOINT): candidate i of every
// palette in one loop step, NG independent LDS reads and compare chains in
// flight; the step count is then the longest list over the wave's lanes and
// the group's palettes.
template <int NG>
__device__ __forceinline__ void argmin_group(float r, float g, float b, const L2E (&E)[NG], bool inside,
                                             const bool (&exh_pal)[NG], const float4* s_pal,
                                             const uint8_t* lvl1, int64_t lvl1_pitch, int p0, int G2,
                                             int K, int (&out)[NG]) {
    int cnt[NG];
    bool slow[NG];
    uint32_t ba[NG];
    int maxc = 0;
#pragma unroll
    for (int q = 0; q < NG; ++q) {
        const bool listed = inside && !exh_pal[q];
        const int c = listed ? (int)(E[q].x & 0xff) : 0;
        slow[q] = !listed || c == kOverflow;
        cnt[q] = slow[q] ? 0 : c;
        maxc = max(maxc, cnt[q]);
        ba[q] = byte_x16(E[q].x, 1);
    }
    bool near[NG];
#pragma unroll
    for (int q = 0; q < NG; ++q) near[q] = false;
#ifdef HQ_ABL_NOLOOP  // timing ablation (wrong results): no candidate walk
    maxc = 1;
#endif
    if (HQ_ANY(maxc > 1)) {
        const f32x2 rg = {r, g};
        const char* base = reinterpret_cast<const char*>(s_pal);
        auto at = [&](int q, uint32_t off) {
            return *reinterpret_cast<const float4*>(base + q * (kMaxK * 16) + off);
        };
        auto cand16 = [&](int q, int i) {  // byte i + 1 of the entry, x16
            const uint32_t w = l2_word(E[q], (i + 1) >> 2);
            return byte_x16(w, (i + 1) & 3);
        };
        float best2[NG], second2[NG];
        // candidate colours are read HQ_ASSIGN_PF steps ahead of their use
        constexpr int PF = HQ_ASSIGN_PF;
        uint32_t an[NG][PF];
        float4 cn[NG][PF];
#pragma unroll
        for (int q = 0; q < NG; ++q) {
            best2[q] = dist2_rank(r, g, b, at(q, ba[q]));
            second2[q] = INFINITY;
#pragma unroll
            for (int d = 0; d < PF; ++d) {
                an[q][d] = cand16(q, 1 + d);
                cn[q][d] = at(q, an[q][d]);
            }
        }
#pragma unroll
        for (int i = 1; i < kL2Cap; ++i) {
            if (!HQ_ANY(i < maxc)) break;
#pragma unroll
            for (int q = 0; q < NG; ++q) {
                const uint32_t ak = an[q][0];
                const float4 c = cn[q][0];
#pragma unroll
                for (int d = 0; d + 1 < PF; ++d) {
                    an[q][d] = an[q][d + 1];
                    cn[q][d] = cn[q][d + 1];
                }
                if (i + PF < kL2Cap) {
                    an[q][PF - 1] = cand16(q, i + PF);
#if HQ_ASSIGN_PRED == 1
                    // only lanes whose list reaches that far read LDS (exec-masked):
                    // the wave walks to its longest list, 6 steps for a mean of 2
                    if (i + PF < cnt[q]) cn[q][PF - 1] = at(q, an[q][PF - 1]);
#elif HQ_ASSIGN_PRED == 2
                    // lanes past their list all read entry 0 (one broadcast address,
                    // no bank conflicts): the wave walks to its longest list
                    cn[q][PF - 1] = at(q, i + PF < cnt[q] ? an[q][PF - 1] : 0u);
#else
                    cn[q][PF - 1] = at(q, an[q][PF - 1]);
#endif
                }
                asm volatile("" ::"v"(c.w));  // one ds_read_b128, not b96
                const float d2 = i < cnt[q] ? dist2_rank_pk(rg, b, c) : INFINITY;
                const bool lt = d2 < best2[q];
                ba[q] = lt ? ak : ba[q];
                second2[q] = __builtin_amdgcn_fmed3f(best2[q], second2[q], d2);
                best2[q] = lt ? d2 : best2[q];
            }
        }
#pragma unroll
        for (int q = 0; q < NG; ++q) near[q] = near_d2(best2[q], second2[q]);
    }
#pragma unroll
    for (int q = 0; q < NG; ++q) {
        out[q] = (int)(ba[q] >> 4);
#ifdef HQ_ABL_NOSLOW  // timing ablation (wrong results): no re-resolution
        const bool s = false;
#else
        const bool s = slow[q] || near[q];
#endif
#ifdef HQ_ASSIGN_TIMING  // diagnostic: lanes re-resolved (near ties, overflows / no list)
        if (near[q]) atomicAdd(&g_asg_slow[0], 1u);
        if (slow[q]) atomicAdd(&g_asg_slow[1], 1u);
#endif
        if (HQ_ANY(s))
            out[q] = argmin_fix(r, g, b, s, out[q], E[q], inside && !exh_pal[q], s_pal + q * kMaxK,
                                lvl1 + (int64_t)(p0 + q) * lvl1_pitch, G2, K);
    }
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

// NG: the palettes of the group a pixel pass serves (4, or P mod 4 for the
// last group, launched on its own): every palette slot is live, so the
// resolve step has no data-dependent exits.  A group below 4 loads only its NG
// 16-B entries of each 64-B level-2 line and keeps NG palette tables.
// (u8_unit, hq_device.h: k/255 bit-exactly from the byte k)

// A pixel's colour while its load is in flight: three planar floats, or the
// packed bytes of an 8-bit image (one dword, one register).
template <bool U8> struct RawPx { float r, g, b; };
template <> struct RawPx<true> { uint32_t v; };
__device__ __forceinline__ uint32_t raw_of(const RawPx<false>&) { return 0u; }
__device__ __forceinline__ uint32_t raw_of(const RawPx<true>& x) { return x.v; }

// Level-2 cell of a packed 8-bit pixel (G2 = 2^lg, lg <= 6): quad_cell's
// min((int)(RN(k/255) G2), G2 - 1) per channel is k >> (8 - lg) for every
// byte k.  Proof: the rounding of k/255 moves k G2/255 by at most 2^-19 while
// a non-integer k G2/255 lies at least 1/255 from an integer (255 is odd,
// G2 a power of two: only k = 0, 255 give integers, and 255 G2/255 = G2 is
// clamped to G2 - 1); floor(k G2/255) = floor(k G2/256) unless some integer j
// has 255 j <= k G2 < 256 j, which needs (-255 j) mod G2 = j < j for j < G2.
__device__ __forceinline__ uint32_t cell_u8(uint32_t v, int lg) {
    const int sh = 8 - lg;
    const uint32_t m = (1u << lg) - 1u;
    return ((((v >> sh) & m) << lg | ((v >> (8 + sh)) & m)) << lg) | ((v >> (16 + sh)) & m);
}


// Chunked palettes (256 < K <= 4096; AssignArgs::nch > 1): a palette of K colours
// is nch sub-palettes of 256 (colours 256 c .. 256 c + 255, the last ones padded
// with copies of colour 0), each with its own grid, and the argmin over K is
// the argmin over the chunks' own argmins: each chunk's winner is its first
// minimum (CL:179-193), and the reference distance of each winner, compared
// in ascending chunk order with a strict <, picks the first chunk that
// attains the global minimum -- the reference's first minimum over all K
// (a padding colour ties colour 0, which chunk 0 holds, and never wins).
// CMB consecutive sub-palettes of a group combine into one 16-bit index per
// pixel.  nch > 4 runs nch / 4 passes over the groups (PASS 1 first, 2 middle,
// 3 last), each comparing its group's winner with the best so far in the
// distance scratch; PASS 0 is a single pass (nch <= 4) and the only one that
// records used bits (nch > 4: used_idx16_kernel from the final indices).
template <int NG, bool U8, int CMB = 1, int PASS = 0>
#ifndef HQ_ASSIGN_WAVES
#define HQ_ASSIGN_WAVES 1
#endif
__global__ __launch_bounds__(256, HQ_ASSIGN_WAVES) void assign_pipe_kernel(AssignArgs a, int grp0, int ngroups) {
    static_assert(NG % CMB == 0 && (CMB == 4 || PASS == 0), "combine sets inside the group; passes: 4 chunks");
    // [NG][kMaxK]: a fixed palette stride, so each palette's base folds into the
    // ds_read_b128 offset field and a candidate's address is its byte << 4
    __shared__ __attribute__((aligned(16))) float4 s_pal[NG * kMaxK];
    // used colours: one byte per colour, set by plain byte stores (a read-test-or
    // of 32-bit words cost an LDS round trip and 5 VALU per pixel and palette;
    // assign 0.1597 -> 0.1578 ms at C3); words by ballot at the flush
    __shared__ __attribute__((aligned(16))) uint8_t s_usedb[NG][kMaxK];
    const int w = xcd_remap(blockIdx.x, a.nblocks * ngroups);
    // group-major: after the relabelling an XCD's contiguous range of
    // workgroups covers one or two groups, so its L2 holds those groups' level-2
    // tables (2 MiB each at G2 = 32) rather than every group's (P = 64: 32 MiB
    // against a 4 MiB L2; the lookups then came from the Infinity Cache)
    const int grp = grp0 + (w / a.nblocks) * a.gstep, blk = w % a.nblocks, tid = threadIdx.x;
#ifdef HQ_ASSIGN_TIMING  // diagnostic build: per-workgroup stamps (wall_clock64, 100 MHz)
    const uint64_t t_start = wall_clock64();
    uint64_t t_fill = 0, t_loop = 0;
#endif
    const int p0 = 4 * grp;
    const uint8_t* lines = a.lvl2 + (int64_t)grp * a.lvl2_gstride;
    const int G2 = a.G2 > 0 ? a.G2 : 4;
    const int lg_g2 = 31 - __builtin_clz(G2);  // (a power of two, hq_set_option "grid")
    // pixel sequence of this thread: a grid stride.  Positions and byte offsets
    // are 32-bit (the host keeps a shard's extended rows below 2^30 pixels), so
    // loads and stores take the scalar-base form.
    const uint32_t n_ext = (uint32_t)a.n_ext, qlast = n_ext - 1;
    const uint32_t cstride = (uint32_t)a.nblocks * 256u;
    const uint32_t qbase = (uint32_t)blk * 256u + (uint32_t)tid;
    // Every lane of a wave runs its lane 0's step count (the largest: qbase
    // grows with the lane): argmin_fix's cooperative loop and butterfly need
    // the whole wave active.  Steps past the image resolve the clamped last
    // pixel again and store nothing.
    const int npx0 = qbase < n_ext ? (int)((n_ext - 1 - qbase) / cstride) + 1 : 0;
    const int npx = __builtin_amdgcn_readfirstlane(npx0);
    auto qpos = [&](int i) { return qbase + (uint32_t)i * cstride; };
    // Loads are unconditional (clamped addresses, results selected afterwards):
    // predicated loads sit behind branches, and the compiler's wait counting
    // then keeps at most one load in flight.
    auto at = [](const float* base, uint32_t q) {
        return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + (q << 2));
    };
    // PASS >= 2: the best reference distance of the earlier passes, per pixel of
    // the group's palette (loaded with the pixel's RGB)
    const float* dist_in = PASS >= 2 ? a.dist + (int64_t)((4 * grp) >> a.lg_nch) * a.idx_pitch : nullptr;
    float pdl[3], pdv[3];  // [NB]: loads in flight, values of pixels being resolved
    auto load_rgb = [&](uint32_t q, RawPx<U8>& x, float& pd) {
        const uint32_t qc = min(q, qlast);
        if constexpr (PASS >= 2) pd = at(dist_in, qc);
        if constexpr (U8) {
            x.v = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(a.rgbx) + (qc << 2));
        } else {
            x.r = at(a.R, qc);
            x.g = at(a.G, qc);
            x.b = at(a.B, qc);
        }
    };
    auto unpack = [&](const RawPx<U8>& x, float& r, float& g, float& b) {
        if constexpr (U8) {
            r = u8_unit(x.v, 0);
            g = u8_unit(x.v, 1);
            b = u8_unit(x.v, 2);
        } else {
            r = x.r;
            g = x.g;
            b = x.b;
        }
    };
    auto lookup = [&](uint32_t q, float r, float g, float b, bool& inside, L2E (&e)[NG], uint32_t raw) {
        // (q past the image: the clamped last pixel, resolved but not stored)
        inside = U8 ? true : r >= 0.f && r <= 1.f && g >= 0.f && g <= 1.f && b >= 0.f && b <= 1.f;
#ifdef HQ_ABL_HASHLOOKUP  // timing ablation (wrong results): a random line, independent of the RGB
        const uint8_t* lb = lines + ((q * 2654435761u) >> 17) * (uint32_t)kL2Line;
#elif defined(HQ_ABL_COHERENT)  // timing ablation (wrong results): runs of 256 consecutive pixels share a cell
        const uint8_t* lb = lines + (((q >> 8) * 40503u) & (uint32_t)(G2 * G2 * G2 - 1)) * (uint32_t)kL2Line;
#else
        // (packed pixels: the cell straight from the bytes, cell_u8)
        const uint8_t* lb = lines + (U8 ? cell_u8(raw, lg_g2) : inside ? (uint32_t)quad_cell(r, g, b, G2) : 0u) *
                                        (uint32_t)kL2Line;
#endif
        // selected by the `listed` flag at use.  8-B entries: two palettes per
        // 16-B load (the L1 access count per pixel, not the bytes, is the cost)
        const uint4* line = reinterpret_cast<const uint4*>(lb);
        if constexpr (kL2Bytes == 16) {
#pragma unroll
            for (int pp = 0; pp < NG; ++pp) e[pp] = line[pp];
        } else {
#pragma unroll
            for (int pp = 0; pp + 1 < NG; pp += 2) {
                const uint4 v = line[pp >> 1];
                l2_set(e[pp], v.x, v.y);
                l2_set(e[pp + 1], v.z, v.w);
            }
            if constexpr (NG & 1) e[NG - 1] = reinterpret_cast<const L2E*>(lb)[NG - 1];
        }
#ifdef HQ_ABL_NOLOOKUP  // timing ablation (wrong results): one fixed entry, lists of 3-4
#pragma unroll
        for (int pp = 0; pp < NG; ++pp) {
            const uint4 f = make_uint4(0x03020103u + (q & 1u), 0x07060504u, 0x0b0a0908u, 0x0f0e0d0cu);
            l2_set(e[pp], f.x, f.y);  // counts 3-4: words 0-1
        }
#endif
    };
    // Pipeline, unrolled by two so every buffer has a fixed register set (a
    // register copy of an in-flight load waits for it: rotating buffers at the
    // loop end serialised the whole pipeline behind an s_waitcnt vmcnt(0)).
    // Step i (parity h = i & 1): RGB(i+1) has landed -> its cell lookup goes out
    // into E[h^1] and its RGB moves to X[h^1]; RGB(i+3) goes out into the freed
    // buffer; pixel i is resolved from E[h], X[h] while those loads fly.  The
    // step body loads nothing conditionally (the rare list overflows and near
    // ties are re-resolved in a called function): a conditional load into a
    // register that a later step overwrites made the compiler wait for every
    // load in flight before that write.
#if HQ_ASSIGN_DEPTH == 2
    // Lookups two pixels ahead (HQ_ASSIGN_DEPTH 2): three buffer sets by i % 3;
    // at step i, E[i%3] and E[(i+1)%3] are in flight, RGB(i+2) and RGB(i+3)
    // too (rb[(i+2)%3], rb[i%3]).
    constexpr int NB = 3;
#else
    constexpr int NB = 2;
#endif
    RawPx<U8> rb[NB];                 // RGB loads in flight
    float xr[NB], xg[NB], xb[NB];     // RGB of pixels being looked up / resolved
    L2E E[NB][NG];
    bool in_[NB];
    uint32_t qq[NB];
#pragma unroll
    for (int j = 0; j < NB - 1; ++j) {
        RawPx<U8> x0;
        load_rgb(qpos(j), x0, pdv[j]);
        unpack(x0, xr[j], xg[j], xb[j]);
        qq[j] = qpos(j);
        lookup(qq[j], xr[j], xg[j], xb[j], in_[j], E[j], raw_of(x0));
    }
#if HQ_ASSIGN_DEPTH == 2
    load_rgb(qpos(2), rb[2], pdl[2]);
    load_rgb(qpos(3), rb[0], pdl[0]);
#else
    load_rgb(qpos(1), rb[1], pdl[1]);
    load_rgb(qpos(2), rb[0], pdl[0]);
#endif
    // The palette table is filled while the first pixels' loads are in flight
    // (the fill used to come first: one more memory round trip per workgroup).
    static_assert(kMaxK == 256, "one table entry per thread and palette");
    // (unconditional: entries past K hold a copy of colour K-1 and are never
    // listed.  A fill skipped by some threads left the prologue's RGB loads in
    // flight on that path, and the loop head's wait, which serves both paths,
    // then drained every lookup in flight on each step.)
#pragma unroll
    for (int pp = 0; pp < NG; ++pp)
        s_pal[pp * kMaxK + tid] = a.pal[(int64_t)(p0 + pp) * kMaxK + min(tid, a.K - 1)];
    if (tid < 64 * NG) reinterpret_cast<uint32_t*>(&s_usedb[0][0])[tid] = 0u;
    __syncthreads();
#ifdef HQ_ASSIGN_TIMING
    t_fill = wall_clock64();
#endif
    uint8_t* idx_base[NG];  // each palette's index image
    bool exh_pal[NG];
#pragma unroll
    for (int pp = 0; pp < NG; ++pp) {
        idx_base[pp] = a.idx + (int64_t)(p0 + pp) * a.idx_pitch;
        exh_pal[pp] = a.pflags[p0 + pp] != 0 || a.G2 == 0;
    }
    auto resolve = [&](int h) {
        const uint32_t q = qq[h];
        int kk[NG];
#if HQ_ASSIGN_JOINT
        argmin_group<NG>(xr[h], xg[h], xb[h], E[h], in_[h], exh_pal, s_pal, a.lvl1, a.lvl1_pitch, p0, G2,
                         a.K, kk);
#else
#pragma unroll
        for (int pp = 0; pp < NG; ++pp) {
            const L2E e1[1] = {E[h][pp]};
            const bool x1[1] = {exh_pal[pp]};
            int k1[1];
            argmin_group<1>(xr[h], xg[h], xb[h], e1, in_[h], x1, s_pal + pp * kMaxK, a.lvl1, a.lvl1_pitch,
                            p0 + pp, G2, a.K, k1);
            kk[pp] = k1[0];
        }
#endif
        if constexpr (CMB == 1) {
#pragma unroll
            for (int pp = 0; pp < NG; ++pp) {
                const int k = kk[pp];
                // non-temporal: streamed out during the kernel rather than left dirty
                // in L2 for the kernel boundary to write back (67 MB per population;
                // ~0.5-1% per evaluation)
                if (q < n_ext) {
                    __builtin_nontemporal_store((uint8_t)k, idx_base[pp] + q);
                    s_usedb[pp][k] = 1;
                }
            }
        } else {
#pragma unroll
            for (int s0 = 0; s0 < NG; s0 += CMB) {
                // the chunks' winners in ascending chunk order, by the reference's
                // distance (ref_dist, CL:186): strict <
                float best = ref_dist(xr[h], xg[h], xb[h], s_pal[s0 * kMaxK + kk[s0]]);
                int bc = 0, k = kk[s0];
#pragma unroll
                for (int c = 1; c < CMB; ++c) {
                    const float d = ref_dist(xr[h], xg[h], xb[h], s_pal[(s0 + c) * kMaxK + kk[s0 + c]]);
                    const bool lt = d < best;
                    best = lt ? d : best;
                    bc = lt ? c : bc;
                    k = lt ? kk[s0 + c] : k;
                }
                const int sp = p0 + s0 + bc;  // the winning sub-palette
                const uint16_t gidx = (uint16_t)(((sp & (a.nch - 1)) << 8) | k);
                const int64_t pal = (int64_t)((p0 + s0) >> a.lg_nch);
                if (q < n_ext) {
                    bool win = true;
                    if constexpr (PASS >= 2) win = best < pdv[h];  // earlier chunks first: strict <
                    if (win) __builtin_nontemporal_store(gidx, a.idx16 + pal * a.idx_pitch + q);
                    if constexpr (PASS == 1 || PASS == 2)
                        if (win) a.dist[pal * a.idx_pitch + q] = best;
                    if constexpr (PASS == 0) {
                        s_usedb[s0 + bc][k] = 1;
                    }
                }
            }
        }
    };
#if HQ_ASSIGN_DEPTH == 2
    auto step = [&](int i, int h) {  // h == i % 3, a compile-time constant at each call
        const int ia = (h + 2) % 3, fi = (h + 1) % 3;  // (not `a`: the kernel's AssignArgs)
        qq[ia] = qpos(i + 2);
        unpack(rb[ia], xr[ia], xg[ia], xb[ia]);  // RGB(i+2): landed
        pdv[ia] = pdl[ia];
        lookup(qq[ia], xr[ia], xg[ia], xb[ia], in_[ia], E[ia], raw_of(rb[ia]));
        load_rgb(qpos(i + 4), rb[fi], pdl[fi]);  // rb[fi] held RGB(i+1), unpacked a step ago
        resolve(h);
    };
    int i = 0;
    for (; i + 3 <= npx; i += 3) {
        step(i, 0);
        step(i + 1, 1);
        step(i + 2, 2);
    }
    if (i < npx) step(i, 0);
    if (i + 1 < npx) step(i + 1, 1);
#else
    auto step = [&](int i, int h) {  // h == i & 1, a compile-time constant at each call
        const int n = h ^ 1;
        qq[n] = qpos(i + 1);
        unpack(rb[n], xr[n], xg[n], xb[n]);  // RGB(i+1): landed, needed now anyway
        pdv[n] = pdl[n];
        lookup(qq[n], xr[n], xg[n], xb[n], in_[n], E[n], raw_of(rb[n]));
        load_rgb(qpos(i + 3), rb[n], pdl[n]);
        resolve(h);
    };
    int i = 0;
    for (; i + 2 <= npx; i += 2) {
        step(i, 0);
        step(i + 1, 1);
    }
    if (i < npx) step(i, 0);
#endif
#ifdef HQ_ASSIGN_TIMING
    t_loop = wall_clock64();
#endif
    __syncthreads();
    // the workgroup's used bits into the palette's 8 words (OR is order-free:
    // the result does not depend on which workgroup gets there first).  A
    // device-scope load first, so only bits nobody has set yet cost an atomic:
    // after the first workgroups every colour of a 256-colour palette is
    // usually in, and 2,000-4,000 workgroups' atomics on the same 32 words
    // serialised at the end of a short (row-block shard) launch.
#ifndef HQ_ABL_NOUSED  // (timing ablation, wrong results: no used-bit flush)
    if constexpr (PASS == 0) {
        // bytes -> words: colour tid of each palette, wave wv's ballot = words
        // 2 wv, 2 wv + 1, staged in LDS so that one wave then flushes all 8 NG
        // words with one load and one atomic instruction (each wave flushing its
        // own words in NG dependent load / atomic round trips held the tail of
        // short launches: shard-of-8 assign 28 -> 59 us)
        static_assert(kMaxK == 256, "one colour per thread at the flush");
        __shared__ uint32_t s_words[NG][8];
        const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
        for (int pp = 0; pp < NG; ++pp) {
            const uint64_t bits = __ballot(s_usedb[pp][tid] != 0);
            if (lane < 2) s_words[pp][2 * wv + lane] = lane ? (uint32_t)(bits >> 32) : (uint32_t)bits;
        }
        __syncthreads();
        if (tid < 8 * NG) {
            const uint32_t m = s_words[tid >> 3][tid & 7];
            uint32_t* gw = &a.used_glob[(blockIdx.x & (kUsedSlots - 1)) * a.used_stride + (p0 + (tid >> 3)) * 8 +
                                        (tid & 7)];
            const uint32_t seen = __hip_atomic_load(gw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (m & ~seen) atomicOr(gw, m);
        }
    }
#endif
#ifdef HQ_ASSIGN_TIMING
    if ((tid & 63) == 0 && w < kAsgStamps) g_asg_t[w][4 + (tid >> 6)] = t_loop;
    if (tid == 0 && w < kAsgStamps) {
        g_asg_t[w][0] = t_start;
        g_asg_t[w][1] = t_fill;
        g_asg_t[w][2] = wall_clock64();
    }
#endif
}

// ----------------------------------------------------------------------------
// used_idx16: grid (blocks, P), block 256 (nch > 4 only: the passes leave the
// used bits to this kernel).  Used bits of palette p from its final 16-bit
// indices (CL:193): an LDS bitmap per workgroup, OR'ed into used copy
// blockIdx.x & 7 at words p * 8 nch ...
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void used_idx16_kernel(AssignArgs a) {
    __shared__ uint32_t s_bits[kMaxKChunked / 32];
    const int p = blockIdx.y, tid = threadIdx.x, wpp = 8 * a.nch;
    for (int i = tid; i < wpp; i += 256) s_bits[i] = 0u;
    __syncthreads();
    const uint16_t* idx = a.idx16 + (int64_t)p * a.idx_pitch;
    for (int64_t q = (int64_t)blockIdx.x * 256 + tid; q < a.n_ext; q += (int64_t)gridDim.x * 256) {
        const uint32_t k = idx[q], bit = 1u << (k & 31);
        if (!(s_bits[k >> 5] & bit)) atomicOr(&s_bits[k >> 5], bit);
    }
    __syncthreads();
    for (int i = tid; i < wpp; i += 256) {
        const uint32_t m = s_bits[i];
        if (m) atomicOr(&a.used_glob[(blockIdx.x & (kUsedSlots - 1)) * a.used_stride + p * wpp + i], m);
    }
}

// ----------------------------------------------------------------------------
// Launcher: the full groups of 4 palettes in one launch, a last group of
// P mod 4 in a second (the profiling events, when set, bracket both).
// Chunked palettes (a.nch > 1; P = sub-palettes): nch = 2 combines pairs, 4
// whole groups; nch = 8, 16 run nch / 4 passes (groups j, j + nch / 4, ...),
// then used_idx16.
// ----------------------------------------------------------------------------
template <bool U8>
void launch_assign_t(const AssignArgs& a0, int P, hipStream_t s) {
    const hipEvent_t ev0 = t_ev_start, ev1 = t_ev_stop;
    AssignArgs a = a0;
    a.gstep = 1;
    if (a.nch > 4) {
        const int npass = a.nch / 4, npal = P / a.nch;
        a.gstep = npass;
        for (int j = 0; j < npass; ++j) {
            t_ev_start = j == 0 ? ev0 : nullptr;
            t_ev_stop = nullptr;
            const dim3 grid((unsigned)(a.nblocks * npal));
            if (j == 0) HQ_LAUNCH((assign_pipe_kernel<4, U8, 4, 1>), grid, dim3(256), 0, s, a, j, npal);
            else if (j + 1 < npass) HQ_LAUNCH((assign_pipe_kernel<4, U8, 4, 2>), grid, dim3(256), 0, s, a, j, npal);
            else HQ_LAUNCH((assign_pipe_kernel<4, U8, 4, 3>), grid, dim3(256), 0, s, a, j, npal);
        }
        t_ev_start = nullptr;
        t_ev_stop = ev1;
        const unsigned ub = (unsigned)std::min<int64_t>(512, (a.n_ext + 4095) / 4096);
        HQ_LAUNCH(used_idx16_kernel, dim3(ub, (unsigned)npal), dim3(256), 0, s, a);
        t_ev_start = ev0;
        return;
    }
    const int full = P / 4, rest = P % 4;
#define HQ_ASG(NG, CMB, NB, G0, NGR) \
    HQ_LAUNCH((assign_pipe_kernel<NG, U8, CMB>), dim3((unsigned)(NB)), dim3(256), 0, s, a, G0, NGR)
    if (full > 0) {
        if (rest) t_ev_stop = nullptr;
        if (a.nch == 4) HQ_ASG(4, 4, a.nblocks * full, 0, full);
        else if (a.nch == 2) HQ_ASG(4, 2, a.nblocks * full, 0, full);
        else HQ_ASG(4, 1, a.nblocks * full, 0, full);
        t_ev_stop = ev1;
        if (rest) t_ev_start = nullptr;
    }
    switch (rest) {  // (nch = 2: rest is 0 or 2; nch = 4: 0)
    case 1: HQ_ASG(1, 1, a.nblocks, full, 1); break;
    case 2:
        if (a.nch == 2) HQ_ASG(2, 2, a.nblocks, full, 1);
        else HQ_ASG(2, 1, a.nblocks, full, 1);
        break;
    case 3: HQ_ASG(3, 1, a.nblocks, full, 1); break;
    default: break;
    }
#undef HQ_ASG
    t_ev_start = ev0;
}

void launch_used_idx16(const AssignArgs& a, int P, hipStream_t s) {
    const unsigned ub = (unsigned)std::min<int64_t>(512, (a.n_ext + 4095) / 4096);
    HQ_LAUNCH(used_idx16_kernel, dim3(ub, (unsigned)P), dim3(256), 0, s, a);
}

hipError_t launch_assign(const AssignArgs& a, int P, hipStream_t s) {
    if (a.rgbx) launch_assign_t<true>(a, P, s);
    else launch_assign_t<false>(a, P, s);
    return hipGetLastError();
}

// Resident workgroups per CU of assign_pipe_kernel<NG> (the auto size of one
// grid-stride round; the packed and planar forms and, for NG = 4, the chunk
// combining forms take the larger register count); 0 if the query fails.
int assign_residency(int NG) {
    auto q = [](auto kern) {
        int n = 0;
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, 256, 0) == hipSuccess ? n : 0;
    };
    switch (NG) {
    case 1: return std::min(q(assign_pipe_kernel<1, false>), q(assign_pipe_kernel<1, true>));
    case 2: return std::min(q(assign_pipe_kernel<2, false>), q(assign_pipe_kernel<2, true>));
    case 3: return std::min(q(assign_pipe_kernel<3, false>), q(assign_pipe_kernel<3, true>));
    default: return std::min(q(assign_pipe_kernel<4, false>), q(assign_pipe_kernel<4, true>));
    }
}

// The same for the chunk-combining forms (chunked palettes, nch = 2 .. 16).
int assign_residency_chunked() {
    auto q = [](auto kern) {
        int n = 0;
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, 256, 0) == hipSuccess ? n : 0;
    };
    int r = std::min(q(assign_pipe_kernel<4, false, 2>), q(assign_pipe_kernel<4, true, 2>));
    r = std::min(r, std::min(q(assign_pipe_kernel<4, false, 4>), q(assign_pipe_kernel<4, true, 4>)));
    r = std::min(r, std::min(q(assign_pipe_kernel<4, false, 4, 2>), q(assign_pipe_kernel<4, true, 4, 2>)));
    return r;
}

}  // namespace hq

#ifdef HQ_ASSIGN_TIMING
// diagnostic build only: the last assign launch's workgroup stamps (wall_clock64 ticks)
extern "C" int hq_debug_assign_slow(unsigned int* out) {  // and resets the counts
    const int e = (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(hq::g_asg_slow), 2 * sizeof(unsigned int));
    const unsigned int z[2] = {0u, 0u};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(hq::g_asg_slow), z, sizeof z);
    return e;
}
extern "C" int hq_debug_assign_stamps(unsigned long long* out, int n) {
    n = n < hq::kAsgStamps ? n : hq::kAsgStamps;
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(hq::g_asg_t), sizeof(unsigned long long) * 8 * (size_t)n);
}
#endif
