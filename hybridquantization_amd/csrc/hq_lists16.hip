// hq_lists16.hip -- native 16-bit candidate lists for chunked palettes of 4 to
// 32 chunks (512 < K <= 8192).  The chunked path (hq_assign.hip) runs one
// grid per 256-colour chunk and nch / 4 assign passes that carry the best
// distance so far through a scratch image: 16 lookups and list walks per pixel
// at K = 4096.  Here one grid covers all K colours at a finer level 2 (64^3
// cells of 1/64: about as many colours per cell as K = 256 has at 32^3) and
// assign makes one lookup and one walk per pixel and palette, writing the
// 16-bit index the chunked cost kernel reads (colour k = chunk k >> 8, entry
// k & 255: the sub-palettes are the palette's colours in order).
//
// The lists are exact in the sense of build_grid (hq_search.hip): every
// colour that can be the reference's argmin (CL:179-193: the first minimum of
// ref_dist in ascending index) for some pixel of a cell is listed.  A cell's
// threshold T is the least upper bound of d^2 over the cell among the
// colours; a colour whose lower bound exceeds T (1 + 1e-5) never wins there.
// The walk ranks the candidates by d^2 and re-resolves a pixel whose runner-up
// lies within 1e-6 relative (a possible tie of the reference's distance) by the
// least (ref_dist, index) over its list: the reference's first minimum.
// Overflowing level-2 entries fall back to the pixel's level-1 list, an
// overflowing level-1 list (or a pixel outside the unit cube, or a palette
// with a non-finite colour) to all K colours, cooperatively by the wave.
#include <mutex>
#include <unordered_map>

#include "hq_device.h"
#include "hq_launch.h"

namespace hq {

// ----------------------------------------------------------------------------
// The grid: one workgroup of 1024 threads per level-0 cell (side 1/4) and
// palette, grid (64, P).  Level 0: the threshold over all K colours (read from
// memory, 4 per thread) and the cell's candidates, compacted into LDS as
// colours + indices.  Level 1: its 64 cells of side 1/16, 4 per wave (the
// wave's lanes over the level-0 candidates, one LDS read per colour for the 4
// cells), the threshold and the list by ballot (positions into that LDS array,
// and the colour indices to memory for assign's fallback).  Level 2: the 4096
// cells of side 1/64 below, one thread per cell; a wave's 64 threads share a
// parent, whose list sits in registers and is broadcast by readlane; each
// entry is written by its thread.
// Each level's candidates are a superset of the colours that can win in its
// cells: a pixel's winner w is within d(x, b) of it for every colour b, so
// w passes the parent's test and then the child's over the parent's list.
// ----------------------------------------------------------------------------
__device__ __forceinline__ float box_min2(float4 c, const float (&lo)[3], float w) {
    return (ax_min2(c.x, lo[0], lo[0] + w) + ax_min2(c.y, lo[1], lo[1] + w)) + ax_min2(c.z, lo[2], lo[2] + w);
}
__device__ __forceinline__ float box_max2(float4 c, const float (&lo)[3], float w) {
    return (ax_max2(c.x, lo[0], lo[0] + w) + ax_max2(c.y, lo[1], lo[1] + w)) + ax_max2(c.z, lo[2], lo[2] + w);
}

constexpr int kN16Threads = 1024;
// SOA: the level-0 candidates as three float planes (12 B per colour: K =
// 8192 fits beside the lists), else float4 (one ds_read_b128 each; the planes
// cost K = 4096 1.4 us)
template <bool SOA, bool TR>
__global__ __launch_bounds__(kN16Threads) void lists16_kernel(Lists16Args a) {
    constexpr int kN16L1Words = SOA ? 256 : 128, kN16L1Cap = kN16L1Words - 1;  // (n16_l1_words)
    // [K] float4 or [3][K] floats, then the colour indices (declared float4: the
    // b128 reads need the 16-B alignment known; a float array left them split)
    extern __shared__ float4 s_cfv[];
    float* const s_cf = reinterpret_cast<float*>(s_cfv);
    float* const s_cx = s_cf;
    float* const s_cy = s_cf + a.K;
    float* const s_cz = s_cf + 2 * a.K;
    float4* const s_c4 = s_cfv;
    auto c0at = [&](int i) {
        if constexpr (SOA) return make_float4(s_cx[i], s_cy[i], s_cz[i], 0.f);
        else return s_c4[i];
    };
    uint16_t* s_k0 = reinterpret_cast<uint16_t*>(s_cf + (SOA ? 3 : 4) * a.K);  // [K] their colour indices
    uint16_t* s_l1 = s_k0 + a.K;                                   // [64][kN16L1Words] positions in the level-0 planes
    __shared__ float s_red[kN16Threads / 64];
    __shared__ int s_n0;
    const int p = blockIdx.y, c0 = blockIdx.x, tid = threadIdx.x, K = a.K;
    const int lane = tid & 63, wv = tid >> 6;
    if (c0 == 0) {  // for the assign and cost kernels that follow
        const int wpp = 8 * a.nch;
        for (int i = tid; i < wpp * kUsedSlots; i += kN16Threads)
            a.used_glob[(i / wpp) * a.used_stride + p * wpp + i % wpp] = 0u;
        if (tid < 4 * kAccSlots) a.acc_zero[((int64_t)(tid >> 2) * acc_pitch(a.P_acc) + p) * 4 + (tid & 3)] = 0ull;
    }
    bool exh = false;
    for (int j = 0; j < a.nch; ++j) exh |= a.pflags[p * a.nch + j] != 0;
    const float4* pal = a.pal + (int64_t)p * a.kpal;
    if (tid == 0) s_n0 = 0;
    // level 0
    // level-0 cell (side 1 / kN16G0) coordinates
    const int C0i = c0 / (kN16G0 * kN16G0), C0j = (c0 / kN16G0) % kN16G0, C0k = c0 % kN16G0;
    const float w0 = 1.0f / kN16G0;
    const float lo0[3] = {(float)C0i * w0, (float)C0j * w0, (float)C0k * w0};
    constexpr int U = (SOA ? kN16MaxK : 4096) / kN16Threads;  // colours per thread (K <= 4096 unless SOA)
    float4 cv[U];
    float m = INFINITY;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int i = tid + kN16Threads * u;
        cv[u] = pal[min(i, K - 1)];
        if (i < K) m = fminf(m, box_max2(cv[u], lo0, w0));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fminf(m, __shfl_xor(m, off, 64));
    if (lane == 0) s_red[wv] = m;
    __syncthreads();
    float t0 = s_red[0];
#pragma unroll
    for (int w = 1; w < kN16Threads / 64; ++w) t0 = fminf(t0, s_red[w]);
    const float thr0 = t0 * HQ_CAND_MARGIN;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int i = tid + kN16Threads * u;
        const bool cand = i < K && box_min2(cv[u], lo0, w0) <= thr0;
        const uint64_t bal = __ballot(cand);
        int base = 0;
        if (lane == 0 && bal) base = atomicAdd(&s_n0, __popcll(bal));
        base = __shfl(base, 0, 64);
        if (cand) {
            const int pos = base + __popcll(bal & ((1ull << lane) - 1ull));
            if constexpr (SOA) {
                s_cx[pos] = cv[u].x;
                s_cy[pos] = cv[u].y;
                s_cz[pos] = cv[u].z;
            } else {
                s_c4[pos] = cv[u];
            }
            s_k0[pos] = (uint16_t)i;
        }
    }
    __syncthreads();
    const int n0 = s_n0;
    // level 1: wave wv takes cells 4 wv .. 4 wv + 3, its lanes the level-0
    // candidates (one LDS read per colour serves the 4 cells); lists in
    // ascending position order by ballot
    const float w1 = 1.0f / kN16G1;
    {
        float lo1[4][3], t1[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int ch = 4 * wv + c;
            lo1[c][0] = (float)(4 * C0i + (ch >> 4)) * w1;
            lo1[c][1] = (float)(4 * C0j + ((ch >> 2) & 3)) * w1;
            lo1[c][2] = (float)(4 * C0k + (ch & 3)) * w1;
            t1[c] = INFINITY;
        }
        for (int i = lane; i < n0; i += 64) {
            const float4 cv = c0at(i);
#pragma unroll
            for (int c = 0; c < 4; ++c) t1[c] = fminf(t1[c], box_max2(cv, lo1[c], w1));
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) t1[c] = fminf(t1[c], __shfl_xor(t1[c], off, 64));
            t1[c] *= HQ_CAND_MARGIN;
        }
        int cnt[4] = {0, 0, 0, 0};
        const uint64_t below = (1ull << lane) - 1ull;
        if (!exh) {
            for (int i0 = 0; i0 < n0; i0 += 64) {
                const int i = i0 + lane;
                const float4 cv = c0at(min(i, n0 - 1));
                const uint16_t kk = s_k0[min(i, n0 - 1)];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const bool cand = i < n0 && box_min2(cv, lo1[c], w1) <= t1[c];
                    const uint64_t bal = __ballot(cand);
                    const int pos = cnt[c] + __popcll(bal & below);
                    if (cand && pos < kN16L1Cap) {
                        const int ch = 4 * wv + c;
                        const int I = 4 * C0i + (ch >> 4), J = 4 * C0j + ((ch >> 2) & 3), L = 4 * C0k + (ch & 3);
                        s_l1[ch * kN16L1Words + 1 + pos] = (uint16_t)i;
                        a.lvl1[((int64_t)p * (kN16G1 * kN16G1 * kN16G1) + (I * kN16G1 + J) * kN16G1 + L) * kN16L1Words +
                               1 + pos] = kk;
                    }
                    cnt[c] += __popcll(bal);
                }
            }
        }
        if (lane < 4) {
            int total = cnt[0];
#pragma unroll
            for (int c = 1; c < 4; ++c) total = lane == c ? cnt[c] : total;
            const int ch = 4 * wv + lane;
            const int I = 4 * C0i + (ch >> 4), J = 4 * C0j + ((ch >> 2) & 3), L = 4 * C0k + (ch & 3);
            const uint16_t h = exh || total > kN16L1Cap ? kN16Ovf : (uint16_t)total;
            s_l1[ch * kN16L1Words] = h;
            a.lvl1[((int64_t)p * (kN16G1 * kN16G1 * kN16G1) + (I * kN16G1 + J) * kN16G1 + L) * kN16L1Words] = h;
        }
    }
    __syncthreads();
    // level 2: wave wv takes parents wv + 16 j; each lane writes the entry of
    // child `lane`.  TR (K > 2048, long parent lists): the bounds formed with
    // the lanes over the parent's list (transposed); else the lane the child,
    // the list's colours broadcast by readlane (the transposed form's fixed
    // cost -- 64 children per slot and a reduction -- is more than short
    // lists' pairs: K = 1024 grid 34 -> 46 us with it, K = 4096 66 -> 60)
    const float w2 = 1.0f / kN16G2;
    auto rl = [](float x, int i) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), i)); };
    for (int j = 0; j < 4; ++j) {
        const int ch = wv + 16 * j, sub = lane;
        const int I2 = 16 * C0i + 4 * (ch >> 4) + (sub >> 4);
        const int J2 = 16 * C0j + 4 * ((ch >> 2) & 3) + ((sub >> 2) & 3);
        const int L2 = 16 * C0k + 4 * (ch & 3) + (sub & 3);
        const float lo2[3] = {(float)I2 * w2, (float)J2 * w2, (float)L2 * w2};
        // up to K = 4096 palette pairs interleaved per cell (one 64-B line holds
        // both entries: assign16 takes two palettes per workgroup); above, a table
        // per palette
        const int64_t cell2 = (I2 * kN16G2 + J2) * kN16G2 + L2, n2 = kN16G2 * kN16G2 * kN16G2;
        uint16_t* out = a.lvl2 + (a.K <= 4096 ? ((((int64_t)(p >> 1) * n2 + cell2) << 1) + (p & 1))
                                              : (int64_t)p * n2 + cell2) * kN16L2Words;
#ifdef HQ_ABL_N16NOL2  // timing ablation of the grid: no level-2 lists (every entry overflows)
        out[0] = kN16Ovf;
        continue;
#endif
        if (exh) {
            out[0] = kN16Ovf;
            continue;
        }
        const uint16_t* sl = s_l1 + ch * kN16L1Words;
        const int c1 = __builtin_amdgcn_readfirstlane((int)sl[0]);
        int cnt = 0;
        if (c1 != kN16Ovf) {
            if constexpr (!TR) {
                // per child: the lane the child; the parent's list in registers
                // (position 64 j + lane in slot j), each colour broadcast by readlane
                constexpr int NSL = (kN16L1Cap + 1) / 64;
                float4 cs[NSL];
                float ks[NSL];
#pragma unroll
                for (int j = 0; j < NSL; ++j) {
                    const int pj = 64 * j + lane < c1 ? sl[1 + 64 * j + lane] : 0;
                    cs[j] = c0at(pj);
                    ks[j] = (float)s_k0[pj];  // (exact: < 2^24)
                }
                // centre form of the bounds (3 VALU per axis): per axis |c - m| + h
                // and max(|c - m| - h, 0), m the box centre (exact), h = half a cell.
                // Each is within 2 ulp of the exact term at the terms' sizes here,
                // which the 1e-5 margin covers with T >= 3 h^2 (a colour at the centre)
                const float h2 = 0.5f * w2;
                const float m0 = lo2[0] + h2, m1 = lo2[1] + h2, m2 = lo2[2] + h2;
                auto bmax = [&](float x, float y, float z) {
                    const float tx = fabsf(x - m0) + h2, ty = fabsf(y - m1) + h2, tz = fabsf(z - m2) + h2;
                    return fmaf(tz, tz, fmaf(ty, ty, tx * tx));
                };
                // (the clamp to [0, 1] is the add's clamp bit, not a v_max; a term
                // above 1 -- a colour outside the unit cube -- only lowers the bound)
                auto bmin = [&](float x, float y, float z) {
                    const float tx = __builtin_amdgcn_fmed3f(fabsf(x - m0) - h2, 0.f, 1.f),
                                ty = __builtin_amdgcn_fmed3f(fabsf(y - m1) - h2, 0.f, 1.f),
                                tz = __builtin_amdgcn_fmed3f(fabsf(z - m2) - h2, 0.f, 1.f);
                    return fmaf(tz, tz, fmaf(ty, ty, tx * tx));
                };
                // the least bmax as an unsigned min of the bit patterns (bmax >= +0,
                // finite): fminf canonicalised the running minimum every iteration
                uint32_t t2u = 0x7f800000u;
#pragma unroll
                for (int j = 0; j < NSL; ++j) {
                    const int nj = min(c1 - 64 * j, 64);
                    for (int i = 0; i < nj; ++i)
                        t2u = min(t2u, __builtin_bit_cast(uint32_t, bmax(rl(cs[j].x, i), rl(cs[j].y, i), rl(cs[j].z, i))));
                }
                const float thr2 = __builtin_bit_cast(float, t2u) * HQ_CAND_MARGIN;
#pragma unroll
                for (int j = 0; j < NSL; ++j) {
                    const int nj = min(c1 - 64 * j, 64);
                    for (int i = 0; i < nj; ++i)
                        if (bmin(rl(cs[j].x, i), rl(cs[j].y, i), rl(cs[j].z, i)) <= thr2) {
                            if (cnt < kN16L2Cap) out[1 + cnt] = (uint16_t)rl(ks[j], i);
                            ++cnt;
                        }
                }
            } else {
                // Transposed: the lanes take the parent's colours (position 64 j +
                // lane in slot j) and the 64 children are unrolled.  A child's
                // bounds are sums of per-axis terms at its 4 x 4 x 4 place in the
                // parent, so a lane forms 4 terms per axis and slot and one FMA per
                // child finishes a bound, in the order of the per-child form
                // (fmaf(tz, tz, fmaf(ty, ty, tx * tx))): the same bits, the same
                // lists.  Centre form of the terms: per axis |c - m| + h and
                // max(|c - m| - h, 0), m the child's centre (exact), h half a cell;
                // each within 2 ulp of the exact term at the sizes here, which the
                // 1e-5 margin covers with T >= 3 h^2 (a colour at the centre).  The
                // clamp to [0, 1] is the add's clamp bit (a term above 1 -- a colour
                // outside the unit cube -- only lowers the bound).
                constexpr int NSL = (kN16L1Cap + 1) / 64;
                const float h2 = 0.5f * w2;
                const int base[3] = {16 * C0i + 4 * (ch >> 4), 16 * C0j + 4 * ((ch >> 2) & 3), 16 * C0k + 4 * (ch & 3)};
                // slot j's colour (read in each pass: held across both, NSL = 4
                // spilled)
                auto colour = [&](int j) { return c0at(64 * j + lane < c1 ? sl[1 + 64 * j + lane] : 0); };
                auto tmax = [&](float c, int ax, int q) { return fabsf(c - ((float)(base[ax] + q) * w2 + h2)) + h2; };
                auto tmin = [&](float c, int ax, int q) {
                    return __builtin_amdgcn_fmed3f(fabsf(c - ((float)(base[ax] + q) * w2 + h2)) - h2, 0.f, 1.f);
                };
                // the least bmax per child: lane-partial minima (unsigned min of the
                // bit patterns: bmax >= +0; a lane past the list gives +inf), then a
                // transposing reduction that leaves child `lane`'s minimum in T[0]
                uint32_t T[64];
#pragma unroll
                for (int sc = 0; sc < 64; ++sc) T[sc] = 0x7f800000u;
#pragma unroll
                for (int j = 0; j < NSL; ++j) {
                    if (64 * j >= c1) break;
                    const float4 c = colour(j);
                    const bool ok = 64 * j + lane < c1;
                    float x2[4], ty[4], tz[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float tx = tmax(c.x, 0, q);
                        x2[q] = tx * tx;
                        ty[q] = tmax(c.y, 1, q);
                        tz[q] = ok ? tmax(c.z, 2, q) : INFINITY;
                    }
#pragma unroll
                    for (int qa = 0; qa < 4; ++qa)
#pragma unroll
                        for (int qb = 0; qb < 4; ++qb) {
                            const float xy = fmaf(ty[qb], ty[qb], x2[qa]);
#pragma unroll
                            for (int qc = 0; qc < 4; ++qc) {
                                const int sc = 16 * qa + 4 * qb + qc;
                                T[sc] = min(T[sc], __builtin_bit_cast(uint32_t, fmaf(tz[qc], tz[qc], xy)));
                            }
                        }
                }
#pragma unroll
                for (int W = 32; W >= 1; W >>= 1) {
                    const bool hi = (lane & W) != 0;
#pragma unroll
                    for (int sc = 0; sc < W; ++sc) {
                        const uint32_t send = hi ? T[sc] : T[sc + W], keep = hi ? T[sc + W] : T[sc];
                        T[sc] = min(keep, (uint32_t)__shfl_xor((int)send, W, 64));
                    }
                }
                const float thr2 = __builtin_bit_cast(float, T[0]) * HQ_CAND_MARGIN;  // child `lane`'s threshold
                // the candidates: per slot and child a ballot over the colours,
                // parked in lane `child` of the slot's mask words
                uint32_t mlo[NSL], mhi[NSL];
#pragma unroll
                for (int j = 0; j < NSL; ++j) {
                    mlo[j] = mhi[j] = 0u;
                    if (64 * j >= c1) continue;
                    const float4 c = colour(j);
                    const bool ok = 64 * j + lane < c1;
                    float x2[4], ty[4], tz[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float tx = tmin(c.x, 0, q);
                        x2[q] = tx * tx;
                        ty[q] = tmin(c.y, 1, q);
                        tz[q] = tmin(c.z, 2, q);
                    }
#pragma unroll
                    for (int qa = 0; qa < 4; ++qa)
#pragma unroll
                        for (int qb = 0; qb < 4; ++qb) {
                            const float xy = fmaf(ty[qb], ty[qb], x2[qa]);
#pragma unroll
                            for (int qc = 0; qc < 4; ++qc) {
                                const int sc = 16 * qa + 4 * qb + qc;
                                const float ts = __builtin_bit_cast(
                                    float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, thr2), sc));
                                const uint64_t bal = __ballot(ok && fmaf(tz[qc], tz[qc], xy) <= ts);
                                mlo[j] = lane == sc ? (uint32_t)bal : mlo[j];
                                mhi[j] = lane == sc ? (uint32_t)(bal >> 32) : mhi[j];
                            }
                        }
                }
                // child `lane`'s list: the set bits in ascending position order
#pragma unroll
                for (int j = 0; j < NSL; ++j) cnt += __popc(mlo[j]) + __popc(mhi[j]);
                if (cnt <= kN16L2Cap) {
                    int n = 0;
#pragma unroll
                    for (int j = 0; j < NSL; ++j) {
                        uint64_t m = ((uint64_t)mhi[j] << 32) | mlo[j];
                        while (m) {
                            const int b = __builtin_ctzll(m);
                            m &= m - 1;
                            out[1 + n++] = s_k0[sl[1 + 64 * j + b]];
                        }
                    }
                }
            }
        } else {  // the parent list overflowed: every level-0 candidate (broadcast LDS reads)
            float t2 = INFINITY;
            for (int i = 0; i < n0; ++i) t2 = fminf(t2, box_max2(c0at(i), lo2, w2));
            const float thr2 = t2 * HQ_CAND_MARGIN;
            for (int i = 0; i < n0; ++i)
                if (box_min2(c0at(i), lo2, w2) <= thr2) {
                    if (cnt < kN16L2Cap) out[1 + cnt] = s_k0[i];
                    ++cnt;
                }
        }
        out[0] = cnt > kN16L2Cap ? kN16Ovf : (uint16_t)cnt;
    }
}

hipError_t launch_lists16_grid(const Lists16Args& a, int P, hipStream_t s) {
    const bool soa = a.K > 4096;
    const size_t lds = ((soa ? 3 : 4) * sizeof(float) + sizeof(uint16_t)) * (size_t)a.K +
                       sizeof(uint16_t) * 64 * n16_l1_words(a.K);
    const dim3 grid(kN16G0 * kN16G0 * kN16G0, (unsigned)P);
    auto go = [&](auto kern) {
        if (!allow_dyn_lds(reinterpret_cast<const void*>(kern), lds)) return hipErrorInvalidConfiguration;
        HQ_LAUNCH(kern, grid, dim3(kN16Threads), lds, s, a);
        return hipGetLastError();
    };
    if (soa) return go(lists16_kernel<true, true>);
    if (a.K > 2048) return go(lists16_kernel<false, true>);
    return go(lists16_kernel<false, false>);
}

// ----------------------------------------------------------------------------
// assign16: grid (nblocks * P), block 1024 (16 waves share the 64 KiB table:
// 256-thread workgroups left one wave per SIMD), XCD-relabelled
// palette-major; the palette in LDS.  A thread's pixels are a grid stride, resolved in batches of
// 4 / NPAL: every RGB load of the batch, then every level-2 entry, then the walks.
// ----------------------------------------------------------------------------
#define HQ_ANY16(c) (__builtin_amdgcn_ballot_w64(c) != 0)
// level-2 cell (64^3) of a pixel in the unit cube; its level-1 cell (16^3) is
// each coordinate >> 2 (floor(64 x) / 4 = floor(16 x): exact scalings)
__device__ __forceinline__ uint32_t quad_cell16(float r, float g, float b) {
    const int i = min((int)(r * (float)kN16G2), kN16G2 - 1), j = min((int)(g * (float)kN16G2), kN16G2 - 1),
              k = min((int)(b * (float)kN16G2), kN16G2 - 1);
    return (uint32_t)((i * kN16G2 + j) * kN16G2 + k);
}

// The reference loop (CL:179-192) for the lanes of a wave in mask s, the whole
// wave on one lane's pixel at a time (as argmin_fix, hq_assign.hip): over its
// level-1 list when it has one, else all K; least (distance, index), a NaN
// distance never winning unless colour 0's is NaN.
__device__ __noinline__ int argmin16_fix(float r, float g, float b, bool s, int cur, const uint16_t* l1,
                                         const float4* s_pal, int K) {
    uint64_t sm = __ballot(s);
    const int lane = (int)__lane_id();
    int result = cur;
    while (sm) {
        const int Ln = __builtin_ctzll(sm);
        sm &= sm - 1;
        const float pr = __shfl(r, Ln, 64), pg = __shfl(g, Ln, 64), pb = __shfl(b, Ln, 64);
        const uint64_t lp = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)((uint64_t)l1 >> 32), Ln, 64) << 32) |
                            (uint32_t)__shfl((int)(uint32_t)(uint64_t)l1, Ln, 64);
        const uint16_t* list = reinterpret_cast<const uint16_t*>(lp);
        const int n = list ? (int)list[0] : K;
        float bd = INFINITY;
        uint32_t bkey = 0xffffffffu;
        for (int j = lane; j < n; j += 64) {
            const int k = list ? (int)list[1 + j] : j;
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
        if (lane == Ln) result = d0 != d0 ? 0 : bk;
    }
    return result;
}

// u16 j of the entry, by selects (a variable j must not index the register
// array: that put the entries in scratch, assign 74 -> 103 us)
template <int NQ>
__device__ __forceinline__ uint32_t u16_at(const uint4 (&E)[NQ], int j) {
    const int w = j >> 1;
    uint32_t v = E[0].x;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        v = w == 4 * q ? E[q].x : v;
        v = w == 4 * q + 1 ? E[q].y : v;
        v = w == 4 * q + 2 ? E[q].z : v;
        v = w == 4 * q + 3 ? E[q].w : v;
    }
    return (j & 1) ? v >> 16 : v & 0xffffu;
}

// NPAL palettes per workgroup (2 up to K = 4096: both tables in LDS, one 64-B
// level-2 line per pixel for both, the pixel read once), batches of 4 / NPAL
// pixels per thread.
template <bool U8, int NPAL>
__global__ __launch_bounds__(kN16Threads) void assign16_kernel(AssignArgs a, int P) {
    extern __shared__ float4 s_pal[];  // [NPAL][K]
    constexpr int KB = 4 / NPAL;
    const int npr = (P + NPAL - 1) / NPAL;
    const int w = xcd_remap(blockIdx.x, a.nblocks * npr);
    const int pr = w / a.nblocks, blk = w % a.nblocks, tid = threadIdx.x, K = a.K;
    const int p0 = NPAL * pr, np = min(NPAL, P - p0);
    bool exh[NPAL];
    uint16_t* idx[NPAL];
#pragma unroll
    for (int q = 0; q < NPAL; ++q) {
        const int p = min(p0 + q, P - 1);
        const float4* pal = a.pal + (int64_t)p * a.kpal;
        for (int i = tid; i < K; i += kN16Threads) s_pal[q * K + i] = pal[i];
        exh[q] = false;
        for (int j = 0; j < a.nch; ++j) exh[q] |= a.pflags[p * a.nch + j] != 0;
        idx[q] = a.idx16 + (int64_t)p * a.idx_pitch;
    }
    __syncthreads();
    // NPAL 2: the pair's level-2 lines (4 x 16 B per cell), palette p0 + q at
    // uint4 2 q; NPAL 1: the palette's own table (2 x 16 B per cell)
    const uint4* l2 = reinterpret_cast<const uint4*>(a.l2n) +
                      (int64_t)(NPAL == 2 ? p0 >> 1 : p0) * (kN16G2 * kN16G2 * kN16G2) * (2 * NPAL);
    const int l1w = n16_l1_words(K);
    const uint32_t n_ext = (uint32_t)a.n_ext, qlast = n_ext - 1;
    const uint32_t cstride = (uint32_t)a.nblocks * (uint32_t)kN16Threads;
    const uint32_t qbase = (uint32_t)blk * (uint32_t)kN16Threads + (uint32_t)tid;
    // every lane runs its lane 0's batch count (argmin16_fix needs the whole wave)
    const int npx0 = qbase < n_ext ? (int)((n_ext - 1 - qbase) / cstride) + 1 : 0;
    const int nb = __builtin_amdgcn_readfirstlane((npx0 + KB - 1) / KB);
    // the next batch's pixels are loaded while this batch's entries are looked
    // up and walked: one exposed memory round trip per batch, not two
    uint32_t nv[KB];          // packed bytes (U8)
    float nr[KB], ng[KB], nbl[KB];  // planar floats
    auto load_batch = [&](int bi) {
#pragma unroll
        for (int u = 0; u < KB; ++u) {
            const uint32_t qc = min(qbase + (uint32_t)(bi * KB + u) * cstride, qlast);
            if constexpr (U8) {
                nv[u] = a.rgbx[qc];
            } else {
                nr[u] = a.R[qc];
                ng[u] = a.G[qc];
                nbl[u] = a.B[qc];
            }
        }
    };
    if (nb > 0) load_batch(0);
    for (int bi = 0; bi < nb; ++bi) {
        float r[KB], g[KB], b[KB];
        uint32_t q[KB];
#pragma unroll
        for (int u = 0; u < KB; ++u) {
            q[u] = qbase + (uint32_t)(bi * KB + u) * cstride;
            if constexpr (U8) {
                r[u] = u8_unit(nv[u], 0);
                g[u] = u8_unit(nv[u], 1);
                b[u] = u8_unit(nv[u], 2);
            } else {
                r[u] = nr[u];
                g[u] = ng[u];
                b[u] = nbl[u];
            }
        }
        bool in_[KB];
        constexpr int NQ = kN16L2Words / 8;  // 16-B pieces per entry
        uint4 E[KB][NPAL][NQ];
#pragma unroll
        for (int u = 0; u < KB; ++u) {
            in_[u] = r[u] >= 0.f && r[u] <= 1.f && g[u] >= 0.f && g[u] <= 1.f && b[u] >= 0.f && b[u] <= 1.f;
            const uint32_t cell = in_[u] ? (uint32_t)quad_cell16(r[u], g[u], b[u]) : 0u;
#pragma unroll
            for (int pq = 0; pq < NPAL; ++pq)
#pragma unroll
                for (int qq = 0; qq < NQ; ++qq) E[u][pq][qq] = l2[2 * NPAL * cell + 2 * pq + qq];
        }
        if (bi + 1 < nb) load_batch(bi + 1);
#pragma unroll
        for (int u = 0; u < KB; ++u)
#pragma unroll
        for (int pq = 0; pq < NPAL; ++pq) {
            if (pq >= np) break;  // (workgroup-uniform: the last pair of an odd population)
            const float4* sp = s_pal + pq * K;
            const uint32_t c = E[u][pq][0].x & 0xffffu;
            const bool slow = !in_[u] || exh[pq] || c == kN16Ovf || c == 0u;
            const int cnt = slow ? 0 : (int)c;
            // ranked by d^2 (dist2_rank: within 3 ulp of dist2); a runner-up within
            // 1e-6 relative is a possible distance tie (near_d2): re-resolved over the list below
            float best2 = INFINITY, second2 = INFINITY;
            int bk = 0;
#pragma unroll
            for (int i = 0; i < kN16L2Cap; ++i) {
                if (!HQ_ANY16(i < cnt)) break;
                const int k = (int)u16_at(E[u][pq], i + 1);
                const float d2 = i < cnt ? dist2_rank(r[u], g[u], b[u], sp[i < cnt ? k : 0]) : INFINITY;
                const bool lt = d2 < best2;
                second2 = __builtin_amdgcn_fmed3f(best2, second2, d2);
                bk = lt ? k : bk;
                best2 = lt ? d2 : best2;
            }
            const bool near = !slow && near_d2(best2, second2);
            if (HQ_ANY16(near)) {
                if (near) {  // the reference distance over the list: least (ref_dist, index)
                    float bd = INFINITY;
                    int bkk = 0x7fffffff;
                    for (int i = 0; i < cnt; ++i) {
                        const int k = (int)u16_at(E[u][pq], i + 1);
                        const float d = ref_dist(r[u], g[u], b[u], sp[k]);
                        if (d < bd || (d == bd && k < bkk)) {
                            bd = d;
                            bkk = k;
                        }
                    }
                    bk = bkk;
                }
            }
            if (HQ_ANY16(slow)) {
                // the level-1 list of the pixel's cell when it has one
                const uint16_t* lst = nullptr;
                if (in_[u] && !exh[pq]) {
                    const int i1 = min((int)(r[u] * (float)kN16G1), kN16G1 - 1);
                    const int j1 = min((int)(g[u] * (float)kN16G1), kN16G1 - 1);
                    const int k1 = min((int)(b[u] * (float)kN16G1), kN16G1 - 1);
                    const uint16_t* e = a.l1n + ((int64_t)(p0 + pq) * (kN16G1 * kN16G1 * kN16G1) +
                                                 (i1 * kN16G1 + j1) * kN16G1 + k1) * l1w;
                    if (e[0] != kN16Ovf) lst = e;
                }
                bk = argmin16_fix(r[u], g[u], b[u], slow, bk, lst, sp, K);
            }
            if (q[u] < n_ext) __builtin_nontemporal_store((uint16_t)bk, idx[pq] + q[u]);
        }
    }
}

void launch_used_idx16(const AssignArgs& a, int P, hipStream_t s);  // (hq_assign.hip)

// assign16 then the used bits from the final indices; the profiling events
// bracket both.
hipError_t launch_assign16(const AssignArgs& a0, int P, hipStream_t s) {
    const hipEvent_t ev0 = t_ev_start, ev1 = t_ev_stop;
    AssignArgs a = a0;
    t_ev_stop = nullptr;
    const int npal = a.K <= 4096 ? 2 : 1;  // two 64 KiB tables fit one workgroup up to K = 4096
    const size_t lds = sizeof(float4) * (size_t)a.K * npal;
    const dim3 grid((unsigned)(a.nblocks * ((P + npal - 1) / npal)));
    bool ok = true;
    auto go = [&](auto kern) {
        ok = allow_dyn_lds(reinterpret_cast<const void*>(kern), lds);
        if (ok) HQ_LAUNCH(kern, grid, dim3(kN16Threads), lds, s, a, P);
    };
    if (npal == 2) {
        if (a.rgbx) go(assign16_kernel<true, 2>);
        else go(assign16_kernel<false, 2>);
    } else {
        if (a.rgbx) go(assign16_kernel<true, 1>);
        else go(assign16_kernel<false, 1>);
    }
    if (!ok) {
        t_ev_start = ev0;
        t_ev_stop = ev1;
        return hipErrorInvalidConfiguration;  // the LDS raise was refused: nothing launched
    }
    t_ev_start = nullptr;
    t_ev_stop = ev1;
    launch_used_idx16(a, P, s);
    t_ev_start = ev0;
    return hipGetLastError();
}

template __global__ void lists16_kernel<true, true>(Lists16Args);
template __global__ void lists16_kernel<false, true>(Lists16Args);
template __global__ void lists16_kernel<false, false>(Lists16Args);
template __global__ void assign16_kernel<true, 1>(AssignArgs, int);
template __global__ void assign16_kernel<false, 1>(AssignArgs, int);
template __global__ void assign16_kernel<true, 2>(AssignArgs, int);
template __global__ void assign16_kernel<false, 2>(AssignArgs, int);

}  // namespace hq
