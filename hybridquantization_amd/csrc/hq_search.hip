// hq_search.hip -- per-iteration kernels of the SWASA search around the
// assign and cost kernels: palette prep (opponent table, duplicates, non-finite
// guard), the device-resident SA step (IM:497-568 with SW:54-101), the exact
// two-level candidate grid of the pruned argmin, and the fixed-order fp64
// finalize (IM:736-768, SW:74-82).
#include "hq_device.h"
#include "hq_launch.h"

#include <mutex>
#include <unordered_map>

namespace hq {

// ----------------------------------------------------------------------------
// prep_palette: grid (P), block 1024.
// ----------------------------------------------------------------------------
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
#ifdef HQ_SA_TIMING
__device__ uint64_t g_sa_t[4];  // block 0's stamps inside the SA step (diagnostic build)
#endif
__device__ __forceinline__ uint32_t dup_hash(float4 c) {
    const uint32_t x = __float_as_uint(c.x == 0.f ? 0.f : c.x);
    const uint32_t y = __float_as_uint(c.y == 0.f ? 0.f : c.y);
    const uint32_t z = __float_as_uint(c.z == 0.f ? 0.f : c.z);
    const uint32_t h = x * 0x9E3779B1u ^ (y * 0x85EBCA77u + 0x27D4EB2Fu) ^ (z * 0xC2B2AE3Du + 0x165667B1u);
    return (h ^ (h >> 15)) & (kDupSlots - 1);
}

// LDS of the prep besides the colour table (the caller's: its own, or the SA
// step's candidate table, which the colours already sit in).
struct PrepLds {
    uint32_t tab[kDupSlots], mn[kDupSlots];
    float lin[3 * kMaxK];
    int nonfinite;
};

// Returns colour k's duplicate flag; `nonfinite` = the palette has a colour
// that is not finite.  write: store the outputs (pal, opp, opp16, dup, pflags)
// of palette p (sa_grid_kernel: one workgroup per palette stores, the others
// only use the flags).
__device__ __forceinline__ bool prep_palette_body(const PaletteArgs& a, int p, float4 c, float4* s, PrepLds& L,
                                                  bool write, bool& nonfinite) {
    // threads 0..K-1 handle colour k = tid; any block size >= K.
    const int tid = threadIdx.x, k = tid;
    uint32_t* s_tab = L.tab;
    uint32_t* s_min = L.mn;
    float* s_lin = L.lin;
    for (int i = tid; i < kDupSlots; i += blockDim.x) { s_tab[i] = ~0u; s_min[i] = ~0u; }
    if (tid == 0) L.nonfinite = 0;
    const bool own = k < a.K;
    if (own) c.w = 0.f;  // SW:49: palettes carry .w = 0
    else c = make_float4(0.f, 0.f, 0.f, 0.f);
    if (own) s[k] = c;
    __syncthreads();
#ifdef HQ_SA_TIMING
    if (tid == 0 && blockIdx.x == 0) g_sa_t[2] = wall_clock64();
#endif
    // linear RGB (CL:85-87), one component per thread: a colour's three powf
    // run on three threads (12 waves) instead of one after another (4 waves)
    for (int t = tid; t < 3 * a.K; t += blockDim.x) {
        const float4 cc = s[t / 3];
        const int ch = t % 3;
        s_lin[t] = srgb_lin(ch == 0 ? cc.x : (ch == 1 ? cc.y : cc.z));
    }
    uint32_t slot = 0;
    if (own) {
        if (!(isfinite(c.x) && isfinite(c.y) && isfinite(c.z))) atomicOr(&L.nonfinite, 1);
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
#ifdef HQ_SA_TIMING
    if (tid == 0 && blockIdx.x == 0) g_sa_t[3] = wall_clock64();
#endif
    const bool dup = own && s_min[slot] < (uint32_t)k;
    nonfinite = L.nonfinite != 0;
    if (own && write) {
        const float lr = s_lin[3 * k], lg = s_lin[3 * k + 1], lb = s_lin[3 * k + 2];
        const float4 opp = make_float4(dot3(lr, lg, lb, c_RGB2Opp + 0),
                                       dot3(lr, lg, lb, c_RGB2Opp + 3),
                                       dot3(lr, lg, lb, c_RGB2Opp + 6), 0.f);
        a.pal[(int64_t)p * kMaxK + k] = c;
        a.opp[(int64_t)p * kMaxK + k] = opp;
        a.opp16[(int64_t)p * kMaxK + k] = make_uint4(split_f16(opp.x), split_f16(opp.y), split_f16(opp.z), 0u);
        a.dup[(int64_t)p * kMaxK + k] = dup ? 1u : 0u;
    }
    if (tid == 0 && write) a.pflags[p] = nonfinite;
    return dup;
}

__global__ __launch_bounds__(1024) void prep_palette_kernel(PaletteArgs a) {
    const int p = blockIdx.x, k = threadIdx.x;
    __shared__ float4 s[kMaxK];
    __shared__ PrepLds L;
    const float4 c = k < a.K ? a.pal_in[(int64_t)p * a.K + k] : make_float4(0.f, 0.f, 0.f, 0.f);
    bool nf;
    (void)prep_palette_body(a, p, c, s, L, true, nf);
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
// MAXF: used flags per thread held in registers (the communicator path).
template <int MAXF>
__device__ __forceinline__ void sa_accept(const SaArgs& a, bool writer, SaShared& s) {
#pragma clang fp contract(off)
    const int tid = threadIdx.x, nt = blockDim.x, P = a.P, K = a.K;
    const int wpp = 8 * a.nch;  // used words per palette (chunked palettes: 8 per chunk)
    const int nf = (P * K + nt - 1) / nt;
    double fv[MAXF];
    constexpr int MAXW = 4;  // used words per thread (wpp P <= 4 nt)
    uint32_t fold_word[MAXW] = {0u, 0u, 0u, 0u};
    if (a.accept && a.fold) {  // the finalize's work, folded: the fixed-point sums, the used bits
        // (all loads issued before the first LDS store: in-order counters)
        const double ein = tid < P ? a.err_in[tid] : 0.0;
#pragma unroll
        for (int j = 0; j < MAXW; ++j) {
            const int e = tid + nt * j;
            if (e < wpp * P) {
                // every rank's kUsedSlots copies (row-block ranks: consecutive blocks)
                for (int r = 0; r < a.nranks; ++r) {
                    const uint32_t* u = a.used_glob + (int64_t)r * kUsedSlots * a.used_stride + e;
                    uint32_t wv[kUsedSlots];
#pragma unroll
                    for (int sl = 0; sl < kUsedSlots; ++sl) wv[sl] = u[sl * a.used_stride];
#pragma unroll
                    for (int sl = 0; sl < kUsedSlots; ++sl) fold_word[j] |= wv[sl];
                }
            }
        }
        // palette pp's sum: lanes 16 pp .. 16 pp + 15 load its kAccSlots slot
        // counters (of every rank) and add them across the lanes (integers: in
        // any order, acc_total's value)
        static_assert(kAccSlots == 16, "one 16-lane group per palette");
        for (int e0 = 0; e0 < P * kAccSlots; e0 += nt) {
            const int e = e0 + tid, pp = e >> 4, sl = e & 15;
            unsigned long long lo = 0, hi = 0, bad = 0;
            if (e < P * kAccSlots) {
                for (int r = 0; r < a.nranks; ++r) {
                    const uint64_t* q = a.acc + r * a.acc_rank_words + ((int64_t)sl * acc_pitch(P) + pp) * 4;
                    lo += q[0];
                    hi += q[1];
                    bad += q[2];
                }
            }
#pragma unroll
            for (int m = 8; m >= 1; m >>= 1) {
                lo += __shfl_xor(lo, m, 64);
                hi += __shfl_xor(hi, m, 64);
                bad += __shfl_xor(bad, m, 64);
            }
            if (sl == 0 && e < P * kAccSlots)
                s.sum[pp] = bad ? __builtin_nan("") : (double)hi * 4096.0 + (double)lo * (1.0 / kAccScale);
        }
        if (tid < P) s.err_in[tid] = ein;
    } else if (a.accept) {
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
        s.best_in = a.init ? 0.0 : *a.best_err_in;
        if (writer && a.generate) { jA = a.jump_A[K * 3 * P]; jC = a.jump_C[K * 3 * P]; }
    }
    if (tid < P) s.unused[tid] = 0;
    __syncthreads();
#ifdef HQ_SA_TIMING
    if (tid == 0 && blockIdx.x == 0) g_sa_t[0] = wall_clock64();
#endif
    if (a.accept && a.fold) {
#pragma unroll
        for (int j = 0; j < MAXW; ++j) {
            const int e = tid + nt * j;
            if (e < wpp * P) {  // unused colours: clear bits below K
                const int nbits = min(max(K - 32 * (e % wpp), 0), 32);
                const uint32_t valid = nbits >= 32 ? ~0u : ((1u << nbits) - 1u);
                const int clear = nbits - __popc(fold_word[j] & valid);
                if (clear) atomicAdd(&s.unused[e / wpp], clear);
            }
        }
    } else if (a.accept) {
        if (nf <= MAXF) {
            // a wave's flags are consecutive: one ballot count per palette it spans
            // (one LDS atomic per wave instead of one per unused colour)
            for (int j = 0; j < nf; ++j) {
                const int e = tid + j * nt, e0 = (tid & ~63) + j * nt;
                const bool z = e < P * K && fv[j] == 0.0;
                const int pe = e / K, plo = e0 / K, phi = min((e0 + 63) / K, P - 1);
                for (int pp = plo; pp <= phi; ++pp) {
                    const int n = __popcll(__ballot(z && pe == pp));
                    if ((tid & 63) == 0 && n) atomicAdd(&s.unused[pp], n);
                }
            }
        } else {
            for (int e = tid; e < P * K; e += nt)
                if (a.out[(int64_t)(e / K) * (1 + K) + 1 + e % K] == 0.0) atomicAdd(&s.unused[e / K], 1);
        }
    }
    if (a.accept) {
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
#ifdef HQ_SA_TIMING
        if (tid == 0 && blockIdx.x == 0) g_sa_t[1] = wall_clock64();
#endif
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
                *a.best_err_out = best;
                *a.seed_out = a.generate ? lcg_jump(seed, jA, jC) : seed;
            }
        }
    } else if (tid == 0) {
        s.best = -1;
        for (int i = 0; i < P; ++i) s.src[i] = -1;
        if (writer) {
            for (int i = 0; i < P; ++i) a.err_out[i] = a.err_in[i];
            *a.best_err_out = s.best_in;
            *a.seed_out = a.generate ? lcg_jump(s.seed, a.jump_A[K * 3 * P], a.jump_C[K * 3 * P]) : s.seed;
        }
    }
    __syncthreads();
}

// Prefetches of a step, issued before the acceptance: member p's candidate and
// kept palette (elements e0 + tid + nt j of its colours, chunk ch's 1,024 floats
// at most) and this thread's jumps to draws t0 + tid + nt j (768 at most), nt =
// 1024 / NPF threads.
template <int NPF>
struct SaPf {
    float cand[NPF], col[NPF];
    uint64_t jA[NPF], jC[NPF], bA = 0, bC = 0;
    __device__ __forceinline__ void load(const SaArgs& a, int p, int ch) {
        const int n4 = 4 * a.K, tid = threadIdx.x, nt = 1024 / NPF;
        const int e0 = a.nch > 1 ? 4 * kMaxK * ch : 0, t0 = a.nch > 1 ? 3 * kMaxK * ch : 0;
#pragma unroll
        for (int j = 0; j < NPF; ++j) {
            const int e = e0 + tid + nt * j, t = t0 + tid + nt * j;
            cand[j] = col[j] = 0.f;
            jA[j] = jC[j] = 0;
            if (e < n4 && tid + nt * j < 4 * kMaxK) {
                if (a.accept) cand[j] = a.cand_in[(int64_t)p * n4 + e];
                col[j] = a.colors_in[(int64_t)p * n4 + e];
            }
            if (a.generate && t < 3 * a.K && tid + nt * j < 3 * kMaxK) {
                jA[j] = a.jump_A[t + 1];
                jC[j] = a.jump_C[t + 1];
            }
        }
        if (a.generate) {
            bA = a.jump_A[3 * a.K * p];
            bC = a.jump_C[3 * a.K * p];
        }
    }
};

// Member p's accepted palette into s_from (LDS, 4K floats; chunked palettes:
// elements e0 .. e0 + 1023 of it, chunk c = e0 / 1024); `lead` also copies it
// to colors_out (and, for p = 0, a new best to best_colors).  The two likely
// sources -- member p's candidate and its kept palette -- were read before the
// acceptance (pf); only a convergence copy from another member's candidate
// reads after it.
template <int NPF>
__device__ __forceinline__ void sa_keep(const SaArgs& a, int p, int e0, bool lead, const SaShared& s,
                                        const SaPf<NPF>& pf, float* s_from) {
    const int n4 = 4 * a.K, tid = threadIdx.x, nt = 1024 / NPF;
    const int ne = a.nch > 1 ? min(4 * kMaxK, n4 - e0) : n4;
    const int src = s.src[p];
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
        const int i = tid + nt * j, e = e0 + i;
        if (i < ne) {
            float v;
            if (src == p) v = pf.cand[j];
            else if (src < 0) v = pf.col[j];
            else v = a.cand_in[(int64_t)src * n4 + e];
            s_from[i] = v;
            if (lead) a.colors_out[(int64_t)p * n4 + e] = v;
        }
    }
    if (lead && p == 0 && s.best >= 0)  // IM:533-536: the best palette so far
        for (int i = tid; i < ne; i += nt) a.best_colors[e0 + i] = a.cand_in[(int64_t)s.best * n4 + e0 + i];
    __syncthreads();
}

// Candidate p into s_cand (.w = 0; cand_out too when `lead`): draw t = 3i + c of
// this palette's block (SW:91-101 neighbours of s_from, or SW:40-52 random).
// Chunked palettes: chunk ch = colours 256 ch .. (draws t0 = 768 ch ..), and
// the chunk's colours past K are copies of candidate colour 0 (pack_chunks'
// padding), drawn again here from its source colour `src0`.
__device__ __forceinline__ float sa_draw(const SaArgs& a, uint64_t st, float from) {
#pragma clang fp contract(off)
    const float u = (float)(int32_t)(st >> 24) / (float)(1 << 24);
    if (a.random) return u;
    const float step = (u * 2 - 1) * a.amax;
    const float x = from + step;
    return x > 0.f ? (x > 1.f ? 1.f : x) : 0.f;  // clampf_java (SW:103-106)
}

template <int NPF>
__device__ __forceinline__ void sa_generate(const SaArgs& a, int p, int ch, const float* s_from,
                                            const float* src0, uint64_t seed, float4* s_cand, bool lead,
                                            const SaPf<NPF>& pf) {
    const int K = a.K, n4 = 4 * K, tid = threadIdx.x, nt = 1024 / NPF;
    // real colours of this chunk: none when the chunk lies wholly past K (K = 600, chunk 3)
    const int k0 = a.nch > 1 ? kMaxK * ch : 0, kn = a.nch > 1 ? max(0, min(kMaxK, K - k0)) : K;
    const uint64_t base = lcg_jump(seed, pf.bA, pf.bC);  // jump_A/C[3Kp], prefetched
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
        const int tt = tid + nt * j, i = tt / 3, c = tt - 3 * i;
        if (tt < 3 * kn) {
            const float v = sa_draw(a, lcg_jump(base, pf.jA[j], pf.jC[j]), s_from[4 * i + c]);
            reinterpret_cast<float*>(s_cand)[4 * i + c] = v;
            if (lead) a.cand_out[(int64_t)p * n4 + 4 * (k0 + i) + c] = v;
        }
    }
    for (int k = tid; k < kn; k += nt) {
        reinterpret_cast<float*>(s_cand)[4 * k + 3] = 0.f;
        if (lead) a.cand_out[(int64_t)p * n4 + 4 * (k0 + k) + 3] = 0.f;
    }
    if (a.nch > 1 && kn < kMaxK) {  // padding: candidate colour 0 (draws 0, 1, 2)
        __shared__ float s_c0[3];
        if (tid < 3) s_c0[tid] = sa_draw(a, lcg_jump(base, a.jump_A[tid + 1], a.jump_C[tid + 1]), src0[tid]);
        __syncthreads();
        for (int k = kn + tid; k < kMaxK; k += nt) s_cand[k] = make_float4(s_c0[0], s_c0[1], s_c0[2], 0.f);
    }
    __syncthreads();
}

// Build with -DHQ_SA_TIMING to print block 0's phase times (accept, keep,
// generate, prep; wall_clock64 ticks of 10 ns) per launch.
// Chunked palettes (a.nch > 1): workgroup p nch + ch keeps, generates and
// preps chunk ch of member p (sub-palette p nch + ch); every workgroup runs the
// acceptance itself.
__global__ __launch_bounds__(1024) void sa_step_kernel(SaArgs a) {
    const int p = blockIdx.x / a.nch, ch = blockIdx.x % a.nch;
    const int K = a.nch > 1 ? kMaxK : a.K;  // colours prepped by this workgroup
    __shared__ SaShared s;
    __shared__ float s_from[4 * kMaxK];
    __shared__ float4 s_cand[kMaxK];
#ifdef HQ_SA_TIMING
    const uint64_t t0 = wall_clock64();
#endif
    SaPf<1> pf;
    pf.load(a, p, ch);
    sa_accept<16>(a, blockIdx.x == 0, s);
#ifdef HQ_SA_TIMING
    const uint64_t t1 = wall_clock64();
#endif
    const int e0 = 4 * kMaxK * ch;
    sa_keep(a, p, e0, true, s, pf, s_from);
#ifdef HQ_SA_TIMING
    const uint64_t t2 = wall_clock64();
#endif
    if (!a.generate) return;
    // chunks past colour 0's: its source colour (the member's accepted colour 0)
    __shared__ float s_src0[3];
    if (a.nch > 1 && ch > 0 && threadIdx.x < 3) {
        const int src = s.src[p], n4 = 4 * a.K;
        s_src0[threadIdx.x] = src >= 0 ? a.cand_in[(int64_t)src * n4 + threadIdx.x]
                                       : a.colors_in[(int64_t)p * n4 + threadIdx.x];
    }
    sa_generate(a, p, ch, s_from, ch > 0 ? s_src0 : s_from, s.seed, s_cand, true, pf);
#ifdef HQ_SA_TIMING
    const uint64_t t3 = wall_clock64();
#endif
    const int k = threadIdx.x;
    __shared__ PrepLds L;
    bool nf;
    (void)prep_palette_body(a.prep, blockIdx.x, k < K ? s_cand[k] : make_float4(0.f, 0.f, 0.f, 0.f), s_cand, L,
                            true, nf);
#ifdef HQ_SA_TIMING
    __syncthreads();
    if (threadIdx.x == 0 && p == 0)
        printf("SA_T %d %d %d %d %d | loads %d exp %d seq %d\n", a.accept, (int)(t1 - t0), (int)(t2 - t1),
               (int)(t3 - t2), (int)(wall_clock64() - t3), (int)(g_sa_t[0] - t0), (int)(g_sa_t[1] - g_sa_t[0]),
               (int)(t1 - g_sa_t[1]));
    if (threadIdx.x == 0 && p == 0)
        printf("SA_P fill %d hash %d rest %d\n", (int)(g_sa_t[2] - t3), (int)(g_sa_t[3] - g_sa_t[2]),
               (int)(wall_clock64() - g_sa_t[3]));
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
// (box bounds ax_min2 / ax_max2 and HQ_CAND_MARGIN: hq_device.h)

// Level-2 entries are interleaved by groups of 4 palettes: the 4 entries of one
// cell sit side by side (32 B at 8 B per entry), so a pixel evaluated under the
// 4 palettes of a group fetches one line instead of 4, in two 16-B loads per
// lane (random lookups are bound by the L1 accesses they cause, not by their
// bytes).  An 8-B entry holds count + 7 indices: after the dominance pruning
// ~0.2% of cells list more (uniform noise, K = 256, G2 = 32); those overflow
// into the reference loop (assign's argmin_fix).
__host__ __device__ __forceinline__ int64_t lvl2_offset(int64_t gstride, int p, int64_t cell) {
    return (int64_t)(p >> 2) * gstride + cell * kL2Line + (p & 3) * kL2Bytes;
}

// Per-axis child terms of the level-2 pass: s_ax[axis][j][i] = the bound of
// parent-list entry i along `axis` for the child at position j (0..3) of the
// cell on that axis.  A child's bound is the sum of its three axis terms, so
// the 64 children share 12 terms per entry instead of 64 x 3.  Pitch 260:
// the children of a wave that differ in position along an axis read rows 4
// banks apart (a plain 256 pitch put them in one bank).
constexpr int kAxPitch = kMaxK + 4;

template <bool MAX>
__device__ __forceinline__ void axis_terms(float (*s_ax)[4][kAxPitch], const float4* s_col,
                                           const uint8_t* s_list, int total, int ci, int cj, int ck,
                                           float inv2) {
    const int t = threadIdx.x;
    if (t < total) {
        const float4 cc = s_col[s_list[t]];
        const float v[3] = {cc.x, cc.y, cc.z};
        const int base[3] = {4 * ci, 4 * cj, 4 * ck};
#pragma unroll
        for (int ax = 0; ax < 3; ++ax)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float lo = (float)(base[ax] + j) * inv2, hi = (float)(base[ax] + j + 1) * inv2;
                s_ax[ax][j][t] = MAX ? ax_max2(v[ax], lo, hi) : ax_min2(v[ax], lo, hi);
            }
    }
}

__device__ __forceinline__ void drop_positions(uint32_t (&w)[4], int& n, uint32_t drop);

// Dominance pruning (exact) of one child entry (w[4], n candidates, quad lane
// q): see the comment in grid_cell_body.
__device__ __forceinline__ void prune_dominated(uint32_t (&w)[4], int& n, const float4* col, int bstar,
                                                const float (&blo)[3], const float (&bhi)[3], int q) {
    const float4 cb = col[bstar];
    const float vb[3] = {cb.x, cb.y, cb.z};
    const float nb = (vb[0] * vb[0] + vb[1] * vb[1]) + vb[2] * vb[2];
    uint32_t drop = 0u;
    // list position i = q + 4t sits in byte (i + 1) & 3 of word (i + 1) >> 2
    const int sh = 8 * ((q + 1) & 3), wo = (q + 1) >> 2;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int i = q + 4 * t;
        if (i >= n) break;
        const uint32_t word = wo ? w[t < 3 ? t + 1 : 3] : w[t];
        const int ka = (int)((word >> sh) & 0xffu);
        if (ka == bstar) continue;
        const float4 ca = col[ka];
        const float va[3] = {ca.x, ca.y, ca.z};
        const float dmax2a = (ax_max2(va[0], blo[0], bhi[0]) + ax_max2(va[1], blo[1], bhi[1])) +
                             ax_max2(va[2], blo[2], bhi[2]);
        const float na = (va[0] * va[0] + va[1] * va[1]) + va[2] * va[2];
        float fmin = na - nb, S = na + nb + dmax2a;
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) {
            const float cc = 2.0f * (vb[ax] - va[ax]);
            const float tl = cc * blo[ax], th = cc * bhi[ax];
            fmin += fminf(tl, th);
            S += fmaxf(fabsf(tl), fabsf(th));
        }
        if (fmin > 1e-5f * S) drop |= 1u << i;
    }
    drop_positions(w, n, drop);
}

// Dominance test of prune_dominated for colour a (bound dmax2a over the box)
// against colour b.
__device__ __forceinline__ bool dominated_by(const float (&va)[3], float dmax2a, const float (&vb)[3],
                                             const float (&blo)[3], const float (&bhi)[3]) {
    const float na = (va[0] * va[0] + va[1] * va[1]) + va[2] * va[2];
    const float nb = (vb[0] * vb[0] + vb[1] * vb[1]) + vb[2] * vb[2];
    float fmin = na - nb, S = na + nb + dmax2a;
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) {
        const float cc = 2.0f * (vb[ax] - va[ax]);
        const float tl = cc * blo[ax], th = cc * bhi[ax];
        fmin += fminf(tl, th);
        S += fmaxf(fabsf(tl), fabsf(th));
    }
    return fmin > 1e-5f * S;
}

// Lists still longer than a stored entry holds (kL2Cap) after prune_dominated
// (~0.2% of cells on uniform noise, K = 256, G2 = 32, 8-B entries): every
// candidate is tested against every other one of its list (the same exact
// test; a colour dominated by any listed colour never wins, and two colours
// cannot dominate each other), which leaves ~1/7 of them overflowing.  The
// quads of such children post their lists (slot: entry words, count, child);
// a wave then takes one list at a time, its lanes testing the n (n - 1)
// ordered pairs (<= 4 per lane), and ORs the drops into the slot.  (One quad
// testing its own pairs held the workgroup: build_grid 13.3 -> 18.2 us.)
struct LongLists {
    uint32_t ent[64][4];
    uint32_t drop[64];
    uint8_t n[64], ch[64];
    int count;
};

__device__ __forceinline__ void prune_long_lists(LongLists& L, const float4* col, int nl, int ci, int cj,
                                                 int ck, float inv2) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int it = wave; it < nl; it += 4) {
        const int chl = L.ch[it], nn = L.n[it];
        const float blo[3] = {(float)(4 * ci + (chl >> 4)) * inv2, (float)(4 * cj + ((chl >> 2) & 3)) * inv2,
                              (float)(4 * ck + (chl & 3)) * inv2};
        const float bhi[3] = {blo[0] + inv2, blo[1] + inv2, blo[2] + inv2};
        const uint8_t* keys = reinterpret_cast<const uint8_t*>(L.ent[it]) + 1;
        for (int pi = lane; pi < nn * nn; pi += 64) {
            const int ia = pi / nn, ib = pi - ia * nn;
            if (ia == ib) continue;
            const float4 ca = col[keys[ia]], cb = col[keys[ib]];
            const float va[3] = {ca.x, ca.y, ca.z}, vb[3] = {cb.x, cb.y, cb.z};
            const float dm = (ax_max2(va[0], blo[0], bhi[0]) + ax_max2(va[1], blo[1], bhi[1])) +
                             ax_max2(va[2], blo[2], bhi[2]);
            if (dominated_by(va, dm, vb, blo, bhi)) atomicOr(&L.drop[it], 1u << ia);
        }
    }
}

// The drop masks of a quad (OR-combined) applied to its entry: kept positions
// move down in ascending order, count byte below them.
__device__ __forceinline__ void drop_positions(uint32_t (&w)[4], int& n, uint32_t drop) {
    drop |= (uint32_t)__shfl_xor((int)drop, 1, 64);
    drop |= (uint32_t)__shfl_xor((int)drop, 2, 64);
    if (drop) {  // rebuild the entry from the kept positions, ascending
        uint32_t x0 = 0u, x1 = 0u, x2 = 0u, x3 = 0u;
        int kept = 0;
#pragma unroll
        for (int i = kL2Build - 1; i >= 0; --i) {
            if (i < n && !((drop >> i) & 1u)) {
                x3 = (x3 << 8) | (x2 >> 24);
                x2 = (x2 << 8) | (x1 >> 24);
                x1 = (x1 << 8) | (x0 >> 24);
                x0 = (x0 << 8) | ((w[(i + 1) >> 2] >> (8 * ((i + 1) & 3))) & 0xffu);
                ++kept;
            }
        }
        // the count's byte goes in below the first kept candidate
        w[3] = (x3 << 8) | (x2 >> 24);
        w[2] = (x2 << 8) | (x1 >> 24);
        w[1] = (x1 << 8) | (x0 >> 24);
        w[0] = x0 << 8;
        n = kept;
    }
}

#ifdef HQ_GRID_TIMING
// diagnostic build: per workgroup start, end, the phase ends (level-1 list,
// pass 1, pass 2, dominance, long lists; wall_clock64 ticks) and the level-1
// list length | long-list count << 16
constexpr int kGridStamps = 65536;
__device__ unsigned long long g_grid_t[kGridStamps][8];
#define HQ_GT_STAMP(i, v)                                                                   \
    do {                                                                                    \
        if (threadIdx.x == 0 && blockIdx.y * gridDim.x + blockIdx.x < (unsigned)kGridStamps) \
            g_grid_t[blockIdx.y * gridDim.x + blockIdx.x][i] = (v);                         \
    } while (0)
#else
#define HQ_GT_STAMP(i, v) ((void)0)
#endif

// LDS of one level-1 cell's grid work.
struct GridLds {
    float4 col[kMaxK];
    float ax[3][4][kAxPitch];
    LongLists lng;  // (8-B entries only)
    uint8_t list[kMaxK];
    float mn[4];
    int wcount[4];
};

// The grid work of level-1 cell `cell` of palette p; thread tid holds colour
// tid (zeros past K) and whether it may be a candidate (prep_palette's
// duplicate flags: an exact duplicate never wins the strict < of CL:186).
__device__ __forceinline__ void grid_cell_body(const GridArgs& a, int p, int cell, float4 c,
                                               bool valid, bool exh, GridLds& L) {
    const int tid = threadIdx.x;
    const int G1 = a.G1, G2 = 4 * G1;
    const int ci = cell / (G1 * G1), cj = (cell / G1) % G1, ck = cell % G1;
    float4* const s_col = L.col;
    uint8_t* const s_list = L.list;
    float* const s_min = L.mn;
    int* const s_wcount = L.wcount;
    float (*const s_ax)[4][kAxPitch] = L.ax;
    LongLists& s_long = L.lng;

    s_col[tid] = c;
    if (kL2Cap < kL2Build && tid == 0) s_long.count = 0;
    const float inv1 = 1.0f / (float)G1;
    const float lo0 = ci * inv1, hi0 = (ci + 1) * inv1;
    const float lo1 = cj * inv1, hi1 = (cj + 1) * inv1;
    const float lo2 = ck * inv1, hi2 = (ck + 1) * inv1;
    float dmin2 = INFINITY, dmax2 = INFINITY;
    if (valid) {
        dmin2 = (ax_min2(c.x, lo0, hi0) + ax_min2(c.y, lo1, hi1)) + ax_min2(c.z, lo2, hi2);
        dmax2 = (ax_max2(c.x, lo0, hi0) + ax_max2(c.y, lo1, hi1)) + ax_max2(c.z, lo2, hi2);
    }
    float m = dmax2;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fminf(m, __shfl_xor(m, off, 64));
    const int wave = tid >> 6, lane = tid & 63;
    if (lane == 0) s_min[wave] = m;
    __syncthreads();
    const float T1 = fminf(fminf(s_min[0], s_min[1]), fminf(s_min[2], s_min[3]));
    const bool cand = valid && dmin2 <= T1 * HQ_CAND_MARGIN;
    const uint64_t bal = __ballot(cand);
    if (lane == 0) s_wcount[wave] = __popcll(bal);
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wave; ++w) base += s_wcount[w];
    const int total = exh ? 0 : s_wcount[0] + s_wcount[1] + s_wcount[2] + s_wcount[3];
    if (cand) s_list[base + __popcll(bal & ((1ull << lane) - 1ull))] = (uint8_t)tid;
    __syncthreads();
    HQ_GT_STAMP(2, wall_clock64());

    uint8_t* l1 = a.lvl1 + (int64_t)p * a.lvl1_pitch + (int64_t)cell * 32;
    const bool ovf1 = exh || total > kL1Cap;
    if (tid < 32) {
        uint8_t v;
        if (tid == 0) v = ovf1 ? kOverflow : (uint8_t)total;
        else v = (!ovf1 && tid - 1 < total) ? s_list[tid - 1] : 0;
        l1[tid] = v;
    }
#ifdef HQ_ABL_GRID_L1ONLY  // timing ablation (wrong results): no level-2 lists
    return;
#endif
    // Level 2: child ch = tid >> 2 of this cell at axis positions (a0, a1, a2),
    // its parent-list positions shared by the 4 threads of a quad (q = tid & 3
    // takes positions q, q+4, ...): T2 and the candidate mask are combined
    // across the quad by shuffles, and each candidate's byte lands at its rank
    // in ascending list order.  Pass 1 reads dmax^2 axis terms, pass 2 dmin^2
    // terms (the same LDS, rewritten between the passes).
    const float inv2 = 1.0f / (float)G2;
    const int ch = tid >> 2, q = tid & 3;
    const int a0 = ch >> 4, a1 = (ch >> 2) & 3, a2 = ch & 3;
    axis_terms<true>(s_ax, s_col, s_list, total, ci, cj, ck, inv2);
    __syncthreads();
    // pass 1: T2 over the whole parent list (which can exceed 31 entries: the
    // level-1 entry then overflows, the children still get lists)
    float t2 = INFINITY;
    int t2pos = 0;  // the parent-list position attaining T2 (the child's closest-in-the-worst-case colour)
    for (int i = q; i < total; i += 4) {
        const float d = (s_ax[0][a0][i] + s_ax[1][a1][i]) + s_ax[2][a2][i];
        if (d < t2) { t2 = d; t2pos = i; }
    }
#pragma unroll
    for (int m = 1; m <= 2; m <<= 1) {
        const float o = __shfl_xor(t2, m, 64);
        const int op = __shfl_xor(t2pos, m, 64);
        if (o < t2 || (o == t2 && op < t2pos)) { t2 = o; t2pos = op; }
    }
    const float thr = t2 * HQ_CAND_MARGIN;
    const int bstar = total > 0 ? (int)s_list[t2pos] : 0;
    __syncthreads();
    HQ_GT_STAMP(3, wall_clock64());
    axis_terms<false>(s_ax, s_col, s_list, total, ci, cj, ck, inv2);
    __syncthreads();
    // pass 2, 32 positions at a time: candidate mask, ranks in list order
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    int n = 0;  // candidates so far (quad-uniform)
    for (int b0 = 0; b0 < total && n <= kL2Build; b0 += 32) {
        uint32_t mine = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int i = b0 + q + 4 * j;
            if (i < total) {
                const float d = (s_ax[0][a0][i] + s_ax[1][a1][i]) + s_ax[2][a2][i];
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
                if (pos <= kL2Build) w[pos >> 2] |= (uint32_t)s_list[b0 + r] << (8 * (pos & 3));
            }
        }
        n += __popc(M);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        w[k] |= (uint32_t)__shfl_xor((int)w[k], 1, 64);
        w[k] |= (uint32_t)__shfl_xor((int)w[k], 2, 64);
    }
    HQ_GT_STAMP(4, wall_clock64());
    // Dominance pruning (exact).  Candidate a of the child's list is dropped
    // when b* -- the colour attaining T2, the child's nearest in the worst
    // case -- is nearer than a to EVERY point of the child box by a margin:
    // f(p) = |p - a|^2 - |p - b|^2 = c . p + |a|^2 - |b|^2 with c = 2 (b - a) is
    // linear, so its minimum over the box is at the corner picked axis by axis.
    // For a pixel p in the box the reference's fp32 d^2 is within ~3e-7
    // relative of the exact one, and its distance (v_sqrt_f32, monotone and
    // within 1 ulp: ref_len, hq_device.h) separates two d^2 that differ by more
    // than 2^-20 relative, so f(p) > 1.1e-6 dmax^2(B, a) makes d_a > d_b
    // strictly: a never wins, not even a tie (CL:179-192).  The test asks f_min > 1e-5 (dmax^2(B, a) + S), S bounding
    // the terms of the fp32 evaluation of f_min (its own rounding is < 1e-6 S).
    // Every reference winner stays listed, so the pruned argmin is unchanged;
    // the lists shrink (uniform noise, K = 256, G2 = 32: mean 2.7 -> 2.05, the
    // longest of 64 pixels' lists 7.9 -> 5.9; against every other candidate
    // instead of b* only: 2.0 / 5.2, at O(n^2) build cost), and with them
    // assign's candidate loop, which runs each wave's longest list.
#ifndef HQ_NO_DOMINANCE
    if (!exh && n >= 2 && n <= kL2Build) {
        const float blo[3] = {(float)(4 * ci + a0) * inv2, (float)(4 * cj + a1) * inv2,
                              (float)(4 * ck + a2) * inv2};
        const float bhi[3] = {blo[0] + inv2, blo[1] + inv2, blo[2] + inv2};
        prune_dominated(w, n, s_col, bstar, blo, bhi, q);
    }
    HQ_GT_STAMP(5, wall_clock64());
    if constexpr (kL2Cap < kL2Build) {
        const bool lng = !exh && n > kL2Cap && n <= kL2Build;  // quad-uniform
        int slot = 0;
        if (lng && q == 0) {
            slot = atomicAdd(&s_long.count, 1);
#pragma unroll
            for (int k = 0; k < 4; ++k) s_long.ent[slot][k] = w[k];
            s_long.drop[slot] = 0u;
            s_long.n[slot] = (uint8_t)n;
            s_long.ch[slot] = (uint8_t)ch;
        }
        __syncthreads();
        const int nl = s_long.count;
        HQ_GT_STAMP(7, (unsigned long long)total | ((unsigned long long)nl << 16));
        if (nl > 0) {  // workgroup-uniform
            prune_long_lists(s_long, s_col, nl, ci, cj, ck, inv2);
            __syncthreads();
            slot = __shfl(slot, (int)(threadIdx.x & 60), 64);
            if (lng) drop_positions(w, n, s_long.drop[slot]);
        }
        HQ_GT_STAMP(6, wall_clock64());
    }
#endif
    if (q == 0) {
#ifdef HQ_ABL_TRUNC  // timing ablation (wrong results): long lists truncated, never overflow
        if (!exh && n > kL2Cap && n <= kL2Build) n = kL2Cap;
#endif
        if (exh || n > kL2Cap) { w[0] = kOverflow; w[1] = w[2] = w[3] = 0; }
        else w[0] |= (uint32_t)n;
        const int ci2 = ci * 4 + a0, cj2 = cj * 4 + a1, ck2 = ck * 4 + a2;
        uint8_t* l2e = a.lvl2 + lvl2_offset(a.lvl2_gstride, p, (int64_t)(ci2 * G2 + cj2) * G2 + ck2);
        if constexpr (kL2Bytes == 16) *reinterpret_cast<uint4*>(l2e) = make_uint4(w[0], w[1], w[2], w[3]);
        else *reinterpret_cast<uint2*>(l2e) = make_uint2(w[0], w[1]);
    }
}


__global__ __launch_bounds__(256) void build_grid_kernel(GridArgs a) {
    const int p = blockIdx.y, tid = threadIdx.x;
#ifdef HQ_GRID_TIMING  // diagnostic build: per-workgroup start / end (wall_clock64, 100 MHz)
    const uint64_t t_start = wall_clock64();
#endif
    if (blockIdx.x == 0 && tid < 8 * kUsedSlots)  // for the assign that follows
        a.used_glob[(tid >> 3) * a.used_stride + p * 8 + (tid & 7)] = 0u;
    if (blockIdx.x == 0 && p % a.nch == 0 && tid < 4 * kAccSlots)  // for the cost kernel
        a.acc_zero[((int64_t)(tid >> 2) * acc_pitch(a.P_acc) + p / a.nch) * 4 + (tid & 3)] = 0ull;
    const bool exh = a.pflags[p] != 0;
    bool valid = false;
    float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tid < a.K) {
        c = a.pal[(int64_t)p * kMaxK + tid];
        valid = !exh && a.dup[(int64_t)p * kMaxK + tid] == 0;
    }
    __shared__ GridLds L;
    grid_cell_body(a, p, blockIdx.x, c, valid, exh, L);
#ifdef HQ_GRID_TIMING
    __syncthreads();
    HQ_GT_STAMP(0, t_start);
    HQ_GT_STAMP(1, wall_clock64());
#endif
}
// ----------------------------------------------------------------------------
// finalize: grid (P), block 1024.  The fixed-point dE sum (acc_total) and the
// used bits -> out[p] = {sum, used[0..K-1]}.
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void finalize_kernel(FinalizeArgs a) {
    constexpr int NT = 1024;
    const int p = blockIdx.x, tid = threadIdx.x;
    double* out = a.out + (int64_t)p * (1 + a.K);
    if (tid == 0) out[0] = acc_total(a.acc, a.P, p);
    if (a.used32) {  // K > 256: the reference's per-colour flags (assign_wide)
        const uint32_t* u = a.used32 + (int64_t)p * a.K;
        for (int k = tid; k < a.K; k += NT) out[1 + k] = u[k] != 0u ? 1.0 : 0.0;
    } else {
        const uint32_t* u = a.used_glob + (int64_t)p * a.wpp;
        for (int k = tid; k < a.K; k += NT) {
            uint32_t w = 0u;
#pragma unroll
            for (int sl = 0; sl < kUsedSlots; ++sl) w |= u[sl * a.used_stride + (k >> 5)];
            out[1 + k] = (w >> (k & 31)) & 1u ? 1.0 : 0.0;
        }
    }
}

// ----------------------------------------------------------------------------
// Launchers
// ----------------------------------------------------------------------------
thread_local hipEvent_t t_ev_start = nullptr, t_ev_stop = nullptr;

bool allow_dyn_lds(const void* fn, size_t bytes) {
    static std::mutex mu;
    static std::unordered_map<const void*, size_t> granted;
    const std::lock_guard<std::mutex> lock(mu);
    size_t& g = granted[fn];
    if (bytes <= g) return true;
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess) return false;
    g = bytes;
    return true;
}
void set_launch_events(hipEvent_t start, hipEvent_t stop) {
    t_ev_start = start;
    t_ev_stop = stop;
}

hipError_t launch_prep_palette(const PaletteArgs& a, int P, hipStream_t s) {
    HQ_LAUNCH(prep_palette_kernel, dim3(P), dim3(1024), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_sa_step(const SaArgs& a, hipStream_t s) {
    HQ_LAUNCH(sa_step_kernel, dim3(a.P * a.nch), dim3(1024), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_build_grid(const GridArgs& a, int P, hipStream_t s) {
    HQ_LAUNCH(build_grid_kernel, dim3(a.G1 * a.G1 * a.G1, P), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_finalize(const FinalizeArgs& a, int P, hipStream_t s) {
    HQ_LAUNCH(finalize_kernel, dim3(P), dim3(1024), 0, s, a);
    return hipGetLastError();
}

}  // namespace hq

#ifdef HQ_GRID_TIMING
// diagnostic build only: the last build_grid launch's workgroup stamps
extern "C" int hq_debug_grid_stamps(unsigned long long* out, int n) {
    n = n < hq::kGridStamps ? n : hq::kGridStamps;
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(hq::g_grid_t), sizeof(unsigned long long) * 8 * (size_t)n);
}
#endif
