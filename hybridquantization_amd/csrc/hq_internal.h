// hq_internal.h -- structs shared by the HIP kernels (hq_kernels.hip) and the
// host runtime (hq_runtime.hip).  Not part of the public ABI (include/hq.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hq {

constexpr int kMaxK = 256;        // u8 palette indices (K <= 256 on the tiled path)
constexpr int kMaxKWide = 1 << 24;  // K > 256: 32-bit indices (the plugin's limit, HQ:192)
constexpr int kMaxKChunked = 16384;  // 256 < K <= 16384: palettes as 256-colour chunks, 16-bit indices
#ifndef HQ_MAX_NCH_FAST
#define HQ_MAX_NCH_FAST 32
#endif
constexpr int kMaxNchFast = HQ_MAX_NCH_FAST;  // chunked palettes of up to 32 chunks run the tiled cost kernel
// chunks of a palette of K colours on the chunked path: a power of two (2 .. 64)
inline int chunk_count(int K) {
    int n = 1;
    while (256 * n < K) n <<= 1;
    return n;
}
constexpr int kMaxTaps = 255;     // generic path limit (2*half+1)
constexpr int kNumFilt = 7;       // separable filter pairs of the S-CIELAB stencil
constexpr int kL1Cap = 31;        // level-1 candidate list capacity (32-B entry)
#ifndef HQ_L2B
#define HQ_L2B 8  // bytes per level-2 entry: 8 (count + 7 indices) or 16 (count + 15)
#endif
constexpr int kL2Bytes = HQ_L2B;
constexpr int kL2Cap = kL2Bytes - 1;  // level-2 candidate list capacity (stored)
constexpr int kL2Build = 15;          // list length build_grid tracks before pruning
constexpr int kL2Line = 4 * kL2Bytes;  // one cell's entries of a group of 4 palettes
constexpr uint8_t kOverflow = 255;

// The 7 separable (vertical, horizontal) filter pairs of the candidate stencil,
// CL:234-306 restated: channel 0 = k1.x (x) k1.x + k2.x (x) k2.x + |k3| (x) k3,
// channel 1 = k1.y (x) k1.y + k2.y (x) k2.y, channel 2 = k1.z (x) k1.z + k2.z (x) k2.z
// (vertical kernel first).  Filter f feeds opponent channel kFiltChan[f].
__host__ __device__ constexpr int filt_chan(int f) { return f < 3 ? 0 : (f < 5 ? 1 : 2); }

template <int T>
struct TapTable {
    float v[kNumFilt][T];  // vertical taps per filter
    float h[kNumFilt][T];  // horizontal taps per filter
};

// Geometry of one (possibly sharded) image on a device.
struct Geom {
    int W, H;        // full image
    int r0, r1;      // owned rows [r0, r1)
    int e0, e1;      // extended rows held on device [e0, e1) (owned +- half, clipped)
    int lab_pitch;   // floats per row of the planar LabRef (multiple of 4)
    int64_t n_ext;   // W * (e1 - e0)
    int64_t idx_pitch;  // bytes per palette in the index buffer (>= n_ext, multiple of 256)
};

struct PaletteArgs {
    const float4* pal_in;   // [P][K] host-uploaded palettes
    float4* pal;            // [P][256] sanitised colours (.w = 0)
    float4* opp;            // [P][256] opponent colour of each palette entry (CL:194-198)
    uint4* opp16;           // [P][256] its channels x 2^14 as (hi, lo) f16 pairs (split_f16), .w = 0
    uint8_t* dup;           // [P][256] 1 if an identical colour exists at a lower index
    int* pflags;            // [P] bit0: non-finite colour present -> exhaustive argmin
    int K;
};

constexpr int kSaMaxP = 64;        // device-resident SWASA: largest population
constexpr int kSaMaxSub = 512;     // ... and sub-palettes (P nch; sa_step's fold: 8 P nch used words <= 4 x 1024)
// Used-colour bits are kept in kUsedSlots copies, used_stride(P) words apart
// (256-B multiples): assign's workgroups OR theirs into copy blockIdx & 7, the
// readers OR the copies.  One copy took every workgroup's atomic at the end of
// the launch (C2, P = 1: 2048 workgroups on one 32-B word set, +14 us).
constexpr int kUsedSlots = 8;
// words per used-bit copy: P palettes x 8 words, rounded up to 64 words (256 B)
inline int used_stride(int P) { return (P * 8 + 63) / 64 * 64; }
// fixed-point dE sums (hq_device.h acc_add): slot counters per palette, and two
// sets used alternately by consecutive evaluations (a set is zeroed by the
// kernel before the evaluation's cost kernel, while the previous set is read)
constexpr int kAccSlots = 16;
// palettes per slot row, a multiple of 8: each slot's counters start a 256-B
// row of their own, so the slots' atomics spread over the memory channels
// rather than queueing on one (P = 1: sixteen 32-B slots shared 512 B)
__host__ __device__ constexpr int acc_pitch(int P) { return (P + 7) & ~7; }
inline size_t acc_words(int P) { return (size_t)kAccSlots * acc_pitch(P) * 4; }

// sa_step_kernel: one accept + generate step of the device-resident SWASA search.
struct SaArgs {
    const double* out;      // [P][1+K] finalize sums + used flags of the last evaluation
    const float* colors_in; // [P][4K] accepted palettes (ping)
    float* colors_out;      // (pong)
    const float* cand_in;   // [P][4K] candidates just evaluated
    float* cand_out;        // [P][4K] next candidates (generate)
    const double* err_in;   // [P] current errors
    double* err_out;
    const uint64_t* seed_in;  // java.util.Random state
    uint64_t* seed_out;
    const double* best_err_in;  // best error so far (ping-ponged like the state: the
    double* best_err_out;       // writer updates it while other workgroups read it)
    float* best_colors;     // [4K]
    const uint64_t* jump_A; // LCG jumps: n steps = A_n s + C_n mod 2^48, n = 0 .. 3K*P
    const uint64_t* jump_C;
    PaletteArgs prep;       // outputs of the palette prep of the next candidates
    // fold (no communicator, or a row-block split): the accept step reads the
    // fixed-point sums and the used bits itself, so no finalize launch sits
    // between the cost kernel and this step.  Row-block ranks: nranks blocks,
    // each rank's own, gathered by one RCCL all-gather (integer sums and OR'ed
    // bits: the same totals in any rank order).
    const uint64_t* acc;    // [nranks][kAccSlots][P][4] (acc_total), acc_rank_words apart
    const uint32_t* used_glob;  // [nranks][kUsedSlots][used_stride]: [P][8 nch] per slot
    int used_stride;
    int fold;
    int nranks;             // rank blocks of acc and used_glob (1 without a communicator)
    int64_t acc_rank_words;
    double n_total;         // pixels of the whole image
    double keep_threshold;  // SW:59-62 -(tanh(num/den))/2 + 0.5 at the accepted iteration
    float temperature;      // SW:54-57 temperature at the accepted iteration
    float amax;             // SW:91-101 max_step_width(ite) / 256 for the generated iteration
    float delta;            // SW:74-82 penalty per unused colour
    int P, K;
    int accept;             // 1: accept the evaluated population first
    int init;               // accept as IM:490-493 (initial population) instead
    int generate;           // 1: generate the next candidates (and prep them)
    int random;             // generate SW:40-52 random colours instead of neighbours
    int convergence;
    int nch;                // chunked palettes: chunks per palette (P nch workgroups), else 1
};

struct GridArgs {
    const float4* pal;
    const uint8_t* dup;
    const int* pflags;
    uint8_t* lvl1;          // [P][G1^3][32]
    uint8_t* lvl2;          // [ceil(P/4)][G2^3][4][kL2Bytes]: a group's 4 entries of a cell side by side
    uint32_t* used_glob;    // [kUsedSlots][used_stride] used-colour bits, zeroed here for the assign
    int used_stride;        // that follows
    int K;
    int G1;                 // level-1 resolution (G2 / 4)
    int64_t lvl1_pitch;     // bytes per palette
    int64_t lvl2_gstride;   // bytes per group of 4 palettes (G2^3 * kL2Line)
    uint64_t* acc_zero;     // the fixed-point sums the following cost kernel adds to, zeroed here
    int P_acc;              // their palettes (P above / nch)
    int nch;                // sub-palettes per palette (chunked palettes), else 1
};

// Native 16-bit candidate lists (hq_lists16.hip) for chunked palettes of 4 to
// 32 chunks (512 < K <= 8192): one grid over all K colours, level 1 at 16^3
// cells (u16 count + 127 or 255 indices), level 2 at 64^3 (u16 count + 15
// indices, 32 B); count kN16Ovf = overflow.
constexpr int kN16G2 = 64, kN16G1 = kN16G2 / 4, kN16G0 = kN16G1 / 4;
// Level-1 entries: 128 u16 (count + 127) up to K = 4096, 256 above (lists at
// K = 8192: mean ~66, a tail past 127); the buffer is sized for the larger.
constexpr int kN16L2Cap = 15, kN16L2Words = kN16L2Cap + 1;  // u16 per entry
constexpr int kN16L1WordsMax = 256;
__host__ __device__ constexpr int n16_l1_words(int K) { return K > 4096 ? 256 : 128; }
constexpr uint16_t kN16Ovf = 0xffff;
constexpr int kN16MinNch = 4;   // chunk counts that take the native lists (option "lists16") ...
constexpr int kN16MaxNch = 32;  // ... up to K = 8192: the palette's 128 KiB table in assign16's LDS
constexpr int kN16MaxK = 256 * kN16MaxNch;

struct Lists16Args {
    const float4* pal;      // [P][kpal] colours (the prepared sub-palettes, contiguous per palette)
    const int* pflags;      // [P nch] sub-palette flags (non-finite colour: exhaustive)
    uint16_t* lvl1;         // [P][16^3][n16_l1_words(K)]
    uint16_t* lvl2;         // [P][64^3][kN16L2Words]
    uint32_t* used_glob;    // [kUsedSlots][used_stride]: [P][8 nch] used-colour bits, zeroed here
    int used_stride;
    uint64_t* acc_zero;     // the fixed-point sums of the cost kernel that follows, zeroed here
    int P_acc;
    int K, kpal, nch;
};

struct AssignArgs {
    const float* R;         // planar, n_ext floats (extended rows)
    const float* G;
    const float* B;
    const uint32_t* rgbx;   // packed 8-bit R,G,B (byte 0..2) of an image whose channels are all
                            // k/255 (exactly, IM:100's int-RGB source), else null
    const float4* pal;      // [P][256]
    const int* pflags;
    const uint8_t* lvl1;
    const uint8_t* lvl2;
    uint8_t* idx;           // [P][idx_pitch]
    uint32_t* used_glob;    // [kUsedSlots][used_stride]: [P][8] used-colour bits per slot, every
    int used_stride;        // workgroup ORs its own into slot blockIdx & 7 (atomics)
    int64_t n_ext;
    int64_t idx_pitch;
    int64_t lvl1_pitch;     // bytes per palette
    int64_t lvl2_gstride;   // bytes per group of 4 palettes (G2^3 * kL2Line)
    int K;
    int G2;                 // 0 = exhaustive
    int nblocks;            // workgroups per palette group
    // chunked palettes (256 < K <= 4096): the P above are sub-palettes, nch per
    // palette (chunk_count), combined into 16-bit indices (hq_assign.hip)
    uint16_t* idx16;        // [P / nch][idx_pitch]
    float* dist;            // [P / nch][idx_pitch] best reference distance (nch > 4 passes)
    int nch = 1, lg_nch = 0;
    int gstep = 1;          // (set by the launcher)
    // native 16-bit lists (hq_lists16.hip): palette p's colours at pal + p kpal
    const uint16_t* l1n = nullptr;
    const uint16_t* l2n = nullptr;
    int kpal = 0;
};

struct CostArgs {
    const uint8_t* idx;     // [P][idx_pitch]
    const uint4* opp16;     // [P][256] split opponent table (PaletteArgs::opp16)
    const void* taps;       // CostTaps<10> x 2 in device memory (build_fast_taps)
    const uint4* vfrag16;   // [trim][4 stacks][hi, lo][64 lanes] f16x8 A fragments of the
                            // vertical taps (build_vpass_f16_stack_fragments; cost_mfma)
    const uint4* vfrag16p;  // [trim][u][4 stacks][hi, lo][64 lanes]: the same taps in the (hi, lo)
                            // pair layout of cost16w (build_vpass_f16_pair_fragments)
    const float* labL;      // planar LabRef, owned rows, pitch lab_pitch
    const float* labA;
    const float* labB;
    uint64_t* acc;          // fixed-point dE sums [kAccSlots][acc_P][4] (acc_add); this launch's
    int acc_P, acc_p0;      // palettes are acc_p0 .. (a group of a larger population: acc_p0 > 0)
    Geom g;
    int K;
    int tiles_x;
    int ntiles;      // tiles of the shard (partial pitch per palette)
    float m_lab[9];  // Opp->XYZ rows / illuminant (CL:124-131), opp2xyz_over_illum()
    float* pix_err;  // test option "pixel_err": [P][pix_pitch] per-pixel dE of the owned rows
    int64_t pix_pitch;  // (null: not written)
};

struct FinalizeArgs {
    const uint64_t* acc;    // fixed-point dE sums [kAccSlots][P][4]
    const uint32_t* used_glob;  // [kUsedSlots][used_stride] used-colour bits (assign)
    int used_stride;
    double* out;            // [P][1+K]
    int P;
    int K;
    const uint32_t* used32; // K > 4096: [P][K] used flags (assign_wide), replaces used_mask
    int wpp;                // used words per palette in used_glob (8; 8 nch for chunked palettes)
};

// Palettes of K > 256 colours (hq_wide.hip).
struct WideArgs {
    const float4* pal_in;   // [P][K] host-uploaded palettes
    float4* pal;            // [P][K] .w = 0
    float4* opp;            // [P][K] opponent colours (CL:194-198)
    int* pflags;            // [P] bit 0: non-finite colour (zeroed before prep)
    const float* R;         // planar extended rows
    const float* G;
    const float* B;
    uint32_t* idx32;        // [P][idx_pitch] 32-bit palette indices
    uint32_t* used32;       // [P][K] used flags (zeroed before assign)
    int64_t n_ext;
    int64_t idx_pitch;      // elements per palette
    int K;
};

// Generic two-pass path (any half-width), one palette per launch.
struct GenArgs {
    const void* idx;         // palette's index image (extended rows): u8, or u32 for K > 256
    const float4* opp;       // palette's opponent table [max(K, 256)]
    const float* k1;         // [T][4]
    const float* k2;         // [T][4]
    const float* k3;         // [T]
    const float* absk3;      // [T]
    float* t;                // [7][n_ext] horizontal results (t1.xyz, t2.xyz, t3)
    const float* labL;
    const float* labA;
    const float* labB;
    uint64_t* acc;           // fixed-point dE sums [kAccSlots][P][4] (acc_add), palette p
    int p, P;
    Geom g;
    int half;
    float m_lab[9];  // Opp->XYZ rows / illuminant (CL:124-131), opp2xyz_over_illum()
    float* pix_err;  // this palette's per-pixel dE of the owned rows (test option), or null
    const float* vtaps;  // tiled path: [7][vtap_pitch] vertical taps per plane, zero-padded
    int vtap_pitch;      // (2 half + 1 rounded up to 16, + 16)
    int hrow4 = 1;       // tiled path: horizontal pass with 4 outputs per thread (gen_hrow4), else gen_hrow
    int hrow_no = 4;     // gen_hrow4's outputs per thread: 4 or 8
    int vtile2 = 1;      // tiled path: double-buffered LDS-DMA vertical pass (gen_vtile2), else gen_vtile
    int vmfma = 1;       // tiled path: the vertical pass on the matrix cores (gen_vmfma, split f16)
    const uint32_t* vtapd = nullptr;  // its duplicated split taps [7][hi, lo][16 S + 16] (build_vtile_dup_taps)
    int hmfma = 1;       // with vmfma: the horizontal pass on the matrix cores too (gen_hmfma)
    int shape = 0;       // matrix-core pair's tile shapes: 0 by grid size, 1 the short forms, 2 the tall ones
    const uint32_t* htapd = nullptr;  // its taps, the same layout (k3 signed: the horizontal t3 taps)
    const float4* htaps = nullptr;  // gen_hrow4: [T][2] (k1.xyz, k3), (k2.xyz, 0) horizontal taps
};

}  // namespace hq
