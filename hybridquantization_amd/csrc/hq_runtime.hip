// hq_runtime.hip -- libhq host runtime: the C ABI of include/hq.h.
//
// One hq_ctx = one GPU, one HIP stream (the reference's single in-order queue,
// IM:58-59), the device-resident image of IM:450-478 (planar RGB of the owned
// rows +- halo, planar LabRef of the owned rows), per-population work buffers,
// and optionally an RCCL communicator for row-block sharding.
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "hq_internal.h"
#include "hq_swasa.h"

#ifndef HQ_COST_TW
#define HQ_COST_TW 128
#endif
#ifndef HQ_SA_GRAPH
#define HQ_SA_GRAPH 0  // (measured slower: C3 0.528 -> 0.540 ms, shard-of-8 0.1035 -> 0.110 ms per step)
#endif

namespace hq {
// launchers from hq_kernels.hip
hipError_t launch_prep_palette(const PaletteArgs&, int P, hipStream_t);
hipError_t launch_sa_step(const SaArgs&, hipStream_t);
void set_launch_events(hipEvent_t start, hipEvent_t stop);
hipError_t launch_build_grid(const GridArgs&, int P, hipStream_t);
hipError_t launch_assign(const AssignArgs&, int P, hipStream_t);
hipError_t launch_lists16_grid(const Lists16Args&, int P, hipStream_t);
hipError_t launch_assign16(const AssignArgs&, int P, hipStream_t);
int assign_residency(int NG);
int assign_residency_chunked();
hipError_t launch_cost_chunked(const CostArgs&, int P, int nch, int de, bool trim, hipStream_t);
void fast_tile_dims(int W, int own_rows, int tile_rows, int tile_w, int* tiles_x, int* ntiles);
void opp2xyz_over_illum(const float inv_illum[3], float m[9]);
hipError_t launch_cost_fast(const CostArgs&, int P, int de, bool trim, int tile_rows, int tile_w, int HB,
                            hipStream_t);
int fast_bucket(int half);
size_t vpass_f16_stack_fragment_halves(int HB);
void build_vpass_f16_pair_fragments(int HB, int H, const float* k1, const float* k2, const float* k3,
                                    const float* absk3, uint16_t* out);
size_t vpass_f16_pair_fragment_halves(int HB);
size_t vtile_dup_tap_words(int H);
void build_vtile_dup_taps(int H, const float* k1, const float* k2, const float* absk3, uint32_t* out);
void build_vpass_f16_stack_fragments(int HB, int H, const float* k1, const float* k2, const float* k3,
                                     const float* absk3, uint16_t* out);
size_t fast_taps_bytes(int HB);
void build_fast_taps(int HB, int H, const float* k1, const float* k2, const float* k3, const float* absk3,
                     void* out);
bool trim_window_ok(const float* k1, int H, int HB);

hipError_t launch_cost_generic(const GenArgs&, int de, int idx_bytes, hipStream_t);
hipError_t launch_cost_tiled_generic(const GenArgs&, int de, int idx_bytes, hipStream_t);
hipError_t launch_prep_wide(const WideArgs&, int P, hipStream_t);
hipError_t launch_assign_wide(const WideArgs&, int P, hipStream_t);
hipError_t launch_finalize(const FinalizeArgs&, int P, hipStream_t);
hipError_t launch_pack_u8(const float*, const float*, const float*, uint32_t*, int*, int64_t, hipStream_t);
hipError_t launch_labref_opp(const float*, const float*, const float*, float4*, int64_t, hipStream_t);
hipError_t launch_xyz_to_opp(const float4*, float4*, int64_t, hipStream_t);
hipError_t launch_rgb_to_xyz(const float*, const float*, const float*, float4*, int64_t, hipStream_t);
hipError_t launch_labref_hconv(const float4*, float4*, const float*, int, int, int, int64_t, hipStream_t);
hipError_t launch_labref_vconv(const float4*, float4*, const float*, int, int, int, const Geom&, hipStream_t);
hipError_t launch_labref_lab(const float4*, float*, float*, float*, float4*, int, int64_t, int,
                             const float*, hipStream_t);
hipError_t launch_lab_to_planar(const float4*, float*, float*, float*, int, int64_t, int, hipStream_t);
hipError_t launch_quantize(const float4*, const float4*, int, int*, float4*, int64_t, hipStream_t);
hipError_t launch_error_image(const float4*, const float4*, float4*, double*, int64_t, int, hipStream_t);
}  // namespace hq

using namespace hq;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t n) {
        if (n <= bytes) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <typename T>
    T* as() const { return static_cast<T*>(p); }
};

struct ProfSlot {
    double ms = 0.0;
    int64_t launches = 0;
};

// Profiling events per evaluation / search iteration: start, stop of grid (0,
// 1), assign (2, 3), cost (4, 5), finalize (6, 7), sa_step (8, 9) and the
// collective (10, 11).
constexpr int kProfEvents = 12;

}  // namespace

struct hq_ctx {
    int device = 0;
    int de_type = HQ_DE_CIE76;
    hipStream_t stream = nullptr;
    std::string err;

    // filters (IM:800-841)
    int taps = 0, half = 0;
    std::vector<float> k1, k2, k3, absk3;
    DevBuf d_k1, d_k2, d_k3, d_absk3;
    DevBuf d_vtaps;    // tiled generic path: [7][vtap_pitch] vertical taps per plane, zero-padded
    int vtap_pitch = 0;
    int fast_hb = 0;   // fast path tap bucket (fast_bucket(half)); 0 = generic path only
    DevBuf d_taps;     // fast path taps, build_fast_taps (the filters centred in the bucket)
    DevBuf d_vfrag16;  // split-f16 MFMA A fragments of the stacked vertical taps
    DevBuf d_vfrag16p; // the same in cost16w's (hi, lo) pair layout
    DevBuf d_vfragm;   // the tiled generic path's matrix-core vertical taps (build_vtile_dup_taps)
    DevBuf d_htaps;    // gen_hrow4's packed horizontal taps [T][2] float4

    // image
    bool have_image = false;
    Geom g{};
    float illum[3] = {0.95047f, 1.0f, 1.0883f};
    DevBuf d_R, d_G, d_B;          // planar, extended rows (n_ext, padded to 4)
    DevBuf d_rgbx;                 // packed 8-bit copy of R,G,B when every channel is k/255
    bool img_u8 = false;
    DevBuf d_labL, d_labA, d_labB;  // planar LabRef, owned rows, lab_pitch

    // population work buffers
    int P_cap = 0, K_cur = 0;
    DevBuf d_pal_in, d_pal, d_opp, d_opp16, d_dup, d_pflags, d_lvl1, d_lvl2, d_idx, d_used_mask,
        d_acc, d_out, d_gen_t;
    // d_acc: two sets of fixed-point dE sums [kAccSlots][P][4] u64 (acc_add), d_used_mask two
    // sets of used bits [kUsedSlots][used_stride]; evaluation n fills set acc_par = n & 1
    int acc_par = 0;
    DevBuf d_pixerr;           // option "pixel_err": [P][n_own] per-pixel dE of the last evaluation
    DevBuf d_idx32, d_used32;  // K > 16384 (hq_wide.hip): 32-bit index images, per-colour used flags
    DevBuf d_idx16, d_dist;    // 256 < K <= 16384 (chunked): 16-bit index images, pass distances
    DevBuf d_l1n, d_l2n;       // the native 16-bit candidate lists (hq_lists16.hip)
    int nch_cur = 1;           // chunks per palette of the population being enqueued (1: K <= 256)
    int last_nch = 1;          // ... of the last evaluation (its index image: u16 when > 1)
    float* h_pal = nullptr;   // pinned [P][K][4]
    double* h_out = nullptr;  // pinned [P][1+K]
    size_t h_pal_bytes = 0, h_out_bytes = 0;
    int last_P = 0;

    // options
    int G2 = 32;           // argmin grid resolution (0 = exhaustive)
    int cost_variant = 0;  // 0 fast tiled (default), 1 generic two-pass (LDS-tiled), 2 the generic
                           // pair per pixel in the reference's summation order
    int cost_rows = 16;    // fast path tiles: 16 x 128 (cost16w_kernel) or 8 x 108 (cost_mfma_kernel)
    int cost_tw = HQ_COST_TW;  // 16-row tiles at HB = 10: 128 (4 waves) or 256 columns (8 waves; slower)
    int gen_hrow4 = 1;     // tiled generic path: 4 outputs per thread in the horizontal pass
    int gen_vtile2 = 1;    // tiled generic path: double-buffered LDS-DMA vertical pass (half <= 64)
    int gen_vmfma = 1;     // tiled generic path: the vertical pass on the matrix cores (half <= 64)
    int gen_hmfma = 1;     // ... and the horizontal pass (gen_hmfma) with it
    int gen_shape = 0;     // their tile shapes: 0 by grid size, 1 short, 2 tall (option gen_tile_shape)
    int gen_hrow_no = 4;   // tiled generic path: horizontal outputs per thread (4 or 8)
    int sa_graph = HQ_SA_GRAPH;  // device-resident search: each run's kernels as one hipGraph
    int assign_blocks_per_cu = 0;  // 0 = auto: assign_pipe_kernel<NG>'s residency (the occupancy
                                   // query, assign_res[NG]), one round of workgroups, each
                                   // thread a grid-stride pixel sequence
    int assign_res[5] = {};   // [NG]
    int assign_res_chunked = 0;  // the chunk-combining forms (NG = 4)
    int psplit = 0;        // with a communicator of N ranks and the whole image on every rank: rank r
                           // evaluates palettes [r P/N, (r+1) P/N), then one all-gather (option
                           // "palette_split"; SURVEY 8e's split of large populations)
    int slice_ranks = 1, slice_rank = 0;  // test only: the same slice without a communicator
    int slice_lo = 0, slice_n = 0;        // the last evaluation's palettes held on this device
    int fold_blocks = 1, fold_block = 0;  // test only: rank blocks of the counters without a communicator
    int lists16 = 1;       // native 16-bit candidate lists: 1 = chunked palettes of 4 to 32 chunks, 2 = 2 .. 32
    int chunked = 1;       // 256 < K <= 16384: palettes as 256-colour chunks through the grid and
                           // tiled kernels (option "chunked"; 0 = the exhaustive K > 256 path)
    int img_u8_path = 1;   // assign reads the packed 8-bit image when there is one (option 'img_u8')
    int shard_solo = 0;    // experiment: a sharded search without a communicator (per-rank timing)
    int sa_device = 1;     // hq_search_*: 1 = SWASA iterations resident on the device (no host
                           // round trip per iteration), 0 = host-driven (one eval call each)
    int pixel_err = 0;     // test option: the cost kernels also write the per-pixel dE
    int trim = 1;          // skip taps < 1e-9 of the peak of the narrow k1 filters
    bool trim_ok = false;  // set by hq_set_filters (the bucket's narrow-filter windows hold)
    bool pal_generic = false;  // this population needs the generic cost path (palette_fits_fast)

    // comm
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;

    // profiling
    bool prof = false;
    ProfSlot prof_assign, prof_cost, prof_grid, prof_finalize, prof_sa, prof_comm;
    // profiling: start/stop of grid, assign, cost, finalize, [sa_step], the collective
    hipEvent_t ev[kProfEvents] = {};
    int num_cu = 256;
    size_t lds_optin = 160 * 1024;  // per-workgroup LDS a kernel may opt into (hq_create's query)
};

struct hq_search {
    hq_ctx* ctx;
    SearchDriver* driver;  // host-driven search (sa_device = 0), else null
    int K;
    // device-resident search: the SWASA state lives on the device, ping-ponged
    // between [0] and [1] by sa_step_kernel; the host keeps the iteration-only
    // quantities (temperature, step width, convergence threshold) in `pol`,
    // whose RNG is unused.
    Swasa* pol = nullptr;
    hq_swasa_params prm{};
    int P = 0, ite = 0, st = 0, cd = 0;  // state and candidate buffer parities
    int nch = 1;                         // chunked palettes (256 < K <= 16384): chunks per palette
    bool fold = false;                   // accept steps reduce the partials (no finalize launch)
    ncclComm_t comm = nullptr;           // the context's communicator at hq_search_create
    float t_acc = 0.f;                   // temperature / threshold of the iteration
    double keep_acc = 0.0;               // whose population awaits acceptance
    DevBuf colors[2], cand[2], err[2], seed[2], best_err[2], best_colors, jA, jC;
    std::vector<hipEvent_t> pev;         // profiling: 8 events per iteration of a run
    hipGraphExec_t gexec = nullptr;      // option sa_graph: the last run's iteration chain
    int gexec_iters = 0;                 // (its iteration count: the topology an update must match)
};

namespace {

int fail(hq_ctx* c, int code, const char* fmt, ...) {
    if (c) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        c->err = buf;
    }
    return code;
}

#define HIP_TRY(ctx, expr)                                                                      \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess)                                                                   \
            return fail((ctx), _e == hipErrorOutOfMemory ? HQ_ERR_NOMEM : HQ_ERR_DEVICE,        \
                        "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, __LINE__); \
    } while (0)

#define NCCL_TRY(ctx, expr)                                                                     \
    do {                                                                                        \
        ncclResult_t _r = (expr);                                                               \
        if (_r != ncclSuccess)                                                                  \
            return fail((ctx), HQ_ERR_COMM, "%s failed: %s", #expr, ncclGetErrorString(_r));    \
    } while (0)

inline int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

int bind(hq_ctx* c) {
    HIP_TRY(c, hipSetDevice(c->device));
    return HQ_OK;
}

// Geometry of the shard [r0, r1) of a (W x H) image with halo `half`.
Geom make_geom(int W, int H, int r0, int r1, int half) {
    Geom g{};
    g.W = W;
    g.H = H;
    g.r0 = r0;
    g.r1 = r1;
    g.e0 = std::max(0, r0 - half);
    g.e1 = std::min(H, r1 + half);
    g.lab_pitch = (int)round_up(W, 4);
    g.n_ext = (int64_t)W * (g.e1 - g.e0);
    g.idx_pitch = round_up(g.n_ext + 4, 256);
    return g;
}

int ensure_pinned(hq_ctx* c, size_t pal_bytes, size_t out_bytes) {
    if (pal_bytes > c->h_pal_bytes) {
        if (c->h_pal) (void)hipHostFree(c->h_pal);
        c->h_pal = nullptr;
        HIP_TRY(c, hipHostMalloc((void**)&c->h_pal, pal_bytes, hipHostMallocDefault));
        c->h_pal_bytes = pal_bytes;
    }
    if (out_bytes > c->h_out_bytes) {
        if (c->h_out) (void)hipHostFree(c->h_out);
        c->h_out = nullptr;
        HIP_TRY(c, hipHostMalloc((void**)&c->h_out, out_bytes, hipHostMallocDefault));
        c->h_out_bytes = out_bytes;
    }
    return HQ_OK;
}

// Upload one plane of the extended rows from a full-image host source with
// stride `sstride` floats between pixels and channel offset `ch`.
void gather_rows(const float* src, int sstride, int ch, const Geom& g, std::vector<float>& dst) {
    dst.assign((size_t)round_up(g.n_ext, 4), 0.0f);
    const int64_t base = (int64_t)g.e0 * g.W;
    for (int64_t i = 0; i < g.n_ext; ++i) dst[i] = src[(base + i) * sstride + ch];
}

int compute_labref_device(hq_ctx* c) {
    // IM:100 RGBtoXYZ + IM:285-370 XYZtoScielab on the extended rows.
    const Geom& g = c->g;
    const int64_t n_own = (int64_t)g.W * (g.r1 - g.r0);
    DevBuf opp, tmp, conv, k3v, ak3v;
    HIP_TRY(c, opp.ensure(sizeof(float4) * g.n_ext));
    HIP_TRY(c, tmp.ensure(sizeof(float4) * g.n_ext));
    HIP_TRY(c, conv.ensure(sizeof(float4) * std::max<int64_t>(n_own, 1)));
    std::vector<float> k3h(4 * c->taps, 0.f), ak3h(4 * c->taps, 0.f);
    for (int t = 0; t < c->taps; ++t) { k3h[4 * t] = c->k3[t]; ak3h[4 * t] = c->absk3[t]; }
    HIP_TRY(c, k3v.ensure(sizeof(float) * k3h.size()));
    HIP_TRY(c, ak3v.ensure(sizeof(float) * ak3h.size()));
    HIP_TRY(c, hipMemcpyAsync(k3v.p, k3h.data(), sizeof(float) * k3h.size(), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(ak3v.p, ak3h.data(), sizeof(float) * ak3h.size(), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, launch_labref_opp(c->d_R.as<float>(), c->d_G.as<float>(), c->d_B.as<float>(),
                                 opp.as<float4>(), g.n_ext, c->stream));
    // IM:319-346 filter by filter: H then V (update for filters 2 and 3)
    const float* hk[3] = {c->d_k1.as<float>(), c->d_k2.as<float>(), k3v.as<float>()};
    const float* vk[3] = {c->d_k1.as<float>(), c->d_k2.as<float>(), ak3v.as<float>()};
    for (int f = 0; f < 3; ++f) {
        const int chans = f < 2 ? 3 : 1;
        HIP_TRY(c, launch_labref_hconv(opp.as<float4>(), tmp.as<float4>(), hk[f], c->half, chans,
                                       g.W, g.n_ext, c->stream));
        HIP_TRY(c, launch_labref_vconv(tmp.as<float4>(), conv.as<float4>(), vk[f], c->half, chans,
                                       f > 0, g, c->stream));
    }
    HIP_TRY(c, launch_labref_lab(conv.as<float4>(), c->d_labL.as<float>(), c->d_labA.as<float>(),
                                 c->d_labB.as<float>(), nullptr, g.W, n_own, g.lab_pitch, c->illum,
                                 c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    opp.release(); tmp.release(); conv.release(); k3v.release(); ak3v.release();
    return HQ_OK;
}

int set_image_common(hq_ctx* c, const std::vector<float>& R, const std::vector<float>& G,
                     const std::vector<float>& B, const float* lab4_full, const float* illum) {
    const Geom& g = c->g;
    const size_t plane = sizeof(float) * (size_t)round_up(g.n_ext, 4);
    HIP_TRY(c, c->d_R.ensure(plane));
    HIP_TRY(c, c->d_G.ensure(plane));
    HIP_TRY(c, c->d_B.ensure(plane));
    HIP_TRY(c, hipMemcpyAsync(c->d_R.p, R.data(), plane, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->d_G.p, G.data(), plane, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->d_B.p, B.data(), plane, hipMemcpyHostToDevice, c->stream));
    // An image whose channels are all exactly k/255 (the reference's int-RGB
    // source, IM:100) is also kept as packed bytes: assign reads 4 B per pixel
    // instead of 12 and rebuilds k/255 exactly (u8_unit).  The check and the
    // packing run on the device (pack_u8_kernel); only a 4-byte flag returns.
    {
        HIP_TRY(c, c->d_rgbx.ensure(sizeof(uint32_t) * (size_t)round_up(g.n_ext, 4)));
        DevBuf flag;
        HIP_TRY(c, flag.ensure(sizeof(int)));
        HIP_TRY(c, hipMemsetAsync(flag.p, 0, sizeof(int), c->stream));
        HIP_TRY(c, launch_pack_u8(c->d_R.as<float>(), c->d_G.as<float>(), c->d_B.as<float>(),
                                  c->d_rgbx.as<uint32_t>(), flag.as<int>(), g.n_ext, c->stream));
        int not_u8 = 1;
        HIP_TRY(c, hipMemcpyAsync(&not_u8, flag.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        flag.release();
        c->img_u8 = not_u8 == 0;
        if (!c->img_u8) c->d_rgbx.release();
    }
    if (illum) std::memcpy(c->illum, illum, sizeof c->illum);
    const int own = g.r1 - g.r0;
    const size_t lplane = sizeof(float) * (size_t)g.lab_pitch * std::max(own, 1);
    HIP_TRY(c, c->d_labL.ensure(lplane));
    HIP_TRY(c, c->d_labA.ensure(lplane));
    HIP_TRY(c, c->d_labB.ensure(lplane));
    HIP_TRY(c, hipMemsetAsync(c->d_labL.p, 0, lplane, c->stream));
    HIP_TRY(c, hipMemsetAsync(c->d_labA.p, 0, lplane, c->stream));
    HIP_TRY(c, hipMemsetAsync(c->d_labB.p, 0, lplane, c->stream));
    if (lab4_full) {
        const int64_t n_own = (int64_t)g.W * own;
        DevBuf tmp;
        HIP_TRY(c, tmp.ensure(sizeof(float4) * n_own));
        HIP_TRY(c, hipMemcpyAsync(tmp.p, lab4_full + (int64_t)g.r0 * g.W * 4, sizeof(float4) * n_own,
                                  hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, launch_lab_to_planar(tmp.as<float4>(), c->d_labL.as<float>(), c->d_labA.as<float>(),
                                        c->d_labB.as<float>(), g.W, n_own, g.lab_pitch, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        tmp.release();
    } else {
        int rc = compute_labref_device(c);
        if (rc) return rc;
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->have_image = true;
    return HQ_OK;
}

int check_geom_args(hq_ctx* c, int w, int h, int r0, int r1) {
    if (!c->taps) return fail(c, HQ_ERR_STATE, "filters not set (call hq_set_filters first)");
    if (w < c->half || h < c->half || w < 1 || h < 1)
        return fail(c, HQ_ERR_ARG, "image %dx%d smaller than the stencil half-width %d", w, h, c->half);
    if (r0 < 0 || r1 > h || r0 >= r1) return fail(c, HQ_ERR_ARG, "bad row range [%d,%d)", r0, r1);
    // the cost kernels address a shard's index image and its fp32 LabRef planes with
    // 32-bit unsigned byte offsets: keep 4 bytes per (padded) pixel below 2^32
    if ((int64_t)(w + 4) * (int64_t)(r1 - r0 + 2 * c->half) >= ((int64_t)1 << 30))
        return fail(c, HQ_ERR_UNSUPPORTED, "shard of %d x %d pixels exceeds 2^30; use more row blocks",
                    w, r1 - r0);
    return HQ_OK;
}

// Assign workgroups per palette group: assign_blocks_per_cu per CU, but no more
// than pixel chunks (256 pixels, one per thread): idle workgroups still fill LDS,
// and after the XCD relabelling they would all sit on the last XCDs (a 512-row
// shard ran assign on half the chip: 0.071 vs 0.053 ms).  (Evening out the
// chunks per workgroup instead -- 1064 workgroups of 2 for 2128 chunks -- was
// slower than 2048 with 80 of them taking a second chunk.)
// assign: one pixel per thread per 256-thread chunk, with one resident round
// of workgroups, makes each thread's pixel sequence a grid stride: every thread
// gets the same number of pixels +-1 (512-row shard 0.1306 -> 0.1261 ms per
// step vs 4 pixels per chunk at 16 workgroups per CU; 4096^2 unchanged).
#ifndef HQ_ASSIGN_MINPX
#define HQ_ASSIGN_MINPX 6
#endif
int assign_blocks(const hq_ctx* c, int P) {
    // at least HQ_ASSIGN_MINPX pixels per thread: a launch's fixed part (table
    // fill, pipeline start, the used-bit flush) is paid per workgroup (C2,
    // 1024^2 P = 1: 2048 workgroups of 2 pixels per thread took 14 us, 1045 of 4
    // took 12.3, 523 of 8 took 8.5; the 512-row shard, 5.5 per thread at 1536
    // workgroups, slowed from 43 to 46 us at 8)
    const int64_t chunk = 256 * HQ_ASSIGN_MINPX;
    const int ng = std::min(P, 4);
    const int res = c->nch_cur > 1 ? c->assign_res_chunked : c->assign_res[ng];
    const int per_cu = c->assign_blocks_per_cu > 0 ? c->assign_blocks_per_cu : res > 0 ? res : 4;
    const int64_t nblocks = (int64_t)c->num_cu * per_cu;
    return (int)std::max<int64_t>(1, std::min<int64_t>(nblocks, (c->g.n_ext + chunk - 1) / chunk));
}

// A row-block split (a communicator, no palette split) keeps one block of
// counters and used bits per rank in each set, [ranks][...]: every rank fills
// its own block, and a device-resident search's one all-gather per iteration
// hands every rank all the blocks, which its accept step folds (no finalize).
// (test options fold_blocks / fold_block: the same layout without a communicator,
// this context filling block fold_block and the others staying zero)
int rank_blocks(const hq_ctx* c) { return c->comm ? (c->psplit ? 1 : c->nranks) : c->fold_blocks; }
int own_block(const hq_ctx* c) { return c->comm ? (rank_blocks(c) > 1 ? c->rank : 0) : c->fold_block; }
// A device-resident search folds the partials in its accept step unless the
// palette split all-gathers finalized rows.
bool search_folds(const hq_ctx* c) { return !(c->comm && c->psplit); }

// Chunked palettes of 4 to 32 chunks take the native 16-bit lists (option lists16).
// Their kernels take up to 144 KiB (lists16_kernel at K = 8192) and 128 KiB
// (assign16_kernel) of dynamic LDS: a device that cannot grant that (less than
// gfx950's 160 KiB per workgroup) keeps the per-chunk grids.
bool use_lists16(const hq_ctx* c) {
    const int min_nch = c->lists16 >= 2 ? 2 : kN16MinNch;  // (2: also 2 and 4 chunks)
    if (!(c->lists16 > 0 && c->G2 > 0 && c->nch_cur >= min_nch && c->nch_cur <= kN16MaxNch)) return false;
    const size_t K = (size_t)kMaxK * c->nch_cur;
    const size_t grid_lds = ((K > 4096 ? 3 : 4) * sizeof(float) + sizeof(uint16_t)) * K +
                            sizeof(uint16_t) * 64 * n16_l1_words((int)K);
    const size_t assign_lds = sizeof(float4) * K * (K <= 4096 ? 2 : 1);
    return std::max(grid_lds, assign_lds) <= c->lds_optin;
}

// The population being enqueued takes the fast tiled cost kernels (else the
// generic pair, whose [7][n_ext] scratch ensure_population then allocates up
// front: nothing may allocate while a search run is captured into a graph).
// Chunked palettes: the 16 x 128 tiles at HB = 10 only.
bool cost_fast(const hq_ctx* c) {
    return c->cost_variant == 0 && c->fast_hb > 0 && !c->pal_generic &&
           (c->nch_cur == 1 || (c->nch_cur <= kMaxNchFast && c->fast_hb == 10 && c->cost_rows == 16 &&
                                c->cost_tw == 128));
}

// Ensure population buffers for P palettes of K colours.
int ensure_population(hq_ctx* c, int P, int K) {
    const Geom& g = c->g;
    if (c->nch_cur > 1) {  // chunked palettes: 16-bit indices, then P nch sub-palettes of 256
        HIP_TRY(c, c->d_idx16.ensure(sizeof(uint16_t) * (size_t)P * g.idx_pitch + 256));
        if (c->nch_cur > 4) HIP_TRY(c, c->d_dist.ensure(sizeof(float) * (size_t)P * g.idx_pitch));
        if (use_lists16(c)) {
            HIP_TRY(c, c->d_l1n.ensure(sizeof(uint16_t) * n16_l1_words(K) * (size_t)P * kN16G1 * kN16G1 * kN16G1));
            // (palette pairs interleaved: an odd population's last pair half empty)
            HIP_TRY(c, c->d_l2n.ensure(sizeof(uint16_t) * kN16L2Words * (size_t)(P + 1) / 2 * 2 * kN16G2 * kN16G2 * kN16G2));
        }
        P *= c->nch_cur;  // (d_out, h_out: P nch (1 + 256) >= P (1 + K) doubles)
        K = kMaxK;
    }
    const int G2 = c->G2 > 0 ? c->G2 : 4;
    const int G1 = G2 / 4;
    const int64_t l1p = round_up((int64_t)G1 * G1 * G1 * 32, 256);
    const int64_t l2g = round_up((int64_t)G2 * G2 * G2 * kL2Line, 256);  // per group of 4 palettes
    const int64_t n_own = (int64_t)g.W * (g.r1 - g.r0);
    HIP_TRY(c, c->d_pal_in.ensure(sizeof(float4) * (size_t)P * K));
    HIP_TRY(c, c->d_pal.ensure(sizeof(float4) * (size_t)P * std::max(K, kMaxK)));
    HIP_TRY(c, c->d_opp.ensure(sizeof(float4) * (size_t)P * std::max(K, kMaxK)));
    if (K > kMaxK) {
        HIP_TRY(c, c->d_idx32.ensure(sizeof(uint32_t) * (size_t)P * g.idx_pitch));
        HIP_TRY(c, c->d_used32.ensure(sizeof(uint32_t) * (size_t)P * K));
    }
    HIP_TRY(c, c->d_opp16.ensure(sizeof(uint4) * (size_t)P * kMaxK));
    HIP_TRY(c, c->d_dup.ensure((size_t)P * kMaxK));
    HIP_TRY(c, c->d_pflags.ensure(sizeof(int) * (size_t)P));
    HIP_TRY(c, c->d_lvl1.ensure((size_t)P * l1p));
    HIP_TRY(c, c->d_lvl2.ensure((size_t)((P + 3) / 4) * l2g));
    // + 256: the cost kernels' interior fills read whole dword pairs, up to 7
    // bytes past a region's last column (past the buffer on the last palette's
    // last row when idx_pitch has no padding)
    HIP_TRY(c, c->d_idx.ensure((size_t)P * g.idx_pitch + 256));
    const size_t rb = (size_t)rank_blocks(c);  // counter / used-bit blocks per set
    HIP_TRY(c, c->d_used_mask.ensure(2 * rb * sizeof(uint32_t) * kUsedSlots * (size_t)used_stride(P)));
    HIP_TRY(c, c->d_acc.ensure(2 * rb * sizeof(uint64_t) * acc_words(P)));
    HIP_TRY(c, c->d_out.ensure(sizeof(double) * (size_t)P * (1 + K)));
    if (c->pixel_err) HIP_TRY(c, c->d_pixerr.ensure(sizeof(float) * (size_t)P * std::max<int64_t>(n_own, 1)));
    // the generic path's [7][n_ext] scratch, here rather than at its first launch: an
    // allocation cannot happen while a search run is being captured into a graph
    if (!cost_fast(c) || K > kMaxK) HIP_TRY(c, c->d_gen_t.ensure(sizeof(float) * 7 * (size_t)g.n_ext + 256));
    return ensure_pinned(c, sizeof(float) * 4 * (size_t)P * K, sizeof(double) * (size_t)P * (1 + K));
}

void prof_add(hq_ctx* c, ProfSlot& s, hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) == hipSuccess) {
        s.ms += ms;
        s.launches += 1;
    } else {
        (void)hipGetLastError();  // an event pair this evaluation never recorded: not a launch error
    }
}

PaletteArgs prep_args(hq_ctx* c, int K) {
    return PaletteArgs{c->d_pal_in.as<float4>(), c->d_pal.as<float4>(), c->d_opp.as<float4>(),
                       c->d_opp16.as<uint4>(), c->d_dup.as<uint8_t>(), c->d_pflags.as<int>(), K};
}

// Enqueue the evaluation of the P prepared palettes (d_pal, d_opp, d_dup,
// d_pflags): grid, assign, cost, finalize into d_out (partial sums + used
// flags), all-reduced if a comm is set.  ev (8 events, or null): start/stop of
// the grid, assign, cost and finalize launches, carried by the launches
// themselves (set_launch_events).
// Counter set `par` of an evaluation of P palettes (P nch sub-palettes Ps).
uint64_t* acc_base(hq_ctx* c, int par, int P) {
    return c->d_acc.as<uint64_t>() + (size_t)par * rank_blocks(c) * acc_words(P);
}
uint32_t* used_base(hq_ctx* c, int par, int Ps) {
    return c->d_used_mask.as<uint32_t>() + (size_t)par * rank_blocks(c) * kUsedSlots * used_stride(Ps);
}
uint64_t* acc_set(hq_ctx* c, int par, int P) { return acc_base(c, par, P) + (size_t)own_block(c) * acc_words(P); }
uint32_t* used_set(hq_ctx* c, int par, int Ps) {
    return used_base(c, par, Ps) + (size_t)own_block(c) * kUsedSlots * used_stride(Ps);
}

GridArgs grid_args(hq_ctx* c, int P, int K, int so = 0) {
    const int G2 = c->G2 > 0 ? c->G2 : 4;
    const int G1 = G2 / 4;
    // (P = sub-palettes; the counters of set c->acc_par)
    const int nch = c->nch_cur;
    // (so: the first of the P sub-palettes in the prepared tables, a palette split's slice)
    return GridArgs{c->d_pal.as<float4>() + (int64_t)so * kMaxK, c->d_dup.as<uint8_t>() + (int64_t)so * kMaxK,
                    c->d_pflags.as<int>() + so, c->d_lvl1.as<uint8_t>(), c->d_lvl2.as<uint8_t>(),
                    used_set(c, c->acc_par, P),
                    used_stride(P), K, G1,
                    round_up((int64_t)G1 * G1 * G1 * 32, 256), round_up((int64_t)G2 * G2 * G2 * kL2Line, 256),
                    acc_set(c, c->acc_par, P / nch), P / nch, nch};
}

// The generic two-pass cost (CL:234-306 per pixel, any half-width) of P
// palettes, one launch pair each: index images at idx_base (u8, or u32 when
// u16 (chunked palettes) or u32, idx_bytes) with c->g.idx_pitch elements per palette, opponent tables of
// opp_stride entries per palette in d_opp.  The cost events time all P pairs.
int enqueue_generic_cost(hq_ctx* c, int P, const void* idx_base, int idx_bytes, int opp_stride,
                         const hipEvent_t* ev, int p_off = 0) {
    const Geom& g = c->g;
    hipStream_t s = c->stream;
    HIP_TRY(c, c->d_gen_t.ensure(sizeof(float) * 7 * (size_t)g.n_ext + 256));
    const int64_t n_own = (int64_t)g.W * (g.r1 - g.r0);
    const float inv[3] = {1.0f / c->illum[0], 1.0f / c->illum[1], 1.0f / c->illum[2]};
    for (int p = 0; p < P; ++p) {
        GenArgs gn{};
        gn.idx = static_cast<const char*>(idx_base) + (int64_t)p * g.idx_pitch * idx_bytes;
        gn.opp = c->d_opp.as<float4>() + (int64_t)(p_off + p) * opp_stride;
        gn.k1 = c->d_k1.as<float>();
        gn.k2 = c->d_k2.as<float>();
        gn.k3 = c->d_k3.as<float>();
        gn.absk3 = c->d_absk3.as<float>();
        gn.t = c->d_gen_t.as<float>();
        gn.labL = c->d_labL.as<float>();
        gn.labA = c->d_labA.as<float>();
        gn.labB = c->d_labB.as<float>();
        gn.acc = acc_set(c, c->acc_par, P);
        gn.p = p;
        gn.P = P;
        gn.g = g;
        gn.half = c->half;
        gn.pix_err = c->pixel_err ? c->d_pixerr.as<float>() + (int64_t)p * n_own : nullptr;
        gn.vtaps = c->d_vtaps.as<float>();
        gn.vtap_pitch = c->vtap_pitch;
        gn.hrow4 = c->gen_hrow4;
        gn.hrow_no = c->gen_hrow_no;
        gn.vtile2 = c->gen_vtile2;
        // split-f16 planes hold |x| < 4 (x 2^14): palettes outside the fast range stay on fp32
        gn.vmfma = c->gen_vmfma && !c->pal_generic;
        gn.vtapd = c->d_vfragm.bytes ? c->d_vfragm.as<uint32_t>() : nullptr;
        gn.hmfma = c->gen_hmfma;
        gn.shape = c->gen_shape;
        gn.htapd = gn.vtapd ? gn.vtapd + vtile_dup_tap_words(c->half) : nullptr;
        gn.htaps = c->d_htaps.as<float4>();
        opp2xyz_over_illum(inv, gn.m_lab);
        // the events span every palette's launch pair: start on the first, stop on the last
        if (ev) set_launch_events(p == 0 ? ev[4] : nullptr, p == P - 1 ? ev[5] : nullptr);
        // cost_variant 2: the per-pixel pair in the reference's summation order
        const hipError_t e = c->cost_variant == 2 ? launch_cost_generic(gn, c->de_type, idx_bytes, s)
                                                  : launch_cost_tiled_generic(gn, c->de_type, idx_bytes, s);
        set_launch_events(nullptr, nullptr);
        HIP_TRY(c, e);
    }
    return HQ_OK;
}

int palette_slice(hq_ctx* c, int P, int* lo, int* n);

// K > 256 (hq_wide.hip): prep, exhaustive argmin into 32-bit indices and
// per-colour used flags, the generic cost, finalize, [all-reduce or, under a
// palette split, all-gather].  A palette split takes the same slice
// [lo, lo + Pl) as enqueue_core: the other ranks' palettes are prepped here
// too (cheap) but neither assigned nor costed, so no rank counts them.
int enqueue_wide(hq_ctx* c, int P, int K, const hipEvent_t* ev) {
    const Geom& g = c->g;
    hipStream_t s = c->stream;
    int lo = 0, Pl = P;
    if (int rc = palette_slice(c, P, &lo, &Pl)) return rc;
    WideArgs wa{c->d_pal_in.as<float4>(), c->d_pal.as<float4>(), c->d_opp.as<float4>(), c->d_pflags.as<int>(),
                c->d_R.as<float>(), c->d_G.as<float>(), c->d_B.as<float>(), c->d_idx32.as<uint32_t>(),
                c->d_used32.as<uint32_t>(), g.n_ext, g.idx_pitch, K};
    c->acc_par ^= 1;
    if (Pl < P && !c->comm)  // test-only slice: the other palettes' rows read as zero
        HIP_TRY(c, hipMemsetAsync(c->d_out.p, 0, sizeof(double) * (size_t)P * (1 + K), s));
    HIP_TRY(c, hipMemsetAsync(acc_set(c, c->acc_par, Pl), 0, sizeof(uint64_t) * acc_words(Pl), s));
    HIP_TRY(c, hipMemsetAsync(c->d_pflags.p, 0, sizeof(int) * (size_t)P, s));
    HIP_TRY(c, launch_prep_wide(wa, P, s));
    HIP_TRY(c, hipMemsetAsync(c->d_used32.p, 0, sizeof(uint32_t) * (size_t)Pl * K, s));
    // the slice's palettes: indices and used flags in rows 0 .. Pl - 1
    WideArgs ws = wa;
    ws.pal += (int64_t)lo * K;
    ws.opp += (int64_t)lo * K;
    ws.pflags += lo;
    if (ev) set_launch_events(ev[2], ev[3]);
    const hipError_t e = launch_assign_wide(ws, Pl, s);
    set_launch_events(nullptr, nullptr);
    HIP_TRY(c, e);
    int rc = enqueue_generic_cost(c, Pl, c->d_idx32.p, 4, K, ev, lo);
    if (rc) return rc;
    FinalizeArgs fa{acc_set(c, c->acc_par, Pl), nullptr, 0, c->d_out.as<double>() + (int64_t)lo * (1 + K), Pl, K,
                    c->d_used32.as<uint32_t>(), 8};
    if (ev) set_launch_events(ev[6], ev[7]);
    const hipError_t ef = launch_finalize(fa, Pl, s);
    set_launch_events(nullptr, nullptr);
    HIP_TRY(c, ef);
    if (c->comm) {
        if (ev) HIP_TRY(c, hipEventRecord(ev[10], s));
        if (c->psplit)
            NCCL_TRY(c, ncclAllGather(c->d_out.as<double>() + (int64_t)lo * (1 + K), c->d_out.p,
                                      (size_t)Pl * (1 + K), ncclFloat64, c->comm, s));
        else
            NCCL_TRY(c, ncclAllReduce(c->d_out.p, c->d_out.p, (size_t)P * (1 + K), ncclFloat64, ncclSum,
                                      c->comm, s));
        if (ev) HIP_TRY(c, hipEventRecord(ev[11], s));
    }
    c->slice_lo = lo;
    c->slice_n = Pl;
    c->last_P = P;
    c->K_cur = K;
    c->last_nch = 1;
    return HQ_OK;
}

// P palettes of K colours.  Chunked palettes (c->nch_cur = nch > 1, 256 < K <=
// 256 nch): the grid and assign run on P nch sub-palettes of 256 colours (d_pal
// etc. hold them, prep_palette made them), assign combines them into 16-bit
// indices, the cost kernel reads those with a 256 nch-entry table.
// The palettes of a P-palette population this device evaluates: a palette
// split (psplit with a communicator of N ranks, or the test-only slice options)
// takes [r P/N, (r+1) P/N) on the whole image; anything else all P.
int palette_slice(hq_ctx* c, int P, int* lo, int* n) {
    int R = 1, r = 0;
    if (c->psplit && c->comm) R = c->nranks, r = c->rank;
    else if (c->slice_ranks > 1) R = c->slice_ranks, r = c->slice_rank;
    *lo = 0;
    *n = P;
    if (R == 1) return HQ_OK;
    if (r < 0 || r >= R) return fail(c, HQ_ERR_ARG, "palette split: rank %d outside [0, %d)", r, R);
    if (P % R) return fail(c, HQ_ERR_ARG, "palette split: population %d not divisible by %d ranks", P, R);
    if (c->g.r0 != 0 || c->g.r1 != c->g.H)
        return fail(c, HQ_ERR_STATE, "palette split: every rank needs the whole image (hq_set_image)");
    *n = P / R;
    *lo = r * *n;
    return HQ_OK;
}

// Each evaluation takes the other counter set than the last one (build_grid
// zeroes it), so an accept step can read the last set while the next is filled.
int enqueue_core(hq_ctx* c, int P, int K, const hipEvent_t* ev, bool fold = false) {
    const Geom& g = c->g;
    hipStream_t s = c->stream;
    const int nch = c->nch_cur, Ks = nch > 1 ? kMaxK : K;
    // the palettes this device evaluates: all, or a palette split's slice [lo, lo + Pl)
    int lo = 0, Pl = P;
    if (int rc = palette_slice(c, P, &lo, &Pl)) return rc;
    const int Ps = Pl * nch, so = lo * nch;  // sub-palettes, the first one's index
    if (Pl < P && !c->comm)  // test-only slice: the other palettes' rows read as zero
        HIP_TRY(c, hipMemsetAsync(c->d_out.p, 0, sizeof(double) * (size_t)P * (1 + K), s));
    c->acc_par ^= 1;
    const GridArgs ga = grid_args(c, Ps, Ks, so);
    auto timed = [&](int slot) {
        if (ev) set_launch_events(ev[2 * slot], ev[2 * slot + 1]);
    };
    auto untimed = [&]() { set_launch_events(nullptr, nullptr); };
    const bool n16 = use_lists16(c);
    if (c->G2 > 0) {  // (build_grid also zeroes the used bits and the sums)
        timed(0);
        const hipError_t e =
            n16 ? launch_lists16_grid(Lists16Args{ga.pal, ga.pflags, c->d_l1n.as<uint16_t>(), c->d_l2n.as<uint16_t>(),
                                                  ga.used_glob, used_stride(Ps), ga.acc_zero, Pl, K, nch * kMaxK, nch},
                                      Pl, s)
                : launch_build_grid(ga, Ps, s);
        untimed();
        HIP_TRY(c, e);
    } else {
        HIP_TRY(c, hipMemsetAsync(ga.used_glob, 0, sizeof(uint32_t) * kUsedSlots * (size_t)used_stride(Ps), s));
        HIP_TRY(c, hipMemsetAsync(ga.acc_zero, 0, sizeof(uint64_t) * acc_words(Pl), s));
    }
    const int nblocks = assign_blocks(c, Ps);
    AssignArgs aa{c->d_R.as<float>(), c->d_G.as<float>(), c->d_B.as<float>(),
                  c->img_u8 && c->img_u8_path ? c->d_rgbx.as<uint32_t>() : nullptr, ga.pal, ga.pflags,
                  c->d_lvl1.as<uint8_t>(), c->d_lvl2.as<uint8_t>(),
                  c->d_idx.as<uint8_t>(), ga.used_glob, used_stride(Ps), g.n_ext, g.idx_pitch,
                  ga.lvl1_pitch, ga.lvl2_gstride, Ks, c->G2, nblocks};
    if (nch > 1) {
        aa.idx16 = c->d_idx16.as<uint16_t>();
        aa.dist = nch > 4 ? c->d_dist.as<float>() : nullptr;
        aa.nch = nch;
        while ((1 << aa.lg_nch) < nch) ++aa.lg_nch;
    }
    if (n16) {  // one palette of K colours per workgroup (its table in LDS)
        aa.l1n = c->d_l1n.as<uint16_t>();
        aa.l2n = c->d_l2n.as<uint16_t>();
        aa.kpal = nch * kMaxK;
        aa.K = K;
        // one resident round of 1024-thread workgroups over the P palettes, >= 4 pixels per thread
        const int ngr = K <= 4096 ? (Pl + 1) / 2 : Pl;  // workgroup groups: palette pairs up to K = 4096
        aa.nblocks = (int)std::max<int64_t>(
            1, std::min<int64_t>(std::max(1, c->num_cu / ngr), (g.n_ext + 4095) / 4096));
    }
    const float inv[3] = {1.0f / c->illum[0], 1.0f / c->illum[1], 1.0f / c->illum[2]};
    const bool fast = cost_fast(c);
    // 8-row tiles (cost_mfma_kernel) exist for the 21-tap bucket only
    const int rows = c->fast_hb == 10 ? c->cost_rows : 16;
    const int tw = c->fast_hb == 10 ? c->cost_tw : 128;  // 256-column tiles: HB = 10 only
    CostArgs ca{};
    if (fast) {
        ca.idx = nch > 1 ? c->d_idx16.as<uint8_t>() : c->d_idx.as<uint8_t>();
        ca.opp16 = c->d_opp16.as<uint4>() + (int64_t)so * kMaxK;
        ca.taps = c->d_taps.p;
        ca.vfrag16 = c->d_vfrag16.as<uint4>();
        ca.vfrag16p = c->d_vfrag16p.as<uint4>();
        ca.labL = c->d_labL.as<float>();
        ca.labA = c->d_labA.as<float>();
        ca.labB = c->d_labB.as<float>();
        ca.acc = ga.acc_zero;
        ca.acc_P = Pl;
        ca.acc_p0 = 0;
        ca.g = g;
        ca.K = K;
        fast_tile_dims(g.W, g.r1 - g.r0, rows, tw, &ca.tiles_x, &ca.ntiles);
        opp2xyz_over_illum(inv, ca.m_lab);
        ca.pix_err = c->pixel_err ? c->d_pixerr.as<float>() : nullptr;
        ca.pix_pitch = (int64_t)g.W * (g.r1 - g.r0);
    }
    timed(1);
    hipError_t e = n16 ? launch_assign16(aa, Pl, s) : launch_assign(aa, Ps, s);
    untimed();
    HIP_TRY(c, e);
    if (fast) {
        timed(2);
        e = nch > 1 ? launch_cost_chunked(ca, Pl, nch, c->de_type, c->trim && c->trim_ok, s)
                    : launch_cost_fast(ca, Pl, c->de_type, c->trim && c->trim_ok, rows, tw, c->fast_hb, s);
        untimed();
        HIP_TRY(c, e);
    } else {
        int rc = nch > 1 ? enqueue_generic_cost(c, Pl, c->d_idx16.p, 2, nch * kMaxK, ev, lo)
                         : enqueue_generic_cost(c, Pl, c->d_idx.p, 1, kMaxK, ev, lo);
        if (rc) return rc;
    }
    if (!fold) {  // (a folding search's accept step reads the sums itself)
        FinalizeArgs fa{ga.acc_zero, ga.used_glob, used_stride(Ps), c->d_out.as<double>() + (int64_t)lo * (1 + K),
                        Pl, K, nullptr, 8 * nch};
        timed(3);
        const hipError_t ef = launch_finalize(fa, Pl, s);
        untimed();
        HIP_TRY(c, ef);
    }
    if (c->comm) {
        // the collective's time (profiling only: an event record between launches
        // idles the GPU a few us, so the timed pass of bench.py records none)
        if (ev) HIP_TRY(c, hipEventRecord(ev[10], s));
        if (fold) {
            // row blocks under a folding search: every rank's counter block and
            // used-bit block to every rank (in place), one group of two
            // all-gathers; the accept step sums the integer counters and ORs the
            // bits of all the blocks itself
            const size_t na = acc_words(Pl), nu = (size_t)kUsedSlots * used_stride(Ps);
            NCCL_TRY(c, ncclGroupStart());
            NCCL_TRY(c, ncclAllGather(acc_set(c, c->acc_par, Pl), acc_base(c, c->acc_par, Pl), na, ncclUint64,
                                      c->comm, s));
            NCCL_TRY(c, ncclAllGather(used_set(c, c->acc_par, Ps), used_base(c, c->acc_par, Ps), nu, ncclUint32,
                                      c->comm, s));
            NCCL_TRY(c, ncclGroupEnd());
        } else if (c->psplit) {  // every rank's slice to every rank (in place; one rank: a no-op)
            NCCL_TRY(c, ncclAllGather(c->d_out.as<double>() + (int64_t)lo * (1 + K), c->d_out.p,
                                      (size_t)Pl * (1 + K), ncclFloat64, c->comm, s));
        } else {  // also with one rank (a no-op copy), so that path is exercised on one GPU
            NCCL_TRY(c, ncclAllReduce(c->d_out.p, c->d_out.p, (size_t)P * (1 + K), ncclFloat64, ncclSum,
                                      c->comm, s));
        }
        if (ev) HIP_TRY(c, hipEventRecord(ev[11], s));
    }
    c->slice_lo = lo;
    c->slice_n = Pl;
    c->last_P = P;
    c->K_cur = K;
    c->last_nch = nch;
    return HQ_OK;
}

// Add one evaluation's kernel times (its events have completed).
void prof_accumulate(hq_ctx* c, const hipEvent_t* ev, bool finalize = true, bool grid = true) {
    if (grid && c->G2 > 0) prof_add(c, c->prof_grid, ev[0], ev[1]);
    prof_add(c, c->prof_assign, ev[2], ev[3]);
    prof_add(c, c->prof_cost, ev[4], ev[5]);
    if (finalize) prof_add(c, c->prof_finalize, ev[6], ev[7]);
    if (c->comm) prof_add(c, c->prof_comm, ev[10], ev[11]);
}

// ... and the SA step that generated it (device-resident search: events 8, 9).
void prof_accumulate_sa(hq_ctx* c, const hipEvent_t* ev) {
    prof_add(c, c->prof_sa, ev[8], ev[9]);
}

// Host-driven evaluation of the P palettes in h_pal: upload, prep, enqueue_core,
// read back d_out into h_out.
int enqueue_eval(hq_ctx* c, int P, int K) {
    hipStream_t s = c->stream;
    const size_t n_in = c->nch_cur > 1 ? (size_t)P * c->nch_cur * kMaxK : (size_t)P * K;
    HIP_TRY(c, hipMemcpyAsync(c->d_pal_in.p, c->h_pal, sizeof(float4) * n_in, hipMemcpyHostToDevice, s));
    const hipEvent_t* ev = c->prof ? c->ev : nullptr;
    int rc;
    if (c->nch_cur > 1) {  // h_pal holds P nch sub-palettes of 256 (pack_chunks)
        HIP_TRY(c, launch_prep_palette(prep_args(c, kMaxK), P * c->nch_cur, s));
        rc = enqueue_core(c, P, K, ev);
    } else if (K > kMaxK) {
        rc = enqueue_wide(c, P, K, ev);
    } else {
        HIP_TRY(c, launch_prep_palette(prep_args(c, K), P, s));
        rc = enqueue_core(c, P, K, ev);
    }
    if (rc) return rc;
    HIP_TRY(c, hipMemcpyAsync(c->h_out, c->d_out.p, sizeof(double) * (size_t)P * (1 + K),
                              hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    if (ev) prof_accumulate(c, ev, true, K <= kMaxK || c->nch_cur > 1);  // (the wide path builds no grid)
    return HQ_OK;
}

int check_eval_args(hq_ctx* c, const float* palettes, int P, int K) {
    if (!c) return HQ_ERR_ARG;
    if (!c->have_image) return fail(c, HQ_ERR_STATE, "no image set (hq_set_image)");
    if (!palettes || P < 1 || K < 1) return fail(c, HQ_ERR_ARG, "bad palettes / P=%d / K=%d", P, K);
    if (K > kMaxKWide)
        return fail(c, HQ_ERR_ARG, "K=%d > %d (the plugin's limit, HQ:192)", K, kMaxKWide);
    if (c->de_type == HQ_DE_CIEDE2000)
        return fail(c, HQ_ERR_UNSUPPORTED, "CIEDE2000 is unimplemented in the reference (CL:227-230)");
    return HQ_OK;
}

// The fast cost kernels take the opponent colours as split f16 of x * 2^14
// (split_f16): |opp| must stay below 65504 / 2^14 ~ 4.  RGB2Opp's largest
// absolute row sum is 0.871, so a palette channel x in [-59, 1.93] keeps
// |opp| < 4 (lin(x) = x / 12.92 below 0.04045, ((x + 0.055) / 1.055)^2.4
// above).  Colours outside [-32, 1.9] -- never produced by the SA, which
// clamps to [0, 1] (SW:103-106), but accepted by hq_eval_population -- and
// non-finite colours send the population to the generic fp32 path.
// [P][K] palettes -> P nch sub-palettes of 256 colours: sub-palette p nch + c
// holds colours 256 c .. 256 c + 255 of palette p, and copies of colour 0 past
// K (a copy of colour 0 ties it and never wins the chunk combine, which keeps
// the first chunk at equal distance; hq_assign.hip).
void pack_chunks(const float* pal, int P, int K, int nch, float* out) {
    for (int p = 0; p < P; ++p)
        for (int k = 0; k < nch * kMaxK; ++k) {
            const float* src = pal + 4 * ((size_t)p * K + (k < K ? k : 0));
            float* dst = out + 4 * ((size_t)p * nch * kMaxK + k);
            dst[0] = src[0]; dst[1] = src[1]; dst[2] = src[2]; dst[3] = src[3];
        }
}

bool palette_fits_fast(const float* pal, int P, int K) {
    for (size_t i = 0, n = (size_t)P * K; i < n; ++i)
        for (int ch = 0; ch < 3; ++ch) {
            const float x = pal[4 * i + ch];
            if (!(x >= -32.0f && x <= 1.9f)) return false;
        }
    return true;
}

int eval_partial_into_hout(hq_ctx* c, const float* palettes, int P, int K) {
    int rc = check_eval_args(c, palettes, P, K);
    if (rc) return rc;
    if ((rc = bind(c))) return rc;
    const bool fits = palette_fits_fast(palettes, P, K);
    // 256 < K <= 16384: chunks of 256 colours through the grid and assign, and the
    // tiled cost kernel up to 32 chunks (the generic pair above).  Palettes outside
    // the fast range (non-finite colours among
    // them) take the exhaustive K > 256 path instead, which keeps the
    // reference's NaN semantics across all K colours.
    c->nch_cur = c->chunked && fits && c->G2 > 0 && K > kMaxK && K <= kMaxKChunked ? chunk_count(K) : 1;
    c->pal_generic = !fits;  // (before ensure_population: it sizes the generic path's scratch)
    if (!(rc = ensure_population(c, P, K))) {
        if (c->nch_cur > 1) pack_chunks(palettes, P, K, c->nch_cur, c->h_pal);
        else std::memcpy(c->h_pal, palettes, sizeof(float) * 4 * (size_t)P * K);
        rc = enqueue_eval(c, P, K);
    }
    c->pal_generic = false;  // device-resident searches generate clamped palettes
    c->nch_cur = 1;
    return rc;
}

}  // namespace

namespace {

// The chunk count of the population being enqueued, for one search call.
struct NchScope {
    hq_ctx* c;
    NchScope(hq_ctx* cc, int nch) : c(cc) { c->nch_cur = nch; }
    ~NchScope() { c->nch_cur = 1; }
};

// The arguments of an SA step: accept the population in cand[cd] (if `accept`,
// its counters in set c->acc_par), then generate the next candidates into
// cand[1 - cd] (if `generate`).
SaArgs sa_args(hq_search* s, bool accept, bool init, bool generate, bool random, float amax) {
    hq_ctx* c = s->ctx;
    SaArgs a{};
    a.out = c->d_out.as<double>();
    a.colors_in = s->colors[s->st].as<float>();
    a.colors_out = s->colors[1 - s->st].as<float>();
    a.cand_in = s->cand[s->cd].as<float>();
    a.cand_out = s->cand[1 - s->cd].as<float>();
    a.err_in = s->err[s->st].as<double>();
    a.err_out = s->err[1 - s->st].as<double>();
    a.seed_in = s->seed[s->st].as<uint64_t>();
    a.seed_out = s->seed[1 - s->st].as<uint64_t>();
    a.best_err_in = s->best_err[s->st].as<double>();
    a.best_err_out = s->best_err[1 - s->st].as<double>();
    a.best_colors = s->best_colors.as<float>();
    a.jump_A = s->jA.as<uint64_t>();
    a.jump_C = s->jC.as<uint64_t>();
    a.prep = prep_args(c, s->nch > 1 ? kMaxK : s->K);
    a.nch = s->nch;
    a.n_total = (double)c->g.W * (double)c->g.H;
    a.keep_threshold = s->keep_acc;
    a.temperature = s->t_acc;
    a.amax = amax;
    a.delta = s->prm.delta;
    a.P = s->P;
    a.K = s->K;
    a.accept = accept;
    a.init = init;
    a.generate = generate;
    a.random = random;
    a.convergence = s->prm.convergence;
    a.acc = acc_base(c, c->acc_par, a.P);
    a.used_glob = used_base(c, c->acc_par, a.P * s->nch);
    a.used_stride = used_stride(a.P * s->nch);
    a.fold = s->fold;
    a.nranks = rank_blocks(c);
    a.acc_rank_words = (int64_t)acc_words(a.P);
    return a;
}

void sa_advance(hq_search* s, bool generate) {
    s->st = 1 - s->st;
    if (generate) s->cd = 1 - s->cd;
}

// One sa_step launch (sa_args).
int enqueue_sa_step(hq_search* s, bool accept, bool init, bool generate, bool random, float amax,
                    const hipEvent_t* ev = nullptr) {
    hq_ctx* c = s->ctx;
    const SaArgs a = sa_args(s, accept, init, generate, random, amax);
    if (ev) set_launch_events(ev[0], ev[1]);
    const hipError_t e = launch_sa_step(a, c->stream);
    set_launch_events(nullptr, nullptr);
    HIP_TRY(c, e);
    sa_advance(s, generate);
    return HQ_OK;
}

int ensure_events(hq_search* s, size_t n) {
    while (s->pev.size() < n) {
        hipEvent_t e;
        HIP_TRY(s->ctx, hipEventCreate(&e));
        s->pev.push_back(e);
    }
    return HQ_OK;
}

int device_search_create(hq_ctx* c, const hq_swasa_params* params, int K, uint64_t seed, hq_search* s) {
    const int P = params->population;
    s->prm = *params;
    s->P = P;
    // no communicator, or row blocks: nothing has to see the finalized sums, so
    // the accept step reads the fixed-point sums itself (one launch less per
    // iteration; row blocks: one all-gather of every rank's counter blocks in
    // place of finalize + the all-reduce of P (1 + K) doubles).  The palette
    // split all-gathers finalized rows.
    s->fold = search_folds(c);
    s->comm = c->comm;
    if (c->slice_ranks > 1 && !c->comm)
        return fail(c, HQ_ERR_STATE, "palette slice without a communicator (test option): no search");
    s->pol = new Swasa(*params, seed);
    const NchScope scope(c, s->nch);
    int rc = ensure_population(c, P, K);
    if (rc) return rc;
    const size_t n4 = (size_t)P * 4 * K;
    for (int i = 0; i < 2; ++i) {
        HIP_TRY(c, s->colors[i].ensure(sizeof(float) * n4));
        HIP_TRY(c, s->cand[i].ensure(sizeof(float) * n4));
        HIP_TRY(c, s->err[i].ensure(sizeof(double) * P));
        HIP_TRY(c, s->seed[i].ensure(sizeof(uint64_t)));
    }
    for (int i = 0; i < 2; ++i) HIP_TRY(c, s->best_err[i].ensure(sizeof(double)));
    HIP_TRY(c, s->best_colors.ensure(sizeof(float) * 4 * K));
    // java.util.Random jumps: n steps = A_n s + C_n (mod 2^48), n = 0 .. 3KP
    const size_t nj = (size_t)3 * K * P + 1;
    std::vector<uint64_t> A(nj), C(nj);
    const uint64_t mask = (1ull << 48) - 1, mult = 0x5DEECE66Dull;
    A[0] = 1;
    C[0] = 0;
    for (size_t n = 1; n < nj; ++n) {
        A[n] = (A[n - 1] * mult) & mask;
        C[n] = (C[n - 1] * mult + 0xBull) & mask;
    }
    HIP_TRY(c, s->jA.ensure(sizeof(uint64_t) * nj));
    HIP_TRY(c, s->jC.ensure(sizeof(uint64_t) * nj));
    HIP_TRY(c, hipMemcpy(s->jA.p, A.data(), sizeof(uint64_t) * nj, hipMemcpyHostToDevice));
    HIP_TRY(c, hipMemcpy(s->jC.p, C.data(), sizeof(uint64_t) * nj, hipMemcpyHostToDevice));
    const uint64_t s0 = (seed ^ mult) & mask;  // JavaRandom::set_seed
    HIP_TRY(c, hipMemcpy(s->seed[0].p, &s0, sizeof s0, hipMemcpyHostToDevice));
    HIP_TRY(c, hipMemset(s->err[0].p, 0, sizeof(double) * P));
    if (rank_blocks(c) > 1 && !c->comm) {  // test layout: the blocks no rank fills read zero
        HIP_TRY(c, hipMemsetAsync(c->d_acc.p, 0, c->d_acc.bytes, c->stream));
        HIP_TRY(c, hipMemsetAsync(c->d_used_mask.p, 0, c->d_used_mask.bytes, c->stream));
    }
    for (int i = 0; i < 2; ++i) HIP_TRY(c, hipMemset(s->best_err[i].p, 0, sizeof(double)));
    s->st = s->cd = 0;
    // IM:385-493: random population (SW:40-52), its evaluation, argmin
    if ((rc = enqueue_sa_step(s, false, false, true, true, 0.f))) return rc;
    if ((rc = enqueue_core(c, P, K, nullptr, s->fold))) return rc;
    if ((rc = enqueue_sa_step(s, true, true, false, false, 0.f))) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    s->ite = 0;
    return HQ_OK;
}

// IM:497-568 for up to `iterations` iterations, all enqueued before one sync.
int device_search_run(hq_search* s, int iterations, int* ran) {
    hq_ctx* c = s->ctx;
    int done = 0, rc;
    // The context may have changed since hq_search_create or the last run (an
    // option such as 'grid' or 'assign_blocks_per_cu', a new image): size its
    // work buffers for the current geometry before enqueueing anything.
    if (!c->have_image) return fail(c, HQ_ERR_STATE, "no image set (hq_set_image)");
    if (c->de_type == HQ_DE_CIEDE2000)
        return fail(c, HQ_ERR_UNSUPPORTED, "CIEDE2000 is unimplemented in the reference (CL:227-230)");
    const NchScope scope(c, s->nch);
    if ((rc = ensure_population(c, s->P, s->K))) return rc;
    if (s->comm != c->comm || s->fold != search_folds(c))
        return fail(c, HQ_ERR_STATE, "communicator or palette split changed after hq_search_create: "
                                     "recreate the search");
    const bool prof = c->prof;
    if (prof && (rc = ensure_events(s, (size_t)kProfEvents * iterations))) return rc;
    // option sa_graph: the run's kernels go into one hipGraph (stream capture),
    // replayed as a whole -- a chain of dependent kernels costs ~2.7 us per
    // kernel from the stream and ~1.8 from a graph (profiles/r04_graph_gap_
    // microbench.txt).  The previous run's executable graph is updated in place
    // when the iteration count (the topology) is the same, else instantiated
    // anew.  Not with profiling events (they ride on the launches).
    const bool graph = c->sa_graph && !prof;
    if (graph) HIP_TRY(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    auto abort_capture = [&](int rc0) {
        if (graph) {
            hipGraph_t gr = nullptr;
            if (hipStreamEndCapture(c->stream, &gr) == hipSuccess && gr) (void)hipGraphDestroy(gr);
        }
        return rc0;
    };
    for (; done < iterations && s->ite < s->prm.imax; ++done) {
        const int ite = ++s->ite;
        s->pol->reduce_temperature_if_necessary(ite);                  // IM:507
        const float amax = s->pol->max_step_width(ite) / 256.0f;       // SW:91-101
        const hipEvent_t* ev = prof ? &s->pev[(size_t)kProfEvents * done] : nullptr;
        // accept the previous iteration's population (none at the first of a run)
        if ((rc = enqueue_sa_step(s, done > 0, false, true, false, amax, ev ? ev + 8 : nullptr)))
            return abort_capture(rc);
        if ((rc = enqueue_core(c, s->P, s->K, ev, s->fold))) return abort_capture(rc);
        s->t_acc = s->pol->temperature();     // SW:54-57 at this iteration
        s->keep_acc = s->pol->keep_threshold(ite);
    }
    if (done > 0 && (rc = enqueue_sa_step(s, true, false, false, false, 0.f))) return abort_capture(rc);
    if (graph) {
        hipGraph_t gr = nullptr;
        HIP_TRY(c, hipStreamEndCapture(c->stream, &gr));
        bool updated = false;
        if (s->gexec && s->gexec_iters == done) {
            hipGraphNode_t err_node = nullptr;
            hipGraphExecUpdateResult res = hipGraphExecUpdateError;
            updated = hipGraphExecUpdate(s->gexec, gr, &err_node, &res) == hipSuccess &&
                      res == hipGraphExecUpdateSuccess;
            if (!updated) (void)hipGetLastError();
        }
        if (!updated) {
            if (s->gexec) (void)hipGraphExecDestroy(s->gexec);
            s->gexec = nullptr;
            const hipError_t e = hipGraphInstantiate(&s->gexec, gr, nullptr, nullptr, 0);
            if (e != hipSuccess) {
                (void)hipGraphDestroy(gr);
                s->gexec = nullptr;
                HIP_TRY(c, e);
            }
            s->gexec_iters = done;
        }
        (void)hipGraphDestroy(gr);
        HIP_TRY(c, hipGraphLaunch(s->gexec, c->stream));
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    for (int i = 0; prof && i < done; ++i) {
        prof_accumulate(c, &s->pev[(size_t)kProfEvents * i], !s->fold);
        prof_accumulate_sa(c, &s->pev[(size_t)kProfEvents * i]);
    }
    if (ran) *ran = done;
    return HQ_OK;
}

}  // namespace

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

int hq_version(void) { return HQ_VERSION; }

const char* hq_status_string(int s) {
    switch (s) {
        case HQ_OK: return "ok";
        case HQ_ERR_ARG: return "invalid argument";
        case HQ_ERR_DEVICE: return "device error";
        case HQ_ERR_STATE: return "invalid state";
        case HQ_ERR_UNSUPPORTED: return "unsupported";
        case HQ_ERR_COMM: return "communication error";
        case HQ_ERR_NOMEM: return "out of memory";
        default: return "unknown status";
    }
}

int hq_device_count(int* count) {
    if (!count) return HQ_ERR_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return HQ_OK;
}

int hq_create(int device, int delta_e_type, hq_ctx** out) {
    if (!out) return HQ_ERR_ARG;
    *out = nullptr;
#ifdef HQ_ABLATION_BUILD
    std::fprintf(stderr, "libhq: ABLATION BUILD (HQ_ABL_*): costs and indices are wrong by design\n");
#endif
    if (delta_e_type < HQ_DE_CIE76 || delta_e_type > HQ_DE_CIEDE2000) return HQ_ERR_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n)
        return HQ_ERR_DEVICE;
    hq_ctx* c = new hq_ctx();
    c->device = device;
    c->de_type = delta_e_type;
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return HQ_ERR_DEVICE;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0) {
        c->num_cu = prop.multiProcessorCount;
        c->lds_optin = std::max(prop.sharedMemPerBlockOptin, prop.sharedMemPerBlock);
    }
    for (int ng = 1; ng <= 4; ++ng) c->assign_res[ng] = assign_residency(ng);
    c->assign_res_chunked = assign_residency_chunked();
    for (auto& e : c->ev) (void)hipEventCreate(&e);
    *out = c;
    return HQ_OK;
}

void hq_destroy(hq_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    for (DevBuf* b : {&c->d_k1, &c->d_k2, &c->d_k3, &c->d_absk3, &c->d_vtaps, &c->d_R, &c->d_G, &c->d_B, &c->d_rgbx,
                      &c->d_labL, &c->d_labA, &c->d_labB, &c->d_pal_in, &c->d_pal, &c->d_opp, &c->d_opp16,
                      &c->d_dup, &c->d_pflags, &c->d_lvl1, &c->d_lvl2, &c->d_idx,
                      &c->d_used_mask, &c->d_acc, &c->d_out, &c->d_gen_t, &c->d_taps,
                      &c->d_vfrag16, &c->d_vfrag16p, &c->d_vfragm, &c->d_htaps, &c->d_idx32, &c->d_used32, &c->d_pixerr, &c->d_idx16, &c->d_dist, &c->d_l1n, &c->d_l2n})
        b->release();
    if (c->h_pal) (void)hipHostFree(c->h_pal);
    if (c->h_out) (void)hipHostFree(c->h_out);
    for (auto& e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* hq_last_error(const hq_ctx* c) { return c ? c->err.c_str() : "null context"; }

int hq_set_filters(hq_ctx* c, int taps, const float* k1, const float* k2, const float* k3,
                   const float* absk3) {
    if (!c) return HQ_ERR_ARG;
    if (taps < 1 || taps > kMaxTaps || !k1 || !k2 || !k3 || !absk3)
        return fail(c, HQ_ERR_ARG, "bad filters (taps=%d)", taps);
    int rc = bind(c);
    if (rc) return rc;
    c->taps = taps;
    c->half = (taps * 4) / 8;  // IM:408 filters4[0].length/8
    if (2 * c->half + 1 != taps)
        return fail(c, HQ_ERR_UNSUPPORTED, "even tap count %d (the reference assumes odd)", taps);
    c->k1.assign(k1, k1 + 4 * taps);
    c->k2.assign(k2, k2 + 4 * taps);
    c->k3.assign(k3, k3 + taps);
    c->absk3.assign(absk3, absk3 + taps);
    HIP_TRY(c, c->d_k1.ensure(sizeof(float) * 4 * taps));
    HIP_TRY(c, c->d_k2.ensure(sizeof(float) * 4 * taps));
    HIP_TRY(c, c->d_k3.ensure(sizeof(float) * taps));
    HIP_TRY(c, c->d_absk3.ensure(sizeof(float) * taps));
    HIP_TRY(c, hipMemcpy(c->d_k1.p, k1, sizeof(float) * 4 * taps, hipMemcpyHostToDevice));
    HIP_TRY(c, hipMemcpy(c->d_k2.p, k2, sizeof(float) * 4 * taps, hipMemcpyHostToDevice));
    HIP_TRY(c, hipMemcpy(c->d_k3.p, k3, sizeof(float) * taps, hipMemcpyHostToDevice));
    HIP_TRY(c, hipMemcpy(c->d_absk3.p, absk3, sizeof(float) * taps, hipMemcpyHostToDevice));
    {  // the tiled generic path's vertical taps per plane (t1.xyz: k1, t2.xyz: k2, t3: |k3|)
        c->vtap_pitch = (taps + 15) / 16 * 16 + 16;
        std::vector<float> vt((size_t)kNumFilt * c->vtap_pitch, 0.f);
        for (int t = 0; t < taps; ++t) {
            for (int ch = 0; ch < 3; ++ch) {
                vt[(size_t)ch * c->vtap_pitch + t] = k1[4 * t + ch];
                vt[(size_t)(3 + ch) * c->vtap_pitch + t] = k2[4 * t + ch];
            }
            vt[(size_t)6 * c->vtap_pitch + t] = absk3[t];
        }
        HIP_TRY(c, c->d_vtaps.ensure(sizeof(float) * vt.size()));
        HIP_TRY(c, hipMemcpy(c->d_vtaps.p, vt.data(), sizeof(float) * vt.size(), hipMemcpyHostToDevice));
        std::vector<float> ht((size_t)8 * taps);
        for (int t = 0; t < taps; ++t) {
            const float v[8] = {k1[4 * t], k1[4 * t + 1], k1[4 * t + 2], k3[t], k2[4 * t], k2[4 * t + 1], k2[4 * t + 2], 0.f};
            std::copy(v, v + 8, ht.begin() + 8 * t);
        }
        HIP_TRY(c, c->d_htaps.ensure(sizeof(float) * ht.size()));
        HIP_TRY(c, hipMemcpy(c->d_htaps.p, ht.data(), sizeof(float) * ht.size(), hipMemcpyHostToDevice));
        // gen_vmfma's vertical taps (t3: |k3|), then gen_hmfma's horizontal ones (t3: k3)
        std::vector<uint32_t> fm(2 * vtile_dup_tap_words(c->half));
        build_vtile_dup_taps(c->half, k1, k2, absk3, fm.data());
        build_vtile_dup_taps(c->half, k1, k2, k3, fm.data() + vtile_dup_tap_words(c->half));
        HIP_TRY(c, c->d_vfragm.ensure(fm.size() * sizeof(uint32_t)));
        HIP_TRY(c, hipMemcpy(c->d_vfragm.p, fm.data(), fm.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    // fast path: the filters centred in the smallest tap bucket that holds them
    // (half-widths up to 24: every dpi / viewing distance of HQ:229-231 up to
    // ~200 dpi at 45 cm); longer filters take the generic path
    c->fast_hb = fast_bucket(c->half);
    c->trim_ok = c->fast_hb > 0 && trim_window_ok(k1, c->half, c->fast_hb);
    if (c->fast_hb > 0) {
        const int HB = c->fast_hb;
        std::vector<uint16_t> f16s(vpass_f16_stack_fragment_halves(HB));
        build_vpass_f16_stack_fragments(HB, c->half, k1, k2, k3, absk3, f16s.data());
        HIP_TRY(c, c->d_vfrag16.ensure(f16s.size() * sizeof(uint16_t)));
        HIP_TRY(c, hipMemcpy(c->d_vfrag16.p, f16s.data(), f16s.size() * sizeof(uint16_t),
                             hipMemcpyHostToDevice));
        std::vector<uint16_t> f16p(vpass_f16_pair_fragment_halves(HB));
        build_vpass_f16_pair_fragments(HB, c->half, k1, k2, k3, absk3, f16p.data());
        HIP_TRY(c, c->d_vfrag16p.ensure(f16p.size() * sizeof(uint16_t)));
        HIP_TRY(c, hipMemcpy(c->d_vfrag16p.p, f16p.data(), f16p.size() * sizeof(uint16_t),
                             hipMemcpyHostToDevice));
        std::vector<char> tb(fast_taps_bytes(HB));
        build_fast_taps(HB, c->half, k1, k2, k3, absk3, tb.data());
        HIP_TRY(c, c->d_taps.ensure(tb.size()));
        HIP_TRY(c, hipMemcpy(c->d_taps.p, tb.data(), tb.size(), hipMemcpyHostToDevice));
    }
    c->have_image = false;  // halo depends on the filters
    return HQ_OK;
}

int hq_set_image_shard(hq_ctx* c, const float* rgba4, const float* lab4, int w, int h,
                       const float* illum, int row_begin, int row_end) {
    if (!c) return HQ_ERR_ARG;
    if (!rgba4) return fail(c, HQ_ERR_ARG, "null image");
    int rc = check_geom_args(c, w, h, row_begin, row_end);
    if (rc) return rc;
    if ((rc = bind(c))) return rc;
    c->g = make_geom(w, h, row_begin, row_end, c->half);
    std::vector<float> R, G, B;
    gather_rows(rgba4, 4, 0, c->g, R);
    gather_rows(rgba4, 4, 1, c->g, G);
    gather_rows(rgba4, 4, 2, c->g, B);
    return set_image_common(c, R, G, B, lab4, illum);
}

int hq_set_image(hq_ctx* c, const float* rgba4, const float* lab4, int w, int h,
                 const float* illum) {
    return hq_set_image_shard(c, rgba4, lab4, w, h, illum, 0, h);
}

int hq_set_image_planar_shard(hq_ctx* c, const float* R, const float* G, const float* B, int w,
                              int h, const float* illum, int row_begin, int row_end) {
    if (!c) return HQ_ERR_ARG;
    if (!R || !G || !B) return fail(c, HQ_ERR_ARG, "null plane");
    int rc = check_geom_args(c, w, h, row_begin, row_end);
    if (rc) return rc;
    if ((rc = bind(c))) return rc;
    c->g = make_geom(w, h, row_begin, row_end, c->half);
    std::vector<float> r, g, b;
    gather_rows(R, 1, 0, c->g, r);
    gather_rows(G, 1, 0, c->g, g);
    gather_rows(B, 1, 0, c->g, b);
    return set_image_common(c, r, g, b, nullptr, illum);
}

int hq_get_labref(hq_ctx* c, float* lab4) {
    if (!c || !lab4) return HQ_ERR_ARG;
    if (!c->have_image) return fail(c, HQ_ERR_STATE, "no image set");
    int rc = bind(c);
    if (rc) return rc;
    const Geom& g = c->g;
    const int own = g.r1 - g.r0;
    std::vector<float> L((size_t)g.lab_pitch * own), A(L.size()), B(L.size());
    HIP_TRY(c, hipMemcpy(L.data(), c->d_labL.p, sizeof(float) * L.size(), hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(A.data(), c->d_labA.p, sizeof(float) * A.size(), hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(B.data(), c->d_labB.p, sizeof(float) * B.size(), hipMemcpyDeviceToHost));
    for (int y = 0; y < own; ++y)
        for (int x = 0; x < g.W; ++x) {
            const size_t s = (size_t)y * g.lab_pitch + x, d = 4 * ((size_t)y * g.W + x);
            lab4[d] = L[s]; lab4[d + 1] = A[s]; lab4[d + 2] = B[s]; lab4[d + 3] = 0.f;
        }
    return HQ_OK;
}

int hq_eval_population_partial(hq_ctx* c, const float* palettes, int P, int K, double* partial) {
    if (!partial) return fail(c, HQ_ERR_ARG, "null output");
    int rc = eval_partial_into_hout(c, palettes, P, K);
    if (rc) return rc;
    std::memcpy(partial, c->h_out, sizeof(double) * (size_t)P * (1 + K));
    return HQ_OK;
}

int hq_eval_population(hq_ctx* c, const float* palettes, int P, int K, float delta,
                       double* costs, int32_t* used) {
    if (!costs) return fail(c, HQ_ERR_ARG, "null output");
    int rc = eval_partial_into_hout(c, palettes, P, K);
    if (rc) return rc;
    // IM:712: averageArray(error) + computePenalty(used).  After an all-reduce
    // the used entries count the ranks using colour k; unused <=> 0.
    const bool full = c->g.r0 == 0 && c->g.r1 == c->g.H;
    if ((!full || c->slice_ranks > 1) && !(c->comm && c->nranks > 1))
        return fail(c, HQ_ERR_STATE, "sharded context or palette slice without a communicator: use "
                                     "hq_eval_population_partial");
    const double n_total = (double)c->g.W * (double)c->g.H;
    for (int p = 0; p < P; ++p) {
        const double* o = c->h_out + (size_t)p * (1 + K);
        double penalty = 0.0;
        for (int k = 0; k < K; ++k) {
            const bool u = o[1 + k] != 0.0;
            if (!u) penalty += delta;
            if (used) used[(size_t)p * K + k] = u ? 1 : 0;
        }
        costs[p] = o[0] / n_total + penalty;
    }
    return HQ_OK;
}

int hq_get_indices(hq_ctx* c, int p, uint8_t* idx) {
    if (!c || !idx) return HQ_ERR_ARG;
    if (p < 0 || p >= c->last_P) return fail(c, HQ_ERR_ARG, "palette %d not in last population", p);
    if (p < c->slice_lo || p >= c->slice_lo + c->slice_n)
        return fail(c, HQ_ERR_ARG, "palette %d was evaluated on another rank (palette split)", p);
    p -= c->slice_lo;
    if (c->K_cur > kMaxK)
        return fail(c, HQ_ERR_STATE, "K=%d > 256: indices are 32-bit (hq_get_indices32)", c->K_cur);
    int rc = bind(c);
    if (rc) return rc;
    const Geom& g = c->g;
    const int64_t off = (int64_t)(g.r0 - g.e0) * g.W;
    const int64_t n_own = (int64_t)g.W * (g.r1 - g.r0);
    HIP_TRY(c, hipMemcpy(idx, c->d_idx.as<uint8_t>() + (int64_t)p * g.idx_pitch + off, n_own,
                         hipMemcpyDeviceToHost));
    return HQ_OK;
}

int hq_get_indices32(hq_ctx* c, int p, uint32_t* idx) {
    if (!c || !idx) return HQ_ERR_ARG;
    if (p < 0 || p >= c->last_P) return fail(c, HQ_ERR_ARG, "palette %d not in last population", p);
    if (p < c->slice_lo || p >= c->slice_lo + c->slice_n)
        return fail(c, HQ_ERR_ARG, "palette %d was evaluated on another rank (palette split)", p);
    p -= c->slice_lo;
    int rc = bind(c);
    if (rc) return rc;
    const Geom& g = c->g;
    const int64_t off = (int64_t)(g.r0 - g.e0) * g.W;
    const int64_t n_own = (int64_t)g.W * (g.r1 - g.r0);
    if (c->last_nch > 1) {  // chunked palettes: 16-bit indices
        std::vector<uint16_t> b((size_t)n_own);
        HIP_TRY(c, hipMemcpy(b.data(), c->d_idx16.as<uint16_t>() + (int64_t)p * g.idx_pitch + off,
                             sizeof(uint16_t) * n_own, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < n_own; ++i) idx[i] = b[i];
        return HQ_OK;
    }
    if (c->K_cur > kMaxK) {
        HIP_TRY(c, hipMemcpy(idx, c->d_idx32.as<uint32_t>() + (int64_t)p * g.idx_pitch + off,
                             sizeof(uint32_t) * n_own, hipMemcpyDeviceToHost));
        return HQ_OK;
    }
    std::vector<uint8_t> b((size_t)n_own);
    HIP_TRY(c, hipMemcpy(b.data(), c->d_idx.as<uint8_t>() + (int64_t)p * g.idx_pitch + off, n_own,
                         hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n_own; ++i) idx[i] = b[i];
    return HQ_OK;
}

int hq_get_pixel_errors(hq_ctx* c, int p, float* err) {
    if (!c || !err) return HQ_ERR_ARG;
    if (!c->pixel_err) return fail(c, HQ_ERR_STATE, "option pixel_err is off");
    if (p < 0 || p >= c->last_P) return fail(c, HQ_ERR_ARG, "palette %d not in last population", p);
    if (p < c->slice_lo || p >= c->slice_lo + c->slice_n)
        return fail(c, HQ_ERR_ARG, "palette %d was evaluated on another rank (palette split)", p);
    p -= c->slice_lo;
    if (c->d_pixerr.bytes < sizeof(float) * (size_t)c->last_P * (size_t)c->g.W * (c->g.r1 - c->g.r0))
        return fail(c, HQ_ERR_STATE, "pixel_err was set after the last evaluation");
    int rc = bind(c);
    if (rc) return rc;
    const int64_t n_own = (int64_t)c->g.W * (c->g.r1 - c->g.r0);
    HIP_TRY(c, hipMemcpy(err, c->d_pixerr.as<float>() + (int64_t)p * n_own, sizeof(float) * n_own,
                         hipMemcpyDeviceToHost));
    return HQ_OK;
}

int hq_rgb_to_xyz(hq_ctx* c, const float* R, const float* G, const float* B, int64_t n,
                  float* xyz4) {
    if (!c || !R || !G || !B || !xyz4 || n < 1) return HQ_ERR_ARG;
    int rc = bind(c);
    if (rc) return rc;
    DevBuf dr, dg, db, dx;
    HIP_TRY(c, dr.ensure(sizeof(float) * n));
    HIP_TRY(c, dg.ensure(sizeof(float) * n));
    HIP_TRY(c, db.ensure(sizeof(float) * n));
    HIP_TRY(c, dx.ensure(sizeof(float4) * n));
    HIP_TRY(c, hipMemcpyAsync(dr.p, R, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(dg.p, G, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(db.p, B, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, launch_rgb_to_xyz(dr.as<float>(), dg.as<float>(), db.as<float>(), dx.as<float4>(), n,
                                 c->stream));
    HIP_TRY(c, hipMemcpyAsync(xyz4, dx.p, sizeof(float4) * n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return HQ_OK;
}

int hq_xyz_to_scielab(hq_ctx* c, const float* xyz4, int w, int h, const float* illum,
                      float* lab4) {
    if (!c || !xyz4 || !lab4) return HQ_ERR_ARG;
    int rc = check_geom_args(c, w, h, 0, h);
    if (rc) return rc;
    if ((rc = bind(c))) return rc;
    const Geom g = make_geom(w, h, 0, h, c->half);
    const int64_t n = (int64_t)w * h;
    DevBuf dxyz, opp, tmp, conv, k3v, ak3v;
    HIP_TRY(c, dxyz.ensure(sizeof(float4) * n));
    HIP_TRY(c, opp.ensure(sizeof(float4) * n));
    HIP_TRY(c, tmp.ensure(sizeof(float4) * n));
    HIP_TRY(c, conv.ensure(sizeof(float4) * n));
    std::vector<float> k3h(4 * c->taps, 0.f), ak3h(4 * c->taps, 0.f);
    for (int t = 0; t < c->taps; ++t) { k3h[4 * t] = c->k3[t]; ak3h[4 * t] = c->absk3[t]; }
    HIP_TRY(c, k3v.ensure(sizeof(float) * k3h.size()));
    HIP_TRY(c, ak3v.ensure(sizeof(float) * ak3h.size()));
    HIP_TRY(c, hipMemcpyAsync(k3v.p, k3h.data(), sizeof(float) * k3h.size(), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(ak3v.p, ak3h.data(), sizeof(float) * ak3h.size(), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(dxyz.p, xyz4, sizeof(float4) * n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, launch_xyz_to_opp(dxyz.as<float4>(), opp.as<float4>(), n, c->stream));
    const float* hk[3] = {c->d_k1.as<float>(), c->d_k2.as<float>(), k3v.as<float>()};
    const float* vk[3] = {c->d_k1.as<float>(), c->d_k2.as<float>(), ak3v.as<float>()};
    for (int f = 0; f < 3; ++f) {
        const int chans = f < 2 ? 3 : 1;
        HIP_TRY(c, launch_labref_hconv(opp.as<float4>(), tmp.as<float4>(), hk[f], c->half, chans,
                                       w, n, c->stream));
        HIP_TRY(c, launch_labref_vconv(tmp.as<float4>(), conv.as<float4>(), vk[f], c->half, chans,
                                       f > 0, g, c->stream));
    }
    const float* il = illum ? illum : c->illum;
    HIP_TRY(c, launch_labref_lab(conv.as<float4>(), nullptr, nullptr, nullptr, dxyz.as<float4>(), w,
                                 n, 0, il, c->stream));
    HIP_TRY(c, hipMemcpyAsync(lab4, dxyz.p, sizeof(float4) * n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return HQ_OK;
}

int hq_quantize(hq_ctx* c, const float* rgba4, int64_t n, const float* colors, int K, float* out4,
                int32_t* used) {
    if (!c || !rgba4 || !colors || !out4 || n < 1 || K < 1) return HQ_ERR_ARG;
    int rc = bind(c);
    if (rc) return rc;
    DevBuf din, dcol, dused, dout;
    HIP_TRY(c, din.ensure(sizeof(float4) * n));
    HIP_TRY(c, dcol.ensure(sizeof(float4) * K));
    HIP_TRY(c, dused.ensure(sizeof(int) * K));
    HIP_TRY(c, dout.ensure(sizeof(float4) * n));
    HIP_TRY(c, hipMemcpyAsync(din.p, rgba4, sizeof(float4) * n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(dcol.p, colors, sizeof(float4) * K, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemsetAsync(dused.p, 0, sizeof(int) * K, c->stream));
    HIP_TRY(c, launch_quantize(din.as<float4>(), dcol.as<float4>(), K, dused.as<int>(),
                               dout.as<float4>(), n, c->stream));
    HIP_TRY(c, hipMemcpyAsync(out4, dout.p, sizeof(float4) * n, hipMemcpyDeviceToHost, c->stream));
    if (used)
        HIP_TRY(c, hipMemcpyAsync(used, dused.p, sizeof(int) * K, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return HQ_OK;
}

int hq_compute_error(hq_ctx* c, const float* orig4, const float* quant4, int64_t n,
                     float* err_img4, double* mean) {
    if (!c || !orig4 || !quant4 || n < 1 || !mean) return HQ_ERR_ARG;
    if (c->de_type == HQ_DE_CIEDE2000)
        return fail(c, HQ_ERR_UNSUPPORTED, "CIEDE2000 is unimplemented in the reference (CL:227-230)");
    int rc = bind(c);
    if (rc) return rc;
    const int64_t nb = (n + 255) / 256;
    DevBuf da, db, de, dp;
    HIP_TRY(c, da.ensure(sizeof(float4) * n));
    HIP_TRY(c, db.ensure(sizeof(float4) * n));
    if (err_img4) HIP_TRY(c, de.ensure(sizeof(float4) * n));
    HIP_TRY(c, dp.ensure(sizeof(double) * nb));
    HIP_TRY(c, hipMemcpyAsync(da.p, orig4, sizeof(float4) * n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(db.p, quant4, sizeof(float4) * n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, launch_error_image(da.as<float4>(), db.as<float4>(), err_img4 ? de.as<float4>() : nullptr,
                                  dp.as<double>(), n, c->de_type, c->stream));
    std::vector<double> parts(nb);
    HIP_TRY(c, hipMemcpyAsync(parts.data(), dp.p, sizeof(double) * nb, hipMemcpyDeviceToHost, c->stream));
    if (err_img4)
        HIP_TRY(c, hipMemcpyAsync(err_img4, de.p, sizeof(float4) * n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    double s = 0.0;
    for (double v : parts) s += v;
    *mean = s / (double)n;  // IM:893
    return HQ_OK;
}

int hq_comm_unique_id(unsigned char id[128]) {
    if (!id) return HQ_ERR_ARG;
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return HQ_ERR_COMM;
    std::memcpy(id, &u, 128);
    return HQ_OK;
}

int hq_comm_init(hq_ctx* c, int nranks, int rank, const unsigned char id[128]) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return HQ_ERR_ARG;
    int rc = bind(c);
    if (rc) return rc;
    if (c->comm) { (void)ncclCommDestroy(c->comm); c->comm = nullptr; }
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    NCCL_TRY(c, ncclCommInitRank(&c->comm, nranks, u, rank));
    c->nranks = nranks;
    c->rank = rank;
    return HQ_OK;
}

int hq_comm_info(hq_ctx* c, int* nranks, int* rank) {
    if (!c || !nranks || !rank) return HQ_ERR_ARG;
    *nranks = 0;
    *rank = -1;
    if (!c->comm) return HQ_OK;
    // what the communicator itself reports, not what hq_comm_init was asked for
    NCCL_TRY(c, ncclCommCount(c->comm, nranks));
    NCCL_TRY(c, ncclCommUserRank(c->comm, rank));
    return HQ_OK;
}

int hq_search_create(hq_ctx* c, const hq_swasa_params* params, int K, uint64_t seed,
                     hq_search** out) {
    if (!c || !params || !out) return HQ_ERR_ARG;
    *out = nullptr;
    if (params->population < 1 || params->imax < 1 || params->iTc < 1 || K < 1)
        return fail(c, HQ_ERR_ARG, "bad SWASA parameters");
    // device-resident: K <= 256, or chunked palettes (256 < K <= 16384); at most
    // kSaMaxP palettes (sa_step's per-palette tables) and kSaMaxSub sub-palettes
    // (its fold reads 8 used words per sub-palette, at most 4 per thread)
    const int nch = K > kMaxK && K <= kMaxKChunked && c->chunked && c->G2 > 0 ? chunk_count(K) : 1;
    const bool device = c->sa_device && params->population <= kSaMaxP && params->population * nch <= kSaMaxSub &&
                        (K <= kMaxK || nch > 1);
    hq_search* s = new hq_search{c, nullptr, K};
    int rc;
    if (device) {
        if (!c->have_image) rc = fail(c, HQ_ERR_STATE, "no image set (hq_set_image)");
        else if (c->de_type == HQ_DE_CIEDE2000)
            rc = fail(c, HQ_ERR_UNSUPPORTED, "CIEDE2000 is unimplemented in the reference (CL:227-230)");
        else rc = bind(c);
        if (rc) {
            hq_search_destroy(s);
            return rc;
        }
        const bool full = c->g.r0 == 0 && c->g.r1 == c->g.H;
        if (!full && !(c->comm && c->nranks > 1) && !c->shard_solo) {
            hq_search_destroy(s);
            return fail(c, HQ_ERR_STATE, "sharded context without a communicator");
        }
        s->nch = nch;
        rc = device_search_create(c, params, K, seed, s);
    } else {
        const float delta = params->delta;
        auto eval = [c, delta](const float* pal, int P, int KK, double* costs) {
            return hq_eval_population(c, pal, P, KK, delta, costs, nullptr);
        };
        s->driver = new SearchDriver(*params, K, seed, eval);
        rc = s->driver->start();
    }
    if (rc) {
        hq_search_destroy(s);
        return rc;
    }
    *out = s;
    return HQ_OK;
}

int hq_search_run(hq_search* s, int iterations, int* ran) {
    if (!s || iterations < 0) return HQ_ERR_ARG;
    if (!s->driver) {
        int rc = bind(s->ctx);
        return rc ? rc : device_search_run(s, iterations, ran);
    }
    return s->driver->run(iterations, ran, nullptr);
}

int hq_search_best(const hq_search* s, float* colors, double* best_error, int* iteration) {
    if (!s) return HQ_ERR_ARG;
    if (!s->driver) {
        hq_ctx* c = s->ctx;
        int rc = bind(c);
        if (rc) return rc;
        if (colors)
            HIP_TRY(c, hipMemcpy(colors, s->best_colors.p, sizeof(float) * 4 * s->K, hipMemcpyDeviceToHost));
        if (best_error)
            HIP_TRY(c, hipMemcpy(best_error, s->best_err[s->st].p, sizeof(double), hipMemcpyDeviceToHost));
        if (iteration) *iteration = s->ite;
        return HQ_OK;
    }
    if (colors) std::copy(s->driver->best_colors().begin(), s->driver->best_colors().end(), colors);
    if (best_error) *best_error = s->driver->best_error();
    if (iteration) *iteration = s->driver->iteration();
    return HQ_OK;
}

void hq_search_destroy(hq_search* s) {
    if (!s) return;
    if (!s->driver && s->ctx) {
        (void)hipSetDevice(s->ctx->device);
        (void)hipStreamSynchronize(s->ctx->stream);
    }
    for (hipEvent_t e : s->pev) (void)hipEventDestroy(e);
    if (s->gexec) (void)hipGraphExecDestroy(s->gexec);
    for (DevBuf* b : {&s->colors[0], &s->colors[1], &s->cand[0], &s->cand[1], &s->err[0], &s->err[1],
                      &s->seed[0], &s->seed[1], &s->best_err[0], &s->best_err[1], &s->best_colors, &s->jA,
                      &s->jC})
        b->release();
    delete s->pol;
    delete s->driver;
    delete s;
}

int hq_profile_enable(hq_ctx* c, int on) {
    if (!c) return HQ_ERR_ARG;
    c->prof = on != 0;
    return HQ_OK;
}

int hq_profile_reset(hq_ctx* c) {
    if (!c) return HQ_ERR_ARG;
    c->prof_assign = c->prof_cost = c->prof_grid = c->prof_finalize = c->prof_sa = c->prof_comm = ProfSlot{};
    return HQ_OK;
}

int hq_profile_get(hq_ctx* c, const char* kernel, double* total_ms, int64_t* launches) {
    if (!c || !kernel) return HQ_ERR_ARG;
    const ProfSlot* s = nullptr;
    if (!std::strcmp(kernel, "assign")) s = &c->prof_assign;
    else if (!std::strcmp(kernel, "cost")) s = &c->prof_cost;
    else if (!std::strcmp(kernel, "grid")) s = &c->prof_grid;
    else if (!std::strcmp(kernel, "finalize")) s = &c->prof_finalize;
    else if (!std::strcmp(kernel, "sa_step")) s = &c->prof_sa;
    else if (!std::strcmp(kernel, "comm")) s = &c->prof_comm;
    else return fail(c, HQ_ERR_ARG, "unknown kernel '%s'", kernel);
    if (total_ms) *total_ms = s->ms;
    if (launches) *launches = s->launches;
    return HQ_OK;
}

int hq_set_option(hq_ctx* c, const char* name, int value) {
    if (!c || !name) return HQ_ERR_ARG;
    if (!std::strcmp(name, "grid")) {
        if (value != 0 && value != 16 && value != 32 && value != 64)
            return fail(c, HQ_ERR_ARG, "grid must be 0, 16, 32 or 64");
        c->G2 = value;
    } else if (!std::strcmp(name, "cost_variant")) {
        if (value < 0 || value > 2) return fail(c, HQ_ERR_ARG, "cost_variant must be 0, 1 or 2");
        c->cost_variant = value;
    } else if (!std::strcmp(name, "trim")) {
        c->trim = value != 0;
    } else if (!std::strcmp(name, "cost_rows")) {
        if (value != 8 && value != 16) return fail(c, HQ_ERR_ARG, "cost_rows must be 8 or 16");
        c->cost_rows = value;
    } else if (!std::strcmp(name, "sa_graph")) {
        c->sa_graph = value != 0;
    } else if (!std::strcmp(name, "gen_hrow_outputs")) {
        if (value != 4 && value != 8) return fail(c, HQ_ERR_ARG, "gen_hrow_outputs must be 4 or 8");
        c->gen_hrow_no = value;
    } else if (!std::strcmp(name, "gen_vmfma")) {
        c->gen_vmfma = value != 0;
    } else if (!std::strcmp(name, "gen_hmfma")) {
        c->gen_hmfma = value != 0;
    } else if (!std::strcmp(name, "gen_tile_shape")) {
        if (value < 0 || value > 2) return fail(c, HQ_ERR_ARG, "gen_tile_shape: 0, 1 or 2");
        c->gen_shape = (int)value;
    } else if (!std::strcmp(name, "gen_vtile2")) {
        c->gen_vtile2 = value != 0;
    } else if (!std::strcmp(name, "gen_hrow4")) {
        c->gen_hrow4 = value != 0;
    } else if (!std::strcmp(name, "cost_tw")) {
        if (value != 128 && value != 256) return fail(c, HQ_ERR_ARG, "cost_tw must be 128 or 256");
        c->cost_tw = value;

    } else if (!std::strcmp(name, "sa_device")) {
        c->sa_device = value != 0;
    } else if (!std::strcmp(name, "shard_solo")) {
        c->shard_solo = value != 0;
    } else if (!std::strcmp(name, "palette_split")) {
        c->psplit = value != 0;
    } else if (!std::strcmp(name, "slice_ranks")) {
        if (value < 1) return fail(c, HQ_ERR_ARG, "slice_ranks must be >= 1");
        c->slice_ranks = value;
    } else if (!std::strcmp(name, "slice_rank")) {
        // (checked against slice_ranks again at each evaluation: the options may come in either order)
        if (value < 0) return fail(c, HQ_ERR_ARG, "slice_rank must be >= 0");
        c->slice_rank = value;
    } else if (!std::strcmp(name, "fold_blocks")) {
        if (value < 1 || value > 64) return fail(c, HQ_ERR_ARG, "fold_blocks in [1, 64]");
        c->fold_blocks = value;
        c->fold_block = 0;
    } else if (!std::strcmp(name, "fold_block")) {
        if (value < 0 || value >= c->fold_blocks) return fail(c, HQ_ERR_ARG, "fold_block in [0, fold_blocks)");
        c->fold_block = value;
    } else if (!std::strcmp(name, "lists16")) {
        if (value < 0 || value > 2) return fail(c, HQ_ERR_ARG, "lists16: 0, 1 or 2");
        c->lists16 = (int)value;
        if (!value) {  // (the lists' 10 MiB per palette are re-allocated when turned on again)
            c->d_l1n.release();
            c->d_l2n.release();
        }
    } else if (!std::strcmp(name, "chunked")) {
        c->chunked = value != 0;
    } else if (!std::strcmp(name, "pixel_err")) {
        c->pixel_err = value != 0;
    } else if (!std::strcmp(name, "img_u8")) {
        c->img_u8_path = value != 0;
    } else if (!std::strcmp(name, "assign_blocks_per_cu")) {
        if (value < 0 || value > 64) return fail(c, HQ_ERR_ARG, "assign_blocks_per_cu in [0,64] (0 = auto)");
        c->assign_blocks_per_cu = value;
    } else {
        return fail(c, HQ_ERR_ARG, "unknown option '%s'", name);
    }
    return HQ_OK;
}

}  // extern "C"
