/*
 * hq.h -- C ABI of libhq, the MI355X-native SWASA dE cost evaluator.
 *
 * Drop-in boundary: every entry point below replaces one method of the
 * reference's JavaCL backend `ImageManipulation` (IM) or its helpers, and is
 * what a JNI shim bound to that class calls (INTEGRATION.md shows the Java
 * side).  Reference files live under
 *   /root/reference/src/plugins/dbrasseur/hybridquantization/
 * with tags IM = ImageManipulation.java, SP = ScielabProcessor.java,
 * SW = SWASA.java, HQ = HybridQuantization.java, CL = OptimizedConvolution.cl.
 *
 * Conventions
 *  - Plain C types only; host pointers are caller-owned and only read/written
 *    for the duration of the call.
 *  - "inline float4" = the reference's RGBA / Lab layout: float[4*N], pixel
 *    p = y*w + x at [4p .. 4p+3], .w = 0 (HQ:279-291 makeinline).
 *  - Palettes: float[4*K] per palette with .w = 0 (SW:40-52); populations are
 *    P palettes back to back.
 *  - Every function returns HQ_OK (0) or a positive HQ_ERR_* code; the message
 *    of the last failure is available from hq_last_error(ctx).  The JNI shim
 *    maps a non-zero status to an exception (IM:79-92 fallback semantics).
 *  - One host thread per context at a time (IM's single in-order queue).
 */
#ifndef HQ_H
#define HQ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HQ_VERSION 1

enum hq_status {
    HQ_OK = 0,
    HQ_ERR_ARG = 1,          /* invalid argument / shape */
    HQ_ERR_DEVICE = 2,       /* HIP runtime failure or no device */
    HQ_ERR_STATE = 3,        /* call order violated (e.g. no image set) */
    HQ_ERR_UNSUPPORTED = 4,  /* valid request outside what this build supports */
    HQ_ERR_COMM = 5,         /* RCCL failure */
    HQ_ERR_NOMEM = 6
};

/* IM:20 enum deltaETypes.  CIE76 is what the plugin always uses (HQ:96, HQ:145). */
enum hq_delta_e { HQ_DE_CIE76 = 0, HQ_DE_CIE94 = 1, HQ_DE_CIEDE2000 = 2 };

/* SP:19 enum Whitepoint */
enum hq_whitepoint { HQ_WP_D50 = 0, HQ_WP_D65 = 1 };

typedef struct hq_ctx hq_ctx;
typedef struct hq_search hq_search;

int hq_version(void);
const char *hq_status_string(int status);
/* Number of visible HIP devices (0 when none).  Never initialises a context. */
int hq_device_count(int *count);

/* IM:52 ImageManipulation(deltaEType, verbose, convergence): binds `device`,
 * creates the context's stream.  Fails with HQ_ERR_DEVICE when no GPU is
 * usable -- the caller's fallback path of IM:79-92. */
int hq_create(int device, int delta_e_type, hq_ctx **out);
/* IM:265 close(): releases every device buffer, stream and communicator. */
void hq_destroy(hq_ctx *ctx);
const char *hq_last_error(const hq_ctx *ctx);

/* SP:66-181 ScielabProcessor constructor (filter design) followed by the
 * packing of IM:800-841.  Host-only.  Writes k1[4*T], k2[4*T] (float4 taps:
 * channel filters (g0j, g1j, g2j, 0)), k3[T] = g02 and absk3[T] = |g02|;
 * *taps = T, illum[3] = whitepoint.  Buffers must hold max_taps taps. */
int hq_design_filters(int dpi, double viewing_distance, int whitepoint, int max_taps,
                      float *k1, float *k2, float *k3, float *absk3, int *taps,
                      float *illum);

/* IM:800 updateOpenCLFilters(filters, absfilters): uploads the packed taps.
 * halfSize = (4*taps)/8 as IM:408. */
int hq_set_filters(hq_ctx *ctx, int taps, const float *k1, const float *k2, const float *k3,
                   const float *absk3);

/* IM:100 RGBtoXYZ: planar R,G,B (n floats each) -> inline XYZ float4 (CL:79-90). */
int hq_rgb_to_xyz(hq_ctx *ctx, const float *R, const float *G, const float *B, int64_t n,
                  float *xyz4);
/* IM:285 XYZtoScielab(XYZ, filters, absfilters, w, illuminant): inline XYZ ->
 * inline S-CIELAB Lab (CL:111-116, CL:2-74 filter by filter, CL:124-145). */
int hq_xyz_to_scielab(hq_ctx *ctx, const float *xyz4, int w, int h, const float *illum,
                      float *lab4);

/* Device-resident state of IM:383 findBestQuantization (IM:450-478):
 * uploads the inline RGBA image and its S-CIELAB (inline Lab float4) once.
 * lab4 may be NULL: the S-CIELAB of the image is then computed on the device
 * (IM:100 + IM:285 semantics).  Requires w, h >= halfSize. */
int hq_set_image(hq_ctx *ctx, const float *rgba4, const float *lab4, int w, int h,
                 const float *illum);
/* Row-block shard of a (w x h) image for multi-GPU evaluation:
 * this context owns rows [row_begin, row_end); rgba4/lab4 point at the FULL
 * image (only the owned rows +- halfSize halo rows are read). */
int hq_set_image_shard(hq_ctx *ctx, const float *rgba4, const float *lab4, int w, int h,
                       const float *illum, int row_begin, int row_end);
/* Same as hq_set_image_shard but planar float R,G,B of the FULL image (no Lab:
 * it is always computed on the device).  Used by bench.py. */
int hq_set_image_planar_shard(hq_ctx *ctx, const float *R, const float *G, const float *B,
                              int w, int h, const float *illum, int row_begin, int row_end);
/* Reads back the device S-CIELAB of the owned rows as inline float4. */
int hq_get_labref(hq_ctx *ctx, float *lab4);

/* IM:620 computeQuantizationErrorPopulation for P palettes of K colours
 * (K in [1, 2^24] as the plugin allows, HQ:192).  K <= 256: the pruned grid
 * argmin and the tiled fast stencil.  256 < K <= 16384: chunked palettes (nch
 * sub-palettes of 256, 16-bit indices; 512 < K <= 8192: one grid of 16-bit
 * candidate lists over all K colours, option "lists16", otherwise a grid and
 * assign pass per chunk; the fast stencil up to K = 8192, the generic one
 * above; option "chunked").  K > 16384,
 * palettes with non-finite colours or
 * outside the fast path's range, option "chunked" 0 or "grid" 0: the exhaustive
 * argmin with 32-bit indices and the generic stencil path.  All give the same
 * indices and used flags (bit-exact) and the same cost (1e-6 relative):
 * costs[p] = mean dE76 + delta * #unused (IM:712, SW:74-82); used[p*K+k] in
 * {0,1} (CL:193), may be NULL.  On a sharded context with a communicator the
 * partial sums are all-reduced over RCCL first. */
int hq_eval_population(hq_ctx *ctx, const float *palettes, int P, int K, float delta,
                       double *costs, int32_t *used);
/* Shard-local partial results without the all-reduce: partial[p*(1+K)] = fp64
 * sum of dE over the owned rows, partial[p*(1+K)+1+k] = 1.0 if colour k is used
 * by an owned-or-halo pixel else 0.0. */
int hq_eval_population_partial(hq_ctx *ctx, const float *palettes, int P, int K,
                               double *partial);
/* Per-pixel palette indices (u8, K <= 256) of the last evaluated population's
 * palette p over the owned rows (w*(row_end-row_begin) bytes).  HQ_ERR_STATE
 * when that population had K > 256 colours. */
int hq_get_indices(hq_ctx *ctx, int p, uint8_t *idx);
/* The same for any K (1 .. 2^24, HQ:192): 32-bit indices, w*(row_end-row_begin)
 * of them -- the reference's int index of CL:172-193. */
int hq_get_indices32(hq_ctx *ctx, int p, uint32_t *idx);
/* Test surface: the per-pixel dE of palette p of the last evaluation over the
 * owned rows (w*(row_end-row_begin) floats) -- the error image the reference
 * reads back per member (IM:663-667, CL:201-209).  Needs option "pixel_err" = 1
 * before that evaluation (the cost kernels then also store it); HQ_ERR_STATE
 * otherwise. */
int hq_get_pixel_errors(hq_ctx *ctx, int p, float *err);

/* IM:770 quantize(inlineImageRGB, colors): chosen colour per pixel (CL:147-170).
 * used (K ints) may be NULL. */
int hq_quantize(hq_ctx *ctx, const float *rgba4, int64_t n, const float *colors, int K,
                float *out4, int32_t *used);
/* IM:858 computeError(original, quantized, errorImage): mean dE (configured
 * type) and errImg4 = (255-e)^2/255^2 replicated in .xyz (IM:886-893). */
int hq_compute_error(hq_ctx *ctx, const float *orig4, const float *quant4, int64_t n,
                     float *err_img4, double *mean);

/* RCCL communicator over xGMI for row-block sharded evaluation.
 * Rank 0 calls hq_comm_unique_id and ships the 128 bytes to every rank. */
int hq_comm_unique_id(unsigned char id[128]);
int hq_comm_init(hq_ctx *ctx, int nranks, int rank, const unsigned char id[128]);
/* The ranks of the context's communicator as RCCL reports them (ncclCommCount,
 * ncclCommUserRank); *nranks = 0 and *rank = -1 without one.  bench.py reports
 * it next to its own world size. */
int hq_comm_info(hq_ctx *ctx, int *nranks, int *rank);

/* SWASA parameters (SW:14-28; GUI defaults HQ:192-224). */
typedef struct hq_swasa_params {
    int population;      /* 4    */
    int imax;            /* 5000 */
    int iTc;             /* 20   */
    float delta;         /* 2    */
    float conv_delay;    /* 0.75 */
    float conv_spread;   /* 0.15 */
    float t0;            /* 20   */
    float alpha;         /* 0.9  */
    float s0;            /* 100  */
    float beta;          /* 5.3  */
    int convergence;     /* 1    */
} hq_swasa_params;

void hq_swasa_default_params(hq_swasa_params *p);

/* IM:383-591 findBestQuantization as a resumable search: create() draws the
 * initial population (SW:40-52) with a java.util.Random-compatible generator
 * seeded with `seed`, evaluates it; run() advances up to `iterations` SA
 * iterations (IM:497-568) and reports how many ran; a JNI caller checks its
 * stop flag between run() calls (IM:499). */
int hq_search_create(hq_ctx *ctx, const hq_swasa_params *params, int K, uint64_t seed,
                     hq_search **out);
int hq_search_run(hq_search *s, int iterations, int *ran);
int hq_search_best(const hq_search *s, float *colors, double *best_error, int *iteration);
void hq_search_destroy(hq_search *s);

/* Host-only SWASA driver with a caller-supplied population evaluator; same
 * policy code as hq_search_*.  Used to test the SA semantics without a GPU.
 * eval(user, palettes[P*K*4], P, K, costs[P]) returns 0 on success.
 * trace (optional) receives per iteration: best_error then the P errors. */
typedef int (*hq_eval_fn)(void *user, const float *palettes, int P, int K, double *costs);
int hq_swasa_search_host(const hq_swasa_params *params, int K, uint64_t seed, int iterations,
                         hq_eval_fn eval, void *user, float *best_colors, double *best_error,
                         double *trace);

/* Kernel timing of the dominant kernels, measured with HIP events on the
 * context stream while enabled (bench.py roofline). */
int hq_profile_enable(hq_ctx *ctx, int on);
/* names: "assign", "cost", "grid", "finalize", "sa_step" (device-resident search), "comm" (the
 * per-evaluation RCCL all-reduce or all-gather, with a communicator); returns total ms and launch
 * count (HIP events on the context stream). */
int hq_profile_get(hq_ctx *ctx, const char *kernel, double *total_ms, int64_t *launches);
int hq_profile_reset(hq_ctx *ctx);

/* Tuning knobs (testing / benchmarking; defaults are the measured best).  They
 * may change between calls, also between hq_search_run calls of one search:
 * every evaluation sizes the context's work buffers for the options and image
 * in force when it is enqueued.
 *   "grid"         argmin pruning resolution G2: 0 = exhaustive, 16, 32 (default), 64
 *   "cost_variant" 0 = fast tiled path (default; filters up to halfSize 24), 1 = generic
 *                  two-pass path, LDS-tiled (any filter length; halfSize > 24 takes it),
 *                  2 = the generic pair per pixel in the reference's summation order
 *   "gen_hrow4"    the LDS-tiled generic path's horizontal pass: 1 (default) = 4 adjacent
 *                  outputs per thread over a sliding window, 0 = one output per thread
 *                  (same planes bit for bit)
 *   "gen_vmfma"    the LDS-tiled generic path's vertical pass (halfSize <= 64) on the matrix
 *                  cores in split f16 (as the fast path's; default 1), 0 = fp32 FMAs (gen_vtile2)
 *   "gen_hmfma"    with gen_vmfma: the horizontal pass on the matrix cores too (default 1;
 *                  palettes in the fast range), 0 = fp32 FMAs (gen_hrow4)
 *   "gen_tile_shape" the matrix-core generic pair's workgroup shapes: 0 (default) by grid size
 *                  (4 row tiles per gen_hmfma workgroup and 128-row gen_vmfma tiles on large
 *                  images), 1 the short forms, 2 the tall forms (same results within the split bars)
 *   "lists16"      chunked palettes: native 16-bit candidate lists (one grid over all K
 *                  colours, one lookup per pixel): 1 (default) for 4 to 32 chunks (512 < K
 *                  <= 8192), 2 for 2 .. 32 chunks, 0 = a grid and assign pass per chunk
 *   "gen_vtile2"   the LDS-tiled generic path's vertical pass (halfSize <= 64): 1 (default) =
 *                  32 x 64 tiles, windows double-buffered by LDS DMA; 0 = 64 x 64 tiles with
 *                  one window at a time (same results bit for bit)
 *   "cost_rows"    fast path tiles: 16 (16 x 128 outputs, default) or 8 (8 x 108)
 *   "cost_tw"      16-row tiles at the default filter width: 128 columns (4 waves,
 *                  default) or 256 (8 waves per workgroup)
 *   "trim"         1 = skip the narrow k1 filters' taps below 1e-9 of their peak
 *                  (default; only when the filters allow it), 0 = all taps
 *   "assign_blocks_per_cu" workgroups per CU of the assign grid (0 = default: one
 *                  resident round, at least 6 pixels per thread)
 *   "img_u8"       1 (default) = assign reads the packed 8-bit copy of an image whose
 *                  channels are all k/255; 0 = the planar floats
 *   "sa_device"    hq_search_*: 1 (default) = the SWASA iterations run on the device
 *                  (accept/generate kernel, no host round trip per iteration; needs
 *                  population <= 64), 0 = host-driven, one evaluation call each
 *   "sa_graph"     hq_search_*: 1 = each run's kernels captured into one hipGraph and
 *                  replayed (0, default: measured slower, 0.540 against 0.528 ms per C3 step)
 *   "shard_solo"   experiment only: let a row-block shard run hq_search_* without a
 *                  communicator (its own partial costs; per-rank timing at N GPUs)
 *   "pixel_err"    test only: 1 = the cost kernels also write the per-pixel dE
 *                  (hq_get_pixel_errors)
 *   "palette_split" 1 = with a communicator of N ranks, each holding the whole image
 *                  (hq_set_image): rank r evaluates palettes [r P/N, (r+1) P/N) and one
 *                  all-gather gives every rank all P results (SURVEY 8e's split of large
 *                  populations; P must divide by N); 0 (default) = row-block shards
 *   "slice_ranks", "slice_rank"  test only: the same palette slice without a
 *                  communicator (hq_eval_population_partial: other rows read 0) */
int hq_set_option(hq_ctx *ctx, const char *name, int value);

#ifdef __cplusplus
}
#endif
#endif /* HQ_H */
