/*
 * ref_cl_host.c -- TEST INFRASTRUCTURE ONLY: runs the reference's own OpenCL
 * kernels (OptimizedConvolution.cl, compiled unmodified for gfx950 by the
 * image's clang from /root/reference by oracle/Makefile into oracle/_ref/) on
 * the MI355X through the ROCm OpenCL runtime, in the order and with the
 * arguments the reference's JavaCL host code uses.  Only the host side is
 * restated here (JavaCL is absent); every per-pixel operation is the
 * reference's kernel code.  This pins the C/numpy oracle and libhq against the
 * reference itself.  Never linked into the product.
 *
 * Host sequences restated (tags: IM = ImageManipulation.java, CL =
 * OptimizedConvolution.cl, under /root/reference/src/plugins/dbrasseur/hybridquantization/):
 *  - hqref_rgb_to_xyz        IM:100-153  (RGB2XYZ, CL:79-90)
 *  - hqref_xyz_to_scielab    IM:285-370  (XYZ2Opp; convolve4Channels x4 and
 *                                         convolve1Channel x2 filter by filter with
 *                                         the update flag; Opp2LAB)
 *  - hqref_eval_population   IM:450-493 + IM:620-727 (per member: used flags
 *                            zeroed, quantizeAndConvertToOpp, computeScielabKernelsTemp,
 *                            computeScielabKernelsEnd with w and h swapped, Opp2LAB, CIEDE;
 *                            the mean of the error image, IM:736-768, here one
 *                            sequential double sum, plus delta * #unused, SW:74-82)
 *  - hqref_quantize          IM:770-798  (quantize, CL:147-170)
 *  - hqref_compute_error     IM:858-884  (CIEDE on two Lab images, CL:201-231)
 * Filters: k1_4 = filters4[0], k2_4 = filters4[1], k3_4 = filters4[2],
 * absk3_4 = absfilters4 (float4 per tap, IM:800-841), k3 = filter3, absk3 =
 * absfilter3 (scalar per tap).  Work sizes: one work item per pixel, local size
 * left to the runtime (JavaCL's enqueueNDRange(queue, int[]{N}), IM:406).
 * The program is built from the binary with no options (the binary was
 * compiled with -DCIE76, IM:63, HQ:96).
 */
#define _POSIX_C_SOURCE 199309L
#define CL_TARGET_OPENCL_VERSION 120
#include <CL/cl.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static cl_context g_ctx;
static cl_command_queue g_q;
static cl_program g_prog;
static cl_device_id g_dev;
static char g_bin[1024];  /* the binary g_prog was built from */
static char g_err[512];

static int fail(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return -1;
}

const char *hqref_error(void) { return g_err; }

/* The context and in-order queue on the first GPU device of the first
 * platform that has one (once). */
static int init_context(void) {
    if (g_ctx) return 0;
    cl_uint np = 0;
    cl_platform_id plats[8];
    if (clGetPlatformIDs(8, plats, &np) != CL_SUCCESS || np == 0) return fail("no OpenCL platform");
    cl_int e = CL_DEVICE_NOT_FOUND;
    for (cl_uint i = 0; i < np && e != CL_SUCCESS; ++i) {
        cl_uint nd = 0;
        e = clGetDeviceIDs(plats[i], CL_DEVICE_TYPE_GPU, 1, &g_dev, &nd);
        if (e == CL_SUCCESS && nd == 0) e = CL_DEVICE_NOT_FOUND;
    }
    if (e != CL_SUCCESS) return fail("no OpenCL GPU device (%d)", e);
    cl_context ctx = clCreateContext(NULL, 1, &g_dev, NULL, NULL, &e);
    if (e != CL_SUCCESS) return fail("clCreateContext %d", e);
    g_q = clCreateCommandQueue(ctx, g_dev, 0, &e);  /* in-order, as JavaCL's default queue (IM:59) */
    if (e != CL_SUCCESS) {
        clReleaseContext(ctx);
        return fail("clCreateCommandQueue %d", e);
    }
    g_ctx = ctx;
    return 0;
}

/* The program from binary_path; a different binary than the current one
 * replaces it (the -DCIE76 and -DCIE94 builds). */
int hqref_init(const char *binary_path) {
    if (g_prog && strcmp(binary_path, g_bin) == 0) return 0;
    if (init_context()) return -1;
    FILE *f = fopen(binary_path, "rb");
    if (!f) return fail("cannot open %s", binary_path);
    fseek(f, 0, SEEK_END);
    const long len = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char *bin = (unsigned char *)malloc((size_t)len);
    if (!bin || fread(bin, 1, (size_t)len, f) != (size_t)len) {
        fclose(f);
        free(bin);
        return fail("cannot read %s", binary_path);
    }
    fclose(f);
    if (g_prog) {
        clReleaseProgram(g_prog);
        g_prog = NULL;
        g_bin[0] = 0;
    }
    const unsigned char *bp = bin;
    const size_t bl = (size_t)len;
    cl_int st = 0, e = 0;
    cl_program prog = clCreateProgramWithBinary(g_ctx, 1, &g_dev, &bl, &bp, &st, &e);
    free(bin);
    if (e != CL_SUCCESS || st != CL_SUCCESS) return fail("clCreateProgramWithBinary %d / %d", e, st);
    e = clBuildProgram(prog, 1, &g_dev, "", NULL, NULL);
    if (e != CL_SUCCESS) {
        char log[256] = {0};
        clGetProgramBuildInfo(prog, g_dev, CL_PROGRAM_BUILD_LOG, sizeof log - 1, log, NULL);
        clReleaseProgram(prog);
        return fail("clBuildProgram %d: %s", e, log);
    }
    g_prog = prog;
    snprintf(g_bin, sizeof g_bin, "%s", binary_path);
    return 0;
}

/* ---- small helpers ---- */
/* Buffer and kernel creation keep the first error in *e (sticky: a later
 * success does not hide an earlier failure; *e starts at CL_SUCCESS). */
static cl_mem buf(size_t bytes, const void *src, cl_int *e) {
    cl_int r = CL_SUCCESS;
    cl_mem m = clCreateBuffer(g_ctx, CL_MEM_READ_WRITE | (src ? CL_MEM_COPY_HOST_PTR : 0), bytes ? bytes : 4,
                              (void *)src, &r);
    if (*e == CL_SUCCESS) *e = r;
    return r == CL_SUCCESS ? m : NULL;
}

static cl_kernel kern(const char *name, cl_int *e) {
    cl_int r = CL_SUCCESS;
    cl_kernel k = clCreateKernel(g_prog, name, &r);
    if (*e == CL_SUCCESS) *e = r;
    return r == CL_SUCCESS ? k : NULL;
}

static void release_mem(cl_mem m) {
    if (m) clReleaseMemObject(m);
}

static int run1d(cl_kernel k, size_t n) {
    const cl_int e = clEnqueueNDRangeKernel(g_q, k, 1, NULL, &n, NULL, 0, NULL, NULL);
    return e == CL_SUCCESS ? 0 : fail("enqueue %d", e);
}

#define ARG(k, i, v) clSetKernelArg((k), (i), sizeof(v), &(v))
#define CHK(x)                                                \
    do {                                                      \
        if ((x) != CL_SUCCESS) { rc = fail("%s failed", #x); goto out; } \
    } while (0)

/* IM:100-153: planar R, G, B -> inline XYZ (CL:79-90). */
int hqref_rgb_to_xyz(const float *R, const float *G, const float *B, int n, float *xyz4) {
    int rc = 0;
    cl_int e = CL_SUCCESS;
    cl_mem r = buf(4 * (size_t)n, R, &e), g = buf(4 * (size_t)n, G, &e), b = buf(4 * (size_t)n, B, &e),
           o = buf(16 * (size_t)n, NULL, &e);
    cl_kernel k = kern("RGB2XYZ", &e);
    if (e != CL_SUCCESS) { rc = fail("RGB2XYZ setup %d", e); goto out; }
    CHK(ARG(k, 0, r)); CHK(ARG(k, 1, g)); CHK(ARG(k, 2, b)); CHK(ARG(k, 3, o));
    if ((rc = run1d(k, (size_t)n))) goto out;
    CHK(clEnqueueReadBuffer(g_q, o, CL_TRUE, 0, 16 * (size_t)n, xyz4, 0, NULL, NULL));
out:
    if (k) clReleaseKernel(k);
    release_mem(r); release_mem(g); release_mem(b); release_mem(o);
    return rc;
}

/* IM:285-370: inline XYZ -> inline S-CIELAB Lab, filter by filter. */
int hqref_xyz_to_scielab(const float *xyz4, int w, int h, const float *k1_4, const float *k2_4,
                         const float *k3_4, const float *absk3_4, int taps, const float *illum, float *lab4) {
    int rc = 0;
    cl_int e = CL_SUCCESS;
    const size_t n = (size_t)w * h, fb = 16 * (size_t)taps;
    const int half = (4 * taps) / 8;  /* IM:299 filters4[0].length / 8 */
    cl_mem in = buf(16 * n, xyz4, &e), opp = buf(16 * n, NULL, &e), conv = buf(16 * n, NULL, &e),
           tmp = buf(16 * n, NULL, &e), lab = buf(16 * n, NULL, &e);
    cl_mem f1 = buf(fb, k1_4, &e), f2 = buf(fb, k2_4, &e), f3 = buf(fb, k3_4, &e), fa = buf(fb, absk3_4, &e);
    cl_kernel kx = kern("XYZ2Opp", &e), c4 = kern("convolve4Channels", &e), c1 = kern("convolve1Channel", &e),
              kl = kern("Opp2LAB", &e);
    if (e != CL_SUCCESS) { rc = fail("XYZtoScielab setup %d", e); goto out; }
    CHK(ARG(kx, 0, in)); CHK(ARG(kx, 1, opp));
    if ((rc = run1d(kx, n))) goto out;
    /* (kernel, filter, horizontal (w, h, update 0, opp -> tmp), then vertical (h, w, update, tmp -> conv)) */
    struct { cl_kernel k; cl_mem f; int upd; } pass[3] = {{c4, f1, 0}, {c4, f2, 1}, {c1, f3, 1}};
    for (int i = 0; i < 3; ++i) {
        const int zero = 0;
        cl_kernel k = pass[i].k;
        CHK(ARG(k, 0, opp)); CHK(ARG(k, 1, pass[i].f)); CHK(ARG(k, 2, half)); CHK(ARG(k, 3, w));
        CHK(ARG(k, 4, h)); CHK(ARG(k, 5, zero)); CHK(ARG(k, 6, tmp));
        if ((rc = run1d(k, n))) goto out;
        cl_mem fv = i == 2 ? fa : pass[i].f;  /* the third filter's vertical pass takes |k3| (IM:343-346) */
        CHK(ARG(k, 0, tmp)); CHK(ARG(k, 1, fv)); CHK(ARG(k, 2, half)); CHK(ARG(k, 3, h));
        CHK(ARG(k, 4, w)); CHK(ARG(k, 5, pass[i].upd)); CHK(ARG(k, 6, conv));
        if ((rc = run1d(k, n))) goto out;
    }
    CHK(ARG(kl, 0, conv)); CHK(ARG(kl, 1, illum[0])); CHK(ARG(kl, 2, illum[1])); CHK(ARG(kl, 3, illum[2]));
    CHK(ARG(kl, 4, lab));
    if ((rc = run1d(kl, n))) goto out;
    CHK(clEnqueueReadBuffer(g_q, lab, CL_TRUE, 0, 16 * n, lab4, 0, NULL, NULL));
out:
    if (kx) clReleaseKernel(kx);
    if (c4) clReleaseKernel(c4);
    if (c1) clReleaseKernel(c1);
    if (kl) clReleaseKernel(kl);
    release_mem(in); release_mem(opp); release_mem(conv); release_mem(tmp);
    release_mem(lab); release_mem(f1); release_mem(f2); release_mem(f3);
    release_mem(fa);
    return rc;
}

/* IM:450-493 set-up + IM:620-727 per member: costs[p] = mean dE + delta * #unused;
 * used[p*K + k] = the reference's int flags; err (P*N floats, may be NULL) = the
 * error images CIEDE writes (IM:663-667). */
int hqref_eval_population(const float *rgba4, const float *lab4, int w, int h, const float *pals4, int P, int K,
                          const float *k1_4, const float *k2_4, const float *k3, const float *absk3, int taps,
                          const float *illum, float delta, double *costs, int32_t *used, float *err) {
    int rc = 0;
    cl_int e = CL_SUCCESS;
    const size_t n = (size_t)w * h;
    const int half = (4 * taps) / 8;  /* IM:408 */
    float *errh = (float *)malloc(4 * n);
    int32_t *uh = (int32_t *)calloc((size_t)K, 4);
    cl_mem comp = buf(16 * n, lab4, &e), rgb = buf(16 * n, rgba4, &e), col = buf(16 * (size_t)K, NULL, &e);
    cl_mem f1 = buf(16 * (size_t)taps, k1_4, &e), f2 = buf(16 * (size_t)taps, k2_4, &e),
           f3 = buf(4 * (size_t)taps, k3, &e), fa = buf(4 * (size_t)taps, absk3, &e);
    cl_mem opp = buf(16 * n, NULL, &e), t1 = buf(16 * n, NULL, &e), t2 = buf(16 * n, NULL, &e),
           t3 = buf(4 * n, NULL, &e), conv = buf(16 * n, NULL, &e), lab = buf(16 * n, NULL, &e),
           usedb = buf(4 * (size_t)K, NULL, &e), errb = buf(4 * n, NULL, &e);
    cl_kernel kq = kern("quantizeAndConvertToOpp", &e), kt = kern("computeScielabKernelsTemp", &e),
              ke = kern("computeScielabKernelsEnd", &e), kl = kern("Opp2LAB", &e), kd = kern("CIEDE", &e);
    if (e != CL_SUCCESS || !errh || !uh) { rc = fail("eval setup %d", e); goto out; }
    /* IM:480-485: the kernels' constant arguments */
    CHK(ARG(kq, 0, rgb)); CHK(ARG(kq, 1, col)); CHK(ARG(kq, 2, K)); CHK(ARG(kq, 3, usedb)); CHK(ARG(kq, 4, opp));
    CHK(ARG(kd, 0, comp)); CHK(ARG(kd, 1, lab)); CHK(ARG(kd, 2, errb));
    CHK(ARG(kl, 0, conv)); CHK(ARG(kl, 1, illum[0])); CHK(ARG(kl, 2, illum[1])); CHK(ARG(kl, 3, illum[2]));
    CHK(ARG(kl, 4, lab));
    CHK(ARG(kt, 0, opp)); CHK(ARG(kt, 1, f1)); CHK(ARG(kt, 2, f2)); CHK(ARG(kt, 3, f3)); CHK(ARG(kt, 4, half));
    CHK(ARG(kt, 5, w)); CHK(ARG(kt, 6, h)); CHK(ARG(kt, 7, t1)); CHK(ARG(kt, 8, t2)); CHK(ARG(kt, 9, t3));
    CHK(ARG(ke, 0, t1)); CHK(ARG(ke, 1, t2)); CHK(ARG(ke, 2, t3)); CHK(ARG(ke, 3, f1)); CHK(ARG(ke, 4, f2));
    CHK(ARG(ke, 5, fa)); CHK(ARG(ke, 6, half)); CHK(ARG(ke, 7, h)); CHK(ARG(ke, 8, w)); CHK(ARG(ke, 9, conv));
    for (int p = 0; p < P; ++p) {
        memset(uh, 0, 4 * (size_t)K);
        CHK(clEnqueueWriteBuffer(g_q, usedb, CL_FALSE, 0, 4 * (size_t)K, uh, 0, NULL, NULL));
        CHK(clEnqueueWriteBuffer(g_q, col, CL_FALSE, 0, 16 * (size_t)K, pals4 + (size_t)p * 4 * K, 0, NULL, NULL));
        if ((rc = run1d(kq, n)) || (rc = run1d(kt, n)) || (rc = run1d(ke, n)) || (rc = run1d(kl, n)) ||
            (rc = run1d(kd, n)))
            goto out;
        CHK(clEnqueueReadBuffer(g_q, usedb, CL_TRUE, 0, 4 * (size_t)K, used ? used + (size_t)p * K : uh, 0, NULL,
                                NULL));
        CHK(clEnqueueReadBuffer(g_q, errb, CL_TRUE, 0, 4 * n, errh, 0, NULL, NULL));
        const int32_t *u = used ? used + (size_t)p * K : uh;
        double s = 0.0;
        for (size_t i = 0; i < n; ++i) s += (double)errh[i];
        int unused = 0;
        for (int k = 0; k < K; ++k) unused += u[k] == 0;
        costs[p] = s / (double)n + (double)unused * (double)delta;
        if (err) memcpy(err + (size_t)p * n, errh, 4 * n);
    }
out:
    if (kq) clReleaseKernel(kq);
    if (kt) clReleaseKernel(kt);
    if (ke) clReleaseKernel(ke);
    if (kl) clReleaseKernel(kl);
    if (kd) clReleaseKernel(kd);
    cl_mem all[] = {comp, rgb, col, f1, f2, f3, fa, opp, t1, t2, t3, conv, lab, usedb, errb};
    for (size_t i = 0; i < sizeof all / sizeof all[0]; ++i)
        if (all[i]) clReleaseMemObject(all[i]);
    free(errh);
    free(uh);
    return rc;
}

/* IM:770-798: the chosen colour of every pixel (CL:147-170) and the used flags. */
int hqref_quantize(const float *rgba4, int n, const float *pal4, int K, float *out4, int32_t *used) {
    int rc = 0;
    cl_int e = CL_SUCCESS;
    int32_t *uh = (int32_t *)calloc((size_t)K, 4);
    cl_mem in = buf(16 * (size_t)n, rgba4, &e), col = buf(16 * (size_t)K, pal4, &e),
           u = buf(4 * (size_t)K, uh, &e), o = buf(16 * (size_t)n, NULL, &e);
    cl_kernel k = kern("quantize", &e);
    if (e != CL_SUCCESS || !uh) { rc = fail("quantize setup %d", e); goto out; }
    CHK(ARG(k, 0, in)); CHK(ARG(k, 1, col)); CHK(ARG(k, 2, K)); CHK(ARG(k, 3, u)); CHK(ARG(k, 4, o));
    if ((rc = run1d(k, (size_t)n))) goto out;
    CHK(clEnqueueReadBuffer(g_q, o, CL_TRUE, 0, 16 * (size_t)n, out4, 0, NULL, NULL));
    CHK(clEnqueueReadBuffer(g_q, u, CL_TRUE, 0, 4 * (size_t)K, used ? used : uh, 0, NULL, NULL));
out:
    if (k) clReleaseKernel(k);
    release_mem(in); release_mem(col); release_mem(u); release_mem(o);
    free(uh);
    return rc;
}

/* Timing of the reference's population evaluation on this GPU (IM:620-727 as the
 * reference runs it: per member the used-flag reset and colour writes, the five
 * kernels, and non-blocking reads of the used flags and the error image; the
 * means on the host once the queue drains -- the reference's worker threads do
 * the same sums while later members run).  Buffers are created once, outside the
 * timed region, as IM:450-493 does once per search.  After one untimed
 * population, `reps` populations are timed: wall_ms = the average wall time of
 * one population; kern_ms[0..4] = the average device time per member of
 * quantizeAndConvertToOpp, computeScielabKernelsTemp, computeScielabKernelsEnd,
 * Opp2LAB and CIEDE (profiling events on a queue of its own). */
static double now_ms(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return 1e3 * (double)t.tv_sec + 1e-6 * (double)t.tv_nsec;
}

int hqref_time_population(const float *rgba4, const float *lab4, int w, int h, const float *pals4, int P, int K,
                          const float *k1_4, const float *k2_4, const float *k3, const float *absk3, int taps,
                          const float *illum, int reps, double *wall_ms, double *kern_ms) {
    int rc = 0;
    cl_int e = CL_SUCCESS;
    const size_t n = (size_t)w * h;
    const int half = (4 * taps) / 8;
    cl_command_queue q = clCreateCommandQueue(g_ctx, g_dev, CL_QUEUE_PROFILING_ENABLE, &e);
    if (e != CL_SUCCESS) return fail("profiling queue %d", e);
    float *errh = (float *)malloc(4 * n * (size_t)P);
    int32_t *uh = (int32_t *)calloc((size_t)K * (size_t)P, 4), *zero = (int32_t *)calloc((size_t)K, 4);
    cl_event *ev = (cl_event *)calloc((size_t)P * 5, sizeof(cl_event));
    cl_mem comp = buf(16 * n, lab4, &e), rgb = buf(16 * n, rgba4, &e), col = buf(16 * (size_t)K, NULL, &e);
    cl_mem f1 = buf(16 * (size_t)taps, k1_4, &e), f2 = buf(16 * (size_t)taps, k2_4, &e),
           f3 = buf(4 * (size_t)taps, k3, &e), fa = buf(4 * (size_t)taps, absk3, &e);
    cl_mem opp = buf(16 * n, NULL, &e), t1 = buf(16 * n, NULL, &e), t2 = buf(16 * n, NULL, &e),
           t3 = buf(4 * n, NULL, &e), conv = buf(16 * n, NULL, &e), lab = buf(16 * n, NULL, &e),
           usedb = buf(4 * (size_t)K, NULL, &e), errb = buf(4 * n, NULL, &e);
    cl_kernel ks[5] = {kern("quantizeAndConvertToOpp", &e), kern("computeScielabKernelsTemp", &e),
                       kern("computeScielabKernelsEnd", &e), kern("Opp2LAB", &e), kern("CIEDE", &e)};
    if (e != CL_SUCCESS || !errh || !uh || !zero || !ev) { rc = fail("timing setup %d", e); goto out; }
    cl_kernel kq = ks[0], kt = ks[1], ke = ks[2], kl = ks[3], kd = ks[4];
    CHK(ARG(kq, 0, rgb)); CHK(ARG(kq, 1, col)); CHK(ARG(kq, 2, K)); CHK(ARG(kq, 3, usedb)); CHK(ARG(kq, 4, opp));
    CHK(ARG(kd, 0, comp)); CHK(ARG(kd, 1, lab)); CHK(ARG(kd, 2, errb));
    CHK(ARG(kl, 0, conv)); CHK(ARG(kl, 1, illum[0])); CHK(ARG(kl, 2, illum[1])); CHK(ARG(kl, 3, illum[2]));
    CHK(ARG(kl, 4, lab));
    CHK(ARG(kt, 0, opp)); CHK(ARG(kt, 1, f1)); CHK(ARG(kt, 2, f2)); CHK(ARG(kt, 3, f3)); CHK(ARG(kt, 4, half));
    CHK(ARG(kt, 5, w)); CHK(ARG(kt, 6, h)); CHK(ARG(kt, 7, t1)); CHK(ARG(kt, 8, t2)); CHK(ARG(kt, 9, t3));
    CHK(ARG(ke, 0, t1)); CHK(ARG(ke, 1, t2)); CHK(ARG(ke, 2, t3)); CHK(ARG(ke, 3, f1)); CHK(ARG(ke, 4, f2));
    CHK(ARG(ke, 5, fa)); CHK(ARG(ke, 6, half)); CHK(ARG(ke, 7, h)); CHK(ARG(ke, 8, w)); CHK(ARG(ke, 9, conv));
    double wall = 0.0, kt_sum[5] = {0, 0, 0, 0, 0};
    for (int r = 0; r <= reps; ++r) {
        const double t0 = now_ms();
        for (int p = 0; p < P; ++p) {
            CHK(clEnqueueWriteBuffer(q, usedb, CL_FALSE, 0, 4 * (size_t)K, zero, 0, NULL, NULL));
            CHK(clEnqueueWriteBuffer(q, col, CL_FALSE, 0, 16 * (size_t)K, pals4 + (size_t)p * 4 * K, 0, NULL,
                                     NULL));
            for (int j = 0; j < 5; ++j) {
                const cl_int ee = clEnqueueNDRangeKernel(q, ks[j], 1, NULL, &n, NULL, 0, NULL, &ev[p * 5 + j]);
                if (ee != CL_SUCCESS) { rc = fail("enqueue %d", ee); goto out; }
            }
            CHK(clEnqueueReadBuffer(q, usedb, CL_FALSE, 0, 4 * (size_t)K, uh + (size_t)p * K, 0, NULL, NULL));
            CHK(clEnqueueReadBuffer(q, errb, CL_FALSE, 0, 4 * n, errh + (size_t)p * n, 0, NULL, NULL));
        }
        CHK(clFinish(q));
        volatile double sink = 0.0;
        for (int p = 0; p < P; ++p) {
            double s = 0.0;
            for (size_t i = 0; i < n; ++i) s += (double)errh[(size_t)p * n + i];
            sink += s;
        }
        const double t1w = now_ms();
        for (int i = 0; i < P * 5; ++i) {
            cl_ulong a = 0, b = 0;
            clGetEventProfilingInfo(ev[i], CL_PROFILING_COMMAND_START, sizeof a, &a, NULL);
            clGetEventProfilingInfo(ev[i], CL_PROFILING_COMMAND_END, sizeof b, &b, NULL);
            if (r > 0) kt_sum[i % 5] += 1e-6 * (double)(b - a);
            clReleaseEvent(ev[i]);
            ev[i] = NULL;
        }
        if (r > 0) wall += t1w - t0;
    }
    *wall_ms = wall / reps;
    for (int j = 0; j < 5; ++j) kern_ms[j] = kt_sum[j] / ((double)reps * P);
out:
    for (int j = 0; j < 5; ++j)
        if (ks[j]) clReleaseKernel(ks[j]);
    if (ev)
        for (int i = 0; i < P * 5; ++i)
            if (ev[i]) clReleaseEvent(ev[i]);
    cl_mem all[] = {comp, rgb, col, f1, f2, f3, fa, opp, t1, t2, t3, conv, lab, usedb, errb};
    for (size_t i = 0; i < sizeof all / sizeof all[0]; ++i)
        if (all[i]) clReleaseMemObject(all[i]);
    clReleaseCommandQueue(q);
    free(errh);
    free(uh);
    free(zero);
    free(ev);
    return rc;
}

/* IM:858-884: the CIEDE kernel (CL:201-231) on two inline Lab images; err = the
 * per-pixel dE it writes (the host's error-image transform and mean, IM:886-893,
 * are the caller's). */
int hqref_compute_error(const float *orig4, const float *quant4, int n, float *err) {
    int rc = 0;
    cl_int e = CL_SUCCESS;
    cl_mem a = buf(16 * (size_t)n, orig4, &e), b = buf(16 * (size_t)n, quant4, &e), o = buf(4 * (size_t)n, NULL, &e);
    cl_kernel k = kern("CIEDE", &e);
    if (e != CL_SUCCESS) { rc = fail("computeError setup %d", e); goto out; }
    CHK(ARG(k, 0, a)); CHK(ARG(k, 1, b)); CHK(ARG(k, 2, o));
    if ((rc = run1d(k, (size_t)n))) goto out;
    CHK(clEnqueueReadBuffer(g_q, o, CL_TRUE, 0, 4 * (size_t)n, err, 0, NULL, NULL));
out:
    if (k) clReleaseKernel(k);
    release_mem(a); release_mem(b); release_mem(o);
    return rc;
}
