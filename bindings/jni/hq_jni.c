/*
 * hq_jni.c -- JNI shim between the plugin's Java ImageManipulation backend
 * (bindings/java/.../ImageManipulation.java) and libhq's C ABI (include/hq.h).
 *
 * Built only where a JDK provides jni.h (`make -C bindings/jni JAVA_HOME=...`);
 * this container has no JDK, so it is not compiled in CI here.  Every native
 * method maps 1:1 to an hq_* call; a non-zero status becomes a Java
 * RuntimeException carrying hq_last_error() (the reference turned OpenCL
 * failures into openCLAvailable = false, IM:79-92: the Java side keeps that for
 * the constructor).  Arrays are pinned with Get/ReleasePrimitiveArrayCritical
 * for the duration of the call only (caller-owned, IM:271-283 semantics).
 * Every array length is checked against what the hq_* call will touch before
 * anything is pinned (IllegalArgumentException), and a failed pin raises
 * OutOfMemoryError, so a mismatched caller never reaches native memory.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/hq.h"

#define JNI_FN(name) Java_plugins_dbrasseur_hybridquantization_ImageManipulation_##name

static void throw_status(JNIEnv *env, hq_ctx *ctx, int status) {
    jclass cls = (*env)->FindClass(env, "java/lang/RuntimeException");
    const char *msg = ctx ? hq_last_error(ctx) : hq_status_string(status);
    if (cls) (*env)->ThrowNew(env, cls, msg && *msg ? msg : hq_status_string(status));
}

static int throw_class(JNIEnv *env, const char *cls_name, const char *msg) {
    jclass cls = (*env)->FindClass(env, cls_name);
    if (cls) (*env)->ThrowNew(env, cls, msg);
    return 1;
}

/* 1 (IllegalArgumentException thrown) unless `a` is non-null and holds at
 * least `need` elements. */
static int bad_len(JNIEnv *env, jarray a, long long need, const char *what) {
    if (!a || need < 0 || (long long)(*env)->GetArrayLength(env, a) < need)
        return throw_class(env, "java/lang/IllegalArgumentException", what);
    return 0;
}

typedef struct {
    jarray arr;
    void *ptr;
} pin_t;

static void *pin(JNIEnv *env, jarray a, pin_t *p) {
    p->arr = a;
    p->ptr = a ? (*env)->GetPrimitiveArrayCritical(env, a, NULL) : NULL;
    return p->ptr;
}

/* 1 (OutOfMemoryError thrown) if a requested pin of a non-null array failed */
static int pin_failed(JNIEnv *env, const pin_t *p, int n) {
    for (int i = 0; i < n; ++i)
        if (p[i].arr && !p[i].ptr)
            return throw_class(env, "java/lang/OutOfMemoryError", "libhq: cannot pin a Java array");
    return 0;
}

static void unpin(JNIEnv *env, pin_t *p, int commit) {
    if (p->arr && p->ptr) (*env)->ReleasePrimitiveArrayCritical(env, p->arr, p->ptr, commit ? 0 : JNI_ABORT);
    p->ptr = NULL;
}

/* IM:52 -> hq_create; returns 0 when no GPU (caller sets openCLAvailable=false) */
JNIEXPORT jlong JNICALL JNI_FN(nCreate)(JNIEnv *env, jclass cls, jint device, jint deType) {
    hq_ctx *ctx = NULL;
    if (hq_create(device, deType, &ctx) != HQ_OK) return 0;
    return (jlong)(intptr_t)ctx;
}

/* IM:265 close() */
JNIEXPORT void JNICALL JNI_FN(nDestroy)(JNIEnv *env, jclass cls, jlong h) {
    hq_destroy((hq_ctx *)(intptr_t)h);
}

/* IM:800 updateOpenCLFilters(filters, absfilters) after Java-side packing */
JNIEXPORT void JNICALL JNI_FN(nSetFilters)(JNIEnv *env, jclass cls, jlong h, jint taps,
                                          jfloatArray k1, jfloatArray k2, jfloatArray k3,
                                          jfloatArray absk3) {
    hq_ctx *ctx = (hq_ctx *)(intptr_t)h;
    if (taps < 1 || bad_len(env, k1, 4LL * taps, "k1: 4*taps floats") ||
        bad_len(env, k2, 4LL * taps, "k2: 4*taps floats") || bad_len(env, k3, taps, "k3: taps floats") ||
        bad_len(env, absk3, taps, "absk3: taps floats")) {
        if (taps < 1) throw_class(env, "java/lang/IllegalArgumentException", "taps < 1");
        return;
    }
    pin_t p[4];
    const float *a = pin(env, k1, &p[0]), *b = pin(env, k2, &p[1]), *c = pin(env, k3, &p[2]),
                *d = pin(env, absk3, &p[3]);
    int st = pin_failed(env, p, 4) ? -1 : hq_set_filters(ctx, taps, a, b, c, d);
    for (int i = 3; i >= 0; --i) unpin(env, &p[i], 0);
    if (st > 0) throw_status(env, ctx, st);
}

/* IM:100 RGBtoXYZ(R, G, B) */
JNIEXPORT void JNICALL JNI_FN(nRGBtoXYZ)(JNIEnv *env, jclass cls, jlong h, jfloatArray R,
                                        jfloatArray G, jfloatArray B, jfloatArray out) {
    hq_ctx *ctx = (hq_ctx *)(intptr_t)h;
    if (!R) { throw_class(env, "java/lang/IllegalArgumentException", "null R"); return; }
    jsize n = (*env)->GetArrayLength(env, R);
    if (n < 1 || bad_len(env, G, n, "G shorter than R") || bad_len(env, B, n, "B shorter than R") ||
        bad_len(env, out, 4LL * n, "out: 4*n floats")) {
        if (n < 1) throw_class(env, "java/lang/IllegalArgumentException", "empty image");
        return;
    }
    pin_t p[4];
    const float *r = pin(env, R, &p[0]), *g = pin(env, G, &p[1]), *b = pin(env, B, &p[2]);
    float *o = pin(env, out, &p[3]);
    int st = pin_failed(env, p, 4) ? -1 : hq_rgb_to_xyz(ctx, r, g, b, n, o);
    unpin(env, &p[3], st == 0);
    for (int i = 2; i >= 0; --i) unpin(env, &p[i], 0);
    if (st > 0) throw_status(env, ctx, st);
}

/* IM:285 XYZtoScielab(XYZ, filters, absfilters, w, illuminant) */
JNIEXPORT void JNICALL JNI_FN(nXYZtoScielab)(JNIEnv *env, jclass cls, jlong h, jfloatArray xyz,
                                            jint w, jfloatArray illum, jfloatArray out) {
    hq_ctx *ctx = (hq_ctx *)(intptr_t)h;
    if (!xyz || w <= 0) { throw_class(env, "java/lang/IllegalArgumentException", "null XYZ or w <= 0"); return; }
    jsize n = (*env)->GetArrayLength(env, xyz) / 4;
    const int hgt = (int)(n / w);
    if (hgt < 1 || bad_len(env, illum, 3, "illuminant: 3 floats") ||
        bad_len(env, out, 4LL * w * hgt, "out: 4*w*h floats")) {
        if (hgt < 1) throw_class(env, "java/lang/IllegalArgumentException", "image shorter than one row");
        return;
    }
    pin_t p[3];
    const float *a = pin(env, xyz, &p[0]), *il = pin(env, illum, &p[1]);
    float *o = pin(env, out, &p[2]);
    int st = pin_failed(env, p, 3) ? -1 : hq_xyz_to_scielab(ctx, a, w, hgt, il, o);
    unpin(env, &p[2], st == 0); unpin(env, &p[1], 0); unpin(env, &p[0], 0);
    if (st > 0) throw_status(env, ctx, st);
}

/* IM:450-478: device-resident inline RGBA image + inline S-CIELAB */
JNIEXPORT void JNICALL JNI_FN(nSetImage)(JNIEnv *env, jclass cls, jlong h, jfloatArray rgba,
                                        jfloatArray lab, jint w, jfloatArray illum) {
    hq_ctx *ctx = (hq_ctx *)(intptr_t)h;
    if (!rgba || w <= 0) { throw_class(env, "java/lang/IllegalArgumentException", "null image or w <= 0"); return; }
    jsize n = (*env)->GetArrayLength(env, rgba) / 4;
    const int hgt = (int)(n / w);
    if (hgt < 1 || (lab && bad_len(env, lab, 4LL * w * hgt, "lab: 4*w*h floats")) ||
        bad_len(env, illum, 3, "illuminant: 3 floats")) {
        if (hgt < 1) throw_class(env, "java/lang/IllegalArgumentException", "image shorter than one row");
        return;
    }
    pin_t p[3];
    const float *a = pin(env, rgba, &p[0]), *b = pin(env, lab, &p[1]), *il = pin(env, illum, &p[2]);
    int st = pin_failed(env, p, 3) ? -1 : hq_set_image(ctx, a, b, w, hgt, il);
    unpin(env, &p[2], 0); unpin(env, &p[1], 0); unpin(env, &p[0], 0);
    if (st > 0) throw_status(env, ctx, st);
}

/* IM:620 computeQuantizationErrorPopulation: palettes[P*4K] -> mean dE per
 * palette (penalty 0: the Java side adds SWASA.computePenalty(used), IM:712)
 * and used[P*K]. */
JNIEXPORT void JNICALL JNI_FN(nEvalPopulation)(JNIEnv *env, jclass cls, jlong h,
                                              jfloatArray palettes, jint P, jint K,
                                              jdoubleArray meanOut, jintArray usedOut) {
    hq_ctx *ctx = (hq_ctx *)(intptr_t)h;
    if (P < 1 || K < 1) { throw_class(env, "java/lang/IllegalArgumentException", "P < 1 or K < 1"); return; }
    if (bad_len(env, palettes, 4LL * P * K, "palettes: P*4K floats") ||
        bad_len(env, meanOut, P, "mean: P doubles") || bad_len(env, usedOut, (long long)P * K, "used: P*K ints"))
        return;
    pin_t p[3];
    const float *a = pin(env, palettes, &p[0]);
    double *m = pin(env, meanOut, &p[1]);
    int32_t *u = (int32_t *)pin(env, usedOut, &p[2]);
    int st = pin_failed(env, p, 3) ? -1 : hq_eval_population(ctx, a, P, K, 0.0f, m, u);
    unpin(env, &p[2], st == 0); unpin(env, &p[1], st == 0); unpin(env, &p[0], 0);
    if (st > 0) throw_status(env, ctx, st);
}

/* IM:770 quantize(inlineImageRGB, colors) */
JNIEXPORT void JNICALL JNI_FN(nQuantize)(JNIEnv *env, jclass cls, jlong h, jfloatArray rgba,
                                        jfloatArray colors, jfloatArray out) {
    hq_ctx *ctx = (hq_ctx *)(intptr_t)h;
    if (!rgba || !colors) { throw_class(env, "java/lang/IllegalArgumentException", "null image or colors"); return; }
    jsize n = (*env)->GetArrayLength(env, rgba) / 4;
    jsize K = (*env)->GetArrayLength(env, colors) / 4;
    if (n < 1 || K < 1 || bad_len(env, out, 4LL * n, "out: 4*n floats")) {
        if (n < 1 || K < 1) throw_class(env, "java/lang/IllegalArgumentException", "empty image or palette");
        return;
    }
    pin_t p[3];
    const float *a = pin(env, rgba, &p[0]), *c = pin(env, colors, &p[1]);
    float *o = pin(env, out, &p[2]);
    int st = pin_failed(env, p, 3) ? -1 : hq_quantize(ctx, a, n, c, K, o, NULL);
    unpin(env, &p[2], st == 0); unpin(env, &p[1], 0); unpin(env, &p[0], 0);
    if (st > 0) throw_status(env, ctx, st);
}

/* IM:858 computeError(original, quantized, errorImage) */
JNIEXPORT jdouble JNICALL JNI_FN(nComputeError)(JNIEnv *env, jclass cls, jlong h,
                                               jfloatArray orig, jfloatArray quant,
                                               jfloatArray errImg) {
    hq_ctx *ctx = (hq_ctx *)(intptr_t)h;
    if (!orig) { throw_class(env, "java/lang/IllegalArgumentException", "null original"); return 0.0; }
    jsize n = (*env)->GetArrayLength(env, orig) / 4;
    if (n < 1 || bad_len(env, quant, 4LL * n, "quantized: 4*n floats") ||
        (errImg && bad_len(env, errImg, 4LL * n, "errorImage: 4*n floats"))) {
        if (n < 1) throw_class(env, "java/lang/IllegalArgumentException", "empty image");
        return 0.0;
    }
    double mean = 0.0;
    pin_t p[3];
    const float *a = pin(env, orig, &p[0]), *b = pin(env, quant, &p[1]);
    float *e = pin(env, errImg, &p[2]);
    int st = pin_failed(env, p, 3) ? -1 : hq_compute_error(ctx, a, b, n, e, &mean);
    unpin(env, &p[2], st == 0); unpin(env, &p[1], 0); unpin(env, &p[0], 0);
    if (st > 0) throw_status(env, ctx, st);
    return mean;
}
