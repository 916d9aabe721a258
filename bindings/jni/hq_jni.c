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

typedef struct {
    jarray arr;
    void *ptr;
} pin_t;

static void *pin(JNIEnv *env, jarray a, pin_t *p) {
    p->arr = a;
    p->ptr = a ? (*env)->GetPrimitiveArrayCritical(env, a, NULL) : NULL;
    return p->ptr;
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
    pin_t a, b, c, d;
    int st = hq_set_filters(ctx, taps, pin(env, k1, &a), pin(env, k2, &b), pin(env, k3, &c),
                            pin(env, absk3, &d));
    unpin(env, &d, 0); unpin(env, &c, 0); unpin(env, &b, 0); unpin(env, &a, 0);
    if (st) throw_status(env, ctx, st);
}

/* IM:100 RGBtoXYZ(R, G, B) */
JNIEXPORT void JNICALL JNI_FN(nRGBtoXYZ)(JNIEnv *env, jclass cls, jlong h, jfloatArray R,
                                        jfloatArray G, jfloatArray B, jfloatArray out) {
    hq_ctx *ctx = (hq_ctx *)(intptr_t)h;
    jsize n = (*env)->GetArrayLength(env, R);
    pin_t a, b, c, o;
    int st = hq_rgb_to_xyz(ctx, pin(env, R, &a), pin(env, G, &b), pin(env, B, &c), n,
                           pin(env, out, &o));
    unpin(env, &o, 1); unpin(env, &c, 0); unpin(env, &b, 0); unpin(env, &a, 0);
    if (st) throw_status(env, ctx, st);
}

/* IM:285 XYZtoScielab(XYZ, filters, absfilters, w, illuminant) */
JNIEXPORT void JNICALL JNI_FN(nXYZtoScielab)(JNIEnv *env, jclass cls, jlong h, jfloatArray xyz,
                                            jint w, jfloatArray illum, jfloatArray out) {
    hq_ctx *ctx = (hq_ctx *)(intptr_t)h;
    jsize n = (*env)->GetArrayLength(env, xyz) / 4;
    pin_t a, i, o;
    int st = hq_xyz_to_scielab(ctx, pin(env, xyz, &a), w, (int)(n / w), pin(env, illum, &i),
                               pin(env, out, &o));
    unpin(env, &o, 1); unpin(env, &i, 0); unpin(env, &a, 0);
    if (st) throw_status(env, ctx, st);
}

/* IM:450-478: device-resident inline RGBA image + inline S-CIELAB */
JNIEXPORT void JNICALL JNI_FN(nSetImage)(JNIEnv *env, jclass cls, jlong h, jfloatArray rgba,
                                        jfloatArray lab, jint w, jfloatArray illum) {
    hq_ctx *ctx = (hq_ctx *)(intptr_t)h;
    jsize n = (*env)->GetArrayLength(env, rgba) / 4;
    pin_t a, b, i;
    int st = hq_set_image(ctx, pin(env, rgba, &a), pin(env, lab, &b), w, (int)(n / w),
                          pin(env, illum, &i));
    unpin(env, &i, 0); unpin(env, &b, 0); unpin(env, &a, 0);
    if (st) throw_status(env, ctx, st);
}

/* IM:620 computeQuantizationErrorPopulation: palettes[P*4K] -> mean dE per
 * palette (penalty 0: the Java side adds SWASA.computePenalty(used), IM:712)
 * and used[P*K]. */
JNIEXPORT void JNICALL JNI_FN(nEvalPopulation)(JNIEnv *env, jclass cls, jlong h,
                                              jfloatArray palettes, jint P, jint K,
                                              jdoubleArray meanOut, jintArray usedOut) {
    hq_ctx *ctx = (hq_ctx *)(intptr_t)h;
    pin_t a, m, u;
    int st = hq_eval_population(ctx, pin(env, palettes, &a), P, K, 0.0f, pin(env, meanOut, &m),
                                (int32_t *)pin(env, usedOut, &u));
    unpin(env, &u, 1); unpin(env, &m, 1); unpin(env, &a, 0);
    if (st) throw_status(env, ctx, st);
}

/* IM:770 quantize(inlineImageRGB, colors) */
JNIEXPORT void JNICALL JNI_FN(nQuantize)(JNIEnv *env, jclass cls, jlong h, jfloatArray rgba,
                                        jfloatArray colors, jfloatArray out) {
    hq_ctx *ctx = (hq_ctx *)(intptr_t)h;
    jsize n = (*env)->GetArrayLength(env, rgba) / 4;
    jsize K = (*env)->GetArrayLength(env, colors) / 4;
    pin_t a, c, o;
    int st = hq_quantize(ctx, pin(env, rgba, &a), n, pin(env, colors, &c), K, pin(env, out, &o), NULL);
    unpin(env, &o, 1); unpin(env, &c, 0); unpin(env, &a, 0);
    if (st) throw_status(env, ctx, st);
}

/* IM:858 computeError(original, quantized, errorImage) */
JNIEXPORT jdouble JNICALL JNI_FN(nComputeError)(JNIEnv *env, jclass cls, jlong h,
                                               jfloatArray orig, jfloatArray quant,
                                               jfloatArray errImg) {
    hq_ctx *ctx = (hq_ctx *)(intptr_t)h;
    jsize n = (*env)->GetArrayLength(env, orig) / 4;
    double mean = 0.0;
    pin_t a, b, e;
    int st = hq_compute_error(ctx, pin(env, orig, &a), pin(env, quant, &b), n, pin(env, errImg, &e), &mean);
    unpin(env, &e, 1); unpin(env, &b, 0); unpin(env, &a, 0);
    if (st) throw_status(env, ctx, st);
    return mean;
}
