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
 * anything is pinned (IllegalArgumentException), and a failed pin releases
 * what is held before raising OutOfMemoryError (pin_all), so a mismatched
 * caller never reaches native memory and no JNI call runs inside a critical
 * region.
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
    jarray arr;  /* may be NULL (optional argument): left unpinned */
    void *ptr;
    int out;     /* written by the call: copied back only when it succeeds */
} pin_t;

/* Pins p[0..n) in order with GetPrimitiveArrayCritical.  JNI allows no other
 * JNI call while a critical region is open, so on the first failed pin this
 * stops, releases every array it already holds (JNI_ABORT), and only then
 * throws OutOfMemoryError -- unless the VM already raised an exception, which
 * is kept.  Returns 0 when every non-null array is pinned. */
static int pin_all(JNIEnv *env, pin_t *p, int n) {
    for (int i = 0; i < n; ++i) p[i].ptr = NULL;
    for (int i = 0; i < n; ++i) {
        if (!p[i].arr) continue;
        p[i].ptr = (*env)->GetPrimitiveArrayCritical(env, p[i].arr, NULL);
        if (!p[i].ptr) {
            for (int j = i - 1; j >= 0; --j)
                if (p[j].ptr) {
                    (*env)->ReleasePrimitiveArrayCritical(env, p[j].arr, p[j].ptr, JNI_ABORT);
                    p[j].ptr = NULL;
                }
            if (!(*env)->ExceptionCheck(env))
                throw_class(env, "java/lang/OutOfMemoryError", "libhq: cannot pin a Java array");
            return 1;
        }
    }
    return 0;
}

/* Releases in reverse order; output arrays are committed only when ok. */
static void unpin_all(JNIEnv *env, pin_t *p, int n, int ok) {
    for (int i = n - 1; i >= 0; --i)
        if (p[i].ptr) {
            (*env)->ReleasePrimitiveArrayCritical(env, p[i].arr, p[i].ptr, ok && p[i].out ? 0 : JNI_ABORT);
            p[i].ptr = NULL;
        }
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
    pin_t p[4] = {{k1, NULL, 0}, {k2, NULL, 0}, {k3, NULL, 0}, {absk3, NULL, 0}};
    if (pin_all(env, p, 4)) return;
    int st = hq_set_filters(ctx, taps, p[0].ptr, p[1].ptr, p[2].ptr, p[3].ptr);
    unpin_all(env, p, 4, st == 0);
    if (st) throw_status(env, ctx, st);
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
    pin_t p[4] = {{R, NULL, 0}, {G, NULL, 0}, {B, NULL, 0}, {out, NULL, 1}};
    if (pin_all(env, p, 4)) return;
    int st = hq_rgb_to_xyz(ctx, p[0].ptr, p[1].ptr, p[2].ptr, n, p[3].ptr);
    unpin_all(env, p, 4, st == 0);
    if (st) throw_status(env, ctx, st);
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
    pin_t p[3] = {{xyz, NULL, 0}, {illum, NULL, 0}, {out, NULL, 1}};
    if (pin_all(env, p, 3)) return;
    int st = hq_xyz_to_scielab(ctx, p[0].ptr, w, hgt, p[1].ptr, p[2].ptr);
    unpin_all(env, p, 3, st == 0);
    if (st) throw_status(env, ctx, st);
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
    pin_t p[3] = {{rgba, NULL, 0}, {lab, NULL, 0}, {illum, NULL, 0}};  /* lab may be NULL */
    if (pin_all(env, p, 3)) return;
    int st = hq_set_image(ctx, p[0].ptr, p[1].ptr, w, hgt, p[2].ptr);
    unpin_all(env, p, 3, st == 0);
    if (st) throw_status(env, ctx, st);
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
    pin_t p[3] = {{palettes, NULL, 0}, {meanOut, NULL, 1}, {usedOut, NULL, 1}};
    if (pin_all(env, p, 3)) return;
    int st = hq_eval_population(ctx, p[0].ptr, P, K, 0.0f, p[1].ptr, (int32_t *)p[2].ptr);
    unpin_all(env, p, 3, st == 0);
    if (st) throw_status(env, ctx, st);
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
    pin_t p[3] = {{rgba, NULL, 0}, {colors, NULL, 0}, {out, NULL, 1}};
    if (pin_all(env, p, 3)) return;
    int st = hq_quantize(ctx, p[0].ptr, n, p[1].ptr, K, p[2].ptr, NULL);
    unpin_all(env, p, 3, st == 0);
    if (st) throw_status(env, ctx, st);
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
    pin_t p[3] = {{orig, NULL, 0}, {quant, NULL, 0}, {errImg, NULL, 1}};  /* errImg may be NULL */
    if (pin_all(env, p, 3)) return 0.0;
    int st = hq_compute_error(ctx, p[0].ptr, p[1].ptr, n, p[2].ptr, &mean);
    unpin_all(env, p, 3, st == 0);
    if (st) throw_status(env, ctx, st);
    return mean;
}
