"""ctypes binding of oracle/_ref/libhq_refcl.so -- TEST INFRASTRUCTURE ONLY.

The reference's own OpenCL kernels (OptimizedConvolution.cl, compiled
unmodified for gfx950 by `make -C oracle ref` from /root/reference into
oracle/_ref/) run on the GPU through the ROCm OpenCL runtime, driven by
ref_cl_host.c, a restatement of the reference's JavaCL host sequences
(IM:100-153, IM:285-370, IM:450-493 + IM:620-727, IM:770-798).  The GPU tests
use it to pin the C/numpy oracle and libhq against the reference itself.
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(_HERE, "_ref")
LIB_PATH = os.path.join(REF_DIR, "libhq_refcl.so")
BIN_PATH = os.path.join(REF_DIR, "optimized_convolution.gfx950.co")  # -DCIE76 (IM:63, HQ:96)
BIN_PATHS = {"cie76": BIN_PATH, "cie94": os.path.join(REF_DIR, "optimized_convolution.cie94.gfx950.co")}
_LIB = None

_f = C.POINTER(C.c_float)
_i32 = C.POINTER(C.c_int32)
_d = C.POINTER(C.c_double)


def _p(a, t=_f):
    return a.ctypes.data_as(t)


def lib():
    """Load the host library and create the OpenCL context on the first GPU
    (raises with the runtime's message if either fails)."""
    global _LIB
    if _LIB is None:
        if not (os.path.exists(LIB_PATH) and os.path.exists(BIN_PATH)):
            raise OSError(f"{REF_DIR}: reference kernels not built (make -C oracle ref, needs /root/reference)")
        lb = C.CDLL(LIB_PATH)
        lb.hqref_error.restype = C.c_char_p
        if lb.hqref_init(BIN_PATH.encode()) != 0:
            raise RuntimeError("reference OpenCL kernels: " + lb.hqref_error().decode())
        _LIB = lb
    return _LIB


def use(variant):
    """Run the -DCIE76 ("cie76", the default) or the -DCIE94 ("cie94") build of the
    reference's kernels from now on (IM:63: the dE type is a build option)."""
    L = lib()
    if L.hqref_init(BIN_PATHS[variant].encode()) != 0:
        raise RuntimeError("reference OpenCL kernels: " + L.hqref_error().decode())


def _check(rc):
    if rc != 0:
        raise RuntimeError("reference OpenCL kernels: " + lib().hqref_error().decode())


def _c32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _filters4(filt):
    """IM:800-841: filters4[0..2] and absfilters4 (float4 per tap), filter3 and
    absfilter3 (scalars)."""
    T = filt.k3.shape[0]
    k3_4 = np.zeros((T, 4), np.float32)
    a3_4 = np.zeros((T, 4), np.float32)
    k3_4[:, 0] = filt.k3
    a3_4[:, 0] = filt.absk3
    return _c32(filt.k1), _c32(filt.k2), k3_4, a3_4, _c32(filt.k3), _c32(filt.absk3), T


def rgb_to_xyz(R, G, B):
    R, G, B = _c32(R), _c32(G), _c32(B)
    out = np.zeros((R.size, 4), np.float32)
    _check(lib().hqref_rgb_to_xyz(_p(R), _p(G), _p(B), R.size, _p(out)))
    return out


def xyz_to_scielab(xyz4, w, filt):
    xyz4 = _c32(xyz4).reshape(-1, 4)
    h = xyz4.shape[0] // w
    k1, k2, k3_4, a3_4, _, _, T = _filters4(filt)
    il = _c32(filt.illum)
    out = np.zeros_like(xyz4)
    _check(lib().hqref_xyz_to_scielab(_p(xyz4), w, h, _p(k1), _p(k2), _p(k3_4), _p(a3_4), T, _p(il), _p(out)))
    return out


def srgb_to_scielab(R, G, B, filt, w):
    """SP:374-381: RGBtoXYZ then XYZtoScielab, both on the reference's kernels."""
    return xyz_to_scielab(rgb_to_xyz(R, G, B), w, filt)


def eval_population(rgba4, lab4, w, pals, filt, delta=2.0, return_err=False):
    """costs [P], used [P, K] (the reference's int flags), and the error images
    [P, N] when asked."""
    rgba4, lab4 = _c32(rgba4).reshape(-1, 4), _c32(lab4).reshape(-1, 4)
    pals = _c32(pals)
    P, K = pals.shape[0], pals.shape[1]
    h = rgba4.shape[0] // w
    k1, k2, _, _, k3, a3, T = _filters4(filt)
    il = _c32(filt.illum)
    costs = np.zeros(P, np.float64)
    used = np.zeros((P, K), np.int32)
    err = np.zeros((P, w * h), np.float32) if return_err else None
    _check(lib().hqref_eval_population(_p(rgba4), _p(lab4), w, h, _p(pals), P, K, _p(k1), _p(k2), _p(k3), _p(a3),
                                       T, _p(il), C.c_float(delta), _p(costs, _d), _p(used, _i32),
                                       _p(err) if return_err else None))
    return (costs, used, err) if return_err else (costs, used)


def quantize(rgba4, pal4):
    """The chosen colour of every pixel (CL:147-170) and the used flags."""
    rgba4, pal4 = _c32(rgba4).reshape(-1, 4), _c32(pal4).reshape(-1, 4)
    out = np.zeros_like(rgba4)
    used = np.zeros(pal4.shape[0], np.int32)
    _check(lib().hqref_quantize(_p(rgba4), rgba4.shape[0], _p(pal4), pal4.shape[0], _p(out), _p(used, _i32)))
    return out, used


KERNELS = ("quantizeAndConvertToOpp", "computeScielabKernelsTemp", "computeScielabKernelsEnd", "Opp2LAB", "CIEDE")


def time_population(rgba4, lab4, w, pals, filt, reps=3):
    """The reference's population evaluation timed on this GPU (hqref_time_population):
    {"wall_ms": one population through the reference's host sequence, error-image
    reads and host means included; "kernel_ms": {kernel: device ms per member}}."""
    rgba4, lab4 = _c32(rgba4).reshape(-1, 4), _c32(lab4).reshape(-1, 4)
    pals = _c32(pals)
    P, K = pals.shape[0], pals.shape[1]
    h = rgba4.shape[0] // w
    k1, k2, _, _, k3, a3, T = _filters4(filt)
    il = _c32(filt.illum)
    wall = C.c_double(0.0)
    kern = np.zeros(5, np.float64)
    _check(lib().hqref_time_population(_p(rgba4), _p(lab4), w, h, _p(pals), P, K, _p(k1), _p(k2), _p(k3), _p(a3),
                                       T, _p(il), int(reps), C.byref(wall), _p(kern, _d)))
    return {"wall_ms": wall.value, "kernel_ms": dict(zip(KERNELS, kern.tolist()))}


def compute_error(orig4, quant4, errorImage=None):
    """IM:858-894 computeError: the CIEDE kernel per pixel, then the host's error
    image ((255 - e)^2 / 255^2 in channels 0-2, computed in float as Java does)
    and mean (one sequential double sum)."""
    orig4, quant4 = _c32(orig4).reshape(-1, 4), _c32(quant4).reshape(-1, 4)
    n = orig4.shape[0]
    err = np.zeros(n, np.float32)
    _check(lib().hqref_compute_error(_p(orig4), _p(quant4), n, _p(err)))
    if errorImage is not None:
        v = ((np.float32(255) - err) * (np.float32(255) - err) / np.float32(255 * 255)).astype(np.float32)
        img = errorImage.reshape(-1, 4)
        img[:, 0] = img[:, 1] = img[:, 2] = v
    s = float(np.cumsum(err, dtype=np.float64)[-1]) if n else 0.0  # sequential, as the Java loop
    return s / n, err
