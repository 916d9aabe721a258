"""ctypes bindings for oracle/libhq_oracle.so -- TEST INFRASTRUCTURE ONLY.

The C restatement (hq_oracle.c) is the fast checker for sizes the numpy oracle
cannot reach in seconds, and the "port" CPU baseline timed by bench.py.
Parity status: pinned against the reference's own OpenCL kernels on the
MI355X (tests/test_refcl.py; oracle/oracle.py header).
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_f = C.POINTER(C.c_float)
_i32 = C.POINTER(C.c_int32)
_d = C.POINTER(C.c_double)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libhq_oracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.hqo_eval.argtypes = [_f, _f, C.c_int, C.c_int, _f, C.c_int, _f, _f, _f, _f, C.c_int,
                               _f, C.c_float, C.c_int, C.c_int, _i32, _i32, _f, _d, _d]
        L.hqo_eval.restype = C.c_int
        L.hqo_assign.argtypes = [_f, C.c_longlong, _f, C.c_int, _i32, _i32]
        L.hqo_assign_mt.argtypes = [_f, C.c_longlong, _f, C.c_int, _i32, _i32, C.c_int]
        L.hqo_assign_mt.restype = C.c_int
        L.hqo_rgb_to_xyz.argtypes = [_f, _f, _f, C.c_longlong, _f]
        L.hqo_xyz_to_scielab.argtypes = [_f, C.c_int, C.c_int, _f, _f, _f, _f, C.c_int, _f, _f]
        L.hqo_xyz_to_scielab.restype = C.c_int
        L.hqo_xyz_to_scielab_mt.argtypes = [_f, C.c_int, C.c_int, _f, _f, _f, _f, C.c_int, _f, _f,
                                            C.c_int]
        L.hqo_xyz_to_scielab_mt.restype = C.c_int
        L.hqo_compute_error.argtypes = [_f, _f, C.c_longlong, _f]
        L.hqo_compute_error.restype = C.c_double
        L.hqo_ref_len_n.argtypes = [_f, C.c_longlong, _f]
        L.hqo_set_sqrt.argtypes = [C.c_void_p]
        L.hqo_set_sqrt.restype = None
        L.hqo_sqrt_calls.restype = C.c_longlong
        _LIB = L
    return _LIB


def _p(a, t=_f):
    return a.ctypes.data_as(t)


def _c32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def assign(rgb4, pal4, nthreads=1):
    """Exhaustive argmin (CL:179-193) -> (idx[N] int32, used[K] int32)."""
    rgb4, pal4 = _c32(rgb4), _c32(pal4)
    n, K = rgb4.shape[0], pal4.shape[0]
    idx = np.zeros(n, np.int32)
    used = np.zeros(K, np.int32)
    if nthreads > 1:
        lib().hqo_assign_mt(_p(rgb4), n, _p(pal4), K, _p(idx, _i32), _p(used, _i32), int(nthreads))
    else:
        lib().hqo_assign(_p(rgb4), n, _p(pal4), K, _p(idx, _i32), _p(used, _i32))
    return idx, used


def srgb_to_scielab(R, G, B, filt, w, nthreads=1):
    """LabRef of a planar image (IM:100-153 + IM:285-370) -> float4 [N,4].
    nthreads splits the rows of each 1-D pass (same arithmetic)."""
    R, G, B = _c32(R), _c32(G), _c32(B)
    n = R.shape[0]
    xyz = np.zeros((n, 4), np.float32)
    lib().hqo_rgb_to_xyz(_p(R), _p(G), _p(B), n, _p(xyz))
    lab = np.zeros((n, 4), np.float32)
    k1, k2, k3, ak3, il = (_c32(filt.k1), _c32(filt.k2), _c32(filt.k3), _c32(filt.absk3),
                           _c32(filt.illum))
    rc = lib().hqo_xyz_to_scielab_mt(_p(xyz), w, n // w, _p(k1), _p(k2), _p(k3), _p(ak3),
                                     filt.half, _p(il), _p(lab), int(nthreads))
    if rc != 0:
        raise ValueError(f"hqo_xyz_to_scielab failed ({rc})")
    return lab


def eval_palette(rgb4, lab4, pal4, filt, w, delta=2.0, depth=4, nthreads=1,
                 return_parts=False):
    """One candidate cost (steps a-h).  Returns cost or (cost, parts)."""
    rgb4, lab4, pal4 = _c32(rgb4), _c32(lab4), _c32(pal4)
    n, K = rgb4.shape[0], pal4.shape[0]
    idx = np.zeros(n, np.int32) if return_parts else None
    err = np.zeros(n, np.float32) if return_parts else None
    used = np.zeros(K, np.int32)
    cost = C.c_double()
    esum = C.c_double()
    k1, k2, k3, ak3, il = (_c32(filt.k1), _c32(filt.k2), _c32(filt.k3), _c32(filt.absk3),
                           _c32(filt.illum))
    rc = lib().hqo_eval(_p(rgb4), _p(lab4), w, n // w, _p(pal4), K, _p(k1), _p(k2), _p(k3),
                        _p(ak3), filt.half, _p(il), float(delta), depth, nthreads,
                        _p(idx, _i32) if idx is not None else None, _p(used, _i32),
                        _p(err) if err is not None else None, C.byref(esum), C.byref(cost))
    if rc != 0:
        raise ValueError(f"hqo_eval failed ({rc})")
    if return_parts:
        return cost.value, dict(idx=idx, used=used, err=err, err_sum=esum.value)
    return cost.value


def compute_error(orig4, quant4):
    orig4, quant4 = _c32(orig4), _c32(quant4)
    n = orig4.shape[0]
    img = np.zeros((n, 4), np.float32)
    e = lib().hqo_compute_error(_p(orig4), _p(quant4), n, _p(img))
    return e, img


def ref_len(dx, dy, dz, dw=None):
    """The argmin distance of hq_oracle.c (ref_len) for arrays of differences."""
    dx = _c32(dx).ravel()
    d4 = np.zeros((dx.size, 4), np.float32)
    d4[:, 0], d4[:, 1], d4[:, 2] = dx, _c32(dy).ravel(), _c32(dz).ravel()
    if dw is not None:
        d4[:, 3] = _c32(dw).ravel()
    out = np.empty(dx.size, np.float32)
    lib().hqo_ref_len_n(_p(d4), dx.size, _p(out))
    return out


def set_sqrt(fn_ptr):
    """The argmin distance's square root: the address of a C function float(float)
    (hw_sqrt.install passes the device's v_sqrt_f32), or None for sqrtf."""
    lib().hqo_set_sqrt(fn_ptr)


def sqrt_calls():
    """How many times the oracle has called the square root set by set_sqrt."""
    return int(lib().hqo_sqrt_calls())
