"""The device's v_sqrt_f32 for the oracles' argmin distance -- TEST INFRASTRUCTURE ONLY.

The reference's distance() on gfx950 ranks colours by v_sqrt_f32 of d^2 (CL:179-192
as its OpenCL build compiles it).  That instruction is not correctly
rounded and has no published definition, so the oracles take it as a parameter;
``install()`` hands them the instruction itself, evaluated on the GPU by
oracle/libhq_hwsqrt.so (hw_sqrt.hip).  The GPU tests install it once per session
(tests/conftest.py); CPU-only runs keep the correctly rounded sqrt.
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np

import c_oracle
import oracle

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        L = C.CDLL(os.path.join(_HERE, "libhq_hwsqrt.so"))
        L.hqhw_sqrt_n.argtypes = [C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_longlong]
        L.hqhw_sqrt_n.restype = C.c_int
        L.hqhw_sqrt1.argtypes = [C.c_float]
        L.hqhw_sqrt1.restype = C.c_float
        _LIB = L
    return _LIB


def sqrt_n(x):
    """v_sqrt_f32 of every element of x (fp32), on the GPU."""
    x = np.ascontiguousarray(x, np.float32).ravel()
    y = np.empty_like(x)
    if x.size:
        rc = lib().hqhw_sqrt_n(x.ctypes.data_as(C.POINTER(C.c_float)), y.ctypes.data_as(C.POINTER(C.c_float)),
                               x.size)
        if rc != 0:
            raise RuntimeError(f"hqhw_sqrt_n: HIP error {rc}")
    return y


def install():
    """Both oracles take v_sqrt_f32 from the GPU from now on."""
    L = lib()
    c_oracle.set_sqrt(C.cast(L.hqhw_sqrt1, C.c_void_p).value)
    oracle.set_sqrt(sqrt_n)


def uninstall():
    c_oracle.set_sqrt(None)
    oracle.set_sqrt(None)
