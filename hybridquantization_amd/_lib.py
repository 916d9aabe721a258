"""ctypes binding of libhq.so (the C ABI declared in include/hq.h).

The library is built in-tree (``hybridquantization_amd/libhq.so``) by
``__graft_entry__.build()`` / ``make -C hybridquantization_amd/csrc``.  There is
no fallback: if the shared library is missing this module raises, so a GPU run
can never silently route through a CPU path.
"""

from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HQ_LIB_PATH") or os.path.join(_HERE, "libhq.so")  # override: A/B builds

HQ_OK = 0
HQ_ERR_ARG = 1
HQ_ERR_DEVICE = 2
HQ_ERR_STATE = 3
HQ_ERR_UNSUPPORTED = 4
HQ_ERR_COMM = 5
HQ_ERR_NOMEM = 6

HQ_DE_CIE76, HQ_DE_CIE94, HQ_DE_CIEDE2000 = 0, 1, 2
HQ_WP_D50, HQ_WP_D65 = 0, 1

_f = C.POINTER(C.c_float)
_d = C.POINTER(C.c_double)
_i32 = C.POINTER(C.c_int32)
_u8 = C.POINTER(C.c_uint8)
_ctx = C.c_void_p


class hq_swasa_params(C.Structure):
    _fields_ = [("population", C.c_int), ("imax", C.c_int), ("iTc", C.c_int),
                ("delta", C.c_float), ("conv_delay", C.c_float), ("conv_spread", C.c_float),
                ("t0", C.c_float), ("alpha", C.c_float), ("s0", C.c_float), ("beta", C.c_float),
                ("convergence", C.c_int)]


EVAL_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, _f, C.c_int, C.c_int, _d)

# name -> (restype, argtypes); the exported surface of include/hq.h
SIGNATURES = {
    "hq_version": (C.c_int, []),
    "hq_status_string": (C.c_char_p, [C.c_int]),
    "hq_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "hq_create": (C.c_int, [C.c_int, C.c_int, C.POINTER(_ctx)]),
    "hq_destroy": (None, [_ctx]),
    "hq_last_error": (C.c_char_p, [_ctx]),
    "hq_design_filters": (C.c_int, [C.c_int, C.c_double, C.c_int, C.c_int, _f, _f, _f, _f,
                                    C.POINTER(C.c_int), _f]),
    "hq_set_filters": (C.c_int, [_ctx, C.c_int, _f, _f, _f, _f]),
    "hq_rgb_to_xyz": (C.c_int, [_ctx, _f, _f, _f, C.c_int64, _f]),
    "hq_xyz_to_scielab": (C.c_int, [_ctx, _f, C.c_int, C.c_int, _f, _f]),
    "hq_set_image": (C.c_int, [_ctx, _f, _f, C.c_int, C.c_int, _f]),
    "hq_set_image_shard": (C.c_int, [_ctx, _f, _f, C.c_int, C.c_int, _f, C.c_int, C.c_int]),
    "hq_set_image_planar_shard": (C.c_int, [_ctx, _f, _f, _f, C.c_int, C.c_int, _f, C.c_int,
                                            C.c_int]),
    "hq_get_labref": (C.c_int, [_ctx, _f]),
    "hq_eval_population": (C.c_int, [_ctx, _f, C.c_int, C.c_int, C.c_float, _d, _i32]),
    "hq_eval_population_partial": (C.c_int, [_ctx, _f, C.c_int, C.c_int, _d]),
    "hq_get_indices": (C.c_int, [_ctx, C.c_int, _u8]),
    "hq_get_indices32": (C.c_int, [_ctx, C.c_int, C.POINTER(C.c_uint32)]),
    "hq_get_pixel_errors": (C.c_int, [_ctx, C.c_int, _f]),
    "hq_quantize": (C.c_int, [_ctx, _f, C.c_int64, _f, C.c_int, _f, _i32]),
    "hq_compute_error": (C.c_int, [_ctx, _f, _f, C.c_int64, _f, _d]),
    "hq_comm_unique_id": (C.c_int, [C.POINTER(C.c_ubyte)]),
    "hq_comm_init": (C.c_int, [_ctx, C.c_int, C.c_int, C.POINTER(C.c_ubyte)]),
    "hq_comm_info": (C.c_int, [_ctx, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "hq_swasa_default_params": (None, [C.POINTER(hq_swasa_params)]),
    "hq_search_create": (C.c_int, [_ctx, C.POINTER(hq_swasa_params), C.c_int, C.c_uint64,
                                   C.POINTER(C.c_void_p)]),
    "hq_search_run": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_int)]),
    "hq_search_best": (C.c_int, [C.c_void_p, _f, _d, C.POINTER(C.c_int)]),
    "hq_search_destroy": (None, [C.c_void_p]),
    "hq_swasa_search_host": (C.c_int, [C.POINTER(hq_swasa_params), C.c_int, C.c_uint64,
                                       C.c_int, EVAL_FN, C.c_void_p, _f, _d, _d]),
    "hq_profile_enable": (C.c_int, [_ctx, C.c_int]),
    "hq_profile_get": (C.c_int, [_ctx, C.c_char_p, _d, C.POINTER(C.c_int64)]),
    "hq_profile_reset": (C.c_int, [_ctx]),
    "hq_set_option": (C.c_int, [_ctx, C.c_char_p, C.c_int]),
}

_LIB = None


class HQError(RuntimeError):
    def __init__(self, status: int, msg: str = ""):
        self.status = status
        super().__init__(f"libhq status {status}: {msg}")


class HQUnavailable(HQError):
    """No usable GPU / library: the reference's IM:79-92 fallback condition."""


def load():
    """Load libhq.so (raises OSError if it has not been built)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} not found: build it with __graft_entry__.build() "
                          "(make -C hybridquantization_amd/csrc); there is no CPU fallback")
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = lib
    return _LIB


def check(status: int, ctx=None):
    if status != HQ_OK:
        lib = load()
        msg = lib.hq_last_error(ctx).decode() if ctx else lib.hq_status_string(status).decode()
        if status == HQ_ERR_DEVICE:
            raise HQUnavailable(status, msg)
        raise HQError(status, msg)


def fptr(a):
    return a.ctypes.data_as(_f)


def dptr(a):
    return a.ctypes.data_as(_d)


def iptr(a):
    return a.ctypes.data_as(_i32)


def u8ptr(a):
    return a.ctypes.data_as(_u8)
