"""Host-side mirror of the reference's ``ImageManipulation`` (IM) backed by libhq.

Method names, argument order and array layouts follow
``src/plugins/dbrasseur/hybridquantization/ImageManipulation.java`` so a caller
of the reference (or its tests) reads the same against this class.  Every
method runs on the GPU through the C ABI of ``include/hq.h``; nothing here
computes pixels on the host.

Layouts (HQ:279-291 ``makeinline``): inline images are ``float32[4*N]`` RGBA /
Lab with ``.w = 0``; palettes are ``float32[4*K]`` (SW:40-52).

Error behaviour: the reference's constructor turns OpenCL failures into
``openCLAvailable = false`` (IM:79-92) and its methods then silently return
zero arrays (IM:392, IM:590, IM:369, IM:797).  This mirror keeps the flag
(``getOpenCLAvailable()``) but raises ``HQUnavailable`` from every compute
method instead of returning zeros.
"""

from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import HQUnavailable, check, dptr, fptr, iptr, load


class deltaETypes:  # IM:20
    CIE76 = _lib.HQ_DE_CIE76
    CIE94 = _lib.HQ_DE_CIE94
    CIEDE2000 = _lib.HQ_DE_CIEDE2000


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def pack_filters(filters, absfilters):
    """IM:800-841 ``updateOpenCLFilters`` packing: Ofilters[3][][] -> k1, k2 (T,4), k3, |k3|."""
    T = len(filters[0][0])
    k1 = np.zeros((T, 4), np.float32)
    k2 = np.zeros((T, 4), np.float32)
    for c in range(3):
        k1[:, c] = filters[c][0]
        k2[:, c] = filters[c][1]
    return k1, k2, _f32(filters[0][2]), _f32(absfilters)


class ImageManipulation:
    """IM:19-895 on libhq (one GPU, one stream)."""

    def __init__(self, deltaEType: int = deltaETypes.CIE76, verbose: bool = False,
                 convergence: bool = True, device: int = 0):
        self._lib = load()  # a missing libhq.so raises here: no silent CPU path
        self.verbose = verbose
        self.convergence = convergence
        self.deltaEType = deltaEType
        self._ctx = C.c_void_p()
        rc = self._lib.hq_create(device, deltaEType, C.byref(self._ctx))
        self.openCLAvailable = rc == _lib.HQ_OK  # IM:54, IM:78
        if rc not in (_lib.HQ_OK, _lib.HQ_ERR_DEVICE):
            check(rc)
        self.openCLFiltersReady = False
        self._filters = None

    # IM:95
    def getOpenCLAvailable(self) -> bool:
        return self.openCLAvailable

    def _require(self):
        if not self.openCLAvailable:
            raise HQUnavailable(_lib.HQ_ERR_DEVICE, "no usable GPU (IM:79-92 condition)")
        return self._ctx

    @property
    def ctx(self):
        return self._require()

    # IM:800
    def updateOpenCLFilters(self, filters, absfilters):
        ctx = self._require()
        k1, k2, k3, ak3 = pack_filters(filters, absfilters)
        check(self._lib.hq_set_filters(ctx, k1.shape[0], fptr(k1), fptr(k2), fptr(k3), fptr(ak3)),
              ctx)
        self._filters = (k1, k2, k3, ak3)
        self.openCLFiltersReady = True

    @property
    def halfSize(self) -> int:  # IM:408
        return (self._filters[0].shape[0] * 4) // 8

    # IM:100
    def RGBtoXYZ(self, R, G, B):
        ctx = self._require()
        R, G, B = _f32(R), _f32(G), _f32(B)
        out = np.zeros(4 * R.shape[0], np.float32)
        check(self._lib.hq_rgb_to_xyz(ctx, fptr(R), fptr(G), fptr(B), R.shape[0], fptr(out)), ctx)
        return out

    # IM:285
    def XYZtoScielab(self, XYZ, filters, absfilters, w, illuminant):
        ctx = self._require()
        if not self.openCLFiltersReady:
            self.updateOpenCLFilters(filters, absfilters)
        XYZ = _f32(XYZ)
        n = XYZ.shape[0] // 4
        lab = np.zeros(4 * n, np.float32)
        il = _f32(illuminant)
        check(self._lib.hq_xyz_to_scielab(ctx, fptr(XYZ), int(w), n // int(w), fptr(il),
                                          fptr(lab)), ctx)
        return lab

    # device-resident image of IM:450-478 (uploaded once per search)
    def setImage(self, rgbInline, labInline, w, illuminant, row_begin=0, row_end=None):
        ctx = self._require()
        rgb = _f32(rgbInline)
        n = rgb.shape[0] // 4
        h = n // int(w)
        lab = _f32(labInline) if labInline is not None else None
        il = _f32(illuminant)
        row_end = h if row_end is None else row_end
        check(self._lib.hq_set_image_shard(ctx, fptr(rgb), fptr(lab) if lab is not None else None,
                                           int(w), h, fptr(il), int(row_begin), int(row_end)),
              ctx)
        self.w, self.h = int(w), h

    def getLabRef(self):
        ctx = self._require()
        out = np.zeros(4 * self.w * self.h, np.float32)
        check(self._lib.hq_get_labref(ctx, fptr(out)), ctx)
        return out

    # IM:620 computeQuantizationErrorPopulation
    def computeQuantizationErrorPopulation(self, colors, delta: float = 2.0, return_used=False):
        """colors: (P, 4K) or list of float[4K] palettes -> costs (P,) [, used (P, K)]."""
        ctx = self._require()
        pal = _f32(np.stack([np.asarray(c, np.float32).reshape(-1) for c in colors]))
        P, K = pal.shape[0], pal.shape[1] // 4
        costs = np.zeros(P, np.float64)
        used = np.zeros((P, K), np.int32)
        check(self._lib.hq_eval_population(ctx, fptr(pal), P, K, float(delta), dptr(costs),
                                           iptr(used)), ctx)
        return (costs, used) if return_used else costs

    def getIndices(self, p: int = 0):
        """u8 palette index per pixel of palette p of the last population (K <= 256)."""
        ctx = self._require()
        out = np.zeros(self.w * self.h, np.uint8)
        check(self._lib.hq_get_indices(ctx, int(p), out.ctypes.data_as(_lib._u8)), ctx)
        return out

    def getPixelErrors(self, p: int = 0):
        """Per-pixel dE of palette p of the last population over the owned rows (the
        error image of IM:663-667); needs setOption("pixel_err", 1) before it."""
        ctx = self._require()
        out = np.zeros(self.w * self.h, np.float32)
        check(self._lib.hq_get_pixel_errors(ctx, int(p), fptr(out)), ctx)
        return out

    def getIndices32(self, p: int = 0):
        """32-bit palette index per pixel of palette p of the last population (any K,
        the int index of CL:172-193)."""
        ctx = self._require()
        out = np.zeros(self.w * self.h, np.uint32)
        check(self._lib.hq_get_indices32(ctx, int(p), out.ctypes.data_as(C.POINTER(C.c_uint32))), ctx)
        return out

    # IM:383
    def findBestQuantization(self, inlinergbOriginal, inlineScielabOriginal, w, nbOfColors,
                             simulatedAnnealing, filters, absfilters, illuminant,
                             iterations=None, stop=None):
        """Full SWASA search (IM:383-591) on the GPU; returns bestColors float[4K].

        ``simulatedAnnealing`` is a :class:`~hybridquantization_amd.swasa.SWASA`;
        ``stop`` is an optional callable polled between chunks (IM:499).
        """
        ctx = self._require()
        if not self.openCLFiltersReady:
            self.updateOpenCLFilters(filters, absfilters)
        # Always upload (IM:450-478 does too): an identity cache keyed on id() can
        # match a new array that reuses a freed one's id, or miss an in-place edit,
        # and the upload is small next to a 5000-iteration search.
        self.setImage(inlinergbOriginal, inlineScielabOriginal, w, illuminant)
        sw = simulatedAnnealing
        params = sw.params()
        handle = C.c_void_p()
        check(self._lib.hq_search_create(ctx, C.byref(params), int(nbOfColors), sw.seed,
                                         C.byref(handle)), ctx)
        try:
            total = params.imax if iterations is None else min(int(iterations), params.imax)
            done = 0
            while done < total:
                if stop is not None and stop():
                    break
                ran = C.c_int()
                chunk = min(64, total - done)
                check(self._lib.hq_search_run(handle, chunk, C.byref(ran)), ctx)
                done += ran.value
                if ran.value == 0:
                    break
            best = np.zeros(4 * int(nbOfColors), np.float32)
            err = C.c_double()
            it = C.c_int()
            check(self._lib.hq_search_best(handle, fptr(best), C.byref(err), C.byref(it)), ctx)
            self.bestError = err.value
            self.iterations = it.value
            if self.verbose:
                print("Final error : %.5f" % err.value)  # IM:589
            return best
        finally:
            self._lib.hq_search_destroy(handle)

    # IM:770
    def quantize(self, inlineImageRGB, colors):
        ctx = self._require()
        rgb = _f32(inlineImageRGB)
        col = _f32(colors)
        n, K = rgb.shape[0] // 4, col.shape[0] // 4
        out = np.zeros_like(rgb)
        used = np.zeros(K, np.int32)
        check(self._lib.hq_quantize(ctx, fptr(rgb), n, fptr(col), K, fptr(out), iptr(used)), ctx)
        self.lastUsedColors = used
        return out

    # IM:858
    def computeError(self, original, quantized, errorImage=None):
        ctx = self._require()
        a, b = _f32(original), _f32(quantized)
        n = a.shape[0] // 4
        img = np.zeros(4 * n, np.float32)
        mean = C.c_double()
        check(self._lib.hq_compute_error(ctx, fptr(a), fptr(b), n, fptr(img), C.byref(mean)), ctx)
        if errorImage is not None:
            errorImage[:] = img
        return mean.value

    # RCCL row-block sharding
    def initComm(self, nranks: int, rank: int, unique_id: bytes):
        ctx = self._require()
        buf = (C.c_ubyte * 128).from_buffer_copy(unique_id)
        check(self._lib.hq_comm_init(ctx, int(nranks), int(rank), buf), ctx)

    def commInfo(self) -> tuple[int, int]:
        """(ranks, this rank) of the context's RCCL communicator as RCCL reports
        them; (0, -1) without one."""
        ctx = self._require()
        n, r = C.c_int(), C.c_int()
        check(self._lib.hq_comm_info(ctx, C.byref(n), C.byref(r)), ctx)
        return n.value, r.value

    @staticmethod
    def commUniqueId() -> bytes:
        buf = (C.c_ubyte * 128)()
        check(load().hq_comm_unique_id(buf))
        return bytes(buf)

    def setOption(self, name: str, value: int):
        ctx = self._require()
        check(self._lib.hq_set_option(ctx, name.encode(), int(value)), ctx)

    # IM:265
    def close(self):
        if self._ctx:
            self._lib.hq_destroy(self._ctx)
            self._ctx = C.c_void_p()
            self.openCLAvailable = False

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
