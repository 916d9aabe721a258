"""Mirror of the reference's ``ScielabProcessor`` (SP) and of the plugin's
``quantization`` flow (HQ:93-137), on libhq.

Filter design (SP:66-181) runs in libhq's host code (``hq_design_filters``);
all pixel work goes through :class:`ImageManipulation` on the GPU.
"""

from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, fptr, load
from .image_manipulation import ImageManipulation, deltaETypes


class Whitepoint:  # SP:19
    D50 = _lib.HQ_WP_D50
    D65 = _lib.HQ_WP_D65


def design_filters(dpi: int = 72, viewingDistance: float = 45.0,
                   whitepoint: int = Whitepoint.D65, max_taps: int = 512):
    """SP:66-181 + IM:800-841 packing -> (k1 (T,4), k2 (T,4), k3 (T,), absk3 (T,), illum (3,))."""
    lib = load()
    k1 = np.zeros(4 * max_taps, np.float32)
    k2 = np.zeros(4 * max_taps, np.float32)
    k3 = np.zeros(max_taps, np.float32)
    ak3 = np.zeros(max_taps, np.float32)
    il = np.zeros(3, np.float32)
    taps = C.c_int()
    check(lib.hq_design_filters(int(dpi), float(np.float32(viewingDistance)), int(whitepoint),
                                max_taps, fptr(k1), fptr(k2), fptr(k3), fptr(ak3),
                                C.byref(taps), fptr(il)))
    T = taps.value
    return (k1[:4 * T].reshape(T, 4).copy(), k2[:4 * T].reshape(T, 4).copy(), k3[:T].copy(),
            ak3[:T].copy(), il)


class ScielabProcessor:
    """SP:18-444 (the parts on the plugin's execution path)."""

    def __init__(self, dpi, viewingDistance, whitepoint, HQ=None, imageProcessor=None):
        k1, k2, k3, ak3, il = design_filters(dpi, viewingDistance, whitepoint)
        self.illuminant = il
        # Ofilters[3][] as in SP:104-107 (channel i, filter j)
        self.Ofilters = [[k1[:, 0].copy(), k2[:, 0].copy(), k3.copy()],
                         [k1[:, 1].copy(), k2[:, 1].copy()],
                         [k1[:, 2].copy(), k2[:, 2].copy()]]
        self.absOfilters = ak3
        self.plugin = HQ
        self.imageProcessing = imageProcessor
        if imageProcessor is not None:
            imageProcessor.updateOpenCLFilters(self.Ofilters, self.absOfilters)  # SP:180

    # SP:374
    def sRGBToScielab(self, image, w):
        xyz = self.imageProcessing.RGBtoXYZ(image[0], image[1], image[2])
        return self.imageProcessing.XYZtoScielab(xyz, self.Ofilters, self.absOfilters, w,
                                                 self.illuminant)

    # SP:383
    def bestColors(self, inlineRGB, inlineSCIELab, w, nbOfColors, simulatedAnnealing, **kw):
        return self.imageProcessing.findBestQuantization(inlineRGB, inlineSCIELab, w, nbOfColors,
                                                         simulatedAnnealing, self.Ofilters,
                                                         self.absOfilters, self.illuminant, **kw)

    # SP:440
    def close(self):
        self.imageProcessing.close()


def makeinline(image):
    """HQ:279-291: planar (3, N) -> inline RGBA float32[4N] with .w = 0."""
    image = np.asarray(image, np.float32)
    out = np.zeros((image.shape[1], 4), np.float32)
    out[:, :3] = image[:3].T
    return out.reshape(-1)


def makeChannels(inline):
    """HQ:293-309."""
    a = np.asarray(inline, np.float32).reshape(-1, 4)
    return [a[:, 0].copy(), a[:, 1].copy(), a[:, 2].copy()]


def quantization(image, w, nbOfColors, swasa, dpi=72, viewingDistance=45.0,
                 whitepoint=Whitepoint.D65, verbose=False, device=0, iterations=None):
    """HQ:93-137 without the GUI: planar float image (3, N) in [0,1] ->
    (quantized planar image (3, N), bestColors float[4K], best error)."""
    ip = ImageManipulation(deltaETypes.CIE76, verbose, swasa.convergence, device=device)
    try:
        inline_rgb = makeinline(image)
        sp = ScielabProcessor(dpi, viewingDistance, whitepoint, None, ip)
        sc_img = sp.sRGBToScielab(image, w)
        best = sp.bestColors(inline_rgb, sc_img, w, nbOfColors, swasa, iterations=iterations)
        q = ip.quantize(inline_rgb, best)
        return np.stack(makeChannels(q)), best, ip.bestError
    finally:
        ip.close()
