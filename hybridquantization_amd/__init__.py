"""hybridquantization_amd -- MI355X-native SWASA dE cost evaluator.

Drop-in for the hot path of Helios77760/HybridQuantization: the candidate
palette cost of the plugin's simulated-annealing search (S-CIELAB dE76 of the
quantized image + unused-colour penalty), evaluated by hand-written gfx950 HIP
kernels in ``libhq.so`` behind the C ABI of ``include/hq.h``.

Python entry points mirror the reference's Java classes:
``ImageManipulation`` (IM), ``ScielabProcessor`` (SP), ``SWASA`` (SW).
"""

from ._lib import HQError, HQUnavailable, LIB_PATH, load  # noqa: F401
from .image_manipulation import ImageManipulation, deltaETypes, pack_filters  # noqa: F401
from .scielab_processor import (ScielabProcessor, Whitepoint, design_filters,  # noqa: F401
                                makeChannels, makeinline, quantization)
from .swasa import SWASA  # noqa: F401

__all__ = ["ImageManipulation", "ScielabProcessor", "SWASA", "deltaETypes", "Whitepoint",
           "design_filters", "makeinline", "makeChannels", "quantization", "HQError",
           "HQUnavailable", "load", "LIB_PATH", "pack_filters"]
