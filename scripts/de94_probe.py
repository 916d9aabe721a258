"""dE94 (CL:217-226): how often is dH^2 = fma(da, da, db db) - dC dC negative in
fp32 (the reference's sqrt then yields NaN, and so does the mean)?  Prints,
per image size and palette, the cost of both dE formulas on the fast and the
generic path, and the NaN pixels of the per-pixel error image."""
import sys
import numpy as np

sys.path.insert(0, ".")
import hybridquantization_amd as hq  # noqa: E402
from oracle import oracle as o  # noqa: E402

for w, h in ((290, 93), (1024, 1024), (2048, 2048)):
    R, G, B = o.synthetic_image(w, h, seed=3)
    rgba = o.inline_rgba(R, G, B).reshape(-1)
    for de in (hq.deltaETypes.CIE76, hq.deltaETypes.CIE94):
        m = hq.ImageManipulation(de, device=0)
        sp = hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
        m.setImage(rgba, None, w, sp.illuminant)
        m.setOption("pixel_err", 1)
        for K in (16, 64, 256):
            pal = o.synthetic_palette(K, 7 + K)
            row = []
            for variant in (0, 1):
                m.setOption("cost_variant", variant)
                c = m.computeQuantizationErrorPopulation([pal.reshape(-1)], 2.0)[0]
                e = m.getPixelErrors(0)
                row.append(f"v{variant} cost {c:.9g} nan_px {int(np.isnan(e).sum())}")
            print(f"{w}x{h} de {int(de)} K {K}: " + "; ".join(row), flush=True)
        m.close()
