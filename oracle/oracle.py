"""CPU oracle for the SWASA dE cost path -- TEST INFRASTRUCTURE ONLY.

This module is a plain numpy restatement of the reference's algorithm, used as
the *checker* for the HIP path.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it.  The product
(``hybridquantization_amd``) never imports anything under ``oracle/``.

PARITY STATUS: **pinned against the reference itself.**  The reference
(Helios77760/HybridQuantization, Java + JavaCL/OpenCL) ships no tests, golden
vectors or fixtures, and its Java host cannot run here (no JVM, no
Icy/EzPlug/JavaCL jars).  Its per-pixel kernels, one
OpenCL C file, are compiled unmodified for gfx950 (oracle/Makefile, into
oracle/_ref/) and run on the MI355X by oracle/ref_cl_host.c, a restatement of
its JavaCL host sequence; tests/test_refcl.py (GPU) checks this oracle and
libhq against them.  Further pins: line-by-line restatement,
self-consistency of the reference's constants (tests/test_oracle.py), and the
agreement of two independent restatements (this file and oracle/hq_oracle.c).

Citation tags (all under /root/reference/src/plugins/dbrasseur/hybridquantization/):
  HQ = HybridQuantization.java, IM = ImageManipulation.java,
  SP = ScielabProcessor.java,   SW = SWASA.java,
  CL = OptimizedConvolution.cl

Numerical contract for the integer output (palette index), CL:179-192 as the
reference's own OpenCL build computes ``distance`` on gfx950 (ref_len):
  d2 = fma(dz, dz, fma(dy, dy, dx*dx)) in fp32, d = v_sqrt_f32(d2) (the rescaled
  form below FLT_MIN), winner = first k with d < best (strict, ascending k).
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

f32 = np.float32

# --------------------------------------------------------------------------
# Constants (transcribed from the reference)
# --------------------------------------------------------------------------

# SP:20-21
D65 = np.array([0.95047, 1.0, 1.0883], dtype=f32)
D50 = np.array([0.966797, 1.0, 0.825188], dtype=f32)
MIN_SAMPPERDEG = 224  # SP:23

# SP:44-53
WEIGHTS = [[1.00327, 0.114416, -0.117686], [0.616725, 0.383275], [0.567885, 0.432115]]
HALFWIDTHS = [[0.05, 0.225, 7.0], [0.0685, 0.826], [0.0920, 0.6451]]

# CL:77 RGB2XYZm
RGB2XYZM = np.array([[0.4124564, 0.3575761, 0.1804375],
                     [0.2126729, 0.7151522, 0.0721750],
                     [0.0193339, 0.1191920, 0.9503041]], dtype=f32)
# CL:110 XYZ2Oppm
XYZ2OPPM = np.array([[0.2787336, 0.7218031, -0.1065520],
                     [-0.4487736, 0.2898056, -0.0771569],
                     [0.0859513, -0.5899859, 0.5011089]], dtype=f32)
# CL:118 Opp2XYZm
OPP2XYZM = np.array([[0.624045, -1.87044, -0.155304],
                     [1.36606, 0.931563, 0.433903],
                     [1.5013, 1.41761, 2.53307]], dtype=f32)
# CL:171 RGB2Oppm
RGB2OPPM = np.array([[0.266413, 0.603167, 0.00113333],
                     [-0.124957, 0.0375879, -0.133381],
                     [-0.0803345, -0.331467, 0.449132]], dtype=f32)
# CL:120-123
LABDELTA3 = f32(216.0) / f32(24389.0)
KAPPA = f32(24389.0) / f32(27.0)


# --------------------------------------------------------------------------
# fp32 helpers
# --------------------------------------------------------------------------

def fma32(a, b, c):
    """fp32 fused multiply-add, emulated via fp64 (a*b exact in fp64)."""
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64)
            + np.asarray(c, np.float64)).astype(f32)


def dot3(v, m_row):
    """float4 dot with .w = 0 (CL dot on float4): ((x*a + y*b) + z*c)."""
    v = np.asarray(v, f32)
    return (v[..., 0] * m_row[0] + v[..., 1] * m_row[1]) + v[..., 2] * m_row[2]


def srgb_lin(x):
    """Gamma expansion as in CL:85-87 / CL:194-196 (fp32 pow)."""
    x = np.asarray(x, f32)
    lo = x / f32(12.92)
    base = (x + f32(0.055)) / f32(1.055)
    with np.errstate(invalid="ignore"):
        # OpenCL pow(float, 2.4f): the exponent is the fp32 literal 2.4f
        hi = np.power(base.astype(np.float64), float(f32(2.4))).astype(f32)
    return np.where(x <= f32(0.04045), lo, hi).astype(f32)


# --------------------------------------------------------------------------
# S-CIELAB filter design  (SP:66-181, gauss SP:238-254, conv1D SP:185-201,
# resize1D SP:203-220, extractWithIndices SP:222-230) + packing IM:800-841
# --------------------------------------------------------------------------

def gauss(halfwidth: np.float32, width: int) -> np.ndarray:
    """SP:238-254 with Java float/double promotion rules."""
    hw = f32(halfwidth)
    alpha = f32(f32(2) * f32(math.sqrt(math.log(2)))) / f32(hw - f32(1))
    res = np.zeros(width, dtype=f32)
    offset = width // 2
    s = 0.0
    for i in range(width):
        d = f32(i - offset)
        e = f32(f32(f32(-alpha) * alpha) * d) * d
        res[i] = f32(math.exp(float(e)))
        s += float(res[i])
    for i in range(width):
        res[i] = f32(float(res[i]) / s)
    return res


def conv1d(data: np.ndarray, filt: np.ndarray) -> np.ndarray:
    """SP:185-201: float accumulation, zero outside, no fma."""
    n = len(data)
    res = np.zeros(n, dtype=f32)
    off = len(filt) // 2
    for i in range(n):
        acc = f32(0)
        for j in range(-off, off + 1):
            if 0 <= i + j < n:
                acc = f32(acc + f32(filt[j + off] * data[i + j]))
        res[i] = acc
    return res


def resize1d(src: np.ndarray, new_size: int) -> np.ndarray:
    """SP:203-220."""
    pad = abs(new_size - len(src)) // 2
    if new_size > len(src):
        res = np.zeros(new_size, dtype=f32)
        res[pad:pad + len(src)] = src
        return res
    return np.array(src[pad:pad + new_size], dtype=f32)


@dataclass
class Filters:
    k1: np.ndarray      # [T,4] float32 (g00, g10, g20, 0)      IM:804-815
    k2: np.ndarray      # [T,4] float32 (g01, g11, g21, 0)
    k3: np.ndarray      # [T]   float32 g02 (signed)            IM:816-826
    absk3: np.ndarray   # [T]   float32 |g02|                   SP:174-178
    half: int           # filters4[0].length/8                  IM:408
    illum: np.ndarray   # [3]   whitepoint                      SP:69-76
    ofilters: list      # raw Ofilters[3][][]

    @property
    def taps(self) -> int:
        return self.k1.shape[0]


def samp_per_deg(dpi: int, viewing_distance: float):
    """SP:79-88 -> (sampPerDeg after uprate, uprate)."""
    spd = int(math.floor(dpi / ((180 / math.pi) * math.atan(2.54 / viewing_distance)) + 0.5))
    if spd < MIN_SAMPPERDEG:
        uprate = int(math.ceil(MIN_SAMPPERDEG * 1.0 / spd))
        spd *= uprate
    else:
        uprate = 1
    return spd, uprate


def design_filters(dpi: int = 72, viewing_distance: float = 45.0,
                   whitepoint: str = "D65") -> Filters:
    """ScielabProcessor constructor SP:66-181, then updateOpenCLFilters IM:800-841."""
    illum = (D50 if whitepoint == "D50" else D65).copy()
    spd, uprate = samp_per_deg(dpi, float(f32(viewing_distance)))
    spreads = [[f32(f32(h) * f32(spd)) for h in row] for row in HALFWIDTHS]
    width = int(math.ceil(spd / 2.0)) * 2 - 1
    of = [[None] * 3, [None] * 2, [None] * 2]
    for i in range(3):
        for j in range(len(of[i])):
            g = gauss(spreads[i][j], width)
            w = f32(WEIGHTS[i][j])
            factor = f32(f32(math.sqrt(abs(float(w)))) * f32(np.sign(w)))
            of[i][j] = (g * factor).astype(f32)
    if uprate > 1:
        upcol = np.array([f32(f32((uprate - abs(uprate - i - 1)) * 1.0) / f32(uprate))
                          for i in range(uprate * 2 - 1)], dtype=f32)
        upcol = resize1d(upcol, len(upcol) + width - 1)
        ups = [[conv1d(of[i][j], upcol) for j in range(len(of[i]))] for i in range(3)]
        s = len(ups[0][0])
        mid = s // 2
        temp = list(range(mid, mid - uprate * (mid // uprate) - 1, -uprate))[: (mid // uprate) + 1]
        temp.reverse()
        downs = []
        j = mid + uprate
        for i in range(2 * (mid // uprate) + 1):
            if i < len(temp):
                downs.append(temp[i])
            else:
                downs.append(j)
                j += uprate
        of = [[ups[i][j][downs].astype(f32) for j in range(len(ups[i]))] for i in range(3)]
    absk3 = np.where(of[0][2] < 0, -of[0][2], of[0][2]).astype(f32)
    T = len(of[0][0])
    k1 = np.zeros((T, 4), dtype=f32)
    k2 = np.zeros((T, 4), dtype=f32)
    for c in range(3):
        k1[:, c] = of[c][0]
        k2[:, c] = of[c][1]
    k3 = of[0][2].astype(f32)
    half = (T * 4) // 8
    return Filters(k1=k1, k2=k2, k3=k3, absk3=absk3, half=half, illum=illum, ofilters=of)


# --------------------------------------------------------------------------
# Per-pixel colour conversions
# --------------------------------------------------------------------------

def rgb_to_xyz(R, G, B):
    """CL:79-90 RGB2XYZ -> float4 [N,4] (.w = 0)."""
    rgb = np.stack([srgb_lin(R), srgb_lin(G), srgb_lin(B)], axis=-1)
    out = np.zeros(rgb.shape[:-1] + (4,), dtype=f32)
    for i in range(3):
        out[..., i] = dot3(rgb, RGB2XYZM[i])
    return out


def xyz_to_opp(xyz):
    """CL:111-116 XYZ2Opp."""
    out = np.zeros_like(xyz, dtype=f32)
    for i in range(3):
        out[..., i] = dot3(xyz, XYZ2OPPM[i])
    return out


def opp_to_lab(opp, illum):
    """CL:124-145 Opp2LAB (cbrt branch, kappa linear branch)."""
    opp = np.asarray(opp, f32)
    X = dot3(opp, OPP2XYZM[0])
    Y = dot3(opp, OPP2XYZM[1])
    Z = dot3(opp, OPP2XYZM[2])

    def f(t):
        t = t.astype(f32)
        lin = (fma32(KAPPA, t, f32(16.0)) / f32(116.0)).astype(f32)
        return np.where(t > LABDELTA3, np.cbrt(t.astype(np.float64)).astype(f32), lin).astype(f32)

    fx = f(X / illum[0])
    fy = f(Y / illum[1])
    fz = f(Z / illum[2])
    out = np.zeros(opp.shape[:-1] + (4,), dtype=f32)
    out[..., 0] = f32(116.0) * fy - f32(16.0)
    out[..., 1] = f32(500.0) * (fx - fy)
    out[..., 2] = f32(200.0) * (fy - fz)
    return out


def ciede76(lab1, lab2):
    """CL:201-209 with -DCIE76: distance(p1.xyz, p2.xyz)."""
    d = (np.asarray(lab1, f32)[..., :3] - np.asarray(lab2, f32)[..., :3]).astype(f32)
    s = (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]
    return np.sqrt(s.astype(f32)).astype(f32)


def ciede94(lab1, lab2):
    """CL:217-226 (-DCIE94 branch); ``sc``/``sh`` use double literals 0.045/0.015."""
    p1 = np.asarray(lab1, np.float64)
    p2 = np.asarray(lab2, np.float64)
    L1, a1, b1 = p1[..., 0], p1[..., 1], p1[..., 2]
    L2, a2, b2 = p2[..., 0], p2[..., 1], p2[..., 2]
    dL = L1 - L2
    c1 = np.sqrt(a1 * a1 + b1 * b1)
    dC = c1 - np.sqrt(a2 * a2 + b2 * b2)
    da, db = a1 - a2, b1 - b2
    dH = np.sqrt(np.maximum(da * da + db * db - dC * dC, 0.0))
    sc = 1 + 0.045 * c1
    sh = 1 + 0.015 * c1
    return np.sqrt(dL * dL + (dC / sc) ** 2 + (dH / sh) ** 2).astype(f32)


def _fma32(a, b, c):
    """fp32 fma(a, b, c): the product is exact in float64, the sum rounds once
    there and once more to fp32 (a double rounding that differs from one fused
    rounding only on rare ties)."""
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(f32)


def ciede94_f32(lab1, lab2):
    """CL:217-226 statement by statement in fp32: fma as one rounding, sc and sh
    from double literals (1 + 0.045 c1 in double, stored as float), and no clamp
    before sqrt(fma(da, da, db db) - dC dC) -- the reference returns NaN where
    rounding makes dH^2 negative (the hue difference below ~1e-4 of the chroma
    difference), and so does this restatement (`ciede94` clamps at 0)."""
    p1 = np.asarray(lab1, f32)
    p2 = np.asarray(lab2, f32)
    L1, a1, b1 = p1[..., 0], p1[..., 1], p1[..., 2]
    L2, a2, b2 = p2[..., 0], p2[..., 1], p2[..., 2]
    with np.errstate(invalid="ignore"):
        dL = (L1 - L2).astype(f32)
        c1 = np.sqrt(_fma32(a1, a1, (b1 * b1).astype(f32)))
        dC = (c1 - np.sqrt(_fma32(a2, a2, (b2 * b2).astype(f32)))).astype(f32)
        da = (a1 - a2).astype(f32)
        db = (b1 - b2).astype(f32)
        dH = np.sqrt((_fma32(da, da, (db * db).astype(f32)) - (dC * dC).astype(f32)).astype(f32))
        sc = (1 + 0.045 * c1.astype(np.float64)).astype(f32)
        sh = (1 + 0.015 * c1.astype(np.float64)).astype(f32)
        dcs = (dC / sc).astype(f32)
        dhs = (dH / sh).astype(f32)
        return np.sqrt(_fma32(dL, dL, _fma32(dcs, dcs, (dhs * dhs).astype(f32)))).astype(f32)


# --------------------------------------------------------------------------
# Separable stencil helpers (reflection CL:256-263)
# --------------------------------------------------------------------------

def reflect_index(n: int, half: int) -> np.ndarray:
    """Index table [n, 2*half+1]: j+i reflected as in CL:256-263."""
    j = np.arange(n)[:, None] + np.arange(-half, half + 1)[None, :]
    j = np.where(j < 0, -j - 1, j)
    j = np.where(j >= n, 2 * n - j - 1, j)
    if (j < 0).any() or (j >= n).any():
        raise ValueError(f"image dimension {n} too small for stencil half-width {half}")
    return j


def _hpass(img, w_taps, half):
    """Horizontal pass on [H, W, C] with per-tap sequential fma (taps [T, C])."""
    H, W, C = img.shape
    idx = reflect_index(W, half)
    acc = np.zeros((H, W, C), dtype=f32)
    for t in range(2 * half + 1):
        acc = fma32(img[:, idx[:, t], :], w_taps[t], acc)
    return acc


def _vpass(img, w_taps, half):
    H, W, C = img.shape
    idx = reflect_index(H, half)
    acc = np.zeros((H, W, C), dtype=f32)
    for t in range(2 * half + 1):
        acc = fma32(img[idx[:, t], :, :], w_taps[t], acc)
    return acc


def xyz_to_scielab(xyz4, filt: Filters, w: int):
    """IM:285-370: XYZ2Opp, filter-by-filter separable convolutions, Opp2LAB.

    xyz4: [N,4] inline float4 (row-major, pixel = y*w + x).  Returns Lab [N,4].
    Accumulation order: conv = V1H1(opp); conv += V2H2(opp); conv.x += V3H3(opp.x)
    (IM:322-346), each pass a sequential per-tap fma (CL:18-29, CL:58-66).
    """
    n = xyz4.shape[0]
    h = n // w
    half = filt.half
    opp = xyz_to_opp(xyz4).reshape(h, w, 4)
    o3 = opp[..., :3]
    c1 = _vpass(_hpass(o3, filt.k1[:, :3], half), filt.k1[:, :3], half)
    c2 = _vpass(_hpass(o3, filt.k2[:, :3], half), filt.k2[:, :3], half)
    conv = (c1 + c2).astype(f32)
    t3 = _hpass(o3[..., :1], filt.k3[:, None], half)
    c3 = _vpass(t3, filt.absk3[:, None], half)
    conv[..., 0] = (conv[..., 0] + c3[..., 0]).astype(f32)
    conv4 = np.zeros((h, w, 4), dtype=f32)
    conv4[..., :3] = conv
    return opp_to_lab(conv4.reshape(n, 4), filt.illum)


def srgb_to_scielab(R, G, B, filt: Filters, w: int):
    """SP:374-381 -> IM.RGBtoXYZ (IM:100) -> IM.XYZtoScielab (IM:285)."""
    return xyz_to_scielab(rgb_to_xyz(R, G, B), filt, w)


# --------------------------------------------------------------------------
# Candidate evaluation: steps a-h of SURVEY section 0
# --------------------------------------------------------------------------

def fma32(a, b, c):
    """fp32 fma(a, b, c) with one rounding: the product is exact in float64, the
    sum is carried as a float64 plus its exact error (TwoSum), and a float64 sum
    that lands exactly on an fp32 midpoint is moved one float64 ulp towards the
    exact value before the rounding to fp32 (round-to-nearest-even otherwise)."""
    x = np.asarray(a, np.float64) * np.asarray(b, np.float64)
    c = np.asarray(c, np.float64)
    s = x + c
    bb = s - x
    err = (x - (s - bb)) + (c - bb)
    r = s.astype(f32)
    rd = r.astype(np.float64)
    other = np.nextafter(r, np.where(rd < s, f32(np.inf), f32(-np.inf))).astype(np.float64)
    mid = (rd != s) & (s == 0.5 * (rd + other)) & (err != 0)
    if np.any(mid):
        s = np.where(mid, np.nextafter(s, s + err), s)
        r = s.astype(f32)
    return r


_SQRT = None  # the device's square root (set_sqrt); None: correctly rounded


def set_sqrt(fn):
    """The square root of the argmin's distance: a function of an fp32 array
    (the GPU tests pass v_sqrt_f32 itself through a test-only helper), or None
    for the correctly rounded one (see ref_len)."""
    global _SQRT
    _SQRT = fn


def _dev_sqrt(x):
    x = np.asarray(x, f32)
    with np.errstate(invalid="ignore"):
        return np.sqrt(x).astype(f32) if _SQRT is None else np.asarray(_SQRT(x), f32)


def ref_len(dx, dy, dz):
    """CL:179-192 distance() as the reference's OpenCL build computes it on gfx950
    (disassembly of its quantize kernels, oracle/_ref), w = 0:
    d2 = fma(dz, dz, fma(dy, dy, dx*dx)); d = sqrt(d2) for FLT_MIN <= d2 < inf
    (and NaN), else the library's rescaled form (components x 2^86, or x 2^-66
    at inf, the same chain, sqrt with an ldexp 32 / -16 step for a subnormal
    sum, and back).  sqrt is the device's v_sqrt_f32 when set_sqrt gave it
    (monotone, within 1 ulp, 1 ulp off on 15.1% of the normal floats), else
    correctly rounded."""
    dx, dy, dz = (np.asarray(v, f32) for v in (dx, dy, dz))
    with np.errstate(over="ignore", under="ignore", invalid="ignore"):
        d2 = fma32(dz, dz, fma32(dy, dy, (dx * dx).astype(f32)))
        small = d2 < f32(2.0 ** -126)
        big = ~small & (d2 != np.inf)
        out = np.empty_like(d2)
        out[big] = _dev_sqrt(d2[big])
        rest = ~big
        if np.any(rest):
            sm = small[rest]
            sc = np.where(sm, f32(2.0 ** 86), f32(2.0 ** -66)).astype(f32)
            x, y, z = ((v[rest] * sc).astype(f32) for v in (dx, dy, dz))
            e = fma32(z, z, fma32(y, y, (x * x).astype(f32)))
            den = e < f32(2.0 ** -126)
            e = np.ldexp(e, np.where(den, 32, 0)).astype(f32)
            r = np.ldexp(_dev_sqrt(e), np.where(den, -16, 0)).astype(f32)
            out[rest] = (r * np.where(sm, f32(2.0 ** -86), f32(2.0 ** 66))).astype(f32)
    return out


def assign(rgb3, palette4):
    """CL:172-193 argmin: the first k whose ref_len distance is below the best
    so far (strict <): a NaN distance never wins unless colour 0's is NaN.

    rgb3: [N,3] fp32, palette4: [K,4].  The .w lanes are 0 on both sides in the
    reference (HQ:288 makeinline, SW:49/99), so the w term of ``distance`` is 0.
    Returns (idx int32 [N], used int32 [K]).
    """
    rgb3 = np.asarray(rgb3, f32)[:, :3]
    pal = np.asarray(palette4, f32)[:, :3]
    K, N = pal.shape[0], rgb3.shape[0]
    idx = np.zeros(N, dtype=np.int32)
    step = max(1, (1 << 22) // K)  # pixels per chunk: K x step distances at a time
    for q0 in range(0, N, step):
        px = rgb3[q0:q0 + step]
        d = (px[None, :, :] - pal[:, None, :]).astype(f32)  # [K, n, 3]
        key = ref_len(d[..., 0].ravel(), d[..., 1].ravel(), d[..., 2].ravel()).reshape(K, -1)
        nan0 = np.isnan(key[0])
        key = np.where(np.isnan(key), f32(np.inf), key)
        ix = np.argmin(key, axis=0).astype(np.int32)  # the first minimum
        ix[nan0] = 0
        idx[q0:q0 + step] = ix
    used = np.zeros(K, dtype=np.int32)
    used[np.unique(idx)] = 1
    return idx, used


def palette_opp(palette4):
    """CL:194-198: gamma + RGB2Oppm of each palette colour -> [K,4]."""
    lin = np.stack([srgb_lin(palette4[:, c]) for c in range(3)], axis=-1)
    out = np.zeros((palette4.shape[0], 4), dtype=f32)
    for i in range(3):
        out[:, i] = dot3(lin, RGB2OPPM[i])
    return out


def candidate_scielab(idx, palette4, filt: Filters, w: int, h: int):
    """Opp of the quantized image -> Temp (CL:234-272) -> End (CL:274-306) -> Opp2LAB.

    Temp:  t1 = sum fma(in, k1), t2 = sum fma(in, k2), t3 = sum fma(in.x, k3)
    End:   out = fma(t1, k1, fma(t2, k2, out)); out.x = fma(t3, |k3|, out.x)
    (End runs with W<->H swapped on the transposed data, IM:485, i.e. the
    vertical pass.)  Returns Lab [N,4].
    """
    half = filt.half
    T = 2 * half + 1
    opp = palette_opp(palette4)[idx].reshape(h, w, 4)[..., :3]
    # horizontal
    hidx = reflect_index(w, half)
    t1 = np.zeros((h, w, 3), f32)
    t2 = np.zeros((h, w, 3), f32)
    t3 = np.zeros((h, w), f32)
    for t in range(T):
        src = opp[:, hidx[:, t], :]
        t1 = fma32(src, filt.k1[t, :3], t1)
        t2 = fma32(src, filt.k2[t, :3], t2)
        t3 = fma32(src[..., 0], filt.k3[t], t3)
    # vertical
    vidx = reflect_index(h, half)
    out = np.zeros((h, w, 3), f32)
    for t in range(T):
        r = vidx[:, t]
        out = fma32(t1[r], filt.k1[t, :3], fma32(t2[r], filt.k2[t, :3], out))
        out[..., 0] = fma32(t3[r], filt.absk3[t], out[..., 0])
    conv4 = np.zeros((h, w, 4), f32)
    conv4[..., :3] = out
    return opp_to_lab(conv4.reshape(h * w, 4), filt.illum)


def shard_partial(rgb3, lab_ref4, palette4, filt: Filters, w: int, h: int, r0: int, r1: int):
    """Row-block shard of the candidate cost: uses only RGB rows
    [r0-half, r1+half) clipped to the image (halo re-quantised locally, reflection
    only at true edges) and LabRef rows [r0, r1).  Returns (fp64 dE sum over the
    owned rows, used flags of the extended rows)."""
    half = filt.half
    e0, e1 = max(0, r0 - half), min(h, r1 + half)
    ext = np.asarray(rgb3, f32).reshape(h, w, 3)[e0:e1].reshape(-1, 3)
    idx, used = assign(ext, palette4)
    opp = palette_opp(palette4)[idx].reshape(e1 - e0, w, 4)[..., :3]
    hidx = reflect_index(w, half)
    T = 2 * half + 1
    t1 = np.zeros((e1 - e0, w, 3), f32)
    t2 = np.zeros((e1 - e0, w, 3), f32)
    t3 = np.zeros((e1 - e0, w), f32)
    for t in range(T):
        src = opp[:, hidx[:, t], :]
        t1 = fma32(src, filt.k1[t, :3], t1)
        t2 = fma32(src, filt.k2[t, :3], t2)
        t3 = fma32(src[..., 0], filt.k3[t], t3)
    vidx = reflect_index(h, half)[r0:r1] - e0
    out = np.zeros((r1 - r0, w, 3), f32)
    for t in range(T):
        r = vidx[:, t]
        out = fma32(t1[r], filt.k1[t, :3], fma32(t2[r], filt.k2[t, :3], out))
        out[..., 0] = fma32(t3[r], filt.absk3[t], out[..., 0])
    conv4 = np.zeros((r1 - r0, w, 4), f32)
    conv4[..., :3] = out
    lab = opp_to_lab(conv4.reshape(-1, 4), filt.illum)
    err = ciede76(np.asarray(lab_ref4, f32).reshape(h, w, 4)[r0:r1].reshape(-1, 4), lab)
    return float(np.sum(err.astype(np.float64))), used


def sum_array(arr, depth: int) -> float:
    """IM:741-768: recursive halving to ``depth``, sequential fp64 leaf sums."""
    def rec(s, e, d):
        if e <= s:
            return 0.0
        if d <= 0:
            return float(np.sum(arr[s:e].astype(np.float64))) if e - s > 0 else 0.0
        m = (s + e) // 2
        return rec(s, m, d - 1) + rec(m, e, d - 1)
    return rec(0, len(arr), depth)


def default_depth(ncpu: int = 8) -> int:
    """IM:738: 32 - Integer.numberOfLeadingZeros(ncpu)."""
    return int(ncpu).bit_length()


def average_array(arr, depth: int = 4) -> float:
    """IM:736-739."""
    return sum_array(np.asarray(arr, f32), depth) / len(arr)


def compute_penalty(used, delta: float) -> float:
    """SW:74-82 (delta is a float field added into a double)."""
    return float(np.count_nonzero(np.asarray(used) == 0)) * float(f32(delta))


def eval_palette(rgb3, lab_ref4, palette4, filt: Filters, w: int, delta: float = 2.0,
                 depth: int = 4, return_parts: bool = False):
    """One candidate cost C(palette) (IM:647-712): mean dE76 + delta * #unused."""
    n = rgb3.shape[0]
    h = n // w
    idx, used = assign(rgb3, palette4)
    lab = candidate_scielab(idx, palette4, filt, w, h)
    err = ciede76(lab_ref4, lab)
    cost = average_array(err, depth) + compute_penalty(used, delta)
    if return_parts:
        return cost, dict(idx=idx, used=used, lab=lab, err=err)
    return cost


def quantize(rgb3, palette4):
    """CL:147-170 / IM:770-798: the chosen colour per pixel as float4."""
    idx, used = assign(rgb3, palette4)
    return palette4[idx].astype(f32), idx, used


def compute_error(orig_lab4, quant_lab4):
    """IM:858-894: mean dE76 (fp64 sequential) and the (255-e)^2/255^2 error image."""
    e = ciede76(orig_lab4, quant_lab4)
    err_img = ((f32(255) - e) * (f32(255) - e) / f32(255 * 255)).astype(f32)
    total = 0.0
    for v in e.astype(np.float64):
        total += v
    return total / len(e), err_img


# --------------------------------------------------------------------------
# SWASA policy (SW:14-116) with java.util.Random-compatible RNG
# --------------------------------------------------------------------------

class JavaRandom:
    """java.util.Random (48-bit LCG): nextFloat = next(24)/2^24, nextDouble 53-bit."""

    MULT = 0x5DEECE66D
    MASK = (1 << 48) - 1

    def __init__(self, seed: int):
        self.seed = (seed ^ self.MULT) & self.MASK

    def next(self, bits: int) -> int:
        self.seed = (self.seed * self.MULT + 0xB) & self.MASK
        r = self.seed >> (48 - bits)
        if r >= 1 << 31:
            r -= 1 << 32  # Java (int) cast: only values with bit 31 set (bits == 32) wrap
        return r

    def next_float(self) -> np.float32:
        return f32(self.next(24) / float(1 << 24))

    def next_double(self) -> float:
        return ((self.next(26) << 27) + self.next(27)) * (1.0 / (1 << 53))


@dataclass
class SwasaParams:
    population: int = 4      # HQ:197
    imax: int = 5000         # HQ:199
    iTc: int = 20            # HQ:214
    delta: float = 2.0       # HQ:201
    conv_delay: float = 0.75  # HQ:206
    conv_spread: float = 0.15  # HQ:208
    t0: float = 20.0         # HQ:212
    alpha: float = 0.9       # HQ:216
    s0: float = 100.0        # HQ:223
    beta: float = 5.3        # HQ:224
    convergence: bool = True  # HQ:204


class Swasa:
    """SW:3-116 restated; all float fields kept in fp32 as in Java."""

    def __init__(self, p: SwasaParams, seed: int):
        self.p = p
        self.rng = JavaRandom(seed)
        self.imax = p.imax
        self.iTc = p.iTc
        self.delta = f32(p.delta)
        self.t0 = f32(p.t0)
        self.alpha = f32(p.alpha)
        self.s0 = f32(p.s0)
        self.beta = f32(p.beta)
        self.conv_delay = f32(p.conv_delay)
        self.conv_rate = f32(p.conv_spread)
        self.reset()

    def reset(self):  # SW:30-34
        self.temperature = self.t0
        self.step_width = self.s0

    def generate_random_colors(self, K):  # SW:40-52
        c = np.zeros((K, 4), dtype=f32)
        for i in range(K):
            c[i, 0] = self.rng.next_float()
            c[i, 1] = self.rng.next_float()
            c[i, 2] = self.rng.next_float()
        return c

    def is_accepted(self, delta_e: float) -> bool:  # SW:54-57
        return delta_e <= 0 or math.exp(-delta_e / float(self.temperature)) > self.rng.next_double()

    def keeps_his_values(self, iteration: int) -> bool:  # SW:59-62
        num = f32(f32(iteration) - f32(self.conv_delay * f32(self.imax)))
        den = f32(self.conv_rate * f32(self.imax))
        return -(math.tanh(float(f32(num / den)))) / 2 + 0.5 > self.rng.next_double()

    def max_step_width(self, i: int) -> np.float32:  # SW:69-72
        e = float(f32(f32(self.beta * f32(i)) / f32(self.imax)))
        return f32(float(f32(f32(2) * self.s0)) / (1 + math.exp(e)))

    def reduce_temperature_if_necessary(self, iteration: int):  # SW:84-89
        if iteration % self.iTc == 0:
            self.temperature = f32(self.temperature * self.alpha)

    def generate_neighboring_colors(self, colors, K, iteration):  # SW:91-101
        amax = f32(self.max_step_width(iteration) / f32(256.0))
        nxt = np.zeros_like(colors)
        for i in range(K):
            for c in range(3):
                u = self.rng.next_float()
                v = f32(colors[i, c] + f32(f32(f32(u * f32(2)) - f32(1)) * amax))
                nxt[i, c] = f32(0) if not v > f32(0) else (f32(1) if v > f32(1) else v)
        return nxt


def argmin_first(arr) -> int:
    """IM:843-856."""
    m = 0
    s = arr[0]
    for i in range(1, len(arr)):
        if s > arr[i]:
            m = i
            s = arr[i]
    return m


def find_best_quantization(eval_population, K: int, sw: Swasa, iterations=None,
                           trace=None):
    """IM:383-591 main loop with a pluggable population evaluator.

    eval_population(list_of_palettes[K,4]) -> list of costs (float).
    Returns (best_colors [K,4], best_error).
    """
    p = sw.p
    P = p.population
    imax = sw.imax if iterations is None else iterations
    sw.reset()
    colors = [sw.generate_random_colors(K) for _ in range(P)]
    current_errors = list(eval_population(colors))
    m = argmin_first(current_errors)
    best_error = current_errors[m]
    best_colors = colors[m].copy()
    for ite in range(1, imax + 1):
        sw.reduce_temperature_if_necessary(ite)
        current = [sw.generate_neighboring_colors(colors[j], K, ite) for j in range(P)]
        errors = list(eval_population(current))
        minerror = float("inf")
        minidx = 0
        for i in range(P):
            if P > 1 and errors[i] < minerror:
                minerror = errors[i]
                minidx = i
            if sw.is_accepted(errors[i] - current_errors[i]):
                current_errors[i] = errors[i]
                colors[i] = current[i].copy()
                if current_errors[i] < best_error:
                    best_error = current_errors[i]
                    best_colors = current[i].copy()
        if p.convergence and P > 1:
            for i in range(P):
                if not sw.keeps_his_values(ite):
                    current_errors[i] = minerror
                    colors[i] = current[minidx].copy()
        if trace is not None:
            trace.append((ite, list(errors), list(current_errors), best_error))
    return best_colors, best_error


# --------------------------------------------------------------------------
# Synthetic inputs
# --------------------------------------------------------------------------

def splitmix64(seed: int, n: int) -> np.ndarray:
    """n outputs of SplitMix64 starting from ``seed`` (vectorised)."""
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def synthetic_image(w: int, h: int, seed: int = 1):
    """u8 uniform per channel -> u8/255.0f; returns planar R, G, B float32 [N]."""
    z = splitmix64(seed, w * h)
    r = (z & np.uint64(0xFF)).astype(np.uint8)
    g = ((z >> np.uint64(8)) & np.uint64(0xFF)).astype(np.uint8)
    b = ((z >> np.uint64(16)) & np.uint64(0xFF)).astype(np.uint8)
    s = f32(255.0)
    return r.astype(f32) / s, g.astype(f32) / s, b.astype(f32) / s


def synthetic_palette(K: int, seed: int):
    """(rng>>40) * 2^-24 in [0,1) like java.util.Random.nextFloat; .w = 0."""
    z = splitmix64(seed, 3 * K)
    v = ((z >> np.uint64(40)).astype(np.float64) * (1.0 / (1 << 24))).astype(f32)
    pal = np.zeros((K, 4), dtype=f32)
    pal[:, :3] = v.reshape(K, 3)
    return pal


def inline_rgba(R, G, B):
    """HQ:279-291 makeinline: planar -> float4 RGBA with .w = 0."""
    out = np.zeros((len(R), 4), dtype=f32)
    out[:, 0], out[:, 1], out[:, 2] = R, G, B
    return out
