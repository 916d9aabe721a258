"""CPU check of u8_unit (hq_assign.hip): the packed-image assign path rebuilds
each channel value k/255 from its byte k as q = k * RN(1/255); r = fma(-q, 255, k);
v = fma(r, RN(1/255), q).  Checked exhaustively against the float division the
host (and the reference, IM:100's int-RGB source) makes, with every fp32
operation rounded exactly (rational arithmetic).  No GPU needed."""

from fractions import Fraction as F

import numpy as np

f32 = np.float32


def rn32(x: F) -> np.float32:
    """x rounded to the nearest float32, ties to even (x > 0 or 0)."""
    if x == 0:
        return f32(0)
    f = f32(float(x))
    cands = [np.nextafter(f, f32(-np.inf)), f, np.nextafter(f, f32(np.inf))]

    def key(c):
        return abs(F(float(c)) - x), int(np.array(c, f32).view(np.uint32)) & 1

    return f32(min(cands, key=key))


def fma32(a, b, c) -> np.float32:
    return rn32(F(float(a)) * F(float(b)) + F(float(c)))


def test_u8_unit_exact_for_all_bytes():
    c = f32(1) / f32(255)
    plain_mul_off = 0
    for k in range(256):
        kf = f32(k)
        want = kf / f32(255)  # IEEE single division, as the host builds the planes
        q = rn32(F(k) * F(float(c)))
        plain_mul_off += q != want
        r = fma32(-q, f32(255), kf)
        v = fma32(r, c, q)
        assert np.array(v, f32).view(np.uint32) == np.array(want, f32).view(np.uint32), k
    assert plain_mul_off > 0  # the correction step is needed
