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


def test_cell_from_bytes_matches_float_cell():
    """cell_u8 (hq_assign.hip): the level-2 cell of a packed 8-bit pixel taken
    from its bytes, k >> (8 - lg G2), equals quad_cell's min((int)(v G2), G2 - 1)
    on v = k/255 rounded to fp32 (the value u8_unit rebuilds), for every byte k
    and every grid the option allows (G2 = 16, 32, 64)."""
    for G2, lg in ((16, 4), (32, 5), (64, 6)):
        for k in range(256):
            v = rn32(F(k, 255))
            cell_f = min(int(np.float32(v * f32(G2))), G2 - 1)  # v * 2^lg is exact in fp32
            assert (k >> (8 - lg)) == cell_f, (G2, k)


def test_fixed_point_sum_is_order_free_and_exact():
    """acc_add / acc_total (hq_device.h): each fp64 partial x in [0, 2^43)
    becomes v = RN(x 2^20), added as (v mod 2^32) to `lo` and (v >> 32) to `hi`;
    the total hi 2^12 + lo 2^-20 equals sum(v) 2^-20 exactly whatever the order
    (integer addition), and stays within 2^-21 per partial of the fp64 sum."""
    rng = np.random.default_rng(3)
    parts = np.concatenate([rng.uniform(0, 4e5, 5000), rng.uniform(0, 1e-3, 100), [0.0, 8.7e12]])
    v = [int(round(float(F(float(x)) * 2 ** 20))) for x in parts]

    def total(order):
        lo = hi = 0
        for i in order:
            lo += v[i] & 0xFFFFFFFF
            hi += v[i] >> 32
        return hi * 4096.0 + lo * (1.0 / 2 ** 20)

    t0 = total(range(len(v)))
    for seed in range(3):
        assert total(np.random.default_rng(seed).permutation(len(v))) == t0
    exact = F(sum(v), 2 ** 20)
    assert abs(F(t0) - exact) <= abs(exact) * F(1, 2 ** 52)  # one final rounding
    assert abs(exact - sum(F(float(x)) for x in parts)) <= len(parts) * F(1, 2 ** 21)
