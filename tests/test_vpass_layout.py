"""CPU check of the vertical stencil's (hi, lo) pair layout (hq_cost.hip
vblock_pair / build_vpass_f16_pair_fragments, cost16w above HB = 10).

For one column and one filter, the kernel computes output rows y = 8 h + o of a
16-row tile (halves h = 0, 1; o = 0..7) as MFMA K steps u = 0..S-1 over the
gathered region rows: lane group g, dword j of step u holds row 4 (4 u + j) + g
(+ 8 for half 1, the window w[4u+2 .. 4u+5]) as its (hi, lo) f16 pair of x * 2^14,
and both A slots of the pair hold one part of the tap t[R - o] * 2^16 (hi in the
first MFMA, lo in the second).  Restated in numpy: every (output row, tap) pair
must be covered exactly once, rows past the region only against zero taps, and
the split products must reproduce the float64 convolution to fp32 accuracy.
Mirrors the kernel's constants; no GPU needed.
"""

import numpy as np
import pytest

V_DATA = np.float32(2.0 ** 14)
V_TAP = np.float32(2.0 ** 16)


def split16(x):
    x = np.asarray(x, np.float32)
    hi = x.astype(np.float16)
    lo = (x - hi.astype(np.float32)).astype(np.float16)
    return hi, lo


def pair_steps(hb):
    return (8 + 2 * hb + 15) // 16


def vpass_pair(x, taps, hb):
    """Output rows 0..15 of one column by the pair layout (float64 accumulate of
    exact f16 x f16 products, as the MFMA's fp32 accumulator does to ~1 ulp)."""
    S, RH, T = pair_steps(hb), 16 + 2 * hb, 2 * hb + 1
    nj = 4 * S + 2
    # gathered rows: w[n] of lane group g = row 4 n + g (rows past the region are
    # clamped to the last one: they only ever meet zero taps)
    xs = x.astype(np.float32) * V_DATA
    out = np.zeros(16)
    hits = np.zeros((16, T), int)
    for h in range(2):
        for o in range(8):
            y = 8 * h + o
            acc = 0.0
            for u in range(S):
                for g in range(4):
                    for j in range(4):
                        n = 4 * u + j + 2 * h  # half 1 reads w[4u+2 ..]
                        assert n < nj
                        row = 4 * n + g
                        r_src = min(row, RH - 1) if 4 * n + 3 >= RH else row
                        x_hi, x_lo = split16(xs[r_src])
                        d = (4 * (4 * u + j) + g) - o  # the fragment's tap index (half 0 reference)
                        t = np.float32(taps[d]) * V_TAP if 0 <= d < T else np.float32(0.0)
                        t_hi, t_lo = split16(t)
                        if 0 <= d < T:
                            assert row == y + d  # half 1: the same d 8 rows further on
                            hits[y, d] += 1
                        else:
                            assert t == 0.0
                        for tp in (t_hi, t_lo):  # the two MFMAs
                            acc += float(tp) * float(x_hi) + float(tp) * float(x_lo)
            out[y] = acc / float(V_DATA) / float(V_TAP)
    return out, hits


@pytest.mark.parametrize("hb", [15, 19, 24])
def test_pair_layout_covers_every_tap_once(hb):
    rng = np.random.default_rng(hb)
    RH, T = 16 + 2 * hb, 2 * hb + 1
    x = rng.uniform(-0.3, 0.9, RH).astype(np.float32)
    taps = rng.normal(0.0, 1.0, T).astype(np.float32) / T
    got, hits = vpass_pair(x, taps, hb)
    assert (hits == 1).all()  # every output row meets every tap exactly once
    ref = np.array([sum(float(taps[d]) * float(x[y + d]) for d in range(T)) for y in range(16)])
    scale = np.abs(taps).sum() * np.abs(x).max()
    np.testing.assert_allclose(got, ref, rtol=0, atol=2e-6 * scale)


def test_pair_steps_and_gathers():
    # rows a lane gathers (4 S + 2) against the 32-row layout's 8 S' + 2
    assert [(hb, pair_steps(hb), 4 * pair_steps(hb) + 2) for hb in (15, 19, 24)] == \
        [(15, 3, 14), (19, 3, 14), (24, 4, 18)]
    for hb in (15, 19, 24):
        assert 16 * pair_steps(hb) >= 8 + 2 * hb  # a half's rows fit its K steps
