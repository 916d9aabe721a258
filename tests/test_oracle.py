"""CPU tests of the oracle: constants, golden fixtures, known answers, and the
agreement of the two independent restatements (numpy and C).

Parity status: the reference ships no vectors, so the fixtures
are oracle-generated (tests/golden/make_golden.py); the oracle itself is pinned
against the reference's own OpenCL kernels run on the MI355X (tests/test_refcl.py,
GPU) and, here, by the java.util.Random known answers.
"""

import json
import os

import numpy as np
import pytest

import c_oracle
import oracle as o

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_reference_constants_self_consistent():
    # RGB2Oppm (CL:171) is XYZ2Oppm (CL:110) . RGB2XYZm (CL:77) rounded to ~6 digits
    prod = o.XYZ2OPPM.astype(np.float64) @ o.RGB2XYZM.astype(np.float64)
    np.testing.assert_allclose(o.RGB2OPPM, prod, rtol=2e-5, atol=2e-6)
    # Opp2XYZm (CL:118) is the inverse of XYZ2Oppm to ~6 significant digits
    inv = np.linalg.inv(o.XYZ2OPPM.astype(np.float64))
    np.testing.assert_allclose(o.OPP2XYZM, inv, rtol=5e-5, atol=5e-5)
    # D65 of SP:20 (note Z = 1.0883, not 1.08883)
    assert o.D65.tolist() == [np.float32(0.95047), np.float32(1.0), np.float32(1.0883)]


def test_default_filter_design():
    f = o.design_filters()
    assert o.samp_per_deg(72, 45.0) == (242, 11)
    assert f.taps == 21 and f.half == 10  # IM:408 halfSize
    # k3 is negative (weight -0.117686) and absk3 = |k3|
    assert (f.k3 < 0).all() and np.array_equal(f.absk3, -f.k3)
    assert (f.k1[:, 3] == 0).all() and (f.k2[:, 3] == 0).all()


@pytest.mark.parametrize("dpi,vd,wp", [(72, 45.0, "D65"), (72, 45.0, "D50"), (96, 60.0, "D65"),
                                       (150, 30.0, "D65")])
def test_filters_golden(dpi, vd, wp):
    g = np.load(os.path.join(GOLD, "filters.npz"))
    f = o.design_filters(dpi, vd, wp)
    tag = f"{dpi}_{int(vd)}_{wp}"
    for name in ("k1", "k2", "k3", "absk3", "illum"):
        np.testing.assert_array_equal(getattr(f, name), g[f"{name}_{tag}"])


def test_java_random_known_answers():
    with open(os.path.join(GOLD, "kat_java_random.json")) as fh:
        kat = json.load(fh)
    assert o.JavaRandom(42).next(32) == kat["seed42_nextInt"]
    assert o.JavaRandom(0).next(32) == kat["seed0_nextInt"]
    assert o.JavaRandom(42).next_double() == kat["seed42_nextDouble"]
    r = o.JavaRandom(1234)
    assert [float(r.next_float()) for _ in range(8)] == kat["seed1234_nextFloat_x8"]


def test_reflect_index_matches_cl():
    idx = o.reflect_index(12, 10)
    assert idx[0, 0] == 9 and idx[0, 9] == 0 and idx[0, 10] == 0   # -10 -> 9, -1 -> 0
    assert idx[11, 20] == 2   # 21 -> 2*12-21-1
    with pytest.raises(ValueError):
        o.reflect_index(9, 10)


@pytest.mark.parametrize("name", ["case_64x48_k16", "case_97x53_k64"])
def test_golden_case_numpy_and_c(name):
    g = np.load(os.path.join(GOLD, f"{name}.npz"))
    w = int(g["w"])
    f = o.design_filters()
    img = g["rgb_u8"].astype(np.float32) / np.float32(255)
    R, G, B = img[:, 0].copy(), img[:, 1].copy(), img[:, 2].copy()
    rgba = o.inline_rgba(R, G, B)
    lab_c = c_oracle.srgb_to_scielab(R, G, B, f, w)
    np.testing.assert_allclose(lab_c, g["lab"], atol=2e-4)
    for p in range(g["palettes"].shape[0]):
        cc, parts = c_oracle.eval_palette(rgba, g["lab"], g["palettes"][p], f, w, return_parts=True)
        np.testing.assert_array_equal(parts["idx"], g["idx"][p])
        np.testing.assert_array_equal(parts["used"], g["used"][p])
        assert abs(cc - g["costs"][p]) <= 1e-6 * abs(g["costs"][p])


def test_golden_256_config1():
    g = np.load(os.path.join(GOLD, "case_256_k16.npz"))
    w = int(g["w"])
    f = o.design_filters()
    img = g["rgb_u8"].astype(np.float32) / np.float32(255)
    R, G, B = img[:, 0].copy(), img[:, 1].copy(), img[:, 2].copy()
    lab = c_oracle.srgb_to_scielab(R, G, B, f, w)
    np.testing.assert_allclose(np.abs(lab[:, :3].astype(np.float64)).sum(0), g["lab_checksum"],
                               rtol=1e-6)
    rgba = o.inline_rgba(R, G, B)
    for p in range(4):
        cc, parts = c_oracle.eval_palette(rgba, lab, g["palettes"][p], f, w, return_parts=True)
        if p == 0:
            np.testing.assert_array_equal(parts["idx"], g["idx0"])
        assert abs(cc - g["costs"][p]) <= 1e-5 * abs(g["costs"][p])


def test_edge_assign_golden():
    g = np.load(os.path.join(GOLD, "edge_assign.npz"))
    for name in ("dup", "clamped", "k1", "k256", "ties"):
        idx, _ = c_oracle.assign(g["px"], g[f"pal_{name}"])
        np.testing.assert_array_equal(idx, g[f"idx_{name}"])


def test_duplicates_lowest_index_wins():
    pal = np.zeros((4, 4), np.float32)
    pal[:, :3] = [[0.2, 0.2, 0.2], [0.7, 0.7, 0.7], [0.2, 0.2, 0.2], [0.7, 0.7, 0.7]]
    px = np.array([[0.21, 0.2, 0.2], [0.69, 0.7, 0.7]], np.float32)
    idx, used = o.assign(px, pal)
    assert idx.tolist() == [0, 1] and used.tolist() == [1, 1, 0, 0]


def test_perfect_palette_cost_is_small_not_zero():
    # LabRef and the candidate path use different matrices/orders
    w, h = 32, 24
    f = o.design_filters()
    rng = np.random.default_rng(0)
    cols = rng.integers(0, 256, (6, 3)).astype(np.float32) / np.float32(255)
    sel = rng.integers(0, 6, w * h)
    R, G, B = cols[sel, 0], cols[sel, 1], cols[sel, 2]
    lab = c_oracle.srgb_to_scielab(R, G, B, f, w)
    pal = np.zeros((6, 4), np.float32)
    pal[:, :3] = cols
    c = c_oracle.eval_palette(o.inline_rgba(R, G, B), lab, pal, f, w)
    assert 0 < c < 5e-3


def test_unused_penalty():
    w, h = 16, 16
    f = o.design_filters()
    R = np.full(w * h, 0.5, np.float32)
    lab = c_oracle.srgb_to_scielab(R, R, R, f, w)
    pal = o.synthetic_palette(8, 3)
    c, parts = c_oracle.eval_palette(o.inline_rgba(R, R, R), lab, pal, f, w, delta=2.0,
                                     return_parts=True)
    assert parts["used"].sum() == 1
    # constant image -> constant quantized image -> uniform dE
    e = parts["err"]
    assert np.ptp(e) < 1e-3 * max(e.max(), 1e-6) + 1e-5
    assert abs(c - (parts["err_sum"] / (w * h) + 2.0 * 7)) < 1e-9


def test_sum_array_tree_matches_sequential():
    a = np.random.default_rng(1).random(10001).astype(np.float32)
    s4 = o.sum_array(a, 4)
    assert abs(s4 - float(np.sum(a.astype(np.float64)))) < 1e-9
    assert o.default_depth(8) == 4 and o.default_depth(16) == 5


def test_swasa_trace_golden():
    g = np.load(os.path.join(GOLD, "swasa_trace.npz"))

    def cost(pal):
        pal = np.asarray(pal, np.float32)[..., :3].astype(np.float64)
        return float(np.sum((pal - 0.3) ** 2) + 0.01 * np.sum(np.sin(pal * 17)))

    sw = o.Swasa(o.SwasaParams(population=4, imax=int(g["imax"])), int(g["seed"]))
    tr = []
    best, err = o.find_best_quantization(lambda ps: [cost(p) for p in ps], int(g["K"]), sw, trace=tr)
    np.testing.assert_array_equal(np.array([[t[3]] + t[1] for t in tr]), g["trace"])
    np.testing.assert_array_equal(best, g["best"])


def test_ciede94_f32_statement():
    """oracle.ciede94_f32 (CL:217-226 in fp32, no clamp) against the float64
    form: within 1e-5 where finite (the cancellation in dH^2 costs a few fp32
    ulp of |dab|^2, divided by 2 dE); NaN exactly where rounding
    makes fma(da, da, db db) - dC dC negative -- a hue-aligned pair (here a
    colour and the same colour scaled towards grey, dH = 0 exactly) is NaN in
    the reference's arithmetic, and identical colours are 0."""
    rng = np.random.default_rng(1)
    n = 4000
    f32 = np.float32
    a, b = (rng.uniform(-60, 60, n).astype(f32) for _ in range(2))
    lab1 = np.stack([rng.uniform(0, 100, n).astype(f32), a, b, np.zeros(n, f32)], -1)
    lab2 = (lab1 + rng.normal(0, 3, lab1.shape)).astype(f32)
    e32, e64 = o.ciede94_f32(lab1, lab2), o.ciede94(lab1, lab2)
    ok = ~np.isnan(e32)
    assert ok.mean() > 0.999
    np.testing.assert_allclose(e32[ok], e64[ok], rtol=1e-6, atol=1e-5)
    # known NaN (fp32 dH^2 = -7.6e-6 for this pair; the float64 form gives 10.36)
    p1 = np.array([[50.0, 53.837933, -44.249878, 0.0]], f32)
    p2 = np.array([[40.0, 45.146347, -37.106186, 0.0]], f32)
    assert np.isnan(o.ciede94_f32(p1, p2)[0])
    assert abs(float(o.ciede94(p1, p2)[0]) - 10.363361) < 1e-4
    k = rng.uniform(0.3, 0.9, n)
    scaled = lab1.copy()
    scaled[:, 1:3] = (lab1[:, 1:3] * k[:, None]).astype(f32)
    assert 0.1 < np.isnan(o.ciede94_f32(lab1, scaled)).mean() < 0.9
    assert (o.ciede94_f32(lab1, lab1) == 0).all()


def test_fma32_is_one_rounding():
    """oracle.fma32 against exact rational arithmetic (Fraction), on random
    operands and on sums built to land near fp32 midpoints."""
    from fractions import Fraction

    rng = np.random.default_rng(5)
    a = rng.standard_normal(3000).astype(np.float32)
    b = rng.standard_normal(3000).astype(np.float32)
    c = rng.standard_normal(3000).astype(np.float32)
    # products whose exact sum sits on or next to a midpoint of the fp32 grid
    c[:1000] = (-(a[:1000].astype(np.float64) * b[:1000]).astype(np.float32)).astype(np.float32)
    c[1000:1500] = np.float32(1.0)
    a[1000:1500] = np.float32(2.0 ** -12) * (1 + rng.integers(0, 8, 500)).astype(np.float32)
    b[1000:1500] = np.float32(2.0 ** -12) + np.float32(2.0 ** -36) * rng.integers(-4, 5, 500).astype(np.float32)
    got = o.fma32(a, b, c)
    for x, y, z, r in zip(a.tolist(), b.tolist(), c.tolist(), got.tolist()):
        exact = Fraction(x) * Fraction(y) + Fraction(z)
        lo = np.float32(float(exact))  # nearest double, then fp32: check r is a nearest fp32
        cand = {float(lo), float(np.nextafter(lo, np.float32(np.inf))), float(np.nextafter(lo, np.float32(-np.inf)))}
        best = min(cand, key=lambda v: (abs(Fraction(v) - exact), np.float32(v).view(np.uint32) & 1))
        assert r == best, (x, y, z, r, best)


def test_ref_len_numpy_matches_c():
    """The two oracles' argmin distance (CL:179-192 as compiled for gfx950),
    correctly rounded sqrt mode: normal, tiny (rescaled x 2^86), subnormal,
    zero and huge (rescaled x 2^-66) differences."""
    rng = np.random.default_rng(8)
    n = 20000
    d = rng.standard_normal((n, 3)).astype(np.float32)
    d[:2000] *= np.float32(1e-21)
    d[2000:3000] *= np.float32(1e-40)
    d[3000:3100] = 0
    d[3100:3200] *= np.float32(3e19)
    d[3200:3300] = np.float32(1.4e-45)
    a = o.ref_len(d[:, 0], d[:, 1], d[:, 2])
    c = c_oracle.ref_len(d[:, 0], d[:, 1], d[:, 2])
    np.testing.assert_array_equal(a.view(np.uint32), c.view(np.uint32))
    # the rescaled forms are the distance to within a few ulp (normal results;
    # a subnormal result is on the subnormal grid)
    ex = np.sqrt(np.sum(d.astype(np.float64) ** 2, axis=1))
    ok = ex > 2.0 ** -126
    assert np.max(np.abs(a[ok] - ex[ok]) / ex[ok]) < 1e-6
    assert np.all(a[ex == 0] == 0) and np.all(np.abs(a[~ok] - ex[~ok]) <= 2.0 ** -149)
