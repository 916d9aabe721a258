"""GPU parity tests: libhq (HIP, gfx950) vs the CPU oracle, through the C ABI.

Bar: palette indices and used flags bit-exact; costs within 1e-4 relative
(the north-star tolerance; we assert tighter where the oracle is fast);
LabRef within 2e-4 absolute on Lab values in [-128, 100].
"""

import os

import numpy as np
import pytest

import c_oracle
import hybridquantization_amd as hq
import oracle as o

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
COST_RTOL = 1e-4  # north-star tolerance on the summed dE cost


@pytest.fixture(scope="module")
def filt():
    return o.design_filters()


@pytest.fixture()
def ip(gpu):
    m = hq.ImageManipulation(hq.deltaETypes.CIE76, device=gpu)
    assert m.getOpenCLAvailable()
    sp = hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    m.illum = sp.illuminant
    yield m
    m.close()


def load_case(name):
    g = np.load(os.path.join(GOLD, f"{name}.npz"))
    img = g["rgb_u8"].astype(np.float32) / np.float32(255)
    return g, img[:, 0].copy(), img[:, 1].copy(), img[:, 2].copy()


# ---------------------------------------------------------------------------
# LabRef / colour conversions (IM:100, IM:285)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["case_64x48_k16", "case_97x53_k64"])
def test_labref_on_device_matches_oracle(ip, name):
    g, R, G, B = load_case(name)
    w = int(g["w"])
    ip.setImage(o.inline_rgba(R, G, B).reshape(-1), None, w, ip.illum)
    lab = ip.getLabRef().reshape(-1, 4)
    np.testing.assert_allclose(lab, g["lab"], atol=2e-4)


def test_rgb_to_xyz_and_xyz_to_scielab(ip, filt):
    g, R, G, B = load_case("case_97x53_k64")
    w = int(g["w"])
    xyz = ip.RGBtoXYZ(R, G, B).reshape(-1, 4)
    np.testing.assert_allclose(xyz, o.rgb_to_xyz(R, G, B), rtol=1e-5, atol=1e-7)
    lab = ip.XYZtoScielab(xyz.reshape(-1), None, None, w, filt.illum).reshape(-1, 4)
    np.testing.assert_allclose(lab, g["lab"], atol=2e-4)


def test_labref_256_checksum(ip):
    g, R, G, B = load_case("case_256_k16")
    ip.setImage(o.inline_rgba(R, G, B).reshape(-1), None, 256, ip.illum)
    lab = ip.getLabRef().reshape(-1, 4)
    np.testing.assert_allclose(np.abs(lab[:, :3].astype(np.float64)).sum(0), g["lab_checksum"],
                               rtol=1e-6)
    np.testing.assert_allclose(lab[:512], g["lab_rows"], atol=2e-4)


# ---------------------------------------------------------------------------
# Candidate evaluation (IM:620-727): golden fixtures
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("grid", [64, 32, 16, 0])
@pytest.mark.parametrize("variant", [(0, 16, 256), (0, 16, 128), (0, 8, 128), (1, 16, 256)])
@pytest.mark.parametrize("name", ["case_64x48_k16", "case_97x53_k64"])
def test_eval_golden(ip, name, grid, variant):
    """(cost_variant, cost_rows, cost_tw): 0 = the fast tiled path (vertical
    passes on the matrix cores in split f16, horizontal pass on VALU) on 16 x 128
    tiles (cost16w_kernel, 4 waves, default), 16 x 256 (8 waves) or 8 x 108 tiles
    (cost_mfma_kernel), 1 = the generic two-pass path; argmin through candidate grids of 64^3, 32^3, 16^3
    cells or exhaustive."""
    g, R, G, B = load_case(name)
    w = int(g["w"])
    ip.setOption("grid", grid)
    ip.setOption("cost_variant", variant[0])
    ip.setOption("cost_rows", variant[1])
    ip.setOption("cost_tw", variant[2])
    ip.setImage(o.inline_rgba(R, G, B).reshape(-1), g["lab"].reshape(-1), w, ip.illum)
    pals = g["palettes"]
    costs, used = ip.computeQuantizationErrorPopulation(pals.reshape(len(pals), -1), 2.0,
                                                        return_used=True)
    np.testing.assert_allclose(costs, g["costs"], rtol=1e-6)
    np.testing.assert_array_equal(used, g["used"])
    for p in range(len(pals)):
        np.testing.assert_array_equal(ip.getIndices(p), g["idx"][p])


def test_eval_config1_256_k16(ip):
    g, R, G, B = load_case("case_256_k16")
    ip.setImage(o.inline_rgba(R, G, B).reshape(-1), None, 256, ip.illum)  # device LabRef
    costs, used = ip.computeQuantizationErrorPopulation(g["palettes"].reshape(4, -1), 2.0,
                                                        return_used=True)
    np.testing.assert_allclose(costs, g["costs"], rtol=1e-5)
    np.testing.assert_array_equal(used, g["used"])
    np.testing.assert_array_equal(ip.getIndices(0), g["idx0"])


def test_eval_config2_1024_k64(ip, filt):
    w = h = 1024
    R, G, B = o.synthetic_image(w, h, seed=1)
    rgba = o.inline_rgba(R, G, B)
    ip.setImage(rgba.reshape(-1), None, w, ip.illum)
    lab_dev = ip.getLabRef().reshape(-1, 4)
    lab = c_oracle.srgb_to_scielab(R, G, B, filt, w)
    np.testing.assert_allclose(lab_dev, lab, atol=2e-4)
    pal = o.synthetic_palette(64, 2)
    cost = ip.computeQuantizationErrorPopulation([pal.reshape(-1)], 2.0)[0]
    ref, parts = c_oracle.eval_palette(rgba, lab, pal, filt, w, nthreads=8, return_parts=True)
    np.testing.assert_array_equal(ip.getIndices(0), parts["idx"].astype(np.uint8))
    assert abs(cost - ref) <= COST_RTOL * abs(ref) * 0.1


def _compare_fast_generic(m, pals, de):
    """Costs and per-pixel dE of the fast path (cost_variant 0) and the generic
    fp32 two-pass path (1) for each palette.  dE76: no NaN, costs to 1e-6
    relative.  dE94: the reference's unclamped dH (CL:217-226) is NaN on the
    rare hue-aligned pixels where fp32 rounding makes dH^2 negative, and which
    pixels depends on the Lab's last bits: the finite pixels must agree, NaNs
    stay below 2e-3 of the pixels, a cost is NaN exactly when one of its pixels
    is, and finite costs agree to 1e-6 (NaN == NaN alone would pass vacuously)."""
    m.setOption("pixel_err", 1)
    for p in pals:
        cost, err = {}, {}
        for variant in (0, 1):
            m.setOption("cost_variant", variant)
            cost[variant] = m.computeQuantizationErrorPopulation([p.reshape(-1)], 2.0)[0]
            err[variant] = m.getPixelErrors(0)
        nan0, nan1 = np.isnan(err[0]), np.isnan(err[1])
        if de == hq.deltaETypes.CIE76:
            assert not nan0.any() and not nan1.any()
        assert nan0.mean() < 2e-3 and nan1.mean() < 2e-3
        ok = ~(nan0 | nan1)
        np.testing.assert_allclose(err[0][ok], err[1][ok], rtol=0, atol=2e-4)
        for v, nan in ((0, nan0), (1, nan1)):
            assert np.isnan(cost[v]) == bool(nan.any())
        if not (nan0.any() or nan1.any()):
            np.testing.assert_allclose(cost[0], cost[1], rtol=1e-6)
    m.setOption("pixel_err", 0)


@pytest.mark.parametrize("rows,tw", [(16, 256), (16, 128), (8, 128)])
@pytest.mark.parametrize("de", [hq.deltaETypes.CIE76, hq.deltaETypes.CIE94])
@pytest.mark.parametrize("trim", [1, 0])
def test_fast_path_matches_generic(gpu, de, trim, rows, tw):
    """The fast path (split-f16 vertical products, hi.hi + hi.lo + lo.hi with ~2^-22
    relative per product dropped; trimmed narrow filters) agrees with the generic
    fp32 two-pass path to 1e-6 relative (the bar is 1e-4) on interior, edge and
    partial tiles (800 columns: two interior 256-column tiles)."""
    w, h = (300, 77) if rows == 8 else (290, 93) if tw == 128 else (800, 93)
    R, G, B = o.synthetic_image(w, h, seed=5)
    m = hq.ImageManipulation(de, device=gpu)
    sp = hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    m.setImage(o.inline_rgba(R, G, B).reshape(-1), None, w, sp.illuminant)
    pals = [o.synthetic_palette(K, 7 + K) for K in (16, 64, 256)]
    m.setOption("trim", trim)
    m.setOption("cost_rows", rows)
    m.setOption("cost_tw", tw)
    _compare_fast_generic(m, pals, de)
    m.close()


@pytest.mark.parametrize("w,h,dpi,vd", [(300, 61, 300, 50.0), (1100, 60, 300, 50.0), (1029, 33, 72, 45.0),
                                         (97, 53, 150, 30.0)])
def test_generic_hrow4_bitwise(gpu, w, h, dpi, vd):
    """The LDS-tiled generic path's horizontal pass with 4 adjacent outputs per
    thread (option gen_hrow4, default) gives the one-output kernel's per-pixel
    dE and sums bit for bit: both sum each output's taps in ascending order.
    The double-buffered vertical pass (gen_vtile2) gives every pixel's dE bit
    for bit too; the matrix-core vertical pass (gen_vmfma, the default for
    half <= 64) agrees within the fast path's bars.
    Segments of 1,024 outputs: 1,100 and 1,029 columns end in partial
    segments; 300 dpi / 50 cm is 103 taps (half 51, not a multiple of 4)."""
    R, G, B = o.synthetic_image(w, h, seed=w * h)
    lib = hq.load()
    m = hq.ImageManipulation(device=gpu)
    sp = hq.ScielabProcessor(dpi, vd, hq.Whitepoint.D65, None, m)
    m.setImage(o.inline_rgba(R, G, B).reshape(-1), None, w, sp.illuminant)
    m.setOption("cost_variant", 1)
    m.setOption("pixel_err", 1)
    K, P = 64, 2
    pals = np.stack([o.synthetic_palette(K, 9 + p) for p in range(P)]).reshape(P, -1)
    res = []
    for h4, v2, vm, no, hm, shape in ((0, 0, 0, 4, 0, 0), (1, 0, 0, 4, 0, 0), (1, 1, 0, 4, 0, 0), (1, 1, 1, 4, 0, 0),
                                      (1, 1, 0, 8, 0, 0), (1, 1, 1, 4, 1, 1), (1, 1, 1, 4, 1, 2)):
        m.setOption("gen_tile_shape", shape)
        m.setOption("gen_hmfma", hm)
        m.setOption("gen_hrow4", h4)
        m.setOption("gen_vtile2", v2)
        m.setOption("gen_vmfma", vm)
        m.setOption("gen_hrow_outputs", no)
        out = np.zeros(P * (1 + K))
        hq._lib.check(lib.hq_eval_population_partial(m.ctx, hq._lib.fptr(np.ascontiguousarray(pals)), P, K,
                                                     out.ctypes.data_as(hq._lib._d)), m.ctx)
        res.append((out, [m.getPixelErrors(p) for p in range(P)]))
    m.close()
    np.testing.assert_array_equal(res[0][0], res[1][0])
    for p in range(P):
        np.testing.assert_array_equal(res[0][1][p], res[1][1][p])
        np.testing.assert_array_equal(res[2][1][p], res[1][1][p])  # gen_vtile2: every pixel bit for bit
        np.testing.assert_array_equal(res[4][1][p], res[2][1][p])  # 8 outputs per thread: the same sums
    # (gen_vtile2's 32 x 64 tiles round their fixed-point partials per tile: 2^-20 each)
    np.testing.assert_allclose(res[2][0], res[1][0], rtol=1e-9)
    assert (res[1][0].reshape(P, 1 + K)[:, 0] > 0).all()
    # gen_vmfma (default): the vertical taps as split-f16 matrix-core products,
    # the fast path's scheme -- the same bars as fast vs generic (per pixel 2e-4,
    # sums 1e-6 relative)
    for p in range(P):
        np.testing.assert_allclose(res[3][1][p], res[2][1][p], rtol=0, atol=2e-4)
    np.testing.assert_allclose(res[3][0].reshape(P, 1 + K)[:, 0], res[2][0].reshape(P, 1 + K)[:, 0], rtol=1e-6)
    np.testing.assert_array_equal(res[3][0].reshape(P, 1 + K)[:, 1:], res[2][0].reshape(P, 1 + K)[:, 1:])
    # gen_hmfma + gen_vmfma (the default): both passes on the matrix cores, in
    # the short (one 16-row tile per gen_hmfma workgroup, 64-row gen_vmfma tiles)
    # and the tall shapes (4 tiles, 128 rows: partial tiles at every size here)
    for r in (5, 6):
        for p in range(P):
            np.testing.assert_allclose(res[r][1][p], res[2][1][p], rtol=0, atol=2e-4)
        np.testing.assert_allclose(res[r][0].reshape(P, 1 + K)[:, 0], res[2][0].reshape(P, 1 + K)[:, 0], rtol=1e-6)
        np.testing.assert_array_equal(res[r][0].reshape(P, 1 + K)[:, 1:], res[2][0].reshape(P, 1 + K)[:, 1:])


@pytest.mark.parametrize("dpi,vd", [(150, 30.0), (96, 60.0), (200, 30.0)])
@pytest.mark.parametrize("de", [hq.deltaETypes.CIE76, hq.deltaETypes.CIE94])
def test_fast_path_matches_generic_wide_buckets(gpu, de, dpi, vd):
    """The tap buckets 15, 19 and 24 (the vertical pass's (hi, lo) pair layout,
    3 and 4 K steps) agree with the generic fp32 two-pass path to 1e-6 relative
    for both dE formulas, on interior, edge and partial tiles."""
    w, h = 290, 93
    R, G, B = o.synthetic_image(w, h, seed=dpi)
    m = hq.ImageManipulation(de, device=gpu)
    sp = hq.ScielabProcessor(dpi, vd, hq.Whitepoint.D65, None, m)
    m.setImage(o.inline_rgba(R, G, B).reshape(-1), None, w, sp.illuminant)
    pals = [o.synthetic_palette(K, 11 + K) for K in (16, 256)]
    _compare_fast_generic(m, pals, de)
    m.close()


# ---------------------------------------------------------------------------
# Viewing geometry (HQ:229-231 dpi / distance -> SP:80-102 tap count -> IM:408
# halfSize): the fast path runs the filters centred in a tap bucket of
# half-width 10, 15, 19 or 24; longer filters take the generic path.
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("dpi,vd,half", [(96, 60.0, 19), (150, 30.0, 15), (72, 30.0, 7),
                                         (100, 55.0, 18), (96, 70.0, 22), (200, 30.0, 20),
                                         (300, 50.0, 51)])
def test_viewing_geometry_vs_oracle(gpu, dpi, vd, half):
    """Non-default dpi / viewing distance on a 256 x 256 and a ragged 301 x 173
    image: device LabRef within 2e-4, every cost within 1e-5 relative of the
    oracle (the bar is 1e-4), indices and used flags bit-exact; the fast path
    (bucketed taps, trimmed or not) equals the generic fp32 two-pass path to
    1e-6 relative, and the LDS-tiled generic pair the per-pixel one."""
    f = o.design_filters(dpi, vd)
    assert f.half == half
    nt = _threads()
    for (w, h) in ((256, 256), (301, 173)):
        R, G, B = o.synthetic_image(w, h, seed=w + dpi)
        rgba = o.inline_rgba(R, G, B)
        m = hq.ImageManipulation(device=gpu)
        sp = hq.ScielabProcessor(dpi, vd, hq.Whitepoint.D65, None, m)
        m.setImage(rgba.reshape(-1), None, w, sp.illuminant)  # device LabRef
        lab_dev = m.getLabRef().reshape(-1, 4)
        lab = c_oracle.srgb_to_scielab(R, G, B, f, w, nthreads=nt)
        np.testing.assert_allclose(lab_dev, lab, atol=2e-4)
        pals = np.stack([o.synthetic_palette(64, 500 + p) for p in range(4)])
        costs, used = m.computeQuantizationErrorPopulation(pals.reshape(4, -1), 2.0, return_used=True)
        for p in range(4):
            ref, parts = c_oracle.eval_palette(rgba, lab_dev, pals[p], f, w, nthreads=nt,
                                               return_parts=True)
            assert abs(costs[p] - ref) <= 1e-5 * abs(ref), (w, p, costs[p], ref)
            np.testing.assert_array_equal(used[p], parts["used"])
            np.testing.assert_array_equal(m.getIndices(p), parts["idx"].astype(np.uint8))
        out = {}
        for variant, trim in ((1, 1), (2, 1), (0, 0), (0, 1)):
            m.setOption("cost_variant", variant)
            m.setOption("trim", trim)
            out[(variant, trim)] = m.computeQuantizationErrorPopulation(pals.reshape(4, -1), 2.0)
        np.testing.assert_array_equal(out[(0, 1)], costs)
        np.testing.assert_allclose(out[(0, 0)], out[(1, 1)], rtol=1e-6)
        np.testing.assert_allclose(out[(0, 1)], out[(1, 1)], rtol=1e-6)
        # the LDS-tiled generic pair against the per-pixel one (reference order)
        np.testing.assert_allclose(out[(1, 1)], out[(2, 1)], rtol=1e-6)
        m.close()


# ---------------------------------------------------------------------------
# argmin edge cases (CL:179-193), bit-exact
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("grid", [64, 32, 16, 0])
def test_assign_edge_cases(ip, grid):
    g = np.load(os.path.join(GOLD, "edge_assign.npz"))
    px = g["px"]  # 4096 pixels -> 64 x 64 image, values partly outside [0, 1]
    ip.setOption("grid", grid)
    ip.setImage(px.reshape(-1), np.zeros_like(px).reshape(-1), 64, ip.illum)
    for name in ("dup", "clamped", "k1", "k256", "ties"):
        pal = g[f"pal_{name}"]
        ip.computeQuantizationErrorPopulation([pal.reshape(-1)], 2.0)
        np.testing.assert_array_equal(ip.getIndices(0), g[f"idx_{name}"], err_msg=name)


@pytest.mark.parametrize("K", [1, 2, 7, 64, 255, 256])
def test_assign_random_and_near_ties(ip, K):
    rng = np.random.default_rng(K)
    w = h = 128
    px = np.zeros((w * h, 4), np.float32)
    px[:, :3] = (rng.integers(0, 256, (w * h, 3)) / 255.0).astype(np.float32)
    pal = o.synthetic_palette(K, 40 + K)
    if K > 4:
        # near-duplicates 1 ulp apart and exact duplicates: stress sqrt-collapse ties
        pal[K // 2, :3] = np.nextafter(pal[0, :3], np.float32(1))
        pal[K // 3, :3] = pal[1, :3]
        pal[K - 1, :3] = px[5, :3]
    ip.setImage(px.reshape(-1), np.zeros_like(px).reshape(-1), w, ip.illum)
    ref_idx, ref_used = c_oracle.assign(px, pal)
    for grid in (64, 32, 16, 0):
        ip.setOption("grid", grid)
        pals = [pal.reshape(-1), pal[::-1].copy().reshape(-1), pal.reshape(-1)]
        _, used = ip.computeQuantizationErrorPopulation(pals, 2.0, return_used=True)
        np.testing.assert_array_equal(ip.getIndices(0), ref_idx.astype(np.uint8))
        np.testing.assert_array_equal(ip.getIndices(2), ref_idx.astype(np.uint8))
        np.testing.assert_array_equal(used[0], ref_used)
        rev_idx, rev_used = c_oracle.assign(px, pal[::-1].copy())
        np.testing.assert_array_equal(ip.getIndices(1), rev_idx.astype(np.uint8))
        np.testing.assert_array_equal(used[1], rev_used)


@pytest.mark.parametrize("grid", [32, 64, 0])
def test_assign_sparse_special_pixels(ip, grid):
    """Lanes that need the reference loop (CL:179-192) -- pixels outside [0, 1],
    NaN or infinite channels, colours equal to a pixel or one ulp apart -- are
    re-resolved by their whole wave when they are few (argmin_coop: the loop
    split over 64 lanes and a (distance, index) butterfly, NaN distances never
    winning unless colour 0's is NaN), by each lane otherwise (a wave of
    specials).  Both must give the oracle's indices and used flags."""
    rng = np.random.default_rng(21)
    w, h = 256, 64
    px = np.zeros((w * h, 4), np.float32)
    px[:, :3] = (rng.integers(0, 256, (w * h, 3)) / 255.0).astype(np.float32)
    specials = [np.nan, np.inf, -np.inf, -0.5, 1.5, 2.0, -0.0]
    for j, i in enumerate(range(0, w * h, 97)):  # sparse: ~one per wave
        px[i, j % 3] = specials[j % len(specials)]
    px[640:704, 0] = np.nan  # a whole wave of NaN pixels: the per-lane path
    px[704:720, 1] = 3.0     # 16 outside pixels in one wave: the cooperative path's limit
    pal = o.synthetic_palette(256, 5)
    pal[7, :3] = px[3, :3]
    pal[8, :3] = np.nextafter(pal[7, :3], np.float32(2))
    pal[100, :3] = pal[9, :3]
    ip.setOption("grid", grid)
    ip.setImage(px.reshape(-1), np.zeros_like(px).reshape(-1), w, ip.illum)
    for p in (pal, pal[::-1].copy()):
        _, used = ip.computeQuantizationErrorPopulation([p.reshape(-1)], 2.0, return_used=True)
        ref_idx, ref_used = c_oracle.assign(px, p)
        np.testing.assert_array_equal(ip.getIndices(0), ref_idx.astype(np.uint8))
        np.testing.assert_array_equal(used[0], ref_used)


@pytest.mark.parametrize("grid", [64, 32, 0])
def test_assign_signed_zero_and_mass_duplicates(ip, grid):
    """Duplicate flags (prep_palette's hash of first occurrences): +0/-0 channels
    compare equal, long runs of one colour, and a palette of only a few distinct
    colours (every slot chain collides) must still give the oracle's indices."""
    rng = np.random.default_rng(11)
    w = h = 64
    px = np.zeros((w * h, 4), np.float32)
    px[:, :3] = (rng.integers(0, 256, (w * h, 3)) / 255.0).astype(np.float32)
    px[:64, :3] = 0.0
    few = o.synthetic_palette(4, 9)
    pal_few = few[rng.integers(0, 4, 256)].copy()
    pal_zero = o.synthetic_palette(64, 12)
    pal_zero[5, :3] = (0.0, 0.25, 0.0)
    pal_zero[9, :3] = (-0.0, 0.25, -0.0)
    pal_zero[2, :3] = (-0.0, -0.0, -0.0)
    pal_zero[40, :3] = (0.0, 0.0, 0.0)
    pal_run = o.synthetic_palette(200, 13)
    pal_run[50:150] = pal_run[60]
    ip.setOption("grid", grid)
    ip.setImage(px.reshape(-1), np.zeros_like(px).reshape(-1), w, ip.illum)
    pals = [pal_few, pal_zero, pal_run]
    for pal in pals:
        ip.computeQuantizationErrorPopulation([pal.reshape(-1)], 2.0)
        ref_idx, _ = c_oracle.assign(px, pal)
        np.testing.assert_array_equal(ip.getIndices(0), ref_idx.astype(np.uint8))


@pytest.mark.parametrize("grid", [64, 32, 16])
def test_assign_clustered_palettes_long_lists(ip, grid):
    """Palettes of a few tight colour clusters: many cells list more colours than
    an 8-B level-2 entry holds, so build_grid's pairwise pass (prune_long_lists)
    and the overflow re-resolution (argmin_fix, cooperative and per-lane) both
    run; indices and used flags equal the oracle's argmin.  P = 4 (one group)."""
    rng = np.random.default_rng(31 + grid)
    w, h, K, P = 256, 192, 256, 4
    px = np.zeros((w * h, 4), np.float32)
    px[:, :3] = (rng.integers(0, 256, (w * h, 3)) / 255.0).astype(np.float32)
    pals = []
    for p in range(P):
        centres = rng.random((2 + 2 * p, 3), dtype=np.float32)
        pal = np.zeros((K, 4), np.float32)
        pal[:, :3] = np.clip(centres[rng.integers(0, len(centres), K)] +
                             rng.normal(0, 0.02 * (p + 1), (K, 3)), 0, 1)
        pals.append(pal)
    pals = np.stack(pals)
    ip.setOption("grid", grid)
    ip.setImage(px.reshape(-1), np.zeros_like(px).reshape(-1), w, ip.illum)
    _, used = ip.computeQuantizationErrorPopulation(pals.reshape(P, -1), 2.0, return_used=True)
    for p in range(P):
        ref_idx, ref_used = c_oracle.assign(px, pals[p])
        np.testing.assert_array_equal(ip.getIndices(p), ref_idx.astype(np.uint8), err_msg=f"palette {p}")
        np.testing.assert_array_equal(used[p], ref_used, err_msg=f"palette {p}")


@pytest.mark.parametrize("P", [1, 2, 3, 5, 6, 8])
def test_assign_group_sizes(ip, P):
    """Groups of 1-4 palettes per pixel pass (P = 5: a full group and a group of
    one).  P = 1, 2, 3 run assign_pipe_kernel<NG = P>, P >= 4 its NG = 4 instance."""
    rng = np.random.default_rng(P)
    w, h, K = 75, 41, 96
    px = np.zeros((w * h, 4), np.float32)
    px[:, :3] = (rng.integers(0, 256, (w * h, 3)) / 255.0).astype(np.float32)
    pals = np.stack([o.synthetic_palette(K, 300 + p) for p in range(P)])
    ip.setImage(px.reshape(-1), np.zeros_like(px).reshape(-1), w, ip.illum)
    _, used = ip.computeQuantizationErrorPopulation(pals.reshape(P, -1), 2.0, return_used=True)
    for p in range(P):
        ref_idx, ref_used = c_oracle.assign(px, pals[p])
        np.testing.assert_array_equal(ip.getIndices(p), ref_idx.astype(np.uint8))
        np.testing.assert_array_equal(used[p], ref_used)


@pytest.mark.parametrize("grid", [64, 32, 16])
def test_grid_margin_adversarial(ip, grid):
    """build_grid's fp32 box bounds and its 1e-5 candidate margin (hq_search.hip)
    on the inputs that sit exactly on the decision boundaries: pixels on cell
    faces i/G2 (and on 0.0 / 1.0) and one ulp either side, palette colours on
    faces and corners, colour pairs mirrored across a face (exactly equidistant
    from the pixels on the face: the lower index must win, CL:186), and colour
    pairs one ulp apart.  Pruned argmin == exhaustive == the oracle, bit for bit,
    indices and used flags (CL:179-193)."""
    rng = np.random.default_rng(2024 + grid)
    w, h = 128, 96
    n = w * h
    faces = (np.arange(grid + 1) / grid).astype(np.float32)  # exact: G2 is a power of two
    vals = np.concatenate([faces, np.nextafter(faces[:-1], np.float32(2)),
                           np.nextafter(faces[1:], np.float32(-1))])
    px = np.zeros((n, 4), np.float32)
    px[:, :3] = rng.choice(vals, size=(n, 3))
    px[:64, :3] = 1.0
    px[64:128, :3] = 0.0
    K = 256
    pals = np.zeros((4, K, 4), np.float32)
    pals[0, :, :3] = rng.choice(faces, size=(K, 3))  # faces and corners
    # mirrored pairs across a face f on one axis; pixels placed on the face
    for i in range(K // 2):
        ax = i % 3
        f = faces[rng.integers(1, grid)]
        d = np.float32(rng.integers(1, 8)) / np.float32(4 * grid)
        base = rng.choice(faces, 3)
        a, b = base.copy(), base.copy()
        a[ax], b[ax] = f - d, f + d
        pals[1, 2 * i, :3], pals[1, 2 * i + 1, :3] = np.clip(a, 0, 1), np.clip(b, 0, 1)
        on = base.copy()
        on[ax] = f
        px[128 + i, :3] = on
    # pairs one ulp apart, on faces and at random points
    c = np.where(rng.random((K // 2, 3)) < 0.5, rng.choice(faces, (K // 2, 3)),
                 rng.random((K // 2, 3), dtype=np.float32)).astype(np.float32)
    pals[2, 0::2, :3] = c
    pals[2, 1::2, :3] = np.nextafter(c, np.float32(2))
    # u8-grid colours with face values mixed in and exact duplicates
    pals[3, :, :3] = (rng.integers(0, 256, (K, 3)) / 255.0).astype(np.float32)
    pals[3, ::7, 0] = rng.choice(faces, len(pals[3, ::7]))
    pals[3, 200:210] = pals[3, 3]
    ip.setImage(px.reshape(-1), np.zeros_like(px).reshape(-1), w, ip.illum)
    refs = [c_oracle.assign(px, pals[p]) for p in range(4)]
    for g in (grid, 0):
        ip.setOption("grid", g)
        _, used = ip.computeQuantizationErrorPopulation(pals.reshape(4, -1), 2.0, return_used=True)
        for p in range(4):
            np.testing.assert_array_equal(ip.getIndices(p), refs[p][0].astype(np.uint8),
                                          err_msg=f"grid {g} palette {p}")
            np.testing.assert_array_equal(used[p], refs[p][1], err_msg=f"grid {g} palette {p}")


def test_out_of_range_palette_takes_generic_path(ip, filt):
    """A palette colour beyond the fast path's split-f16 range (G = 2.5: its
    opponent value x 2^14 overflows f16) is routed to the generic fp32 path
    (palette_fits_fast, hq_runtime.hip): a finite cost equal to the oracle's,
    indices bit-exact.  The SA itself only produces colours in [0, 1]."""
    g, R, G, B = load_case("case_97x53_k64")
    w = int(g["w"])
    rgba = o.inline_rgba(R, G, B)
    ip.setImage(rgba.reshape(-1), g["lab"].reshape(-1), w, ip.illum)
    pal = g["palettes"][0].copy()
    pal[3, 1] = 2.5
    pal[5, 2] = -40.0
    pals = np.stack([pal, g["palettes"][1]])
    costs = ip.computeQuantizationErrorPopulation(pals.reshape(2, -1), 2.0)
    for p in range(2):
        ref, parts = c_oracle.eval_palette(rgba, g["lab"], pals[p], filt, w, return_parts=True)
        assert np.isfinite(costs[p]) and abs(costs[p] - ref) <= 1e-6 * abs(ref), (p, costs[p], ref)
        np.testing.assert_array_equal(ip.getIndices(p), parts["idx"].astype(np.uint8))


def test_out_of_range_palette_every_pixel(ip, filt):
    """Every colour of the palette beyond the split-f16 range (G + 2.2), so
    every pixel's filtered error is out of the matrix-core range: the generic
    path keeps both passes in fp32 (gn.vmfma off for such populations,
    hq_runtime.hip) and the cost equals the oracle's."""
    g, R, G, B = load_case("case_97x53_k64")
    w = int(g["w"])
    rgba = o.inline_rgba(R, G, B)
    ip.setImage(rgba.reshape(-1), g["lab"].reshape(-1), w, ip.illum)
    pal = g["palettes"][0].copy()
    pal[:, 1] += 2.2
    pal[:, 0] -= 0.5
    pals = np.stack([pal, g["palettes"][1]])
    costs = ip.computeQuantizationErrorPopulation(pals.reshape(2, -1), 2.0)
    for p in range(2):
        ref, parts = c_oracle.eval_palette(rgba, g["lab"], pals[p], filt, w, return_parts=True)
        assert np.isfinite(costs[p]) and abs(costs[p] - ref) <= 1e-6 * abs(ref), (p, costs[p], ref)
        np.testing.assert_array_equal(ip.getIndices(p), parts["idx"].astype(np.uint8))


@pytest.mark.parametrize("K,P", [(257, 2), (300, 3), (600, 2), (1024, 2), (1500, 1), (4096, 2)])
def test_wide_palette_vs_oracle(gpu, filt, K, P):
    """K > 256 (the plugin allows up to 2^24, HybridQuantization.java:192).  The
    palettes run as 256-colour chunks (16-bit indices) and the tiled cost
    kernel: K = 257 and 300 (2 chunks, P odd leaves a group of two
    sub-palettes) through a grid and assign pass per chunk, chunk winners
    combined by the reference distance; K = 600 to 4096 (4 to 16 chunks)
    through the native 16-bit candidate lists (lists16_kernel +
    assign16_kernel, one grid over all K colours; level 2 transposed above
    K = 2048).  K > 4096: test_large_palettes_vs_oracle.  Indices and used flags bit-exact
    against the oracle's argmin (CL:172-193), costs within 1e-5 relative (the
    bar is 1e-4), on a 256 x 256 image with duplicate colours (also across
    chunks), colours one ulp apart and colours equal to pixels (exact ties)."""
    w = h = 256
    R, G, B = o.synthetic_image(w, h, seed=K)
    rgba = o.inline_rgba(R, G, B)
    m = hq.ImageManipulation(device=gpu)
    hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    m.setImage(rgba.reshape(-1), None, w, filt.illum)
    lab = m.getLabRef().reshape(-1, 4)
    pals = np.stack([o.synthetic_palette(K, 900 + p) for p in range(P)])
    pals[0, K // 2, :3] = np.nextafter(pals[0, 3, :3], np.float32(1))
    pals[0, K - 1] = pals[0, 7]
    pals[-1, 100:110, :3] = rgba[1000:1010, :3]
    pals[-1, K - 5:, :3] = rgba[1000:1005, :3]  # same colours again at higher indices
    costs, used = m.computeQuantizationErrorPopulation(pals.reshape(P, -1), 2.0, return_used=True)
    nt = _threads()
    for p in range(P):
        ref, parts = c_oracle.eval_palette(rgba, lab, pals[p], filt, w, nthreads=nt, return_parts=True)
        assert abs(costs[p] - ref) <= 1e-5 * abs(ref), (p, costs[p], ref)
        np.testing.assert_array_equal(used[p], parts["used"])
        np.testing.assert_array_equal(m.getIndices32(p), parts["idx"].astype(np.uint32))
    with pytest.raises(hq.HQError):
        m.getIndices(0)  # u8 indices only exist for K <= 256
    lib = hq.load()  # kernel timing on: the wide path records no grid events, and must not fail
    lib.hq_profile_enable(m.ctx, 1)
    c2 = m.computeQuantizationErrorPopulation(pals.reshape(P, -1), 2.0)
    c3 = m.computeQuantizationErrorPopulation(pals.reshape(P, -1), 2.0)
    lib.hq_profile_enable(m.ctx, 0)
    np.testing.assert_array_equal(c2, costs)
    np.testing.assert_array_equal(c3, costs)
    m.close()


@pytest.mark.parametrize("K", [512, 1024, 2048, 4096, 3000, 8192, 5000, 16384, 10000])
def test_chunked_palettes_match_exhaustive(gpu, filt, K):
    """The chunked K > 256 path (grid per 256-colour chunk, winners combined by
    the reference distance, hq_assign.hip) against the exhaustive one (option
    chunked 0, hq_wide.hip) on a 512 x 384 image: indices bit for bit, used
    flags equal, costs within 1e-6 relative -- with the ties a chunk boundary
    can split: colours of chunk 0 repeated at the same position of every other
    chunk, a colour one ulp from one in another chunk, pixels equal to palette
    colours, and near-black / near-white colours."""
    w, h = 512, 384
    R, G, B = o.synthetic_image(w, h, seed=K + 7)
    rgba = o.inline_rgba(R, G, B)
    pal = o.synthetic_palette(K, 4242).copy()
    for c in range(1, K // 256):
        pal[256 * c + 5] = pal[5]                     # exact duplicates across chunks
        pal[256 * c + 9, :3] = np.nextafter(pal[9, :3], np.float32(2))
    pal[K - 20:K - 10, :3] = rgba[5000:5010, :3]      # pixel colours in the last chunk
    pal[30:40, :3] = rgba[5000:5010, :3]              # ... and in chunk 0 (ties: chunk 0 wins)
    pal[K - 3, :3] = 0.0
    pal[K - 2, :3] = 1.0
    pals = np.stack([pal, o.synthetic_palette(K, 77)])
    m = hq.ImageManipulation(device=gpu)
    hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    m.setImage(rgba.reshape(-1), None, w, filt.illum)
    res = {}
    for chunked in (1, 0):
        m.setOption("chunked", chunked)
        costs, used = m.computeQuantizationErrorPopulation(pals.reshape(2, -1), 2.0, return_used=True)
        res[chunked] = (costs, used, [m.getIndices32(p) for p in range(2)])
    for p in range(2):
        np.testing.assert_array_equal(res[1][2][p], res[0][2][p])
        np.testing.assert_array_equal(res[1][1][p], res[0][1][p])
    np.testing.assert_allclose(res[1][0], res[0][0], rtol=1e-6)
    m.close()


@pytest.mark.parametrize("K,img_u8,mode", [(2048, 1, 1), (4096, 0, 1), (1500, 1, 1), (600, 1, 2), (300, 0, 2),
                                            (8192, 1, 1), (6000, 0, 1)])
def test_lists16_match_chunked_and_exhaustive(gpu, filt, K, img_u8, mode):
    """The native 16-bit candidate lists (option lists16, default from 4 to 32
    chunks: one grid over all K colours, hq_lists16.hip) against the per-chunk
    grids (lists16 0) and the exhaustive path (chunked 0): indices bit for bit,
    used flags equal, costs within 1e-6.  Palette 0 is clustered -- every
    colour in a box of side 0.08 around a grey that many pixels sit in, so
    level-2 entries and level-1 lists overflow into their fallbacks (the
    pixel's level-1 list, all K colours) -- palette 1 uniform, palette 2 the
    uniform one with duplicates across chunks, palette 3 the uniform one
    stretched to [-0.3, 1.3] (colours outside the unit cube: the level-2
    lower bound's clamp); planar float pixels (img_u8 0) and packed bytes.
    Mode 2 takes 2 chunks too."""
    w, h = 320, 200
    R, G, B = o.synthetic_image(w, h, seed=K)
    R[: h // 2] = np.clip(0.45 + 0.06 * (R[: h // 2] - 0.5), 0, 1)  # half the image near the cluster
    G[: h // 2] = np.clip(0.5 + 0.06 * (G[: h // 2] - 0.5), 0, 1)
    B[: h // 2] = np.clip(0.55 + 0.06 * (B[: h // 2] - 0.5), 0, 1)
    R, G, B = (np.round(x * 255) / 255 for x in (R, G, B))
    rgba = o.inline_rgba(R, G, B)
    rng = np.random.default_rng(K)
    clus = o.synthetic_palette(K, 5).copy()
    clus[:, :3] = (np.array([0.45, 0.5, 0.55]) + 0.08 * (rng.random((K, 3)) - 0.5)).astype(np.float32)
    uni = o.synthetic_palette(K, 6)
    dup = uni.copy()
    for c in range(1, K // 256):
        dup[256 * c + 3] = dup[3]
    far = uni.copy()
    far[:, :3] = (1.6 * far[:, :3] - 0.3).astype(np.float32)
    pals = np.stack([clus, uni, dup, far])
    m = hq.ImageManipulation(device=gpu)
    hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    m.setImage(rgba.reshape(-1), None, w, filt.illum)
    m.setOption("img_u8", img_u8)
    res = {}
    for name, opts in (("n16", {"lists16": mode, "chunked": 1}), ("chunk", {"lists16": 0, "chunked": 1}),
                       ("exh", {"lists16": 1, "chunked": 0})):
        for k, v in opts.items():
            m.setOption(k, v)
        costs, used = m.computeQuantizationErrorPopulation(pals.reshape(len(pals), -1), 2.0, return_used=True)
        res[name] = (costs, used, [m.getIndices32(p) for p in range(len(pals))])
    m.close()
    for other in ("chunk", "exh"):
        for p in range(len(pals)):
            np.testing.assert_array_equal(res["n16"][2][p], res[other][2][p])
            np.testing.assert_array_equal(res["n16"][1][p], res[other][1][p])
        np.testing.assert_allclose(res["n16"][0], res[other][0], rtol=1e-6)


@pytest.mark.parametrize("K,opts", [
    (5000, {}),                     # native 16-bit lists (level 2 transposed above 2048), cost16w NCH = 32
    (8192, {}),                     # ... at the lists' largest K
    (10000, {}),                    # per-chunk grids (64 chunks) + the generic cost pair
    (16384, {}),                    # ... at the chunked path's largest K
    (20000, {}),                    # K > 16384: prep_wide + assign_wide, 32-bit indices
    (5000, {"chunked": 0}),         # the exhaustive assign_wide path at a chunkable K
    (3000, {"chunked": 0, "grid": 0}),
])
def test_large_palettes_vs_oracle(gpu, filt, K, opts):
    """Every K > 4096 path against the oracle's argmin (CL:172-193) and cost, not
    only against another HIP path (VERDICT r5 Missing 2): indices bit for bit,
    used flags equal, costs within 1e-5 relative, on a 320 x 200 image whose
    upper half sits in a small cluster of colours.  Palettes: clustered around
    that cluster (level-2 / level-1 lists overflow), uniform with exact
    duplicates across chunks and one-ulp neighbours in other chunks, pixel
    colours at a low and a high index (exact ties: the lower index wins), and
    the uniform palette stretched to [-0.3, 1.3] (colours outside the unit
    cube).  K up to 2^24 is allowed by the plugin (HybridQuantization.java:192)."""
    w, h = 320, 200
    R, G, B = o.synthetic_image(w, h, seed=K + 3)
    R[: h // 2] = np.clip(0.45 + 0.06 * (R[: h // 2] - 0.5), 0, 1)
    G[: h // 2] = np.clip(0.5 + 0.06 * (G[: h // 2] - 0.5), 0, 1)
    B[: h // 2] = np.clip(0.55 + 0.06 * (B[: h // 2] - 0.5), 0, 1)
    R, G, B = ((np.round(x * 255) / 255).astype(np.float32) for x in (R, G, B))
    rgba = o.inline_rgba(R, G, B)
    rng = np.random.default_rng(K)
    clus = o.synthetic_palette(K, 15).copy()
    clus[:, :3] = (np.array([0.45, 0.5, 0.55]) + 0.08 * (rng.random((K, 3)) - 0.5)).astype(np.float32)
    uni = o.synthetic_palette(K, 16).copy()
    for c in range(1, K // 256):
        uni[256 * c + 3] = uni[3]                                      # duplicates across chunks
        uni[256 * c + 11, :3] = np.nextafter(uni[11, :3], np.float32(2))  # one ulp from chunk 0's
    uni[40:50, :3] = rgba[40000:40010, :3]                             # pixel colours, low index ...
    uni[K - 12:K - 2, :3] = rgba[40000:40010, :3]                      # ... and again at a high one
    far = o.synthetic_palette(K, 17).copy()
    far[:, :3] = (1.6 * far[:, :3] - 0.3).astype(np.float32)
    pals = np.stack([clus, uni, far])
    P = len(pals)
    m = hq.ImageManipulation(device=gpu)
    hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    m.setImage(rgba.reshape(-1), None, w, filt.illum)
    for k, v in opts.items():
        m.setOption(k, v)
    lab = m.getLabRef().reshape(-1, 4)
    costs, used = m.computeQuantizationErrorPopulation(pals.reshape(P, -1), 2.0, return_used=True)
    idx = [m.getIndices32(p) for p in range(P)]
    m.close()
    nt = _threads()
    for p in range(P):
        ref, parts = c_oracle.eval_palette(rgba, lab, pals[p], filt, w, nthreads=nt, return_parts=True)
        np.testing.assert_array_equal(idx[p], parts["idx"].astype(np.uint32), err_msg=f"palette {p}")
        np.testing.assert_array_equal(used[p], parts["used"], err_msg=f"palette {p}")
        assert abs(costs[p] - ref) <= 1e-5 * abs(ref), (p, costs[p], ref)


def test_wide_palette_search_runs_host_driven(ip, filt):
    """A SWASA search with K > 256 runs the host-driven loop (the device-resident
    step keeps palettes in LDS, K <= 256) on the wide evaluation path and follows
    the same native driver fed with oracle costs."""
    w, h, K = 40, 32, 300
    R, G, B = o.synthetic_image(w, h, seed=21)
    rgba = o.inline_rgba(R, G, B)
    lab = c_oracle.srgb_to_scielab(R, G, B, filt, w)
    ip.setImage(rgba.reshape(-1), lab.reshape(-1), w, filt.illum)
    sw = hq.SWASA(population=2, imax=6, seed=31, t0=0.5)
    best = ip.findBestQuantization(rgba.reshape(-1), lab.reshape(-1), w, K, sw, None, None, filt.illum)
    gpu_err = ip.bestError

    def ev(ps):
        return [c_oracle.eval_palette(rgba, lab, p, filt, w) for p in ps]

    hbest, herr, _ = hq.SWASA(population=2, imax=6, seed=31, t0=0.5).search_host(K, ev)
    assert abs(gpu_err - herr) <= 1e-5 * abs(herr)
    np.testing.assert_array_equal(best, hbest)


@pytest.mark.parametrize("P", [1, 4, 6])
def test_used_flags_from_sparse_pixels(gpu, filt, P):
    """Used flags are OR'ed into 8 words per palette by every assign workgroup
    (device-scope atomics, hq_assign.hip): a colour used by a single pixel in
    one corner of a 2048 x 2048 image -- one workgroup on one XCD -- must still
    be flagged, and one used nowhere must not (CL:193).  Mostly-grey image with
    200 isolated pixels of their own colours spread over the image."""
    w = h = 2048
    rng = np.random.default_rng(17 + P)
    R = np.full(w * h, 0.5, np.float32)
    G = R.copy()
    B = R.copy()
    K = 256
    pals = np.zeros((P, K, 4), np.float32)
    where = rng.choice(w * h, 200, replace=False)
    cols = (rng.integers(0, 256, (200, 3)) / 255.0).astype(np.float32)
    R[where], G[where], B[where] = cols[:, 0], cols[:, 1], cols[:, 2]
    for p in range(P):
        pals[p, :, :3] = (rng.integers(0, 256, (K, 3)) / 255.0).astype(np.float32)
        pals[p, 0, :3] = 0.5  # the grey
        sel = rng.choice(200, 100, replace=False)
        pals[p, 1 + np.arange(100), :3] = cols[sel]
    m = _planar_ctx(gpu, R, G, B, w, h, filt.illum)
    _, used = m.computeQuantizationErrorPopulation(pals.reshape(P, -1), 2.0, return_used=True)
    m.close()
    rgba = o.inline_rgba(R, G, B)
    for p in range(P):
        _, ref_used = c_oracle.assign(rgba, pals[p], nthreads=_threads())
        np.testing.assert_array_equal(used[p], ref_used, err_msg=f"palette {p}")
        assert 50 < ref_used.sum() < 200


@pytest.mark.parametrize("K", [16, 600])
def test_nonfinite_palette_falls_back_exactly(ip, K):
    """Non-finite colours: the reference loop verbatim (K <= 256), or the
    exhaustive K > 256 path instead of the chunked one (a NaN colour 0 of a
    later chunk would stop that chunk's own loop, CL:186, not the reference's)."""
    w = h = 32
    px = np.zeros((w * h, 4), np.float32)
    px[:, :3] = np.random.default_rng(3).random((w * h, 3), dtype=np.float32)
    pal = o.synthetic_palette(K, 5)
    pal[3, 1] = np.nan
    pal[7, 0] = np.inf
    if K > 256:
        pal[256, 2] = np.nan  # colour 0 of chunk 1
    ip.setImage(px.reshape(-1), np.zeros_like(px).reshape(-1), w, ip.illum)
    ip.computeQuantizationErrorPopulation([pal.reshape(-1)], 2.0)
    ref_idx, _ = c_oracle.assign(px, pal)
    np.testing.assert_array_equal(ip.getIndices32(0), ref_idx.astype(np.uint32))


# ---------------------------------------------------------------------------
# Row-block sharding: shards' partials add up to the full image
# ---------------------------------------------------------------------------
def test_row_block_shards_sum_to_full(gpu, filt):
    w, h, K, P = 96, 90, 32, 3
    R, G, B = o.synthetic_image(w, h, seed=4)
    rgba = o.inline_rgba(R, G, B).reshape(-1)
    pals = np.stack([o.synthetic_palette(K, 60 + p) for p in range(P)]).reshape(P, -1)
    full = hq.ImageManipulation(device=gpu)
    hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, full)
    full.setImage(rgba, None, w, filt.illum)
    lib = hq.load()
    ref = np.zeros(P * (1 + K))
    hq._lib.check(lib.hq_eval_population_partial(full.ctx, hq._lib.fptr(pals), P, K,
                                                 hq._lib.dptr(ref)), full.ctx)
    for nshards in (2, 3, 7):
        bounds = np.linspace(0, h, nshards + 1).astype(int)
        acc = np.zeros(P * (1 + K))
        for r0, r1 in zip(bounds[:-1], bounds[1:]):
            sh = hq.ImageManipulation(device=gpu)
            hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, sh)
            sh.setImage(rgba, None, w, filt.illum, row_begin=r0, row_end=r1)
            part = np.zeros(P * (1 + K))
            hq._lib.check(lib.hq_eval_population_partial(sh.ctx, hq._lib.fptr(pals), P, K,
                                                         hq._lib.dptr(part)), sh.ctx)
            acc += part
            sh.close()
        acc = acc.reshape(P, 1 + K)
        refp = ref.reshape(P, 1 + K)
        np.testing.assert_allclose(acc[:, 0], refp[:, 0], rtol=1e-6)
        np.testing.assert_array_equal(acc[:, 1:] > 0, refp[:, 1:] > 0)
    full.close()


def test_rccl_single_rank_allreduce(gpu, filt):
    """The multi-GPU path on one GPU: libhq's own RCCL communicator (unique id,
    ncclCommInitRank, the fp64 all-reduce on the context stream) with one rank
    leaves the costs and used flags unchanged."""
    w, h, K, P = 80, 64, 48, 4
    R, G, B = o.synthetic_image(w, h, seed=6)
    rgba = o.inline_rgba(R, G, B).reshape(-1)
    pals = np.stack([o.synthetic_palette(K, 80 + p) for p in range(P)]).reshape(P, -1)
    m = hq.ImageManipulation(device=gpu)
    hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    m.setImage(rgba, None, w, filt.illum, row_begin=0, row_end=h)
    c0, u0 = m.computeQuantizationErrorPopulation(pals, 2.0, return_used=True)
    m.initComm(1, 0, hq.ImageManipulation.commUniqueId())
    c1, u1 = m.computeQuantizationErrorPopulation(pals, 2.0, return_used=True)
    np.testing.assert_array_equal(c1, c0)
    np.testing.assert_array_equal(u1, u0)
    m.close()


# ---------------------------------------------------------------------------
# Final quantize (IM:770) and error image (IM:858)
# ---------------------------------------------------------------------------
def test_quantize_matches_oracle(ip):
    g, R, G, B = load_case("case_97x53_k64")
    rgba = o.inline_rgba(R, G, B)
    pal = g["palettes"][0]
    q = ip.quantize(rgba.reshape(-1), pal.reshape(-1)).reshape(-1, 4)
    ref, idx, used = o.quantize(rgba[:, :3], pal)
    np.testing.assert_array_equal(q, ref)
    np.testing.assert_array_equal(ip.lastUsedColors, used)


@pytest.mark.parametrize("de", [hq.deltaETypes.CIE76, hq.deltaETypes.CIE94])
def test_compute_error_matches_oracle(gpu, de):
    g, R, G, B = load_case("case_97x53_k64")
    m = hq.ImageManipulation(de, device=gpu)
    rng = np.random.default_rng(0)
    other = (g["lab"] + rng.normal(0, 2, g["lab"].shape)).astype(np.float32)
    other[:, 3] = 0
    img = np.zeros(g["lab"].size, np.float32)
    mean = m.computeError(g["lab"].reshape(-1), other.reshape(-1), img)
    e = o.ciede76(g["lab"], other) if de == hq.deltaETypes.CIE76 else o.ciede94(g["lab"], other)
    assert abs(mean - float(np.mean(e.astype(np.float64)))) < 1e-5 * float(np.mean(e))
    np.testing.assert_allclose(img.reshape(-1, 4)[:, 0],
                               ((255 - e) * (255 - e) / (255 * 255)).astype(np.float32), rtol=1e-5)
    m.close()


# ---------------------------------------------------------------------------
# SA search on the GPU (IM:383-591) vs the same native driver on oracle costs
# ---------------------------------------------------------------------------
def test_search_matches_host_driver_on_oracle_costs(ip, filt):
    w, h, K = 48, 40, 8
    R, G, B = o.synthetic_image(w, h, seed=8)
    rgba = o.inline_rgba(R, G, B)
    lab = c_oracle.srgb_to_scielab(R, G, B, filt, w)
    ip.setImage(rgba.reshape(-1), lab.reshape(-1), w, filt.illum)
    sw = hq.SWASA(population=3, imax=40, seed=77, t0=0.5)
    best = ip.findBestQuantization(rgba.reshape(-1), lab.reshape(-1), w, K, sw, None, None,
                                   filt.illum)
    gpu_err = ip.bestError

    def ev(ps):
        return [c_oracle.eval_palette(rgba, lab, p, filt, w) for p in ps]

    hbest, herr, _ = hq.SWASA(population=3, imax=40, seed=77, t0=0.5).search_host(K, ev)
    # identical decisions unless an acceptance test lands within fp32 noise
    assert abs(gpu_err - herr) <= 1e-5 * abs(herr)
    np.testing.assert_array_equal(best, hbest)


@pytest.mark.parametrize("P,K", [(1, 16), (3, 16), (4, 16), (2, 600), (3, 1500), (4, 5000), (2, 8192),
                                 (64, 256), (8, 16384), (32, 3000), (64, 600)])
def test_device_search_matches_host_driven(gpu, filt, P, K):
    """The device-resident SWASA loop (sa_step_kernel: acceptance, convergence,
    java.util.Random draws by jump table, neighbour generation) follows the
    host-driven driver's trajectory exactly on the same GPU costs, across
    resumed run() calls and up to imax.  K = 600 and 1500: chunked palettes
    (one workgroup per chunk keeps, draws and preps its colours; the padding
    of the last chunks is candidate colour 0, drawn again).  The extremes of
    the device-resident limits (kSaMaxP = 64 palettes, kSaMaxSub = 512
    sub-palettes): P = 8 at K = 16384 (64 chunks: per-chunk grids and the
    generic cost pair), P = 32 at K = 3000 and P = 64 at K = 600 (the
    accept step's used-bit fold at 4 words per thread, 8 P nch > 1024)."""
    import ctypes as C
    w, h = 96, 64
    R, G, B = o.synthetic_image(w, h, seed=9)
    m = hq.ImageManipulation(device=gpu)
    hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    m.setImage(o.inline_rgba(R, G, B).reshape(-1), None, w, filt.illum)
    lib = hq.load()
    res = {}
    for dev in (0, 1):  # host-driven; device-resident
        m.setOption("sa_device", dev)
        sw = hq.SWASA(population=P, imax=50, seed=5 + P, t0=0.05)
        params = sw.params()
        handle = C.c_void_p()
        hq._lib.check(lib.hq_search_create(m.ctx, C.byref(params), K, sw.seed, C.byref(handle)), m.ctx)
        ran = C.c_int()
        total = 0
        for chunk in (17, 1, 40):  # the last call stops at imax
            hq._lib.check(lib.hq_search_run(handle, chunk, C.byref(ran)), m.ctx)
            total += ran.value
        best = np.zeros(4 * K, np.float32)
        err = C.c_double()
        it = C.c_int()
        hq._lib.check(lib.hq_search_best(handle, hq._lib.fptr(best), C.byref(err), C.byref(it)), m.ctx)
        lib.hq_search_destroy(handle)
        res[dev] = (best, err.value, it.value, total)
    assert res[1][2] == res[0][2] == res[1][3] == res[0][3] == 50
    assert res[1][1] == res[0][1]
    np.testing.assert_array_equal(res[1][0], res[0][0])
    m.close()


@pytest.mark.parametrize("P", [1, 4])
def test_device_search_de94_nan_costs(gpu, filt, P):
    """dE94 costs of a realistic image are NaN (the reference's unclamped dH,
    CL:222; see test_pixel_errors_de94_vs_oracle).  The reference's loop then
    runs on IEEE comparisons: argmin (IM:843-855) keeps member 0, isAccepted
    (SW:54-57) rejects a NaN difference after drawing its random number, a NaN
    never beats the best (IM:529) and the convergence copy takes member 0 with
    minerror = Double.MAX_VALUE (IM:518-545).  The device-resident loop and the
    host-driven driver must follow that trajectory identically; while no
    candidate has a finite cost, the best palette stays the initial member 0's
    (its error NaN).  (A rare candidate with no NaN pixel is finite and then
    becomes the best, as in the reference.)"""
    import ctypes as C
    w, h, K = 256, 128, 16
    R, G, B = o.synthetic_image(w, h, seed=19)
    m = hq.ImageManipulation(hq.deltaETypes.CIE94, device=gpu)
    hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    m.setImage(o.inline_rgba(R, G, B).reshape(-1), None, w, filt.illum)
    lib = hq.load()
    res = {}
    for dev in (0, 1):  # host-driven; device-resident
        m.setOption("sa_device", dev)
        sw = hq.SWASA(population=P, imax=30, seed=40 + P, t0=0.05)
        params = sw.params()
        handle = C.c_void_p()
        hq._lib.check(lib.hq_search_create(m.ctx, C.byref(params), K, sw.seed, C.byref(handle)), m.ctx)
        best = np.zeros((2, 4 * K), np.float32)
        err = C.c_double()
        it = C.c_int()
        ran = C.c_int()
        for j, chunk in enumerate((1, 29)):
            hq._lib.check(lib.hq_search_run(handle, chunk, C.byref(ran)), m.ctx)
            hq._lib.check(lib.hq_search_best(handle, hq._lib.fptr(best[j]), C.byref(err), C.byref(it)), m.ctx)
        lib.hq_search_destroy(handle)
        res[dev] = (best, err.value, it.value)
    print(f"P={P}: best error host {res[0][1]!r} device {res[1][1]!r}")
    assert res[0][2] == res[1][2] == 30
    assert res[0][1] == res[1][1] or (np.isnan(res[0][1]) and np.isnan(res[1][1]))
    np.testing.assert_array_equal(res[1][0], res[0][0])
    if np.isnan(res[0][1]):  # no finite cost in the run: member 0's initial palette stays the best
        np.testing.assert_array_equal(res[0][0][0], res[0][0][1])
    m.close()


@pytest.mark.parametrize("split", [0, 1])
def test_device_search_with_single_rank_comm(gpu, filt, split):
    """The multi-GPU search loop on one GPU: with libhq's RCCL communicator
    split 0 (row blocks) all-gathers every rank's fixed-point counter and
    used-bit blocks between the cost kernel and sa_step (no finalize), split 1
    (option palette_split) all-gathers finalized rows after finalize; with
    one rank the trajectory must be the one without a communicator.  The last
    10 iterations run profiled: the collective is event-timed once per
    iteration ("comm", bench.py's N > 1 line), and only with a communicator."""
    import ctypes as C
    w, h, K, P = 80, 72, 24, 4
    R, G, B = o.synthetic_image(w, h, seed=12)
    lib = hq.load()
    res = []
    for comm in (False, True):
        m = hq.ImageManipulation(device=gpu)
        hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
        m.setImage(o.inline_rgba(R, G, B).reshape(-1), None, w, filt.illum)
        m.setOption("palette_split", split)
        if comm:
            m.initComm(1, 0, hq.ImageManipulation.commUniqueId())
        sw = hq.SWASA(population=P, imax=40, seed=21, t0=0.05)
        params = sw.params()
        handle = C.c_void_p()
        hq._lib.check(lib.hq_search_create(m.ctx, C.byref(params), K, sw.seed, C.byref(handle)), m.ctx)
        ran = C.c_int()
        hq._lib.check(lib.hq_search_run(handle, 30, C.byref(ran)), m.ctx)
        assert ran.value == 30
        lib.hq_profile_reset(m.ctx)
        lib.hq_profile_enable(m.ctx, 1)
        hq._lib.check(lib.hq_search_run(handle, 10, C.byref(ran)), m.ctx)
        lib.hq_profile_enable(m.ctx, 0)
        for stage, want in (("comm", 10 if comm else 0), ("cost", 10), ("sa_step", 10)):
            ms, n = C.c_double(), C.c_int64()
            hq._lib.check(lib.hq_profile_get(m.ctx, stage.encode(), C.byref(ms), C.byref(n)), m.ctx)
            assert n.value == want and (ms.value > 0) == (want > 0), (stage, comm, n.value, ms.value)
        best = np.zeros(4 * K, np.float32)
        err = C.c_double()
        it = C.c_int()
        hq._lib.check(lib.hq_search_best(handle, hq._lib.fptr(best), C.byref(err), C.byref(it)), m.ctx)
        lib.hq_search_destroy(handle)
        m.close()
        res.append((best, err.value, it.value))
    assert res[0][2] == res[1][2] == 40
    assert res[0][1] == res[1][1]
    np.testing.assert_array_equal(res[0][0], res[1][0])


@pytest.mark.parametrize("K,P", [(24, 4), (600, 3)])
def test_device_search_folds_rank_blocks(gpu, filt, K, P):
    """The row-block layout of the counters (one block of fixed-point sums and
    used bits per rank, each rank filling its own, the accept step summing and
    OR'ing all of them after the all-gather) on one context: test options
    fold_blocks / fold_block put this context's block at position r of R and
    leave the others zero, as an all-gather of ranks that own no pixels would.
    The device-resident trajectory must be the one of the plain layout at any
    (R, r), and a host-driven evaluation (finalize of its own block) too."""
    import ctypes as C
    w, h = 80, 72
    R, G, B = o.synthetic_image(w, h, seed=13)
    lib = hq.load()
    pals = np.stack([o.synthetic_palette(K, 30 + p) for p in range(P)]).reshape(P, -1)
    res = []
    for nb, b in ((1, 0), (2, 1), (3, 0), (8, 5), (8, 7)):
        m = hq.ImageManipulation(device=gpu)
        hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
        m.setImage(o.inline_rgba(R, G, B).reshape(-1), None, w, filt.illum)
        m.setOption("fold_blocks", nb)
        m.setOption("fold_block", b)
        costs = m.computeQuantizationErrorPopulation(pals, 2.0)
        sw = hq.SWASA(population=P, imax=25, seed=23, t0=0.05)
        params = sw.params()
        handle = C.c_void_p()
        hq._lib.check(lib.hq_search_create(m.ctx, C.byref(params), K, sw.seed, C.byref(handle)), m.ctx)
        ran = C.c_int()
        hq._lib.check(lib.hq_search_run(handle, 25, C.byref(ran)), m.ctx)
        best = np.zeros(4 * K, np.float32)
        err = C.c_double()
        it = C.c_int()
        hq._lib.check(lib.hq_search_best(handle, hq._lib.fptr(best), C.byref(err), C.byref(it)), m.ctx)
        lib.hq_search_destroy(handle)
        m.close()
        res.append((costs, best, err.value, it.value))
    for r in res[1:]:
        np.testing.assert_array_equal(r[0], res[0][0])
        assert r[2] == res[0][2] and r[3] == res[0][3] == 25
        np.testing.assert_array_equal(r[1], res[0][1])


@pytest.mark.parametrize("K,P,ranks,opts", [(64, 8, 2, {}), (64, 8, 4, {}), (256, 12, 3, {}), (600, 4, 2, {}),
                                             (5000, 4, 2, {}), (600, 4, 2, {"chunked": 0}),
                                             (300, 6, 3, {"grid": 0}), (2048, 4, 2, {}), (600, 4, 2, {"lists16": 2})])
def test_palette_slices_sum_to_full(gpu, filt, K, P, ranks, opts):
    """The palette split (option palette_split with a communicator):
    rank r evaluates palettes [r P/N, (r+1) P/N) of the whole image.  Here the
    ranks are contexts on one GPU with the test-only slice options: each slice's
    rows of hq_eval_population_partial equal the full evaluation's bit for bit
    (sums and used flags; the other rows read 0), and so do the indices of the
    slice's palettes; K = 600 runs chunked palettes.  K = 5000, chunked 0 and
    grid 0 run the wide (exhaustive K > 256) path, which must take the same
    slice (a rank that evaluated every palette would count each N times)."""
    w, h = 160, 120
    R, G, B = o.synthetic_image(w, h, seed=K + P)
    rgba = o.inline_rgba(R, G, B).reshape(-1)
    pals = np.stack([o.synthetic_palette(K, 40 + p) for p in range(P)]).reshape(P, -1)
    lib = hq.load()

    def run(slice_rank):
        m = hq.ImageManipulation(device=gpu)
        hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
        m.setImage(rgba, None, w, filt.illum)
        for k, v in opts.items():
            m.setOption(k, v)
        if slice_rank is not None:
            m.setOption("slice_ranks", ranks)
            m.setOption("slice_rank", slice_rank)
        out = np.zeros(P * (1 + K))
        hq._lib.check(lib.hq_eval_population_partial(m.ctx, hq._lib.fptr(np.ascontiguousarray(pals)), P, K,
                                                     out.ctypes.data_as(hq._lib._d)), m.ctx)
        idx = {}
        n = P // ranks
        lo = 0 if slice_rank is None else slice_rank * n
        for p in range(P):
            if slice_rank is None or lo <= p < lo + n:
                idx[p] = m.getIndices32(p)
            else:
                with pytest.raises(hq.HQError):
                    m.getIndices32(p)
        m.close()
        return out.reshape(P, 1 + K), idx

    full, idx_full = run(None)
    n = P // ranks
    for r in range(ranks):
        part, idx = run(r)
        rows = slice(r * n, (r + 1) * n)
        np.testing.assert_array_equal(part[rows], full[rows])
        others = np.ones(P, bool)
        others[rows] = False
        assert not part[others].any()
        for p, v in idx.items():
            np.testing.assert_array_equal(v, idx_full[p])


def test_palette_slice_rank_out_of_range(gpu, filt):
    """slice_rank must lie in [0, slice_ranks): a rank past the last slice is
    refused with HQ_ERR_ARG before anything is enqueued (it would address
    palette rows past the population)."""
    w, h, K, P = 64, 48, 16, 4
    R, G, B = o.synthetic_image(w, h, seed=5)
    rgba = o.inline_rgba(R, G, B).reshape(-1)
    pals = np.stack([o.synthetic_palette(K, 2 + p) for p in range(P)]).reshape(P, -1)
    m = hq.ImageManipulation(device=gpu)
    hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    m.setImage(rgba, None, w, filt.illum)
    with pytest.raises(hq.HQError):
        m.setOption("slice_rank", -1)
    lib = hq.load()
    out = np.zeros(P * (1 + K))

    def partial():
        return lib.hq_eval_population_partial(m.ctx, hq._lib.fptr(np.ascontiguousarray(pals)), P, K,
                                              out.ctypes.data_as(hq._lib._d))

    m.setOption("slice_ranks", 2)
    m.setOption("slice_rank", 2)
    assert partial() == hq._lib.HQ_ERR_ARG and "outside" in lib.hq_last_error(m.ctx).decode()
    m.setOption("slice_rank", 1)
    assert partial() == 0
    rows = out.reshape(P, 1 + K)
    assert not rows[:2].any() and (rows[2:, 0] > 0).all()  # rows 0, 1: the other slice
    m.close()


# ---------------------------------------------------------------------------
# Full-size properties (4096^2, K = 256): determinism, grid == exhaustive,
# fast == generic, shards == full.
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("w,h,P", [(1003, 517, 4), (1003, 517, 3), (37, 29, 5)])
def test_assign_workgroup_count_invariance(gpu, filt, w, h, P):
    """The assign grid (option assign_blocks_per_cu: 1 to 64 workgroups per CU)
    only changes which workgroup takes which pixels.  The reference run uses
    the default, 0 = auto (one resident round from the occupancy query, at
    least HQ_ASSIGN_MINPX pixels per thread); indices, used flags and costs at
    every listed count must equal it bit for bit, also when an image has
    fewer pixel chunks than workgroups (37 x 29)."""
    K = 256
    R, G, B = o.synthetic_image(w, h, seed=11)
    m = _planar_ctx(gpu, R, G, B, w, h, filt.illum)
    pals = np.stack([o.synthetic_palette(K, 40 + p) for p in range(P)]).reshape(P, -1)
    ref_c, ref_used = m.computeQuantizationErrorPopulation(pals, 2.0, return_used=True)
    ref_idx = [m.getIndices(p) for p in range(P)]
    for nb in (1, 5, 64, 16):
        m.setOption("assign_blocks_per_cu", nb)
        c, used = m.computeQuantizationErrorPopulation(pals, 2.0, return_used=True)
        np.testing.assert_array_equal(c, ref_c, err_msg=f"blocks {nb}")
        np.testing.assert_array_equal(used, ref_used, err_msg=f"blocks {nb}")
        for p in range(P):
            np.testing.assert_array_equal(m.getIndices(p), ref_idx[p], err_msg=f"blocks {nb} palette {p}")
    m.close()


@pytest.mark.parametrize("off_lattice", [False, True])
def test_packed_image_path(gpu, filt, off_lattice):
    """An image whose channels are all k/255 (the reference's int-RGB source)
    is also kept as packed bytes, and assign reads those (4 B per pixel instead
    of 12, k/255 rebuilt by u8_unit); option img_u8 = 0 forces the planar floats.
    Both give the same indices, used flags and costs, and the indices are the
    exhaustive oracle argmin.  An image with one value off the k/255 lattice is
    kept planar only (both settings then take the same path).  P = 5 runs a
    group of 4 and a group of 1 (two assign launches)."""
    w, h, K, P = 301, 203, 256, 5
    R, G, B = o.synthetic_image(w, h, seed=31)
    if off_lattice:
        R = R.copy()
        R[7] = np.float32(0.5)
        G[1000] = np.nextafter(G[1000], np.float32(2))
    m = _planar_ctx(gpu, R, G, B, w, h, filt.illum)
    pals = np.stack([o.synthetic_palette(K, 60 + p) for p in range(P)])
    pals[4, 17, :3] = [R[9], G[9], B[9]]  # a colour on a pixel
    c1, used1 = m.computeQuantizationErrorPopulation(pals.reshape(P, -1), 2.0, return_used=True)
    idx1 = [m.getIndices(p) for p in range(P)]
    m.setOption("img_u8", 0)
    c0, used0 = m.computeQuantizationErrorPopulation(pals.reshape(P, -1), 2.0, return_used=True)
    np.testing.assert_array_equal(c0, c1)
    np.testing.assert_array_equal(used0, used1)
    px = np.stack([R, G, B, np.zeros_like(R)], 1)
    for p in range(P):
        np.testing.assert_array_equal(m.getIndices(p), idx1[p])
        ref_idx, ref_used = c_oracle.assign(px, pals[p])
        np.testing.assert_array_equal(idx1[p], ref_idx.astype(np.uint8), err_msg=f"palette {p}")
        np.testing.assert_array_equal(used1[p], ref_used)
    m.close()


def test_full_size_properties(gpu, filt):
    w = h = 4096
    K = 256
    R, G, B = o.synthetic_image(w, h, seed=1)
    m = hq.ImageManipulation(device=gpu)
    hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    lib = hq.load()
    hq._lib.check(lib.hq_set_image_planar_shard(m.ctx, hq._lib.fptr(R), hq._lib.fptr(G),
                                                hq._lib.fptr(B), w, h, hq._lib.fptr(filt.illum),
                                                0, h), m.ctx)
    m.w, m.h = w, h
    pals = np.stack([o.synthetic_palette(K, 2 + p) for p in range(2)]).reshape(2, -1)
    c1 = m.computeQuantizationErrorPopulation(pals, 2.0)
    idx1 = m.getIndices(1)
    c2 = m.computeQuantizationErrorPopulation(pals, 2.0)
    np.testing.assert_array_equal(c1, c2)  # deterministic reduction
    m.setOption("grid", 0)
    c3 = m.computeQuantizationErrorPopulation(pals, 2.0)
    np.testing.assert_array_equal(m.getIndices(1), idx1)  # pruned == exhaustive argmin
    np.testing.assert_array_equal(c3, c1)

    m.setOption("grid", 64)
    m.setOption("cost_rows", 8)
    c8 = m.computeQuantizationErrorPopulation(pals, 2.0)
    np.testing.assert_allclose(c8, c1, rtol=1e-6)  # 8-row tiles == 16-row tiles
    m.setOption("cost_rows", 16)
    m.setOption("cost_tw", 256)
    c256 = m.computeQuantizationErrorPopulation(pals, 2.0)
    np.testing.assert_allclose(c256, c1, rtol=1e-6)  # 256-column tiles == 128-column tiles
    m.setOption("cost_tw", 128)
    m.setOption("cost_rows", 16)
    m.setOption("cost_variant", 1)
    c4 = m.computeQuantizationErrorPopulation(pals, 2.0)
    np.testing.assert_allclose(c4, c1, rtol=1e-6)  # generic two-pass == fast path
    m.setOption("cost_variant", 0)
    m.setOption("trim", 0)  # all 21 taps of the narrow filters
    c5 = m.computeQuantizationErrorPopulation(pals, 2.0)
    np.testing.assert_allclose(c5, c1, rtol=1e-7)
    assert np.all(np.isfinite(c1)) and np.all(c1 > 0)
    m.close()


@pytest.mark.parametrize("rows,tw", [(16, 256), (16, 128), (8, 128)])
def test_alternating_populations_bitwise(gpu, filt, rows, tw):
    """Two different populations evaluated alternately give, every time,
    bitwise the costs and used flags of their first evaluation (no state of one
    evaluation -- partials, used masks, level-2 lines -- leaks into the next),
    and agree with the generic two-pass path."""
    w = h = 4096
    K, P = 256, 4
    R, G, B = o.synthetic_image(w, h, seed=3)
    m = _planar_ctx(gpu, R, G, B, w, h, filt.illum)
    m.setOption("cost_rows", rows)
    m.setOption("cost_tw", tw)
    pops = [np.stack([o.synthetic_palette(K, 40 + 10 * s + p) for p in range(P)]).reshape(P, -1)
            for s in range(2)]
    first = [m.computeQuantizationErrorPopulation(pp, 2.0, return_used=True) for pp in pops]
    for it in range(6):
        c, u = m.computeQuantizationErrorPopulation(pops[it & 1], 2.0, return_used=True)
        np.testing.assert_array_equal(c, first[it & 1][0])
        np.testing.assert_array_equal(u, first[it & 1][1])
    assert not np.array_equal(first[0][0], first[1][0])
    m.setOption("cost_variant", 1)
    for s in range(2):
        c, u = m.computeQuantizationErrorPopulation(pops[s], 2.0, return_used=True)
        np.testing.assert_allclose(c, first[s][0], rtol=1e-6)
        np.testing.assert_array_equal(u, first[s][1])
    m.close()


# ---------------------------------------------------------------------------
# BASELINE.json configs at their full sizes against the oracle (C3, C4, C5).
# The C oracle runs one 4096^2/K=256 evaluation in about 1 s on 16 threads.
# ---------------------------------------------------------------------------
def _threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def _planar_ctx(gpu, R, G, B, w, h, illum, r0=0, r1=None):
    m = hq.ImageManipulation(device=gpu)
    hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    r1 = h if r1 is None else r1
    lib = hq.load()
    hq._lib.check(lib.hq_set_image_planar_shard(m.ctx, hq._lib.fptr(R), hq._lib.fptr(G),
                                                hq._lib.fptr(B), w, h, hq._lib.fptr(illum),
                                                r0, r1), m.ctx)
    m.w, m.h = w, r1 - r0
    return m


def test_config3_4096_k256_p4_vs_oracle(gpu, filt):
    """C3 (4096x4096, K = 256, P = 4 per launch, the bench's population): the
    device LabRef equals the oracle's to 2e-4; every palette's cost is within
    1e-4 relative of the oracle's end to end (oracle LabRef on the oracle side,
    device LabRef on the device side); every palette's indices and used flags
    bit-exact."""
    w = h = 4096
    K, P = 256, 4
    R, G, B = o.synthetic_image(w, h, seed=1)
    m = _planar_ctx(gpu, R, G, B, w, h, filt.illum)
    pals = np.stack([o.synthetic_palette(K, 2 + p) for p in range(P)])
    costs, used = m.computeQuantizationErrorPopulation(pals.reshape(P, -1), 2.0, return_used=True)
    idx = {p: m.getIndices(p) for p in range(P)}
    lab_dev = m.getLabRef().reshape(-1, 4)
    m.close()
    nt = _threads()
    lab = c_oracle.srgb_to_scielab(R, G, B, filt, w, nthreads=nt)
    np.testing.assert_allclose(lab_dev, lab, atol=2e-4)
    del lab_dev
    rgba = o.inline_rgba(R, G, B)
    for p in range(P):
        ref, parts = c_oracle.eval_palette(rgba, lab, pals[p], filt, w, nthreads=nt,
                                           return_parts=True)
        assert abs(costs[p] - ref) <= COST_RTOL * abs(ref), (p, costs[p], ref)
        np.testing.assert_array_equal(used[p], parts["used"])
        if p in idx:
            np.testing.assert_array_equal(idx[p], parts["idx"].astype(np.uint8))


def test_config5_p64_one_launch(gpu, filt):
    """C5 (4096x4096, K = 256, P = 64 palettes in one launch): every cost and
    used flag is bit-identical to 64 separate single-palette evaluations (same
    per-tile partials, same fixed-order sum); all 64 palettes' used flags and 8
    palettes' indices equal the oracle's argmin, and palettes 0, 31 and 63's
    costs match the oracle (device LabRef as the oracle's input: LabRef parity
    at this size is test_config3's)."""
    w = h = 4096
    K, P = 256, 64
    R, G, B = o.synthetic_image(w, h, seed=1)
    m = _planar_ctx(gpu, R, G, B, w, h, filt.illum)
    pals = np.stack([o.synthetic_palette(K, 100 + p) for p in range(P)])
    costs, used = m.computeQuantizationErrorPopulation(pals.reshape(P, -1), 2.0, return_used=True)
    checked = (0, 9, 18, 27, 36, 45, 54, 63)
    idx = {p: m.getIndices(p) for p in checked}
    assert np.all(np.isfinite(costs))
    for p in range(P):
        c1, u1 = m.computeQuantizationErrorPopulation(pals[p].reshape(1, -1), 2.0, return_used=True)
        assert c1[0] == costs[p], p
        np.testing.assert_array_equal(u1[0], used[p])
    lab = m.getLabRef().reshape(-1, 4)
    m.close()
    rgba = o.inline_rgba(R, G, B)
    nt = _threads()
    for p in range(P):  # every palette's used flags against the oracle's argmin
        ref_idx, ref_used = c_oracle.assign(rgba, pals[p], nthreads=nt)
        np.testing.assert_array_equal(used[p], ref_used, err_msg=f"palette {p}")
        if p in idx:
            np.testing.assert_array_equal(idx[p], ref_idx.astype(np.uint8), err_msg=f"palette {p}")
    for p in (0, 31, 63):
        ref, parts = c_oracle.eval_palette(rgba, lab, pals[p], filt, w, nthreads=nt,
                                           return_parts=True)
        assert abs(costs[p] - ref) <= COST_RTOL * abs(ref), (p, costs[p], ref)


def test_config4_8192_shards_sum_to_full(gpu, filt):
    """C4 (8192x8192, K = 256, row-block shards of 8 GPUs): the partials of the
    eight 1024-row shards (each with its +-10 halo rows, evaluated in its own
    context) sum to the full-image evaluation (fp64 sums to 1e-9 relative, used
    flags exact), the device LabRef equals the oracle's at 8192^2 (2e-4), and the
    full image matches the oracle on one palette (cost, used flags, indices)."""
    w = h = 8192
    K, P, N = 256, 4, 8
    R, G, B = o.synthetic_image(w, h, seed=1)
    pals = np.stack([o.synthetic_palette(K, 2 + p) for p in range(P)]).reshape(P, -1)
    lib = hq.load()
    full = _planar_ctx(gpu, R, G, B, w, h, filt.illum)
    ref = np.zeros(P * (1 + K))
    hq._lib.check(lib.hq_eval_population_partial(full.ctx, hq._lib.fptr(pals), P, K,
                                                 hq._lib.dptr(ref)), full.ctx)
    idx0 = full.getIndices(0)
    lab = full.getLabRef().reshape(-1, 4)
    full.close()
    acc = np.zeros(P * (1 + K))
    for r in range(N):
        sh = _planar_ctx(gpu, R, G, B, w, h, filt.illum, r * h // N, (r + 1) * h // N)
        part = np.zeros(P * (1 + K))
        hq._lib.check(lib.hq_eval_population_partial(sh.ctx, hq._lib.fptr(pals), P, K,
                                                     hq._lib.dptr(part)), sh.ctx)
        acc += part
        sh.close()
    acc, ref = acc.reshape(P, 1 + K), ref.reshape(P, 1 + K)
    np.testing.assert_allclose(acc[:, 0], ref[:, 0], rtol=1e-9)
    np.testing.assert_array_equal(acc[:, 1:] > 0, ref[:, 1:] > 0)
    lab_ref = c_oracle.srgb_to_scielab(R, G, B, filt, w, nthreads=_threads())
    np.testing.assert_allclose(lab, lab_ref, atol=2e-4)  # device LabRef at 8192^2
    del lab_ref
    rgba = o.inline_rgba(R, G, B)
    del R, G, B
    cost, parts = c_oracle.eval_palette(rgba, lab, pals[0].reshape(K, 4), filt, w,
                                        nthreads=_threads(), return_parts=True)
    used0 = ref[0, 1:] > 0
    dev_cost = ref[0, 0] / (w * h) + 2.0 * np.count_nonzero(~used0)
    assert abs(dev_cost - cost) <= COST_RTOL * abs(cost)
    np.testing.assert_array_equal(used0, parts["used"] > 0)
    np.testing.assert_array_equal(idx0, parts["idx"].astype(np.uint8))


def test_search_survives_option_and_image_changes(gpu, filt):
    """Options and the image may change between hq_search_run calls: the search
    re-sizes the context's work buffers for the current geometry (a finer grid,
    more assign workgroups, a larger image) instead of writing past them, and a
    context whose image was invalidated (new filters) reports HQ_ERR_STATE."""
    import ctypes as C
    K, P = 32, 4
    R, G, B = o.synthetic_image(64, 48, seed=3)
    m = _planar_ctx(gpu, R, G, B, 64, 48, filt.illum)
    lib = hq.load()
    sw = hq.SWASA(population=P, imax=100, seed=9, t0=0.05)
    params = sw.params()
    handle = C.c_void_p()
    hq._lib.check(lib.hq_search_create(m.ctx, C.byref(params), K, sw.seed, C.byref(handle)), m.ctx)
    ran = C.c_int()
    hq._lib.check(lib.hq_search_run(handle, 5, C.byref(ran)), m.ctx)
    m.setOption("grid", 64)
    m.setOption("assign_blocks_per_cu", 32)
    hq._lib.check(lib.hq_search_run(handle, 5, C.byref(ran)), m.ctx)
    R2, G2, B2 = o.synthetic_image(700, 300, seed=4)
    hq._lib.check(lib.hq_set_image_planar_shard(m.ctx, hq._lib.fptr(R2), hq._lib.fptr(G2),
                                                hq._lib.fptr(B2), 700, 300,
                                                hq._lib.fptr(filt.illum), 0, 300), m.ctx)
    hq._lib.check(lib.hq_search_run(handle, 5, C.byref(ran)), m.ctx)
    assert ran.value == 5
    err = C.c_double()
    hq._lib.check(lib.hq_search_best(handle, None, C.byref(err), None), m.ctx)
    assert np.isfinite(err.value) and err.value > 0
    k1, k2, k3, ak3 = (np.ascontiguousarray(x, np.float32) for x in
                       (filt.k1, filt.k2, filt.k3, filt.absk3))
    hq._lib.check(lib.hq_set_filters(m.ctx, k1.shape[0], hq._lib.fptr(k1), hq._lib.fptr(k2),
                                     hq._lib.fptr(k3), hq._lib.fptr(ak3)), m.ctx)
    assert lib.hq_search_run(handle, 1, C.byref(ran)) == hq._lib.HQ_ERR_STATE
    lib.hq_search_destroy(handle)
    m.close()


# ---------------------------------------------------------------------------
# Per-pixel parity of the stencil (CL:234-306), Opp->Lab (CL:118-145) and dE
# (CL:201-209): the cost kernels' per-pixel dE (test option pixel_err) against
# the oracle's error image, not only through the mean.
# ---------------------------------------------------------------------------
def _dark_case(w, h, seed):
    """A synthetic image with a near-black block (u8 0..6) and a palette whose
    second half is near-black colours: the filtered opponent values there fall
    in Opp->Lab's linear segment (t <= 216/24389, CL:137-143)."""
    R, G, B = o.synthetic_image(w, h, seed=seed)
    rng = np.random.default_rng(seed)
    y0, x0 = h // 4, w // 5
    for P_ in (R, G, B):
        blk = P_.reshape(h, w)[y0:y0 + h // 2, x0:x0 + w // 2]
        blk[...] = rng.integers(0, 7, blk.shape).astype(np.float32) / np.float32(255)
    return R, G, B


def exact_pixel_err(idx, pal, lab_ref, f, w, h, lab_only=False):
    """The per-pixel dE of CL:194-198 (palette -> opponent), CL:234-306 (both
    stencil passes, reflection CL:256-263), CL:118-145 (Opp->Lab) and CL:201-209
    (dE76), evaluated in float64 from the same fp32 inputs (palette, taps,
    LabRef): the exact value that both fp32 paths -- the reference's order in
    the oracle and the GPU's -- approximate.  lab_only: the candidate's float64
    Lab (n x 3) instead of dE76."""
    d = np.float64
    p = pal[:, :3].astype(d)
    lin = np.where(p <= 0.04045, p / 12.92, ((p + 0.055) / 1.055) ** float(np.float32(2.4)))
    img = (lin @ o.RGB2OPPM.astype(d).T)[np.asarray(idx, np.int64)].reshape(h, w, 3)
    half = f.half
    hidx, vidx = o.reflect_index(w, half), o.reflect_index(h, half)
    k1, k2 = f.k1[:, :3].astype(d), f.k2[:, :3].astype(d)
    k3, ak3 = np.asarray(f.k3, d), np.asarray(f.absk3, d)
    t1 = np.zeros((h, w, 3)); t2 = np.zeros((h, w, 3)); t3 = np.zeros((h, w))
    for t in range(2 * half + 1):
        src = img[:, hidx[:, t], :]
        t1 += src * k1[t]
        t2 += src * k2[t]
        t3 += src[..., 0] * k3[t]
    out = np.zeros((h, w, 3))
    for t in range(2 * half + 1):
        r = vidx[:, t]
        out += t1[r] * k1[t] + t2[r] * k2[t]
        out[..., 0] += t3[r] * ak3[t]
    xyz = out.reshape(-1, 3) @ o.OPP2XYZM.astype(d).T / np.asarray(f.illum[:3], d)
    lin_seg = (d(o.KAPPA) * xyz + 16.0) / 116.0
    fx = np.where(xyz > d(o.LABDELTA3), np.cbrt(xyz), lin_seg)
    lab = np.stack([116.0 * fx[:, 1] - 16.0, 500.0 * (fx[:, 0] - fx[:, 1]), 200.0 * (fx[:, 1] - fx[:, 2])], -1)
    if lab_only:
        return lab
    return np.sqrt(((np.asarray(lab_ref, d).reshape(-1, 4)[:, :3] - lab) ** 2).sum(-1))


def _pal_with_dark(K, seed):
    pal = o.synthetic_palette(K, seed).copy()
    rng = np.random.default_rng(seed)
    pal[K // 2:, :3] = rng.integers(0, 7, (K - K // 2, 3)).astype(np.float32) / np.float32(255)
    return pal


@pytest.mark.parametrize("variant", [(0, 16), (0, 8), (1, 16), (2, 16)])
@pytest.mark.parametrize("case", ["case_64x48_k16", "case_97x53_k64", "dark_256_9660", "dark_193x131_7245",
                                  "dark_256_30050", "dark_200x136_15030", "dark_160x144_20030"])
def test_pixel_errors_vs_oracle(gpu, case, variant):
    """(cost_variant, cost_rows): the default 16 x 128 tiles (cost16w), the 8 x 108
    tiles (cost_mfma), the LDS-tiled generic pair and the per-pixel generic pair
    (the reference's summation order); 300 dpi / 50 cm (half 51) takes the
    generic path whatever the variant.  Every pixel's dE -- border
    pixels (reflection, CL:256-263), pixels in the linear Lab segment, edge and
    partial tiles -- within 2e-4 absolute of the oracle's error image (same
    LabRef on both sides), at most 2x the oracle's own worst distance from a
    float64 evaluation and 1.5x its mean (the comment below says why the bar is
    relative to float64), and the indices bit-exact."""
    if case.startswith("case_"):
        g, R, G, B = load_case(case)
        w, h = int(g["w"]), int(g["h"])
        f = o.design_filters()
        dpi, vd = 72, 45.0
        pals = [p for p in g["palettes"]]
        lab = g["lab"].astype(np.float32)
    else:
        dims, geo = case.split("_")[1], case.split("_")[2]
        w, h = (int(v) for v in dims.split("x")) if "x" in dims else (int(dims), int(dims))
        # (96/60: tap bucket 19, 150/30: 15, 200/30: 24 -- the pair layout's 3 and 4 K steps)
        dpi, vd = {"9660": (96, 60.0), "7245": (72, 45.0), "30050": (300, 50.0), "15030": (150, 30.0),
                   "20030": (200, 30.0)}[geo]
        f = o.design_filters(dpi, vd)
        R, G, B = _dark_case(w, h, seed=w + h)
        pals = [_pal_with_dark(64, 900 + w), _pal_with_dark(256, 901 + w)]
        lab = c_oracle.srgb_to_scielab(R, G, B, f, w, nthreads=_threads())
    rgba = o.inline_rgba(R, G, B)
    m = hq.ImageManipulation(device=gpu)
    sp = hq.ScielabProcessor(dpi, vd, hq.Whitepoint.D65, None, m)
    m.setOption("pixel_err", 1)
    m.setOption("cost_variant", variant[0])
    m.setOption("cost_rows", variant[1])
    m.setImage(rgba.reshape(-1), lab.reshape(-1), w, sp.illuminant)
    dark_lin = 0
    for pal in pals:  # one population per palette (K differs between them)
        K = pal.shape[0]
        m.computeQuantizationErrorPopulation([pal.reshape(-1)], 2.0)
        ref, parts = c_oracle.eval_palette(rgba, lab, pal, f, w, nthreads=_threads(), return_parts=True)
        np.testing.assert_array_equal(m.getIndices(0), parts["idx"].astype(np.uint8))
        err = m.getPixelErrors(0)
        # Tolerance.  a = 500 (fx - fy) and b = 200 (fy - fz) (CL:143-145) turn one
        # ulp of f (1.2e-7 near 1) into 6e-5 of dE, so two fp32 orders of the same
        # sums cannot agree to 2e-5: the oracle alone is up to ~1e-4 (mean ~1.3e-5)
        # from the float64 value.  Both fp32 paths are therefore measured against
        # the float64 evaluation of the same inputs: the GPU's per-pixel error may
        # be at most 2x the oracle's worst pixel and 1.5x its mean (measured: at
        # most 1.56x and 1.23x over these cases; 4x before the cube root moved to
        # unscaled t, hq_device.h lab_f_fast), and every pixel within 2e-4 of
        # the oracle's.
        ex = exact_pixel_err(parts["idx"], pal, lab, f, w, h)
        e_gpu, e_orc = np.abs(err - ex), np.abs(parts["err"] - ex)
        stats = (f"{case} K={K} variant {variant}: |gpu-exact| max {e_gpu.max():.3g} mean {e_gpu.mean():.3g}; "
                 f"|oracle-exact| max {e_orc.max():.3g} mean {e_orc.mean():.3g}")
        print(stats)
        np.testing.assert_allclose(err, parts["err"], rtol=0, atol=2e-4, err_msg=stats)
        assert e_gpu.max() <= 2 * e_orc.max(), stats
        assert e_gpu.mean() <= 1.5 * e_orc.mean(), stats
        dark_lin += int(np.count_nonzero(parts["idx"] >= K // 2)) if not case.startswith("case_") else 0
    if not case.startswith("case_"):
        assert dark_lin > 1000  # the near-black colours were chosen (linear-segment Lab)
    m.close()


def _de94_exact(lab_ref, lab):
    """CL:217-226 in float64 on float64 Lab; also returns dH^2 and da^2 + db^2."""
    p1 = np.asarray(lab_ref, np.float64).reshape(-1, 4)[:, :3]
    L1, a1, b1 = p1[:, 0], p1[:, 1], p1[:, 2]
    L2, a2, b2 = lab[:, 0], lab[:, 1], lab[:, 2]
    c1 = np.hypot(a1, b1)
    dC = c1 - np.hypot(a2, b2)
    dab2 = (a1 - a2) ** 2 + (b1 - b2) ** 2
    dH2 = dab2 - dC * dC
    e = np.sqrt((L1 - L2) ** 2 + (dC / (1 + 0.045 * c1)) ** 2 + np.maximum(dH2, 0) / (1 + 0.015 * c1) ** 2)
    return e, dH2, dab2


@pytest.mark.parametrize("variant", [(0, 16), (0, 8), (1, 16), (2, 16)])
@pytest.mark.parametrize("case", ["case_97x53_k64", "dark_193x131_7245", "dark_256_9660", "dark_200x136_15030",
                                  "dark_160x144_20030"])
def test_pixel_errors_de94_vs_oracle(gpu, case, variant):
    """dE94 (CL:217-226) per pixel against the oracle's fp32 statement of it
    (oracle.ciede94_f32 on the oracle's candidate Lab) and a float64 evaluation.
    The reference's dH = sqrt(fma(da, da, db db) - dC dC) has no clamp: where
    fp32 rounding makes the argument negative (the hue difference ~1e-4 of the
    colour difference or less; ~3e-4 of the pixels of a synthetic image) it is
    NaN, the pixel's dE is NaN, and so is the mean (IM:736-768).  The GPU keeps
    that: a NaN pixel on either side must have a float64 dH^2 within rounding of
    0, the cost is NaN exactly when a pixel is, and every finite pixel meets
    dE76's bars (2x the oracle's worst distance from float64, 1.5x its mean)."""
    if case.startswith("case_"):
        g, R, G, B = load_case(case)
        w, h = int(g["w"]), int(g["h"])
        f = o.design_filters()
        dpi, vd = 72, 45.0
        pals = [p for p in g["palettes"]]
        lab = g["lab"].astype(np.float32)
    else:
        dims, geo = case.split("_")[1], case.split("_")[2]
        w, h = (int(v) for v in dims.split("x")) if "x" in dims else (int(dims), int(dims))
        dpi, vd = {"9660": (96, 60.0), "7245": (72, 45.0), "15030": (150, 30.0), "20030": (200, 30.0)}[geo]
        f = o.design_filters(dpi, vd)
        R, G, B = _dark_case(w, h, seed=w + h)
        pals = [_pal_with_dark(64, 900 + w), _pal_with_dark(256, 901 + w)]
        lab = c_oracle.srgb_to_scielab(R, G, B, f, w, nthreads=_threads())
    rgba = o.inline_rgba(R, G, B)
    m = hq.ImageManipulation(hq.deltaETypes.CIE94, device=gpu)
    sp = hq.ScielabProcessor(dpi, vd, hq.Whitepoint.D65, None, m)
    m.setOption("pixel_err", 1)
    m.setOption("cost_variant", variant[0])
    m.setOption("cost_rows", variant[1])
    m.setImage(rgba.reshape(-1), lab.reshape(-1), w, sp.illuminant)
    for pal in pals:
        K = pal.shape[0]
        cost = m.computeQuantizationErrorPopulation([pal.reshape(-1)], 2.0)[0]
        _, parts = c_oracle.eval_palette(rgba, lab, pal, f, w, nthreads=_threads(), return_parts=True)
        np.testing.assert_array_equal(m.getIndices(0), parts["idx"].astype(np.uint8))
        err = m.getPixelErrors(0)
        e_orc = o.ciede94_f32(lab, o.candidate_scielab(parts["idx"], pal, f, w, h))
        ex, dH2, dab2 = _de94_exact(lab, exact_pixel_err(parts["idx"], pal, lab, f, w, h, lab_only=True))
        nan_g, nan_o = np.isnan(err), np.isnan(e_orc)
        # a NaN needs dH^2 within rounding of 0: fp32 Lab is ~1e-4 from float64
        # in a and b (the 500x and 200x of CL:143-145), moving dH^2 by ~2e-4 |dab|
        near0 = np.abs(dH2) <= 1e-3 * (np.sqrt(dab2) + 1.0)
        assert near0[nan_g].all() and near0[nan_o].all()
        assert nan_g.mean() < 2e-3
        ok = ~(nan_g | nan_o)
        d_gpu, d_orc = np.abs(err[ok] - ex[ok]), np.abs(e_orc[ok] - ex[ok])
        stats = (f"{case} K={K} variant {variant}: NaN px gpu {int(nan_g.sum())} oracle {int(nan_o.sum())}; "
                 f"|gpu-exact| max {d_gpu.max():.3g} mean {d_gpu.mean():.3g}; "
                 f"|oracle-exact| max {d_orc.max():.3g} mean {d_orc.mean():.3g}")
        print(stats)
        np.testing.assert_allclose(err[ok], e_orc[ok], rtol=0, atol=2e-4, err_msg=stats)
        assert d_gpu.max() <= 2 * d_orc.max(), stats
        assert d_gpu.mean() <= 1.5 * d_orc.mean(), stats
        assert np.isnan(cost) == bool(nan_g.any()), stats
        if not nan_g.any():  # the mean (IM:736-768) and the penalty
            used = np.bincount(parts["idx"], minlength=K)[:K] > 0
            ref = float(np.mean(ex)) + float(np.count_nonzero(~used)) * 2.0
            assert abs(cost - ref) <= 1e-5 * ref, stats
    m.close()


@pytest.mark.parametrize("w,h", [(10, 10), (11, 37), (37, 11), (129, 17)])
@pytest.mark.parametrize("K,P", [(1, 1), (2, 5), (3, 2), (255, 3)])
def test_small_images_and_palettes_vs_oracle(gpu, filt, w, h, K, P):
    """Edge shapes against the oracle: images down to the stencil's half-width
    (10 x 10: every pixel's window reflects at both edges, CL:256-263), images
    smaller than one 16 x 128 tile in either direction, ragged tiles, and
    palettes of 1, 2, 3 and 255 colours (a one-colour palette: every pixel
    index 0, no penalty).  Indices and used flags bit-exact, costs within 1e-5."""
    R, G, B = o.synthetic_image(w, h, seed=w * 131 + h + K)
    rgba = o.inline_rgba(R, G, B)
    pals = np.stack([o.synthetic_palette(K, 500 + p) for p in range(P)])
    m = hq.ImageManipulation(device=gpu)
    hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    m.setImage(rgba.reshape(-1), None, w, filt.illum)
    lab = m.getLabRef().reshape(-1, 4)
    costs, used = m.computeQuantizationErrorPopulation(pals.reshape(P, -1), 2.0, return_used=True)
    idx = [m.getIndices(p) for p in range(P)]
    m.close()
    for p in range(P):
        ref, parts = c_oracle.eval_palette(rgba, lab, pals[p], filt, w, return_parts=True)
        np.testing.assert_array_equal(idx[p], parts["idx"].astype(np.uint8))
        np.testing.assert_array_equal(used[p], parts["used"])
        assert abs(costs[p] - ref) <= 1e-5 * abs(ref), (p, costs[p], ref)
