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
@pytest.mark.parametrize("variant", [(0, 11), (0, 10), (0, 9), (0, 7), (0, 8), (0, 6), (0, 4), (0, 5), (0, 2), (0, 0), (0, 1), (0, 3), (1, 0)])
@pytest.mark.parametrize("name", ["case_64x48_k16", "case_97x53_k64"])
def test_eval_golden(ip, name, grid, variant):
    """(cost_variant, cost_tile): 8-row tiles with the row-pair horizontal pass
    (in two channel groups: default, and with the vertical passes on the matrix cores;
    all filters at once, 2 or 4 columns per item), row-layout 8-row tiles, 16-row
    tiles, the split vertical pass, the vertical pass on the matrix cores
    (split-f16 products), the generic two-pass path."""
    g, R, G, B = load_case(name)
    w = int(g["w"])
    ip.setOption("grid", grid)
    ip.setOption("cost_variant", variant[0])
    ip.setOption("cost_tile", variant[1])
    ip.setOption("assign_rep", (1, 4, 16)[grid % 3])
    ip.setImage(o.inline_rgba(R, G, B).reshape(-1), g["lab"].reshape(-1), w, ip.illum)
    pals = g["palettes"]
    costs, used = ip.computeQuantizationErrorPopulation(pals.reshape(len(pals), -1), 2.0,
                                                        return_used=True)
    np.testing.assert_allclose(costs, g["costs"], rtol=1e-6)
    np.testing.assert_array_equal(used, g["used"])
    for p in range(len(pals)):
        np.testing.assert_array_equal(ip.getIndices(p), g["idx"][p])


@pytest.mark.parametrize("bands", [2, 3, 16])
@pytest.mark.parametrize("tile", [11, 10, 9, 7, 6, 8])
@pytest.mark.parametrize("name", ["case_64x48_k16", "case_97x53_k64"])
def test_eval_golden_banded(ip, name, tile, bands):
    """The banded pipeline (assign of row band j+1 on a second stream beside the
    cost of band j) gives the unbanded results bit for bit: same indices, same
    per-tile partials summed in the same order, same used masks."""
    g, R, G, B = load_case(name)
    w = int(g["w"])
    ip.setOption("cost_tile", tile)
    ip.setOption("bands", bands)
    ip.setOption("band_cpb", 1 + bands % 3)
    ip.setImage(o.inline_rgba(R, G, B).reshape(-1), g["lab"].reshape(-1), w, ip.illum)
    pals = g["palettes"]
    costs, used = ip.computeQuantizationErrorPopulation(pals.reshape(len(pals), -1), 2.0,
                                                        return_used=True)
    np.testing.assert_allclose(costs, g["costs"], rtol=1e-6)
    np.testing.assert_array_equal(used, g["used"])
    for p in range(len(pals)):
        np.testing.assert_array_equal(ip.getIndices(p), g["idx"][p])
    ip.setOption("bands", 0)
    c0 = ip.computeQuantizationErrorPopulation(pals.reshape(len(pals), -1), 2.0)
    np.testing.assert_array_equal(costs, c0)


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


@pytest.mark.parametrize("de", [hq.deltaETypes.CIE76, hq.deltaETypes.CIE94])
@pytest.mark.parametrize("trim", [1, 0])
def test_mfma_passes_match_valu(gpu, de, trim):
    """cost_tile 7 runs the vertical taps on the matrix cores in split f16
    (hi.hi + hi.lo + lo.hi, ~2^-22 relative per product dropped), cost_tile 8 both
    passes; their costs agree with cost_tile 6's fp32 VALU passes to 1e-6 relative
    (the bar is 1e-4)."""
    w, h = 300, 77  # interior, edge and partial tiles
    R, G, B = o.synthetic_image(w, h, seed=5)
    m = hq.ImageManipulation(de, device=gpu)
    sp = hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    m.setImage(o.inline_rgba(R, G, B).reshape(-1), None, w, sp.illuminant)
    pals = [o.synthetic_palette(K, 7 + K) for K in (16, 64, 256)]
    m.setOption("trim", trim)
    out = {}
    for tile in (6, 7, 8, 9, 10, 11):
        m.setOption("cost_tile", tile)
        out[tile] = np.array([m.computeQuantizationErrorPopulation([p.reshape(-1)], 2.0)[0]
                              for p in pals])
    np.testing.assert_allclose(out[7], out[6], rtol=1e-6)
    np.testing.assert_allclose(out[8], out[6], rtol=1e-6)
    np.testing.assert_allclose(out[9], out[6], rtol=1e-6)
    np.testing.assert_allclose(out[10], out[6], rtol=1e-6)
    np.testing.assert_allclose(out[11], out[6], rtol=1e-6)
    m.close()


# ---------------------------------------------------------------------------
# argmin edge cases (CL:179-193), bit-exact
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("grid", [64, 32, 16, 0])
@pytest.mark.parametrize("group_batch", [(1, 0), (1, 4), (1, 8), (4, 1), (4, 2), (4, 3), (4, 5)])
def test_assign_edge_cases(ip, grid, group_batch):
    g = np.load(os.path.join(GOLD, "edge_assign.npz"))
    px = g["px"]  # 4096 pixels -> 64 x 64 image, values partly outside [0, 1]
    ip.setOption("grid", grid)
    ip.setOption("assign_group", group_batch[0])
    ip.setOption("assign_batch", group_batch[1])
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
    for grid, group, rep, batch in ((64, 1, 4, 0), (32, 4, 4, 0), (32, 2, 4, 0), (32, 4, 1, 0),
                                    (16, 4, 2, 0), (0, 1, 16, 0), (32, 1, 1, 4), (32, 1, 1, 8),
                                    (64, 1, 1, 8), (0, 1, 1, 4), (32, 4, 1, 1), (32, 4, 1, 2),
                                    (64, 4, 1, 2), (16, 4, 1, 1), (0, 4, 1, 2), (32, 4, 1, 3),
                                    (64, 4, 1, 3), (0, 4, 1, 3), (32, 4, 1, 5), (64, 4, 1, 5),
                                    (16, 4, 1, 5), (0, 4, 1, 5)):
        ip.setOption("grid", grid)
        ip.setOption("assign_group", group)
        ip.setOption("assign_rep", rep)
        ip.setOption("assign_batch", batch)
        pals = [pal.reshape(-1), pal[::-1].copy().reshape(-1), pal.reshape(-1)]
        _, used = ip.computeQuantizationErrorPopulation(pals, 2.0, return_used=True)
        np.testing.assert_array_equal(ip.getIndices(0), ref_idx.astype(np.uint8))
        np.testing.assert_array_equal(ip.getIndices(2), ref_idx.astype(np.uint8))
        np.testing.assert_array_equal(used[0], ref_used)
        rev_idx, rev_used = c_oracle.assign(px, pal[::-1].copy())
        np.testing.assert_array_equal(ip.getIndices(1), rev_idx.astype(np.uint8))
        np.testing.assert_array_equal(used[1], rev_used)


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


@pytest.mark.parametrize("batch", [5, 3])
@pytest.mark.parametrize("P", [1, 2, 3, 5, 8])
def test_assign_group_sizes(ip, P, batch):
    """Groups of 1-4 palettes per pixel pass (P = 5: a full group and a group of
    one; the lane kernel then runs 64 / ng pixels per wave instruction).  P = 1,
    2, 3 run assign_pipe_kernel<NG = P>, P >= 4 its NG = 4 instance."""
    rng = np.random.default_rng(P)
    w, h, K = 75, 41, 96
    px = np.zeros((w * h, 4), np.float32)
    px[:, :3] = (rng.integers(0, 256, (w * h, 3)) / 255.0).astype(np.float32)
    pals = np.stack([o.synthetic_palette(K, 300 + p) for p in range(P)])
    ip.setOption("assign_group", 4)
    ip.setOption("assign_batch", batch)
    ip.setImage(px.reshape(-1), np.zeros_like(px).reshape(-1), w, ip.illum)
    _, used = ip.computeQuantizationErrorPopulation(pals.reshape(P, -1), 2.0, return_used=True)
    for p in range(P):
        ref_idx, ref_used = c_oracle.assign(px, pals[p])
        np.testing.assert_array_equal(ip.getIndices(p), ref_idx.astype(np.uint8))
        np.testing.assert_array_equal(used[p], ref_used)


def test_nonfinite_palette_falls_back_exactly(ip):
    w = h = 32
    px = np.zeros((w * h, 4), np.float32)
    px[:, :3] = np.random.default_rng(3).random((w * h, 3), dtype=np.float32)
    pal = o.synthetic_palette(16, 5)
    pal[3, 1] = np.nan
    pal[7, 0] = np.inf
    ip.setImage(px.reshape(-1), np.zeros_like(px).reshape(-1), w, ip.illum)
    ip.computeQuantizationErrorPopulation([pal.reshape(-1)], 2.0)
    ref_idx, _ = c_oracle.assign(px, pal)
    np.testing.assert_array_equal(ip.getIndices(0), ref_idx.astype(np.uint8))


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
    lib.hq_eval_population_partial(full.ctx, hq._lib.fptr(pals), P, K, hq._lib.dptr(ref))
    for nshards in (2, 3, 7):
        bounds = np.linspace(0, h, nshards + 1).astype(int)
        acc = np.zeros(P * (1 + K))
        for r0, r1 in zip(bounds[:-1], bounds[1:]):
            sh = hq.ImageManipulation(device=gpu)
            hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, sh)
            sh.setImage(rgba, None, w, filt.illum, row_begin=r0, row_end=r1)
            sh.setOption("bands", nshards)  # banded pipeline inside a shard
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


@pytest.mark.parametrize("P", [1, 3, 4])
def test_device_search_matches_host_driven(gpu, filt, P):
    """The device-resident SWASA loop (sa_step_kernel: acceptance, convergence,
    java.util.Random draws by jump table, neighbour generation) follows the
    host-driven driver's trajectory exactly on the same GPU costs, across
    resumed run() calls and up to imax."""
    import ctypes as C
    w, h, K = 96, 64, 16
    R, G, B = o.synthetic_image(w, h, seed=9)
    m = hq.ImageManipulation(device=gpu)
    hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    m.setImage(o.inline_rgba(R, G, B).reshape(-1), None, w, filt.illum)
    lib = hq.load()
    res = {}
    for dev in (0, 1, 2):  # host-driven; device, SA step fused with the grid; device, unfused
        m.setOption("sa_device", int(dev > 0))
        m.setOption("sa_fuse_grid", int(dev < 2))
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
    for dev in (1, 2):
        assert res[dev][2] == res[0][2] == res[dev][3] == res[0][3] == 50
        assert res[dev][1] == res[0][1]
        np.testing.assert_array_equal(res[dev][0], res[0][0])
    m.close()


def test_device_search_with_single_rank_comm(gpu, filt):
    """The multi-GPU search loop on one GPU: with libhq's RCCL communicator the
    all-reduce sits between finalize and sa_step in every iteration; with one
    rank the trajectory must be the one without a communicator."""
    import ctypes as C
    w, h, K, P = 80, 72, 24, 4
    R, G, B = o.synthetic_image(w, h, seed=12)
    lib = hq.load()
    res = []
    for comm in (False, True):
        m = hq.ImageManipulation(device=gpu)
        hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
        m.setImage(o.inline_rgba(R, G, B).reshape(-1), None, w, filt.illum)
        if comm:
            m.initComm(1, 0, hq.ImageManipulation.commUniqueId())
        sw = hq.SWASA(population=P, imax=30, seed=21, t0=0.05)
        params = sw.params()
        handle = C.c_void_p()
        hq._lib.check(lib.hq_search_create(m.ctx, C.byref(params), K, sw.seed, C.byref(handle)), m.ctx)
        ran = C.c_int()
        hq._lib.check(lib.hq_search_run(handle, 30, C.byref(ran)), m.ctx)
        best = np.zeros(4 * K, np.float32)
        err = C.c_double()
        it = C.c_int()
        hq._lib.check(lib.hq_search_best(handle, hq._lib.fptr(best), C.byref(err), C.byref(it)), m.ctx)
        lib.hq_search_destroy(handle)
        m.close()
        res.append((best, err.value, ran.value))
    assert res[0][2] == res[1][2] == 30
    assert res[0][1] == res[1][1]
    np.testing.assert_array_equal(res[0][0], res[1][0])


# ---------------------------------------------------------------------------
# Full-size properties (4096^2, K = 256): determinism, grid == exhaustive,
# fast == generic, shards == full.
# ---------------------------------------------------------------------------
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
    for bands in (2, 5, 16):  # banded pipeline: bit-identical
        m.setOption("bands", bands)
        cb = m.computeQuantizationErrorPopulation(pals, 2.0)
        np.testing.assert_array_equal(m.getIndices(1), idx1)
        np.testing.assert_array_equal(cb, c1)
    m.setOption("bands", 0)
    for batch in (3, 5):  # assign: pixel-per-lane and (pixel, palette)-per-lane pipelines
        m.setOption("assign_batch", batch)
        cb = m.computeQuantizationErrorPopulation(pals, 2.0)
        np.testing.assert_array_equal(m.getIndices(1), idx1)
        np.testing.assert_array_equal(cb, c1)
    m.setOption("grid", 64)
    for variant, tile in ((1, 0), (0, 0), (0, 1), (0, 2), (0, 3), (0, 4), (0, 5), (0, 6), (0, 8), (0, 9), (0, 10), (0, 11)):
        m.setOption("cost_variant", variant)
        m.setOption("cost_tile", tile)
        c4 = m.computeQuantizationErrorPopulation(pals, 2.0)
        np.testing.assert_allclose(c4, c1, rtol=1e-6)  # generic == every tile configuration
    m.setOption("cost_variant", 0)
    m.setOption("trim", 0)  # all 21 taps of the narrow filters
    c5 = m.computeQuantizationErrorPopulation(pals, 2.0)
    np.testing.assert_allclose(c5, c1, rtol=1e-7)
    assert np.all(np.isfinite(c1)) and np.all(c1 > 0)
    m.close()
