"""Parity against the reference itself: the reference's own OpenCL kernels
(OptimizedConvolution.cl, compiled unmodified for gfx950 by `make -C oracle
ref` into oracle/_ref/, run on the MI355X through the ROCm OpenCL runtime by
oracle/ref_cl_host.c, a restatement of the JavaCL host sequences IM:100-153,
IM:285-370, IM:450-493 + IM:620-727, IM:770-798) against libhq through the C
ABI, and against the C oracle that the other tests use as their checker.

Bars: chosen colours (the reference's `quantize`, CL:147-170: its distance()
argmin with strict <) and used flags bit-exact; costs within 1e-6 relative
(the north-star bar is 1e-4); per-pixel dE within 3e-4 absolute of the
reference's error image (CL:201-209; libhq and the oracle each sum the stencil
in their own fp32 order); LabRef within 2e-4 absolute (IM:285-370).
"""

import os

import numpy as np
import pytest

import c_oracle
import hybridquantization_amd as hq
import oracle as o
import ref_cl

pytestmark = pytest.mark.gpu

PIX_ATOL = 3e-4


@pytest.fixture(scope="module")
def filt():
    return o.design_filters()


@pytest.fixture(scope="module")
def refk(gpu):
    # The build needs the reference's source tree (make -C oracle ref, run by
    # build() when it is present); a checkout without it cannot run these.  A
    # build that is present but does not run on the GPU fails, with the
    # runtime's message.
    if not all(os.path.exists(p) for p in (ref_cl.LIB_PATH, *ref_cl.BIN_PATHS.values())):
        pytest.skip("reference kernels not built (oracle/_ref: make -C oracle ref needs the reference tree)")
    ref_cl.lib()
    return ref_cl


def _threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def _ctx(gpu, rgba, lab, w, illum, dpi=72, dist=45.0, **opts):
    m = hq.ImageManipulation(device=gpu)
    hq.ScielabProcessor(dpi, dist, hq.Whitepoint.D65, None, m)
    m.setImage(rgba.reshape(-1), None if lab is None else lab.reshape(-1), w, illum)
    for k, v in opts.items():
        m.setOption(k, v)
    return m


@pytest.mark.parametrize("w,h", [(97, 53), (256, 256), (333, 217), (1024, 640)])
def test_labref_matches_reference_kernels(gpu, refk, filt, w, h):
    """IM:100 RGBtoXYZ + IM:285 XYZtoScielab on the reference's kernels (filter by
    filter, the update flag) against libhq's device LabRef and the oracle's."""
    R, G, B = o.synthetic_image(w, h, seed=w + h)
    ref = refk.srgb_to_scielab(R, G, B, filt, w)
    m = _ctx(gpu, o.inline_rgba(R, G, B), None, w, filt.illum)
    lab = m.getLabRef().reshape(-1, 4)
    m.close()
    np.testing.assert_allclose(lab[:, :3], ref[:, :3], atol=2e-4)
    np.testing.assert_allclose(c_oracle.srgb_to_scielab(R, G, B, filt, w)[:, :3], ref[:, :3], atol=2e-4)


@pytest.mark.parametrize("w,h,K,P", [(256, 256, 16, 4), (97, 53, 64, 2), (333, 217, 256, 3), (1024, 512, 256, 2),
                                     (320, 200, 600, 2), (320, 200, 2048, 1), (128, 96, 4096, 2),
                                     (96, 64, 20000, 1), (10, 10, 16, 2), (11, 37, 5, 3), (64, 48, 1, 2),
                                     (64, 48, 2, 2)])
def test_costs_match_reference_kernels(gpu, refk, filt, w, h, K, P):
    """computeQuantizationErrorPopulation on the reference's kernels (IM:620-727)
    against libhq's evaluation and the C oracle's, on the same LabRef (the
    reference's): costs, used flags, the per-pixel dE of palette 0, and the
    chosen colours (the reference's quantize kernel) -- at C1 (256^2, K = 16, P =
    4), K = 256 on ragged images, chunked palettes (K = 600, 2048), native 16-bit
    lists (K = 4096), the exhaustive 32-bit path (K = 20000 > 16384), images as
    small as the stencil's half-width (10 x 10, 11 x 37: reflection at both
    edges of every row and column), and K = 1, 2, 5."""
    R, G, B = o.synthetic_image(w, h, seed=3 * w + K)
    rgba = o.inline_rgba(R, G, B)
    lab = refk.srgb_to_scielab(R, G, B, filt, w)
    pals = np.stack([o.synthetic_palette(K, 40 + p) for p in range(P)])
    rc, ru, re = refk.eval_population(rgba, lab, w, pals, filt, return_err=True)
    m = _ctx(gpu, rgba, lab, w, filt.illum, pixel_err=1)
    costs, used = m.computeQuantizationErrorPopulation(pals.reshape(P, -1), 2.0, return_used=True)
    idx = [m.getIndices32(p) for p in range(P)]
    pe0 = m.getPixelErrors(0)
    m.close()
    np.testing.assert_allclose(costs, rc, rtol=1e-6)
    np.testing.assert_array_equal(used > 0, ru != 0)
    assert np.abs(pe0 - re[0]).max() <= PIX_ATOL
    for p in range(P):
        q, qu = refk.quantize(rgba, pals[p])
        np.testing.assert_array_equal(pals[p][idx[p]], q)
        np.testing.assert_array_equal(qu != 0, ru[p] != 0)
    oc, parts = c_oracle.eval_palette(rgba, lab, pals[0], filt, w, nthreads=_threads(), return_parts=True)
    assert abs(oc - rc[0]) <= 1e-6 * rc[0]
    assert np.abs(parts["err"] - re[0]).max() <= PIX_ATOL


@pytest.mark.parametrize("dpi,dist", [(96, 60.0), (150, 30.0), (200, 30.0), (72, 30.0), (300, 50.0), (300, 100.0)])
def test_viewing_geometries_match_reference_kernels(gpu, refk, dpi, dist):
    """Other viewing geometries (HQ:229-231): halfSize 19, 15, 20 and 7 (the
    tiled kernel's 19-, 15-, 24- and 10-tap buckets), 51 (the generic
    matrix-core pair) and 102 (205 taps: the generic fp32 pair).  Up to 103
    taps the costs agree within 1e-6 and every pixel within 3e-4; at 205 taps
    two fp32 orders of each pixel's 2 x 205-tap sums drift further apart, so
    the costs are held to 1e-5 and to a float64 evaluation of the same inputs:
    libhq no further from it than the reference (x 1.5)."""
    from test_gpu import exact_pixel_err

    f = o.design_filters(dpi, dist)
    w, h, K, P = 301, 173, 64, 2
    R, G, B = o.synthetic_image(w, h, seed=dpi)
    rgba = o.inline_rgba(R, G, B)
    lab = refk.srgb_to_scielab(R, G, B, f, w)
    pals = np.stack([o.synthetic_palette(K, 60 + p) for p in range(P)])
    rc, ru, re = refk.eval_population(rgba, lab, w, pals, f, return_err=True)
    m = _ctx(gpu, rgba, None, w, f.illum, dpi=dpi, dist=dist, pixel_err=1)
    np.testing.assert_allclose(m.getLabRef().reshape(-1, 4)[:, :3], lab[:, :3], atol=2e-4)
    m.close()
    m = _ctx(gpu, rgba, lab, w, f.illum, dpi=dpi, dist=dist, pixel_err=1)
    costs, used = m.computeQuantizationErrorPopulation(pals.reshape(P, -1), 2.0, return_used=True)
    pe = [m.getPixelErrors(p) for p in range(P)]
    idx = [m.getIndices(p) for p in range(P)]
    m.close()
    np.testing.assert_array_equal(used > 0, ru != 0)
    if f.half <= 64:
        np.testing.assert_allclose(costs, rc, rtol=1e-6)
        for p in range(P):
            assert np.abs(pe[p] - re[p]).max() <= PIX_ATOL
        return
    np.testing.assert_allclose(costs, rc, rtol=1e-5)
    for p in range(P):
        ex = exact_pixel_err(idx[p], pals[p], lab, f, w, h)
        assert np.abs(pe[p] - re[p]).max() <= 10 * PIX_ATOL
        d_hq, d_ref = abs(float(np.mean(pe[p], dtype=np.float64)) - float(np.mean(ex))), \
            abs(float(np.mean(re[p], dtype=np.float64)) - float(np.mean(ex)))
        print(f"{dpi}/{dist} palette {p}: |mean - float64| libhq {d_hq:.3g} reference {d_ref:.3g}")
        assert d_hq <= 1.5 * d_ref + 1e-7


def _adversarial(G2=32):
    """Pixels on the level-2 cell faces i/G2 and one ulp either side; palettes:
    0 colours on faces and corners, 1 colour pairs mirrored across a face (exact
    ties), 2 colour pairs one ulp apart, 3 exact duplicates and colours equal to
    pixels."""
    rng = np.random.default_rng(77)
    w, h = 128, 96
    n = w * h
    faces = (np.arange(G2 + 1) / G2).astype(np.float32)
    vals = np.concatenate([faces, np.nextafter(faces[:-1], np.float32(2)), np.nextafter(faces[1:], np.float32(-1))])
    px = np.zeros((n, 4), np.float32)
    px[:, :3] = rng.choice(vals, size=(n, 3))
    K = 256
    pals = np.zeros((4, K, 4), np.float32)
    pals[0, :, :3] = rng.choice(faces, size=(K, 3))
    for i in range(K // 2):
        ax = i % 3
        f = faces[rng.integers(1, G2)]
        d = np.float32(rng.integers(1, 8)) / np.float32(4 * G2)
        base = rng.choice(faces, 3)
        a, b = base.copy(), base.copy()
        a[ax], b[ax] = f - d, f + d
        pals[1, 2 * i, :3], pals[1, 2 * i + 1, :3] = np.clip(a, 0, 1), np.clip(b, 0, 1)
        on = base.copy()
        on[ax] = f
        px[i, :3] = on
    c = rng.random((K // 2, 3), dtype=np.float32)
    pals[2, 0::2, :3] = c
    pals[2, 1::2, :3] = np.nextafter(c, np.float32(2))
    pals[3, :, :3] = (rng.integers(0, 256, (K, 3)) / 255.0).astype(np.float32)
    pals[3, 200:210] = pals[3, 3]
    pals[3, 100:110, :3] = px[500:510, :3]
    pals[3, 240:250, :3] = px[500:510, :3]
    return px, pals, w


def test_adversarial_argmin_matches_reference_kernels(gpu, refk, filt):
    """The argmin's decision boundaries on the reference's own distance()
    (CL:179-192, compiled for gfx950: fma-chain d^2, v_sqrt_f32): pixels on
    level-2 cell faces and one ulp either side, mirrored pairs (exact ties: the
    lower index wins), one-ulp pairs (ties that v_sqrt_f32 forms between
    different d^2), duplicates, pixel-equal colours and pixels one subnormal
    ulp from a colour (the rescaled form).  libhq's chosen colours (pruned grid
    and exhaustive) equal the reference quantize kernel's bit for bit, and the
    used flags too."""
    px, pals, w = _adversarial()
    for g in (32, 0):
        m = _ctx(gpu, px, np.zeros_like(px), w, filt.illum, grid=g)
        _, used = m.computeQuantizationErrorPopulation(pals.reshape(4, -1), 2.0, return_used=True)
        idx = [m.getIndices(p) for p in range(4)]
        m.close()
        for p in range(4):
            q, qu = refk.quantize(px, pals[p])
            np.testing.assert_array_equal(pals[p][idx[p]], q, err_msg=f"grid {g} palette {p}")
            np.testing.assert_array_equal(used[p] > 0, qu != 0, err_msg=f"grid {g} palette {p}")


def test_oracles_match_reference_argmin(gpu, refk):
    """The two oracles' argmin (hq_oracle.c and oracle.py, with the device's
    v_sqrt_f32 installed by the gpu fixture) against the reference's quantize
    kernel on the adversarial palettes: identical choices.  With the correctly
    rounded sqrt instead, the oracles split some of the ties v_sqrt_f32 forms."""
    import hw_sqrt

    px, pals, _ = _adversarial()
    calls0 = c_oracle.sqrt_calls()
    for p in range(4):
        q, _ = refk.quantize(px, pals[p])
        ci, _ = c_oracle.assign(px, pals[p])
        ni, _ = o.assign(px[:, :3], pals[p])
        np.testing.assert_array_equal(pals[p][ci], q, err_msg=f"C oracle, palette {p}")
        np.testing.assert_array_equal(pals[p][ni], q, err_msg=f"numpy oracle, palette {p}")
    assert c_oracle.sqrt_calls() > calls0  # the near ties went through v_sqrt_f32
    hw_sqrt.uninstall()
    try:
        diff = sum(int(np.any(pals[p][c_oracle.assign(px, pals[p])[0]] != refk.quantize(px, pals[p])[0], axis=1).sum())
                   for p in range(4))
    finally:
        hw_sqrt.install()
    assert diff > 0


def test_hw_sqrt_monotone_within_one_ulp(gpu):
    """The properties the argmin's re-resolution window rests on: v_sqrt_f32 is
    monotone and within 1 ulp of the correctly rounded root (a stride-61 sample
    of the normal floats plus runs of consecutive ones; the exhaustive count is
    in profiles/r06_sqrt_probe.json), and not correctly rounded (0x00806001)."""
    import hw_sqrt

    bits = np.concatenate([np.arange(0x00800000, 0x7F800000, 61, dtype=np.uint32),
                           np.arange(0x3F800000, 0x3F800000 + 200000, dtype=np.uint32),
                           np.arange(0x00806001, 0x00806001 + 4096, dtype=np.uint32)])
    x = bits.view(np.float32)
    y = hw_sqrt.sqrt_n(x)
    cr = np.sqrt(x.astype(np.float64)).astype(np.float32)  # double sqrt rounded to fp32: correctly rounded
    ulps = np.abs(y.view(np.int32).astype(np.int64) - cr.view(np.int32).astype(np.int64))
    assert ulps.max() <= 1
    assert 0.05 < np.mean(ulps) < 0.3
    order = np.argsort(bits, kind="stable")
    assert np.all(np.diff(y[order]) >= 0)
    assert y[bits == 0x00806001][0].view(np.uint32) == 0x20002FF7


def test_config3_4096_matches_reference_kernels(gpu, refk, filt):
    """BASELINE config 3's shape (4096^2, K = 256) through the reference's kernels:
    LabRef, two palettes' costs and used flags, and palette 0's chosen colour for
    every one of the 16.8 M pixels."""
    w = h = 4096
    R, G, B = o.synthetic_image(w, h, seed=1)
    rgba = o.inline_rgba(R, G, B)
    lab = refk.srgb_to_scielab(R, G, B, filt, w)
    pals = np.stack([o.synthetic_palette(256, 2 + p) for p in range(2)])
    rc, ru = refk.eval_population(rgba, lab, w, pals, filt)
    m = _ctx(gpu, rgba, None, w, filt.illum)
    np.testing.assert_allclose(m.getLabRef().reshape(-1, 4)[:, :3], lab[:, :3], atol=2e-4)
    m.close()
    m = _ctx(gpu, rgba, lab, w, filt.illum)
    costs, used = m.computeQuantizationErrorPopulation(pals.reshape(2, -1), 2.0, return_used=True)
    idx0 = m.getIndices(0)
    m.close()
    np.testing.assert_allclose(costs, rc, rtol=1e-6)
    np.testing.assert_array_equal(used > 0, ru != 0)
    q, _ = refk.quantize(rgba, pals[0])
    np.testing.assert_array_equal(pals[0][idx0], q)


@pytest.mark.parametrize("name,size,K,P,dpi,dist", [("C3", 4096, 256, 4, 72, 45.0), ("C1", 256, 16, 4, 72, 45.0),
                                                     ("C2", 1024, 64, 1, 72, 45.0), ("C5", 4096, 256, 64, 72, 45.0),
                                                     ("C3 at 96 dpi / 60 cm", 4096, 256, 4, 96, 60.0)])
def test_reference_kernels_timed_against_libhq(gpu, refk, name, size, K, P, dpi, dist):
    """The reference's own population evaluation on this MI355X (its five kernels per
    member, IM:620-727) beside libhq's, at the BASELINE configs' shapes: the same
    work, the same inputs.  libhq's population (one call through the C ABI, costs
    read back) must take less time than the reference's kernels alone.  With
    HQ_REFCL_TIMING_OUT set, one JSON line per config is appended there."""
    import json
    import time

    filt = o.design_filters(dpi, dist)
    w = h = size
    R, G, B = o.synthetic_image(w, h, seed=1)
    rgba = o.inline_rgba(R, G, B)
    lab = refk.srgb_to_scielab(R, G, B, filt, w)
    pals = np.stack([o.synthetic_palette(K, 2 + p) for p in range(P)])
    ref = refk.time_population(rgba, lab, w, pals, filt, reps=2 if P > 8 else 3)
    ref_kernels_ms = P * sum(ref["kernel_ms"].values())
    m = _ctx(gpu, rgba, lab, w, filt.illum, dpi=dpi, dist=dist)
    flat = pals.reshape(P, -1)
    m.computeQuantizationErrorPopulation(flat, 2.0)
    reps = 5 if P > 8 else 20
    t0 = time.perf_counter()
    for _ in range(reps):
        m.computeQuantizationErrorPopulation(flat, 2.0)
    hq_ms = 1e3 * (time.perf_counter() - t0) / reps
    m.close()
    px_evals = w * h * P
    out = {
        "config": {"workload": f"{name} population evaluation", "size": w, "K": K, "P": P, "dpi": dpi,
                   "distance_cm": dist, "halfSize": filt.half},
        "reference_opencl_on_mi355x": {
            "wall_ms_per_population": ref["wall_ms"],
            "kernel_ms_per_member": ref["kernel_ms"],
            "kernels_ms_per_population": ref_kernels_ms,
            "mpx_evals_per_s_kernels": px_evals / ref_kernels_ms / 1e3,
            "mpx_evals_per_s_wall": px_evals / ref["wall_ms"] / 1e3,
        },
        "libhq": {"ms_per_population": hq_ms, "mpx_evals_per_s": px_evals / hq_ms / 1e3,
                  "note": "one hq_eval_population call through the C ABI, costs read back (host API)"},
        "speedup_vs_reference_kernels": ref_kernels_ms / hq_ms,
        "speedup_vs_reference_wall": ref["wall_ms"] / hq_ms,
    }
    path = os.environ.get("HQ_REFCL_TIMING_OUT")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(out) + "\n")
    print(json.dumps(out))
    assert hq_ms < ref["wall_ms"], out
    # (under a kernel-trace profiler the OpenCL event timestamps are not the
    # kernels' own: only a kernel time that is a plausible share of the wall
    # time is held to this)
    if ref_kernels_ms > 0.05 * ref["wall_ms"]:
        assert hq_ms < ref_kernels_ms, out


@pytest.mark.parametrize("w,h,dpi,dist", [(256, 256, 72, 45.0), (193, 131, 96, 60.0)])
def test_de94_matches_reference_kernels(gpu, refk, w, h, dpi, dist):
    """dE94 (CL:217-226) against the reference's -DCIE94 build (IM:63): per pixel
    and per palette.  Its dH = sqrt(fma(da, da, db db) - dC dC) has no clamp,
    so a pixel whose hue difference is within rounding of 0 is NaN, and which
    pixels those are depends on the last bits of each side's Lab: a NaN pixel on
    either side must have a float64 dH^2 within rounding of 0; every other pixel
    agrees within 3e-4; a cost is NaN exactly when one of its pixels is; used
    flags bit-exact."""
    from test_gpu import _de94_exact, exact_pixel_err

    f = o.design_filters(dpi, dist)
    R, G, B = o.synthetic_image(w, h, seed=w + dpi)
    rgba = o.inline_rgba(R, G, B)
    lab = refk.srgb_to_scielab(R, G, B, f, w)
    pals = np.stack([o.synthetic_palette(64, 70 + p) for p in range(2)])
    refk.use("cie94")
    try:
        rc, ru, re = refk.eval_population(rgba, lab, w, pals, f, return_err=True)
    finally:
        refk.use("cie76")
    m = hq.ImageManipulation(hq.deltaETypes.CIE94, device=gpu)
    hq.ScielabProcessor(dpi, dist, hq.Whitepoint.D65, None, m)
    m.setOption("pixel_err", 1)
    m.setImage(rgba.reshape(-1), lab.reshape(-1), w, f.illum)
    costs, used = m.computeQuantizationErrorPopulation(pals.reshape(2, -1), 2.0, return_used=True)
    errs = [m.getPixelErrors(p) for p in range(2)]
    idxs = [m.getIndices(p) for p in range(2)]
    m.close()
    np.testing.assert_array_equal(used > 0, ru != 0)
    n_nan = 0
    for p in range(2):
        err, ref = errs[p], re[p]
        _, dH2, dab2 = _de94_exact(lab, exact_pixel_err(idxs[p], pals[p], lab, f, w, h, lab_only=True))
        near0 = np.abs(dH2) <= 1e-3 * (np.sqrt(dab2) + 1.0)
        nan_g, nan_r = np.isnan(err), np.isnan(ref)
        assert near0[nan_g].all() and near0[nan_r].all()
        ok = ~(nan_g | nan_r)
        assert np.abs(err[ok] - ref[ok]).max() <= PIX_ATOL
        assert np.isnan(costs[p]) == bool(nan_g.any()) and np.isnan(rc[p]) == bool(nan_r.any())
        if not (nan_g.any() or nan_r.any()):
            assert abs(costs[p] - rc[p]) <= 1e-6 * rc[p]
        n_nan += int(nan_g.sum() + nan_r.sum())
    print(f"dE94 {w}x{h} {dpi}/{dist}: NaN pixels (libhq + reference) {n_nan}")


def test_quantize_and_compute_error_match_reference_kernels(gpu, refk, filt):
    """The plugin's last two calls (HQ:93-137): quantize (IM:770-798, CL:147-170)
    with pixels and colours whose .w is not 0 -- the reference's distance() then
    takes the w term too, and the chosen colour is copied whole -- and
    computeError (IM:858-894: CIEDE between the original's and the quantized
    image's S-CIELAB, the host's error image and mean).  Chosen colours and used
    flags bit-exact; the mean within 1e-6 relative, the error image within 1e-5."""
    w, h, K = 211, 157, 64
    rng = np.random.default_rng(31)
    R, G, B = o.synthetic_image(w, h, seed=5)
    rgba = o.inline_rgba(R, G, B)
    rgba[:, 3] = rng.random(w * h, dtype=np.float32)
    pal = o.synthetic_palette(K, 9)
    pal[:, 3] = rng.random(K, dtype=np.float32)
    m = hq.ImageManipulation(device=gpu)
    q = m.quantize(rgba.reshape(-1), pal.reshape(-1)).reshape(-1, 4)
    used = m.lastUsedColors.copy()
    rq, ru = refk.quantize(rgba, pal)
    np.testing.assert_array_equal(q, rq)
    np.testing.assert_array_equal(used != 0, ru != 0)
    lab0 = refk.srgb_to_scielab(R, G, B, filt, w)
    lab1 = refk.srgb_to_scielab(rq[:, 0], rq[:, 1], rq[:, 2], filt, w)
    img = np.zeros(4 * w * h, np.float32)
    mean = m.computeError(lab0.reshape(-1), lab1.reshape(-1), img)
    m.close()
    rimg = np.zeros(4 * w * h, np.float32)
    rmean, _ = refk.compute_error(lab0, lab1, rimg)
    assert abs(mean - rmean) <= 1e-6 * rmean
    np.testing.assert_allclose(img.reshape(-1, 4)[:, :3], rimg.reshape(-1, 4)[:, :3], rtol=0, atol=1e-5)


@pytest.mark.parametrize("w,h,K,P,imax,seed,t0", [(96, 64, 16, 3, 40, 77, 0.5), (128, 96, 32, 4, 150, 5, 0.05)])
def test_search_on_reference_kernels_matches_device_search(gpu, refk, filt, w, h, K, P, imax, seed, t0):
    """The plugin's whole search (IM:383-591 with SW:14-116, restated by
    oracle.find_best_quantization and checked bit for bit against libhq's native
    driver by tests/test_capi.py) with every population evaluated by the
    reference's own kernels (IM:620-727) on the MI355X, against libhq's
    device-resident search (sa_step_kernel) on its own costs: the same best
    palette and error -- the costs agree to ~1e-7, so every acceptance
    decision is the same unless one lands within that of its threshold."""
    R, G, B = o.synthetic_image(w, h, seed=8)
    rgba = o.inline_rgba(R, G, B)
    lab = refk.srgb_to_scielab(R, G, B, filt, w)

    def ref_eval(ps):
        return list(refk.eval_population(rgba, lab, w, np.stack(ps), filt)[0])

    osw = o.Swasa(o.SwasaParams(population=P, imax=imax, t0=t0), seed)
    ob, oe = o.find_best_quantization(ref_eval, K, osw)
    m = _ctx(gpu, rgba, lab, w, filt.illum)
    m.setOption("sa_device", 1)
    sw = hq.SWASA(population=P, imax=imax, seed=seed, t0=t0)
    best = m.findBestQuantization(rgba.reshape(-1), lab.reshape(-1), w, K, sw, None, None, filt.illum)
    err = m.bestError
    m.close()
    assert abs(err - oe) <= 1e-6 * oe
    np.testing.assert_array_equal(np.asarray(best, np.float32).reshape(K, 4), ob)


def test_compute_error_de94_matches_reference_kernels(gpu, refk, filt):
    """computeError (IM:858-894) with dE94: the reference's -DCIE94 CIEDE kernel
    against libhq's.  Its unclamped dH (CL:222) is NaN where the hue difference
    is within rounding of 0; the two sides may disagree on which of those
    pixels turn NaN (last bits), so: the finite pixels agree within 1e-4, and
    NaN pixels are rare on both sides (< 2e-3) and the mean is NaN exactly when
    a pixel is."""
    w, h, K = 160, 120, 32
    R, G, B = o.synthetic_image(w, h, seed=12)
    rgba = o.inline_rgba(R, G, B)
    pal = o.synthetic_palette(K, 13)
    rq, _ = refk.quantize(rgba, pal)
    lab0 = refk.srgb_to_scielab(R, G, B, filt, w)
    lab1 = refk.srgb_to_scielab(rq[:, 0], rq[:, 1], rq[:, 2], filt, w)
    refk.use("cie94")
    try:
        rmean, rerr = refk.compute_error(lab0, lab1)
    finally:
        refk.use("cie76")
    m = hq.ImageManipulation(hq.deltaETypes.CIE94, device=gpu)
    img = np.zeros(4 * w * h, np.float32)
    mean = m.computeError(lab0.reshape(-1), lab1.reshape(-1), img)
    m.close()
    e = np.float32(255) - np.sqrt(img.reshape(-1, 4)[:, 0].astype(np.float64) * (255.0 * 255.0))  # back from (255 - e)^2 / 255^2
    nan_r = np.isnan(rerr)
    nan_g = np.isnan(img.reshape(-1, 4)[:, 0])
    assert nan_r.mean() < 2e-3 and nan_g.mean() < 2e-3
    ok = ~(nan_r | nan_g)
    assert np.abs(e[ok] - rerr[ok]).max() <= 1e-3
    assert np.isnan(mean) == bool(nan_g.any()) and np.isnan(rmean) == bool(nan_r.any())
    if not (nan_g.any() or nan_r.any()):
        assert abs(mean - rmean) <= 1e-6 * rmean
