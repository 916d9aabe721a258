"""CPU tests of the C ABI library: it loads, exports every symbol declared in
include/hq.h, and its host-only parts (filter design, SWASA driver) agree with
the oracle.  No compute call here touches a GPU."""

import ctypes
import os
import re

import numpy as np
import pytest

import hybridquantization_amd as hq
import oracle as o
from hybridquantization_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def header_symbols():
    src = open(os.path.join(ROOT, "include", "hq.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(hq_[a-z0-9_]+)\s*\(", src))
    names.discard("hq_eval_fn")
    return sorted(names)


def test_library_exports_every_header_symbol():
    lib = hq.load()
    syms = header_symbols()
    assert len(syms) >= 30
    for name in syms:
        assert hasattr(lib, name), name
    # the ctypes signature table covers exactly the header surface
    assert set(_lib.SIGNATURES) == set(syms)


def test_status_and_version():
    lib = hq.load()
    assert lib.hq_version() == 1
    assert lib.hq_status_string(0) == b"ok"
    n = ctypes.c_int(-1)
    assert lib.hq_device_count(ctypes.byref(n)) == 0 and n.value >= 0


@pytest.mark.parametrize("dpi,vd,wp", [(72, 45.0, "D65"), (72, 45.0, "D50"), (96, 60.0, "D65"),
                                       (150, 30.0, "D65")])
def test_design_filters_bitexact_with_oracle(dpi, vd, wp):
    k1, k2, k3, ak3, il = hq.design_filters(dpi, vd, hq.Whitepoint.D50 if wp == "D50" else hq.Whitepoint.D65)
    g = np.load(os.path.join(GOLD, "filters.npz"))
    tag = f"{dpi}_{int(vd)}_{wp}"
    np.testing.assert_array_equal(k1, g[f"k1_{tag}"])
    np.testing.assert_array_equal(k2, g[f"k2_{tag}"])
    np.testing.assert_array_equal(k3, g[f"k3_{tag}"])
    np.testing.assert_array_equal(ak3, g[f"absk3_{tag}"])
    np.testing.assert_array_equal(il, g[f"illum_{tag}"])


def test_design_filters_rejects_bad_args():
    lib = hq.load()
    buf = np.zeros(64, np.float32)
    taps = ctypes.c_int()
    p = _lib.fptr(buf)
    assert lib.hq_design_filters(0, 45.0, 1, 16, p, p, p, p, ctypes.byref(taps), p) == _lib.HQ_ERR_ARG
    # 300 dpi at 100 cm needs 205 taps: too many for a 16-tap buffer
    assert lib.hq_design_filters(300, 100.0, 1, 16, p, p, p, p, ctypes.byref(taps), p) == \
        _lib.HQ_ERR_UNSUPPORTED
    assert taps.value == 205


def _cost(pal):
    pal = np.asarray(pal, np.float32)[..., :3].astype(np.float64)
    return float(np.sum((pal - 0.3) ** 2) + 0.01 * np.sum(np.sin(pal * 17)))


def test_native_swasa_driver_matches_golden_trace():
    g = np.load(os.path.join(GOLD, "swasa_trace.npz"))
    sw = hq.SWASA(population=int(g["population"]), imax=int(g["imax"]), seed=int(g["seed"]))
    best, err, trace = sw.search_host(int(g["K"]), lambda ps: [_cost(p) for p in ps])
    np.testing.assert_array_equal(trace, g["trace"])
    np.testing.assert_array_equal(best.reshape(-1, 4), g["best"])
    assert err == float(g["best_error"])


@pytest.mark.parametrize("P,conv,K", [(1, True, 4), (3, False, 8), (6, True, 3)])
def test_native_swasa_driver_matches_oracle(P, conv, K):
    sw = hq.SWASA(population=P, imax=150, seed=99 + P, convergence=conv, t0=0.05, iTc=7)
    best, err, trace = sw.search_host(K, lambda ps: [_cost(p) for p in ps])
    osw = o.Swasa(o.SwasaParams(population=P, imax=150, convergence=conv, t0=0.05, iTc=7), 99 + P)
    tr = []
    ob, oe = o.find_best_quantization(lambda ps: [_cost(p) for p in ps], K, osw, trace=tr)
    np.testing.assert_array_equal(trace, np.array([[t[3]] + t[1] for t in tr]))
    np.testing.assert_array_equal(best.reshape(K, 4), ob)
    assert err == oe


def test_swasa_driver_propagates_evaluator_errors():
    sw = hq.SWASA(population=2, imax=10, seed=1)

    def bad(ps):
        raise ValueError("boom")

    with pytest.raises(ValueError):
        sw.search_host(4, bad)


def test_no_gpu_means_unavailable_not_silent():
    n = ctypes.c_int(0)
    hq.load().hq_device_count(ctypes.byref(n))
    if n.value > 0:
        pytest.skip("a GPU is present")
    ip = hq.ImageManipulation()
    assert ip.getOpenCLAvailable() is False  # IM:79-92 condition
    with pytest.raises(hq.HQUnavailable):
        ip.RGBtoXYZ(np.zeros(4, np.float32), np.zeros(4, np.float32), np.zeros(4, np.float32))


def test_pack_filters_matches_im800():
    f = o.design_filters()
    k1, k2, k3, ak3 = hq.pack_filters(f.ofilters, f.absk3)
    np.testing.assert_array_equal(k1, f.k1)
    np.testing.assert_array_equal(k2, f.k2)
    np.testing.assert_array_equal(k3, f.k3)
    np.testing.assert_array_equal(ak3, f.absk3)


CSRC = os.path.join(ROOT, "hybridquantization_amd", "csrc")


def test_every_ablation_switch_is_guarded():
    """Every HQ_ABL_* name used in the kernel sources is in hq_device.h's
    #error guard, so no ablation (wrong results by design) builds by accident."""
    guard = open(os.path.join(CSRC, "hq_device.h")).read()
    guard = guard[guard.index("#if !defined(HQ_ABLATION_BUILD)"):guard.index("#error")]
    listed = set(re.findall(r"defined\((HQ_ABL_\w+)\)", guard))
    used = set()
    for f in os.listdir(CSRC):
        if f.endswith((".hip", ".h", ".cpp")) and f != "hq_device.h":
            used |= set(re.findall(r"\b(HQ_ABL_\w+)", open(os.path.join(CSRC, f)).read()))
    assert used, "no ablation switches found (the scan is broken)"
    assert used <= listed, sorted(used - listed)


def test_ablation_define_without_opt_in_fails_to_compile():
    """A stray -DHQ_ABL_* (without HQ_ABLATION_BUILD) stops the build."""
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    cmd = [hipcc, "--offload-arch=gfx950", "-std=c++17", "-E", "-o", os.devnull, os.path.join(CSRC, "hq_wide.hip")]
    assert subprocess.run(cmd, capture_output=True).returncode == 0
    bad = subprocess.run(cmd + ["-DHQ_ABL_NOFILL"], capture_output=True, text=True)
    assert bad.returncode != 0 and "HQ_ABLATION_BUILD" in bad.stderr
    assert subprocess.run(cmd + ["-DHQ_ABL_NOFILL", "-DHQ_ABLATION_BUILD"], capture_output=True).returncode == 0
