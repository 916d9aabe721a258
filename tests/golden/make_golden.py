"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

Provenance: the reference (Java + JavaCL) holds no tests, fixtures or golden
vectors and its Java host cannot run in this container, so every
expected value here comes from the oracle's restatement of the reference
semantics (oracle/oracle.py, cross-checked against oracle/hq_oracle.c), with
the correctly rounded square root (oracle.ref_len).  The oracle is pinned
against the reference's own OpenCL kernels on the MI355X by tests/test_refcl.py
(GPU); the java.util.Random known answers in kat_java_random.json are published
outputs of the JDK class.

Run:  python tests/golden/make_golden.py
"""

from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import c_oracle  # noqa: E402
import oracle as o  # noqa: E402

FILTER_SETTINGS = [(72, 45.0, "D65"), (72, 45.0, "D50"), (96, 60.0, "D65"), (150, 30.0, "D65")]


def u8_image(w, h, seed):
    z = o.splitmix64(seed, w * h)
    return np.stack([(z >> np.uint64(8 * c)) & np.uint64(0xFF) for c in range(3)], axis=1).astype(np.uint8)


def from_u8(img):
    f = img.astype(np.float32) / np.float32(255.0)
    return f[:, 0].copy(), f[:, 1].copy(), f[:, 2].copy()


def filters():
    out = {}
    for dpi, vd, wp in FILTER_SETTINGS:
        f = o.design_filters(dpi, vd, wp)
        tag = f"{dpi}_{int(vd)}_{wp}"
        out[f"k1_{tag}"] = f.k1
        out[f"k2_{tag}"] = f.k2
        out[f"k3_{tag}"] = f.k3
        out[f"absk3_{tag}"] = f.absk3
        out[f"illum_{tag}"] = f.illum
    np.savez_compressed(os.path.join(HERE, "filters.npz"), **out)


def case(name, w, h, K, P, seed_img, store_full_idx=True):
    f = o.design_filters()
    img = u8_image(w, h, seed_img)
    R, G, B = from_u8(img)
    rgba = o.inline_rgba(R, G, B)
    lab = o.srgb_to_scielab(R, G, B, f, w)
    lab_c = c_oracle.srgb_to_scielab(R, G, B, f, w)
    assert np.abs(lab - lab_c).max() < 1e-3
    pals = np.stack([o.synthetic_palette(K, 2 + p) for p in range(P)])
    costs, err_sums, idxs, useds = [], [], [], []
    for p in range(P):
        c, parts = o.eval_palette(rgba[:, :3], lab, pals[p], f, w, return_parts=True)
        cc, pc = c_oracle.eval_palette(rgba, lab, pals[p], f, w, return_parts=True)
        assert np.array_equal(parts["idx"], pc["idx"])
        assert abs(c - cc) <= 1e-6 * abs(c)
        costs.append(c)
        err_sums.append(float(np.sum(parts["err"].astype(np.float64))))
        idxs.append(parts["idx"].astype(np.uint8))
        useds.append(parts["used"].astype(np.uint8))
    data = dict(w=np.int32(w), h=np.int32(h), K=np.int32(K), rgb_u8=img, palettes=pals,
                costs=np.array(costs), err_sums=np.array(err_sums), used=np.stack(useds),
                lab_checksum=np.abs(lab[:, :3].astype(np.float64)).sum(axis=0),
                lab_rows=lab[: 2 * w].copy())
    if store_full_idx:
        data["idx"] = np.stack(idxs)
        data["lab"] = lab
    else:
        data["idx0"] = idxs[0]
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **data)


def edge_cases():
    """Index-only edge cases (CL:179-193 semantics)."""
    rng = np.random.default_rng(7)
    n = 4096
    px = rng.random((n, 3), dtype=np.float32)
    px[:64] = rng.uniform(-0.5, 1.5, (64, 3)).astype(np.float32)  # outside [0,1]
    px[64:80] = np.float32(0.0)
    px[80:96] = np.float32(1.0)
    rgba = np.zeros((n, 4), np.float32)
    rgba[:, :3] = px
    cases = {}
    # duplicates: every colour repeated (lowest index must win)
    base = o.synthetic_palette(32, 11)
    dup = np.concatenate([base, base, base[::-1]], axis=0)[:96]
    # clamped colours (SW:96-98 produce exact 0/1 channels)
    clamped = o.synthetic_palette(64, 12)
    clamped[::3, 0] = 0.0
    clamped[1::3, 1] = 1.0
    clamped[2::5, :3] = 1.0
    # K = 1 and K = 256
    k1 = o.synthetic_palette(1, 13)
    k256 = o.synthetic_palette(256, 14)
    # equidistant ties: colours symmetric around pixel grid points
    ties = np.zeros((8, 4), np.float32)
    ties[:, :3] = np.array([[0.5 + dx, 0.5 + dy, 0.5 + dz] for dx in (-0.25, 0.25)
                            for dy in (-0.25, 0.25) for dz in (-0.25, 0.25)], np.float32)
    for name, pal in dict(dup=dup, clamped=clamped, k1=k1, k256=k256, ties=ties).items():
        idx, used = o.assign(px, pal)
        cidx, cused = c_oracle.assign(rgba, pal)
        assert np.array_equal(idx, cidx) and np.array_equal(used, cused)
        cases[f"pal_{name}"] = pal
        cases[f"idx_{name}"] = idx.astype(np.uint8)
    # tie pixels: grid points equidistant to several colours
    tie_px = np.full((8, 4), 0.5, np.float32)
    tie_px[:, 3] = 0
    cases["px"] = rgba
    np.savez_compressed(os.path.join(HERE, "edge_assign.npz"), **cases)


def swasa_trace():
    """Native-vs-oracle SWASA policy fixture with a synthetic deterministic cost."""
    def cost(pal):
        pal = np.asarray(pal, np.float32)[..., :3].astype(np.float64)
        return float(np.sum((pal - 0.3) ** 2) + 0.01 * np.sum(np.sin(pal * 17)))

    sw = o.Swasa(o.SwasaParams(population=4, imax=200), 1234)
    tr = []
    best, err = o.find_best_quantization(lambda ps: [cost(p) for p in ps], 8, sw, trace=tr)
    trace = np.array([[t[3]] + t[1] for t in tr])
    np.savez_compressed(os.path.join(HERE, "swasa_trace.npz"), best=best, best_error=err,
                        trace=trace, seed=1234, K=8, population=4, imax=200)


def java_random_kat():
    """Known outputs of java.util.Random (JDK), and the oracle's values for them."""
    kat = {
        "seed42_nextInt": -1170105035,      # new Random(42).nextInt()
        "seed0_nextInt": -1155484576,       # new Random(0).nextInt()
        "seed42_nextDouble": 0.7275636800328681,  # new Random(42).nextDouble()
    }
    r = o.JavaRandom(42)
    assert r.next(32) == kat["seed42_nextInt"]
    assert o.JavaRandom(0).next(32) == kat["seed0_nextInt"]
    assert o.JavaRandom(42).next_double() == kat["seed42_nextDouble"]
    seq = o.JavaRandom(1234)
    kat["seed1234_nextFloat_x8"] = [float(seq.next_float()) for _ in range(8)]
    with open(os.path.join(HERE, "kat_java_random.json"), "w") as fh:
        json.dump(kat, fh, indent=1)


if __name__ == "__main__":
    c_oracle.build()
    filters()
    case("case_64x48_k16", 64, 48, 16, 2, seed_img=1)
    case("case_256_k16", 256, 256, 16, 4, seed_img=5, store_full_idx=False)
    case("case_97x53_k64", 97, 53, 64, 2, seed_img=9)
    edge_cases()
    swasa_trace()
    java_random_kat()
    print("golden fixtures written to", HERE)
