"""Profiling driver: repeated population evaluations at a given size (for rocprofv3).

python scripts/profile_eval.py [--size 4096] [--K 256] [--P 4] [--evals 10] [--opt NAME=VALUE ...]
Prints per-kernel HIP-event averages and the end-to-end eval time.
"""

import argparse
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import hybridquantization_amd as hq  # noqa: E402
from hybridquantization_amd import _lib  # noqa: E402
from bench import synthetic_planes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--K", type=int, default=256)
    ap.add_argument("--P", type=int, default=4)
    ap.add_argument("--evals", type=int, default=10)
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="libhq option (include/hq.h hq_set_option), repeatable")
    ap.add_argument("--rows", type=int, default=0,
                    help="evaluate only the row shard [0, rows) of the image (an N-GPU rank's share)")
    ap.add_argument("--lib", default=None, help="alternative libhq build (scripts/ablate.py)")
    args = ap.parse_args()
    if args.lib:
        _lib.LIB_PATH = os.path.abspath(args.lib)
    lib = hq.load()
    m = hq.ImageManipulation(device=0)
    sp = hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    for kv in args.opt:
        k, v = kv.split("=", 1)
        m.setOption(k, int(v))
    W = H = args.size
    R, G, B = synthetic_planes(W, H, 1)
    rows = args.rows or H
    _lib.check(lib.hq_set_image_planar_shard(m.ctx, _lib.fptr(R), _lib.fptr(G), _lib.fptr(B), W, H,
                                             _lib.fptr(sp.illuminant), 0, rows), m.ctx)
    rng = np.random.default_rng(0)
    pals = np.zeros((args.P, args.K, 4), np.float32)
    pals[..., :3] = rng.random((args.P, args.K, 3), dtype=np.float32)
    costs = np.zeros(args.P)
    flat = pals.reshape(-1)
    part = np.zeros(args.P * (1 + args.K))
    if rows < H:  # a shard without a communicator: partial sums
        def evaluate():
            _lib.check(lib.hq_eval_population_partial(m.ctx, _lib.fptr(flat), args.P, args.K,
                                                      _lib.dptr(part)), m.ctx)
    else:
        def evaluate():
            _lib.check(lib.hq_eval_population(m.ctx, _lib.fptr(flat), args.P, args.K, 2.0,
                                              _lib.dptr(costs), None), m.ctx)
    evaluate()
    phases = getattr(lib, "hq_debug_phases", None) if args.lib else None
    ph = (C.c_ulonglong * 8)()
    if phases is not None:
        phases(ph, 1)
    lib.hq_profile_enable(m.ctx, 1)
    t0 = time.perf_counter()
    for _ in range(args.evals):
        evaluate()
    el = time.perf_counter() - t0
    out = []
    for k in ("grid", "assign", "cost", "finalize"):
        ms = C.c_double()
        n = C.c_int64()
        lib.hq_profile_get(m.ctx, k.encode(), C.byref(ms), C.byref(n))
        out.append(f"{k}={ms.value / max(n.value, 1):.4f}ms")
    print(f"{os.path.basename(args.lib or 'libhq.so')} size={W} K={args.K} P={args.P} opts={args.opt}: "
          f"{el / args.evals * 1e3:.3f} ms/eval-population, "
          f"{W * rows * args.P * args.evals / el / 1e6:.1f} Mpx*evals/s (rows {rows})  ", " ".join(out),
          "costs", costs.tolist())
    if phases is not None:
        phases(ph, 0)
        n = max(ph[7], 1)
        names = ["prologue", "barrier1", "vpass", "barrier2", "hpass+lab", "reduce"]
        print("per-wave cycles:", " ".join(f"{nm}={ph[i] / n:.0f}" for i, nm in enumerate(names)),
              f"waves={ph[7]}")
    m.close()


if __name__ == "__main__":
    main()
