"""Diagnostic: per-workgroup stamps of assign_pipe_kernel (a library built with
-DHQ_ASSIGN_TIMING, HQ_LIB_PATH) over a few evaluations at GT_SIZE^2 (rows
GT_ROWS of it, default all), K = 256, P = GT_P: the dispatch spread, the time
to the table fill barrier, the pixel loop and the end, of the last evaluation."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "run":
    sys.path.insert(0, ROOT)
    import numpy as np
    import bench
    import hybridquantization_amd as hq
    from hybridquantization_amd import _lib
    lib = hq.load()
    m = hq.ImageManipulation(device=0)
    sp = hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    W = int(os.environ.get("GT_SIZE", "4096"))
    rows = int(os.environ.get("GT_ROWS", str(W)))
    P = int(os.environ.get("GT_P", "4"))
    R, G, B = bench.synthetic_planes(W, W)
    _lib.check(lib.hq_set_image_planar_shard(m.ctx, _lib.fptr(R), _lib.fptr(G), _lib.fptr(B), W, W,
                                             _lib.fptr(sp.illuminant), 0, rows), m.ctx)
    rng = np.random.default_rng(1)
    for it in range(3):
        pal = rng.random((P, 256, 4), dtype=np.float32)
        pal[..., 3] = 0
        print("EVAL", it, flush=True)
        m.computeQuantizationErrorPopulation(pal.reshape(P, -1), 2.0)
    m.close()
    sys.exit(0)
out = subprocess.run([sys.executable, __file__, "run"], capture_output=True, text=True, timeout=300).stdout
last = [l.split() for l in out.split("EVAL")[-1].splitlines() if l.startswith("ASG_T")]
st, fi, lo, en = ([int(x[k]) for x in last] for k in (3, 4, 5, 6))
t0 = min(st)


def q(v):
    v = sorted(v)
    return "min %.2f med %.2f p90 %.2f max %.2f" % (v[0], v[len(v) // 2], v[int(len(v) * 0.9)], v[-1])


print(f"{len(last)} workgroups; end of the last {(max(en) - t0) / 100:.2f} us after the first start")
print("start     ", q([(s - t0) / 100 for s in st]))
print("to fill   ", q([(f - s) / 100 for s, f in zip(st, fi)]))
print("loop      ", q([(l - f) / 100 for f, l in zip(fi, lo)]))
print("flush     ", q([(e - l) / 100 for l, e in zip(lo, en)]))
print("end       ", q([(e - t0) / 100 for e in en]))
