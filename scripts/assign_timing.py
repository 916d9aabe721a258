"""Diagnostic: per-workgroup stamps of assign_pipe_kernel (a library built with
-DHQ_ASSIGN_TIMING, HQ_LIB_PATH; stamps kept in device memory, read back by
hq_debug_assign_stamps) over a few evaluations at GT_SIZE^2 (rows GT_ROWS of
it, default all), K = 256, P = GT_P: the dispatch spread, the time to the table
fill barrier, the pixel loop and the end, of the last evaluation."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "run":
    sys.path.insert(0, ROOT)
    import ctypes as C
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
        if rows < W:  # a row-block shard: the partial evaluation (no communicator)
            part = np.zeros(P * 257, np.float64)
            _lib.check(lib.hq_eval_population_partial(m.ctx, _lib.fptr(pal.reshape(-1)), P, 256,
                                                      _lib.dptr(part)), m.ctx)
        else:
            m.computeQuantizationErrorPopulation(pal.reshape(P, -1), 2.0)
    slow = np.zeros(2, np.uint32)
    lib.hq_debug_assign_slow.argtypes = [C.c_void_p]
    lib.hq_debug_assign_slow(slow.ctypes.data)
    print("SLOW %d %d" % (int(slow[0]), int(slow[1])))
    buf = np.zeros((16384, 8), np.uint64)
    lib.hq_debug_assign_stamps.argtypes = [C.c_void_p, C.c_int]
    lib.hq_debug_assign_stamps(buf.ctypes.data, 16384)
    m.close()
    n = int((buf[:, 2] > 0).sum())
    for r in buf[:n]:
        print("ASG_T 0 0 " + " ".join(str(int(x)) for x in r))
    sys.exit(0)
res = subprocess.run([sys.executable, __file__, "run"], capture_output=True, text=True, timeout=300)
last = [l.split() for l in res.stdout.splitlines() if l.startswith("ASG_T")]
if not last:
    sys.exit("no stamps:\n" + res.stderr[-2000:])
st, fi, en = ([int(x[k]) for x in last] for k in (3, 4, 5))
wr = [[int(x[k]) for k in (6, 7, 8, 9)] for x in last]  # each wave's loop end (0: not stamped)
wl = [[y for y in w if y] for w in wr]
t0 = min(st)


def q(v):
    v = sorted(v)
    return "min %.2f med %.2f p90 %.2f max %.2f" % (v[0], v[len(v) // 2], v[int(len(v) * 0.9)], v[-1])


sl = [l for l in res.stdout.splitlines() if l.startswith("SLOW")]
if sl:
    print("lanes re-resolved over the 3 evaluations: near ties %s, overflow or no list %s" % tuple(sl[0].split()[1:]))
print(f"{len(last)} workgroups; end of the last {(max(en) - t0) / 100:.2f} us after the first start")
print("start            ", q([(s - t0) / 100 for s in st]))
print("to fill          ", q([(f - s) / 100 for s, f in zip(st, fi)]))
print("wave loops       ", q([(x - f) / 100 for f, w in zip(fi, wl) for x in w]))
print("wave spread in wg", q([(max(w) - min(w)) / 100 for w in wl if w]))
print("end              ", q([(e - t0) / 100 for e in en]))
n = len(last)
per_x = n // 8
for x in range(8):  # XCD x holds workgroups [x n/8, (x+1) n/8) after xcd_remap
    sl = range(x * per_x, (x + 1) * per_x)
    print(f"xcd {x}: wave loops", q([(y - fi[i]) / 100 for i in sl for y in wl[i]]),
          " end", q([(en[i] - t0) / 100 for i in sl]))
for k in range(4):  # wave index in the workgroup
    v = [(wr[i][k] - fi[i]) / 100 for i in range(n) if wr[i][k]]
    print(f"wave {k}: {len(v)} stamped", q(v) if v else "")
# by dispatch order within an XCD (position s of the workgroup in its XCD's range)
for part in range(4):
    sl = [i for i in range(n) if (i % per_x) * 4 // per_x == part]
    print(f"dispatch quarter {part}:", q([(y - fi[i]) / 100 for i in sl for y in wl[i]]))
