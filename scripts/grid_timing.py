"""Diagnostic: per-workgroup start/end stamps of build_grid (a library built with
-DHQ_GRID_TIMING, HQ_LIB_PATH; stamps kept in device memory, read back by
hq_debug_grid_stamps) over a few 4096^2 / K=256 / P=4 evaluations; prints the
dispatch spread and the workgroup durations of the last one."""
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
    R, G, B = bench.synthetic_planes(W, W)
    _lib.check(lib.hq_set_image_planar_shard(m.ctx, _lib.fptr(R), _lib.fptr(G), _lib.fptr(B), W, W,
                                             _lib.fptr(sp.illuminant), 0, W), m.ctx)
    rng = np.random.default_rng(1)
    for it in range(3):
        pal = rng.random((4, 256, 4), dtype=np.float32)
        pal[..., 3] = 0
        m.computeQuantizationErrorPopulation(pal.reshape(4, -1), 2.0)
    import ctypes as C
    n = 4 * 512
    buf = np.zeros((n, 8), np.uint64)
    lib.hq_debug_grid_stamps.argtypes = [C.c_void_p, C.c_int]
    lib.hq_debug_grid_stamps(buf.ctypes.data, n)
    m.close()
    for i, r in enumerate(buf):
        print("GRID_T %d %d %s" % (i // 512, i % 512, " ".join(str(int(x)) for x in r)))
    sys.exit(0)
res = subprocess.run([sys.executable, __file__, "run"], capture_output=True, text=True, timeout=300)
last = [l.split() for l in res.stdout.splitlines() if l.startswith("GRID_T")]
if not last:
    sys.exit("no stamps:\n" + res.stderr[-2000:])
st = [int(x[3]) for x in last]
en = [int(x[4]) for x in last]
t0 = min(st)
durs = sorted((e - s) / 100.0 for s, e in zip(st, en))  # 100 MHz ticks -> us
starts = sorted((s - t0) / 100.0 for s in st)
print(f"{len(last)} workgroups; start spread {starts[-1]:.2f} us (50% by {starts[len(starts)//2]:.2f}); "
      f"end {max((e - t0) / 100.0 for e in en):.2f} us")
print("duration us: min %.2f med %.2f p90 %.2f max %.2f" % (durs[0], durs[len(durs) // 2],
                                                           durs[int(len(durs) * 0.9)], durs[-1]))
# phases (stamps 2..6: level-1 list, pass 1, pass 2, dominance, long lists) of the
# slowest 5% of workgroups against the median ones, and their level-1 list lengths
rows = []
for x in last:
    v = [int(t) for t in x[3:11]]
    if len(v) < 8 or v[6] == 0:
        continue
    ph = [(v[2] - v[0]) / 100.0, (v[3] - v[2]) / 100.0, (v[4] - v[3]) / 100.0, (v[5] - v[4]) / 100.0,
          (v[6] - v[5]) / 100.0, (v[1] - v[6]) / 100.0]
    rows.append(((v[1] - v[0]) / 100.0, ph, v[7] & 0xFFFF, v[7] >> 16))
rows.sort(key=lambda r: r[0])
if rows:
    def summ(sel, name):
        import statistics as st
        print(f"{name} ({len(sel)} wg): dur {st.mean(r[0] for r in sel):.2f} us; phases l1/pass1/pass2/dom/long/tail "
              + " ".join(f"{st.mean(r[1][k] for r in sel):.2f}" for k in range(6))
              + f"; level-1 list {st.mean(r[2] for r in sel):.1f}; long lists {st.mean(r[3] for r in sel):.2f}")
    n = len(rows)
    summ(rows[int(n * 0.45):int(n * 0.55)], "median")
    summ(rows[int(n * 0.95):], "slowest 5%")
