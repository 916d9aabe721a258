"""Multi-process libhq (GPU): two processes, each with its own hq_ctx on device 0
owning half the rows (hq_set_image_planar_shard), exchange their partials over
gloo and must reproduce the single-context full evaluation.  The control path
is the one bench.py runs at N > 1 (hybridquantization_amd.dist: shard bounds,
unique-id broadcast, MAX over ranks); two ranks cannot share one GPU in RCCL,
so the fp64 partials are all-reduced over gloo instead of libhq's ncclAllReduce.
"""

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

W, H, K, P = 160, 131, 48, 3


def _inputs():
    import oracle as o

    R, G, B = o.synthetic_image(W, H, seed=31)
    pals = np.stack([o.synthetic_palette(K, 90 + p) for p in range(P)]).reshape(P, -1)
    return R, G, B, pals


def _context(R, G, B, r0, r1):
    import hybridquantization_amd as hq

    m = hq.ImageManipulation(device=0)
    sp = hq.ScielabProcessor(72, 45.0, hq.Whitepoint.D65, None, m)
    lib = hq.load()
    hq._lib.check(lib.hq_set_image_planar_shard(m.ctx, hq._lib.fptr(R), hq._lib.fptr(G),
                                                hq._lib.fptr(B), W, H,
                                                hq._lib.fptr(sp.illuminant), r0, r1), m.ctx)
    return m, lib


def _worker(rank, world, port, out):
    import sys
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "oracle")]
    import torch.distributed as dist

    import hybridquantization_amd as hq
    from hybridquantization_amd import dist as hqd

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t0 = time.perf_counter()
    R, G, B, pals = _inputs()
    r0, r1 = hqd.shard_rows(H, world, rank)
    m, lib = _context(R, G, B, r0, r1)
    part = np.zeros(P * (1 + K))
    hq._lib.check(lib.hq_eval_population_partial(m.ctx, hq._lib.fptr(pals), P, K,
                                                 hq._lib.dptr(part)), m.ctx)
    total = hqd.allreduce_partials(dist, part)
    uid = hqd.broadcast_unique_id(dist, rank, hq.ImageManipulation.commUniqueId)
    el = hqd.max_over_ranks(dist, time.perf_counter() - t0 + rank)  # rank 1 reports +1 s
    m.close()
    out.put((rank, total, uid, el, (r0, r1)))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_process_shards_allreduce_to_full(gpu):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=100) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # the control path: contiguous bounds, one unique id everywhere, one MAX
    assert [r[4] for r in res] == [(0, H // 2), (H // 2, H)]
    assert res[0][2] == res[1][2] and len(res[0][2]) == 128
    assert res[0][3] == res[1][3] and res[0][3] >= 1.0
    np.testing.assert_array_equal(res[0][1], res[1][1])
    total = res[0][1].reshape(P, 1 + K)

    import hybridquantization_amd as hq

    R, G, B, pals = _inputs()
    m, lib = _context(R, G, B, 0, H)
    ref = np.zeros(P * (1 + K))
    hq._lib.check(lib.hq_eval_population_partial(m.ctx, hq._lib.fptr(pals), P, K,
                                                 hq._lib.dptr(ref)), m.ctx)
    costs, used = m.computeQuantizationErrorPopulation(pals, 2.0, return_used=True)
    m.close()
    ref = ref.reshape(P, 1 + K)
    # H // 2 = 65 rows is not a multiple of the 16-row cost16w tile: the shards' tiles
    # group the pixels differently from the full image's, so the fp32 per-item
    # sums inside a tile round differently (~1e-9); aligned shards agree to 1e-9
    # (test_gpu.py::test_config4_8192_shards_sum_to_full)
    np.testing.assert_allclose(total[:, 0], ref[:, 0], rtol=1e-7)
    np.testing.assert_array_equal(total[:, 1:] > 0, ref[:, 1:] > 0)
    # the cost assembled from the all-reduced partials, as hq_eval_population does
    c = total[:, 0] / (W * H) + 2.0 * np.count_nonzero(total[:, 1:] == 0, axis=1)
    np.testing.assert_allclose(c, costs, rtol=1e-7)
    np.testing.assert_array_equal(total[:, 1:] > 0, used > 0)


def _bench(args, timeout=300):
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args], env=env, cwd=root,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_gpus_1_prints_one_line(gpu):
    """bench.py --gpus 1 (the driver's BENCH form) stays a single process with
    today's line, plus the split and the communicator's rank count (none)."""
    import json

    r = _bench(["--gpus", "1", "--steps", "3", "--warmup", "1", "--size", "256", "--K", "16",
                "--population", "2", "--no-cpu-baseline", "--no-full-search"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # stdout carries the line and nothing else
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["value"] > 0
    assert d["split"] == "none" and d["rccl_ranks"] == 0 and "launcher" not in d
    assert d["roofline"]["kernel_avg_ms"] > 0


def test_bench_launcher_refuses_more_gpus_than_visible(gpu):
    import ctypes

    import hybridquantization_amd as hq

    n = ctypes.c_int()
    hq.load().hq_device_count(ctypes.byref(n))
    r = _bench(["--gpus", str(n.value + 1), "--steps", "1", "--size", "256", "--K", "16",
                "--no-cpu-baseline", "--no-full-search"], timeout=200)
    assert r.returncode == 2
    assert f"only {n.value} GPU(s) visible" in r.stderr


def test_bench_shard_with_comm_keeps_stdout_to_one_line(gpu):
    """A shard step with a one-rank RCCL communicator (--shard-comm): RCCL prints
    its version banner to stdout at communicator set-up; bench.py routes native
    output to stderr so stdout stays the one JSON line.  The step carries the
    collective ("comm" timed) and the communicator reports one rank."""
    import json

    r = _bench(["--steps", "3", "--warmup", "1", "--size", "512", "--K", "16", "--population", "2",
                "--shard-of", "2", "--shard-comm", "--no-cpu-baseline", "--no-full-search"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["rccl_ranks"] == 1 and d["config"]["shard_comm"] is True
    assert d["kernel_avg_ms"]["comm"] > 0 and d["kernel_avg_ms"]["finalize"] == 0
