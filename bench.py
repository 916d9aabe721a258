"""bench.py -- SWASA dE cost evaluation throughput on MI355X.

Metric (BASELINE.json): Mpixel*evals/s of the SWASA dE cost at 4096x4096, K=256.
A "step" is one SWASA iteration of the native search (IM:497-568): neighbour
generation for P palettes, evaluation of the P candidate costs on the GPU
(palette prep + exact grid, argmin, S-CIELAB stencil + dE76, fixed-order fp64
reduction), when N > 1 the RCCL all-gather of every rank's fixed-point
counter blocks (row blocks) or of the palette split's result rows, and the
acceptance step.  value = W*H*P*steps / max-over-ranks wall time (strong
scaling: the 4096^2 image is row-block sharded over the N GPUs).

Run: python bench.py [--gpus N] [--steps K] [--warmup W].  N > 1 runs one
process per GPU: under torch.distributed.run (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*
set; WORLD_SIZE must equal N), or, when WORLD_SIZE is unset, bench.py starts
the N rank processes itself (launch_ranks: the parent imports neither torch nor
libhq, so nothing touches the GPU before the ranks exist) and relays rank 0's
line.
"""

from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3    # vector FP32 spec


def synthetic_planes(w, h, seed=1):
    """SplitMix64 u8 per channel -> u8/255.0f; same as oracle.synthetic_image."""
    with np.errstate(over="ignore"):
        i = np.arange(1, w * h + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    s = np.float32(255.0)
    return [((z >> np.uint64(8 * c)) & np.uint64(0xFF)).astype(np.float32) / s for c in range(3)]


def measured_traffic(size, K, P, grid, world, kernel, dpi=72, distance=45.0, with_source=False):
    """HBM bytes per launch of `kernel` from the newest committed PMC passes
    whose config matches this run (image size, K, P, grid and viewing
    geometry): any profiles/rNN*hbm_traffic.json, newest = the highest round,
    then the latest `generated` stamp (scripts/pmc_traffic.py), then the name.
    None when no file matches (a file with an empty config never does)."""
    import glob
    import re

    cands = []
    for path in glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]*hbm_traffic.json")):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        c = d.get("config") or {}
        if world != 1 or (c.get("size"), c.get("K"), c.get("P"), c.get("grid")) != (size, K, P, grid):
            continue
        if (c.get("dpi", 72), float(c.get("distance", 45.0))) != (dpi, float(distance)):
            continue
        hit = next((int(v["traffic_bytes"]) for name, v in sorted(d.get("kernels", {}).items())
                    if name.startswith("hq::" + kernel)), None)
        if hit is not None:
            rnd = int(re.match(r"r(\d\d)", os.path.basename(path)).group(1))
            cands.append(((rnd, str(d.get("generated", "")), os.path.basename(path)), hit))
    if not cands:
        return (None, None) if with_source else None
    key, hit = max(cands)
    return (hit, key[2]) if with_source else hit


def cost_accounting(half, K, grid, opts):
    """The cost kernel that runs for a geometry / palette size / options, and its
    flops per pixel-evaluation: nominal = the reference's stencil, 7 separable
    filters x 2 passes x (2 half + 1) taps x 2 flops, + Opp->Lab / dE76 ~ 40 (628 at
    the default half 10); executed = the fast path's filters centred in its tap
    bucket HB (2 HB + 1 taps), the narrow k1 filters over their trimmed windows
    only (hq_cost.hip trim_w); the generic path runs the filters as designed.
    Returns (kernel name, bucket HB or 0, chunked, nominal, executed)."""
    rows = int(opts.get("cost_rows", 16))
    variant = int(opts.get("cost_variant", 0))
    hb = next((b for b in (10, 15, 19, 24) if half <= b), 0)
    # K <= 256: u8 indices; 256 < K <= 16384: chunked palettes, 16-bit indices, the
    # tiled kernel at HB = 10 with 16 x 128 tiles only, up to 32 chunks; above: 32-bit indices
    chunked = 256 < K <= 16384 and int(opts.get("chunked", 1)) != 0 and grid > 0
    nch = 1 << max(0, (K - 1).bit_length() - 8) if chunked else 1  # chunk_count: 256-colour chunks
    tw_opt = int(opts.get("cost_tw", 128))
    generic = (variant != 0 or hb == 0 or (K > 256 and not chunked)
               or (chunked and (hb != 10 or rows != 16 or tw_opt != 128 or nch > 32)))
    trim_w = {10: (3, 4, 5), 15: (4, 5, 7), 19: (5, 7, 9), 24: (6, 9, 12)}
    if generic:
        # cost_variant 2: the per-pixel pair; otherwise the LDS-tiled pair
        # (variant 1, the LDS-tiled pair: both passes on the matrix cores up to half 64)
        vm = half <= 64 and int(opts.get("gen_vmfma", 1))
        kernel = ("gen_hpass_kernel+gen_vpass_kernel" if variant == 2 else
                  "gen_hmfma_kernel+gen_vmfma_kernel" if vm and int(opts.get("gen_hmfma", 1)) else
                  "gen_hrow4_kernel+gen_vmfma_kernel" if vm else
                  "gen_hrow4_kernel+gen_vtile2_kernel" if half <= 64 else "gen_hrow4_kernel+gen_vtile_kernel")
        taps_exec = 7 * (2 * half + 1)
    else:
        kernel = "cost_mfma_kernel" if rows == 8 and hb == 10 else "cost16w_kernel"
        trim = int(opts.get("trim", 1)) != 0
        taps_exec = 4 * (2 * hb + 1) + (sum(2 * t + 1 for t in trim_w[hb]) if trim else 3 * (2 * hb + 1))
    return kernel, (0 if generic else hb), chunked, 7 * 2 * (2 * half + 1) * 2 + 40, 2 * 2 * taps_exec + 40


def use_palette_split(split, P, world):
    """N > 1: the palette split (whole image, P / N palettes per rank, one
    all-gather) when asked, or under 'auto' when P >= 8 N and N divides P (C5:
    1.23x faster per rank than the row split); else row blocks."""
    if world <= 1:
        return False
    return split == "palettes" or (split == "auto" and P >= 8 * world and P % world == 0)


def profiled_stages(world, comm=False):
    """hq_profile_get names of one search iteration: the kernels, and at N > 1
    (or with a one-rank communicator, --shard-comm) the collective ("comm": the
    RCCL all-gather of the counter blocks or of the palette split's rows,
    event-timed)."""
    return ("sa_step", "grid", "assign", "cost", "finalize") + (("comm",) if world > 1 or comm else ())


def kernel_profile(prof, world, max_over_ranks=None):
    """{stage: (avg ms, launches)} of this rank -> (kernel_avg_ms of this rank,
    the MAX over ranks of each average or None at N = 1).  max_over_ranks maps
    a {stage: ms} dict to the element-wise max over the process group."""
    avg = {k: round(v[0], 4) for k, v in prof.items()}
    if world <= 1 or max_over_ranks is None:
        return avg, None
    mx = max_over_ranks({k: v[0] for k, v in prof.items()})
    return avg, {k: round(v, 4) for k, v in mx.items()}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args):
    """BASELINE.md's CPU plan on this host's cores: the C restatement of the
    reference's semantics (oracle/hq_oracle.c, 'port'; the reference's own Java
    path computes no cost without OpenCL, IM:392, IM:590).  The headline value
    is the same-shape eval (4096^2, K = 256) on the box's CPU share for one GPU;
    also timed: the C1 256^2 / K = 16 and C2 1024^2 / K = 64 evaluation loops
    on those threads, and one thread on a 1024^2 / K = 256 sample.  LabRef is setup, not timed (the
    eval's work does not depend on its values, so a zero LabRef is used)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import c_oracle  # checker/baseline only
    import oracle as o

    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    # every core this process may use, capped at the box's CPU share for one GPU
    # (OMP_NUM_THREADS, 16 on the GPU boxes, whose nproc shows the whole machine)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = int(os.environ.get("HQ_CPU_THREADS", "0")) or min(usable or 1, share or usable or 1)
    f = o.design_filters()

    def rate(w, K, nthreads, seconds, max_evals):
        R, G, B = o.synthetic_image(w, w, seed=1)
        rgba = o.inline_rgba(R, G, B)
        lab = np.zeros_like(rgba)
        c_oracle.eval_palette(rgba, lab, o.synthetic_palette(K, 1), f, w, nthreads=nthreads)  # warm
        evals, t0 = 0, time.perf_counter()
        while True:
            c_oracle.eval_palette(rgba, lab, o.synthetic_palette(K, 2 + evals), f, w, nthreads=nthreads)
            evals += 1
            el = time.perf_counter() - t0
            if el >= seconds or evals >= max_evals:
                return w * w * evals / el / 1e6, evals, el

    v, n, el = rate(args.size, args.K, threads, args.cpu_seconds, 64)
    c1, n1, el1 = rate(256, 16, threads, 2.0, 4096)
    c2, n2, el2 = rate(1024, 64, threads, 3.0, 4096)
    st, ns, els = rate(1024, args.K, 1, 4.0, 64)
    # Every usable core of the node is NOT timed: a GPU box is one GPU's share
    # of a shared node (OMP_NUM_THREADS = 16) and worker pools must stay inside
    # that share.  The linear projection from the measured per-thread rate is
    # reported as such, next to the measured numbers it is derived from.
    all_cores = {"measured": False, "usable_cpus": usable, "threads_timed": threads,
                 "projected_linear_value": round(v / threads * usable, 3) if usable else None,
                 "reason": "the box's CPU share for one GPU is OMP_NUM_THREADS threads; the node's "
                           "other cores belong to other jobs, so only the share is timed"}
    if os.environ.get("HQ_CPU_ALL_CORES") == "1" and usable and usable != threads:
        va, na, ela = rate(args.size, args.K, usable, args.cpu_seconds, 64)
        all_cores = {"measured": True, "value": round(va, 3), "threads": usable, "evals": na,
                     "seconds": round(ela, 2)}
    ref_gpu = reference_kernels_on_gpu(args)
    return {"value": round(v, 3), "unit": "Mpixel*evals/s", "cores": threads, "kind": "port",
            "nproc": os.cpu_count(), "usable_cpus": usable, "cpu_share": share or None,
            "cpu_model": _cpu_model(),
            "sample": f"{args.size}x{args.size} image, K={args.K}: {n} candidate evaluations on "
                      f"{threads} threads in {el:.1f} s (C restatement oracle/hq_oracle.c: "
                      f"exhaustive argmin, S-CIELAB stencil, Lab, dE76, fp64 sum)",
            "c1_256_k16": {"value": round(c1, 3), "evals": n1, "seconds": round(el1, 2),
                           "threads": threads},
            "c2_1024_k64": {"value": round(c2, 3), "evals": n2, "seconds": round(el2, 2),
                            "threads": threads},
            "all_cores": all_cores,
            "single_thread_1024_k256": {"value": round(st, 3), "evals": ns,
                                        "seconds": round(els, 2), "threads": 1},
            "reference_kernels_on_this_gpu": ref_gpu}


def reference_kernels_on_gpu(args, reps=3, timeout=180):
    """The reference's own population evaluation on this GPU, same shape: its
    OpenCL kernels (OptimizedConvolution.cl, compiled unmodified for gfx950 into
    oracle/_ref by `make -C oracle ref`) driven in the order of its JavaCL host
    code (IM:620-727, oracle/ref_cl_host.c).  Part of the baseline leg, after
    the timed region, in a child process under a time limit (an OpenCL runtime
    that misbehaves can neither hang nor fail the run: its error is reported).
    The LabRef input is zeros: the reference's work does not depend on its
    values."""
    import subprocess

    cmd = [sys.executable, os.path.abspath(__file__), "--ref-kernels-child",
           json.dumps({"size": args.size, "K": args.K, "P": args.population, "seed": args.seed,
                       "dpi": args.dpi, "distance": args.distance, "reps": reps})]
    try:
        res = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
        lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
        if res.returncode != 0 or not lines:
            return {"value": None, "error": f"exit {res.returncode}: {res.stderr.strip()[-300:]}"}
        return json.loads(lines[-1])
    except subprocess.TimeoutExpired:
        return {"value": None, "error": f"timed out after {timeout} s"}
    except Exception as e:  # noqa: BLE001 -- a baseline, never the run's outcome
        return {"value": None, "error": f"{type(e).__name__}: {e}"}


def _ref_kernels_child(spec):
    """Child of reference_kernels_on_gpu: prints one JSON object."""
    c = json.loads(spec)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as o
    import ref_cl  # the reference's kernels (baseline only)

    R, G, B = synthetic_planes(c["size"], c["size"], seed=c["seed"])
    rgba = o.inline_rgba(R.ravel(), G.ravel(), B.ravel())
    del R, G, B
    pals = np.stack([o.synthetic_palette(c["K"], 2 + p) for p in range(c["P"])])
    t = ref_cl.time_population(rgba, np.zeros_like(rgba), c["size"], pals, o.design_filters(c["dpi"], c["distance"]),
                               reps=c["reps"])
    px_evals = c["size"] * c["size"] * c["P"]
    kern_ms = c["P"] * sum(t["kernel_ms"].values())
    print(json.dumps({"value": round(px_evals / kern_ms / 1e3, 2), "unit": "Mpixel*evals/s",
                      "wall_value": round(px_evals / t["wall_ms"] / 1e3, 2),
                      "kernel_ms_per_population": round(kern_ms, 4), "wall_ms_per_population": round(t["wall_ms"], 3),
                      "kernel_ms_per_member": {k: round(v, 4) for k, v in t["kernel_ms"].items()},
                      "reps": c["reps"], "kind": "reference",
                      "sample": f"{c['size']}x{c['size']}, K={c['K']}, P={c['P']}: the reference's five kernels per "
                                "member (value: their device time) and its host sequence with the error-image reads "
                                "and host means (wall_value)"}))


GPU_MODULES = ("torch", "hybridquantization_amd")


def gpu_modules_loaded():
    """Modules in this process that could touch the GPU (the launcher must have none)."""
    return sorted(m for m in sys.modules if m.split(".")[0] in GPU_MODULES)


def _free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpus():
    """Visible HIP devices, counted in a child process (this one stays GPU-free)."""
    import subprocess

    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(f"bench.py: counting the visible GPUs failed: {r.stderr.strip()[-400:]}")
    return int(r.stdout.strip().splitlines()[-1])


def launch_ranks(n, argv, dry_run=False):
    """--gpus N > 1 with WORLD_SIZE unset: start N rank processes of this script,
    one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1 and
    a free port), wait for them all, print rank 0's JSON line with a `launcher`
    record, and return the exit status (non-zero if any rank failed; the other
    ranks are then stopped).  Nothing here imports torch or libhq."""
    import subprocess
    import tempfile

    before = gpu_modules_loaded()
    if not dry_run:
        have = visible_gpus()
        if n > have:
            print(f"bench.py: --gpus {n} but only {have} GPU(s) visible", file=sys.stderr, flush=True)
            return 2
    port = _free_port()
    out0 = tempfile.TemporaryFile(mode="w+")
    procs = []
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                       HQ_BENCH_LAUNCHER=str(os.getpid()))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                          stdout=out0 if r == 0 else sys.stderr))
        rc = 0
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 1
                    print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    for q in live:
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    out0.seek(0)
    lines = [ln for ln in out0.read().splitlines() if ln.startswith("{")]
    if rc != 0:
        return rc
    if len(lines) != 1:
        print(f"bench.py: rank 0 printed {len(lines)} JSON lines, expected 1", file=sys.stderr, flush=True)
        return 1
    line = json.loads(lines[0])
    line["launcher"] = {"by": "bench.py", "ranks": n, "master": f"127.0.0.1:{port}",
                        "parent_gpu_modules": before}
    print(json.dumps(line), flush=True)
    return 0


def dry_run_worker(world, rank):
    """--dry-run: the rank wiring alone (gloo, no libhq, no GPU).  Rank 0 prints
    one line with the ranks it saw over the process group."""
    import torch
    import torch.distributed as dist

    env = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "world": world, "pid": os.getpid()}
    if os.environ.get("HQ_DRY_RUN_FAIL_RANK") == str(rank):  # test: one rank dies before the rendezvous
        raise SystemExit(3)
    seen = [env]
    if world > 1:
        dist.init_process_group("gloo")
        seen = [None] * world
        dist.all_gather_object(seen, env)
        dist.barrier()
    if rank == 0:
        print(json.dumps({"metric": "Mpixel*evals/s (SWASA dE cost) at 4096x4096 K=256", "dry_run": True,
                          "n_gpus": world, "ranks_seen": seen, "torch": torch.__version__}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def full_search(lib, _lib, m, K, P, seed, sa_device, restore):
    """BASELINE config 3 as the plugin runs it: one SWASA search of imax = 5000
    iterations with the default schedule (HQ:197-224), P palettes per
    iteration.  Returns wall time, iterations and the best error found; the
    context's sa_device option is set back to `restore` (the run's own value)."""
    import hybridquantization_amd as hq

    m.setOption("sa_device", sa_device)
    sw = hq.SWASA(population=P, seed=seed)
    params = sw.params()
    s = C.c_void_p()
    t0 = time.perf_counter()
    _lib.check(lib.hq_search_create(m.ctx, C.byref(params), K, sw.seed, C.byref(s)), m.ctx)
    ran = C.c_int()
    _lib.check(lib.hq_search_run(s, params.imax, C.byref(ran)), m.ctx)
    best = np.zeros(4 * K, np.float32)
    err = C.c_double()
    it = C.c_int()
    _lib.check(lib.hq_search_best(s, _lib.fptr(best), C.byref(err), C.byref(it)), m.ctx)
    wall = time.perf_counter() - t0
    lib.hq_search_destroy(s)
    m.setOption("sa_device", restore)
    return {"wall_s": round(wall, 3), "iterations": it.value, "best_error": err.value}, best


def main():
    if len(sys.argv) == 3 and sys.argv[1] == "--ref-kernels-child":
        _ref_kernels_child(sys.argv[2])
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of this node; default WORLD_SIZE or 1.  N > 1 with WORLD_SIZE unset: "
                         "bench.py starts the N rank processes itself")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--K", type=int, default=256)
    ap.add_argument("--population", type=int, default=4)
    ap.add_argument("--grid", type=int, default=32)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--dpi", type=int, default=72, help="viewing geometry (HQ:229-231): screen dpi")
    ap.add_argument("--distance", type=float, default=45.0, help="viewing distance in cm")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="extra libhq option (hq.h), repeatable; for experiments")
    ap.add_argument("--shard-of", type=int, default=0, metavar="N",
                    help="experiment: run rank 0's row block of an N-way split on one GPU, "
                         "no collective (per-rank step time at N GPUs)")
    ap.add_argument("--shard-comm", action="store_true",
                    help="with --shard-of: a one-rank RCCL communicator, so each step carries the "
                         "collective path (the all-gather of the counter blocks)")
    ap.add_argument("--split", choices=["auto", "rows", "palettes"], default="auto",
                    help="N > 1: row-block shards + one all-reduce, or each rank the whole image and P/N "
                         "palettes + one all-gather (SURVEY 8e); auto: palettes when P >= 8 N and N "
                         "divides P (C5: 1.23x faster per rank, DESIGN.md 5), else rows")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-full-search", action="store_true",
                    help="skip the imax = 5000 search of BASELINE config 3 (extra keys)")
    ap.add_argument("--dry-run", action="store_true",
                    help="test the rank wiring only: gloo process group, no libhq, no GPU")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus is not None and args.gpus < 1:
            raise SystemExit(f"bench.py: --gpus {args.gpus}")
        if args.gpus is not None and args.gpus > 1:  # this process only launches and relays
            sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.dry_run))
        world = 1
    else:
        world = int(env_world)
        if args.gpus is not None and args.gpus != world:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one process per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        dry_run_worker(world, rank)
        return
    # The job's stdout carries exactly one JSON line (rank 0's).  Native
    # libraries print to fd 1 on their own -- RCCL's version banner at
    # communicator set-up -- so fd 1 goes to stderr for the run and the line is
    # written to the saved stdout at the end.
    sys.stdout.flush()
    line_fd = os.dup(1)
    os.dup2(2, 1)
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        have = torch.cuda.device_count()
        if local >= have:
            raise SystemExit(f"bench.py: rank {rank} needs GPU {local} (LOCAL_RANK) but {have} are visible")
        torch.cuda.set_device(local)
        dist.init_process_group("gloo")  # control plane only; data path is libhq's RCCL comm

    import hybridquantization_amd as hq
    from hybridquantization_amd import _lib
    from hybridquantization_amd import dist as hqd

    lib = hq.load()
    W = H = args.size
    m = hq.ImageManipulation(hq.deltaETypes.CIE76, device=local)
    if not m.getOpenCLAvailable():
        raise RuntimeError("bench.py: libhq could not open the GPU")
    sp = hq.ScielabProcessor(args.dpi, args.distance, hq.Whitepoint.D65, None, m)
    m.setOption("grid", args.grid)
    if args.shard_of > 0:
        m.setOption("shard_solo", 1)
    opts = dict(kv.split("=", 1) for kv in args.opt)
    for k, v in opts.items():
        m.setOption(k, int(v))
    sa_device = int(opts.get("sa_device", 1))
    R, G, B = synthetic_planes(W, H, seed=args.seed)
    psplit = use_palette_split(args.split, args.population, world)
    if psplit:
        hqd.palette_slice(args.population, world, rank)  # (raises unless the population divides)
        m.setOption("palette_split", 1)
    r0, r1 = (0, H) if psplit else hqd.shard_rows(H, args.shard_of if args.shard_of > 0 else world, rank)
    _lib.check(lib.hq_set_image_planar_shard(m.ctx, _lib.fptr(R), _lib.fptr(G), _lib.fptr(B), W, H,
                                             _lib.fptr(sp.illuminant), r0, r1), m.ctx)
    del R, G, B
    if world > 1:
        hqd.init_comm(m, dist, world, rank)
    elif args.shard_of > 0 and args.shard_comm:
        m.initComm(1, 0, m.commUniqueId())
    rccl_ranks, rccl_rank = m.commInfo()  # (0, -1): no communicator (one GPU)
    if (world > 1 or (args.shard_of > 0 and args.shard_comm)) and (rccl_ranks, rccl_rank) != (world, rank):
        raise RuntimeError(f"bench.py: RCCL communicator has {rccl_ranks} ranks (rank {rccl_rank}), "
                           f"expected {world} (rank {rank})")

    P = args.population
    # which BASELINE.json config this run's shape is (configs[2] is the default)
    shape = (W, args.K, P)
    cfg_name = {(4096, 256, 4): "BASELINE config 3", (1024, 64, 1): "BASELINE config 2",
                (8192, 256, 4): "BASELINE config 4", (4096, 256, 64): "BASELINE config 5",
                (256, 16, 4): "BASELINE config 1"}.get(shape, "not a BASELINE config")
    # BASELINE config 3's real search (imax = 5000, default schedule) is its own
    # measurement (extra key `full_search_c3`).  It runs before the benchmark's
    # search: the GPU's clocks take ~0.1 s of sustained load to settle, and a
    # timed region of a few steps straight after set-up measured ~7% slow (20
    # vs 100 steps: 0.72 vs 0.67 ms).  At N > 1 every rank runs it, device-
    # resident with the communicator (the same path as the timed steps).
    search_line = None
    if not args.no_full_search:
        dev, bdev = full_search(lib, _lib, m, args.K, P, args.seed, 1, sa_device)
        where = (f"rows [{r0}, {r1}) of an {args.shard_of}-way split, "
                 f"{'a one-rank communicator' if args.shard_comm else 'no collective'}" if args.shard_of > 0
                 else f"{world} GPU(s)")
        label = "BASELINE config 3" if shape == (4096, 256, 4) else f"full search ({cfg_name})"
        search_line = {"config": f"{label}: {W}x{H}, K={args.K}, P={P}, imax=5000, "
                                 "default SWASA schedule (HQ:197-224), seed "
                                 f"{args.seed}, {where}",
                       "device_resident": dev,
                       "ms_per_iteration_device": round(dev["wall_s"] / max(dev["iterations"], 1) * 1e3, 4)}
        if world == 1 and args.shard_of == 0:  # the host-driven driver must agree bit for bit
            host, bhost = full_search(lib, _lib, m, args.K, P, args.seed, 0, sa_device)
            search_line["host_driven"] = host
            search_line["device_host_agree"] = bool(dev["best_error"] == host["best_error"]
                                                    and np.array_equal(bdev, bhost)
                                                    and dev["iterations"] == host["iterations"])

    sw = hq.SWASA(population=args.population, imax=10 ** 9, seed=args.seed)
    params = sw.params()
    search = C.c_void_p()
    _lib.check(lib.hq_search_create(m.ctx, C.byref(params), args.K, sw.seed, C.byref(search)), m.ctx)
    ran = C.c_int()
    _lib.check(lib.hq_search_run(search, args.warmup, C.byref(ran)), m.ctx)

    def sync_all():
        if world > 1:
            import torch

            torch.cuda.synchronize()
            dist.barrier()

    # Timed region: the search loop alone.  Kernel times come from a second pass of
    # the same number of steps with HIP events on the context stream: an event
    # between two kernels leaves the GPU idle ~5-10 us (measured in the rocprofv3
    # timeline), ~4% of a step, so they stay out of the timed region.
    sync_all()
    t0 = time.perf_counter()
    _lib.check(lib.hq_search_run(search, args.steps, C.byref(ran)), m.ctx)
    sync_all()
    elapsed = time.perf_counter() - t0
    lib.hq_profile_reset(m.ctx)
    lib.hq_profile_enable(m.ctx, 1)
    _lib.check(lib.hq_search_run(search, args.steps, C.byref(ran)), m.ctx)
    lib.hq_profile_enable(m.ctx, 0)
    if world > 1:
        elapsed = hqd.max_over_ranks(dist, elapsed)

    prof = {}
    for k in profiled_stages(world, rccl_ranks > 0):
        ms = C.c_double()
        n = C.c_int64()
        lib.hq_profile_get(m.ctx, k.encode(), C.byref(ms), C.byref(n))
        prof[k] = (ms.value / max(n.value, 1), n.value)
    kernel_avg, kernel_max = kernel_profile(prof, world, dist and (lambda v: hqd.max_each_over_ranks(dist, v)))
    best = np.zeros(4 * args.K, np.float32)
    berr = C.c_double()
    it = C.c_int()
    lib.hq_search_best(search, _lib.fptr(best), C.byref(berr), C.byref(it))
    lib.hq_search_destroy(search)

    n_own = W * (r1 - r0)
    value = W * H * P * args.steps / elapsed / 1e6
    if args.shard_of > 0:  # experiment: one rank's rows only (per-rank rate, not a job total)
        value = n_own * P * args.steps / elapsed / 1e6
    # Dominant kernel: the cost kernel (S-CIELAB stencil + Opp->Lab + dE76).  With P > 1
    # palettes per launch its HBM bytes (LabRef once + P index images) amortise
    # and FP32 VALU bounds it; its flops: cost_accounting.
    half = m.halfSize
    kernel, hb, chunked, flops_nominal, flops_exec = cost_accounting(half, args.K, args.grid, opts)
    cost_ms = prof["cost"][0]
    P_dev = hqd.palette_slice(P, world, rank)[1] if psplit else P  # palettes one device's cost kernel evaluates
    alg_flops = n_own * P_dev * flops_nominal
    exec_flops = n_own * P_dev * flops_exec
    achieved_tf = alg_flops / (cost_ms * 1e-3) / 1e12 if cost_ms > 0 else 0.0
    exec_tf = exec_flops / (cost_ms * 1e-3) / 1e12 if cost_ms > 0 else 0.0
    alg_bytes = n_own * (12 + P_dev * (1 if args.K <= 256 else 2 if chunked else 4))
    hbm_gbs = alg_bytes / (cost_ms * 1e-3) / 1e9 if cost_ms > 0 else 0.0
    traffic, traffic_src = measured_traffic(W, args.K, P, args.grid, world, kernel.split("+")[0],
                                            args.dpi, args.distance, with_source=True)
    # whole-evaluation view: the metric's 24 B/px-eval HBM-read roofline
    eval_roof_mpx = HBM_PEAK_GBS * 1e9 / 24.0 / 1e6 * world
    out = {
        "metric": "Mpixel*evals/s (SWASA dE cost) at 4096x4096 K=256",
        "value": round(value, 2),
        "unit": "Mpixel*evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (SplitMix64 u8 RGB image, java.util.Random-seeded SWASA palettes)",
        "config": {"workload": f"SWASA search iteration, {W}x{H} RGB image, K={args.K}, "
                               f"population P={P} palettes per step ({cfg_name})",
                   "image": f"{W}x{H}", "K": args.K, "population": P,
                   "parallelism": (f"palette split x{world} + RCCL all-gather" if psplit else
                                   f"row-block x{world} + RCCL all-reduce" if world > 1 else "1 GPU"),
                   "argmin_grid": args.grid,
                   **({"dpi": args.dpi, "distance_cm": args.distance}
                      if (args.dpi, args.distance) != (72, 45.0) else {}),
                   **({"shard_of": args.shard_of, "rows": [r0, r1], "shard_comm": bool(args.shard_comm)}
                      if args.shard_of > 0 else {}),
                   **({"options": args.opt} if args.opt else {})},
        "roofline": {"bound": "valu", "achieved": round(achieved_tf, 2), "peak": FP32_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(achieved_tf / FP32_PEAK_TFLOPS, 4),
                     "traffic": traffic, "traffic_source": traffic_src and f"profiles/{traffic_src}",
                     "kernel": kernel, "kernel_avg_ms": round(cost_ms, 4),
                     "flops_per_px_eval": flops_nominal, "exec_flops_per_px_eval": flops_exec,
                     "half": half, "tap_bucket": hb or None,
                     "alg_flops_per_launch": alg_flops, "exec_flops_per_launch": exec_flops,
                     "frac_executed_taps": round(exec_tf / FP32_PEAK_TFLOPS, 4),
                     "alg_bytes_per_launch": alg_bytes, "hbm_GBs_alg": round(hbm_gbs, 1),
                     "hbm_frac": round(hbm_gbs / HBM_PEAK_GBS, 4),
                     "note": "fp32-accurate stencil: vertical taps on the matrix cores as split-f16 "
                             "products (hi*hi+hi*lo+lo*hi, fp32 accumulate), horizontal taps, Lab and dE on "
                             "FP32 VALU.  bound valu: the compute roof is the FP32 vector peak, 157.3 TFLOP/s "
                             "(the f32 MFMA peak is the same number on gfx950); achieved = the nominal "
                             "7*2*(2 half+1)*2 + 40 flop/px-eval of the reference's stencil + Lab/dE (628 at "
                             "half 10) over the kernel time (all P palettes' launches); frac_executed_taps = "
                             "the flops the kernel executes (bucket taps, trimmed narrow filters); hbm_frac = the kernel's algorithmic bytes (LabRef 12 B + P index bytes "
                             "per pixel) over its time against 8 TB/s; traffic = HBM bytes/launch from the "
                             "committed rocprofv3 FETCH_SIZE(x2)+WRITE_SIZE passes when their config matches; "
                             "kernel_avg_ms: HIP events carried by the launches on the context stream over a "
                             "second pass of the same steps, right after the timed one (events idle the GPU "
                             "~5-10 us each, so the timed pass has none)"},
        "split": "palettes" if psplit else "rows" if world > 1 else "none",
        "rccl_ranks": rccl_ranks,
        "metric_hbm_roofline_frac": round(value / eval_roof_mpx, 4),
        "kernel_avg_ms": kernel_avg,
        **({"kernel_avg_ms_max_over_ranks": kernel_max} if kernel_max is not None else {}),
        "best_error": berr.value,
    }
    if search_line is not None and rank == 0:
        out["full_search_c3"] = search_line
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args)
        ref = out["cpu_baseline"].get("reference_kernels_on_this_gpu") or {}
        if ref.get("value"):  # this line's value over the reference's own kernels on this GPU
            ref["libhq_over_reference"] = round(value / ref["value"], 2)
    m.close()
    sys.stdout.flush()
    if rank == 0:
        os.write(line_fd, (json.dumps(out) + "\n").encode())
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
