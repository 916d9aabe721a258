"""bench.py --gpus N: the launcher starts N rank processes itself (CPU, gloo
dry run: no libhq, no GPU), relays rank 0's one JSON line, and fails loudly
when a rank fails or --gpus disagrees with WORLD_SIZE."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra)
    return env


def _run(args, env, timeout=240):
    return subprocess.run([sys.executable, BENCH, *args], env=env, capture_output=True, text=True,
                          timeout=timeout, cwd=ROOT)


def test_launcher_starts_n_ranks_and_relays_one_line():
    r = _run(["--gpus", "2", "--dry-run"], _env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["dry_run"] is True and d["n_gpus"] == 2
    seen = sorted(d["ranks_seen"], key=lambda e: e["rank"])
    assert [e["rank"] for e in seen] == [0, 1]
    assert [e["local_rank"] for e in seen] == [0, 1]
    assert all(e["world"] == 2 for e in seen)
    assert len({e["pid"] for e in seen}) == 2
    # the launcher itself never imported torch or libhq before the ranks started
    assert d["launcher"]["ranks"] == 2 and d["launcher"]["by"] == "bench.py"
    assert d["launcher"]["parent_gpu_modules"] == []
    assert d["launcher"]["master"].startswith("127.0.0.1:")


def test_launcher_fails_when_a_rank_fails():
    r = _run(["--gpus", "2", "--dry-run"], _env(HQ_DRY_RUN_FAIL_RANK="1"), timeout=120)
    assert r.returncode != 0
    assert "rank 1 exited with 3" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "3", "--dry-run"], _env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0
    assert "--gpus 3 but WORLD_SIZE=2" in r.stderr


def test_single_rank_dry_run_needs_no_launcher():
    r = _run(["--dry-run"], _env())
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1 and "launcher" not in d


def test_launcher_module_has_no_gpu_imports():
    """Importing bench.py (what the launcher process runs) pulls in neither torch
    nor the libhq package."""
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "print(bench.gpu_modules_loaded())" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "[]"


def test_reference_baseline_never_fails_the_run():
    """bench.py's timing of the reference's own kernels runs in a child process
    under a time limit; without a GPU (or without the build) it reports an
    error in the line instead of raising."""
    import argparse

    sys.path.insert(0, ROOT)
    import bench

    args = argparse.Namespace(size=64, K=16, population=2, seed=1, dpi=72, distance=45.0)
    out = bench.reference_kernels_on_gpu(args, reps=1, timeout=120)
    assert out["value"] is None and out["error"]
