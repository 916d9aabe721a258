"""Control plane of the sharded evaluation.

One process per GPU.  torch.distributed (gloo) carries only control data:
the 128-byte RCCL unique id from rank 0 to every rank, and the MAX of the
ranks' timings.  The data path runs inside libhq on its own RCCL communicator
over xGMI: per SWASA iteration either one fp64 all-reduce of P * (1 + K)
partial sums (row-block split) or one all-gather of each rank's P / N result
rows (palette split, option "palette_split").  bench.py and the
multi-process tests call these same functions.
"""

from __future__ import annotations


def shard_rows(H: int, world: int, rank: int) -> tuple[int, int]:
    """Rows [r0, r1) owned by `rank` of a `world`-way row-block split of H rows."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} of world {world}")
    return rank * H // world, (rank + 1) * H // world


def palette_slice(P: int, world: int, rank: int) -> tuple[int, int]:
    """Palettes [lo, lo + n) that `rank` evaluates under the palette split
    (hq_runtime.hip palette_slice): an equal slice of the population, every
    rank holding the whole image; P must be a multiple of the world size."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} of world {world}")
    if P % world:
        raise ValueError(f"palette split: population {P} not divisible by {world} ranks")
    n = P // world
    return rank * n, n


def allgather_rows(dist, rows, world: int):
    """The palette split's exchange: every rank's [n, 1 + K] result rows,
    concatenated in rank order ([P, 1 + K]) -- ncclAllGather in libhq, here
    over gloo for tests."""
    import numpy as np
    import torch

    t = torch.from_numpy(np.ascontiguousarray(rows, dtype=np.float64)).clone()
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return torch.cat(out).numpy()


def broadcast_unique_id(dist, rank: int, make_id) -> bytes:
    """Rank 0 calls make_id() (hq_comm_unique_id) and ships the 128 bytes to every
    rank over the (gloo) process group `dist`; every rank returns them."""
    import torch

    uid = torch.zeros(128, dtype=torch.uint8)
    if rank == 0:
        raw = bytes(make_id())
        if len(raw) != 128:
            raise ValueError("an RCCL unique id is 128 bytes")
        uid = torch.frombuffer(bytearray(raw), dtype=torch.uint8).clone()
    dist.broadcast(uid, 0)
    return bytes(uid.numpy().tobytes())


def init_comm(m, dist, world: int, rank: int) -> None:
    """libhq's RCCL communicator for context `m` (an ImageManipulation) of rank
    `rank` in a world of `world` processes, one GPU each."""
    uid = broadcast_unique_id(dist, rank, m.commUniqueId)
    m.initComm(world, rank, uid)


def max_over_ranks(dist, value: float) -> float:
    """MAX of a per-rank float (the bench's elapsed time) over the process group."""
    import torch

    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def max_each_over_ranks(dist, values: dict) -> dict:
    """Element-wise MAX of a per-rank {name: float} (the same keys on every rank,
    e.g. bench.py's per-kernel averages) over the process group."""
    import torch

    keys = sorted(values)
    t = torch.tensor([float(values[k]) for k in keys], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return {k: float(v) for k, v in zip(keys, t.tolist())}


def allreduce_partials(dist, partial):
    """Sum of the ranks' hq_eval_population_partial outputs (numpy fp64 [P*(1+K)])
    over the process group: the exchange libhq does with ncclAllReduce, here over
    gloo for processes that share one GPU (tests)."""
    import numpy as np
    import torch

    t = torch.from_numpy(np.ascontiguousarray(partial, dtype=np.float64)).clone()
    dist.all_reduce(t)
    return t.numpy()
