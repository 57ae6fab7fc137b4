"""Multi-GPU sharding of the packet-build path.

Packets shard by iteration index: seeds depend only on (seq, k), so every
rank builds an independent, disjoint range and the concatenation over ranks
equals a single-GPU build.  The only exchange is the reference's global
counter (total_pckts / total_bytes, sequence.c:12-14, 633-642), all-reduced
once per epoch over torch.distributed (RCCL on GPUs, gloo on CPU)."""
from typing import Tuple


def shard(first_iter: int, n_iter: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous split of [first_iter, first_iter + n_iter): rank g gets
    [g*N/G, (g+1)*N/G) (strong scaling of a fixed job)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    a = first_iter + n_iter * rank // world
    b = first_iter + n_iter * (rank + 1) // world
    return a, b - a


def step_first_iter(step: int, rank: int, world: int, n_per_rank: int) -> int:
    """Weak scaling (bench.py): step s of rank r builds iterations
    [(s*world + r) * n, ... + n) — disjoint over ranks and steps."""
    return (step * world + rank) * n_per_rank


def allreduce_counters(pckts, bytes_, device="cpu"):
    """Sum per-sequence {packets, bytes} u64 counters over all ranks."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([[int(p), int(b)] for p, b in zip(pckts, bytes_)], dtype=torch.int64, device=device)
    dist.all_reduce(t)
    return [int(x) for x in t[:, 0].tolist()], [int(x) for x in t[:, 1].tolist()]
