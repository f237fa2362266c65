"""Multi-GPU sharding of a JPEG batch: images are independent, so each rank
(one process per GPU) decodes its own shard with no data-path collective; the only exchange is a
final gather of per-image results (statuses, dims) over RCCL/xGMI (backend "nccl" on ROCm), or
gloo for the CPU tests.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple


def shard_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous image range [start, stop) of `rank`; sizes differ by at most one."""
    if world <= 0 or not 0 <= rank < world or n_total < 0:
        raise ValueError("bad shard arguments")
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard_by_size(sizes: Sequence[int], world: int) -> List[List[int]]:
    """Greedy longest-first split of image indices by compressed size, for skewed batches:
    decode time tracks the entropy-coded bytes. Each shard keeps ascending index order."""
    if world <= 0:
        raise ValueError("world must be positive")
    loads = [0] * world
    shards: List[List[int]] = [[] for _ in range(world)]
    for i in sorted(range(len(sizes)), key=lambda k: (-sizes[k], k)):
        r = min(range(world), key=lambda q: (loads[q], q))
        shards[r].append(i)
        loads[r] += sizes[i]
    return [sorted(s) for s in shards]


def gather_results(local, dist_mod, group=None):
    """All-gather a per-rank 1-D tensor of equal length (e.g. int32 statuses) and return the
    concatenation in rank order. The tensor must live where the backend expects it (CUDA/HIP
    for nccl=RCCL, CPU for gloo)."""
    world = dist_mod.get_world_size(group)
    if world == 1:
        return local
    import torch
    parts = [torch.empty_like(local) for _ in range(world)]
    dist_mod.all_gather(parts, local, group=group)
    return torch.cat(parts)
