"""Multi-GPU sharding of a JPEG batch: images are independent, so each rank
(one process per GPU) decodes its own shard with no data-path collective; the only exchange is a
final gather of per-image records {status, width, height, ncomp, checksum64} over RCCL/xGMI
(backend "nccl" on ROCm), or gloo for the CPU tests. Shards may differ in size (shard_by_size):
the gather pads every rank's records to the largest shard.

Record tensors are int64 [n, 5]: status, width, height, ncomp, checksum (the uint64 checksum's
bit pattern). Device records come from icx_jpeg_records (libicx, a kernel over each decoded
image); `checksum64` restates the checksum in numpy for checks on the host.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


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


def checksum64(data) -> int:
    """sum_k w_k * (2k + 1) mod 2^64 over the little-endian uint32 words w_k of `data` (the last
    one zero-padded): the records' checksum of a decoded image (include/icx.h icx_record)."""
    b = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data.reshape(-1).view(np.uint8)
    pad = (-len(b)) % 4
    if pad:
        b = np.concatenate([b, np.zeros(pad, np.uint8)])
    w = b.view("<u4").astype(np.uint64)
    k = np.arange(len(w), dtype=np.uint64)
    with np.errstate(over="ignore"):
        return int((w * (np.uint64(2) * k + np.uint64(1))).sum(dtype=np.uint64))


def records_from_numpy(rec) -> "torch.Tensor":
    """icx RECORD_DTYPE array -> int64 [n, 5] tensor (checksum as its int64 bit pattern)."""
    import torch
    out = np.zeros((len(rec), 5), np.int64)
    for j, f in enumerate(("status", "width", "height", "ncomp")):
        out[:, j] = rec[f]
    out[:, 4] = rec["checksum"].view(np.int64)
    return torch.from_numpy(out)


def gather_records(local, dist_mod, group=None):
    """All-gather every rank's int64 [n_r, 5] record tensor, n_r may differ per rank: the
    shard sizes are exchanged first, each rank's records are padded to the largest shard and
    gathered with one all_gather_into_tensor, and the padding is dropped. Returns the
    concatenation in rank order and the per-rank counts. The tensor must live where the
    backend expects it (device memory for nccl = RCCL, host for gloo)."""
    import torch
    world = dist_mod.get_world_size(group)
    if world == 1:
        return local, [int(local.shape[0])]
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    counts = torch.empty(world, dtype=torch.int64, device=local.device)
    dist_mod.all_gather_into_tensor(counts, n, group=group)
    cnt = [int(c) for c in counts.cpu()]
    m = max(cnt)
    pad = torch.zeros((m, 5), dtype=torch.int64, device=local.device)
    pad[: local.shape[0]] = local
    full = torch.empty((world * m, 5), dtype=torch.int64, device=local.device)
    dist_mod.all_gather_into_tensor(full, pad, group=group)
    return torch.cat([full[r * m: r * m + cnt[r]] for r in range(world)]), cnt
