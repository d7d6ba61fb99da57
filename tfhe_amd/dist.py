"""Multi-GPU plumbing for the PBS path: one process per GPU, torch.distributed.

Independent PBS shard embarrassingly across ranks: the only collective on the data
path is NONE; the key set is broadcast once (RCCL over xGMI with the "nccl" backend, gloo on CPU
for tests), and chained circuits gather output ciphertexts between levels (all_gather).

These helpers take torch tensors and a process group; they never call the HIP library, so the
same code is exercised by the world-size-2 gloo tests on CPU.
"""
from __future__ import annotations

from typing import Callable, List, Tuple

import numpy as np


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, stop) slice of `total` units for `rank` (sizes differ by at most one)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def broadcast_keys(bsk, ksk, src: int = 0, group=None) -> float:
    """Broadcast the (int64-viewed) BSK and KSK tensors from `src` in place; returns ms spent
    (device-synchronous for CUDA tensors)."""
    import time

    import torch
    import torch.distributed as dist

    cuda = bsk.is_cuda
    if cuda:
        torch.cuda.synchronize(bsk.device)
    t0 = time.perf_counter()
    dist.broadcast(bsk, src=src, group=group)
    dist.broadcast(ksk, src=src, group=group)
    if cuda:
        torch.cuda.synchronize(bsk.device)
    return (time.perf_counter() - t0) * 1e3


def _gather_device(local, group):
    """Where the all_gather buffers must live for the group's backend: device memory for "nccl" (RCCL over xGMI:
    a host tensor would be refused), host memory for gloo (its all_gather takes CPU tensors only)."""
    import torch
    import torch.distributed as dist

    if dist.get_backend(group) == "nccl":
        return local.device if local.is_cuda else torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def sharded_map(global_in, fn: Callable, group=None):
    """Apply `fn` (a batched per-rank kernel: (B_r, ...) -> (B_r, ...)) to this rank's contiguous shard
    of `global_in` (same tensor on every rank) and all_gather the shards back in order.

    `global_in` may be a host tensor or a device tensor (a device-resident circuit level); the result is on the
    device of fn's output.  Under "nccl" the gather runs on device buffers (RCCL), under gloo through host
    buffers.  Used for chained circuits (one tree level per call); for the throughput bench every rank owns its
    batch and no gather is needed."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    total = global_in.shape[0]
    lo, hi = shard_range(total, world, rank)
    local = fn(global_in[lo:hi])
    sizes = [shard_range(total, world, r) for r in range(world)]
    width = local.shape[1:]
    maxrows = max(b - a for a, b in sizes)
    gdev = _gather_device(local, group)
    padded = torch.zeros((maxrows,) + tuple(width), dtype=local.dtype, device=gdev)
    padded[: local.shape[0]] = local.to(gdev)
    bufs: List = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(bufs, padded, group=group)
    return torch.cat([bufs[r][: b - a] for r, (a, b) in enumerate(sizes)], dim=0).to(local.device)


def rank_batch_seed(base_seed: int, rank: int) -> int:
    """Per-rank input seed (weak scaling: each rank encrypts its own batch)."""
    return base_seed + rank


def tree_levels(n_leaves: int) -> List[int]:
    """Comparisons per level of a binary reduction tree over n_leaves (e.g. 256 -> 128,64,...,1)."""
    out = []
    while n_leaves > 1:
        out.append(n_leaves // 2)
        n_leaves = n_leaves // 2 + (n_leaves % 2)
    return out


def as_u64(t) -> np.ndarray:
    return t.cpu().numpy().view(np.uint64)
