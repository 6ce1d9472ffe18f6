"""Pair-space and query sharding across GPUs (one process per GPU, torch.distributed).

versusAll's unordered pairs are the row-major upper triangle of the N x N product; row a holds
N-1-a pairs.  Ranks take contiguous row blocks balanced by pair count; the
pair blocks are independent, so the only exchange is the final gather of each rank's results
(RCCL all-gather over xGMI on GPUs, gloo on CPU for tests).  RCCL has no all-gather-v, so
blocks are padded to the largest one.  versusReference shards its queries the same way
(contiguous equal blocks, references replicated on every rank).
"""

from __future__ import annotations

from typing import Callable

import numpy as np


def tri_row_start(a: int, n: int) -> int:
    return a * (2 * n - a - 1) // 2


def shard_rows(n: int, world: int) -> list[tuple[int, int]]:
    """Row ranges [r0, r1) per rank with nearly equal pair counts."""
    total = n * (n - 1) // 2
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        lo, hi = bounds[-1], n
        while lo < hi:  # smallest row whose start >= target
            mid = (lo + hi) // 2
            if tri_row_start(mid, n) >= target:
                hi = mid
            else:
                lo = mid + 1
        bounds.append(lo)
    bounds.append(n)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def shard_pairs(n: int, world: int) -> list[tuple[int, int]]:
    """(k0, count) of each rank's contiguous block of the linear pair index."""
    out = []
    for r0, r1 in shard_rows(n, world):
        k0 = tri_row_start(r0, n)
        out.append((k0, tri_row_start(r1, n) - k0))
    return out


def gather_blocks(local, counts: list[int], group=None, device=None, dst: int | None = None):
    """Gather variable-length leading-dim blocks in rank order.

    ``local`` has shape (counts[rank], ...): a numpy array, or a torch tensor already on the
    collective's device (no host round trip).  Uses torch.distributed (the default group's backend:
    nccl = RCCL on ROCm GPUs, gloo on CPU).  RCCL has no variable-size gather, so blocks are padded to
    the largest one.  dst None: every rank receives the concatenation (all-gather); dst = r: only rank
    r does (a gather: the other ranks return None and receive nothing)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    pad = max(counts) if counts else 0
    if isinstance(local, torch.Tensor):
        t = local if device is None else local.to(device)
        tail = tuple(t.shape[1:])
        if t.shape[0] != pad:
            tp = torch.zeros((pad,) + tail, dtype=t.dtype, device=t.device)
            tp[: t.shape[0]] = t
            t = tp
    else:
        tail = tuple(local.shape[1:])
        buf = np.zeros((pad,) + tail, dtype=local.dtype)
        buf[: local.shape[0]] = local
        t = torch.from_numpy(buf)
        if device is not None:
            t = t.to(device)
    if dst is None:
        outs = torch.empty((world * pad,) + tail, dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(outs, t, group=group)
    else:
        parts = [torch.empty_like(t) for _ in range(world)] if rank == dst else None
        dist.gather(t, gather_list=parts, dst=dst, group=group)
        if rank != dst:
            return None
        outs = torch.cat(parts, dim=0)
    outs = outs.cpu().numpy().reshape((world, pad) + tail)
    return np.concatenate([outs[r, : counts[r]] for r in range(world)], axis=0)


def distributed_all_pairs(n: int, compute: Callable[[int, int], np.ndarray], group=None, device=None) -> np.ndarray:
    """Every rank computes its pair block with ``compute(k0, count)`` and receives all blocks.

    Returns the full (n(n-1)/2, ...) result in pair-index order on every rank."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    blocks = shard_pairs(n, world)
    k0, cnt = blocks[rank]
    local = compute(k0, cnt)
    return gather_blocks(local, [c for _, c in blocks], group=group, device=device)


def shard_range(n: int, world: int) -> list[tuple[int, int]]:
    """Contiguous, nearly equal [lo, hi) blocks of n rows (versusReference queries)."""
    return [(n * r // world, n * (r + 1) // world) for r in range(world)]


def distributed_rows(n: int, compute: Callable[[int, int], np.ndarray], group=None, device=None) -> np.ndarray:
    """Every rank computes ``compute(q0, q1)`` (rows [q0, q1), shape (q1 - q0, ...)) for its
    block and receives every block: the full (n, ...) result on every rank."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    blocks = shard_range(n, world)
    q0, q1 = blocks[rank]
    return gather_blocks(compute(q0, q1), [hi - lo for lo, hi in blocks], group=group, device=device)


def world_info() -> tuple[bool, int]:
    """(distributed run with more than one rank, rank)."""
    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            return True, dist.get_rank()
    except Exception:
        pass
    return False, 0
