"""Multi-GPU plumbing of the batch path: one process per GPU, scans sharded
across ranks with no data-path collective, then one all-gather of the resulting 6-DoF poses
(7 doubles per scan) over RCCL (torch.distributed "nccl") for local-map stitching.

The same functions run on CPU tensors with the gloo backend (tests/test_multirank.py).
"""
from __future__ import annotations

import numpy as np


def shard_range(n_total: int, rank: int, world: int):
    """Contiguous, balanced slice [lo, hi) of n_total items owned by `rank`."""
    base, rem = divmod(n_total, world)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def gather_poses(local_poses: np.ndarray, out_tensor, device=None):
    """All-gather (B, 7) float64 poses from every rank into out_tensor (world, B, 7)."""
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(local_poses, dtype=np.float64))
    if device is not None:
        t = t.to(device, non_blocking=True)
    dist.all_gather_into_tensor(out_tensor, t.unsqueeze(0))
    return out_tensor


def max_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
