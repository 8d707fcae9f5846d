"""Multi-GPU frame sharding (one process per GPU, torch.distributed).

Rig captures (time steps) are independent, so a stream of captures is sharded round-robin over
the ranks and every rank stitches its own with its own plan: no collective touches the data path
(SURVEY.md section 8e).  The only exchanges are control-plane ones -- a barrier and a max-reduce of
timings -- and, optionally, gathering finished mosaics to one consumer rank (RCCL over xGMI when
the process group is "nccl": one point-to-point transfer per peer, straight into the consumer's
buffer).
"""
from __future__ import annotations

from typing import List, Sequence


def shard_frames(n_frames: int, rank: int, world: int) -> List[int]:
    """Capture indices rank `rank` of `world` processes stitches (capture f -> rank f % world)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("rank %d outside world %d" % (rank, world))
    return list(range(rank, n_frames, world))


def max_over_ranks(values: Sequence[float], device=None) -> List[float]:
    """Element-wise max over all ranks (the slowest rank defines the job's time)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.cpu()]


def gather_mosaics(local, dst: int = 0):
    """Collect every rank's finished mosaics (same shape on every rank) on rank `dst`.

    Returns the list of per-rank tensors on `dst` (rank order), None elsewhere.  Point-to-point
    sends to the consumer, not a ring collective: each peer's transfer uses its own xGMI link.
    """
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [local]
    world, rank = dist.get_world_size(), dist.get_rank()
    if rank == dst:
        out = [local if r == dst else torch.empty_like(local) for r in range(world)]
        reqs = [dist.irecv(out[r], src=r) for r in range(world) if r != dst]
        for q in reqs:
            q.wait()
        return out
    dist.send(local, dst=dst)
    return None
