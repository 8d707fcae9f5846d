"""Multi-GPU frame sharding (one process per GPU, torch.distributed).

Rig captures (time steps) are independent, so a stream of captures is sharded round-robin over
the ranks and every rank stitches its own with its own plan: no collective touches the data path
(SURVEY.md section 8e).  The only exchanges are control-plane ones -- a barrier and a max-reduce of
timings -- and, optionally, gathering finished mosaics to one consumer rank (RCCL over xGMI when
the process group is "nccl": one point-to-point transfer per peer, straight into the consumer's
buffer).
"""
from __future__ import annotations

import time
from typing import List, Sequence


def shard_frames(n_frames: int, rank: int, world: int) -> List[int]:
    """Capture indices rank `rank` of `world` processes stitches (capture f -> rank f % world)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("rank %d outside world %d" % (rank, world))
    return list(range(rank, n_frames, world))


# A check every rank runs before each collective of these helpers (bench.py guarded(): a rank whose
# line failed tells the others at their next collective instead of leaving them to time out)
_GUARD = None


def set_collective_guard(fn):
    """fn() runs before every collective below (None: no check); returns the previous one."""
    global _GUARD
    prev, _GUARD = _GUARD, fn
    return prev


def _guard():
    if _GUARD is not None:
        _GUARD()


def max_over_ranks(values: Sequence[float], device=None) -> List[float]:
    """Element-wise max over all ranks (the slowest rank defines the job's time)."""
    import torch
    import torch.distributed as dist
    _guard()
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.cpu()]


def gather_mosaics(local, dst: int = 0, bufs=None):
    """Collect every rank's finished mosaics (same shape on every rank) on rank `dst`.

    Returns the list of per-rank tensors on `dst` (rank order), None elsewhere.  Point-to-point
    sends to the consumer, not a ring collective: each peer's transfer uses its own xGMI link.
    bufs (on `dst`): preallocated receive tensors, one per peer in rank order (reused across
    calls); fresh ones otherwise.
    """
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [local]
    _guard()
    world, rank = dist.get_world_size(), dist.get_rank()
    if rank == dst:
        peers = iter(bufs) if bufs is not None else None
        out = [local if r == dst else (next(peers) if peers else torch.empty_like(local))
               for r in range(world)]
        reqs = [dist.irecv(out[r], src=r) for r in range(world) if r != dst]
        for q in reqs:
            q.wait()
        return out
    dist.send(local, dst=dst)
    return None


def mcs_group(device: int):
    """The libmcs RCCL group (mcs_group_create) of this torch.distributed job: rank 0's
    unique id reaches every rank through the process group; collective."""
    import torch.distributed as dist
    from . import _capi
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    box = [_capi.Group.unique_id() if rank == 0 else None]
    if world > 1:
        _guard()
        dist.broadcast_object_list(box, src=0)
    return _capi.Group(world, rank, box[0], device)


def gather_mosaics_group(group, local, recv=None, dst: int = 0, stream: int = 0):
    """Every rank's mosaics (contiguous tensor `local`, same size everywhere) to rank `dst`
    through mcs_group_gather: recv (on dst) = a (world, *local.shape) tensor, rank r's at
    recv[r].  Enqueued on `stream`."""
    _guard()
    group.gather(local.data_ptr(), local.numel() * local.element_size(),
                 recv.data_ptr() if recv is not None else 0, dst, stream)
    return recv


def timed_loop(step, steps: int, warmup: int, sync, record=None) -> float:
    """The bench contract's timed region on this rank: `warmup` untimed steps, then exactly
    `steps` timed ones bracketed on both sides by (sync, barrier, sync); returns this rank's
    wall seconds (reduce with max_over_ranks).  record(i, "start"|"end") brackets step i (HIP
    events on the kernels' stream)."""
    import torch.distributed as dist
    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    for _ in range(warmup):
        step()
    sync()
    if multi:
        _guard()
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        if record:
            record(i, "start")
        step()
        if record:
            record(i, "end")
    sync()
    if multi:
        dist.barrier()
    sync()
    return time.perf_counter() - t0


def job_rate(units_per_step_per_rank: float, steps: int, seconds_max: float, world: int) -> float:
    """Whole-job throughput: the units every rank processed over the slowest rank's time."""
    return world * units_per_step_per_rank * steps / seconds_max


CHECKSUM_CHUNK = 1 << 24     # bytes per slice: 64 MB of int32 temporaries, whatever the batch


def checksum(t, chunk: int = CHECKSUM_CHUNK) -> int:
    """Order-sensitive 63-bit checksum of a u8 tensor's bytes, computed where the tensor lives;
    used to verify gathered mosaics against their producers.

    sum_i byte_i * ((i + 1) mod 65521) mod 2^63, taken slice by slice: per slice of `chunk` bytes
    the products (< 2^24) in int32 and their int64 sum, so a 1.3 GB batch needs 2 x 64 MB of
    temporaries instead of 10 GB of int64 ones."""
    import torch
    flat = t.reshape(-1)
    n = flat.numel()
    base = torch.arange(min(chunk, max(n, 1)), device=flat.device, dtype=torch.int32)
    total = 0
    for o in range(0, n, chunk):
        m = min(chunk, n - o)
        w = base[:m] + ((o + 1) % 65521)
        w = torch.remainder(w, 65521)
        total += int((flat[o:o + m].to(torch.int32) * w).sum(dtype=torch.int64).item())
    return total & ((1 << 63) - 1)


def max_abs_over_ranks(mine, device=None):
    """Max over ranks of each rank's own max |product - oracle| (None where a rank did not
    check; None overall when no rank did)."""
    v = -1.0 if mine is None else float(mine)
    got = max_over_ranks([v], device=device)[0]
    return None if got < 0 else int(got)


def gather_and_verify(local, dst: int = 0, bufs=None, device=None):
    """gather_mosaics + a checksum-of-checksums check: every rank's checksum of what it sent is
    all-gathered, and `dst` compares them with checksums of what it received.  Returns
    (mosaics on dst or None, ok on every rank)."""
    import torch
    import torch.distributed as dist
    got = gather_mosaics(local, dst, bufs)
    world = dist.get_world_size() if dist.is_initialized() else 1
    mine = torch.tensor([checksum(local)], dtype=torch.int64, device=device)
    sums = [torch.zeros_like(mine) for _ in range(world)]
    if world > 1:
        dist.all_gather(sums, mine)
    else:
        sums = [mine]
    ok = True
    if got is not None:
        ok = all(checksum(g) == int(s.item()) for g, s in zip(got, sums))
    flag = torch.tensor([1 if ok else 0], dtype=torch.int64, device=device)
    if world > 1:
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return got, bool(flag.item())
