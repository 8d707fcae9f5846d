"""Multi-process sharding on CPU (gloo, world size 2): captures are split without overlap or gaps,
timings reduce to the slowest rank, and mosaics gather onto the consumer rank intact."""
import os
import socket

import pytest

from multicamera_stitching_amd.shard import shard_frames


def test_shard_frames_partition():
    for world in (1, 2, 3, 8):
        for n in (0, 1, 7, 64):
            got = sorted(f for r in range(world) for f in shard_frames(n, r, world))
            assert got == list(range(n))
    with pytest.raises(ValueError):
        shard_frames(4, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from multicamera_stitching_amd import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = shard.shard_frames(10, rank, world)
        t = shard.max_over_ranks([0.5 + rank, 3.0 - rank])
        # a fake "mosaic" per rank: its capture indices painted into a small u8 image
        mosaic = torch.zeros((4, 6, 3), dtype=torch.uint8)
        for i, f in enumerate(mine):
            mosaic.view(-1)[i] = f
        got = shard.gather_mosaics(mosaic, dst=0)
        if rank == 0:
            flat = sorted(int(v) for g in got for v in g.view(-1)[:5].tolist())
            q.put(("ok", t, flat, [list(g.shape) for g in got]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gloo_world2_sharding_reduce_gather():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    status, t, flat, shapes = q.get(timeout=5)
    assert status == "ok"
    assert t == [1.5, 3.0]
    assert flat == list(range(10))
    assert shapes == [[4, 6, 3], [4, 6, 3]]


def test_checksum_chunked_equals_definition():
    """shard.checksum slice by slice (int32 products, int64 sums) = the position-weighted sum
    sum_i b_i ((i + 1) mod 65521) mod 2^63, for slice sizes that do and do not divide the data."""
    import numpy as np
    import torch
    from multicamera_stitching_amd import shard
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, size=200_003, dtype=np.uint8)
    w = (np.arange(1, a.size + 1, dtype=np.int64) % 65521)
    want = int((a.astype(np.int64) * w).sum()) & ((1 << 63) - 1)
    t = torch.from_numpy(a)
    for chunk in (1 << 24, 65536, 1000, 7):
        assert shard.checksum(t, chunk=chunk) == want
    assert shard.checksum(t.reshape(-1)[:0]) == 0
