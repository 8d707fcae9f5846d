"""Two ranks of the libmcs RCCL group on ONE GPU (gloo carries the unique id): does the
gather deliver rank 1's bytes to rank 0?  (RCCL may refuse two ranks on one device.)"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    from multicamera_stitching_amd import _capi, shard
    g = shard.mcs_group(0)
    src = torch.full((1 << 20,), rank + 7, dtype=torch.uint8, device="cuda:0")
    recv = torch.zeros((world, 1 << 20), dtype=torch.uint8, device="cuda:0") if rank == 0 else None
    shard.gather_mosaics_group(g, src, recv, 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    if rank == 0:
        print("gather ok:", all(bool((recv[r] == r + 7).all()) for r in range(world)), flush=True)
    g.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
