"""C3 probe: resident estimation throughput of rig jobs that carry B captures each (one job over
4 B cameras: capture q's cameras at 4q .. 4q + 3; the pairs across a capture boundary are
computed and ignored).  Estimate only (no stitch), D jobs in flight.  A feasibility measurement
for multi-capture rig jobs: prints one line per (B, D)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,2,3")
    ap.add_argument("--depths", default="4")
    ap.add_argument("--captures", type=int, default=600)
    args = ap.parse_args()
    import torch
    from multicamera_stitching_amd import _capi, rig
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from estimate_bench import world
    W, Hh, N = 1920, 1080, 4
    C = rig.camera_models(N, W, Hh, seed=0)
    frames = rig.world_frames(C, W, Hh, 3, seed=0, world_fn=world)
    dev = torch.device("cuda", 0)
    base = torch.stack([torch.from_numpy(f) for f in frames]).to(dev)
    for B in [int(b) for b in args.batches.split(",")]:
        for D in [int(d) for d in args.depths.split(",")]:
            sets = [base.repeat(B, 1, 1, 1).contiguous() for _ in range(D)]
            ptrs = [[t.data_ptr() for t in s] for s in sets]
            jobs = [_capi.RigJob(N * B, W, Hh, 3) for _ in range(D)]
            njobs = max(D, args.captures // B)
            ref = None
            t0 = None
            for i in range(njobs + D):
                if i == D:   # (warm: the first round builds graphs)
                    t0 = time.perf_counter()
                s = i % D
                if i >= D:
                    H, st = jobs[s].wait()
                    if ref is None:
                        ref = [None if h is None else h.copy() for h in H]
                if i < njobs:
                    jobs[s].submit(ptrs[s])
            dt = time.perf_counter() - t0
            # every capture's pairs equal capture 0's (the same frames): the batched job's results
            same = all((ref[q * N + k] is None) == (ref[k] is None) and
                       (ref[k] is None or np.array_equal(ref[q * N + k], ref[k]))
                       for q in range(B) for k in range(N - 1))
            print(json.dumps({"captures_per_job": B, "depth": D,
                              "captures_per_s": round(njobs * B / dt, 1),
                              "pairs_equal_across_batch": same}), flush=True)
            for j in jobs:
                j.close()
            del sets


if __name__ == "__main__":
    main()
