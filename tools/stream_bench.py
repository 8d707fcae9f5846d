"""End-to-end streaming throughput (host frames in, host mosaics out) through mcs_stream_*:
pinned staging, H2D / stitch (hipGraph) / D2H on three streams.  SURVEY.md 8 C5: 4-camera
3840x2160 video; also the 4 x 1920x1080 rig.  Prints one JSON line per configuration."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(w, h, blend, depth, frames, graphs=True):
    from multicamera_stitching_amd import _capi, rig
    from multicamera_stitching_amd.StitcherClass import _stage_desc
    st, images, _ = rig.calibrated_stitcher(4, w, h, 3, seed=0)
    cams = [images[label] for label in st.img_labels]
    plan = _capi.Plan([_stage_desc(sb) for sb in st.stitchers], w, h, 3, 1)
    plan.set_blend(blend)
    pipe = _capi.StreamPipeline(plan, depth=depth, use_graphs=graphs)
    out = [np.empty(plan.out_shape(), np.uint8) for _ in range(depth)]
    ring = []
    for _ in range(depth):                      # warm-up
        ring.append(pipe.submit(cams))
    for s in ring:
        pipe.wait(s, out[s])
    ring = []
    t0 = time.perf_counter()
    for f in range(frames):
        if len(ring) == depth:
            s = ring.pop(0)
            pipe.wait(s, out[s])
        ring.append(pipe.submit(cams))
    while ring:
        s = ring.pop(0)
        pipe.wait(s, out[s])
    dt = time.perf_counter() - t0
    pipe.close()
    mpix = plan.out_w * plan.out_h / 1e6
    in_mb = sum(c.nbytes for c in cams) / 1e6
    return {"cams": f"4x{w}x{h}x3", "blend": blend, "depth": depth, "graphs": graphs,
            "frames": frames, "fps": round(frames / dt, 1),
            "mpix_per_s": round(frames * mpix / dt, 1),
            "pcie_gb_per_s": round(frames * (in_mb + mpix * 3) / dt / 1e3, 2)}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    for (w, h) in ((1920, 1080), (3840, 2160)):
        for blend in (0, 2):
            for depth, graphs in ((1, False), (3, False), (3, True)):
                print(json.dumps(run(w, h, blend, depth, a.frames, graphs)), flush=True)
