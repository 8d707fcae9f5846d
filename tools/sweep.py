"""Kernel time vs captures per launch (fixed per-launch cost vs per-capture cost)."""
import os, sys, json
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from multicamera_stitching_amd import rig, _capi
from multicamera_stitching_amd.StitcherClass import _stage_desc

st, images, _ = rig.calibrated_stitcher(4, 1920, 1080, 3, seed=0)
cams = [images[l] for l in st.img_labels]
plan = _capi.Plan([_stage_desc(sb) for sb in st.stitchers], 1920, 1080, 3, 1)
Fmax = 64
dev = torch.device("cuda", 0)
d_cams = [torch.from_numpy(c).to(dev).unsqueeze(0).repeat(Fmax, 1, 1, 1).contiguous() for c in cams]
pitch = (plan.out_w * 3 + 255) // 256 * 256
out = torch.empty((Fmax, plan.out_h, pitch), dtype=torch.uint8, device=dev)
s = torch.cuda.Stream()
plan.prepare(s.cuda_stream)
print("plan stats", plan.stats(), flush=True)
res = {}
for F in [1, 2, 4, 8, 16, 32, 64]:
    ts = []
    for it in range(12):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        plan.stitch_device([t.data_ptr() for t in d_cams], [t[0].numel() for t in d_cams],
                           out.data_ptr(), pitch, out[0].numel(), F, s.cuda_stream)
        b.record(s)
        torch.cuda.synchronize()
        if it >= 2:
            ts.append(a.elapsed_time(b))
    res[F] = float(np.median(ts))
    print(F, "%.4f ms" % res[F], "%.2f us/capture" % (res[F] * 1000 / F), flush=True)
print(json.dumps(res))
