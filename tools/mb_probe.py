"""Multi-band launch timing probe: the C2 rig's multi-band launch over 64 captures with distinct
camera frames per capture (normal) and with every capture reading the same frames (frame
stride 0: data L2/TLB-warm), and the paste-only launch for reference."""
import os, sys, json
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from multicamera_stitching_amd import rig, _capi
from multicamera_stitching_amd.StitcherClass import _stage_desc

st, images, _ = rig.calibrated_stitcher(4, 1920, 1080, 3, seed=0)
cams = [images[l] for l in st.img_labels]
F = 64
dev = torch.device("cuda", 0)
d_cams = [torch.from_numpy(c).to(dev).unsqueeze(0).repeat(F, 1, 1, 1).contiguous() for c in cams]
s = torch.cuda.Stream()
res = {}
for mode, name in [(_capi.MCS_BLEND_NONE, "paste"), (_capi.MCS_BLEND_MULTIBAND, "multiband")]:
    plan = _capi.Plan([_stage_desc(sb) for sb in st.stitchers], 1920, 1080, 3, 1)
    plan.set_blend(mode)
    pitch = (plan.out_w * 3 + 255) // 256 * 256
    out = torch.empty((F, plan.out_h, pitch), dtype=torch.uint8, device=dev)
    plan.prepare(s.cuda_stream)
    for fs_name, strides in [("distinct", [t[0].numel() for t in d_cams]), ("same", [0] * 4)]:
        ts = []
        for it in range(12):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            plan.stitch_device([t.data_ptr() for t in d_cams], strides, out.data_ptr(), pitch,
                               out[0].numel(), F, s.cuda_stream)
            b.record(s)
            torch.cuda.synchronize()
            if it >= 2:
                ts.append(a.elapsed_time(b))
        res[f"{name}_{fs_name}"] = float(np.median(ts))
        print(name, fs_name, "%.4f ms" % res[f"{name}_{fs_name}"], flush=True)
print(json.dumps(res))
