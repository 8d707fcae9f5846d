"""Diagnostics: where does the GPU mosaic differ from a golden fixture?"""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import goldens
from multicamera_stitching_amd import _capi

print("runtime:", _capi.hip_runtime(), "devices:", _capi.device_count())
for name in goldens.names():
    meta, frames, out = goldens.load(name)
    cams = goldens.sorted_cams(meta, frames)
    plan = goldens.plan_for(meta, cams)
    got = plan.stitch_host(cams)
    d = np.abs(got.astype(int) - out.astype(int))
    if d.ndim == 3:
        d = d.max(-1)
    bad = np.argwhere(d > 0)
    fl = plan.describe()
    print(name, "out", got.shape, "bad px", len(bad), "rects", fl["rect"], "off", fl["off_x"], fl["off_y"])
    if len(bad):
        print("   first bad (y,x):", bad[:5].tolist(), "last:", bad[-3:].tolist())
        print("   rows with bad:", sorted(set(bad[:, 0].tolist()))[:20])
        print("   cols range:", bad[:, 1].min(), bad[:, 1].max())
