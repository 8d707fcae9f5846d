import sys
import numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import goldens
from multicamera_stitching_amd import _capi
res = {}
for name in ["tiny_blocks", "pair_affineish", "labels_lex"]:
    meta, frames, out = goldens.load(name)
    cams = goldens.sorted_cams(meta, frames)
    plan = goldens.plan_for(meta, cams)
    res[name] = plan.stitch_host(cams)
    res[name + "_again"] = plan.stitch_host(cams)
np.savez("gpurun_out/dump.npz", **res)
print("saved")
