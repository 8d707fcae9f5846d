import ctypes, sys
import numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import goldens
from multicamera_stitching_amd import _capi
L = _capi.load()
res = {}
for name in ["tiny_blocks", "labels_lex", "pair_affineish"]:
    meta, frames, out = goldens.load(name)
    cams = [np.ascontiguousarray(c) for c in goldens.sorted_cams(meta, frames)]
    plan = goldens.plan_for(meta, cams)
    dbg = np.zeros((plan.out_h, plan.out_w, 4), np.int32)
    ptrs = (ctypes.c_void_p * len(cams))(*[c.ctypes.data for c in cams])
    rc = L.mcs__debug_pixels(plan.handle, ptrs, dbg.ctypes.data_as(ctypes.c_void_p))
    res[name] = dbg
    print(name, rc)
np.savez("gpurun_out/dbg_pixels.npz", **res)
