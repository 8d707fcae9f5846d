import ctypes, sys
import numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import goldens
from multicamera_stitching_amd import _capi
L = _capi.load()
L.mcs__kparams_size.restype = ctypes.c_size_t
n = L.mcs__kparams_size()
for name in ["tiny_blocks", "fail_mid"]:
    meta, frames, out = goldens.load(name)
    cams = goldens.sorted_cams(meta, frames)
    plan = goldens.plan_for(meta, cams)
    dv = np.zeros(n, np.uint8); hv = np.zeros(n, np.uint8)
    rc = L.mcs__echo_kparams(plan.handle, dv.ctypes.data_as(ctypes.c_void_p), hv.ctypes.data_as(ctypes.c_void_p))
    diff = np.nonzero(dv != hv)[0]
    print(name, "rc", rc, "size", n, "differing bytes:", len(diff), diff[:40].tolist())
    print(" host st0 ints:", hv[312+72:312+120].view(np.int32).tolist())
    print(" dev  st0 ints:", dv[312+72:312+120].view(np.int32).tolist())
