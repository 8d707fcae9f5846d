"""ORB host-path probe: one 1080p BGR frame through mcs_orb_detect_host serially (median of 50)
and four frames from four threads, beside a plain pageable / pinned 6.2 MB upload."""
import os, sys, time, json
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from concurrent.futures import ThreadPoolExecutor
from multicamera_stitching_amd import _capi, rig

W, H = 1920, 1080
g = rig.corner_texture(H, W, seed=0).astype(np.uint8)
frames = [np.ascontiguousarray(np.stack([np.roll(g, 7 * k, 1)] * 3, -1)) for k in range(4)]
res = {}


def med(fn, n=50):
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts)) * 1e3


for _ in range(5):
    _capi.orb_detect(frames[0], 2000, 8, 1.2, 20)
res["orb_1frame_serial_ms"] = med(lambda: _capi.orb_detect(frames[0], 2000, 8, 1.2, 20))
pool = ThreadPoolExecutor(4)
list(pool.map(lambda f: _capi.orb_detect(f, 2000, 8, 1.2, 20), frames))
res["orb_4frames_4threads_ms"] = med(lambda: list(pool.map(
    lambda f: _capi.orb_detect(f, 2000, 8, 1.2, 20), frames)))
d = torch.empty(frames[0].nbytes, dtype=torch.uint8, device="cuda")
src = torch.from_numpy(frames[0].reshape(-1))
pin = src.pin_memory()
for name, s in [("upload_pageable_ms", src), ("upload_pinned_ms", pin)]:
    def up():
        d.copy_(s, non_blocking=True)
        torch.cuda.synchronize()
    up()
    res[name] = med(up)
print(json.dumps({k: round(v, 4) for k, v in res.items()}))
