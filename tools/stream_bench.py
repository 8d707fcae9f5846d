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


def link_probe(in_bytes, out_bytes, reps=20):
    """The host link's ceiling on this box, with the pipeline's own transfer sizes: pinned
    hipMemcpyAsync H2D alone, D2H alone, and both at once on two streams (GB/s)."""
    import torch
    h_in = torch.empty(in_bytes, dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(out_bytes, dtype=torch.uint8, pin_memory=True)
    d_in = torch.empty(in_bytes, dtype=torch.uint8, device="cuda")
    d_out = torch.empty(out_bytes, dtype=torch.uint8, device="cuda")
    s_up, s_down = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(up, down):
        for warm in (True, False):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(2 if warm else reps):
                if up:
                    with torch.cuda.stream(s_up):
                        d_in.copy_(h_in, non_blocking=True)
                if down:
                    with torch.cuda.stream(s_down):
                        h_out.copy_(d_out, non_blocking=True)
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        return round(reps * ((in_bytes if up else 0) + (out_bytes if down else 0)) / dt / 1e9, 2)

    return {"h2d_gbs": timed(True, False), "d2h_gbs": timed(False, True),
            "bidir_gbs": timed(True, True)}


def host_copy_gbs(nbytes, reps=10):
    """Single-thread host memcpy rate (numpy copy) for the submit()/wait() copies."""
    a = np.ones(nbytes, np.uint8)
    b = np.empty_like(a)
    np.copyto(b, a)
    t0 = time.perf_counter()
    for _ in range(reps):
        np.copyto(b, a)
    return round(reps * nbytes / (time.perf_counter() - t0) / 1e9, 2)


def run(w, h, blend, depth, frames, graphs=True, zero_copy=False, link=None):
    """zero_copy: frames written into the pinned slots in place (input_views, once per slot:
    a producer decoding straight into them) and mosaics read from the pinned slots
    (wait(copy=False)); otherwise numpy frames in, numpy mosaics out (two host memcpys per
    capture on the submitting thread)."""
    from multicamera_stitching_amd import _capi, rig
    from multicamera_stitching_amd.StitcherClass import _stage_desc
    st, images, _ = rig.calibrated_stitcher(4, w, h, 3, seed=0)
    cams = [images[label] for label in st.img_labels]
    plan = _capi.Plan([_stage_desc(sb) for sb in st.stitchers], w, h, 3, 1)
    plan.set_blend(blend)
    pipe = _capi.StreamPipeline(plan, depth=depth, use_graphs=graphs)
    out = [np.empty(plan.out_shape(), np.uint8) for _ in range(depth)]
    if zero_copy:
        for slot in range(depth):
            for v, c in zip(pipe.input_views(slot), cams):
                v[...] = c

    def submit():
        return pipe.submit_inplace() if zero_copy else pipe.submit(cams)

    def collect(s):
        if zero_copy:
            pipe.wait(s, copy=False)
        else:
            pipe.wait(s, out[s])
    ring = []
    for _ in range(depth):                      # warm-up
        ring.append(submit())
    for s in ring:
        collect(s)
    ring = []
    t0 = time.perf_counter()
    for f in range(frames):
        if len(ring) == depth:
            collect(ring.pop(0))
        ring.append(submit())
    while ring:
        collect(ring.pop(0))
    dt = time.perf_counter() - t0
    if zero_copy:   # the slots still hold capture 0's frames: check the last mosaic
        want = plan.stitch_host(cams)
        assert np.array_equal(pipe.output_view((frames - 1) % depth), want)
    pipe.close()
    mpix = plan.out_w * plan.out_h / 1e6
    in_mb = sum(c.nbytes for c in cams) / 1e6
    gbs = frames * (in_mb + mpix * 3) / dt / 1e3
    res = {"cams": f"4x{w}x{h}x3", "blend": blend, "depth": depth, "graphs": graphs,
           "zero_copy": zero_copy, "frames": frames, "fps": round(frames / dt, 1),
           "mpix_per_s": round(frames * mpix / dt, 1), "pcie_gb_per_s": round(gbs, 2)}
    if link is not None:
        res["link_ceiling_gbs"] = link["bidir_gbs"]
        res["frac_of_link"] = round(gbs / link["bidir_gbs"], 3)
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--sizes", default="1920x1080,3840x2160")
    ap.add_argument("--summary", action="store_true",
                    help="also print one closing JSON line holding every configuration's line")
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    lines = []
    for size in a.sizes.split(","):
        w, h = (int(v) for v in size.split("x"))
        in_b = 4 * w * h * 3
        out_b = int(3.23 * w) * (h + h // 40) * 3       # about the rig's mosaic size
        link = link_probe(in_b, out_b)
        link.update(cams=f"4x{w}x{h}x3", host_memcpy_gbs=host_copy_gbs(in_b))
        print(json.dumps({"link_probe": link}), flush=True)
        lines.append({"link_probe": link})
        for blend in (0, 2):
            for depth, graphs, zc in ((1, False, False), (3, True, False), (3, True, True)):
                r = run(w, h, blend, depth, a.frames, graphs, zc, link)
                print(json.dumps(r), flush=True)
                lines.append(r)
    if a.summary:
        print(json.dumps({"metric": "streamed rig captures/s (C5: host frames in, host mosaics "
                                    "out, mcs_stream_*)", "unit": "fps", "lines": lines}))
