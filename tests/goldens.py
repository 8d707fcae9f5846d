"""Loader for the fixtures in tests/golden (made by tests/golden/gen_golden.py, which executes
the reference's StitcherClass.py)."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def names():
    return sorted(os.path.basename(p)[:-5] for p in glob.glob(os.path.join(GOLDEN, "*.json")))


def load(name):
    """(meta, calibration frames by label, reference output)."""
    meta, frames, _, out = load_full(name)
    return meta, frames, out


def load_full(name):
    """(meta, calibration frames, frames passed to Stitcher.stitch, reference output).  The two
    frame sets differ for the resize cases (frames off their calibrated shape)."""
    meta = json.load(open(os.path.join(GOLDEN, name + ".json")))
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    frames = {lab: z["cam%d" % i] for i, lab in enumerate(meta["labels"])}
    stitch = {lab: z["scam%d" % i] if "scam%d" % i in z else frames[lab]
              for i, lab in enumerate(meta["labels"])}
    return meta, frames, stitch, z["out"]


def calibrated_hw(meta):
    """Calibrated (h, w) of each camera in sorted-label order (None: never read)."""
    st = meta["stages"]
    hw = [None] * (len(st) + 1)
    for i, s in enumerate(st):
        if s["calibrated"]:
            if hw[0] is None:
                hw[0] = tuple(s["BimgSize"][:2])
            hw[i + 1] = tuple(s["AimgSize"][:2])
    return hw


def resized_for_oracle(meta, cams):
    """The frames as the reference's stages see them after its cv2.resize branch (:226-233)."""
    from oracle import oracle
    out = []
    for c, hw in zip(cams, calibrated_hw(meta)):
        if hw is not None and tuple(c.shape[:2]) != hw:
            c = oracle.resize_linear(c, (hw[1], hw[0]))
        out.append(c)
    return out


def sorted_cams(meta, frames):
    return [frames[label] for label in meta["img_labels"]]


def stage_desc(s, meta, cams, i):
    from multicamera_stitching_amd import _capi
    d = _capi.StageDesc()
    if not s["calibrated"]:
        d.a_w, d.a_h = cams[i + 1].shape[1], cams[i + 1].shape[0]
        return d
    d.H[:] = list(np.array(s["cachedAH"], np.float64).reshape(9))
    d.calibrated = 1
    d.canvas_w, d.canvas_h = s["ABSize"]
    d.b_x, d.b_y = s["Bpts"][0]
    d.b_w, d.b_h = s["BimgSize"][1], s["BimgSize"][0]
    d.a_w, d.a_h = s["AimgSize"][1], s["AimgSize"][0]
    d.super_mode = int(meta["super_mode"])
    d.x_lim0, d.x_lim1 = s["x_limits"]
    d.y_lim0, d.y_lim1 = s["y_limits"]
    return d


def plan_for(meta, cams, interp=1, device=0, channels=None):
    """Plan of the fixture's chain; cams: calibration frames (sorted-label order)."""
    from multicamera_stitching_amd import _capi
    descs = [stage_desc(s, meta, cams, i) for i, s in enumerate(meta["stages"])]
    ch = channels or (1 if cams[0].ndim == 2 else cams[0].shape[2])
    return _capi.Plan(descs, cams[0].shape[1], cams[0].shape[0], ch, interp, device)


def oracle_stages(meta):
    out = []
    for s in meta["stages"]:
        if not s["calibrated"]:
            continue
        out.append(dict(H=np.array(s["cachedAH"]), canvas_w=s["ABSize"][0],
                        canvas_h=s["ABSize"][1], bx=s["Bpts"][0][0], by=s["Bpts"][0][1],
                        super_mode=meta["super_mode"], x_limits=s["x_limits"],
                        y_limits=s["y_limits"]))
    return out


def used_cams(meta, cams):
    return [cams[0]] + [cams[i + 1] for i, s in enumerate(meta["stages"]) if s["calibrated"]]
