#!/usr/bin/env python3
"""Graph-cut seams per plan (8 x 1920x1080 on a 6912 x 1080 cylinder,
the 1/4 seam grid): mcs_plan_find_seams end to end (device sampling + the pairwise max-flows),
device push-relabel by default or the host Dinic with MCS_SEAM_FLOW=host; labels checked against
the CPU restatement (oracle/orc_seam.c via oracle.blend_stitch_cyl) unless --no-check.  One JSON
line."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-check", action="store_true")
    args = ap.parse_args()
    from multicamera_stitching_amd import rig, _capi
    cams, frames, g = rig.cylinder_rig(8, 1920, 1080, 1100.0, 3, seed=0, jitter_deg=0.5)
    plan = _capi.Plan.cylindrical(cams, g["out_w"], g["out_h"], g["f_cyl"], g["u0"], g["v0"], 3)
    plan.find_seams(frames, scale_log2=args.k)          # warm-up (module load, first touch)
    ts = []
    for _ in range(args.reps):
        t = time.perf_counter()
        plan.find_seams(frames, scale_log2=args.k)
        ts.append(time.perf_counter() - t)
    lab = plan.seam_labels()
    line = {"metric": "graph-cut seams per plan (C4: 8 x 1920x1080 cylinder, 1/%d grid)" % (1 << args.k),
            "ms_per_plan": round(float(np.median(ts)) * 1e3, 2), "reps": args.reps,
            "grid": list(lab.shape),
            "max_flow": "host Dinic" if os.environ.get("MCS_SEAM_FLOW") == "host" else
                        "device push-relabel",
            "stats_pairs_push_relabel_globalrelabels_us": plan.seam_stats()}
    if not args.no_check:
        from oracle import oracle
        _, want = oracle.blend_stitch_cyl(cams, g["out_w"], g["out_h"], g["f_cyl"], g["u0"],
                                          g["v0"], frames, 2, seam_k=args.k, want_seams=True)
        line["labels_equal_oracle"] = bool(np.array_equal(lab, want))
    print(json.dumps(line))


if __name__ == "__main__":
    main()
