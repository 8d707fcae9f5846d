"""Summarise tools/experiments/gpu_pmc_c3.sh: per kernel family of the C3 estimation path, dispatches and
per-dispatch counter averages, HBM bytes (FETCH_SIZE x 2 per the gfx950 correction + WRITE_SIZE)
and the derived ratios of pmc_summary.  Writes profiles/r02_pmc_c3.json (argv[1] overrides)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MCS_PMC_DIR", os.path.join(ROOT, "gpurun_out", "pmc_c3"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_summary as ps  # noqa: E402

FAMILIES = ["mcs_orb_gray", "mcs_resize", "mcs_orb_pyramid", "mcs_orb_level", "mcs_orb_select",
            "mcs_orb_describe", "mcs_hamming_knn2", "mcs_ransac", "mcs_rig_knn2", "mcs_rig_match",
            "mcs_rig_ransac", "mcs_rig_best", "mcs_direct"]


def main(out):
    sys.path.insert(0, ROOT)
    from multicamera_stitching_amd import _capi
    args = os.environ.get("C3_ARGS", "--steps 10 --warmup 2 --threads 1")
    res = {"workload": "C3: tools/estimate_bench.py " + args +
                       " (4 x 1080p ORB 2000 features, 3 pairs kNN-2 + RANSAC per capture"
                       + (", stitched" if "--stitch" in args else "") + ")",
           "build_id": _capi.build_id(), "per_kernel": {}}
    for fam in FAMILIES:
        avg = ps.family_counters(fam)
        _, n = ps.family_counters(fam, totals=True)
        if not avg:
            continue
        d = ps.derived(avg)
        d["dispatches"] = n
        d["counters_per_dispatch"] = avg
        res["per_kernel"][fam] = d
    text = json.dumps(res, indent=1, sort_keys=True)
    print(text)
    with open(out, "w") as f:
        f.write(text + "\n")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r02_pmc_c3.json"))
