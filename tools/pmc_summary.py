"""Summarise tools/gpu_pmc.sh output: per-launch averages of every counter for the streaming
kernel, HBM bytes per launch (FETCH_SIZE x 2 per the gfx950 correction in MI355X_MICROARCH.md,
+ WRITE_SIZE; both KiB-denominated) and from the sized read-request counts, derived ratios.  Writes profiles/pmc_latest.json (read by
bench.py's roofline.traffic when the workload matches) and prints a text summary."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PMC = os.environ.get("MCS_PMC_DIR", os.path.join(ROOT, "gpurun_out", "pmc"))


def _window_start(rows):
    """First dispatch of the bench's own launches in one pass: after the last plan prepare
    (mcs_prepare_* / mcs_cyl_prepare_*).  Earlier stitch dispatches belong to the Stitcher's
    calibration (its own small plans) and are not bench launches."""
    last = -1
    for r in rows:
        if "prepare" in r["Kernel_Name"]:
            last = max(last, int(r["Dispatch_Id"]))
    return last + 1


def family_counters(prefix, totals=False):
    """Per-dispatch averages of every counter over the bench-launch dispatches of kernels named
    prefix* (totals=True: (sum over the dispatches, dispatches per pass))."""
    vals = defaultdict(lambda: defaultdict(float))     # (pass, dispatch) -> counter -> value
    for f in sorted(glob.glob(os.path.join(PMC, "pass*", "**", "*counter_collection.csv"),
                              recursive=True)):
        p = f.split(os.sep)[len(PMC.split(os.sep))]
        rows = list(csv.DictReader(open(f)))
        start = _window_start(rows)
        for r in rows:
            if not r["Kernel_Name"].startswith(prefix) or int(r["Dispatch_Id"]) < start:
                continue
            vals[(p, int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
    per_counter = defaultdict(list)
    passes = defaultdict(int)
    for (p, _), cs in vals.items():
        passes[p] += 1
        for c, v in cs.items():
            per_counter[c].append(v)
    if totals:
        n = max(passes.values()) if passes else 0
        return {c: sum(v) * n / max(len(v), 1) for c, v in per_counter.items()}, n
    return {c: sum(v) / len(v) for c, v in per_counter.items()}


def derived(avg):
    res = {}
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        fetch = avg["FETCH_SIZE"] * 1024 * 2
        write = avg["WRITE_SIZE"] * 1024
        res.update(fetch_bytes=fetch, write_bytes=write, hbm_bytes=int(fetch + write))
    if "TCC_EA0_RDREQ_sum" in avg and "TCC_EA0_RDREQ_128B_sum" in avg:
        # read bytes from the sized request counts (32 / 64 / 128-B requests of the L2's memory
        # side): no width assumption, unlike FETCH_SIZE x 2 (which is exact only when every
        # request is 128 B)
        n, n64, n128 = (avg["TCC_EA0_RDREQ_sum"], avg["TCC_EA0_RDREQ_64B_sum"],
                        avg["TCC_EA0_RDREQ_128B_sum"])
        sized = 128 * n128 + 64 * n64 + 32 * max(n - n64 - n128, 0)
        res.update(read_bytes_sized=sized, read_req_128b_frac=n128 / max(n, 1),
                   read_req_64b_frac=n64 / max(n, 1))
        if "WRITE_SIZE" in avg:
            res["hbm_bytes_sized"] = int(sized + avg["WRITE_SIZE"] * 1024)
    if "SQ_WAVE_CYCLES" in avg:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS"):
            if c in avg:
                res[c + "_frac"] = avg[c] / avg["SQ_WAVE_CYCLES"]
    if "SQ_WAVES" in avg:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM"):
            if c in avg:
                res[c + "_per_wave"] = avg[c] / avg["SQ_WAVES"]
    if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_LDS_IDX_ACTIVE" in avg:
        res["lds_bank_conflict_frac"] = avg["SQ_LDS_BANK_CONFLICT"] / max(avg["SQ_LDS_IDX_ACTIVE"], 1)
    if "TCC_HIT_sum" in avg:
        res["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"], 1)
    return res


def main(prefixes=("mcs_stream_c3",), workload=None, out=None, launches=None):
    """Launches = the bench launches of each counter pass (tools/gpu_pmc.sh: --steps 3 --warmup 1
    = 4, $MCS_PMC_LAUNCHES overrides; the PMC runs use bench.py --no-paste-ref so only the
    measured plan dispatches, and a multi-band launch streams its tiles in two dispatches); HBM
    bytes per launch = every family's FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE over its
    dispatches, / launches."""
    if launches is None:
        launches = int(os.environ.get("MCS_PMC_LAUNCHES", "4"))
    sys.path.insert(0, ROOT)
    from multicamera_stitching_amd import _capi
    # the kernels these counters belong to: bench.py reports "traffic" only for this build
    res = {"kernels": list(prefixes), "workload": workload, "build_id": _capi.build_id(),
           "per_kernel": {}}
    total = total_sized = 0
    res["launches_per_pass"] = launches
    for pre in prefixes:
        avg = family_counters(pre)
        tot, n = family_counters(pre, totals=True)
        d = derived(avg)
        d["counters_per_dispatch"] = avg
        d["dispatches_per_launch"] = n / launches
        per_launch = derived({c: v / launches for c, v in tot.items()})
        d["hbm_bytes_per_launch"] = per_launch.get("hbm_bytes")
        d["hbm_bytes_sized_per_launch"] = per_launch.get("hbm_bytes_sized")
        res["per_kernel"][pre] = d
        total += per_launch.get("hbm_bytes", 0)
        total_sized += per_launch.get("hbm_bytes_sized", 0)
    res["hbm_bytes_per_launch"] = int(total) if total else None
    res["hbm_bytes_sized_per_launch"] = int(total_sized) if total_sized else None
    text = json.dumps(res, indent=1, sort_keys=True)
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    wl = sys.argv[1] if len(sys.argv) > 1 else "4x1920x1080x3-linear-super0-F64-multiband"
    kernels = (sys.argv[2].split(",") if len(sys.argv) > 2
               else ["mcs_stream_c3", "mcs_mb_bands", "mcs_mb_levels_c3", "mcs_mb_blend_c3"])
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "profiles", "pmc_latest.json")
    main(prefixes=kernels, workload=wl, out=out)
