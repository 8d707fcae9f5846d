"""Per-dispatch statistics of the bench's TIMED launches from a rocprofv3 kernel trace.

    python tools/trace_stats.py <rocprofv3 output dir | kernel_trace.csv> [--bench-line line.json]
                                [--out x.json] [--trim trimmed.csv]

The bench run must set MCS_BENCH_MARKERS=1: bench.py then launches a tiny spin kernel on its
stream right before the first and right after the last timed launch of the main plan, and the
same around the paste-only reference launches.  Only mcs_* dispatches between a pair of markers
count (calibration stitches, plan preparation, warm-up and the parity check are excluded).

Per window: every mcs_* kernel's dispatch count, mean / median / min / max duration (us); per
launch the span from its first dispatch's start to its last dispatch's end (the same quantity
the bench's HIP events bracket, minus event overhead).  With --bench-line (the JSON line of the
same run) the roofline fractions are recomputed from those spans and the line's algorithmic
bytes (SURVEY.md 8d B_frame and the touched-pixel figure).  --trim writes the raw trace rows
(every column) of the dispatches inside the marker windows, markers included: the committed
record of the timed launches.
"""
import argparse
import csv
import glob
import json
import os
from statistics import mean, median

HBM_PEAK = 8000.0


def load(d):
    """Dispatches (start, end, name) of a rocprofv3 output directory or one kernel_trace.csv."""
    rows = []
    files = [d] if os.path.isfile(d) else glob.glob(os.path.join(d, "**", "*kernel_trace.csv"),
                                                     recursive=True)
    for f in files:
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def windows(rows):
    """(start, end) of each marker pair, in trace order."""
    ts = [r for r in rows if "spin" in r[2].lower() or "sleep" in r[2].lower()]
    return [(ts[i][1], ts[i + 1][0]) for i in range(0, len(ts) - 1, 2)]


def launches(disp, steps):
    """Split a window's dispatches (start-time order) into its `steps` launches: consecutive
    launches do not overlap (each one's first kernel waits for the previous one's join), so equal
    consecutive chunks when the count divides; otherwise a launch starts at each dispatch of the
    window's first kernel name."""
    if not disp:
        return []
    if steps and len(disp) % steps == 0:
        k = len(disp) // steps
        return [disp[i:i + k] for i in range(0, len(disp), k)]
    first = disp[0][2]
    out, cur = [], []
    for d in disp:
        if d[2] == first and cur:
            out.append(cur)
            cur = []
        cur.append(d)
    out.append(cur)
    return out


def summarize(disp):
    per = {}
    for s, e, n in disp:
        per.setdefault(n, []).append((e - s) / 1e3)
    return {n: {"dispatches": len(v), "mean_us": round(mean(v), 2), "median_us": round(median(v), 2),
                "min_us": round(min(v), 2), "max_us": round(max(v), 2)}
            for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))}


def trim(d, wins, out):
    """The raw kernel_trace.csv rows whose dispatch lies inside one of the windows (or is one of
    their markers), in start-time order."""
    files = [d] if os.path.isfile(d) else glob.glob(os.path.join(d, "**", "*kernel_trace.csv"),
                                                     recursive=True)
    keep, fields = [], None
    for f in files:
        rd = csv.DictReader(open(f))
        fields = fields or rd.fieldnames
        for r in rd:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if any(t0 - 10**6 <= s and e <= t1 + 10**6 for t0, t1 in wins):
                keep.append(r)
    keep.sort(key=lambda r: int(r["Start_Timestamp"]))
    with open(out, "w", newline="") as fo:
        w = csv.DictWriter(fo, fieldnames=fields)
        w.writeheader()
        w.writerows(keep)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--bench-line")
    ap.add_argument("--out")
    ap.add_argument("--trim")
    a = ap.parse_args()
    rows = load(a.trace_dir)
    line = json.load(open(a.bench_line)) if a.bench_line else None
    steps = line["steps"] if line else None
    res = {"trace": os.path.relpath(a.trace_dir), "windows": []}
    for wi, (t0, t1) in enumerate(windows(rows)):
        disp = [r for r in rows if r[0] >= t0 and r[1] <= t1 and r[2].startswith("mcs_")]
        ls = launches(disp, steps)
        spans = [max(x[1] for x in l) - min(x[0] for x in l) for l in ls]
        w = {"window": ["timed launches (main plan)", "paste-only reference launches"][min(wi, 1)],
             "launches": len(ls), "launch_span_us_mean": round(mean(spans) / 1e3, 2) if spans else None,
             "kernels": summarize(disp)}
        if line and spans:
            rf = line["roofline"]
            ms = mean(spans) / 1e6
            b = rf["algorithmic_bytes_per_launch"]
            bt = rf.get("touched", {}).get("algorithmic_bytes_per_launch")
            w["frac_bframe"] = round(b / (ms * 1e-3) / 1e9 / HBM_PEAK, 4)
            if bt:
                w["frac_touched"] = round(bt / (ms * 1e-3) / 1e9 / HBM_PEAK, 4)
        res["windows"].append(w)
    if line:
        rf = line["roofline"]
        res["bench_line"] = {"kernel_ms_per_launch": rf["kernel_ms_per_launch"], "frac": rf["frac"],
                             "stream_kernel": rf.get("stream_kernel"),
                             "build_id": rf.get("build_id")}
    if a.trim:
        trim(a.trace_dir, windows(rows), a.trim)
    txt = json.dumps(res, indent=1)
    if a.out:
        open(a.out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
