"""Copies one tools/gpu_r05_final.sh (or r04 / r03) run's outputs from gpurun_out/ into profiles/<prefix>_*
(the committed record; gpurun_out/ is scratch).  Usage: python tools/save_record.py r03b_final"""
import glob
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G, P = os.path.join(ROOT, "gpurun_out"), os.path.join(ROOT, "profiles")
pre = sys.argv[1]


def cp(src, dst):
    s = os.path.join(G, src)
    if os.path.exists(s):
        shutil.copy(s, os.path.join(P, f"{pre}_{dst}"))
        print(src, "->", f"{pre}_{dst}")


def last_json(src, dst):
    s = os.path.join(G, src)
    if not os.path.exists(s):
        return
    lines = [ln for ln in open(s) if ln.startswith("{")]
    if lines:
        open(os.path.join(P, f"{pre}_{dst}"), "w").write(lines[-1])
        print(src, "->", f"{pre}_{dst}")


cp("bench_line.json", "bench_line.json")
cp("bench_line_paste.json", "bench_line_paste.json")
cp("bench_line_cyl.json", "bench_line_cylinder.json")
for n in ("mb", "paste", "cyl"):
    cp(f"trace_stats_{n}.json", f"trace_stats_{n}.json")
    cp(f"trace_{n}_line.json", f"trace_line_{n}.json")
    for f in glob.glob(os.path.join(G, f"trace_{n}", "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(P, f"{pre}_kernel_stats_{n}.csv"))
    cp(f"trace_{n}_trimmed.csv", f"kernel_trace_{n}.csv")   # (tools/trace_stats.py --trim)
cp("pmc_summary.txt", "pmc_summary.txt")
cp("pmc_latest.json", "pmc_latest.json")
cp("pmc_summary_cyl.txt", "pmc_summary_cyl.txt")
cp("pmc_latest_cyl.json", "pmc_latest_cyl.json")
for f in ("pmc_latest.json", "pmc_latest_cyl.json"):
    if os.path.exists(os.path.join(G, f)):
        shutil.copy(os.path.join(G, f), os.path.join(P, f))
last_json("c3_serial.log", "c3_serial.json")
last_json("c3_overlap.log", "c3_overlap_depth4.json")
last_json("c3_resident.log", "c3_resident_depth4.json")
last_json("c3_resident_pystitch.log", "c3_resident_depth4_python_stitch.json")
last_json("c3_estimate.log", "c3_estimate_only.json")
last_json("match.log", "match_bench.json")
last_json("seam.log", "seam_c4.json")
cp("stream.log", "stream_pipeline.jsonl")
cp("copy_probe.txt", "copy_probe.txt")
for f in glob.glob(os.path.join(G, "trace_c3", "**", "*kernel_stats.csv"), recursive=True):
    shutil.copy(f, os.path.join(P, f"{pre}_kernel_stats_c3.csv"))
s = os.path.join(G, "pytest_gpu.log")
if os.path.exists(s):
    tail = [ln for ln in open(s) if "passed" in ln or "failed" in ln][-1:]
    open(os.path.join(P, f"{pre}_gpu_tests_summary.txt"), "w").writelines(tail)
