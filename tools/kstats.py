"""Print the mcs_* kernels of a rocprofv3 --kernel-trace --stats directory: calls, average and
median duration (us), share of the total."""
import csv
import glob
import os
import sys
from collections import defaultdict
from statistics import median

d = sys.argv[1]
trace = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
dur = defaultdict(list)
for f in trace:
    for r in csv.DictReader(open(f)):
        dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in dur.values())
for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    if not n.startswith("mcs_"):
        continue
    print(f"{n[:34]:34s} calls {len(v):5d} avg {sum(v)/len(v):9.1f} med {median(v):9.1f} "
          f"share {100*sum(v)/tot:5.1f}%")
