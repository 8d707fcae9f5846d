"""Timeline of the timed launches in a rocprofv3 kernel trace (bench run with MCS_BENCH_MARKERS=1):
per dispatch between the first pair of marker (spin) kernels its start / end relative to the
window's start and its duration, in microseconds.  python tools/timeline.py <trace dir> [n]"""
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from trace_stats import load   # noqa: E402


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    rows = load(d)
    marks = [i for i, r in enumerate(rows) if "spin_kernel" in r[2]]
    a, b = marks[0], marks[1]
    win = rows[a + 1:b]
    t0 = win[0][0]
    for s, e, name in win[-n:]:
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  {name[:48]}")


if __name__ == "__main__":
    main()
