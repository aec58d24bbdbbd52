#!/usr/bin/env python3
"""One steady-state training step from a rocprofv3 --kernel-trace CSV, launch by launch: duration, gap
to the previous launch's end, grid, and running time (the bench step is the block of launches that ends
at the last adam_kernel; the step before it is used so that the tail of the run is excluded).

usage: python tools/step_timeline.py <kt_kernel_trace.csv> [--step -2]
"""
import csv
import re
import sys


def short(name):
    m = re.search(r"(\w+_kernel)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main():
    path = sys.argv[1]
    which = int(sys.argv[sys.argv.index("--step") + 1]) if "--step" in sys.argv else -2
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    hi = ends[which]
    lo = ends[which - 1] + 1
    step = rows[lo:hi + 1]
    t0 = int(step[0]["Start_Timestamp"])
    prev_end = int(rows[lo - 1]["End_Timestamp"])
    busy = gaps = 0
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = s - prev_end
        busy += e - s
        gaps += max(gap, 0)
        print(f"{(s - t0) / 1e3:9.1f}us {(e - s) / 1e3:8.1f}us gap {gap / 1e3:6.1f}  grid {int(r['Grid_Size_X']):8d}  "
              f"{short(r['Kernel_Name'])[:70]}")
        prev_end = e
    print(f"launches {len(step)}  kernel time {busy / 1e6:.3f} ms  gaps {gaps / 1e6:.3f} ms  "
          f"span {(int(step[-1]['End_Timestamp']) - t0) / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
