#!/usr/bin/env python3
"""Per-kernel time breakdown from a rocprofv3 `--stats -f csv` kernel_stats file.

usage: python tools/kstats.py <prefix>_kernel_stats.csv [steps]
Prints each kernel's calls, mean duration and total per step (total / steps).
"""
import csv
import re
import sys


def short(name):
    m = re.search(r"(\w+_kernel)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:52]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    for r in rows:
        t = float(r["TotalDurationNs"])
        if t / tot < 0.002:
            continue
        print(f"{short(r['Name'])[:52]:<52} calls={int(r['Calls']):5d} avg={float(r['AverageNs']) / 1e3:9.1f}us "
              f"per_step={t / 1e6 / steps:7.2f}ms {100 * t / tot:5.1f}%")
    print(f"total per step: {tot / 1e6 / steps:.2f} ms")


if __name__ == "__main__":
    main()
