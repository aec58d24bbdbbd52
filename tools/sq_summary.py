#!/usr/bin/env python3
"""Per-kernel SQ counter summary of a rocprofv3 --pmc pass (counter_collection.csv): sums per kernel name and the
ratios that say where a kernel's wave time goes. usage: python tools/sq_summary.py <counter_collection.csv> [top]"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    acc = defaultdict(lambda: defaultdict(float))
    seen = defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        d = int(r["Dispatch_Id"])
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if d not in seen[k]:
            seen[k].add(d)
            acc[k]["_ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    rows = sorted(acc.items(), key=lambda kv: -kv[1]["_ns"])[:top]
    for k, c in rows:
        n = len(seen[k])
        wave = c.get("SQ_WAVE_CYCLES", 0.0)
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        line = f"{k[:70]:70s} n={n:4d} avg {c['_ns'] / n / 1e3:8.1f} us"
        if gui:
            # MFMA busy per SIMD-cycle of the kernel (1024 SIMDs; GRBM_GUI_ACTIVE counts GPU cycles)
            line += f"  mfma_busy/simd_cycle {mf / (gui * 1024):.3f}"
        if wave:
            line += (f"  wait_any {c.get('SQ_WAIT_ANY', 0) / wave:.3f}  wait_inst {c.get('SQ_WAIT_INST_ANY', 0) / wave:.3f}"
                     f"  active_inst {c.get('SQ_ACTIVE_INST_ANY', 0) / wave:.3f}")
        print(line)


if __name__ == "__main__":
    main()
