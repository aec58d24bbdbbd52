#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc / --kernel-trace CSVs per kernel (our kernels only).

usage: python tools/pmc_summary.py DIR [prefix ...]
Reads DIR/<prefix>_counter_collection.csv for every prefix (default: all in DIR) and
DIR/*_kernel_trace.csv, groups dispatches by (kernel short name, grid size) and prints per-dispatch
means plus derived ratios:
  lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  wait/issue/active = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
  clock_GHz = GRBM_GUI_ACTIVE / 8 / duration
  fetch_GB / write_GB: FETCH_SIZE (x2, gfx950 wide-read correction) and WRITE_SIZE, KiB -> GB
"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.search(r"(\w+_kernel)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main():
    d = sys.argv[1]
    prefixes = sys.argv[2:]
    files = [os.path.join(d, f"{p}_counter_collection.csv") for p in prefixes] if prefixes else \
        glob.glob(os.path.join(d, "*_counter_collection.csv"))
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in files:
        for r in csv.DictReader(open(f)):
            if "adipose" in r["Kernel_Name"] or "at::native" in r["Kernel_Name"]:
                continue
            key = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            acc[key]["_dur_" + r["Counter_Name"]].append(dur)
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "*_kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            gs = int(r.get("Grid_Size") or int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]))
            dur[(short(r["Kernel_Name"]), gs)].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    for key in sorted(acc):
        c = {k: sum(v) / len(v) for k, v in acc[key].items()}
        out = [f"{key[0]:<44} grid={key[1]:<8}"]
        if key in dur:
            out.append(f"t={1e3 * sorted(dur[key])[len(dur[key]) // 2]:.3f}ms")
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if n in c:
                    out.append(f"{n[3:].lower()}={c[n] / wc:.2f}")
        if c.get("SQ_LDS_IDX_ACTIVE"):
            out.append(f"lds_conflict={c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_LDS_IDX_ACTIVE']:.3f}")
        if "GRBM_GUI_ACTIVE" in c:
            out.append(f"clock={c['GRBM_GUI_ACTIVE'] / 8 / c['_dur_GRBM_GUI_ACTIVE'] / 1e9:.2f}GHz")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                out.append(f"mfma_busy/(gui*128)={c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['GRBM_GUI_ACTIVE'] * 128):.3f}")
        if "FETCH_SIZE" in c:
            out.append(f"fetch={2 * c['FETCH_SIZE'] * 1024 / 1e9:.3f}GB")
        if "WRITE_SIZE" in c:
            out.append(f"write={c['WRITE_SIZE'] * 1024 / 1e9:.3f}GB")
        print(" ".join(out))


if __name__ == "__main__":
    main()
