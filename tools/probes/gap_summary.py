#!/usr/bin/env python3
"""Summarise gap_probe's kernel trace: per (writer cache policy, MB written) the writer's duration and the gap from its
end to the start of the tiny kernel that follows it (median over repetitions)."""
import csv
import statistics
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sizes = [0, 4, 16, 64, 256, 1024]
    res = {}
    i = 0
    k = 0
    seq = []
    while i + 1 < len(rows):
        a, b = rows[i], rows[i + 1]
        if "writer" in a["Kernel_Name"] and "tiny" in b["Kernel_Name"]:
            aux = a["Kernel_Name"].split("writer<")[1].split(">")[0]
            seq.append((aux, int(a["End_Timestamp"]) - int(a["Start_Timestamp"]),
                        int(b["Start_Timestamp"]) - int(a["End_Timestamp"])))
            i += 2
        else:
            i += 1
    for j, (aux, dur, gap) in enumerate(seq):
        mb = sizes[(j // 5) % len(sizes)]
        res.setdefault((aux, mb), []).append((dur, gap))
    # every consecutive pair that involves a fat kernel: (first, second) -> gaps
    pairs = {}
    for a, b in zip(rows, rows[1:]):
        if "fat" in a["Kernel_Name"] or "fat" in b["Kernel_Name"]:
            key = (a["Kernel_Name"].split("(")[0][-24:], b["Kernel_Name"].split("(")[0][-24:])
            pairs.setdefault(key, []).append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
    for (x, y), g in pairs.items():
        print(f"{x:>24} -> {y:<24} gap median {statistics.median(g):6.2f} us (n={len(g)})")
    print(f"{'aux':>4} {'MB':>5} {'writer us':>10} {'gap us':>8} {'GB/s':>8}")
    for (aux, mb), v in sorted(res.items(), key=lambda kv: (int(kv[0][0]), kv[0][1])):
        d = statistics.median(x[0] for x in v) / 1e3
        g = statistics.median(x[1] for x in v) / 1e3
        print(f"{aux:>4} {mb:>5} {d:10.1f} {g:8.2f} {mb * 1.048576e3 / d if d else 0:8.0f}")


if __name__ == "__main__":
    main(sys.argv[1])
