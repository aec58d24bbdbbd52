#!/usr/bin/env python3
"""Inter-kernel gaps between library conv launches issued back to back (no host work in between beyond the ctypes
call): alternating a level-2 persistent forward and a level-0 halo forward, 30 launches; run under rocprofv3
--kernel-trace and summarise with gap_summary-style pairing (printed by --summary <trace.csv>)."""
import csv
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run():
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd import ops
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(1)
    x0 = torch.randn(4, 1024, 1024, 64, generator=g).to(dev, torch.bfloat16)
    w0 = (torch.randn(64, 576, generator=g) * 0.03).to(dev, torch.bfloat16)
    o0 = torch.empty(4, 1024, 1024, 64, dtype=torch.bfloat16, device=dev)
    x2 = torch.randn(4, 256, 256, 256, generator=g).to(dev, torch.bfloat16)
    w2 = (torch.randn(256, 2304, generator=g) * 0.03).to(dev, torch.bfloat16)
    o2 = torch.empty(4, 256, 256, 256, dtype=torch.bfloat16, device=dev)
    a1 = torch.empty_like(x0)
    sc = torch.ones(64, device=dev)
    st = torch.zeros(6, 64, device=dev)
    for rep in range(2):
        torch.cuda.synchronize()
        for i in range(15):
            ops.conv_fwd(x0, w0, 64, out=o0)
            ops.conv_fwd(x2, w2, 256, out=o2)
        for i in range(10):   # elementwise between convs
            ops.bn_apply(x0, sc, sc, a1)
            ops.conv_fwd(a1, w0, 64, out=o0)
        # phase 2: with the bench's per-launch event timing
        timer = ops.LaunchTimer()
        ops.set_launch_timer(timer)
        for i in range(10):
            ops.conv_fwd(x0, w0, 64, out=o0)
            ops.conv_fwd(x2, w2, 256, out=o2)
        ops.set_launch_timer(None)
        timer.summary()
        # phase 3: statistics in the epilogue, deferred fold + finalize (the training forward's sequence)
        for i in range(10):
            ops.conv_fwd(a1, w0, 64, out=o0, bn_stats=(st[0], st[1]), defer_fold=True)
            ops.bn_finalize(4 * 1024 * 1024, st[0], st[1], sc, sc, 1e-3, 0.01, st[2], st[3], st[4], st[5], None,
                            None, fold=True)
            ops.bn_apply(o0, st[2], st[3], a1)
        torch.cuda.synchronize()


def summary(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    pairs = {}
    for a, b in zip(rows, rows[1:]):
        ka = a["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-40:]
        kb = b["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-40:]
        pairs.setdefault((ka, kb), []).append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
    for (x, y), gaps in sorted(pairs.items(), key=lambda kv: -len(kv[1])):
        print(f"{x:>40} -> {y:<40} n={len(gaps):3d} gap median {statistics.median(gaps):7.2f} us  min {min(gaps):6.2f}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        summary(sys.argv[2])
    else:
        run()
