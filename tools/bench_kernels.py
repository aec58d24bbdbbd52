#!/usr/bin/env python3
"""Per-layer conv kernel microbenchmark (A/B of kernel variants in ONE process, interleaved rounds).

For the unet_bn L5 / 1024^2 / B=4 layer shapes: forward, data-gradient and weight-gradient launches,
timed with HIP events; reports TFLOP/s per variant. A variant is a comma-separated list of native
options (ops.set_option), variants are separated by ';', e.g.
  --variants "conv_fast=2,fwd_tap64=0;fwd_tap64=1;fwd_tap64=2"
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--variants", default="conv_fast=2,fwd_tap64=0;conv_fast=2,fwd_tap64=1")
    p.add_argument("--kinds", default="fwd,wgrad", help="fwd, fwd_stats, bnr (data gradient with the fused "
                   "BatchNorm-backward reduction), wgrad")
    p.add_argument("--layers", default="", help="comma-separated substrings selecting layer shapes")
    p.add_argument("--batch", type=int, default=4)
    p.add_argument("--blas", action="store_true",
                   help="add a hipBLASLt (torch.matmul) dense GEMM of the same M x N x K as a reference arm")
    args = p.parse_args()
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd import ops

    dev = torch.device("cuda", 0)
    B = args.batch
    # (name, S, Cin, Cout): 3x3 convs of unet_bn L5 (one per (level, shape) class)
    shapes = [("L0 64->64", 1024, 64, 64), ("L0 128->64", 1024, 128, 64), ("L1 128->128", 512, 128, 128),
              ("L2 256->256", 256, 256, 256), ("L3 512->512", 128, 512, 512), ("L4 1024->1024", 64, 1024, 1024),
              ("L3 1024->512", 128, 1024, 512), ("L4 1024->512", 64, 1024, 512), ("L1 256->128", 512, 256, 128),
              ("L0 in8->64", 1024, 8, 64)]   # the input layer (8-channel source: cin8 kernels)
    if args.layers:
        keys = args.layers.split(",")
        shapes = [sh for sh in shapes if any(k in sh[0] for k in keys)]
    variants = list(range(len(args.variants.split(";"))))
    settings = [[(kv.split("=")[0], int(kv.split("=")[1])) for kv in v.split(",") if kv]
                for v in args.variants.split(";")]
    kinds = args.kinds.split(",")
    print(json.dumps({"variants": {f"v{i}": args.variants.split(";")[i] for i in variants}}), flush=True)
    res = {}
    for name, S, cin, cout in shapes:
        K = 9 * cin
        Kpad = (K + 31) // 32 * 32
        x = torch.randn(B, S, S, cin, device=dev).to(torch.bfloat16)
        W = (torch.randn(((cout + 63) // 64 * 64), Kpad, device=dev) * 0.02).to(torch.bfloat16)
        y = torch.empty(B, S, S, cout, device=dev, dtype=torch.bfloat16)
        dW = torch.zeros(((cout + 63) // 64 * 64), Kpad, device=dev)
        # BatchNorm operands: forward statistics (fwd_stats) and the data gradient's fused BN-backward
        # reduction (bnr: z = the pre-BN output of the layer below, same shape as y)
        st = (torch.zeros(cout, device=dev), torch.zeros(cout, device=dev))
        z = torch.randn(B, S, S, cout, device=dev).to(torch.bfloat16)
        vec = [torch.rand(cout, device=dev) + 0.5 for _ in range(4)]
        bnr = (z, vec[0], vec[1], vec[2], vec[3], torch.zeros(cout, device=dev), torch.zeros(cout, device=dev))
        flops = 2.0 * B * S * S * cout * K
        if args.blas:   # dense GEMM of the same shape: x2d (M x K) @ Wt (K x N), no im2col gather
            a2 = torch.randn(B * S * S, K, device=dev, dtype=torch.bfloat16)
            b2 = torch.randn(K, cout, device=dev, dtype=torch.bfloat16)
            for _ in range(3):
                a2 @ b2
            bl = []
        for kind in kinds:
            for v in variants:
                res.setdefault((name, kind, v), [])
        for r in range(args.rounds):
            for v in variants:
                for k_ in {kk for st in settings for kk, _ in st}:
                    ops.set_option(k_, None)      # every variant starts from the defaults
                for k_, v_ in settings[v]:
                    ops.set_option(k_, v_)
                if r == 0 and "fwd" in kinds:   # every variant's forward output against variant 0's
                    ops.conv_fwd(x, W, cout, out=y)
                    torch.cuda.synchronize()
                    if v == 0:
                        y0 = y.clone()
                    else:
                        d = (y.float() - y0.float()).abs().max().item()
                        print(json.dumps({"layer": name, "variant": v, "fwd_max_abs_diff_vs_v0": d}), flush=True)
                for kind in kinds:
                    fn = {"fwd": lambda: ops.conv_fwd(x, W, cout, out=y),
                          "fwd_stats": lambda: ops.conv_fwd(x, W, cout, out=y, bn_stats=st),
                          "bnr": lambda: ops.conv_fwd(x, W, cout, out=y, bn_reduce=bnr),
                          "wgrad": lambda: ops.conv_wgrad(x, y, dW, cout)}[kind]
                    fn()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.reps):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    ms = e0.elapsed_time(e1) / args.reps
                    res[(name, kind, v)].append(ms)
            if args.blas:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    a2 @ b2
                e1.record()
                torch.cuda.synchronize()
                bl.append(e0.elapsed_time(e1) / args.reps)
        if args.blas:
            ms = min(bl)
            print(json.dumps({"layer": name, "kind": "hipblaslt_gemm", "ms": round(ms, 4),
                              "tflops": round(flops / ms / 1e9, 1)}), flush=True)
            del a2, b2
        for kind in kinds:
            line = {"layer": name, "kind": kind}
            for v in variants:
                ms = min(res[(name, kind, v)])
                line[f"v{v}_ms"] = round(ms, 4)
                line[f"v{v}_tflops"] = round(flops / ms / 1e9, 1)
            print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
