#!/usr/bin/env python3
"""ConvTranspose 2x2/s2 microbenchmark at the unet_bn L5 / 1024^2 / B=4 decoder shapes (dec{i}_up):
forward (1x1 GEMM + pixel-shuffle store), data gradient (stride-2 4-tap gather, optionally with the fused
BatchNorm-backward reduction) and weight gradient; variants of native options interleaved in ONE process
(';'-separated, each a ','-separated list of name=value), HIP-event timed. Reports ms, TFLOP/s and the
algorithmic HBM GB/s (operands read once, outputs written once).

    python tools/bench_convt.py --variants "fwd_tap64=1;fwd_tap64=5"
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
    p.add_argument("--variants", default="fwd_tap64=1")
    p.add_argument("--kinds", default="fwd,dgrad,dgrad_bnr,wgrad")
    p.add_argument("--batch", type=int, default=4)
    args = p.parse_args()
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd import ops

    dev = torch.device("cuda", 0)
    B = args.batch
    # (name, low-resolution size S, Cin (= ch(i+1)), Cout (= ch(i)))
    shapes = [("dec0_up", 512, 128, 64), ("dec1_up", 256, 256, 128), ("dec2_up", 128, 512, 256),
              ("dec3_up", 64, 1024, 512)]
    settings = [[(kv.split("=")[0], int(kv.split("=")[1])) for kv in v.split(",") if kv]
                for v in args.variants.split(";")]
    keys = {k for st in settings for k, _ in st}
    kinds = args.kinds.split(",")
    print(json.dumps({"variants": {f"v{i}": v for i, v in enumerate(args.variants.split(";"))}}), flush=True)
    for name, S, cin, cout in shapes:
        N = 4 * cout
        x = torch.randn(B, S, S, cin, device=dev).to(torch.bfloat16)                 # ConvT input
        Wf = (torch.randn(N, cin, device=dev) * 0.05).to(torch.bfloat16)           # [4*Cout][Cin]
        Wd = (torch.randn(cin + 0, 4 * cout, device=dev) * 0.05).to(torch.bfloat16)  # [Cin][4*Cout]
        t = torch.empty(B, 2 * S, 2 * S, cout, device=dev, dtype=torch.bfloat16)   # ConvT output
        dt = torch.randn(B, 2 * S, 2 * S, cout, device=dev).to(torch.bfloat16)
        dA = torch.empty(B, S, S, cin, device=dev, dtype=torch.bfloat16)
        z = torch.randn(B, S, S, cin, device=dev).to(torch.bfloat16)
        vec = [torch.rand(cin, device=dev) + 0.5 for _ in range(4)]
        dg, dbt = torch.zeros(cin, device=dev), torch.zeros(cin, device=dev)
        dW = torch.zeros(N, cin, device=dev)
        bias = torch.zeros(cout, device=dev)
        flops = 2.0 * B * S * S * cin * N
        nbytes = {"fwd": 2 * (x.numel() + t.numel()), "dgrad": 2 * (dt.numel() + dA.numel()),
                  "dgrad_bnr": 2 * (dt.numel() + dA.numel() + z.numel()), "wgrad": 2 * (x.numel() + dt.numel())}
        fns = {
            "fwd": lambda: ops.conv_fwd(x, Wf, N, out=t, bias=bias, kh=1, kw=1, pad=0, out_mode=1, shuffle_c=cout),
            "dgrad": lambda: ops.conv_fwd(dt, Wd, cin, out=dA, kh=2, kw=2, dil=1, pad=0, stride=2, Ho=S, Wo=S),
            "dgrad_bnr": lambda: ops.conv_fwd(dt, Wd, cin, out=dA, kh=2, kw=2, dil=1, pad=0, stride=2, Ho=S, Wo=S,
                                              bn_reduce=(z, vec[0], vec[1], vec[2], vec[3], dg, dbt)),
            "wgrad": lambda: ops.conv_wgrad(x, dt, dW, N, kh=1, kw=1, pad=0, shuffle_c=cout),
        }
        res = {}
        outs0 = {}
        for r in range(args.rounds):
            for v, st in enumerate(settings):
                for k_ in keys:
                    ops.set_option(k_, None)
                for k_, v_ in st:
                    ops.set_option(k_, v_)
                for kind in kinds:
                    fn = fns[kind]
                    if r == 0:   # outputs of every variant against variant 0 (forward / data gradient)
                        if kind == "wgrad":
                            ops.fill(dW, 0.0)
                        fn()
                        torch.cuda.synchronize()
                        o = {"fwd": t, "dgrad": dA, "dgrad_bnr": dA, "wgrad": dW}[kind].float().clone()
                        if v == 0:
                            outs0[kind] = o
                        else:
                            d = (o - outs0[kind]).abs().max().item() / max(outs0[kind].abs().max().item(), 1e-12)
                            print(json.dumps({"layer": name, "kind": kind, "variant": v, "rel_diff_vs_v0": d}),
                                  flush=True)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.reps):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    res.setdefault((kind, v), []).append(e0.elapsed_time(e1) / args.reps)
        for kind in kinds:
            line = {"layer": name, "kind": kind}
            for v in range(len(settings)):
                ms = min(res[(kind, v)])
                line[f"v{v}_ms"] = round(ms, 4)
                line[f"v{v}_tflops"] = round(flops / ms / 1e9, 1)
                line[f"v{v}_GBps"] = round(nbytes[kind] / ms / 1e6, 1)
                line[f"v{v}_kernel"] = None
            print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
