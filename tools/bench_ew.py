#!/usr/bin/env python3
"""HBM-bound pass micro-benchmark (GPU box): BatchNorm apply / backward-apply / backward-reduce and the
2x2 max-pool at the unet_bn L5 1024^2 B=4 level shapes. Prints one JSON line per (op, level) with the
average launch time and the achieved HBM rate on the op's minimum traffic.
usage: python tools/bench_ew.py [--reps 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--batch", type=int, default=4)
    p.add_argument("--opt", action="append", default=[], help="name=value native option (repeatable)")
    p.add_argument("--ops", default="", help="comma list of ops to run (default all)")
    args = p.parse_args()
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd import ops

    dev = "cuda"
    B = args.batch
    for o in args.opt:
        k, v = o.split("=")
        ops.set_option(k, int(v))
    only = set(args.ops.split(",")) if args.ops else None

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.reps

    for lvl in range(5):
        H = 1024 >> lvl
        C = 64 << lvl
        z = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        dA = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        out = torch.empty_like(z)
        vec = lambda v=1.0: torch.full((C,), v, device=dev, dtype=torch.float32)  # noqa: E731
        sc, sh, mean, inv = vec(1.1), vec(0.05), vec(0.01), vec(0.9)
        gamma, dg, db = vec(1.0), vec(0.3), vec(0.2)
        n = z.numel()
        rows = [
            ("bn_apply", lambda: ops.bn_apply(z, sc, sh, out), 4 * n),
            ("bn_bwd_apply", lambda: ops.bn_bwd_apply(dA, z, sc, sh, mean, inv, gamma, dg, db, B * H * H, out), 6 * n),
            ("bn_bwd_reduce", lambda: ops.bn_bwd_reduce(dA, z, sc, sh, mean, inv, dg, db), 4 * n),
        ]
        if lvl < 4:
            pooled = torch.empty(B, H // 2, H // 2, C, device=dev, dtype=torch.bfloat16)
            rows.append(("maxpool_fwd", lambda: ops.maxpool2_fwd(z, pooled), 2 * n + 2 * n // 4))
        for name, fn, nbytes in rows:
            if only and name not in only:
                continue
            ms = timed(fn)
            print(json.dumps({"op": name, "level": lvl, "shape": [B, H, H, C], "ms": round(ms, 4),
                              "TB_s": round(nbytes / ms / 1e9, 3), "opts": args.opt}), flush=True)
        del z, dA, out


if __name__ == "__main__":
    main()
