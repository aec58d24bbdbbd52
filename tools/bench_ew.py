#!/usr/bin/env python3
"""Microbenchmark of the bandwidth-bound (non-GEMM) kernels of the unet_bn L5 / 1024^2 / B=4 bf16 step at
their level-0 / level-1 shapes, HIP-event timed, with the algorithmic HBM bytes of each (operands read
once, outputs written once) and the achieved GB/s. Native-option variants interleave in one process
(';'-separated, each a ','-separated list of name=value); library builds A/B through tools/ab_libs.sh.

    python tools/bench_ew.py --ops head_bwd_bnr,pool_bwd_bnr
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
    p.add_argument("--variants", default="")
    p.add_argument("--ops", default="head_bwd_bnr,pool_bwd_bnr,bn_bwd_apply,bn_apply,bn_apply_pool")
    p.add_argument("--levels", default="0,1")
    p.add_argument("--batch", type=int, default=4)
    args = p.parse_args()
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd import ops

    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    settings = [[(kv.split("=")[0], int(kv.split("=")[1])) for kv in v.split(",") if kv]
                for v in args.variants.split(";")]
    keys = {k for st in settings for k, _ in st}
    print(json.dumps({"variants": {f"v{i}": v for i, v in enumerate(args.variants.split(";"))}}), flush=True)
    B = args.batch
    for lev in [int(x) for x in args.levels.split(",")]:
        S, C = 1024 >> lev, 64 << lev
        g = torch.Generator(device=dev).manual_seed(lev)
        t = lambda *sh: torch.randn(*sh, device=dev, generator=g).to(bf)   # noqa: E731
        z, dA, add, out, act = t(B, S, S, C), t(B, S, S, C), t(B, S, S, C), t(B, S, S, C), t(B, S, S, C)
        dpool, pool = t(B, S // 2, S // 2, C), t(B, S // 2, S // 2, C)
        vec = lambda: torch.rand(C, device=dev, generator=g) + 0.5   # noqa: E731
        sc, sh, mu, ist, gam = vec(), vec() - 1.0, vec() - 1.0, vec(), vec()
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        M = B * S * S
        pr = torch.rand(M, device=dev, generator=g)
        dpr = torch.randn(M, device=dev, generator=g)
        Wh, gw, gb = torch.randn(C, device=dev, generator=g) * 0.1, torch.zeros(C, device=dev), torch.zeros(1, device=dev)
        E = M * C * 2   # bytes of one full-resolution bf16 map
        table = {
            "head_bwd_bnr": (lambda: ops.head_bwd(z, Wh, pr, dpr, gw, gb, cin=C, softmax2=False, dx=out, bn=(sc, sh),
                                                  bn_reduce=(mu, ist, dg, db)), 2 * E + 8 * M),
            "head_bwd_bnr_nodx": (lambda: ops.head_bwd(z, Wh, pr, dpr, gw, gb, cin=C, softmax2=False, dx=None,
                                                       bn=(sc, sh), bn_reduce=(mu, ist, dg, db)), E + 8 * M),
            "bn_bwd_apply_head": (lambda: ops.bn_bwd_apply_head(Wh, pr, dpr, z, sc, sh, mu, ist, gam, dg, db, float(M),
                                                                out, cin=C), 2 * E + 8 * M),
            "pool_bwd_bnr": (lambda: ops.maxpool2_bwd(act, dpool, out, addend=add,
                                                      bn_reduce=(z, sc, sh, mu, ist, dg, db)), 3 * E + E // 4),
            "pool_bwd_bnr_src": (lambda: ops.maxpool2_bwd(act, dpool, out, addend=add, argmax_from_z=False,
                                                          bn_reduce=(z, sc, sh, mu, ist, dg, db)), 4 * E + E // 4),
            "bn_bwd_apply": (lambda: ops.bn_bwd_apply(dA, z, sc, sh, mu, ist, gam, dg, db, float(M), out), 3 * E),
            "bn_apply": (lambda: ops.bn_apply(z, sc, sh, out), 2 * E),
            "bn_apply_pool": (lambda: ops.bn_apply_maxpool2(z, sc, sh, act, pool), 2 * E + E // 4),
        }
        res = {}
        for r in range(args.rounds):
            for v, st in enumerate(settings):
                for k_ in keys:
                    ops.set_option(k_, None)
                for k_, v_ in st:
                    ops.set_option(k_, v_)
                for name in args.ops.split(","):
                    fn = table[name][0]
                    fn()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.reps):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    res.setdefault((name, v), []).append(e0.elapsed_time(e1) / args.reps)
        for name in args.ops.split(","):
            line = {"level": lev, "op": name, "bytes": table[name][1]}
            for v in range(len(settings)):
                ms = min(res[(name, v)])
                line[f"v{v}_us"] = round(ms * 1e3, 1)
                line[f"v{v}_GBps"] = round(table[name][1] / ms / 1e6, 1)
            print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
