#!/usr/bin/env python3
"""Whole-step sweep of native options in ONE process (unet_bn bench step, or --preset adipose_v3): arms are
';'-separated option lists (name=value,...; "base" = defaults), run round-robin so that box drift hits every arm
alike; every arm first resets all options any arm names. Prints ms/step per round, min and median per arm."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--arms", required=True)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--steps", type=int, default=8)
    p.add_argument("--preset", default="unet_bn", choices=["unet_bn", "adipose_v3"])
    p.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    args = p.parse_args()
    import numpy as np
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd import ops
    from adipose_amd.data import synthetic_batch
    from adipose_amd.nets import UNetBN
    from adipose_amd.trainer import LossConfig, Trainer
    dev = torch.device("cuda", 0)
    if args.preset == "adipose_v3":
        from adipose_amd.data import to_gray
        from adipose_amd.nets import AdiposeV3Net
        B = 2
        net = AdiposeV3Net(B, 1024, dtype=args.dtype, device=dev, seed=865)
        tr = Trainer(net, LossConfig(), lr=1e-4)
        xs, ys = synthetic_batch(B, 1024, channels=3, seed=865)
        xs = to_gray(xs.astype("float32"))
    else:
        B = 4
        net = UNetBN(B, 1024, levels=5, base=64, in_ch=3, dtype=args.dtype, device=dev, seed=865)
        tr = Trainer(net, LossConfig(use_hard_mining=False), lr=1e-4)
        xs, ys = synthetic_batch(B, 1024, channels=3, seed=865)
    x = torch.from_numpy(((xs - xs.mean()) / (xs.std() + 1e-10)).astype(np.float32)).to(dev)
    y = torch.from_numpy(ys).to(dev)
    arms = [a.strip() for a in args.arms.split(";")]
    parsed = [[(kv.split("=")[0], int(kv.split("=")[1])) for kv in a.split(",") if kv and a != "base"] for a in arms]
    names = sorted({k for arm in parsed for k, _ in arm})

    def apply(i):
        for n in names:
            ops.set_option(n, None)
        for k, v in parsed[i]:
            ops.set_option(k, v)

    for i in range(len(arms)):
        apply(i)
        for _ in range(2):
            tr.train_step(x, y)
    res = [[] for _ in arms]
    for _ in range(args.rounds):
        for i in range(len(arms)):
            apply(i)
            tr.train_step(x, y)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                tr.train_step(x, y)
            torch.cuda.synchronize()
            res[i].append((time.perf_counter() - t0) / args.steps * 1e3)
    apply(0)
    base = sorted(res[0])[len(res[0]) // 2]
    for a, r in zip(arms, res):
        med = sorted(r)[len(r) // 2]
        print(f"{a:50s} ms/step {[round(t, 3) for t in r]} min {min(r):.3f} median {med:.3f} ({(med / base - 1) * 100:+.2f} %)",
              flush=True)


if __name__ == "__main__":
    main()
