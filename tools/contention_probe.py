#!/usr/bin/env python3
"""How the bench step (unet_bn L5, 1024^2, B=4, bf16) reacts to CUs held by another stream's kernel, as RCCL's
blocks hold CUs while the data-parallel step's gradient buckets are all-reduced (one GPU stands in: a
sleep-only kernel on a side stream, K blocks of 64 threads with 96 KiB of LDS each, so that none of the step's
persistent blocks can share their CU). Each sample: the side kernel (about `--spin-ms` long) is launched, then
one training step on the default stream; the step's wall time is compared with steps without it. A step that
only lost K of 256 CUs for the spin's duration grows by about spin_ms * K / 256; a persistent kernel whose
late blocks wait for a held CU grows by up to its own duration.
usage: python tools/contention_probe.py [--blocks 0,8,16,32,64] [--spin-ms 20] [--rounds 3]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--blocks", default="0,8,16,32,64")
    p.add_argument("--spin-ms", type=float, default=20.0)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--opt", action="append", default=[], help="name=value native option")
    args = p.parse_args()
    import numpy as np
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd.data import synthetic_batch
    from adipose_amd.nets import UNetBN
    from adipose_amd.trainer import LossConfig, Trainer

    from adipose_amd import ops
    for kv in args.opt:
        ops.set_option(kv.split("=")[0], int(kv.split("=")[1]))
    spin = ctypes.CDLL(os.path.join(ROOT, "tools", "libspin.so"))
    dev = torch.device("cuda", 0)
    B, S = 4, 1024
    net = UNetBN(B, S, levels=5, base=64, in_ch=3, dtype="bf16", device=dev, seed=865)
    tr = Trainer(net, LossConfig(use_hard_mining=False), lr=1e-4)
    xs, ys = synthetic_batch(B, S, channels=3, seed=865)
    xs = xs.astype(np.float32)
    x = torch.from_numpy((xs - xs.mean()) / (xs.std() + 1e-10)).to(dev).contiguous()
    y = torch.from_numpy(ys).to(dev).contiguous()
    side = torch.cuda.Stream(device=dev)
    # s_sleep 127 = 127 x 64 clocks; calibrate the iteration count on the idle GPU
    for _ in range(3):
        tr.train_step(x, y)
    torch.cuda.synchronize()
    spin.spin_launch(1, 10, 98304, ctypes.c_void_p(side.cuda_stream))   # (first launch: attribute, module load)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    spin.spin_launch(1, 2000, 98304, ctypes.c_void_p(side.cuda_stream))
    torch.cuda.synchronize()
    per_iter_ms = (time.perf_counter() - t0) * 1e3 / 2000
    iters = max(1, int(args.spin_ms / per_iter_ms))
    res = {"spin_iter_ms": round(per_iter_ms, 5), "iters": iters}

    def step(k):
        torch.cuda.synchronize()
        t = time.perf_counter()
        if k:
            spin.spin_launch(k, iters, 98304, ctypes.c_void_p(side.cuda_stream))
        tr.train_step(x, y)
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3

    ks = [int(v) for v in args.blocks.split(",")]
    times = {k: [] for k in ks}
    for _ in range(args.rounds):
        for k in ks:   # alternating, so drift hits every arm alike
            times[k].append(step(k))
    torch.cuda.synchronize()
    t = time.perf_counter()
    spin.spin_launch(1, iters, 98304, ctypes.c_void_p(side.cuda_stream))
    torch.cuda.synchronize()
    res["spin_ms"] = round((time.perf_counter() - t) * 1e3, 3)
    base = min(times[0]) if 0 in times else None
    for k in ks:
        res[f"K{k}"] = {"ms": [round(v, 3) for v in times[k]], "min": round(min(times[k]), 3),
                        "extra_ms": round(min(times[k]) - base, 3) if base else None,
                        "cu_share_model_ms": round(res["spin_ms"] * k / 256, 3)}
    res["opts"] = args.opt
    print(json.dumps(res))


if __name__ == "__main__":
    main()
