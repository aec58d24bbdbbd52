#!/usr/bin/env python3
"""How the bench step (unet_bn L5, 1024^2, B=4, bf16) reacts to CUs held by another stream's kernel, as RCCL's
blocks hold CUs while the data-parallel step's gradient buckets are all-reduced (one GPU stands in: a
sleep-only kernel on a side stream, K blocks of 64 threads with 96 KiB of LDS each, so that none of the step's
persistent blocks can share their CU). Each sample: the side kernel (about `--spin-ms` long) is launched, then
one training step on the default stream; the step's wall time is compared with steps without it. A step that
only lost K of 256 CUs for the spin's duration grows by about spin_ms * K / 256; a persistent kernel whose
late blocks wait for a held CU grows by up to its own duration.
usage: python tools/contention_probe.py [--blocks 0,8,16,32,64] [--spin-ms 20] [--rounds 3]

--buckets: the data-parallel schedule instead of one long hold. The step runs with the Trainer's gradient buckets
(trainer.plan_buckets, 16 MB), and each bucket's all-reduce is stood in for by a side-stream sleep kernel of
--bucket-ms holding K CUs, started when the backward has finished the bucket's layers (overlap) or all of them at
the end of the backward (after), as RCCL's kernels would be on a node. Arms: static tile lists / claimed tiles
(option dp_claim) x overlap / after; "exposed_model_ms" is what the buckets cost run back to back on an idle chip.
usage: python tools/contention_probe.py --buckets [--blocks 8,32] [--bucket-ms 0.3] [--rounds 3]
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
    p.add_argument("--buckets", action="store_true")
    p.add_argument("--bucket-ms", type=float, default=0.3)
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

    if args.buckets:
        return bucket_probe(args, tr, x, y, spin, side, per_iter_ms, res, ops)
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


class _Done:
    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        import torch
        torch.cuda.current_stream().wait_event(self.ev)


def bucket_probe(args, tr, x, y, spin, side, per_iter_ms, res, ops):
    """The Trainer's bucket schedule with each all-reduce replaced by a CU-holding sleep on a side stream."""
    import torch
    from adipose_amd import trainer as trmod
    iters = max(1, int(args.bucket_ms / per_iter_ms))
    state = {"k": 0}

    class SpinBuckets(trmod.GradBuckets):
        def __init__(self, net, overlap):   # no process group: one GPU stands in for a rank
            self.group, self.overlap, self.world = None, overlap, 1
            self.buckets = trmod.plan_buckets(net.ps, 16 << 20)
            self.ps, self.works = net.ps, []

        def _launch(self, i):
            self.launched[i] = True
            ev = torch.cuda.Event()
            ev.record()
            side.wait_event(ev)
            spin.spin_launch(state["k"], iters, 98304, ctypes.c_void_p(side.cuda_stream))
            done = torch.cuda.Event()
            done.record(side)
            self.works.append(_Done(done))

    real_all_reduce = trmod.dist.all_reduce
    trmod.dist.all_reduce = lambda *a, **k: None   # the Dice-sum reduce: 24 doubles, no CUs worth holding
    arms = {}
    ks = [int(v) for v in args.blocks.split(",") if int(v) > 0]
    sb = {ov: SpinBuckets(tr.net, ov) for ov in (True, False)}
    res["n_buckets"] = len(sb[True].buckets)
    res["bucket_iters"] = iters

    def step():
        torch.cuda.synchronize()
        t = time.perf_counter()
        tr.train_step(x, y)
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3

    try:
        for _ in range(2):
            for claim in (0, 1):
                ops.set_option("dp_claim", claim)
                tr.buckets = None
                arms.setdefault(f"none/claim{claim}", []).append(step())
                for k in ks:
                    state["k"] = k
                    for ov in (True, False):
                        tr.buckets = sb[ov]
                        step()    # warm
                        for _ in range(args.rounds):
                            arms.setdefault(f"K{k}/claim{claim}/{'overlap' if ov else 'after'}", []).append(step())
    finally:
        trmod.dist.all_reduce = real_all_reduce
        tr.buckets = None
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(res["n_buckets"]):
        spin.spin_launch(8, iters, 98304, ctypes.c_void_p(side.cuda_stream))
    torch.cuda.synchronize()
    res["exposed_model_ms"] = round((time.perf_counter() - t) * 1e3, 3)
    base = {c: min(arms[f"none/claim{c}"]) for c in (0, 1)}
    for name, v in arms.items():
        c = int(name.split("claim")[1][0])
        res[name] = {"min": round(min(v), 3), "extra_ms": round(min(v) - base[c], 3), "n": len(v)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
