#!/usr/bin/env python3
"""Where does the train step's wall time go outside the kernels? (diagnostic, GPU box)

Times the bench workload (unet_bn L5 1024^2 B=4 bf16) three ways: eager steps without the bench's
launch timer, the host-side issue time of those steps (no synchronisation between them), and replays
of ONE step captured in a HIP graph. usage: python tools/graph_probe.py [--steps 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--batch", type=int, default=4)
    args = p.parse_args()
    import numpy as np
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd.data import synthetic_batch
    from adipose_amd.nets import UNetBN
    from adipose_amd.trainer import LossConfig, Trainer

    dev = torch.device("cuda", 0)
    B, S = args.batch, 1024
    net = UNetBN(B, S, levels=5, base=64, in_ch=3, dtype="bf16", device=dev, seed=865)
    tr = Trainer(net, LossConfig(use_hard_mining=False), lr=1e-4)
    xs, ys = synthetic_batch(B, S, channels=3, seed=865)
    xs = xs.astype(np.float32)
    x = torch.from_numpy((xs - xs.mean()) / (xs.std() + 1e-10)).to(dev).contiguous()
    y = torch.from_numpy(ys).to(dev).contiguous()
    out = {}
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            tr.train_step(x, y)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()

    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.train_step(x, y)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out["eager_ms"] = (t2 - t0) * 1e3 / args.steps
    out["host_issue_ms"] = (t1 - t0) * 1e3 / args.steps

    # the same with bench.py's per-launch HIP-event timer on every conv launch
    from adipose_amd import ops
    timer = ops.LaunchTimer()
    ops.set_launch_timer(timer)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.train_step(x, y)
    torch.cuda.synchronize()
    out["eager_timer_ms"] = (time.perf_counter() - t0) * 1e3 / args.steps
    ops.set_launch_timer(None)

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        tr.train_step(x, y)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        g.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out["graph_ms"] = (t2 - t0) * 1e3 / args.steps
    out["graph_host_ms"] = (t1 - t0) * 1e3 / args.steps
    out["tiles_per_s_eager"] = B / out["eager_ms"] * 1e3
    out["tiles_per_s_graph"] = B / out["graph_ms"] * 1e3
    print(json.dumps({k: round(v, 3) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
