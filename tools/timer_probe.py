#!/usr/bin/env python3
"""Cost of the bench's per-launch event timing (arm events: every conv launch; dom: the dominant kernel's only) (ops.LaunchTimer: a HIP event pair around the main kernel of every conv
launch) on the unet_bn bench step: alternating blocks of steps with and without it, in one process."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd import ops
    from adipose_amd.data import synthetic_batch
    from adipose_amd.nets import UNetBN
    from adipose_amd.trainer import LossConfig, Trainer
    dev = torch.device("cuda", 0)
    net = UNetBN(4, 1024, levels=5, base=64, in_ch=3, dtype="bf16", device=dev, seed=865)
    tr = Trainer(net, LossConfig(use_hard_mining=False), lr=1e-4)
    xs, ys = synthetic_batch(4, 1024, channels=3, seed=865)
    x = torch.from_numpy(((xs - xs.mean()) / (xs.std() + 1e-10)).astype(np.float32)).to(dev)
    y = torch.from_numpy(ys).to(dev)
    for _ in range(3):
        tr.train_step(x, y)
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    nst = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    res = {"events": [], "plain": [], "dom": []}
    for _ in range(rounds):
        for arm in ("plain", "events", "dom"):
            timer = (ops.LaunchTimer() if arm == "events" else
                     ops.LaunchTimer(only="igemm_wgrad_halopair_kernel<6, 0>") if arm == "dom" else None)
            torch.cuda.synchronize()
            ops.set_launch_timer(timer)
            t0 = time.perf_counter()
            for _ in range(nst):
                tr.train_step(x, y)
            torch.cuda.synchronize()
            res[arm].append((time.perf_counter() - t0) / nst * 1e3)
            ops.set_launch_timer(None)
            if timer is not None:
                timer.summary()
    for k, v in res.items():
        print(k, "ms/step", [round(t, 3) for t in v], "min", round(min(v), 3), "median",
              round(sorted(v)[len(v) // 2], 3), flush=True)


if __name__ == "__main__":
    main()
