#!/usr/bin/env python3
"""The bench step (unet_bn L5 1024^2 B=4 bf16) run N times with or without the bench's per-launch event timing
(--timer), for rocprofv3 --kernel-trace + tools/step_timeline.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


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
    for _ in range(2):
        tr.train_step(x, y)
    torch.cuda.synchronize()
    timer = ops.LaunchTimer() if "--timer" in sys.argv else None
    ops.set_launch_timer(timer)
    for _ in range(4):
        tr.train_step(x, y)
    torch.cuda.synchronize()
    ops.set_launch_timer(None)


if __name__ == "__main__":
    main()
