"""Repeatability probe: the same f32 unet_bn gradient computed N times in one process (after an
adipose train step that leaves stale data in recycled memory). Differences beyond atomic-order noise
(~1e-6 relative) point at a race or an uninitialised read."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _adipose_pkg  # noqa: E402,F401
from adipose_amd import ops  # noqa: E402
from adipose_amd.nets import AdiposeV3Net, UNetBN  # noqa: E402
from adipose_amd.trainer import LossConfig, Trainer  # noqa: E402
from oracle import torch_ref as R  # noqa: E402

DEV = "cuda"


def adipose_steps():
    w = R.adipose_v3_keras_weights(seed=865)
    net = AdiposeV3Net(2, 32, dtype="f32", device=DEV)
    net.set_weights(w)
    net.dropout_rate = 0.0
    tr = Trainer(net, LossConfig(), lr=1e-3)
    g = torch.Generator().manual_seed(8)
    x = torch.randn(2, 32, 32, generator=g)
    y = (torch.rand(2, 32, 32, generator=g) > 0.5).float()
    for _ in range(2):
        tr.train_step(x.to(DEV), y.to(DEV))
    torch.cuda.synchronize()


def unet_grads(dtype):
    B, S, L = 2, 32, 3
    w = R.unet_bn_keras_weights(levels=L, base=16, in_ch=3, seed=5)
    g = torch.Generator().manual_seed(9)
    x = torch.randn(B, S, S, 3, generator=g)
    y = (torch.rand(B, S, S, generator=g) > 0.6).float()
    net = UNetBN(B, S, levels=L, base=16, in_ch=3, dtype=dtype, device=DEV)
    net.set_weights(w)
    tr = Trainer(net, LossConfig(use_hard_mining=False))
    ops.prep_input(x.to(DEV), net.acts(B)["x"], mean=0.0, std=1.0)
    outs = net.forward(B, train=True)
    grads = tr.loss_and_grads(outs, y.to(DEV))
    ops.fill(net.ps.grad, 0.0)
    net.backward(grads)
    torch.cuda.synchronize()
    return {n: [a.copy() for a in net.get_layer_grads(n)] for n in net.layers}


def main():
    adipose_steps()
    runs = [unet_grads("f32") for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4)]
    worst = {}
    for n in runs[0]:
        for si in range(len(runs[0][n])):
            ref = runs[0][n][si]
            scale = max(np.abs(ref).max(), 1e-20)
            d = max(np.abs(r[n][si] - ref).max() for r in runs[1:]) / scale
            worst[(n, si)] = d
    top = sorted(worst.items(), key=lambda kv: -kv[1])[:6]
    print("max relative spread across repetitions:", [(k, f"{v:.2e}") for k, v in top])


if __name__ == "__main__":
    main()
