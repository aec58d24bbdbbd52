"""Localise f32 gradient differences of the unet_bn preset vs the oracle (per tensor)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _adipose_pkg  # noqa: E402,F401
from adipose_amd import ops  # noqa: E402
from adipose_amd.nets import UNetBN  # noqa: E402
from adipose_amd.trainer import LossConfig, Trainer  # noqa: E402
from oracle import torch_ref as R  # noqa: E402

DEV = "cuda"
B, S, L = 2, 32, 3
w = R.unet_bn_keras_weights(levels=L, base=16, in_ch=3, seed=5)
g = torch.Generator().manual_seed(9)
x = torch.randn(B, S, S, 3, generator=g)
yy, xx = torch.meshgrid(torch.arange(S), torch.arange(S), indexing="ij")
y = torch.zeros(B, S, S)
for b in range(B):
    cy, cx = torch.randint(0, S, (2,), generator=g)
    y[b] = (((yy - cy) ** 2 + (xx - cx) ** 2) < (S / 3) ** 2).float()
net = UNetBN(B, S, levels=L, base=16, in_ch=3, dtype="f32", device=DEV)
net.set_weights(w)
tr = Trainer(net, LossConfig(use_hard_mining=False))
a = net.acts(B)
ops.prep_input(x.to(DEV), a["x"], mean=0.0, std=1.0)
outs = net.forward(B, train=True)
grads = tr.loss_and_grads(outs, y.to(DEV))
ops.fill(net.ps.grad, 0.0)
net.backward(grads)
torch.cuda.synchronize()

# oracle with retained intermediate grads
W = {k: [torch.tensor(v, requires_grad=True) for v in vs] for k, vs in w.items()}
inter = {}


def keep(name, t):
    t.retain_grad()
    inter[name] = t
    return t


def blk(name, inp):
    k, gm, bt = W[name]
    z = keep("z/" + name, R.conv2d_same(inp, k, None, relu=False))
    return keep("a/" + name, R.bn_relu_train(z, gm, bt))


skips, h = [], x
for i in range(L):
    h = blk(f"enc{i}_conv2", blk(f"enc{i}_conv1", h))
    if i < L - 1:
        skips.append(h)
        h = R.maxpool2(h)
for i in range(L - 2, -1, -1):
    k, b = W[f"dec{i}_up"]
    u = torch.nn.functional.conv_transpose2d(h.permute(0, 3, 1, 2), k, b, stride=2).permute(0, 2, 3, 1)
    h = blk(f"dec{i}_conv2", blk(f"dec{i}_conv1", torch.cat([skips[i], u], -1)))
k, b = W["head"]
p = torch.sigmoid(R.conv1x1(h, k, b))[..., 0]
loss = R.combined_loss_standard(y, p)
loss.backward()


def rel(a_, b_):
    a_, b_ = torch.as_tensor(a_).float(), torch.as_tensor(b_).float()
    return (a_ - b_).abs().max().item() / max(b_.abs().max().item(), 1e-20)


print("p", rel(outs["main_out"].cpu(), p.detach()))
bufmap = {"enc0_conv1": ("z0_1", "dz_z0_1", "dA_z0_1"), "enc0_conv2": ("z0_2", "dz_z0_2", "dA_z0_2"),
          "enc1_conv1": ("z1_1", "dz_z1_1", "dA_z1_1"), "enc1_conv2": ("z1_2", "dz_z1_2", "dA_z1_2"),
          "dec0_conv1": ("y0_1", "dz_y0_1", "dA_y0_1"), "dec0_conv2": ("y0_2", "dz_y0_2", "y0_2")}
for name, (zk, dzk, dak) in bufmap.items():
    z = a[zk].cpu()
    da = net.buf("g/" + dak, tuple(a[zk].shape), a[zk].dtype).cpu()
    # (enc0_conv1's dz is not stored with the fused BN-backward weight gradient: nothing reads it)
    dzs = "n/a"
    if not (name == "enc0_conv1" and net.fuse_bn_wgrad):
        dz = net.buf("g/" + dzk, tuple(a[zk].shape), a[zk].dtype).cpu()
        dzs = f"{rel(dz, inter['z/' + name].grad):.2e}"
    print(name, "z", f"{rel(z, inter['z/' + name].detach()):.2e}",
          "dA", f"{rel(da, inter['a/' + name].grad):.2e}", "dz", dzs)
for name, ts in W.items():
    got = net.get_layer_grads(name)
    print("grad", name, [f"{rel(gi, t.grad):.2e}" for gi, t in zip(got, ts)])
st = net.st["enc0_conv1"].cpu().numpy()
zz = inter["z/enc0_conv1"].detach()
print("mean", np.abs(st[4][:16] - zz.mean((0, 1, 2)).numpy()).max(), "invstd",
      np.abs(st[5][:16] - 1 / torch.sqrt(zz.var((0, 1, 2), unbiased=False) + 1e-5).numpy()).max())
