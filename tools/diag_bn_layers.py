"""One-off: which unet_bn layer's BatchNorm statistics differ between two training steps of one bf16 network
(same weights, no optimizer step): per-layer max relative difference of mean / invstd, and the outputs."""
import sys
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import _adipose_pkg  # noqa: E402,F401
import test_gpu_network as T  # noqa: E402
from oracle import torch_ref as R  # noqa: E402
from adipose_amd.nets import UNetBN  # noqa: E402
from adipose_amd.trainer import LossConfig, Trainer  # noqa: E402

B, L, S = 2, 3, 64
w = R.unet_bn_keras_weights(levels=L, base=64, in_ch=3, seed=5)
x, y = T.synth_batch(B, S, C=3, seed=9)
for backward in (False, True):
    net = UNetBN(B, S, levels=L, base=64, in_ch=3, dtype="bf16", device="cuda")
    net.set_weights(w)
    tr = Trainer(net, LossConfig(use_hard_mining=False))
    runs = []
    for step in range(6):
        o, _ = T._unet_bn_step(net, tr, x, y, B, backward=backward)
        st = {n: torch.stack([v.detach().clone() for v in net.st[n][:6]]).cpu() for n in net.st}
        runs.append((o["main_out"].cpu().clone(), st))
    p0, s0 = runs[0]
    for i, (p, s) in enumerate(runs[1:], 1):
        bad = []
        for n in s0:
            d = ((s[n] - s0[n]).abs() / (s0[n].abs() + 1e-6)).amax(1)
            if d.max() > 1e-5:
                bad.append((n, [round(float(v), 6) for v in d]))
        print("backward", backward, "step", i, "out max %.3g mean %.3g" % ((p - p0).abs().max(), (p - p0).abs().mean()),
              bad[:6], flush=True)
