"""One-off: run-to-run spread of the unet_bn training forward (bf16 / f32, base 64, 64^2, B=2): fresh networks,
the same network twice, and each fallback flag, each against the f32 torch oracle."""
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
ref = R.unet_bn_forward(x, w, levels=L).float()
for dtype in ("bf16", "f32"):
    outs = []
    for tag, flag in (("fresh0", None), ("fresh1", None), ("fuse_head_bn", "fuse_head_bn"), ("fresh2", None),
                      ("pool_argmax_from_z", "pool_argmax_from_z"), ("fuse_bn_fold", "fuse_bn_fold")):
        net = UNetBN(B, S, levels=L, base=64, in_ch=3, dtype=dtype, device="cuda")
        net.set_weights(w)
        if flag:
            setattr(net, flag, False)
        tr = Trainer(net, LossConfig(use_hard_mining=False))
        o, _ = T._unet_bn_step(net, tr, x, y, B)
        p = o["main_out"].cpu().clone()
        o2, _ = T._unet_bn_step(net, tr, x, y, B)
        p2 = o2["main_out"].cpu().clone()
        outs.append((tag, p))
        print(dtype, tag, "vs oracle max %.3g mean %.3g" % ((p - ref).abs().max(), (p - ref).abs().mean()))
        print(dtype, tag, "same-net repeat max %.3g mean %.3g" % ((p - p2).abs().max(), (p - p2).abs().mean()),
              flush=True)
        del net, tr
    t0, p0 = outs[0]
    for tag, p in outs[1:]:
        d = (p - p0).abs()
        print(dtype, t0, "vs", tag, "max %.3g mean %.3g" % (d.max(), d.mean()), flush=True)
