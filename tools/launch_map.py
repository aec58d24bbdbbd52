#!/usr/bin/env python3
"""Which kernel each conv launch of one training step runs on (layer shape, epilogue flags -> adp_last_kernel),
for finding launches that miss the persistent kernels. usage: python tools/launch_map.py [--preset adipose_v3]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--preset", default="adipose_v3", choices=["adipose_v3", "unet_bn"])
    p.add_argument("--batch", type=int, default=2)
    p.add_argument("--size", type=int, default=1024)
    p.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    args = p.parse_args()
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd import _lib, ops
    from adipose_amd.data import synthetic_batch
    from adipose_amd.nets import AdiposeV3Net, UNetBN
    from adipose_amd.trainer import LossConfig, Trainer
    dev = torch.device("cuda", 0)
    B, S = args.batch, args.size
    if args.preset == "unet_bn":
        net = UNetBN(B, S, levels=5, base=64, in_ch=3, dtype=args.dtype, device=dev, seed=865)
        tr = Trainer(net, LossConfig(use_hard_mining=False))
        xs, ys = synthetic_batch(B, S, channels=3, seed=865)
    else:
        from adipose_amd.data import to_gray
        net = AdiposeV3Net(B, S, dtype=args.dtype, device=dev, seed=865)
        tr = Trainer(net, LossConfig())
        xs, ys = synthetic_batch(B, S, channels=3, seed=865)
        xs = to_gray(xs.astype("float32"))
    x = torch.from_numpy((xs - xs.mean()) / (xs.std() + 1e-10)).float().to(dev)
    y = torch.from_numpy(ys).to(dev)
    tr.train_step(x, y)
    torch.cuda.synchronize()
    log = []
    for fn in ("conv_fwd", "conv_wgrad"):
        orig = getattr(ops, fn)

        def wrap(*a, _o=orig, _fn=fn, **k):
            r = _o(*a, **k)
            flags = ",".join(n for n in ("addend", "mask", "mask2", "accum", "bn_stats", "bn_reduce", "bn_apply", "out2")
                             if k.get(n) is not None) + (f",dil={k['dil']}" if k.get("dil", 1) != 1 else "") + \
                (",up" if k.get("up") else "") + (f",drop={k['dropout_rate']}" if k.get("dropout_rate") else "")
            nout = a[3] if _fn == "conv_wgrad" else a[2]   # (conv_fwd: srcA, W, nout; conv_wgrad: srcA, dY, dW, nout)
            log.append((_fn, tuple(a[0].shape), nout, flags,
                        _lib.lib().adp_last_kernel().decode()))
            return r
        setattr(ops, fn, wrap)
    tr.train_step(x, y)
    torch.cuda.synchronize()
    for e in log:
        print(f"{e[0]:10s} src={str(e[1]):24s} nout={e[2]!s:6s} {e[3]:32s} {e[4]}")


if __name__ == "__main__":
    main()
