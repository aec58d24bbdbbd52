#!/usr/bin/env python3
"""Same-process A/B of two host-schedule variants of the bench step (unet_bn L5, 1024^2, B=4, bf16):
alternating timed blocks so that clock drift and device variance hit both arms alike.
  --variant pack: per-layer forward-weight packs (old) vs one flat cast (UNetEngine.pack_forward_weights)
  --variant pool: bn_apply + maxpool2_fwd (old) vs the fused adp_bn_apply_maxpool2
  --variant head: materialised dec0_conv2 activation + adp_bn_bwd_reduce (old) vs BN-on-load head and
                  adp_head_sigmoid_bwd_bnr (UNetBN.fuse_head_bn)
  --variant fold: conv-side BatchNorm statistic fold + finalize (old) vs the fold fused into the finalize
                  (UNetBN.fuse_bn_fold)
  --variant headdA: head backward storing dA (old) vs dA recomputed by adp_bn_bwd_apply_head
                  (UNetBN.head_recompute_dA)
  --variant bnwgrad: adp_bn_bwd_apply + weight gradient (old) vs adp_conv_wgrad_bn (UNetBN.fuse_bn_wgrad)
  --variant side: every weight gradient on the backward's stream (old) vs the off-critical-path ones on a second
                  stream (UNetBN.wgrad_side)
  --variant opt --opts "a=1;a=0": two native option settings (';'-separated, each ','-separated name=value)
(the round-1 "stat" arm, per-layer statistic fills vs one arena fill, measured neutral:
profiles/r01i_ab_stat_arena.txt; only the arena path remains)"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variant", default="pack", choices=["pack", "pool", "head", "fold", "headdA", "bnwgrad", "side", "opt"])
    p.add_argument("--opts", default="")
    p.add_argument("--side", action="store_true", help="UNetBN.wgrad_side in both arms (default: off in both)")
    p.add_argument("--rounds", type=int, default=4)
    p.add_argument("--steps", type=int, default=8)
    p.add_argument("--preset", default="unet_bn", choices=["unet_bn", "adipose_v3"],
                   help="adipose_v3: the reference topology (1024^2, B=2; --variant opt only)")
    p.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    args = p.parse_args()
    import numpy as np
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd import ops
    from adipose_amd.data import synthetic_batch
    from adipose_amd.nets import Dense, UNetBN, UNetEngine
    from adipose_amd.trainer import LossConfig, Trainer

    dev = torch.device("cuda", 0)
    UNetBN.wgrad_side = args.side   # (both arms; --variant side overrides per arm)
    if args.preset == "adipose_v3":
        from adipose_amd.data import to_gray
        from adipose_amd.nets import AdiposeV3Net
        assert args.variant == "opt", "adipose_v3 runs the option A/B only"
        net = AdiposeV3Net(2, 1024, dtype=args.dtype, device=dev, seed=865)
        tr = Trainer(net, LossConfig(), lr=1e-4)
        xs, ys = synthetic_batch(2, 1024, channels=3, seed=865)
        xs = to_gray(xs.astype("float32"))
    else:
        net = UNetBN(4, 1024, levels=5, base=64, in_ch=3, dtype=args.dtype, device=dev, seed=865)
        tr = Trainer(net, LossConfig(use_hard_mining=False), lr=1e-4)
        xs, ys = synthetic_batch(4, 1024, channels=3, seed=865)
    x = torch.from_numpy(((xs - xs.mean()) / (xs.std() + 1e-10)).astype(np.float32)).to(dev)
    y = torch.from_numpy(ys).to(dev)
    if args.variant == "pack":
        owner, attr = UNetEngine, "pack_forward_weights"
        new = UNetEngine.pack_forward_weights

        def old(self):
            for l in self.layers.values():
                if isinstance(l, Dense):
                    dst = self.buf("wf_old/" + l.name, (l.Npad, l.Kpad))
                    ops.pack_weights(self.ps.view(l.name + "/W"), dst, 0)
                    self._packed[l.name] = dst
    elif args.variant == "head":
        owner, attr, old, new = UNetBN, "fuse_head_bn", False, True
    elif args.variant == "fold":
        owner, attr, old, new = UNetBN, "fuse_bn_fold", False, True
    elif args.variant == "headdA":
        owner, attr, old, new = UNetBN, "head_recompute_dA", False, True
    elif args.variant == "bnwgrad":
        owner, attr, old, new = UNetBN, "fuse_bn_wgrad", False, True
    elif args.variant == "side":
        owner, attr, old, new = UNetBN, "wgrad_side", False, True
    elif args.variant == "opt":
        class _Opts:   # setattr(owner, attr, settings) applies a native option setting
            def __setattr__(self, _, st):
                for kv in st.split(","):
                    if kv:
                        ops.set_option(kv.split("=")[0], int(kv.split("=")[1]))
        owner, attr = _Opts(), "opts"
        old, new = args.opts.split(";")
    else:
        owner, attr = ops, "bn_apply_maxpool2"
        new = ops.bn_apply_maxpool2

        def old(z, scale, shift, act, pool):
            ops.bn_apply(z, scale, shift, act)
            ops.maxpool2_fwd(act, pool)
            return act
    arms = {"A (old)": old, "B (new)": new}
    for fn in arms.values():
        setattr(owner, attr, fn)
        for _ in range(3):
            tr.train_step(x, y)
    res = {k: [] for k in arms}
    for _ in range(args.rounds):
        for k, fn in arms.items():
            setattr(owner, attr, fn)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                tr.train_step(x, y)
            torch.cuda.synchronize()
            res[k].append((time.perf_counter() - t0) / args.steps * 1e3)
    for k, v in res.items():
        print(k, "ms/step", [round(t, 3) for t in v], "min", round(min(v), 3), flush=True)


if __name__ == "__main__":
    main()
