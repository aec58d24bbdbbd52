#!/usr/bin/env python3
"""Timing probe of the level-0 conv2 with the BatchNorm-ReLU applied on load (halo forward EPI 6) against the plain
launch and the bn_apply pass it replaces (unet_bn L0: 4 x 1024^2 x 64 -> 64, statistics). Arms: plain conv on the
activation; bn_apply alone; the fused launch; the fused launch without its activation stores (fwd_debug bit 12,
timing only: run with ADP_LIB_PATH=ab/libadipose_ablation.so from tools/build_ablation_lib.sh, the product library
ignores the option); the fused launch without the halo apply VALU is not separable. Prints ms per launch (20 launches,
median of 5 repeats).""" 
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd import ops
    dev = torch.device("cuda", 0)
    N, S, C = 4, 1024, 64
    g = torch.Generator().manual_seed(3)
    z = (torch.randn(N, S, S, C, generator=g) * 2).to(dev, torch.bfloat16)
    act = torch.empty_like(z)
    sc = (torch.rand(C, generator=g) + 0.5).to(dev)
    sh = (torch.randn(C, generator=g) * 0.5).to(dev)
    W = (torch.randn(64, 9 * C, generator=g) * 0.03).to(dev, torch.bfloat16)
    out = torch.empty(N, S, S, 64, dtype=torch.bfloat16, device=dev)
    st = torch.zeros(2, 64, device=dev)

    def plain():
        ops.conv_fwd(act, W, 64, out=out, bn_stats=(st[0], st[1]))

    def apply():
        ops.bn_apply(z, sc, sh, act)

    def fused():
        ops.conv_fwd(z, W, 64, out=out, bn_stats=(st[0], st[1]), bnA=(sc, sh), act_out=act)

    def fused_nostore():
        ops.set_option("fwd_debug", 4096)
        try:
            fused()
        finally:
            ops.set_option("fwd_debug", None)

    arms = {"plain conv": plain, "bn_apply": apply, "fused": fused, "fused, no act stores": fused_nostore}
    for fn in arms.values():
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    res = {k: [] for k in arms}
    for _ in range(5):
        for k, fn in arms.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / 20)
    for k, v in res.items():
        v.sort()
        print(f"{k:24s} {v[len(v) // 2]:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
