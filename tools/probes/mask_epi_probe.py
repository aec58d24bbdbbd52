#!/usr/bin/env python3
"""Epilogue cost of the adipose_v3 data-gradient launches (mask / addend epilogues on the tap64 kernel), f32 and bf16:
the launch as is and with fwd_debug bit 4 (no epilogue; timing only -- run with ADP_LIB_PATH=ab/libadipose_ablation.so
from tools/build_ablation_lib.sh). Prints ms per launch (median of 5 x 10)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd import _lib, ops
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(5)
    cases = [("f32 L0 64->64 mask", torch.float32, 2, 1024, 64, 64, True, False),
             ("f32 L0 64->64 plain", torch.float32, 2, 1024, 64, 64, False, False),
             ("f32 L2 192->192 mask+add", torch.float32, 2, 256, 192, 192, True, True),
             ("bf16 L2 192->192 mask+add", torch.bfloat16, 2, 256, 192, 192, True, True),
             ("bf16 L1 96->96 mask", torch.bfloat16, 2, 512, 128, 128, True, False)]
    for name, dt, N, S, cin, cout, mask, add in cases:
        x = torch.randn(N, S, S, cin, generator=g).to(dev, dt)
        W = (torch.randn(ops.round_up(cout, 64), ops.round_up(9 * cin, 32), generator=g) * 0.03).to(dev, dt)
        o = torch.empty(N, S, S, cout, dtype=dt, device=dev)
        mk = (torch.rand(N, S, S, cout, generator=g) > 0.4).to(dev, dt) if mask else None
        ad = torch.randn(N, S, S, cout, generator=g).to(dev, dt) if add else None
        res = {}
        for dbg in (0, 16):
            ops.set_option("fwd_debug", dbg)
            try:
                ts = []
                for _ in range(5):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(10):
                        ops.conv_fwd(x, W, cout, out=o, mask=mk, addend=ad)
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) / 10)
                ts.sort()
                res[dbg] = ts[2]
                kname = _lib.lib().adp_last_kernel().decode()
            finally:
                ops.set_option("fwd_debug", None)
        print(f"{name:28s} {kname[:60]:60s} full {res[0]:.4f} ms  no-epilogue {res[16]:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
