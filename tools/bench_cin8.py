#!/usr/bin/env python3
"""Input-layer (one 8-channel source) forward conv timing at the unet_bn 1024^2 B=4 shape, over native
option variants: python tools/bench_cin8.py "fwd_cin8=0;cin8_waves=4096;cin8_waves=16384" """
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd import ops
    from adipose_amd._lib import lib
    from adipose_amd.nets import Dense

    variants = (sys.argv[1] if len(sys.argv) > 1 else "fwd_cin8=0;fwd_cin8=1").split(";")
    B, S, cout = 4, 1024, 64
    l = Dense("t", [3], cout)
    W = torch.randn(64, (9 * 8 + 31) // 32 * 32, device="cuda").to(torch.bfloat16)
    x = torch.randn(B, S, S, 8, device="cuda").to(torch.bfloat16)
    out = torch.empty(B, S, S, 64, device="cuda", dtype=torch.bfloat16)
    s1 = torch.zeros(64, device="cuda")
    s2 = torch.zeros(64, device="cuda")
    b = torch.zeros(64, device="cuda")
    for v in variants:
        opts = [kv for kv in v.split(",") if "=" in kv]
        for kv in opts:
            k, val = kv.split("=")
            ops.set_option(k, int(val))
        st = None if "nostats" in v else (s1, s2)
        fn = lambda: ops.conv_fwd(x, W, l.Nout, out=out, bias=b, bn_stats=st)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        name = lib().adp_last_kernel().decode()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(json.dumps({"variant": v, "kernel": name, "ms": round(ms, 4),
                          "TB_s": round((out.numel() * 2 + x.numel() * 2) / ms / 1e9, 3)}), flush=True)
        for kv in opts:
            ops.set_option(kv.split("=")[0], None)


if __name__ == "__main__":
    main()
