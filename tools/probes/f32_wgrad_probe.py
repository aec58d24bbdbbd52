#!/usr/bin/env python3
"""Per-launch time of the f32 halo weight gradients (igemm_wgrad_halo_f32_kernel / _dil_kernel) on adipose_v3's f32
1024^2 B=2 layer shapes, with option variants: ms per launch (median of 5 x 10, HIP events), TFLOP/s of the real
channel products and of the products the kernel computes (64-row output blocks x 32-channel chunks, zero-tail
chunks on 16 columns)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd import _lib, ops
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(5)
    variants = [v for v in (sys.argv[1] if len(sys.argv) > 1 else "wgrad_f32_halo_grid=256").split(";")]
    # name, N, S (output), source strides, source real channels, Nout stride, Nout real, up, dil
    cases = [("L0 44->44", 2, 1024, [64], [44], 64, 44, False, 1),
             ("L0 44+44->44", 2, 1024, [64, 64], [44, 44], 64, 44, False, 1),
             ("L0 up 88->44", 2, 1024, [96], [88], 64, 44, True, 1),
             ("L1 44->88", 2, 512, [64], [44], 96, 88, False, 1),
             ("L1 88->88", 2, 512, [96], [88], 96, 88, False, 1),
             ("L1 88+88->88", 2, 512, [96, 96], [88, 88], 96, 88, False, 1),
             ("L1 up 176->88", 2, 512, [192], [176], 96, 88, True, 1),
             ("L2 176->176", 2, 256, [192], [176], 192, 176, False, 1),
             ("L2 176+176->176", 2, 256, [192, 192], [176, 176], 192, 176, False, 1),
             ("L3 176->352", 2, 128, [192], [176], 352, 352, False, 1),
             ("L3 352->352 d2", 2, 128, [352], [352], 352, 352, False, 2)]
    for name, N, S, parts, reals, nst, nreal, up, dil in cases:
        Ss = S // 2 if up else S
        xs = []
        for c, r in zip(parts, reals):
            t = torch.zeros(N, Ss, Ss, c, device=dev)
            t[..., :r] = torch.randn(N, Ss, Ss, r, generator=g).to(dev)
            xs.append(t)
        dY = torch.zeros(N, S, S, nst, device=dev)
        dY[..., :nreal] = torch.randn(N, S, S, nreal, generator=g).to(dev)
        cin = sum(parts)
        dW = torch.zeros(ops.round_up(nst, 64), ops.round_up(9 * cin, 32), device=dev)
        real = (reals[0], reals[1] if len(reals) > 1 else 0, nreal)
        flop_real = 2.0 * N * S * S * nreal * 9 * sum(reals)
        out = []
        for v in variants:
            kv = [(s.split("=")[0], int(s.split("=")[1])) for s in v.split(",") if s]
            for k, val in kv:
                ops.set_option(k, val)
            try:
                def run():
                    ops.conv_wgrad(xs[0], dY, dW, nst, srcB=xs[1] if len(xs) > 1 else None, up=up, dil=dil,
                                   real=real)
                run()
                torch.cuda.synchronize()
                kname = _lib.lib().adp_last_kernel().decode()
                ts = []
                for _ in range(5):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(10):
                        run()
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) / 10)
                ts.sort()
                ms = ts[2]
            finally:
                for k, _ in kv:
                    ops.set_option(k, None)
            out.append(f"[{v}] {ms:.3f} ms {flop_real / ms / 1e9:.1f} TF-real {kname}")
        print(f"{name:16s} " + " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
