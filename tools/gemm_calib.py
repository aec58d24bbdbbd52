"""Calibration: hipBLASLt (torch.matmul) bf16 GEMM rate on the implicit-GEMM shapes of the unet_bn L5
1024^2 B=4 3x3 convs (M = B*H*W pixels, K = 9*Cin, N = Cout), random operands, after a warm-up so the
clock has settled. The dense library GEMM is the practical ceiling the conv kernels are measured against.

    python tools/gemm_calib.py
"""
import time

import torch


def rate(M, K, N, iters=20):
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(5):
        c = a @ b
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        c = a @ b
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    del c
    return 2.0 * M * K * N / dt / 1e12, dt * 1e3


def main():
    # spin the clock down to its loaded state first (~2 s of dense GEMM)
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2.0:
        a @ a
    torch.cuda.synchronize()
    shapes = [("L0 64->64", 4 * 1024 * 1024, 576, 64), ("L1 128->128", 4 * 512 * 512, 1152, 128),
              ("L2 256->256", 4 * 256 * 256, 2304, 256), ("L3 512->512", 4 * 128 * 128, 4608, 512),
              ("L4 1024->1024", 4 * 64 * 64, 9216, 1024), ("L3 dec 1024->512", 4 * 128 * 128, 9216, 512),
              ("square 8192", 8192, 8192, 8192)]
    for name, M, K, N in shapes:
        tf, ms = rate(M, K, N)
        print(f"{name:18s} M={M:8d} K={K:5d} N={N:5d}  {ms:7.3f} ms  {tf:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
