#!/usr/bin/env python3
"""bench_infer.py — inference benchmarks of BASELINE.json configs[3] (sliding window + 8-way TTA on an
8192x8192 synthetic WSI, 1024^2 tiles, 75 % overlap, tile rows sharded across GPUs) and the plain
1024^2 forward of the reference network.

Workload (config 4): the reference network (`adipose_v3`, train_adipose_unet_v3.py:660-758, random
Keras-default init, seed 865) evaluated exactly as full_evaluation_enhanced.py's
SlidingWindowInference.predict_with_sliding_window (:286-329) with TTA 'full' (:522-600) and Gaussian
blending (:115-183): 29 x 29 = 841 tile positions x 8 views = 6,728 tile forwards per WSI. The WSI
is resident in HBM before timing; the blended probability map stays in HBM (its D2H copy is outside
the timed region). With N ranks (torchrun) every rank takes a contiguous band of tile rows and the
blend canvases are SUM-all-reduced over RCCL (predictor.SlidingWindowInference).

Usage: python bench_infer.py [--mode wsi|tiles] [--size 8192] [--dtype bf16|f32] [--steps K] [--warmup W]
Rank 0 prints ONE JSON line with a `roofline` object for the dominant conv kernel.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MI355X_PEAK = {"bf16": 2500.0, "f32": 157.3}
# forward FLOPs of adipose_v3 per 1024^2 tile: 2 x 448.2 GMAC (counted from the layer list)
V3_FWD_GFLOP_1024 = 896.3


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--mode", default="wsi", choices=["wsi", "tiles"])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--size", type=int, default=8192, help="WSI side (mode wsi)")
    p.add_argument("--tile", type=int, default=1024)
    p.add_argument("--overlap", type=float, default=0.75)
    p.add_argument("--tta", default="full", choices=["none", "minimal", "basic", "full"])
    p.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    p.add_argument("--cpad", type=lambda v: tuple(int(x) for x in v.split(",")), default=None, help="channel-stride granule per level, e.g. 8,8,64,64 (bf16 default: predictor.INFER_CPAD)")
    p.add_argument("--batch", type=int, default=8, help="tile x view forwards per batched launch")
    p.add_argument("--steps", type=int, default=1, help="WSIs (mode wsi) / batches (mode tiles) timed")
    p.add_argument("--warmup", type=int, default=1)
    return p.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import _adipose_pkg  # noqa: F401
    from adipose_amd import ops
    from adipose_amd.data import synthetic_tile, to_gray
    from adipose_amd.nets import AdiposeV3Net
    from adipose_amd.predictor import INFER_CPAD, HipUnetPredictor, SlidingWindowInference

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    T = args.tile
    cpad = args.cpad or (INFER_CPAD if args.dtype == "bf16" else None)
    net = AdiposeV3Net(1, T, dtype=args.dtype, device=dev, seed=865, deep_supervision=False, cpad=cpad)
    pred = HipUnetPredictor(net, max_batch=args.batch)
    rng = np.random.default_rng(865)
    if args.mode == "wsi":
        # synthetic WSI: an 8 x 8 mosaic of independently drawn histology-like 1024^2 tiles (gray)
        S = args.size
        n = (S + T - 1) // T
        wsi = np.zeros((n * T, n * T), np.float32)
        for i in range(n):
            for j in range(n):
                wsi[i * T:(i + 1) * T, j * T:(j + 1) * T] = to_gray(synthetic_tile(rng, T, 3)[0])
        wsi = wsi[:S, :S]
        mean, std = float(wsi.mean()), float(wsi.std())
        img = torch.from_numpy(np.ascontiguousarray(wsi)).to(dev)
        sw = SlidingWindowInference(T, args.overlap, "gaussian", process_group=dist.group.WORLD if world > 1 else None,
                                    verbose=False)
        npos = len(sw.extract_tile_positions((S, S)))
        use_tta = args.tta != "none"
        nviews = {"none": 1, "minimal": 2, "basic": 4, "full": 8}[args.tta]

        def step():
            return sw.predict_with_sliding_window(img, pred, mean, std, use_tta=use_tta,
                                                  tta_mode=args.tta if use_tta else "basic", return_device=True)
        forwards = npos * nviews
        unit_name = "WSI/s"
    else:
        tiles = [to_gray(synthetic_tile(rng, T, 3)[0]).astype(np.float32) for _ in range(args.batch)]
        mean, std = float(np.mean(tiles)), float(np.std(tiles))
        dtiles = [torch.from_numpy(t).to(dev) for t in tiles]

        def step():
            return pred.predict_views(dtiles, mean, std, [0])
        forwards = args.batch
        unit_name = "tiles/s"

    for _ in range(args.warmup):
        out = step()
    torch.cuda.synchronize()
    timer = ops.LaunchTimer()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ops.set_launch_timer(timer)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ops.set_launch_timer(None)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    checksum = float(out.double().sum().item())
    summ = timer.summary()
    if rank == 0:
        dom = max(summ.items(), key=lambda kv: kv[1][2])
        (kname, dcode), (n, flops, ms) = dom
        dname = "bf16" if dcode == 1 else "f32"
        achieved = flops / (ms * 1e-3) / 1e12
        tot_ms = sum(v[2] for v in summ.values())
        # forward FLOPs executed per tile (all ranks): the wsi mode counts every rank's forwards
        fwd_gflop = V3_FWD_GFLOP_1024 * (T / 1024.0) ** 2
        per_fwd_ms = elapsed * 1e3 / (args.steps * (forwards if args.mode == "tiles" else forwards))
        line = {
            "metric": ("8192^2 WSI/s (sliding window 75% overlap + 8-way TTA)" if args.mode == "wsi"
                       else "1024^2 tiles/s (forward)"),
            "value": round(args.steps / elapsed if args.mode == "wsi" else args.steps * forwards / elapsed, 6),
            "unit": unit_name, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong" if args.mode == "wsi" else "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (seeded histology-like gray mosaic, resident in HBM)",
            "config": {"workload": (f"adipose_v3 SW+TTA({args.tta}) {args.size}^2 WSI, tile {T}, overlap {args.overlap}"
                                    if args.mode == "wsi" else f"adipose_v3 forward {T}^2 B={args.batch}"),
                       "tile_positions": npos if args.mode == "wsi" else None,
                       "tile_forwards_per_step": forwards, "batch": args.batch,
                       "parallelism": f"tile-rows x{world}" if args.mode == "wsi" else f"replicas x{world}"},
            "tile_forwards_per_s": round(args.steps * forwards / elapsed, 3),
            "fwd_tflops_effective": round(args.steps * forwards * fwd_gflop / elapsed / 1e3, 2),
            "ms_per_tile_forward": round(per_fwd_ms, 4),
            "checksum": checksum,
            "roofline": {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 2),
                         "peak": MI355X_PEAK[dname], "unit": "TFLOP/s", "frac": round(achieved / MI355X_PEAK[dname], 4),
                         "avg_launch_ms": round(ms / n, 4), "launches": n,
                         "conv_share_of_time": round(tot_ms / (elapsed * 1e3), 4),
                         "per_kernel": {k[0]: {"launches": v[0], "avg_ms": round(v[2] / v[0], 4),
                                               "tflops": round(v[1] / (v[2] * 1e-3) / 1e12, 2)}
                                        for k, v in sorted(summ.items(), key=lambda kv: -kv[1][2])}},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
