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

MI355X_PEAK = {"bf16": 2500.0, "f32": 157.3, "fp8": 5000.0}
DNAME = {0: "f32", 1: "bf16", 2: "fp8"}
# forward FLOPs of adipose_v3 per 1024^2 tile: 2 x 448.2 GMAC (counted from the layer list)
V3_FWD_GFLOP_1024 = 896.3


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--mode", default="wsi", choices=["wsi", "tiles", "fp8"])
    p.add_argument("--opt", action="append", default=[], help="name=value native option (A/B experiments only)")
    p.add_argument("--levels", type=int, default=5, help="unet_bn levels (mode fp8)")
    p.add_argument("--train-steps", type=int, default=60, help="mode fp8: bf16 training steps before the comparison")
    p.add_argument("--fp8-level0", type=int, default=1, help="mode fp8: level 0 in fp8 too (0: bf16, as in round 3)")
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


def fp8_main(args):
    """BASELINE.json configs[4]: fp8 (CDNA4 block-scaled MFMA) forward of the 1024^2 unet_bn network on one
    GPU, Dice within 1e-2 of bf16. The network (L5, base 64, random Keras-default init, seed 865) is first
    trained for --train-steps bf16 steps on synthetic histology tiles so that weights and BatchNorm running
    statistics are those of a fitted model; then a held-out synthetic batch is predicted in bf16 and in fp8
    and both are scored against its masks (calculate_pixel_metrics, threshold 0.5)."""
    import numpy as np
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd import ops
    from adipose_amd.data import synthetic_batch
    from adipose_amd.metrics import calculate_pixel_metrics
    from adipose_amd.nets import UNetBN
    from adipose_amd.trainer import LossConfig, Trainer

    for kv in args.opt:
        ops.set_option(kv.split("=")[0], int(kv.split("=")[1]))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, S = args.batch, args.tile
    net = UNetBN(B, S, levels=args.levels, base=64, in_ch=3, dtype="bf16", device=dev, seed=865)
    net.fp8_level0 = bool(args.fp8_level0)
    tr = Trainer(net, LossConfig(use_hard_mining=False), lr=1e-3)
    batches = []
    for k in range(2):
        xs, ys = synthetic_batch(B, S, channels=3, seed=865 + k)
        batches.append((xs.astype(np.float32), ys))
    mean = float(np.mean([b[0].mean() for b in batches]))
    std = float(np.mean([b[0].std() for b in batches]))
    dev_batches = [(torch.from_numpy((x - mean) / (std + 1e-10)).to(dev), torch.from_numpy(y).to(dev))
                   for x, y in batches]
    t0 = time.perf_counter()
    for i in range(args.train_steps):
        tr.train_step(*dev_batches[i % 2])
    torch.cuda.synchronize()
    train_s = time.perf_counter() - t0
    xv, yv = synthetic_batch(B, S, channels=3, seed=865 + 10_000)
    xvd = torch.from_numpy((xv.astype(np.float32) - mean) / (std + 1e-10)).to(dev)
    ops.prep_input(xvd, net.acts(B)["x"], mean=0.0, std=1.0)

    def run(fn, steps):
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        timer = ops.LaunchTimer()
        ops.set_launch_timer(timer)
        t = time.perf_counter()
        for _ in range(steps):
            out = fn()
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        ops.set_launch_timer(None)
        return out["main_out"].clone(), el, timer.summary()

    steps = max(args.steps, 5)
    p16, el16, _ = run(lambda: net.forward(B, train=False), steps)
    p8, el8, summ = run(lambda: net.forward_fp8(B), steps)
    y = yv.astype(np.float32)
    d16 = [calculate_pixel_metrics(p16[b].cpu().numpy(), y[b])["dice_score"] for b in range(B)]
    d8 = [calculate_pixel_metrics(p8[b].cpu().numpy(), y[b])["dice_score"] for b in range(B)]
    agree = [calculate_pixel_metrics(p8[b].cpu().numpy(), (p16[b].cpu().numpy() > 0.5).astype(np.float32))["dice_score"]
             for b in range(B)]
    f8 = {k: v for k, v in summ.items() if k[1] == 2}
    dom = max(f8.items(), key=lambda kv: kv[1][2])
    (kname, dcode), (n, flops, ms, _nb) = dom
    achieved = flops / (ms * 1e-3) / 1e12
    line = {
        "metric": "1024^2 tiles/s (fp8 forward) + Dice vs bf16", "value": round(steps * B / el8, 3), "unit": "tiles/s",
        "n_gpus": 1, "steps": steps, "warmup": args.warmup, "ms_per_step": round(el8 / steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp8 (e4m3fn)",
        "data": "synthetic (seeded histology-like tiles, resident in HBM)",
        "config": {"workload": f"unet_bn L{args.levels} base64 {S}x{S}x3 forward B={B} (BASELINE configs[4])",
                   "train_steps_before_eval": args.train_steps, "train_s": round(train_s, 2),
                   "fp8_layers": sorted(net._packed8), "fp8_level0": net.fp8_level0, "batch": B},
        "bf16_tiles_per_s": round(steps * B / el16, 3), "fp8_speedup": round(el16 / el8, 4),
        "dice_bf16": round(float(np.mean(d16)), 5), "dice_fp8": round(float(np.mean(d8)), 5),
        "dice_delta": round(abs(float(np.mean(d8)) - float(np.mean(d16))), 6),
        "dice_fp8_vs_bf16_masks": round(float(np.mean(agree)), 5),
        "max_abs_dprob": round((p8 - p16).abs().max().item(), 5),
        "roofline": {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 2), "peak": MI355X_PEAK["fp8"],
                     "unit": "TFLOP/s", "frac": round(achieved / MI355X_PEAK["fp8"], 4),
                     "avg_launch_ms": round(ms / n, 4), "launches": n,
                     "per_kernel": {f"{k[0]} [{DNAME[k[1]]}]": {"launches": v[0], "avg_ms": round(v[2] / v[0], 4),
                                                               "tflops": round(v[1] / (v[2] * 1e-3) / 1e12, 2)}
                                    for k, v in sorted(summ.items(), key=lambda kv: -kv[1][2])}},
    }
    print(json.dumps(line), flush=True)


def main():
    args = parse()
    if args.mode == "fp8":
        if args.batch == 8 and args.tile == 1024:
            args.batch = 4
        return fp8_main(args)
    import numpy as np
    import torch
    import torch.distributed as dist

    import _adipose_pkg  # noqa: F401
    from adipose_amd import ops
    from adipose_amd.data import synthetic_tile, to_gray
    from adipose_amd.nets import AdiposeV3Net
    from adipose_amd.predictor import INFER_CPAD, HipUnetPredictor, SlidingWindowInference
    for kv in args.opt:
        ops.set_option(kv.split("=")[0], int(kv.split("=")[1]))

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
    checksum = float(out.double().sum().item()) if out is not None else None   # (wsi: the frame is on rank 0)
    summ = timer.summary()
    if rank == 0:
        dom = max(summ.items(), key=lambda kv: kv[1][2])
        (kname, dcode), (n, flops, ms, _nb) = dom
        dname = DNAME[dcode]
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
