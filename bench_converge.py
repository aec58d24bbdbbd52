#!/usr/bin/env python3
"""bench_converge.py — Dice@val of the MI355X-native training step, measured as the reference measures it.

The reference validates on held-out tiles every epoch and monitors `val_main_out_dice_coef`
(Segmentation/train_adipose_unet_v3.py:1267, :1316-1324): Keras' `dice_coef` (src/utils/model.py:93-98,
(2 sum(yp) + 1) / (sum(y) + sum(p) + 1) over the whole batch, no threshold) averaged over the validation batches.
This script trains on a seeded stream of DISTINCT synthetic histology tiles (a pool of --pool tiles drawn without
a repeated batch, each draw under a random dihedral view: 8 x pool distinct inputs), evaluates every --eval-every
steps on the separate 64-tile seeded val stream of SURVEY.md §8d (seed 865 + 10000), and reports:

  * dice_val: the Keras val_main_out_dice_coef (mean over val batches), plus the thresholded per-tile Dice of
    calculate_pixel_metrics (full_evaluation_enhanced.py:721-785, threshold 0.5) on the same tiles;
  * the training time (eval passes excluded) and steps to reach --target, and the curve;
  * --fp8 (unet_bn, BASELINE configs[4]): the fp8 forward's Dice on the same val tiles and its delta to bf16.

Default workload: BASELINE configs[2] on one GPU (unet_bn L5 base 64, 1024^2 x 3, bf16, B = 4), BCE + Dice,
Adam lr 1e-3. Prints ONE JSON line (progress lines go to stderr)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--preset", default="unet_bn", choices=["unet_bn", "adipose_v3"])
    p.add_argument("--levels", type=int, default=5)
    p.add_argument("--size", type=int, default=1024)
    p.add_argument("--batch", type=int, default=4)
    p.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    p.add_argument("--pool", type=int, default=256, help="distinct training tiles (seed 865 stream)")
    p.add_argument("--val", type=int, default=64, help="val tiles (seed 865 + 10000 stream)")
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--max-steps", type=int, default=1500)
    p.add_argument("--max-seconds", type=float, default=150.0, help="training time budget (eval excluded)")
    p.add_argument("--eval-every", type=int, default=100)
    p.add_argument("--target", type=float, default=0.9, help="val_main_out_dice_coef to time")
    p.add_argument("--fp8", action="store_true", help="unet_bn: also the fp8 forward's Dice on the val tiles")
    p.add_argument("--hard", action="store_true",
                   help="the harder synthetic task (data.synthetic_tile_hard: packed touching cells, torn membranes, "
                        "stroma, non-fat lumens, stain noise) instead of the ellipse tiles")
    return p.parse_args()


def log(msg):
    print(msg, file=sys.stderr, flush=True)


def main():
    print(json.dumps(converge(parse(), log=log)), flush=True)


def converge(args, log=log):
    """Train a fresh network on the seeded distinct-tile stream and validate on the 64-tile val stream; returns
    the result line (a dict). `args` carries the fields of parse() (bench.py builds one for its Dice leg)."""
    import numpy as np
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd import _lib, ops
    from adipose_amd.data import synthetic_tile, to_gray
    from adipose_amd.metrics import calculate_pixel_metrics
    from adipose_amd.nets import AdiposeV3Net, UNetBN
    from adipose_amd.trainer import LossConfig, Trainer
    from bench import workload_label

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, S = args.batch, args.size
    gray = args.preset == "adipose_v3"

    def stream(seed, n, what):
        rng = np.random.default_rng(seed)
        xs, ys = [], []
        t0 = time.perf_counter()
        for i in range(n):
            x, y = synthetic_tile(rng, S, 3)
            xs.append(to_gray(x).astype(np.float32) if gray else x)
            ys.append(y)
            if (i + 1) % 32 == 0:
                log(f"{what}: {i + 1}/{n} tiles ({time.perf_counter() - t0:.1f} s)")
        return np.stack(xs), np.stack(ys)

    if getattr(args, "hard", False):   # generated on the device (torch, outside every timed step)
        from adipose_amd.data import synthetic_stream_hard

        def stream_hard(seed, n, what):
            t0 = time.perf_counter()
            x, y = synthetic_stream_hard(seed, n, S, 3, device=dev)
            if gray:
                x = (x[..., 0].float() * 0.299 + x[..., 1].float() * 0.587 + x[..., 2].float() * 0.114)
            torch.cuda.synchronize()
            log(f"{what}: {n} hard tiles ({time.perf_counter() - t0:.1f} s)")
            return x, y

        XP, YP = stream_hard(865, args.pool, "train pool")
        XV, YV = stream_hard(865 + 10_000, args.val, "val")
        mean, std = float(XP.float().mean()), float(XP.float().std())
    else:
        xp, yp = stream(865, args.pool, "train pool")
        xv, yv = stream(865 + 10_000, args.val, "val")
        mean, std = float(xp.astype(np.float32).mean()), float(xp.astype(np.float32).std())
        # resident in HBM: the pool as stored (u8 RGB / f32 gray), normalised per batch on the device
        XP = torch.from_numpy(xp).to(dev)
        YP = torch.from_numpy(yp.astype(np.float32)).to(dev)
        XV = torch.from_numpy(xv).to(dev)
        YV = torch.from_numpy(yv.astype(np.float32)).to(dev)

    if args.preset == "unet_bn":
        net = UNetBN(B, S, levels=args.levels, base=64, in_ch=3, dtype=args.dtype, device=dev, seed=865)
        cfg = LossConfig(use_hard_mining=False)
    else:
        net = AdiposeV3Net(B, S, dtype=args.dtype, device=dev, seed=865)
        cfg = LossConfig()
    wl = workload_label(args)   # the same label as the throughput line of bench.py
    tr = Trainer(net, cfg, lr=args.lr)

    def norm(x):
        return ((x.float() - mean) / (std + 1e-10)).contiguous()

    g = torch.Generator().manual_seed(865)

    def batch():
        """B distinct pool tiles (an epoch-wise permutation), each under a random dihedral view."""
        nonlocal perm, pos
        if pos + B > len(perm):
            perm, pos = torch.randperm(args.pool, generator=g).tolist(), 0
        idx = perm[pos:pos + B]
        pos += B
        xs, ys = [], []
        for i in idx:
            v = int(torch.randint(0, 8, (1,), generator=g))
            x, y = XP[i], YP[i]
            if v & 4:
                x, y = x.flip(1), y.flip(1)
            x, y = torch.rot90(x, v & 3, (0, 1)), torch.rot90(y, v & 3, (0, 1))
            xs.append(x)
            ys.append(y)
        return norm(torch.stack(xs)), torch.stack(ys).contiguous()

    perm, pos = [], 1 << 30

    def evaluate(fp8=False):
        """val_main_out_dice_coef (Keras: batch-global dice_coef, mean over val batches) and the thresholded
        per-tile Dice (calculate_pixel_metrics at 0.5)."""
        kd, td = [], []
        for b0 in range(0, args.val, B):
            x, y = norm(XV[b0:b0 + B]), YV[b0:b0 + B]
            ops.prep_input(x, net.acts(B)["x"], mean=0.0, std=1.0)
            p = (net.forward_fp8(B) if fp8 else net.forward(B, train=False))["main_out"].float()
            kd.append(((2 * (y * p).sum() + 1) / (y.sum() + p.sum() + 1)).item())
            td.extend(calculate_pixel_metrics(p[k].contiguous(), y[k].contiguous())["dice_score"] for k in range(B))
        return float(np.mean(kd)), float(np.mean(td))

    curve = []
    t_train, step, hit = 0.0, 0, None
    d0 = evaluate()
    curve.append({"step": 0, "train_s": 0.0, "dice_val": round(d0[0], 5), "dice_val_thr": round(d0[1], 5)})
    log(f"step 0: dice_val {d0[0]:.4f} (thresholded {d0[1]:.4f})")
    while step < args.max_steps and t_train < args.max_seconds:
        xb, yb = batch()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = min(args.eval_every, args.max_steps - step)
        for k in range(n):
            tr.train_step(xb, yb)
            if k % 25 == 24:   # (the time budget holds inside an eval interval too)
                torch.cuda.synchronize()
                if t_train + time.perf_counter() - t0 >= args.max_seconds:
                    n = k + 1
                    break
            if k + 1 < n:
                xb, yb = batch()
        torch.cuda.synchronize()
        t_train += time.perf_counter() - t0
        step += n
        loss = tr.read_metrics()["loss"]
        d = evaluate()
        curve.append({"step": step, "train_s": round(t_train, 3), "train_loss": round(loss, 5),
                      "dice_val": round(d[0], 5), "dice_val_thr": round(d[1], 5)})
        log(f"step {step}: {t_train:.1f} s train, loss {loss:.4f}, dice_val {d[0]:.4f} (thresholded {d[1]:.4f})")
        if hit is None and d[0] >= args.target:
            hit = {"step": step, "train_s": round(t_train, 3)}
    final = curve[-1]
    task = "hard synthetic histology (data.synthetic_tile_hard)" if getattr(args, "hard", False) else \
        "synthetic histology (ellipse tiles, data.synthetic_tile)"
    line = {"metric": "Dice@val (val_main_out_dice_coef) after 1024^2 training", "workload": wl,
            "build": _lib.lib().adp_source_hash().decode()[:16],
            "data": f"{task}: {args.pool} distinct seeded train tiles x 8 dihedral views, "
                    f"{args.val} seeded val tiles (SURVEY §8d); dataset z-score",
            "optimizer": f"Adam lr {args.lr}", "loss": "BCE + Dice" if args.preset == "unet_bn" else "OHEM + DS",
            "dice_val": final["dice_val"], "dice_val_thr": final["dice_val_thr"],
            "best_dice_val": max(c["dice_val"] for c in curve), "steps": step, "train_seconds": round(t_train, 3),
            "tiles_per_s_incl_feed": round(step * B * (S / 1024.0) ** 2 / t_train, 3) if t_train else None,
            "target": args.target, "time_to_target": hit, "curve": curve}
    if args.fp8:
        if args.preset != "unet_bn":
            raise SystemExit("--fp8: the fp8 forward is the unet_bn preset's (BASELINE configs[4])")
        d8 = evaluate(fp8=True)
        line["fp8"] = {"dice_val": round(d8[0], 5), "dice_val_thr": round(d8[1], 5),
                       "delta_dice_val": round(d8[0] - final["dice_val"], 7),
                       "delta_dice_val_thr": round(d8[1] - final["dice_val_thr"], 7)}
    if getattr(args, "f32_eval", False) and args.dtype == "bf16":
        # the same trained weights (f32 masters) and BatchNorm running statistics in an f32 twin of the network:
        # the bf16 forward's Dice against the reference precision's on the same val tiles (round-5 VERDICT item 8)
        if args.preset == "unet_bn":
            twin = UNetBN(B, S, levels=args.levels, base=64, in_ch=3, dtype="f32", device=dev, seed=865)
        else:
            twin = AdiposeV3Net(B, S, dtype="f32", device=dev, seed=865)
        if twin.ps.flat.numel() != net.ps.flat.numel():
            line["f32"] = {"error": "the f32 twin packs its weights differently"}
        else:
            twin.ps.flat.copy_(net.ps.flat)
            for k, (rm, rv) in getattr(net, "running", {}).items():
                twin.running[k][0].copy_(rm)
                twin.running[k][1].copy_(rv)
            keep = net
            net = twin
            try:
                d32 = evaluate()
            finally:
                net = keep
            line["f32"] = {"dice_val": round(d32[0], 5), "dice_val_thr": round(d32[1], 5),
                           "delta_bf16_minus_f32": round(final["dice_val"] - d32[0], 7),
                           "delta_bf16_minus_f32_thr": round(final["dice_val_thr"] - d32[1], 7)}
            if args.fp8:
                line["fp8"]["delta_vs_f32"] = round(line["fp8"]["dice_val"] - d32[0], 7)
        del twin
        torch.cuda.empty_cache()
    return line


if __name__ == "__main__":
    main()
