#!/usr/bin/env python3
"""bench.py — 1024^2 tiles/sec (train) of the MI355X-native U-Net step.

Workload (BASELINE.json configs[2], the configuration the metric "1024^2 tiles/sec (train)" is quoted
on; it fits one GPU): `unet_bn` 5-level U-Net, base 64 channels, 1024x1024x3 synthetic histology
tiles, bf16 compute (f32 accumulate, f32 master weights), batch 4 per GPU, pure data parallel (weak
scaling). One step = prep -> forward -> BCE+Dice loss/grad -> backward -> RCCL gradient all-reduce
(N>1, bucketed, overlapped with backward) -> Adam, on inputs already resident in HBM.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N>1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N)
Rank 0 prints ONE JSON line (plus `roofline` and `cpu_baseline` objects).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MI355X_PEAK = {"bf16": 2500.0, "f32": 157.3, "fp8": 5000.0}   # TFLOP/s dense (MI355X_MICROARCH.md chip table)
POST_STEPS = 2   # steps after the timed region with every GEMM launch timed (roofline per_kernel table)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--preset", default="unet_bn", choices=["unet_bn", "adipose_v3"])
    p.add_argument("--batch", type=int, default=4, help="tiles per GPU")
    p.add_argument("--size", type=int, default=1024)
    p.add_argument("--levels", type=int, default=5)
    p.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    p.add_argument("--cpad", type=lambda v: tuple(int(x) for x in v.split(",")), default=None, help="adipose_v3 channel-stride granule (default 64 for bf16)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-dice", action="store_true", help="skip the Dice@val leg (profiling runs)")
    p.add_argument("--dice-steps", type=int, default=2000,
                   help="Dice@val leg: training steps (a fixed count, so the value is one number per build on any box)")
    p.add_argument("--dice-seconds", type=float, default=90.0,
                   help="Dice@val leg: time cap on the training (the step count normally ends it first)")
    p.add_argument("--opt", action="append", default=[], help="name=value native option (A/B experiments only)")
    p.add_argument("--allreduce", default="overlap", choices=["overlap", "after"],
                   help="N > 1: gradient buckets all-reduced as the backward completes them (default) or all after it")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="collective backend for N > 1 (nccl = RCCL; gloo only to rehearse the multi-rank plumbing with "
                        "several ranks on one GPU)")
    return p.parse_args()


def host_threads():
    """Host threads for the CPU baseline: the CPUs this process may run on (sched_getaffinity), capped by
    the cgroup CPU quota when one is set (a GPU box shows the whole machine's CPUs but grants a share);
    returns (threads, description)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    n = min(aff, quota) if quota else aff
    return n, f"{aff} CPUs in the affinity mask" + (f", cgroup quota {quota} CPUs" if quota else ", no cgroup quota")


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, min_seconds=10.0, max_steps=60):
    """The reference's path on the host cores (BASELINE.md:30-44): the oracle's CPU fp32 restatement of
    AdiposeUNetV3 (oracle/torch_ref.py, train_adipose_unet_v3.py:660-758) training at BASELINE configs[0]
    (256x256 gray tiles, batch 2, fp32): forward, OHEM main + 0.4/0.3 deep-supervision BCE+Dice losses
    (compile_model :780-879), backward, Keras Adam. One untimed warm-up step, then steps until >= min_seconds
    and >= 3 steps. Reported in 1024^2-tile equivalents (16 256^2 tiles = one 1024^2 tile: the same FLOPs)."""
    import torch

    from oracle import torch_ref as R

    threads, tdesc = host_threads()
    torch.set_num_threads(threads)
    S, B = 256, 2
    g = torch.Generator().manual_seed(865)
    w = R.adipose_v3_keras_weights(seed=865)
    W = {k: [torch.tensor(v, requires_grad=True) for v in vs] for k, vs in w.items()}
    x = torch.randn(B, S, S, generator=g)
    y = (torch.rand(B, S, S, generator=g) > 0.7).float()
    params = [p for vs in W.values() for p in vs]
    opt = R.KerasAdam(params, lr=1e-4)

    def step():
        for p in params:
            p.grad = None
        R.ds_total_loss(y, R.adipose_v3_forward(x, W)).backward()
        opt.step([p.grad for p in params])

    step()   # warm-up (first-call allocations, thread pool start)
    n, t0 = 0, time.perf_counter()
    while n < 3 or (time.perf_counter() - t0 < min_seconds and n < max_steps):
        step()
        n += 1
    dt = time.perf_counter() - t0
    tiles = n * B * (S / 1024.0) ** 2
    return {"value": round(tiles / dt, 6), "unit": "1024^2 tiles/s (train, 1024^2-equivalent)", "cores": threads,
            "kind": "port", "cpu_model": cpu_model(),
            "sample": f"oracle adipose_v3 (reference topology) fp32 train steps at BASELINE configs[0]: {S}x{S} gray, "
                      f"B={B}, OHEM + deep-supervision losses, Keras Adam; 1 warm-up + {n} timed steps in {dt:.2f} s "
                      f"({n * B / dt:.3f} {S}^2 tiles/s); torch CPU, {threads} threads ({tdesc})"}


def gpu_same_workload(dev, min_seconds=3.0):
    """The CPU baseline's own workload on the GPU (round-5 VERDICT item 6): the product path's adipose_v3 (reference
    topology) f32 train step at BASELINE configs[0] (256x256 gray, B=2, OHEM + deep-supervision losses, Adam), so the
    baseline compares the same network and precision, not the headline's unet_bn bf16. Same 1024^2-equivalent unit."""
    import numpy as np
    import torch

    from adipose_amd.data import synthetic_batch, to_gray
    from adipose_amd.nets import AdiposeV3Net
    from adipose_amd.trainer import LossConfig, Trainer

    S, B = 256, 2
    net = AdiposeV3Net(B, S, dtype="f32", device=dev, seed=865)
    tr = Trainer(net, LossConfig(), lr=1e-4)
    xs, ys = synthetic_batch(B, S, channels=3, seed=865)
    xs = to_gray(xs.astype(np.float32))
    x = torch.from_numpy((xs - xs.mean()) / (xs.std() + 1e-10)).to(dev).contiguous()
    y = torch.from_numpy(ys).to(dev).contiguous()
    for _ in range(3):
        tr.train_step(x, y)
    torch.cuda.synchronize()
    n, t0 = 0, time.perf_counter()
    while n < 10 or time.perf_counter() - t0 < min_seconds:
        for _ in range(10):
            tr.train_step(x, y)
        n += 10
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    del tr, net
    torch.cuda.empty_cache()
    return {"value": round(n * B * (S / 1024.0) ** 2 / dt, 4), "unit": "1024^2 tiles/s (train, 1024^2-equivalent)",
            "ms_per_step": round(dt / n * 1e3, 3),
            "workload": "adipose_v3 (reference topology) 256x256x1 f32 B=2 (BASELINE configs[0]) on this GPU, "
                        f"{n} steps after 3 warm-up"}


def workload_label(args):
    """What this run trains, and which BASELINE.json config it is (if any)."""
    if args.preset == "unet_bn":
        wl = f"unet_bn L{args.levels} base64 {args.size}x{args.size}x3 {args.dtype} B={args.batch}/GPU"
        cfg = {(5, 1024, 4, "bf16"): 2, (4, 512, 8, "bf16"): 1}.get((args.levels, args.size, args.batch, args.dtype))
    else:
        wl = f"adipose_v3 (reference topology) {args.size}x{args.size}x1 {args.dtype} B={args.batch}/GPU"
        cfg = 0 if (args.size, args.batch, args.dtype) == (256, 2, "f32") else None
    return wl + (f" (BASELINE configs[{cfg}])" if cfg is not None else " (not a BASELINE config)")


def committed_traffic(kernel, workload, build):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary of THIS workload
    (profiles/<round>_traffic.json, written by tools/profile_round.sh from rocprofv3 FETCH_SIZE / WRITE_SIZE passes
    of the bench command, with the workload label and library build record of that run under "_meta");
    (None, None, None) when no summary of this workload holds the kernel — a profile of another workload is
    never used. The third value says whether the profiled library build is the one running now."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")))
    hits = []
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        meta = d.get("_meta") or {}
        if meta.get("workload") != workload:
            continue
        e = d.get(kernel)
        if e and e.get("traffic_bytes") is not None:
            hits.append((int(e["traffic_bytes"]), os.path.basename(f), meta.get("build") == build))
    # a summary of the running build first (file names sort by round, not by time within a round), else the last
    for h in hits:
        if h[2]:
            return h
    return hits[0] if hits else (None, None, None)


def dice_leg(args):
    """Dice@val of THIS build, measured in this process after the timed steps (round-4 VERDICT item 5): a fresh
    network of the benched workload (seed 865) trains --dice-steps steps (2000; round 6: a step count instead of 45 s,
    so that boxes of different speed report the same value for one build) on a pool of 128 distinct tiles of the
    hard synthetic task (data.synthetic_tile_hard; x 8 dihedral views) and is validated on its 64-tile seeded val
    stream as the reference monitors val_main_out_dice_coef (train_adipose_unet_v3.py:1267, :1316-1324; Keras
    dice_coef, src/utils/model.py:93-98, mean over val batches), plus the thresholded per-tile Dice of
    calculate_pixel_metrics; unet_bn also reports the fp8 forward (BASELINE configs[4]) on the same val tiles.
    The throughput steps train one resident batch, which says nothing about Dice."""
    from bench_converge import converge

    a = argparse.Namespace(preset=args.preset, levels=args.levels, size=args.size, batch=args.batch, dtype=args.dtype,
                           pool=128, val=64, lr=1e-3, max_steps=args.dice_steps, max_seconds=args.dice_seconds,
                           eval_every=400, target=0.9, fp8=args.preset == "unet_bn", hard=True, f32_eval=True)
    r = converge(a, log=lambda m: print(m, file=sys.stderr, flush=True))
    out = {k: r.get(k) for k in ("dice_val", "best_dice_val", "dice_val_thr", "steps", "train_seconds", "fp8", "f32",
                                  "build", "data")}
    out["curve"] = [(c["step"], c["dice_val"]) for c in r["curve"]]
    out["same_build"] = True   # (measured by this process on the library it benched)
    return out


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import _adipose_pkg  # noqa: F401
    from adipose_amd import _lib, ops
    from adipose_amd.data import synthetic_batch
    from adipose_amd.nets import AdiposeV3Net, UNetBN
    from adipose_amd.trainer import LossConfig, Trainer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.dist_backend == "gloo":   # rehearsal: ranks share the visible GPUs
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    for kv in args.opt:
        ops.set_option(kv.split("=")[0], int(kv.split("=")[1]))
    B, S = args.batch, args.size
    if args.preset == "unet_bn":
        net = UNetBN(B, S, levels=args.levels, base=64, in_ch=3, dtype=args.dtype, device=dev, seed=865)
        cfg = LossConfig(use_hard_mining=False)
        C = 3
    else:
        net = AdiposeV3Net(B, S, dtype=args.dtype, device=dev, seed=865, cpad=args.cpad)
        cfg = LossConfig()
        C = None
    tr = Trainer(net, cfg, lr=1e-4, distributed=world > 1, overlap_allreduce=args.allreduce == "overlap")

    # synthetic histology tiles, resident in HBM before timing (per-rank shard of the data)
    xs, ys = synthetic_batch(B, S, channels=3, seed=865 + rank)
    xs = xs.astype(np.float32)
    if C is None:
        from adipose_amd.data import to_gray
        xs = to_gray(xs)
    mean, std = float(xs.mean()), float(xs.std())
    x = torch.from_numpy((xs - mean) / (std + 1e-10)).to(dev).contiguous()
    y = torch.from_numpy(ys).to(dev).contiguous()

    # the last warm-up step times every GEMM launch to find the dominant kernel; the timed region then brackets
    # only that kernel's launches with event pairs (each pair costs the step ~4 us: all ~65 of a unet_bn step
    # cost it 1.3 %, profiles/r06l_timer_probe.log), and the other kernels' figures come from POST_STEPS
    # steps after the timed region with every launch timed
    dom_name = None
    for i in range(args.warmup):
        wt = ops.LaunchTimer() if i == args.warmup - 1 else None
        if wt is not None:
            ops.set_launch_timer(wt)
        tr.train_step(x, y)
        if wt is not None:
            ops.set_launch_timer(None)
            ws = wt.summary()
            if ws:
                dom_name = max(ws.items(), key=lambda kv: kv[1][2])[0][0]
    torch.cuda.synchronize()

    timer = ops.LaunchTimer(only=dom_name)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ops.set_launch_timer(timer)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.train_step(x, y)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    ops.set_launch_timer(None)
    elapsed = t1 - t0
    comm = None
    if world > 1:   # max over ranks; the per-rank times and the communicator's own rank count go into the line
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        per_rank = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(per_rank, t)
        ones = torch.ones(1, device=dev)
        dist.all_reduce(ones)   # (a live check: the sum over the communicator's ranks)
        comm = {"backend": dist.get_backend(), "ranks": dist.get_world_size(), "allreduce_check": int(ones.item()),
                "per_rank_ms_per_step": [round(v.item() / args.steps * 1e3, 3) for v in per_rank]}
        elapsed = max(v.item() for v in per_rank)
        world = dist.get_world_size()
    met = tr.read_metrics()

    summ = timer.summary()
    post = ops.LaunchTimer()   # (every rank: the steps all-reduce)
    ops.set_launch_timer(post)
    for _ in range(POST_STEPS):
        tr.train_step(x, y)
    ops.set_launch_timer(None)
    psumm = post.summary()
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    tiles = B * world * args.steps * (S / 1024.0) ** 2
    value = tiles / elapsed
    # roofline of the dominant kernel: the GEMM kernel instantiation with the largest total time
    # (names as rocprofv3 prints them; profiles/ holds the matching --kernel-trace --stats summary)
    dom = max(summ.items(), key=lambda kv: kv[1][2])
    (kname, dcode), (n, flops, ms, abytes) = dom
    dname = {0: "f32", 1: "bf16", 2: "fp8"}[dcode]
    achieved = flops / (ms * 1e-3) / 1e12
    step_ms = elapsed * 1e3 / args.steps
    # (per step: POST_STEPS steps after the timed region, every GEMM launch timed)
    per_kernel = {k[0]: {"launches": v[0], "avg_ms": round(v[2] / v[0], 4),
                         "tflops": round(v[1] / (v[2] * 1e-3) / 1e12, 2),
                         "alg_gbs": round(v[3] / (v[2] * 1e-3) / 1e9, 1),
                         "share_of_step": round(v[2] / POST_STEPS / step_ms, 4)}
                  for k, v in sorted(psumm.items(), key=lambda kv: -kv[1][2])}
    wl = workload_label(args)
    build = _lib.lib().adp_source_hash().decode()[:16]
    traffic, tsrc, same_build = committed_traffic(kname, wl, build)
    alg_bytes = abytes / n
    roof = {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 2),
            "peak": MI355X_PEAK[dname], "unit": "TFLOP/s", "frac": round(achieved / MI355X_PEAK[dname], 4),
            "traffic": traffic, "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": tsrc,
            "traffic_same_build": same_build,
            "algorithmic_bytes": round(alg_bytes),
            "traffic_over_algorithmic": round(traffic / alg_bytes, 3) if traffic and alg_bytes else None,
            "avg_launch_ms": round(ms / n, 4), "launches": n,
            "flops_per_launch": round(flops / n / 1e9, 3),
            "timing": ("the dominant kernel's launches of the timed region (HIP event pairs on its stream); "
                       f"per_kernel and the GEMM totals from {POST_STEPS} steps after it with every GEMM launch timed"),
            "gemm_share_of_step": round(sum(v[2] for v in psumm.values()) / POST_STEPS / step_ms, 4),
            "gemm_tflops_all": round(sum(v[1] for v in psumm.values()) / (sum(v[2] for v in psumm.values()) * 1e-3) / 1e12, 2),
            "per_kernel": per_kernel}
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args)
        except Exception as e:  # report, never fake
            cpu = {"value": None, "error": repr(e)}
        try:   # the like-for-like comparison: the CPU baseline's own network and precision on this GPU
            del tr, net, x, y
            torch.cuda.empty_cache()
            tr = net = x = y = None
            g = gpu_same_workload(dev)
            cpu["gpu_same_workload"] = g
            if cpu.get("value"):
                cpu["gpu_over_cpu_same_workload"] = round(g["value"] / cpu["value"], 1)
        except Exception as e:  # report, never fake
            cpu["gpu_same_workload"] = {"value": None, "error": repr(e)}
    dice = None
    if world == 1 and not args.no_dice:
        tr = net = x = y = None
        torch.cuda.empty_cache()
        try:
            dice = dice_leg(args)
        except Exception as e:  # report, never fake
            dice = {"dice_val": None, "error": repr(e)}
    line = {
        "metric": "1024^2 tiles/sec (train)", "value": round(value, 4), "unit": "tiles/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic (seeded histology-like tiles, resident in HBM)",
        "config": {"workload": wl, "preset": args.preset, "levels": args.levels if args.preset == "unet_bn" else 4,
                   "tile": S, "batch_per_gpu": B, "global_batch": B * world, "parallelism": f"dp{world}",
                   "allreduce": args.allreduce if world > 1 else None},
        "comm": comm,
        "build": build,
        "train_loss": round(met["loss"], 5), "dice_val": dice,
        "roofline": roof, "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
