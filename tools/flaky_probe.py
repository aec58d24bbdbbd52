"""Repeat the unet_bn f32 forward+backward parity case of tests/test_gpu_network.py many times in one
process and report, per repetition, the worst per-layer relative gradient error against the CPU oracle
and the run-to-run spread of the GPU gradients (localises an intermittent mismatch to a layer).

    python tools/flaky_probe.py [--reps 30] [--base 16] [--size 32] [--dtype f32]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _adipose_pkg  # noqa: E402,F401

import numpy as np  # noqa: E402
import torch  # noqa: E402

from adipose_amd import ops  # noqa: E402
from adipose_amd.nets import UNetBN  # noqa: E402
from adipose_amd.trainer import LossConfig, Trainer  # noqa: E402
from oracle import torch_ref as R  # noqa: E402
from tests.test_gpu_network import synth_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--base", type=int, default=16)
    ap.add_argument("--size", type=int, default=32)
    ap.add_argument("--levels", type=int, default=3)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--seed", type=int, default=33, help="data seed (9: the ill-conditioned round-1 case)")
    ap.add_argument("--fresh", type=int, default=1, help="1: new net per repetition, 0: reuse one net")
    args = ap.parse_args()
    B, L, S = 2, args.levels, args.size
    w = R.unet_bn_keras_weights(levels=L, base=args.base, in_ch=3, seed=5)
    x, y = synth_batch(B, S, C=3, seed=args.seed)
    W = {k: [torch.tensor(v, requires_grad=True) for v in vs] for k, vs in w.items()}
    p = R.unet_bn_forward(x, W, levels=L)
    R.combined_loss_standard(y, p).backward()
    # backward order of the GPU schedule: decoder level 0 first ... encoder level 0 last
    names = list(W.keys())
    first = None
    worst_all = 0.0
    net = None
    for rep in range(args.reps):
        if net is None or args.fresh:
            net = UNetBN(B, S, levels=L, base=args.base, in_ch=3, dtype=args.dtype, device="cuda")
            net.set_weights(w)
            tr = Trainer(net, LossConfig(use_hard_mining=False))
        else:
            net.set_weights(w)
        a = net.acts(B)
        ops.prep_input(x.to("cuda"), a["x"], mean=0.0, std=1.0)
        outs = net.forward(B, train=True)
        grads = tr.loss_and_grads(outs, y.to("cuda"))
        ops.fill(net.ps.grad, 0.0)
        net.backward(grads)
        torch.cuda.synchronize()
        errs = {}
        cur = {}
        for name in names:
            got = net.get_layer_grads(name)
            cur[name] = got
            for si, (gi, t) in enumerate(zip(got, W[name])):
                r = (torch.as_tensor(gi) - t.grad).abs().max().item() / max(t.grad.abs().max().item(), 1e-12)
                errs[(name, si)] = r
        worst = max(errs.values())
        worst_all = max(worst_all, worst)
        bad = [(k, round(v, 5)) for k, v in errs.items() if v >= 2e-3]
        spread = 0.0
        if first is None:
            first = cur
        else:
            for name in names:
                for gi, g0 in zip(cur[name], first[name]):
                    d = abs(torch.as_tensor(gi) - torch.as_tensor(g0)).max().item()
                    spread = max(spread, d / max(abs(torch.as_tensor(g0)).max().item(), 1e-12))
        fw = (outs["main_out"].cpu() - p.detach()).abs().max().item()
        bad.sort(key=lambda kv: -kv[1])
        print(f"rep {rep:3d} fwd {fw:.2e} worst {worst:.3e} spread-vs-rep0 {spread:.3e} bad {bad[:8]}", flush=True)
        # every persistent buffer (creation order = first-use order of the schedule) against rep 0's
        snap = {str(k[0]): t.detach().float().cpu().clone() for k, t in net._bufs.items()}
        if rep == 0:
            snap0 = snap
            grad0 = net.ps.grad.cpu().clone()
        elif spread > 1e-3:
            for k, t in snap.items():
                t0 = snap0.get(k)
                if t0 is None or t0.shape != t.shape:
                    continue
                d = (t - t0).abs()
                rel = d.max().item() / max(t0.abs().max().item(), 1e-12)
                if rel > 2e-5:
                    idx = torch.nonzero(d == d.max())[0].tolist()
                    print(f"    differing buffer {k} {tuple(t.shape)} rel {rel:.3e} at {idx} "
                          f"n_diff {(d > 1e-3 * t0.abs().max()).sum().item()}", flush=True)
            for n_, (o, shp, _) in net.ps.entries.items():
                if n_.endswith("/gamma") or n_.endswith("/beta"):
                    cnt = int(np.prod(shp))
                    d_ = (net.ps.grad.cpu()[o:o + cnt] - grad0[o:o + cnt])
                    chans = torch.nonzero(d_.abs() > 1e-4 * grad0[o:o + cnt].abs().max()).flatten().tolist()
                    if chans:
                        print(f"    {n_}: channels {chans[:16]} deltas {[round(d_[c].item(), 7) for c in chans[:6]]}")
            gd = (net.ps.grad.cpu() - grad0).abs()
            nz = torch.nonzero(gd > 1e-4 * grad0.abs().max()).flatten().tolist()
            for off in nz[:5]:
                owner = [n for n, (o, shp, _) in net.ps.entries.items() if o <= off < o + int(np.prod(shp))]
                print(f"    grad flat[{off}] {grad0[off].item():.6g} -> {net.ps.grad[off].item():.6g} {owner}")
    print(f"worst over reps {worst_all:.3e}")


if __name__ == "__main__":
    main()
