"""One training step of the U-Net hot path on the GPU: forward -> BCE+Dice / OHEM loss + gradient ->
backward -> (DP) RCCL gradient all-reduce overlapped with the backward convs -> fused Adam.

Semantics follow the reference's Keras training (Segmentation/train_adipose_unet_v3.py):
  * loss selection and deep-supervision weights: compile_model :780-879 (main/aux1/aux2 = 1.0/0.4/0.3)
  * losses: dice_loss :217-225 (batch-global), combined_loss_standard :228-241, label smoothing
    :244-279, OHEM :282-363 (per-ROW BCE, k = int(H * ratio) rows per image)
  * Adam(lr, beta 0.9/0.999, eps 1e-7) / AdamW(weight_decay=0.01) :800-806 (Keras 2.13 update rule)
  * encoder freezing (phase 1): freeze_encoder_layers :760-772 — frozen layers get no gradient and
    no optimizer update; their data-gradients are not even computed.

Data parallel (new; the reference is single-GPU): one process per GPU. The loss is
normalised with GLOBAL counts and the Dice sums (Σyp, Σy, Σp per head) are all-reduced before the
loss gradient, so the summed per-rank gradients equal the single-device gradient of the global batch
exactly; gradients are SUM-all-reduced in buckets launched as soon as the backward pass has finished
every layer of a bucket (RCCL runs on its own stream, overlapping the remaining backward kernels).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from . import ops


@dataclass
class LossConfig:
    use_hard_mining: bool = True
    hard_example_ratio: float = 0.7
    use_label_smoothing: bool = False
    epsilon_pos: float = 0.03
    epsilon_neg: float = 0.07
    ds_weight_main: float = 1.0
    ds_weight_aux1: float = 0.4
    ds_weight_aux2: float = 0.3
    main_ohem_override: bool | None = None  # unet_bn preset: plain BCE+Dice

    def head_specs(self, outputs):
        """[(name, weight, ohem)] in the order of the network outputs."""
        specs = [("main_out", self.ds_weight_main if len(outputs) > 1 else 1.0,
                  self.use_hard_mining if self.main_ohem_override is None else self.main_ohem_override)]
        if "aux_out1" in outputs:
            specs += [("aux_out1", self.ds_weight_aux1, False), ("aux_out2", self.ds_weight_aux2, False)]
        return specs


def dp_row_normaliser(world, batch_local, rows_kept):
    """Denominator of every per-row BCE coefficient under data parallelism: the GLOBAL number of kept
    rows (world x local batch x rows kept per image), so the per-rank row terms sum to the reference's
    single-device mean over the whole batch (Keras SUM_OVER_BATCH_SIZE of the per-row BCE; the OHEM
    top-k mean of train_adipose_unet_v3.py:282-318). The Dice term is made batch-global by
    all-reducing its three sums before the gradient (Trainer.loss_and_grads)."""
    return float(world * batch_local * rows_kept)


def plan_buckets(ps, bucket_bytes):
    """[(layer names, lo, hi)]: the flat gradient buffer cut into spans of about bucket_bytes, in the order the
    backward pass completes them (from the end of the buffer), each span whole layers."""
    spans = {}   # layer -> [start, end) span in the flat buffer (a layer's params are contiguous)
    for name, (off, shape, _) in ps.entries.items():
        lname = name.rsplit("/", 1)[0]
        n = int(np.prod(shape))
        lo, hi = spans.get(lname, (off, off))
        spans[lname] = (min(lo, off), max(hi, off + ops.round_up(n, 64)))
    order = sorted(spans.items(), key=lambda kv: kv[1][0], reverse=True)
    buckets = []
    cur, cur_lo, cur_hi = [], None, None
    for lname, (lo, hi) in order:
        if cur and (cur_hi - lo) * 4 > bucket_bytes:
            buckets.append((set(cur), cur_lo, cur_hi))
            cur, cur_hi = [], None
        cur.append(lname)
        cur_lo = lo
        cur_hi = hi if cur_hi is None else cur_hi
    if cur:
        buckets.append((set(cur), cur_lo, cur_hi))
    return buckets


class GradBuckets:
    """Bucketed, backward-overlapped SUM all-reduce over the flat gradient buffer. overlap=False launches every
    bucket at finish() instead (the same sums): while an RCCL bucket holds CUs, a persistent conv kernel's
    blocks that find no free CU run after the others, so an overlapped bucket can cost as much as an exposed one
    (profiles/r03_contention_probe.txt); the switch is there to measure both on a multi-GPU node."""

    def __init__(self, net, bucket_bytes=16 << 20, group=None, overlap=True, launch_group=2):
        self.group = group
        self.overlap = overlap
        self.world = dist.get_world_size(group)
        self.buckets = plan_buckets(net.ps, bucket_bytes)
        self.ps = net.ps
        self.net = net
        self.works = []
        # buckets whose layers are done wait until launch_group of them are ready (or the backward ends) and go out
        # together behind ONE flush of the deferred weight-gradient reductions (round 6): with a flush per bucket the
        # backward's batched reductions were split into as many launches as buckets
        self.launch_group = max(1, int(launch_group))
        self.queued = []
        self.launches = 0   # (flush + launch points of the last backward)

    def begin(self, frozen=()):
        self.pending = [set(b[0]) - set(frozen) for b in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.works = []
        self.queued = []
        self.launches = 0

    def ready(self, lname):
        if not self.overlap:
            return
        for i, p in enumerate(self.pending):
            if lname in p:
                p.discard(lname)
                if not p and not self.launched[i] and i not in self.queued:
                    self.queued.append(i)
        if len(self.queued) >= self.launch_group:
            self._launch_queued()

    def _launch_queued(self):
        if not self.queued:
            return
        self.launches += 1
        if getattr(self.net, "_deferring", False):   # the buckets' gradients are final after the recorded reductions
            ops.wgrad_flush()
            ops.wgrad_defer(True)
        for i in self.queued:
            _, lo, hi = self.buckets[i]
            self.launched[i] = True
            self.works.append(dist.all_reduce(self.ps.grad[lo:hi], op=dist.ReduceOp.SUM, group=self.group,
                                              async_op=True))
        self.queued = []

    def _launch(self, i):
        if not self.launched[i] and i not in self.queued:
            self.queued.append(i)
        self._launch_queued()

    def abort(self):
        """Error path of a backward: the buckets already issued may still read the gradient buffer on the RCCL
        stream; the current stream waits for them before anything (the next step's zero-fill) writes it."""
        for w in self.works:
            w.wait()
        self.works = []

    def finish(self):
        # every gradient is final here: reduce any bucket a ready-hook did not launch (a layer that never
        # reported, or frozen-only buckets, whose zero gradients are harmless to sum)
        for i, done in enumerate(self.launched):
            if not done and i not in self.queued:
                self.queued.append(i)
        self._launch_queued()
        for w in self.works:
            w.wait()  # current stream waits on the RCCL stream
        self.works = []


class Trainer:
    """Owns optimizer state and loss buffers for one UNetEngine."""

    def __init__(self, net, loss_cfg: LossConfig | None = None, *, optimizer="adam", lr=1e-4, beta1=0.9,
                 beta2=0.999, eps=1e-7, weight_decay=0.01, process_group=None, distributed=None,
                 bucket_bytes=16 << 20, overlap_allreduce=True):
        self.net = net
        self.cfg = loss_cfg or LossConfig()
        self.opt = optimizer.lower()
        self.lr, self.b1, self.b2, self.eps = lr, beta1, beta2, eps
        self.wd = weight_decay if self.opt == "adamw" else 0.0
        dev = net.device
        self.m = torch.zeros_like(net.ps.flat)
        self.v = torch.zeros_like(net.ps.flat)
        self.iterations = 0
        self.distributed = dist.is_available() and dist.is_initialized() if distributed is None else distributed
        self.group = process_group
        self.world = dist.get_world_size(process_group) if self.distributed else 1
        self.buckets = (GradBuckets(net, bucket_bytes, process_group, overlap=overlap_allreduce)
                        if self.distributed and self.world > 1 else None)
        # (data parallel keeps the persistent kernels' static tile lists: with the bucket schedule -- each bucket's
        # all-reduce holding CUs for a fraction of a millisecond -- static lists cost the overlapped step +0.4-0.5 ms
        # against +0.7 ms with claimed tiles, whose kernels are 3-11 % slower on an idle chip, and +1.9-2.2 ms for
        # the exposed all-reduce: profiles/r04c_bucket_probe.log, DESIGN.md §5. Option dp_claim=1 turns claiming on.)
        self.stats = torch.zeros((3, 8), dtype=torch.float64, device=dev)   # per head: loss_rows sums
        self.lossbuf = torch.zeros(4, dtype=torch.float64, device=dev)
        self._dp = {}
        self._frozen = ()

    # -------------------------------------------------------------------------- freezing
    def set_frozen(self, names):
        """Freeze layers (no grads, no updates). Encoder freezing = AdiposeUNetV3.freeze_encoder_layers."""
        self._frozen = tuple(names)
        if hasattr(self.net, "frozen_encoder"):
            self.net.frozen_encoder = bool(names)

    def trainable_ranges(self):
        """Contiguous [lo, hi) ranges of the flat buffer that the optimizer updates."""
        ps = self.net.ps
        frozen = set(self._frozen)
        rngs = []
        for name, (off, shape, _) in ps.entries.items():
            if name.rsplit("/", 1)[0] in frozen:
                continue
            hi = off + ops.round_up(int(np.prod(shape)), 64)
            if rngs and rngs[-1][1] == off:
                rngs[-1][1] = hi
            else:
                rngs.append([off, hi])
        return rngs

    # ------------------------------------------------------------------------------ loss
    def _dpbuf(self, name, shape):
        t = self._dp.get((name, shape))
        if t is None:
            t = torch.zeros(shape, dtype=torch.float32, device=self.net.device)
            self._dp[(name, shape)] = t
        return t

    def loss_and_grads(self, outputs, y, *, compute_grad=True):
        """Loss (device scalars) and dL/dp for every head; y: (B,S,S) f32 labels on device."""
        cfg = self.cfg
        B, H, W = y.shape
        specs = cfg.head_specs(outputs)
        ops.fill(self.stats.view(torch.float32), 0.0)
        ops.fill(self.lossbuf.view(torch.float32), 0.0)
        rows = {}
        for i, (name, w, ohem) in enumerate(specs):
            rb = self._dpbuf("rows/" + name, (B * H,))
            ops.loss_rows(outputs[name], y, rb, self.stats[i], smooth=cfg.use_label_smoothing,
                          eps_pos=cfg.epsilon_pos, eps_neg=cfg.epsilon_neg)
            rows[name] = rb
        if self.buckets is not None or (self.distributed and self.world > 1):
            dist.all_reduce(self.stats, op=dist.ReduceOp.SUM, group=self.group)
        grads = {}
        for i, (name, w, ohem) in enumerate(specs):
            k = int(np.float32(H) * np.float32(cfg.hard_example_ratio)) if ohem else H
            coef = self._dpbuf("coef/" + name, (B * H,))
            ops.loss_select(rows[name], coef, self.lossbuf[i:i + 1], N=B, H=H, W=W, ohem=ohem,
                            keep_ratio=cfg.hard_example_ratio, weight=w, norm_rows=dp_row_normaliser(self.world, B, k))
            if compute_grad:
                dp = self._dpbuf("dp/" + name, (B, H, W))
                ops.loss_grad(outputs[name], y, coef, self.stats[i], dp, weight=w, smooth=cfg.use_label_smoothing,
                              eps_pos=cfg.epsilon_pos, eps_neg=cfg.epsilon_neg)
                grads[name] = dp
        self._specs = specs
        return grads

    def read_metrics(self):
        """Host read-back (synchronises): total loss, per-head losses, dice_coef and accuracy of main."""
        st = self.stats.cpu().numpy()
        lb = self.lossbuf.clone()
        if self.distributed and self.world > 1:
            dist.all_reduce(lb, op=dist.ReduceOp.SUM, group=self.group)
        lb = lb.cpu().numpy()
        out = {}
        total = 0.0
        for i, (name, w, _) in enumerate(self._specs):
            dice = 1.0 - (2 * st[i, 0] + 1) / (st[i, 1] + st[i, 2] + 1)
            li = lb[i] / w + dice if w else 0.0
            out[name + "_loss"] = float(li)
            total += w * li
        out["loss"] = float(total)
        out["main_out_dice_coef"] = float((2 * st[0, 3] + 1) / (st[0, 4] + st[0, 5] + 1))
        out["main_out_binary_accuracy"] = float(st[0, 6] / self._npix) if getattr(self, "_npix", 0) else float("nan")
        return out

    # ------------------------------------------------------------------------------ step
    def train_step(self, x_norm, y, *, lr=None):
        """x_norm: (B,S,S) or (B,S,S,C) normalised f32 device tensor; y: (B,S,S) f32 labels."""
        net = self.net
        B = y.shape[0]
        a = net.acts(B)
        ops.bn_fold_reset()   # a failed earlier step may have left a deferred BatchNorm fold pending
        ops.prep_input(x_norm, a["x"], mean=0.0, std=1.0)
        self.iterations += 1
        outs = net.forward(B, train=True, seed=self.iterations)
        grads = self.loss_and_grads(outs, y)
        self._npix = B * y.shape[1] * y.shape[2] * self.world
        ops.fill(net.ps.grad, 0.0)
        if self.buckets is not None:
            self.buckets.begin(frozen=self._frozen)
            net.grad_hook = self.buckets.ready
        try:
            net.backward(grads)
        except BaseException:
            if self.buckets is not None:
                self.buckets.abort()
            raise
        finally:
            net.grad_hook = None
        if self.buckets is not None:
            self.buckets.finish()
        self.apply_gradients(lr)

    def apply_gradients(self, lr=None):
        lr = self.lr if lr is None else lr
        ps = self.net.ps
        for lo, hi in self.trainable_ranges():
            ops.adam(ps.flat[lo:hi], ps.grad[lo:hi], self.m[lo:hi], self.v[lo:hi], lr=lr, beta1=self.b1,
                     beta2=self.b2, eps=self.eps, step=self.iterations, weight_decay=self.wd)

    def eval_step(self, x_norm, y):
        net = self.net
        B = y.shape[0]
        a = net.acts(B)
        ops.prep_input(x_norm, a["x"], mean=0.0, std=1.0)
        outs = net.forward(B, train=False)
        self.loss_and_grads(outs, y, compute_grad=False)
        self._npix = B * y.shape[1] * y.shape[2] * self.world
        return outs


def cosine_warmup_lr(epoch, max_lr, min_lr, warmup_epochs, total_epochs):
    """CosineAnnealingWithWarmup.on_epoch_begin (train_adipose_unet_v3.py:393-404)."""
    if epoch < warmup_epochs:
        return (max_lr / warmup_epochs) * (epoch + 1)
    progress = (epoch - warmup_epochs) / (total_epochs - warmup_epochs)
    return min_lr + 0.5 * (max_lr - min_lr) * (1 + math.cos(math.pi * progress))
