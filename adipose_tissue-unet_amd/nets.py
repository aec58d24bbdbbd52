"""U-Net presets as explicit, preallocated GPU schedules over the libadipose_hip kernels.

Two presets share the same kernels:

* ``adipose_v3`` — the reference network, AdiposeUNetV3.build_model
  (Segmentation/train_adipose_unet_v3.py:660-758; identical copies segmentation_inference.py:88-146,
  full_evaluation_enhanced.py:1163-1264): 1-channel input, base width 44, 3 poolings, dilated
  bottleneck (dilations 1..32 summed), nearest-upsample+conv decoder with skip concats, Dropout(0.3),
  2-class softmax main head (+ two sigmoid deep-supervision heads with bilinear resize).
* ``unet_bn`` — the north-star network of BASELINE.json configs 2/3/5 (no reference code):
  L levels, base 64, [conv3x3 -> BatchNorm -> ReLU] x 2 blocks, 2x2 max-pool, ConvTranspose 2x2/s2
  upsampling + skip concat, 1x1 conv + sigmoid head.

Nothing here runs torch compute: torch tensors are only HBM allocations; every op is a C-ABI call.
All activations for a fixed (batch, size) are allocated once (HBM is 288 GB; no allocator churn in
the step), so a whole step can be captured in a HIP graph.

Parameter layout: one flat f32 master buffer (+ same-layout grad / Adam buffers). A dense layer owns
``W`` packed [Npad][Kpad] (see include/adipose_hip.h) and ``b``; Keras HWIO kernels map onto it by
``keras_to_packed`` / ``packed_to_keras`` so `.weights.h5`-style name/slot I/O is 1:1.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np
import torch

from . import ops
from .ops import round_up


def r8(c):
    return round_up(c, 8)


# --------------------------------------------------------------------------------- parameters
class ParamStore:
    """Flat f32 parameter buffer with named views; grads/moments share the layout."""

    def __init__(self):
        self.entries = OrderedDict()
        self.total = 0
        self.flat = None
        self.grad = None

    def add(self, name, shape, init="zeros"):
        n = int(np.prod(shape))
        self.entries[name] = (self.total, tuple(shape), init)
        self.total += round_up(n, 64)  # 256-B aligned slices
        return name

    def allocate(self, device):
        self.flat = torch.zeros(self.total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=device)

    def view(self, name, buf=None):
        off, shape, _ = self.entries[name]
        b = self.flat if buf is None else buf
        return b[off:off + int(np.prod(shape))].view(shape)

    def gview(self, name):
        return self.view(name, self.grad)


class Dense:
    """A GEMM-lowered layer: 3x3 conv (any dilation, optional nearest-x2 input, optional concat) or
    ConvTranspose 2x2/s2. Keras names/shapes are kept for checkpoint interop."""

    def __init__(self, name, cin_parts, cout, *, k=3, dil=1, up=False, bias=True, bn=False, transpose=False,
                 relu=True, cpad=8, in_pad=None):
        """cpad: channel-stride granule of the output (and, unless in_pad says otherwise, the input)
        tensors; 64 puts every 64-deep K step inside one tap (the tap64 / halo kernels)."""
        self.name = name
        self.cin_parts = list(cin_parts)
        self.cin_s = [round_up(c, in_pad or cpad) for c in cin_parts]
        self.Cin_s = sum(self.cin_s)
        self.cout = cout
        self.cout_s = round_up(cout, cpad)
        self.k = 1 if transpose else k
        self.dil = dil
        self.up = up
        self.bias = bias
        self.bn = bn
        self.relu = relu
        self.transpose = transpose
        if transpose:
            self.taps = 1
            self.Nout = 4 * self.cout_s
        else:
            self.taps = k * k
            self.Nout = self.cout_s
        self.K = self.taps * self.Cin_s
        self.Kpad = round_up(self.K, 32)
        self.Npad = round_up(self.Nout, 64)
        # data-gradient launch: rows = forward input channels, K = taps * forward out channels
        self.dtaps = 4 if transpose else self.taps
        self.dK = self.dtaps * self.cout_s
        self.dKpad = round_up(self.dK, 32)
        # real channel counts of the forward / data-gradient launches (ops.conv_fwd real=: the pad weight columns and
        # rows are zeros, which the f32 tap kernel may skip)
        self.real_fwd = (cin_parts[0], cin_parts[1] if len(cin_parts) > 1 else 0, cout)
        self.real_dgrad = (cout, 0, cin_parts[0] if len(cin_parts) == 1 else 0)
        # (+64 rows for concat inputs so the decoder-only row slice of a split data-gradient stays
        #  a valid [Npad][Kpad] operand)
        self.dNpad = round_up(self.Cin_s, 64) + (64 if len(self.cin_parts) > 1 else 0)

    # -- parameter registration
    def register(self, ps: ParamStore):
        ps.add(self.name + "/W", (self.Npad, self.Kpad), init="glorot")
        if self.bias:
            ps.add(self.name + "/b", (self.cout_s,))
        if self.bn:
            ps.add(self.name + "/gamma", (self.cout_s,), init="ones")
            ps.add(self.name + "/beta", (self.cout_s,))

    def fan(self):
        cin = sum(self.cin_parts)
        if self.transpose:
            return cin * 4, self.cout * 4   # torch-style fan for ConvTranspose (in*k*k, out*k*k)
        return cin * self.taps, self.cout * self.taps

    def keras_shapes(self):
        cin = sum(self.cin_parts)
        if self.transpose:  # torch ConvTranspose2d layout (Cin, Cout, 2, 2)
            return (cin, self.cout, 2, 2), (self.cout,)
        return (self.k, self.k, cin, self.cout), (self.cout,)

    def _cmap(self):
        """logical input channel -> packed input channel index"""
        m = []
        base = 0
        for c, cs in zip(self.cin_parts, self.cin_s):
            m.extend(range(base, base + c))
            base += cs
        return np.asarray(m)

    def keras_to_packed(self, kernel):
        kernel = np.asarray(kernel, dtype=np.float32)
        Wp = np.zeros((self.Npad, self.Kpad), np.float32)
        cm = self._cmap()
        if self.transpose:
            cin, cout = kernel.shape[:2]
            for dy in range(2):
                for dx in range(2):
                    sub = dy * 2 + dx
                    # Wp[sub*cout_s + co][ci] = kernel[ci, co, dy, dx]
                    Wp[sub * self.cout_s: sub * self.cout_s + cout][:, cm] = kernel[:, :, dy, dx].T
            return Wp
        k = self.k
        for ky in range(k):
            for kx in range(k):
                t = ky * k + kx
                blk = kernel[ky, kx]  # (cin, cout)
                Wp[: self.cout, t * self.Cin_s + cm] = blk.T
        return Wp

    def packed_to_keras(self, Wp):
        Wp = np.asarray(Wp, dtype=np.float32)
        cm = self._cmap()
        kshape, _ = self.keras_shapes()
        out = np.zeros(kshape, np.float32)
        if self.transpose:
            for dy in range(2):
                for dx in range(2):
                    sub = dy * 2 + dx
                    out[:, :, dy, dx] = Wp[sub * self.cout_s: sub * self.cout_s + self.cout][:, cm].T
            return out
        k = self.k
        for ky in range(k):
            for kx in range(k):
                t = ky * k + kx
                out[ky, kx] = Wp[: self.cout, t * self.Cin_s + cm].T
        return out


class Head:
    """1x1 conv head: softmax over 2 classes keeping class 1, or a 1-channel sigmoid."""

    def __init__(self, name, cin, nout):
        self.name, self.cin, self.nout = name, cin, nout

    def register(self, ps):
        ps.add(self.name + "/W", (self.nout, self.cin), init="glorot")
        ps.add(self.name + "/b", (self.nout,))

    def fan(self):
        return self.cin, self.nout

    def keras_shapes(self):
        return (1, 1, self.cin, self.nout), (self.nout,)

    def keras_to_packed(self, kernel):
        return np.ascontiguousarray(np.asarray(kernel, np.float32)[0, 0].T)

    def packed_to_keras(self, Wp):
        return np.asarray(Wp, np.float32).T.reshape(1, 1, self.cin, self.nout)


# ------------------------------------------------------------------------------ base engine
class UNetEngine:
    """Common machinery: params, per-step weight packing, Keras-name weight I/O, buffers."""

    preset = None

    def __init__(self, batch, size, *, dtype="bf16", device="cuda", seed=865):
        self.B = batch
        self.S = size
        self.dt = torch.bfloat16 if dtype == "bf16" else torch.float32
        self.dtype_name = dtype
        self.device = torch.device(device)
        self.seed = seed
        self.ps = ParamStore()
        self.layers = OrderedDict()
        self.build_layers()
        for l in self.layers.values():
            l.register(self.ps)
        self.ps.allocate(self.device)
        self._packed = {}
        self._bufs = {}
        self.step_count = 0
        self.init_weights(seed)

    # -- to implement per preset
    def build_layers(self):
        raise NotImplementedError

    # -- weights
    def init_weights(self, seed):
        """Keras defaults: glorot_uniform kernels, zero biases (BN: gamma 1, beta 0)."""
        rng = np.random.default_rng(seed)
        for l in self.layers.values():
            fi, fo = l.fan()
            lim = math.sqrt(6.0 / (fi + fo))
            kshape, _ = l.keras_shapes()
            kern = rng.uniform(-lim, lim, size=kshape).astype(np.float32)
            arrs = [kern]
            for slot in self._slots(l.name)[1:]:
                arrs.append((np.ones if slot == "gamma" else np.zeros)(l.keras_shapes()[1], np.float32))
            self.set_layer_weights(l.name, arrs)

    def _slots(self, name):
        """Keras-style variable slots of a layer: kernel, [bias], [gamma, beta]."""
        slots = ["W"]
        if (name + "/b") in self.ps.entries:
            slots.append("b")
        if (name + "/gamma") in self.ps.entries:
            slots += ["gamma", "beta"]
        return slots

    def set_layer_weights(self, name, arrays):
        """Keras-style set: arrays = [kernel, bias] (conv/head), [kernel, gamma, beta] (conv+BN)."""
        l = self.layers[name]
        slots = self._slots(name)
        if len(arrays) != len(slots):
            raise ValueError(f"{name}: expected {len(slots)} arrays ({slots}), got {len(arrays)}")
        Wp = l.keras_to_packed(arrays[0])
        self.ps.view(name + "/W").copy_(torch.from_numpy(Wp))
        for slot, arr in zip(slots[1:], arrays[1:]):
            v = self.ps.view(f"{name}/{slot}")
            v.zero_()
            v[: len(arr)].copy_(torch.from_numpy(np.asarray(arr, np.float32)))

    def get_layer_weights(self, name, buf=None):
        l = self.layers[name]
        Wp = self.ps.view(name + "/W", buf).detach().cpu().numpy()
        out = [l.packed_to_keras(Wp)]
        n = l.cout if isinstance(l, Dense) else l.nout
        for slot in self._slots(name)[1:]:
            out.append(self.ps.view(f"{name}/{slot}", buf).detach().cpu().numpy()[:n].copy())
        return out

    def get_layer_grads(self, name):
        return self.get_layer_weights(name, self.ps.grad)

    def get_weights(self):
        return OrderedDict((n, self.get_layer_weights(n)) for n in self.layers)

    def set_weights(self, wd):
        for n, arrs in wd.items():
            if n in self.layers:
                self.set_layer_weights(n, arrs)

    def count_params(self):
        tot = 0
        for l in self.layers.values():
            ks, bs = l.keras_shapes()
            tot += int(np.prod(ks)) + (int(np.prod(bs)) if (l.name + "/b") in self.ps.entries else 0)
            if isinstance(l, Dense) and l.bn:
                tot += 2 * l.cout
        return tot

    # -- buffers
    def buf(self, key, shape, dtype=None):
        """Persistent HBM buffer, allocated once per (name, shape, dtype)."""
        dtype = dtype or self.dt
        k = (key, tuple(shape), dtype)
        t = self._bufs.get(k)
        if t is None:
            t = torch.zeros(shape, dtype=dtype, device=self.device)
            self._bufs[k] = t
        return t

    grad_hook = None  # called with a layer name once that layer's parameter gradients are final

    def _grad_ready(self, name):
        if self.grad_hook is not None:
            self.grad_hook(name)

    def acts(self, batch):
        """Activation set for a batch size (allocated once, reused every step)."""
        if not hasattr(self, "_acts"):
            self._acts = {}
        if batch not in self._acts:
            self._acts[batch] = self.alloc(batch)
        self.a = self._acts[batch]
        if hasattr(self, "_sts"):
            self.st = self._sts[batch]
        return self.a

    def zero(self, t):
        if t.dtype == torch.float32:
            ops.fill(t, 0.0)
        else:
            ops.fill(t.view(torch.float32) if t.numel() % 2 == 0 else t, 0.0)

    def pack_forward_weights(self):
        """Per step: master f32 -> compute-dtype forward layout for every dense layer. The forward layout
        of a layer is its master layout, so bf16 is ONE cast of the whole flat parameter buffer into a
        flat mirror (one launch instead of one per layer); the layers' weights are views into it."""
        if self.dt != torch.float32:
            mirror = self.buf("wf/flat", (self.ps.total,))
            ops.cast(self.ps.flat, mirror)
        for l in self.layers.values():
            if not isinstance(l, Dense):
                continue
            self._packed[l.name] = self.ps.view(l.name + "/W", None if self.dt == torch.float32 else mirror)

    def pack_dgrad_weights(self, names):
        """Flipped / transposed data-gradient weights of the named layers, batched into one launch
        (adp_pack_weights_batch: ConvT = 1 tap over 4*C outputs, conv = 9 flipped taps)."""
        jobs = []
        for n in names:
            l = self.layers[n]
            dst = self.buf("wd/" + n, (l.dNpad, l.dKpad))
            jobs.append((self.ps.view(n + "/W"), dst, 1 if l.transpose else l.taps, l.Cin_s,
                         l.Nout if l.transpose else l.cout_s))
            self._packed["d/" + n] = dst
        if jobs:
            ops.pack_weights_batch(jobs)

    def Wf(self, name):
        return self._packed[name]

    def Wd(self, name):
        return self._packed["d/" + name]

    def bias(self, name):
        key = name + "/b"
        return self.ps.view(key) if key in self.ps.entries else None

    # conv helpers -----------------------------------------------------------------------
    def conv(self, l, srcA, out, *, srcB=None, bnA=None, bnB=None, dropout=0.0, seed=0, accum=None,
             bn_stats=None, defer_fold=False, act_out=None):
        if l.transpose:
            return ops.conv_fwd(srcA, self.Wf(l.name), l.Nout, out=out, bias=self.bias(l.name), kh=1, kw=1,
                                pad=0, bnA=bnA, out_mode=1, shuffle_c=l.cout_s)
        return ops.conv_fwd(srcA, self.Wf(l.name), l.Nout, out=out, srcB=srcB, bnA=bnA, bnB=bnB,
                            bias=self.bias(l.name) if l.bias else None, up=l.up, kh=l.k, kw=l.k, dil=l.dil,
                            relu=l.relu and not l.bn, dropout_rate=dropout, dropout_seed=seed, accum=accum,
                            bn_stats=bn_stats, defer_fold=defer_fold, act_out=act_out, real=l.real_fwd)

    def wgrad(self, l, srcA, dZ, *, srcB=None, bnA=None, bnB=None, bias_grad=True, bn_apply=None):
        dW = self.ps.gview(l.name + "/W")
        dB = self.ps.gview(l.name + "/b") if bias_grad and (l.name + "/b") in self.ps.entries else None
        if l.transpose:
            ops.conv_wgrad(srcA, dZ, dW, l.Nout, dB=dB, bnA=bnA, kh=1, kw=1, pad=0, shuffle_c=l.cout_s)
        else:
            ops.conv_wgrad(srcA, dZ, dW, l.Nout, dB=dB, srcB=srcB, bnA=bnA, bnB=bnB, up=l.up, kh=l.k, kw=l.k,
                           dil=l.dil, bn_apply=bn_apply, real=l.real_fwd)
        self._grad_ready(l.name)

    def dgrad(self, l, dZ, out, *, Ho=None, Wo=None, addend=None, mask=None, mask_scale=1.0, split=False,
              out2=None, mask2=None, mask2_scale=1.0, skip_first=False, bn_reduce=None, bn_stats=None):
        """Data gradient of a dense layer: a forward-shaped launch over dZ with repacked weights.
        bn_reduce: fuse the BatchNorm-backward reduction of the layer `out` is the gradient of.
        bn_stats: per-channel sums (and sums of squares) of the stored gradient (split stores included)."""
        Wd = self.Wd(l.name)
        if l.transpose:
            # input coord = 2*o + (dy,dx): 4 taps, stride 2, over the ConvT output gradient
            return ops.conv_fwd(dZ, Wd, l.Cin_s, out=out, kh=2, kw=2, dil=1, pad=0, stride=2,
                                Ho=dZ.shape[1] // 2, Wo=dZ.shape[2] // 2, addend=addend, mask=mask,
                                mask_scale=mask_scale, bn_reduce=bn_reduce)
        # forward dilation d, 'same' padding: data gradient is the same gather with flipped taps
        if split and skip_first:
            # only the second (decoder) part of a concat input is needed: offset the weight rows
            Wsub = Wd[l.cin_s[0]:]
            return ops.conv_fwd(dZ, Wsub, l.cin_s[1], out=out2, kh=l.k, kw=l.k, dil=l.dil, mask=mask2,
                                mask_scale=mask2_scale, real=(l.cout, 0, l.cin_parts[1]))
        if split:
            return ops.conv_fwd(dZ, Wd, l.Cin_s, out=out, kh=l.k, kw=l.k, dil=l.dil, out_mode=2, out2=out2,
                                split_c=l.cin_s[0], addend=addend, mask=mask, mask_scale=mask_scale,
                                mask2=mask2, mask2_scale=mask2_scale, bn_stats=bn_stats, real=(l.cout, 0, 0))
        return ops.conv_fwd(dZ, Wd, l.Cin_s, out=out, kh=l.k, kw=l.k, dil=l.dil, addend=addend, mask=mask,
                            mask_scale=mask_scale, bn_reduce=bn_reduce, real=l.real_dgrad)


# --------------------------------------------------------------------------------- adipose_v3
class AdiposeV3Net(UNetEngine):
    """AdiposeUNetV3 (train_adipose_unet_v3.py:660-758) generalised in the tile size S."""

    preset = "adipose_v3"
    ENCODER = ("down1_conv1", "down1_conv2", "down2_conv1", "down2_conv2", "down3_conv1", "down3_conv2")

    def __init__(self, batch, size, *, dtype="bf16", device="cuda", seed=865, init_nb=44, dropout_rate=0.3,
                 deep_supervision=True, cpad=None):
        self.nb = init_nb
        self.dropout_rate = dropout_rate
        self.ds = deep_supervision
        # channel-stride granule per resolution level (int = all levels): a 64 granule stores 44/88/176/352
        # as 64/128/192/384 so those levels run on the tap64 / halo MFMA kernels (the pad channels are exact
        # zeros: zero weights and biases in, ReLU(0) = 0 out, zero gradients back); 8 keeps 48/88/176/352 on
        # the generic LDS-DMA kernels. f32 uses 32 (64/96/192/352): every 32-channel K step then lies in one
        # tap, which puts the forward and data-gradient launches on the LDS-DMA tap kernel's f32 form.
        if cpad is None:
            cpad = 64 if dtype == "bf16" else 32
        cpad = tuple(cpad) if isinstance(cpad, (tuple, list)) else (int(cpad),)
        self.cpad = cpad * 4 if len(cpad) == 1 else cpad   # one granule: every level
        assert size % 8 == 0, "adipose_v3 needs S % 8 == 0 (3 poolings)"
        super().__init__(batch, size, dtype=dtype, device=device, seed=seed)

    def build_layers(self):
        nb = self.nb
        L = self.layers

        def D(name, lin, cin_parts, lout, cout, **kw):
            in_pad = 8 if lin is None else self.cpad[lin]
            L[name] = Dense(name, cin_parts, cout, cpad=self.cpad[lout], in_pad=in_pad, **kw)

        D("down1_conv1", None, [1], 0, nb)
        D("down1_conv2", 0, [nb], 0, nb)
        D("down2_conv1", 0, [nb], 1, 2 * nb)
        D("down2_conv2", 1, [2 * nb], 1, 2 * nb)
        D("down3_conv1", 1, [2 * nb], 2, 4 * nb)
        D("down3_conv2", 2, [4 * nb], 2, 4 * nb)
        for i, d in enumerate((1, 2, 4, 8, 16, 32)):
            D(f"dilate{i + 1}", 2 if i == 0 else 3, [4 * nb if i == 0 else 8 * nb], 3, 8 * nb, dil=d)
        D("up3_conv1", 3, [8 * nb], 2, 4 * nb, up=True)
        D("up3_conv2", 2, [4 * nb, 4 * nb], 2, 4 * nb)
        D("up3_conv3", 2, [4 * nb], 2, 4 * nb)
        D("up2_conv1", 2, [4 * nb], 1, 2 * nb, up=True)
        D("up2_conv2", 1, [2 * nb, 2 * nb], 1, 2 * nb)
        D("up2_conv3", 1, [2 * nb], 1, 2 * nb)
        D("up1_conv1", 1, [2 * nb], 0, nb, up=True)
        D("up1_conv2", 0, [nb, nb], 0, nb)
        D("up1_conv3", 0, [nb], 0, nb)
        if self.ds:
            L["aux_out1"] = Head("aux_out1", 4 * nb, 1)
            L["aux_out2"] = Head("aux_out2", 2 * nb, 1)
        L["output_softmax"] = Head("output_softmax", nb, 2)

    # -------------------------------------------------------------------------- forward
    def alloc(self, B):
        S, nb = self.S, self.nb
        s = [S, S // 2, S // 4, S // 8]
        c = [round_up(k * nb, self.cpad[i]) for i, k in enumerate((1, 2, 4, 8))]
        a = {}
        a["x"] = self.buf("x", (B, S, S, 8))
        a["d1a"] = self.buf("d1a", (B, s[0], s[0], c[0]))
        a["d1"] = self.buf("d1", (B, s[0], s[0], c[0]))
        a["p1"] = self.buf("p1", (B, s[1], s[1], c[0]))
        a["d2a"] = self.buf("d2a", (B, s[1], s[1], c[1]))
        a["d2"] = self.buf("d2", (B, s[1], s[1], c[1]))
        a["p2"] = self.buf("p2", (B, s[2], s[2], c[1]))
        a["d3a"] = self.buf("d3a", (B, s[2], s[2], c[2]))
        a["d3"] = self.buf("d3", (B, s[2], s[2], c[2]))
        a["p3"] = self.buf("p3", (B, s[3], s[3], c[2]))
        for i in range(1, 7):
            a[f"dl{i}"] = self.buf(f"dl{i}", (B, s[3], s[3], c[3]))
        a["dsum"] = self.buf("dsum", (B, s[3], s[3], c[3]))   # f32 networks: the accumulator itself
        for lvl, (sz, cc) in zip((3, 2, 1), ((s[2], c[2]), (s[1], c[1]), (s[0], c[0]))):
            for j in ("a", "b", ""):
                a[f"u{lvl}{j}"] = self.buf(f"u{lvl}{j}", (B, sz, sz, cc))
        a["p_main"] = self.buf("p_main", (B, S, S), torch.float32)
        if self.ds:
            a["s_aux1"] = self.buf("s_aux1", (B, s[2], s[2]), torch.float32)
            a["s_aux2"] = self.buf("s_aux2", (B, s[1], s[1]), torch.float32)
            a["p_aux1"] = self.buf("p_aux1", (B, S, S), torch.float32)
            a["p_aux2"] = self.buf("p_aux2", (B, S, S), torch.float32)
        return a

    def forward(self, batch=None, *, train=False, seed=0, pack=True):
        """Run the network on acts(batch)['x'] (NHWC, prepped by ops.prep_input).
        Returns dict of f32 probability maps (views of persistent buffers)."""
        a = self.acts(batch or self.B)
        if pack:
            self.pack_forward_weights()
        L = self.layers
        r = self.dropout_rate if train else 0.0
        sd = (seed * 7919 + 17) & 0xFFFFFFFF
        self.conv(L["down1_conv1"], a["x"], a["d1a"])
        self.conv(L["down1_conv2"], a["d1a"], a["d1"])
        ops.maxpool2_fwd(a["d1"], a["p1"])
        self.conv(L["down2_conv1"], a["p1"], a["d2a"])
        self.conv(L["down2_conv2"], a["d2a"], a["d2"])
        ops.maxpool2_fwd(a["d2"], a["p2"])
        self.conv(L["down3_conv1"], a["p2"], a["d3a"])
        self.conv(L["down3_conv2"], a["d3a"], a["d3"])
        ops.maxpool2_fwd(a["d3"], a["p3"])
        # the Add of the six dilated outputs: f32 networks accumulate in the convs' epilogues; bf16 ones sum
        # the six stored maps in one pass (the same f32 sum of the same bf16 values, rounded once), which
        # keeps the dilated convs on the persistent kernel (no read-modify-write epilogue) and moves
        # 7 x 4 bytes per element less than accumulate + cast
        acc = a["dsum"] if self.dt == torch.float32 else None
        if acc is not None:
            self.zero(acc)
        self.conv(L["dilate1"], a["p3"], a["dl1"], dropout=r, seed=sd + 1, accum=acc)
        for i in range(2, 7):
            self.conv(L[f"dilate{i}"], a[f"dl{i - 1}"], a[f"dl{i}"], accum=acc)
        if acc is None:
            ops.sum_bf16([a[f"dl{i}"] for i in range(1, 7)], a["dsum"])
        self.conv(L["up3_conv1"], a["dsum"], a["u3a"])
        self.conv(L["up3_conv2"], a["d3"], a["u3b"], srcB=a["u3a"])
        self.conv(L["up3_conv3"], a["u3b"], a["u3"], dropout=r, seed=sd + 2)
        self.conv(L["up2_conv1"], a["u3"], a["u2a"])
        self.conv(L["up2_conv2"], a["d2"], a["u2b"], srcB=a["u2a"])
        self.conv(L["up2_conv3"], a["u2b"], a["u2"], dropout=r, seed=sd + 3)
        self.conv(L["up1_conv1"], a["u2"], a["u1a"])
        self.conv(L["up1_conv2"], a["d1"], a["u1b"], srcB=a["u1a"])
        self.conv(L["up1_conv3"], a["u1b"], a["u1"], dropout=r, seed=sd + 4)
        h = L["output_softmax"]
        ops.head_fwd(a["u1"], self.ps.view("output_softmax/W"), self.ps.view("output_softmax/b"), a["p_main"],
                     cin=h.cin, softmax2=True)
        out = {"main_out": a["p_main"]}
        if self.ds:
            for k, src, sb, pb in (("aux_out1", "u3", "s_aux1", "p_aux1"), ("aux_out2", "u2", "s_aux2", "p_aux2")):
                hh = L[k]
                ops.head_fwd(a[src], self.ps.view(k + "/W"), self.ps.view(k + "/b"), a[sb], cin=hh.cin,
                             softmax2=False)
                ops.resize_bilinear_fwd(a[sb], a[pb])
                out[k] = a[pb]
        self._train_fwd = train
        return out

    # ------------------------------------------------------------------------- backward
    def trainable(self, name):
        return not (self.frozen_encoder and name in self.ENCODER)

    frozen_encoder = False

    def backward(self, grads_out):
        """The backward pass; its deterministic weight-gradient reductions are deferred (ops.wgrad_defer) and launched
        together at its end (one launch instead of one per layer); every gradient is final when it returns."""
        ops.wgrad_defer(True)
        self._deferring = True
        try:
            return self._backward(grads_out)
        finally:
            self._deferring = False
            ops.wgrad_flush()

    def _backward(self, grads_out):
        """grads_out: {'main_out': dL/dp (B,S,S) f32, 'aux_out1': ..., 'aux_out2': ...}.
        Accumulates parameter gradients into self.ps.grad (caller zeroes)."""
        a, L = self.a, self.layers
        r = self.dropout_rate if self._train_fwd else 0.0
        keep = 1.0 / (1.0 - r) if r > 0 else 1.0
        full = not self.frozen_encoder
        names = [n for n, l in L.items() if isinstance(l, Dense)]
        self.pack_dgrad_weights([n for n in names if n != "down1_conv1" and (full or n not in self.ENCODER)
                                 and (full or n != "dilate1")])
        g = {}

        def gb(key, like, dtype=None):
            t = self.buf("g/" + key, tuple(like.shape), dtype or like.dtype)
            return t

        # heads
        h = L["output_softmax"]
        g["u1"] = gb("u1", a["u1"])
        ops.head_bwd(a["u1"], self.ps.view("output_softmax/W"), a["p_main"], grads_out["main_out"],
                     self.ps.gview("output_softmax/W"), self.ps.gview("output_softmax/b"), cin=h.cin, softmax2=True,
                     dx=g["u1"], mask=a["u1"], mask_scale=keep)
        self._grad_ready("output_softmax")
        aux_dx = {}
        if self.ds:
            for k, src, sb, pb in (("aux_out1", "u3", "s_aux1", "p_aux1"), ("aux_out2", "u2", "s_aux2", "p_aux2")):
                hh = L[k]
                ds = self.buf("g/" + sb, tuple(a[sb].shape), torch.float32)
                ops.resize_bilinear_bwd(grads_out[k], ds)
                dx = gb("aux/" + src, a[src])
                ops.head_bwd(a[src], self.ps.view(k + "/W"), a[sb], ds, self.ps.gview(k + "/W"),
                             self.ps.gview(k + "/b"), cin=hh.cin, softmax2=False, dx=dx)
                self._grad_ready(k)
                aux_dx[src] = dx
        # decoder level 1 (full resolution)
        self._dec_level(1, g, "u1", "d1", aux_dx.get("u2"), keep, full)
        self._dec_level(2, g, "u2", "d2", aux_dx.get("u3"), keep, full)
        self._dec_level(3, g, "u3", "d3", None, keep, full)
        # bottleneck: g['dsum'] = dL/d(sum) (no activation on the Add)
        dsum = g["dsum"]
        dz = gb("dz6", a["dl6"])
        ops.add_mask(dsum, dz, mask=a["dl6"])
        for i in range(6, 1, -1):
            l = L[f"dilate{i}"]
            self.wgrad(l, a[f"dl{i - 1}"], dz)
            nz = gb(f"dz{i - 1}", a[f"dl{i - 1}"])
            self.dgrad(l, dz, nz, addend=dsum, mask=a[f"dl{i - 1}"], mask_scale=keep if i == 2 else 1.0)
            dz = nz
        self.wgrad(L["dilate1"], a["p3"], dz)
        if not full:
            return
        gp3 = gb("p3", a["p3"])
        self.dgrad(L["dilate1"], dz, gp3)
        # encoder: pool backward merges the concat-skip gradient and applies the ReLU mask
        for lvl, pin in ((3, "p2"), (2, "p1"), (1, "x")):
            dd = gb(f"d{lvl}", a[f"d{lvl}"])
            ops.maxpool2_bwd(a[f"d{lvl}"], g[f"p{lvl}"] if lvl < 3 else gp3, dd, addend=g[f"skip{lvl}"],
                             mask=a[f"d{lvl}"])
            l2, l1 = L[f"down{lvl}_conv2"], L[f"down{lvl}_conv1"]
            self.wgrad(l2, a[f"d{lvl}a"], dd)
            dz1 = gb(f"d{lvl}a", a[f"d{lvl}a"])
            self.dgrad(l2, dd, dz1, mask=a[f"d{lvl}a"])
            self.wgrad(l1, a[pin], dz1)
            if lvl > 1:
                gp = gb(f"p{lvl - 1}", a[f"p{lvl - 1}"])
                self.dgrad(l1, dz1, gp)
                g[f"p{lvl - 1}"] = gp

    def _dec_level(self, lvl, g, uname, dname, aux_add, keep, full):
        """Backward through up{lvl}_conv3 / conv2 (concat) / conv1 (upsample)."""
        a, L = self.a, self.layers
        c3, c2, c1 = L[f"up{lvl}_conv3"], L[f"up{lvl}_conv2"], L[f"up{lvl}_conv1"]
        if lvl == 1:
            dz3 = g["u1"]          # head backward already applied the u1 ReLU/dropout mask
        else:
            dz3 = g[uname]
        self.wgrad(c3, a[f"u{lvl}b"], dz3)
        dz2 = self.buf(f"g/u{lvl}b", tuple(a[f"u{lvl}b"].shape))
        self.dgrad(c3, dz3, dz2, mask=a[f"u{lvl}b"])
        self.wgrad(c2, a[dname], dz2, srcB=a[f"u{lvl}a"])
        dz1 = self.buf(f"g/u{lvl}a", tuple(a[f"u{lvl}a"].shape))
        if full:
            skip = self.buf(f"g/skip{lvl}", tuple(a[dname].shape))
            self.dgrad(c2, dz2, skip, split=True, out2=dz1, mask2=a[f"u{lvl}a"])
            g[f"skip{lvl}"] = skip
        else:
            self.dgrad(c2, dz2, None, split=True, skip_first=True, out2=dz1, mask2=a[f"u{lvl}a"])
        # conv1 reads the nearest-upsampled source
        src = {3: "dsum", 2: "u3", 1: "u2"}[lvl]
        self.wgrad(c1, a[src], dz1)
        Sup = a[f"u{lvl}a"].shape[1]
        gup = self.buf(f"g/up{lvl}", (a["x"].shape[0], Sup, Sup, a[src].shape[3]))
        self.dgrad(c1, dz1, gup)
        dsrc = self.buf(f"g/{src}", tuple(a[src].shape))
        if lvl == 3:
            ops.upsample2_bwd(gup, dsrc)
            g["dsum"] = dsrc
        else:
            ops.upsample2_bwd(gup, dsrc, addend=aux_add, mask=a[src], mask_scale=keep)
            g[src] = dsrc


# ------------------------------------------------------------------------------------ unet_bn
class UNetBN(UNetEngine):
    """North-star U-Net (BASELINE.json configs 2/3/5): L levels, base 64, Conv-BN-ReLU x2 blocks,
    MaxPool 2x2, ConvTranspose 2x2/s2 + concat, 1x1 sigmoid head. BatchNorm uses batch statistics
    in training (momentum 0.1, eps 1e-5, PyTorch semantics) and running statistics in eval."""

    preset = "unet_bn"
    # dec0_conv2's BatchNorm+ReLU applied on load by the head (forward) and its BatchNorm-backward
    # reduction fused into the head backward; False: materialised activation + adp_bn_bwd_reduce
    fuse_head_bn = True
    # the training conv leaves its BatchNorm sums in the replica scratch and the finalize folds them (one
    # launch); False: the conv's own fold launch, then the finalize
    fuse_bn_fold = True
    fuse_eval_bn = True   # eval forwards: BatchNorm + ReLU folded into the conv epilogues (False: z + apply pass)
    # with fuse_head_bn: the head backward stores no dA for dec0_conv2; that layer's BatchNorm-backward
    # apply recomputes it from p, dL/dp and the head weights (adp_bn_bwd_apply_head, bit-identical dz)
    head_recompute_dA = True
    # each layer's BatchNorm-backward apply (dz from dA, z) handed to its weight-gradient launch
    # (adp_conv_wgrad_bn: computed inside the halo weight-gradient kernel on levels 0-1, which also stores
    # dz for the data gradient); False: adp_bn_bwd_apply, then the weight gradient re-reads dz
    fuse_bn_wgrad = True
    # training forward, 64-channel levels: conv2 reads conv1's pre-BatchNorm output and applies
    # relu(bn(.)) on load, storing the activation for the backward itself (adp_conv_io.act_outA: the persistent halo
    # forward's EPI 6) instead of an adp_bn_apply pass between the convs; the same bits
    fuse_bn_load = True
    # the encoder pool backward recomputes its argmax from z (relu(z*scale+shift), rounded as stored) instead of
    # reading the stored activation
    pool_argmax_from_z = True

    def __init__(self, batch, size, *, levels=5, base=64, in_ch=3, dtype="bf16", device="cuda", seed=865,
                 bn_eps=1e-5, bn_momentum=0.1):
        self.levels = levels
        self.base = base
        self.in_ch = in_ch
        self.bn_eps = bn_eps
        self.bn_momentum = bn_momentum
        assert size % (1 << (levels - 1)) == 0
        super().__init__(batch, size, dtype=dtype, device=device, seed=seed)
        self.running = {}
        for n, l in self.layers.items():
            if isinstance(l, Dense) and l.bn:
                self.running[n] = (torch.zeros(l.cout_s, device=self.device),
                                   torch.ones(l.cout_s, device=self.device))

    def ch(self, i):
        return self.base << i

    def build_layers(self):
        L = self.layers
        Lv = self.levels
        cin = self.in_ch
        for i in range(Lv):
            c = self.ch(i)
            L[f"enc{i}_conv1"] = Dense(f"enc{i}_conv1", [cin], c, bias=False, bn=True)
            L[f"enc{i}_conv2"] = Dense(f"enc{i}_conv2", [c], c, bias=False, bn=True)
            cin = c
        for i in range(Lv - 2, -1, -1):
            c = self.ch(i)
            L[f"dec{i}_up"] = Dense(f"dec{i}_up", [self.ch(i + 1)], c, transpose=True, relu=False)
            L[f"dec{i}_conv1"] = Dense(f"dec{i}_conv1", [c, c], c, bias=False, bn=True)
            L[f"dec{i}_conv2"] = Dense(f"dec{i}_conv2", [c], c, bias=False, bn=True)
        L["head"] = Head("head", self.ch(0), 1)

    def alloc(self, B):
        S = self.S
        a = {"x": self.buf("x", (B, S, S, 8))}
        st = {}
        for i in range(self.levels):
            s, c = S >> i, self.ch(i)
            for key in ([f"z{i}_1", f"z{i}_2"] + ([f"y{i}_1", f"y{i}_2"] if i < self.levels - 1 else [])):
                a[key] = self.buf(key, (B, s, s, c))          # conv output (pre-BN), kept for BN backward
                a["a" + key] = self.buf("a" + key, (B, s, s, c))  # relu(bn(z)), read by every consumer
            if i < self.levels - 1:
                a[f"pool{i}"] = self.buf(f"pool{i}", (B, s // 2, s // 2, c))
                a[f"t{i}"] = self.buf(f"t{i}", (B, s, s, c))
        a["p"] = self.buf("p", (B, S, S), torch.float32)
        # the per-step f32 accumulators live in one arena of two parts, each zeroed by ONE fill (instead of a
        # fill launch per BatchNorm layer / per ConvTranspose bias-gradient sum): the forward part, per BN
        # layer (6, C) = sum, sq, scale, shift, mean, invstd, is filled at the start of every training
        # forward; the backward part, per decoder level (2, Cin_s) channel sums of the concat data gradient,
        # at the start of every backward (so a backward never depends on what the forward zeroed)
        bn = [(n, l.cout_s) for n, l in self.layers.items() if isinstance(l, Dense) and l.bn]
        ts = [(i, self.layers[f"dec{i}_conv1"].Cin_s) for i in range(self.levels - 1)]
        nbn = sum(6 * c for _, c in bn)
        arena = self.buf("stat_arena", (nbn + sum(2 * c for _, c in ts),), torch.float32)
        off = 0
        for n, c in bn:
            st[n] = arena[off:off + 6 * c].view(6, c)
            off += 6 * c
        self.dtsum = {}
        for i, c in ts:
            self.dtsum[i] = arena[off:off + 2 * c].view(2, c)
            off += 2 * c
        self._stat_fwd = arena[:nbn]
        self._stat_bwd = arena[nbn:]
        self.st = st  # batch-independent shapes: shared by every activation set
        return a

    def bnvec(self, name):
        s = self.st[name]
        return (s[2], s[3])

    def _bn_conv(self, name, srcA, out, act, *, srcB=None, train=True, pool=None, bnA=None, act_in=None):
        """conv -> BN statistics (epilogue) -> scale/shift -> act = relu(bn(out)) materialised (and, with
        pool, its 2x2 max-pool in the same pass; act=None: not materialised, the consumer applies it on
        load). bnA / act_in (training): srcA is the previous layer's pre-BatchNorm output, applied on load and
        stored to act_in by this conv (fuse_bn_load)."""
        l = self.layers[name]
        s = self.st[name]
        if train:
            # s[:2] was zeroed with the forward part of the stat arena at the start of this training forward
            # the conv leaves its statistics in the accumulator replicas; the finalize folds them (one launch)
            fold = self.fuse_bn_fold
            self.conv(l, srcA, out, srcB=srcB, bn_stats=(s[0], s[1]), defer_fold=fold, bnA=bnA, act_out=act_in)
            count = out.shape[0] * out.shape[1] * out.shape[2]
            rm, rv = self.running[name]
            ops.bn_finalize(count, s[0], s[1], self.ps.view(name + "/gamma"), self.ps.view(name + "/beta"),
                            self.bn_eps, self.bn_momentum, s[2], s[3], s[4], s[5], rm, rv, fold=fold)
        else:
            rm, rv = self.running[name]
            # eval: count < 0 -> (sum, sqsum) are read as (running mean, running var)
            ops.bn_finalize(-1.0, rm, rv, self.ps.view(name + "/gamma"), self.ps.view(name + "/beta"),
                            self.bn_eps, 0.0, s[2], s[3], s[4], s[5], None, None)
            if self.fuse_eval_bn and act is not None:
                self._conv_eval_folded(l, srcA, act, srcB=srcB)
                if pool is not None:
                    ops.maxpool2_fwd(act, pool)
                return
            self.conv(l, srcA, out, srcB=srcB)
        if pool is not None:
            ops.bn_apply_maxpool2(out, s[2], s[3], act, pool)
        elif act is not None:
            ops.bn_apply(out, s[2], s[3], act)

    def _conv_eval_folded(self, l, srcA, act, *, srcB=None):
        """Eval conv with its BatchNorm folded in: forward weights scaled per output channel by the BN scale
        (adp_scale_rows, in the compute dtype), BN shift as the bias, ReLU in the epilogue: act = relu(bn(z))
        in one launch, no z and no apply pass (the BN vectors of the layer are final: bn_finalize ran)."""
        s = self.st[l.name]
        Wm = self.ps.view(l.name + "/W")
        We = self.buf("we/" + l.name, tuple(Wm.shape), self.dt)
        ops.scale_rows(Wm, s[2], We)
        ops.conv_fwd(srcA, We, l.Nout, out=act, srcB=srcB, bias=s[3], up=l.up, kh=l.k, kw=l.k, dil=l.dil,
                     relu=True)

    def forward(self, batch=None, *, train=False, seed=0, pack=True):
        a = self.acts(batch or self.B)
        if pack:
            self.pack_forward_weights()
        if train:
            ops.fill(self._stat_fwd, 0.0)
        Lv = self.levels
        src = a["x"]
        def bnl(i):   # conv2 of level i applies conv1's BatchNorm-ReLU on load (the persistent halo forward's shapes)
            return train and self.fuse_bn_load and self.dt == torch.bfloat16 and self.ch(i) == 64
        for i in range(Lv):
            if bnl(i):
                self._bn_conv(f"enc{i}_conv1", src, a[f"z{i}_1"], None, train=train)
                self._bn_conv(f"enc{i}_conv2", a[f"z{i}_1"], a[f"z{i}_2"], a[f"az{i}_2"], train=train,
                              pool=a[f"pool{i}"] if i < Lv - 1 else None, bnA=self.bnvec(f"enc{i}_conv1"),
                              act_in=a[f"az{i}_1"])
            else:
                self._bn_conv(f"enc{i}_conv1", src, a[f"z{i}_1"], a[f"az{i}_1"], train=train)
                self._bn_conv(f"enc{i}_conv2", a[f"az{i}_1"], a[f"z{i}_2"], a[f"az{i}_2"], train=train,
                              pool=a[f"pool{i}"] if i < Lv - 1 else None)
            if i < Lv - 1:
                src = a[f"pool{i}"]
        prev = a[f"az{Lv - 1}_2"]
        for i in range(Lv - 2, -1, -1):
            self.conv(self.layers[f"dec{i}_up"], prev, a[f"t{i}"])
            f = bnl(i)
            self._bn_conv(f"dec{i}_conv1", a[f"az{i}_2"], a[f"y{i}_1"], None if f else a[f"ay{i}_1"],
                          srcB=a[f"t{i}"], train=train)
            # level 0: relu(bn(y0_2)) is only read by the head, which applies it on load (same rounding); eval
            # with the BatchNorm folded into the convs materialises it in the conv epilogue instead
            head_bn = self.fuse_head_bn and (train or not self.fuse_eval_bn)
            fuse = i == 0 and head_bn
            self._bn_conv(f"dec{i}_conv2", a[f"y{i}_1"] if f else a[f"ay{i}_1"], a[f"y{i}_2"],
                          None if fuse else a[f"ay{i}_2"], train=train,
                          bnA=self.bnvec(f"dec{i}_conv1") if f else None, act_in=a[f"ay{i}_1"] if f else None)
            prev = a[f"ay{i}_2"]
        if self.fuse_head_bn and (train or not self.fuse_eval_bn):
            ops.head_fwd(a["y0_2"], self.ps.view("head/W"), self.ps.view("head/b"), a["p"], cin=self.ch(0),
                         softmax2=False, bn=self.bnvec("dec0_conv2"))
        else:
            ops.head_fwd(prev, self.ps.view("head/W"), self.ps.view("head/b"), a["p"], cin=self.ch(0),
                         softmax2=False)
        self._train_fwd = train
        return {"main_out": a["p"]}

    # ------------------------------------------------------------------ fp8 inference (configs[4])
    fp8_level0 = True   # forward_fp8: level 0 in fp8 too (the 64-channel fp8 halo kernel; False: bf16 as in round 3)

    def _fp8_acts(self, B):
        """fp8 e4m3 twins of the activations the fp8 convs read: every level >= 1 (channel strides >= 128) and,
        with fp8_level0, level 0 (64 channels: enc0_conv1's output, pool0, the decoder's concat halves and
        dec0_conv1's output; dec0_conv2's output stays bf16 for the head)."""
        a = self.acts(B)
        q = {}
        if self.fp8_level0 and self.levels > 1:
            for k in ("az0_1", "az0_2", "pool0", "t0", "ay0_1"):
                q[k] = self.buf("q/" + k, tuple(a[k].shape), ops.FP8_DTYPE)
        for i in range(1, self.levels):
            keys = [f"az{i}_1", f"az{i}_2"]
            if i < self.levels - 1:
                keys += [f"ay{i}_1", f"ay{i}_2", f"t{i}", f"pool{i}"]
            for k in keys:
                q[k] = self.buf("q/" + k, tuple(a[k].shape), ops.FP8_DTYPE)
        return q

    def pack_fp8_weights(self):
        """fp8 forward weights + per-output-channel scales for every layer whose input channel strides are
        multiples of 128 (one 128-channel K step per tap) and every 3x3 layer over 64-channel sources (the fp8
        halo kernel: tap pairs, or the two halves of a concat, per 128-deep K step)."""
        self._packed8 = {}
        for n, l in self.layers.items():
            wide = all(c % 128 == 0 for c in l.cin_s) and l.K % 128 == 0 if isinstance(l, Dense) else False
            c64 = isinstance(l, Dense) and not l.transpose and l.k == 3 and all(c == 64 for c in l.cin_s)
            if wide or c64:
                dst = self.buf("w8/" + n, (l.Npad, l.Kpad), ops.FP8_DTYPE)
                sc = self.buf("w8s/" + n, (l.Npad,), torch.float32)
                ops.pack_weights_fp8(self.ps.view(n + "/W"), dst, sc)
                self._packed8[n] = (dst, sc)

    def _conv_any(self, l, srcA, out, *, srcB=None):
        """Eval conv: fp8 kernel when the operands are fp8, else the bf16 path (no BN statistics)."""
        if srcA.dtype != ops.FP8_DTYPE:
            return self.conv(l, srcA, out, srcB=srcB)
        W8, ws = self._packed8[l.name]
        if l.transpose:
            return ops.conv_fwd(srcA, W8, l.Nout, out=out, bias=self.bias(l.name), kh=1, kw=1, pad=0, out_mode=1,
                                shuffle_c=l.cout_s, w_scale=ws)
        return ops.conv_fwd(srcA, W8, l.Nout, out=out, srcB=srcB, bias=self.bias(l.name) if l.bias else None,
                            kh=l.k, kw=l.k, dil=l.dil, relu=l.relu and not l.bn, w_scale=ws)

    def _bn_conv_eval(self, name, srcA, z, act, *, srcB=None):
        l = self.layers[name]
        s = self.st[name]
        rm, rv = self.running[name]
        ops.bn_finalize(-1.0, rm, rv, self.ps.view(name + "/gamma"), self.ps.view(name + "/beta"),
                        self.bn_eps, 0.0, s[2], s[3], s[4], s[5], None, None)
        if srcA.dtype != ops.FP8_DTYPE and self.fuse_eval_bn and (act.dtype != ops.FP8_DTYPE or l.Cin_s == 8):
            # (bf16 operands; an fp8 act only from the input layer, whose kernel stores fp8 itself)
            self._conv_eval_folded(l, srcA, act, srcB=srcB)
            return
        if srcA.dtype == ops.FP8_DTYPE and self.fuse_eval_bn:
            # eval BatchNorm folded into the fp8 conv: dequantisation scale x BN scale, BN shift as the bias,
            # ReLU in the epilogue, the next conv's fp8 (or bf16) operand stored directly (no z, no apply pass)
            W8, ws = self._packed8[name]
            wsb = self.buf("w8sb/" + name, tuple(ws.shape), torch.float32)
            ops.vec_mul(ws[:l.Nout], s[2], wsb)
            ops.conv_fwd(srcA, W8, l.Nout, out=act, srcB=srcB, bias=s[3], kh=l.k, kw=l.k, dil=l.dil, relu=True,
                         w_scale=wsb)
            return
        self._conv_any(l, srcA, z, srcB=srcB)
        if act.dtype == ops.FP8_DTYPE:
            ops.bn_apply_fp8(z, s[2], s[3], act)
        else:
            ops.bn_apply(z, s[2], s[3], act)

    def forward_fp8(self, batch=None, *, pack=True):
        """Eval forward with fp8 e4m3 activations and weights on every conv whose inputs have >= 128
        channels (levels >= 1: ~78 % of the forward FLOPs); the input conv, level 0 and the head stay bf16.
        Conv outputs (pre-BN) are bf16, BatchNorm-ReLU writes the fp8 operand of the next conv."""
        if self.dt != torch.bfloat16:
            raise ops.AdpError("forward_fp8 needs a bf16 network (its level-0 path)")
        B = batch or self.B
        a = self.acts(B)
        q = self._fp8_acts(B)
        if pack:
            self.pack_forward_weights()
            self.pack_fp8_weights()

        def act(key):
            return q.get(key, a[key])
        Lv = self.levels
        src = a["x"]
        for i in range(Lv):
            self._bn_conv_eval(f"enc{i}_conv1", src, a[f"z{i}_1"], act(f"az{i}_1"))
            self._bn_conv_eval(f"enc{i}_conv2", act(f"az{i}_1"), a[f"z{i}_2"], act(f"az{i}_2"))
            if i < Lv - 1:
                ops.maxpool2_fwd(act(f"az{i}_2"), act(f"pool{i}"))
                src = act(f"pool{i}")
        prev = act(f"az{Lv - 1}_2")
        for i in range(Lv - 2, -1, -1):
            self._conv_any(self.layers[f"dec{i}_up"], prev, act(f"t{i}"))
            self._bn_conv_eval(f"dec{i}_conv1", act(f"az{i}_2"), a[f"y{i}_1"], act(f"ay{i}_1"), srcB=act(f"t{i}"))
            self._bn_conv_eval(f"dec{i}_conv2", act(f"ay{i}_1"), a[f"y{i}_2"], act(f"ay{i}_2"))
            prev = act(f"ay{i}_2")
        ops.head_fwd(prev, self.ps.view("head/W"), self.ps.view("head/b"), a["p"], cin=self.ch(0), softmax2=False)
        self._train_fwd = False
        return {"main_out": a["p"]}

    def _bn_red(self, name, z):
        """bn_reduce argument for a dgrad launch whose output is the gradient of relu(bn_name(z))."""
        s = self.st[name]
        return (z, s[2], s[3], s[4], s[5], self.ps.gview(name + "/gamma"), self.ps.gview(name + "/beta"))

    def _bn_bwd_wgrad(self, name, dA, z, dz, l, srcA, srcB=None):
        """_bn_bwd(reduced=True) of layer `name` followed by the weight gradient of conv l over its dz."""
        cin = srcA.shape[-1] + (srcB.shape[-1] if srcB is not None else 0)
        if getattr(self, "_side", None) is not None and dz is not None and cin > 64:
            # (wider than one 64-channel chunk: the library would run the apply and the plain kernel anyway)
            self._bn_bwd(name, dA, z, dz, reduced=True)
            self._side_wgrad(l, srcA, dz, srcB=srcB)
            return
        if not self.fuse_bn_wgrad:
            self._bn_bwd(name, dA, z, dz, reduced=True)
            self.wgrad(l, srcA, dz, srcB=srcB)
            return
        s = self.st[name]
        count = z.shape[0] * z.shape[1] * z.shape[2]
        self.wgrad(l, srcA, dz, srcB=srcB,
                   bn_apply=(dA, z, s[2], s[3], s[4], s[5], self.ps.view(name + "/gamma"),
                             self.ps.gview(name + "/gamma"), self.ps.gview(name + "/beta"), count))

    def _bn_bwd(self, name, dA, z, dz, reduced=False):
        """dA: gradient wrt relu(bn(z)) -> dz, and gamma/beta grads (already summed by the producer of
        dA when reduced=True)."""
        s = self.st[name]
        dg, db = self.ps.gview(name + "/gamma"), self.ps.gview(name + "/beta")
        if not reduced:
            ops.bn_bwd_reduce(dA, z, s[2], s[3], s[4], s[5], dg, db)
        count = z.shape[0] * z.shape[1] * z.shape[2]
        ops.bn_bwd_apply(dA, z, s[2], s[3], s[4], s[5], self.ps.view(name + "/gamma"), dg, db, count, dz)

    # wgrad_side: the weight gradients that nothing on the backward's critical path waits for (every one but the
    # BatchNorm-fused forms, which produce the dz their data gradient reads) run on a second stream, event-ordered
    # after the dz they read, so that their tails, slab writes and launch gaps overlap the data-gradient chain.
    # Single-process only (the bucketed all-reduce orders on the issuing stream): with a grad_hook it stays off.
    # Measured -0.5..-0.6 % per step, the same bits (profiles/r05p_side_ab.log, r05q_side_ab.log). Off by default:
    # with two streams the kernels overlap, and every per-kernel duration (rocprofv3's, and the HIP-event timing the
    # bench's roofline divides by) then includes the time shared with the other stream (the halo weight gradient
    # reads 462 instead of 282 us), so no kernel's roofline fraction can be measured in the step.
    wgrad_side = False

    def backward(self, grads_out):
        """The backward pass; its deterministic weight-gradient reductions are deferred (ops.wgrad_defer) and launched
        together at its end (one launch instead of one per layer); every gradient is final when it returns."""
        side = None
        if self.wgrad_side and self.grad_hook is None:
            if getattr(self, "_side_stream", None) is None:
                self._side_stream = torch.cuda.Stream(device=self.device)
            side = self._side_stream
        self._side = side
        ops.wgrad_defer(True)
        if side is not None:
            with torch.cuda.stream(side):
                ops.wgrad_defer(True)
        self._deferring = True
        try:
            return self._backward(grads_out)
        finally:
            self._deferring = False
            ops.wgrad_flush()
            if side is not None:
                with torch.cuda.stream(side):
                    ops.wgrad_flush()
                torch.cuda.current_stream().wait_stream(side)
            self._side = None

    def _side_wgrad(self, l, srcA, dZ, **kw):
        """self.wgrad on the side stream (wgrad_side), ordered after everything issued so far on this one."""
        side = getattr(self, "_side", None)
        if side is None:
            return self.wgrad(l, srcA, dZ, **kw)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self.wgrad(l, srcA, dZ, **kw)

    def _backward(self, grads_out):
        a, L = self.a, self.layers
        Lv = self.levels
        self.pack_dgrad_weights([n for n, l in L.items() if isinstance(l, Dense) and n != "enc0_conv1"])

        def gb(key, like):
            return self.buf("g/" + key, tuple(like.shape), like.dtype)

        # head: dA = dL/d(relu(bn(y0_2)))
        # (dec0_conv2's BatchNorm-backward reduction over dA fused into the head backward)
        recompute = self.fuse_head_bn and self.head_recompute_dA
        dA = None if recompute else gb("y0_2", a["y0_2"])
        s0 = self.st["dec0_conv2"]
        if not self.fuse_head_bn:
            ops.head_bwd(a["ay0_2"], self.ps.view("head/W"), a["p"], grads_out["main_out"],
                         self.ps.gview("head/W"), self.ps.gview("head/b"), cin=self.ch(0), softmax2=False, dx=dA)
            ops.bn_bwd_reduce(dA, a["y0_2"], s0[2], s0[3], s0[4], s0[5], self.ps.gview("dec0_conv2/gamma"),
                              self.ps.gview("dec0_conv2/beta"))
        else:
            ops.head_bwd(a["y0_2"], self.ps.view("head/W"), a["p"], grads_out["main_out"], self.ps.gview("head/W"),
                         self.ps.gview("head/b"), cin=self.ch(0), softmax2=False, dx=dA,
                         bn=self.bnvec("dec0_conv2"), bn_reduce=(s0[4], s0[5], self.ps.gview("dec0_conv2/gamma"),
                                                                 self.ps.gview("dec0_conv2/beta")))
        self._grad_ready("head")
        ops.fill(self._stat_bwd, 0.0)
        skip_grad = {}
        cur_dA = dA
        bott_dA = None
        # decoder, from level 0 down to the bottleneck
        for i in range(0, Lv - 1):
            dz = gb(f"dz_y{i}_2", a[f"y{i}_2"])
            # level 0's dA comes from the head, deeper levels' from the ConvT dgrad (reduction fused in both)
            if cur_dA is None:   # level 0, head_recompute_dA
                s2 = self.st["dec0_conv2"]
                y = a["y0_2"]
                ops.bn_bwd_apply_head(self.ps.view("head/W"), a["p"], grads_out["main_out"], y, s2[2], s2[3], s2[4],
                                      s2[5], self.ps.view("dec0_conv2/gamma"), self.ps.gview("dec0_conv2/gamma"),
                                      self.ps.gview("dec0_conv2/beta"), y.shape[0] * y.shape[1] * y.shape[2], dz,
                                      cin=self.ch(0))
            l2 = L[f"dec{i}_conv2"]
            if cur_dA is None:
                self._side_wgrad(l2, a[f"ay{i}_1"], dz)
            else:
                self._bn_bwd_wgrad(f"dec{i}_conv2", cur_dA, a[f"y{i}_2"], dz, l2, a[f"ay{i}_1"])
            dA1 = gb(f"dA_y{i}_1", a[f"y{i}_1"])
            self.dgrad(l2, dz, dA1, bn_reduce=self._bn_red(f"dec{i}_conv1", a[f"y{i}_1"]))
            dz1 = gb(f"dz_y{i}_1", a[f"y{i}_1"])
            l1 = L[f"dec{i}_conv1"]
            self._bn_bwd_wgrad(f"dec{i}_conv1", dA1, a[f"y{i}_1"], dz1, l1, a[f"az{i}_2"], srcB=a[f"t{i}"])
            sk = gb(f"skip{i}", a[f"z{i}_2"])
            dt = gb(f"dt{i}", a[f"t{i}"])
            # the ConvTranspose bias gradient (sum of dt over pixels) comes out of this launch's epilogue
            # channel sums (channels >= split_c are dt) instead of a separate pass over dt
            lu = L[f"dec{i}_up"]
            tsum = self.dtsum[i]   # zeroed with the backward part of the stat arena above
            self.dgrad(l1, dz1, sk, split=True, out2=dt, bn_stats=(tsum[0], tsum[1]))
            gb_up = self.ps.gview(lu.name + "/b")
            c0 = l1.cin_s[0]
            ops.add_mask(gb_up, gb_up, b=tsum[0, c0:c0 + gb_up.numel()])
            skip_grad[i] = sk
            # ConvTranspose dec{i}_up reads the previous level's activation
            pact = a[f"ay{i + 1}_2"] if i + 1 < Lv - 1 else a[f"az{Lv - 1}_2"]
            self._side_wgrad(lu, pact, dt, bias_grad=False)
            dAp = gb(f"dA_up{i}", pact)
            if i + 1 < Lv - 1:
                red = self._bn_red(f"dec{i + 1}_conv2", a[f"y{i + 1}_2"])
            else:
                red = self._bn_red(f"enc{Lv - 1}_conv2", a[f"z{Lv - 1}_2"])
            self.dgrad(lu, dt, dAp, bn_reduce=red)
            if i + 1 < Lv - 1:
                cur_dA = dAp
            else:
                bott_dA = dAp
        # bottleneck + encoder, from the deepest level up to level 0
        dpool = None
        for i in range(Lv - 1, -1, -1):
            z2, z1 = a[f"z{i}_2"], a[f"z{i}_1"]
            if i < Lv - 1:
                # dA of enc{i}_conv2 = concat-skip part + pool backward (argmax on the activation)
                dA2 = gb(f"dA_z{i}_2", z2)
                # pool backward + skip gradient, with enc{i}_conv2's BN-backward reduction fused in
                ops.maxpool2_bwd(a[f"az{i}_2"], dpool, dA2, addend=skip_grad[i],
                                 bn_reduce=self._bn_red(f"enc{i}_conv2", z2), argmax_from_z=self.pool_argmax_from_z)
            else:
                dA2 = bott_dA
            dz2 = gb(f"dz_z{i}_2", z2)
            l2 = L[f"enc{i}_conv2"]
            self._bn_bwd_wgrad(f"enc{i}_conv2", dA2, z2, dz2, l2, a[f"az{i}_1"])
            dA1 = gb(f"dA_z{i}_1", z1)
            self.dgrad(l2, dz2, dA1, bn_reduce=self._bn_red(f"enc{i}_conv1", z1))
            # (the input layer has no data gradient: with the fused BN-backward weight gradient nothing reads
            # its dz, which is then never stored)
            dz1 = gb(f"dz_z{i}_1", z1) if i > 0 or not self.fuse_bn_wgrad else None
            l1 = L[f"enc{i}_conv1"]
            src = a["x"] if i == 0 else a[f"pool{i - 1}"]
            self._bn_bwd_wgrad(f"enc{i}_conv1", dA1, z1, dz1, l1, src)
            if i > 0:
                dpool = gb(f"dpool{i - 1}", a[f"pool{i - 1}"])
                self.dgrad(l1, dz1, dpool)
