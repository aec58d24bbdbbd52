"""CPU fp32 restatement of the reference hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker / CPU baseline. The product path (adipose_amd) never calls it.

Parity status: the reference's arithmetic lives in TensorFlow 2.13 / Keras 2.13, which is not
installed here (ordinary ImportError) — so the TF-level numerics below are a
restatement that follows the reference files line by line; "parity unpinned vs TF2.13" for the
network/loss arithmetic. The numpy-level evaluation functions (metrics, sliding window, blending,
TTA) are pinned by golden vectors generated from the reference itself (tests/golden/).

Layout: tensors are NHWC (Keras channels_last) on the CPU; kernels are Keras HWIO.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

KEPS = 1e-7  # keras.backend.epsilon()


# ----------------------------------------------------------------------------- layer helpers
def conv2d_same(x, kernel, bias=None, dilation=1, relu=True):
    """Keras Conv2D(filters, k, padding='same', dilation_rate=d, activation='relu')
    (train_adipose_unet_v3.py:668-709). x NHWC, kernel HWIO."""
    k = kernel.shape[0]
    pad = dilation * (k // 2)
    w = kernel.permute(3, 2, 0, 1)  # OIHW
    y = F.conv2d(x.permute(0, 3, 1, 2), w, bias, padding=pad, dilation=dilation)
    y = y.permute(0, 2, 3, 1)
    return F.relu(y) if relu else y


def upsample_nearest2(x):
    """UpSampling2D((2,2)) (:691,698,705): repeat rows and columns."""
    return x.repeat_interleave(2, dim=1).repeat_interleave(2, dim=2)


def maxpool2(x):
    """MaxPooling2D((2,2), strides=(2,2)) (:670,674,678), 'valid'."""
    return F.max_pool2d(x.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1)


def resize_bilinear_half_pixel(x, size):
    """tf.image.resize(x, size, 'bilinear') == half-pixel centres, no antialias (:716-726).
    For upsampling, torch bilinear(align_corners=False) clamps negative source coordinates to 0,
    which yields the same value as TF's lower=max(floor,0)/upper=min(ceil,n-1)/lerp=in-floor(in)."""
    y = F.interpolate(x.permute(0, 3, 1, 2), size=size, mode="bilinear", align_corners=False)
    return y.permute(0, 2, 3, 1)


def conv1x1(x, kernel, bias):
    return torch.einsum("nhwc,co->nhwo", x, kernel[0, 0]) + bias


# --------------------------------------------------------------------------------- networks
ADIPOSE_LAYERS = (
    ["down1_conv1", "down1_conv2", "down2_conv1", "down2_conv2", "down3_conv1", "down3_conv2"]
    + [f"dilate{i}" for i in range(1, 7)]
    + [f"up{l}_conv{j}" for l in (3, 2, 1) for j in (1, 2, 3)])


def adipose_v3_keras_weights(seed=865, init_nb=44, deep_supervision=True):
    """Glorot-uniform kernels and N(0, 0.01) biases (Keras would start biases at zero; non-zero biases exercise
    the bias paths) with Keras shapes, keyed by Keras layer name."""
    rng = np.random.default_rng(seed)
    nb = init_nb
    shapes = {
        "down1_conv1": (1, nb), "down1_conv2": (nb, nb), "down2_conv1": (nb, 2 * nb),
        "down2_conv2": (2 * nb, 2 * nb), "down3_conv1": (2 * nb, 4 * nb), "down3_conv2": (4 * nb, 4 * nb),
        "dilate1": (4 * nb, 8 * nb), "up3_conv1": (8 * nb, 4 * nb), "up3_conv2": (8 * nb, 4 * nb),
        "up3_conv3": (4 * nb, 4 * nb), "up2_conv1": (4 * nb, 2 * nb), "up2_conv2": (4 * nb, 2 * nb),
        "up2_conv3": (2 * nb, 2 * nb), "up1_conv1": (2 * nb, nb), "up1_conv2": (2 * nb, nb), "up1_conv3": (nb, nb),
    }
    for i in range(2, 7):
        shapes[f"dilate{i}"] = (8 * nb, 8 * nb)
    w = {}
    for name in ADIPOSE_LAYERS:
        ci, co = shapes[name]
        lim = math.sqrt(6.0 / (9 * ci + 9 * co))
        w[name] = [rng.uniform(-lim, lim, (3, 3, ci, co)).astype(np.float32),
                   rng.normal(0, 0.01, co).astype(np.float32)]
    heads = {"output_softmax": (nb, 2)}
    if deep_supervision:
        heads.update({"aux_out1": (4 * nb, 1), "aux_out2": (2 * nb, 1)})
    for name, (ci, co) in heads.items():
        lim = math.sqrt(6.0 / (ci + co))
        w[name] = [rng.uniform(-lim, lim, (1, 1, ci, co)).astype(np.float32),
                   rng.normal(0, 0.01, co).astype(np.float32)]
    return w


def adipose_v3_forward(x, weights, deep_supervision=True, dropout_masks=None):
    """AdiposeUNetV3.build_model (train_adipose_unet_v3.py:660-758), generalised in S.
    x: (B, S, S) normalised float32. Dropout is identity unless masks are given (inference / parity).
    Returns dict main_out / aux_out1 / aux_out2 of (B, S, S)."""
    t = lambda a: a if torch.is_tensor(a) else torch.as_tensor(np.asarray(a))  # noqa: E731
    W = {k: [t(v[0]), t(v[1])] for k, v in weights.items()}
    S = x.shape[1]
    h = x.reshape(x.shape[0], S, S, 1)

    def c(name, inp, dil=1):
        return conv2d_same(inp, W[name][0], W[name][1], dilation=dil)

    def drop(name, v):
        if dropout_masks and name in dropout_masks:
            return v * dropout_masks[name]
        return v

    d1 = c("down1_conv2", c("down1_conv1", h))
    d2 = c("down2_conv2", c("down2_conv1", maxpool2(d1)))
    d3 = c("down3_conv2", c("down3_conv1", maxpool2(d2)))
    p3 = maxpool2(d3)
    dl = [drop("dropout_dilate1", c("dilate1", p3))]
    for i, dil in zip(range(2, 7), (2, 4, 8, 16, 32)):
        dl.append(c(f"dilate{i}", dl[-1], dil))
    s = dl[0] + dl[1] + dl[2] + dl[3] + dl[4] + dl[5]
    u3 = c("up3_conv1", upsample_nearest2(s))
    u3 = drop("dropout_up3", c("up3_conv3", c("up3_conv2", torch.cat([d3, u3], -1))))
    u2 = c("up2_conv1", upsample_nearest2(u3))
    u2 = drop("dropout_up2", c("up2_conv3", c("up2_conv2", torch.cat([d2, u2], -1))))
    u1 = c("up1_conv1", upsample_nearest2(u2))
    u1 = drop("dropout_up1", c("up1_conv3", c("up1_conv2", torch.cat([d1, u1], -1))))
    z = conv1x1(u1, W["output_softmax"][0], W["output_softmax"][1])
    out = {"main_out": torch.softmax(z, -1)[..., 1]}
    if deep_supervision:
        a1 = torch.sigmoid(conv1x1(u3, W["aux_out1"][0], W["aux_out1"][1]))
        a2 = torch.sigmoid(conv1x1(u2, W["aux_out2"][0], W["aux_out2"][1]))
        out["aux_out1"] = resize_bilinear_half_pixel(a1, (S, S))[..., 0]
        out["aux_out2"] = resize_bilinear_half_pixel(a2, (S, S))[..., 0]
    return out


def unet_bn_keras_weights(levels=5, base=64, in_ch=3, seed=865):
    """Weights for the north-star BN U-Net (no reference code): conv kernels HWIO, ConvT (Cin,Cout,2,2)."""
    rng = np.random.default_rng(seed)
    w = {}
    cin = in_ch
    ch = lambda i: base << i  # noqa: E731
    for i in range(levels):
        c = ch(i)
        for j, ci in ((1, cin), (2, c)):
            lim = math.sqrt(6.0 / (9 * ci + 9 * c))
            w[f"enc{i}_conv{j}"] = [rng.uniform(-lim, lim, (3, 3, ci, c)).astype(np.float32),
                                    (1 + rng.normal(0, 0.1, c)).astype(np.float32),
                                    rng.normal(0, 0.1, c).astype(np.float32)]
        cin = c
    for i in range(levels - 2, -1, -1):
        c = ch(i)
        lim = math.sqrt(6.0 / (4 * ch(i + 1) + 4 * c))
        w[f"dec{i}_up"] = [rng.uniform(-lim, lim, (ch(i + 1), c, 2, 2)).astype(np.float32),
                           rng.normal(0, 0.01, c).astype(np.float32)]
        for j, ci in ((1, 2 * c), (2, c)):
            lim = math.sqrt(6.0 / (9 * ci + 9 * c))
            w[f"dec{i}_conv{j}"] = [rng.uniform(-lim, lim, (3, 3, ci, c)).astype(np.float32),
                                    (1 + rng.normal(0, 0.1, c)).astype(np.float32),
                                    rng.normal(0, 0.1, c).astype(np.float32)]
    lim = math.sqrt(6.0 / (base + 1))
    w["head"] = [rng.uniform(-lim, lim, (1, 1, base, 1)).astype(np.float32), np.zeros(1, np.float32)]
    return w


def bn_relu_train(z, gamma, beta, eps=1e-5, record=None):
    """record: optional list; gets {"margin": min |pre-ReLU value|, "mean", "var_unbiased"} of this layer
    appended (test conditioning: an element within float rounding of the ReLU kink takes either
    subgradient; running statistics: momentum updates use the unbiased batch variance)."""
    mean = z.mean(dim=(0, 1, 2))
    var = z.var(dim=(0, 1, 2), unbiased=False)
    pre = (z - mean) / torch.sqrt(var + eps) * gamma + beta
    if record is not None:
        record.append({"margin": pre.detach().abs().min().item(), "mean": mean.detach().clone(),
                       "var_unbiased": z.detach().var(dim=(0, 1, 2), unbiased=True)})
    return F.relu(pre)


def unet_bn_forward(x, weights, levels=5, record=None):
    """x: (B,S,S,C_in) NHWC; training-mode BatchNorm (batch statistics). Returns (B,S,S) sigmoid.
    record: optional list, receives one entry per BatchNorm layer in execution order (bn_relu_train)."""
    t = lambda a: a if torch.is_tensor(a) else torch.as_tensor(np.asarray(a))  # noqa: E731
    W = {k: [t(v) for v in vs] for k, vs in weights.items()}

    def blk(name, inp):
        k, g, b = W[name]
        return bn_relu_train(conv2d_same(inp, k, None, relu=False), g, b, record=record)

    skips = []
    h = x
    for i in range(levels):
        h = blk(f"enc{i}_conv2", blk(f"enc{i}_conv1", h))
        if i < levels - 1:
            skips.append(h)
            h = maxpool2(h)
    for i in range(levels - 2, -1, -1):
        k, b = W[f"dec{i}_up"]
        u = F.conv_transpose2d(h.permute(0, 3, 1, 2), k, b, stride=2).permute(0, 2, 3, 1)
        h = blk(f"dec{i}_conv2", blk(f"dec{i}_conv1", torch.cat([skips[i], u], -1)))
    k, b = W["head"]
    return torch.sigmoid(conv1x1(h, k, b))[..., 0]


# ----------------------------------------------------------------------------------- losses
def keras_bce_rows(y, p):
    """keras.losses.binary_crossentropy (Keras 2.13): clip p to [eps, 1-eps], then
    -(y log(p+eps) + (1-y) log(1-p+eps)), mean over the LAST axis -> (B, H)."""
    pc = torch.clamp(p, KEPS, 1.0 - KEPS)
    bce = -(y * torch.log(pc + KEPS) + (1 - y) * torch.log(1 - pc + KEPS))
    return bce.mean(-1)


def dice_loss(y, p):
    """train_adipose_unet_v3.py:217-225 (batch-global, clipped p)."""
    pc = torch.clamp(p, KEPS, 1.0 - KEPS)
    inter = (y * pc).sum()
    return 1.0 - (2.0 * inter + 1.0) / (y.sum() + pc.sum() + 1.0)


def combined_loss_standard(y, p):
    """:228-241 -> mean over (B,H) of row BCE + dice (Keras SUM_OVER_BATCH_SIZE reduction)."""
    return keras_bce_rows(y, p).mean() + dice_loss(y, p)


def smooth_labels(y, eps_pos=0.03, eps_neg=0.07):
    return y * (1.0 - eps_pos - eps_neg) + eps_neg


def combined_loss_with_label_smoothing(y, p, eps_pos=0.03, eps_neg=0.07):
    """:244-279"""
    ys = smooth_labels(y, eps_pos, eps_neg)
    return keras_bce_rows(ys, p).mean() + dice_loss(ys, p)


def ohem_loss(y, p, keep_ratio=0.7):
    """online_hard_example_mining_loss :282-318. 'per-pixel' BCE is per ROW (mean over last axis);
    k = int(float32(H) * keep_ratio) rows per image; mean of the selected row losses + global dice."""
    rows = keras_bce_rows(y, p)
    H = rows.shape[1]
    k = int(np.float32(H) * np.float32(keep_ratio))
    top = torch.topk(rows, k, dim=1).values
    return top.mean() + dice_loss(y, p)


def ohem_loss_with_smoothing(y, p, keep_ratio=0.7, eps_pos=0.03, eps_neg=0.07):
    """:321-363"""
    ys = smooth_labels(y, eps_pos, eps_neg)
    rows = keras_bce_rows(ys, p)
    k = int(np.float32(rows.shape[1]) * np.float32(keep_ratio))
    return torch.topk(rows, k, dim=1).values.mean() + dice_loss(ys, p)


def ds_total_loss(y, outs, *, use_hard_mining=True, keep_ratio=0.7, use_label_smoothing=False, eps_pos=0.03,
                  eps_neg=0.07, w_main=1.0, w_aux1=0.4, w_aux2=0.3):
    """compile_model (:808-855): weighted sum over main_out / aux_out1 / aux_out2."""
    if use_label_smoothing and use_hard_mining:
        fm = lambda a, b: ohem_loss_with_smoothing(a, b, keep_ratio, eps_pos, eps_neg)  # noqa: E731
        fa = lambda a, b: combined_loss_with_label_smoothing(a, b, eps_pos, eps_neg)  # noqa: E731
    elif use_label_smoothing:
        fm = fa = lambda a, b: combined_loss_with_label_smoothing(a, b, eps_pos, eps_neg)  # noqa: E731
    elif use_hard_mining:
        fm = lambda a, b: ohem_loss(a, b, keep_ratio)  # noqa: E731
        fa = combined_loss_standard
    else:
        fm = fa = combined_loss_standard
    total = w_main * fm(y, outs["main_out"])
    if "aux_out1" in outs:
        total = total + w_aux1 * fa(y, outs["aux_out1"]) + w_aux2 * fa(y, outs["aux_out2"])
    return total


def dice_coef(y, p):
    """src/utils/model.py:93-98 (no clipping, whole batch)."""
    return (2.0 * (y * p).sum() + 1.0) / (y.sum() + p.sum() + 1.0)


def binary_accuracy(y, p, threshold=0.5):
    return (y == (p > threshold).to(p.dtype)).to(torch.float32).mean()


# ------------------------------------------------------- rest of the model.py loss / metric surface
def jaccard_coef(y, p):
    """src/utils/model.py:8-12 (axis=[0,-1,-2] of a (B,H,W) tensor: one scalar)."""
    inter = (y * p).sum()
    return (inter + KEPS) / ((y + p).sum() - inter + KEPS)


def jaccard_coef_int(y, p):
    """model.py:14-19: round(clip(p, 0, 1)) in the intersection, raw p in the sum (quirk kept)."""
    inter = (y * torch.round(torch.clamp(p, 0.0, 1.0))).sum()
    return (inter + KEPS) / ((y + p).sum() - inter + KEPS)


def avg_pool_same(x4, k):
    """K.pool2d(x4, (k, k), strides=(1, 1), padding='same', pool_mode='avg') on a channels_last (N, D1, D2, C)
    tensor: TF's SAME average pooling divides by the number of VALID elements in each window."""
    xc = x4.permute(0, 3, 1, 2)
    r = k // 2
    s = F.avg_pool2d(xc, k, stride=1, padding=r, count_include_pad=False)
    return s.permute(0, 2, 3, 1)


def border_weight(y, k=21):
    """The weight map of weighted_dice_loss / weighted_bce_dice_loss (model.py:104-116, 140-151):
    y (B,H,W) -> expand_dims(0) = (1,B,H,W), pooled over (B,H) with W as channels (the reference's quirk);
    border = (avg > 0.005) * (avg < 0.995); weight = 1 + 2 * border renormalised by sum(ones)/sum(weight).
    Returns the (1,B,H,W) weight."""
    y4 = y[None]
    avg = avg_pool_same(y4, k)
    border = (avg > 0.005).to(y.dtype) * (avg < 0.995).to(y.dtype)
    weight = torch.ones_like(avg)
    w0 = weight.sum()
    weight = weight + border * 2
    w1 = weight.sum()
    return weight * (w0 / w1)


def weighted_dice_coeff(y, p, weight):
    """model.py:120-125 (y and p broadcast against weight's (1,B,H,W))."""
    w = weight * weight
    return (2.0 * (w * (y * p)).sum() + 1.0) / ((w * y).sum() + (w * p).sum() + 1.0)


def weighted_bce_loss(y, p, weight):
    """model.py:127-136; max(-l, 0) written as where(-l >= 0, -l, 0) so its subgradient at l = 0 is TF's
    (tf.maximum routes the gradient to its first argument on ties; torch.maximum would split it)."""
    pc = torch.clamp(p, KEPS, 1.0 - KEPS)
    lg = torch.log(pc / (1.0 - pc))
    relu_neg = torch.where(-lg >= 0, -lg, torch.zeros_like(lg))
    loss = (1.0 - y) * lg + (1.0 + (weight - 1.0) * y) * (torch.log(1.0 + torch.exp(-torch.abs(lg))) + relu_neg)
    return loss.sum() / weight.sum()


def weighted_dice_loss(y, p):
    """model.py:103-118 (y expanded to (1,B,H,W) before the pool and the coefficient)."""
    wt = border_weight(y)
    return 1.0 - weighted_dice_coeff(y[None], p, wt)


def weighted_bce_dice_loss(y, p):
    """model.py:139-153"""
    wt = border_weight(y)
    y4 = y[None]
    return weighted_bce_loss(y4, p, wt) + (1.0 - weighted_dice_coeff(y4, p, wt))


def metric_helpers(y, p):
    """model.py:21-91 on (B,H,W) tensors: argmax / argmin over the last axis (first occurrence)."""
    at, ap = torch.argmax(y, -1), torch.argmax(p, -1)
    it, ip = torch.argmin(y, -1), torch.argmin(p, -1)
    ytf, ypf = at.double(), ap.double()
    tp = torch.round(torch.clamp(ytf * ypf, 0, 1)).sum()
    pp = torch.round(torch.clamp(ypf, 0, 1)).sum()
    pos = torch.round(torch.clamp(ytf, 0, 1)).sum()
    prec = tp / (pp + KEPS)
    rec = tp / (pos + KEPS)
    return {"mean_diff": (p.double().mean() - y.double().mean()).item(), "act_mean": p.double().mean().item(),
            "act_min": p.min().item(), "act_max": p.max().item(), "act_std": p.double().std(unbiased=False).item(),
            "tru_pos": int((at * ap).sum()), "fls_pos": int(torch.clamp(ap - at, 0, 1).sum()),
            "tru_neg": int((it * ip).sum()), "fls_neg": int(torch.clamp(ip - it, 0, 1).sum()),
            "precision_onehot": prec.item(), "recall_onehot": rec.item(),
            "fmeasure_onehot": (2 * (prec * rec) / (prec + rec + KEPS)).item()}


# --------------------------------------------------------------------------------- optimizer
class KerasAdam:
    """Keras 2.13 Adam / AdamW update_step (optimizer_experimental), for parity tests."""

    def __init__(self, params, lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-7, weight_decay=0.0):
        self.p = params
        self.lr, self.b1, self.b2, self.eps, self.wd = lr, beta1, beta2, eps, weight_decay
        self.m = [torch.zeros_like(x) for x in params]
        self.v = [torch.zeros_like(x) for x in params]
        self.t = 0

    @torch.no_grad()
    def step(self, grads):
        self.t += 1
        alpha = self.lr * math.sqrt(1 - self.b2 ** self.t) / (1 - self.b1 ** self.t)
        for p, g, m, v in zip(self.p, grads, self.m, self.v):
            if self.wd:
                p -= p * self.wd * self.lr
            m += (g - m) * (1 - self.b1)
            v += (g * g - v) * (1 - self.b2)
            p -= m * alpha / (torch.sqrt(v) + self.eps)
