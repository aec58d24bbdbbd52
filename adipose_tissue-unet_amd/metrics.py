"""Loss / metric surface of the reference, computed by the libadipose_hip reduction kernels.

Callables take ``(y_true, y_pred)`` (B,H,W) float32 tensors (device tensors, or numpy arrays which
are uploaded) and return Python floats, mirroring:
  src/utils/model.py:8-19, 93-101    jaccard_coef, jaccard_coef_int, dice_coef, dice_coef_loss
  train_adipose_unet_v3.py:217-363   dice_loss, combined_loss_standard, combined_loss_with_label_smoothing,
                                     online_hard_example_mining_loss(_with_smoothing)
  Keras binary_accuracy (compile_model metrics :852-854)
  src/utils/model.py:21-91            mean_diff, act_mean/min/max/std, tru_pos, fls_pos, tru_neg, fls_neg,
                                     precision_onehot, recall_onehot, fmeasure_onehot
  src/utils/model.py:103-153          weighted_dice_loss, weighted_dice_coeff, weighted_bce_loss,
                                     weighted_bce_dice_loss (+ their gradients: weighted_loss_and_grad)
  full_evaluation_enhanced.py:721-785 calculate_pixel_metrics (tp/fp/fn/tn counted on the GPU)
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops
from ._lib import call, ptr, stream_ptr

KEPS = 1e-7


def _dev(t):
    if isinstance(t, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(t, dtype=np.float32))
    if not t.is_cuda:
        t = t.cuda()
    t = t.float().contiguous()
    if t.dim() == 2:
        t = t[None]
    return t


def _stats(y_true, y_pred, *, smooth=False, eps_pos=0.03, eps_neg=0.07):
    y, p = _dev(y_true), _dev(y_pred)
    if y.shape != p.shape:
        raise ValueError(f"shape mismatch {tuple(y.shape)} vs {tuple(p.shape)}")
    N, H, W = p.shape
    rows = torch.empty(N * H, dtype=torch.float32, device=p.device)
    st = torch.empty(8, dtype=torch.float64, device=p.device)
    ops.fill(st.view(torch.float32), 0.0)
    ops.loss_rows(p, y, rows, st, smooth=smooth, eps_pos=eps_pos, eps_neg=eps_neg)
    return y, p, rows, st


def _bce_part(rows, N, H, W, ohem, keep_ratio):
    coef = torch.empty(N * H, dtype=torch.float32, device=rows.device)
    out = torch.empty(1, dtype=torch.float64, device=rows.device)
    ops.fill(out.view(torch.float32), 0.0)
    k = int(np.float32(H) * np.float32(keep_ratio)) if ohem else H
    ops.loss_select(rows, coef, out, N=N, H=H, W=W, ohem=ohem, keep_ratio=keep_ratio, weight=1.0, norm_rows=N * k)
    return out.item()


def _dice_loss_from(st):
    s = st.cpu().numpy()
    return 1.0 - (2.0 * s[0] + 1.0) / (s[1] + s[2] + 1.0)


def dice_coef(y_true, y_pred):
    """(2Σyp+1)/(Σy+Σp+1), no clipping, whole batch (model.py:93-98)."""
    s = _stats(y_true, y_pred)[3].cpu().numpy()
    return float((2.0 * s[3] + 1.0) / (s[4] + s[5] + 1.0))


def dice_coef_loss(y_true, y_pred):
    return -dice_coef(y_true, y_pred)


def jaccard_coef(y_true, y_pred):
    """model.py:8-12; axis=[0,-1,-2] on a (B,H,W) tensor reduces everything to one scalar."""
    s = _stats(y_true, y_pred)[3].cpu().numpy()
    inter, tot = s[3], s[4] + s[5]
    return float((inter + KEPS) / (tot - inter + KEPS))


def jaccard_coef_int(y_true, y_pred):
    """model.py:14-19: round(clip(p)) in the intersection but raw p in the sum (reference quirk)."""
    s = _stats(y_true, y_pred)[3].cpu().numpy()
    inter, tot = s[7], s[4] + s[5]
    return float((inter + KEPS) / (tot - inter + KEPS))


def binary_accuracy(y_true, y_pred, threshold=0.5):
    y, p, _, st = _stats(y_true, y_pred)
    if threshold != 0.5:
        raise ValueError("binary_accuracy kernel uses the Keras default threshold 0.5")
    return float(st[6].item() / p.numel())


def dice_loss(y_true, y_pred):
    """train_adipose_unet_v3.py:217-225 (clipped p, batch-global)."""
    return float(_dice_loss_from(_stats(y_true, y_pred)[3]))


def combined_loss_standard(y_true, y_pred):
    """:228-241 = mean(row BCE) + dice_loss."""
    y, p, rows, st = _stats(y_true, y_pred)
    N, H, W = p.shape
    return float(_bce_part(rows, N, H, W, False, 0.7) + _dice_loss_from(st))


def combined_loss_with_label_smoothing(y_true, y_pred, epsilon_pos=0.03, epsilon_neg=0.07):
    """:244-279"""
    y, p, rows, st = _stats(y_true, y_pred, smooth=True, eps_pos=epsilon_pos, eps_neg=epsilon_neg)
    N, H, W = p.shape
    return float(_bce_part(rows, N, H, W, False, 0.7) + _dice_loss_from(st))


def online_hard_example_mining_loss(y_true, y_pred, keep_ratio=0.7):
    """:282-318 (row-level top-k, k = int(H*keep_ratio) per image, + global dice)."""
    y, p, rows, st = _stats(y_true, y_pred)
    N, H, W = p.shape
    return float(_bce_part(rows, N, H, W, True, keep_ratio) + _dice_loss_from(st))


def online_hard_example_mining_loss_with_smoothing(y_true, y_pred, keep_ratio=0.7, epsilon_pos=0.03,
                                                   epsilon_neg=0.07):
    """:321-363"""
    y, p, rows, st = _stats(y_true, y_pred, smooth=True, eps_pos=epsilon_pos, eps_neg=epsilon_neg)
    N, H, W = p.shape
    return float(_bce_part(rows, N, H, W, True, keep_ratio) + _dice_loss_from(st))


# ------------------------------------------------------------- model.py metric helpers (:21-91)
def _value_stats(x):
    x = _dev(x)
    work = torch.empty(1024 * 40, dtype=torch.uint8, device=x.device)
    out = torch.empty(4, dtype=torch.float64, device=x.device)
    call("adp_value_stats", x.numel(), ptr(x), ptr(work), ptr(out), stream_ptr())
    return out.cpu().numpy()   # mean, min, max, population std


def act_mean(y_true, y_pred):
    return float(_value_stats(y_pred)[0])


def act_min(y_true, y_pred):
    return float(_value_stats(y_pred)[1])


def act_max(y_true, y_pred):
    return float(_value_stats(y_pred)[2])


def act_std(y_true, y_pred):
    """K.std: population standard deviation."""
    return float(_value_stats(y_pred)[3])


def mean_diff(y_true, y_pred):
    return float(_value_stats(y_pred)[0] - _value_stats(y_true)[0])


def _onehot_counts(y_true, y_pred):
    y, p = _dev(y_true), _dev(y_pred)
    if y.shape != p.shape:
        raise ValueError(f"shape mismatch {tuple(y.shape)} vs {tuple(p.shape)}")
    W = p.shape[-1]
    out = torch.zeros(7, dtype=torch.int64, device=p.device)
    call("adp_onehot_counts", p.numel() // W, W, ptr(y), ptr(p), ptr(out), stream_ptr())
    return [int(v) for v in out.cpu().tolist()]


def tru_pos(y_true, y_pred):
    """sum argmax(y) * argmax(p) over the last axis (model.py:36-41)."""
    return _onehot_counts(y_true, y_pred)[0]


def fls_pos(y_true, y_pred):
    return _onehot_counts(y_true, y_pred)[1]


def tru_neg(y_true, y_pred):
    return _onehot_counts(y_true, y_pred)[2]


def fls_neg(y_true, y_pred):
    return _onehot_counts(y_true, y_pred)[3]


def precision_onehot(y_true, y_pred):
    c = _onehot_counts(y_true, y_pred)
    return float(np.float32(c[4]) / (np.float32(c[5]) + np.float32(KEPS)))


def recall_onehot(y_true, y_pred):
    c = _onehot_counts(y_true, y_pred)
    return float(np.float32(c[4]) / (np.float32(c[6]) + np.float32(KEPS)))


def fmeasure_onehot(y_true, y_pred):
    p, r = np.float32(precision_onehot(y_true, y_pred)), np.float32(recall_onehot(y_true, y_pred))
    return float(2 * (p * r) / (p + r + np.float32(KEPS)))


# ---------------------------------------------------------------- weighted losses (:103-153)
def border_weight(y_true, ksize=21):
    """(weight (B,H,W) before renormalisation, sum of it) of weighted_dice_loss (model.py:104-116): the
    21x21 'same' average of y expanded to (1,B,H,W), i.e. pooled over (B,H) per W, TF's pad-excluding count."""
    y = _dev(y_true)
    B, H, W = y.shape
    tmp = torch.empty_like(y)
    wt = torch.empty_like(y)
    wsum = torch.zeros(1, dtype=torch.float64, device=y.device)
    call("adp_border_weight", B, H, W, int(ksize), ptr(y), ptr(tmp), ptr(wt), ptr(wsum), stream_ptr())
    return wt, wsum


def _wstats(y, p, wt, wsum):
    st = torch.zeros(5, dtype=torch.float64, device=p.device)
    call("adp_weighted_loss_stats", p.numel(), ptr(y), ptr(p), ptr(wt), ptr(wsum), ptr(st), stream_ptr())
    return st


def weighted_dice_coeff(y_true, y_pred, weight):
    """model.py:120-125 with an explicit weight (B,H,W) or (1,B,H,W) (used as given, no renormalisation)."""
    y, p, w = _dev(y_true), _dev(y_pred), _dev(weight).reshape(_dev(y_pred).shape).contiguous()
    one = torch.full((1,), float(w.numel()), dtype=torch.float64, device=p.device)   # ratio 1
    s = _wstats(y, p, w, one).cpu().numpy()
    return float((2.0 * s[0] + 1.0) / (s[1] + s[2] + 1.0))


def weighted_bce_loss(y_true, y_pred, weight):
    """model.py:127-136 with an explicit weight (used as given)."""
    y, p, w = _dev(y_true), _dev(y_pred), _dev(weight).reshape(_dev(y_pred).shape).contiguous()
    one = torch.full((1,), float(w.numel()), dtype=torch.float64, device=p.device)
    s = _wstats(y, p, w, one).cpu().numpy()
    return float(s[3] / s[4])


def weighted_loss_and_grad(y_true, y_pred, *, bce=True, ksize=21):
    """weighted_bce_dice_loss (bce=True, model.py:139-153) or weighted_dice_loss (bce=False, :103-118):
    (loss, dL/dp as a device tensor shaped like y_pred)."""
    y, p = _dev(y_true), _dev(y_pred)
    if y.shape != p.shape:
        raise ValueError(f"shape mismatch {tuple(y.shape)} vs {tuple(p.shape)}")
    wt, wsum = border_weight(y, ksize)
    st = _wstats(y, p, wt, wsum)
    dp = torch.empty_like(p)
    call("adp_weighted_loss_grad", p.numel(), ptr(y), ptr(p), ptr(wt), ptr(wsum), ptr(st), 1.0 if bce else 0.0, 1.0,
         ptr(dp), stream_ptr())
    s = st.cpu().numpy()
    loss = 1.0 - (2.0 * s[0] + 1.0) / (s[1] + s[2] + 1.0)
    if bce:
        loss += s[3] / s[4]
    return float(loss), dp


def weighted_dice_loss(y_true, y_pred):
    return weighted_loss_and_grad(y_true, y_pred, bce=False)[0]


def weighted_bce_dice_loss(y_true, y_pred):
    return weighted_loss_and_grad(y_true, y_pred, bce=True)[0]


# ------------------------------------------------------------------------------ evaluation
def pixel_counts(pred, true, threshold=0.5):
    """(tp, fp, fn, tn) of (pred > threshold) vs (true > 0.5), counted on the GPU (int64)."""
    p, t = _dev(pred), _dev(true)
    c = torch.zeros(4, dtype=torch.int64, device=p.device)
    ops.pixel_counts(p, t, float(threshold), c)
    return tuple(int(v) for v in c.cpu().tolist())


def metrics_from_counts(tp, fp, fn, tn):
    """Ratios of full_evaluation_enhanced.py:763-785 (float64, +1e-10 guards)."""
    precision = tp / (tp + fp + 1e-10)
    sensitivity = tp / (tp + fn + 1e-10)
    specificity = tn / (tn + fp + 1e-10)
    accuracy = (tp + tn) / (tp + fp + fn + tn + 1e-10)
    f1 = 2 * tp / (2 * tp + fp + fn + 1e-10)
    jaccard = tp / (tp + fp + fn + 1e-10)
    return {"dice_score": float(f1), "jaccard_index": float(jaccard), "sensitivity": float(sensitivity),
            "specificity": float(specificity), "precision": float(precision), "f1_score": float(f1),
            "accuracy": float(accuracy), "tp": int(tp), "fp": int(fp), "fn": int(fn), "tn": int(tn)}


def calculate_pixel_metrics(pred, true, threshold=0.5):
    """full_evaluation_enhanced.py:721-785, counts from the GPU; both-empty -> all 1.0."""
    tp, fp, fn, tn = pixel_counts(pred, true, threshold)
    if tp + fp == 0 and tp + fn == 0:
        return {"dice_score": 1.0, "jaccard_index": 1.0, "sensitivity": 1.0, "specificity": 1.0,
                "precision": 1.0, "f1_score": 1.0, "accuracy": 1.0, "tp": 0, "fp": 0, "fn": 0, "tn": int(tn)}
    return metrics_from_counts(tp, fp, fn, tn)
