"""Loss / metric surface of the reference, computed by the libadipose_hip reduction kernels.

Callables take ``(y_true, y_pred)`` (B,H,W) float32 tensors (device tensors, or numpy arrays which
are uploaded) and return Python floats, mirroring:
  src/utils/model.py:8-19, 93-101    jaccard_coef, jaccard_coef_int, dice_coef, dice_coef_loss
  train_adipose_unet_v3.py:217-363   dice_loss, combined_loss_standard, combined_loss_with_label_smoothing,
                                     online_hard_example_mining_loss(_with_smoothing)
  Keras binary_accuracy (compile_model metrics :852-854)
  full_evaluation_enhanced.py:721-785 calculate_pixel_metrics (tp/fp/fn/tn counted on the GPU)
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops

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
