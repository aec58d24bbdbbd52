"""Evaluation surface of Segmentation/full_evaluation_enhanced.py on the HIP engine.

Same names, arguments, return values and printed summaries as the reference:
  resolve_weights_path / _find_best_weights_in_dir / _detect_deep_supervision   :401-520
  ComprehensiveMetrics                                                           :602-644
  set_deterministic_seeds, extract_slide_id, load_training_stats                 :647-713
  calculate_pixel_metrics (metrics.py, GPU counts), calculate_boundary_metrics,
  calculate_auc_metrics                                                          :721-888
  optimize_threshold_f1_slide_level / optimize_threshold_f1                      :891-980
  bootstrap_confidence_interval / safe_bootstrap_ci                              :983-1018
  create_4panel_visualization, sample_tiles, categorize_by_dice                  :1021-1153
  BoundaryRefiner                                                                :332-393
  read_image_gray, load_validation_data                                          :1356-1443
  run_publication_evaluation                                                     :1446-1958

MI355X-first differences (same results): predictions stay float32 device tensors until a CPU-only
metric needs them; the threshold search counts every threshold of the grid for a tile in ONE GPU pass
(adp_threshold_hist) instead of one numpy pass per threshold, ROC / PR AUC in one sort-and-scan GPU pass
(adp_auc_metrics), boundary metrics from exact GPU distance transforms (adp_boundary_metrics). cv2, tifffile, skimage and matplotlib are not
installed here: images/masks are read with PIL, skimage.morphology.binary_erosion is restated with
scipy.ndimage (cross footprint, border_value=1, as skimage 0.21 does), the 4-panel figure is drawn without
cv2/matplotlib, and the BoundaryRefiner runs on the GPU with OpenCV's documented semantics restated (csrc/refine.hip;
its pixel output vs cv2 is "parity unpinned").
"""
from __future__ import annotations

import ctypes as C
import json
import os
import time
import warnings
from collections import defaultdict
from dataclasses import dataclass
from datetime import datetime
from pathlib import Path
import math
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from . import ops
from .metrics import calculate_pixel_metrics, metrics_from_counts

# ------------------------------------------------------------------------------ checkpoints
_SUFFIXES = (".weights.h5", ".weights.safetensors")   # Keras 2.13 files first (this build writes them)
_WEIGHT_CANDIDATES_BEST = ["weights_best_overall", "phase2_best", "phase1_best", "best_model", "model_best",
                           "weights_best"]
_WEIGHT_CANDIDATES_EMA = ["weights_ema", "ema_weights_phase2", "ema_weights"]


def _find_best_weights_in_dir(ckpt_dir: Path, use_ema: bool = False) -> Optional[Path]:
    """:471-490 (each candidate as .weights.h5, then as an earlier build's .weights.safetensors)."""
    def first(names):
        for n in names:
            for suf in _SUFFIXES:
                p = ckpt_dir / (n + suf)
                if p.exists():
                    return p
        return None
    hit = first(_WEIGHT_CANDIDATES_EMA if use_ema else _WEIGHT_CANDIDATES_BEST)
    if hit is not None:
        return hit
    if use_ema:
        print("⚠️  EMA weights not found, falling back to best weights")
        hit = first(_WEIGHT_CANDIDATES_BEST)
        if hit is not None:
            return hit
    files = (sorted(ckpt_dir.glob("*.weights.h5")) + sorted(ckpt_dir.glob("*.weights.safetensors"))
             + sorted(ckpt_dir.glob("*.h5")))
    return files[0] if files else None


def resolve_weights_path(weights_arg: str, use_ema: bool = False) -> Tuple[str, str]:
    """:401-453"""
    if not weights_arg:
        raise ValueError("❌ --weights argument is required.\nPlease specify path to trained model weights.")
    roots = ["checkpoints", "segmentation", "classifier_runs"]
    if Path(weights_arg).is_dir():
        ckpt_dir = weights_arg
        if Path(ckpt_dir).name in roots:
            raise ValueError(f"❌ Cannot use root checkpoint directory: {ckpt_dir}\n"
                             f"Please specify a specific checkpoint directory")
        f = _find_best_weights_in_dir(Path(ckpt_dir), use_ema=use_ema)
        if f is None:
            raise FileNotFoundError(f"No {'EMA' if use_ema else 'best'} weights files found in directory: {ckpt_dir}")
        return str(f), ckpt_dir
    ckpt_dir = str(Path(weights_arg).parent)
    if Path(ckpt_dir).name in roots:
        raise ValueError(f"❌ Weights file appears to be in root checkpoint directory: {ckpt_dir}\n"
                         f"Weights should be in a timestamped checkpoint subdirectory.")
    return weights_arg, ckpt_dir


def _detect_deep_supervision(ckpt_dir: Path) -> bool:
    """:493-520 — string match in training_settings.log."""
    f = Path(ckpt_dir) / "training_settings.log"
    if not f.exists():
        return False
    try:
        content = f.read_text()
        return "use_deep_supervision: True" in content or "deep_supervision: True" in content
    except Exception as e:  # noqa: BLE001 (reference: warn and fall back)
        print(f"⚠️  Could not read training settings: {e}")
    return False


@dataclass
class ComprehensiveMetrics:
    """:602-644"""
    dice_score: float
    dice_ci: Tuple[float, float]
    jaccard_index: float
    jaccard_ci: Tuple[float, float]
    sensitivity: float
    sensitivity_ci: Tuple[float, float]
    specificity: float
    specificity_ci: Tuple[float, float]
    precision: float
    precision_ci: Tuple[float, float]
    f1_score: float
    f1_ci: Tuple[float, float]
    accuracy: float
    accuracy_ci: Tuple[float, float]
    roc_auc: float
    roc_auc_ci: Tuple[float, float]
    pr_auc: float
    pr_auc_ci: Tuple[float, float]
    hausdorff95: float
    hausdorff95_ci: Tuple[float, float]
    assd: float
    assd_ci: Tuple[float, float]
    n_slides: int
    n_tiles: int
    optimal_threshold: float


def set_deterministic_seeds(seed: int = 1337):
    """:647-655 (TF flags replaced by torch's)."""
    import random
    os.environ["PYTHONHASHSEED"] = str(seed)
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)


def extract_slide_id(tile_path: str) -> str:
    """:658-678"""
    stem = Path(tile_path).stem
    parts = stem.split("_")
    if len(parts) >= 2 and parts[-2].startswith("r") and parts[-1].startswith("c"):
        return "_".join(parts[:-2])
    if parts[-1].startswith(("r", "c")):
        return "_".join(parts[:-1])
    return stem


def load_training_stats(checkpoint_dir: str) -> Tuple[float, float]:
    """:681-713 — required (FileNotFoundError)."""
    p = Path(checkpoint_dir) / "normalization_stats.json"
    if not p.exists():
        raise FileNotFoundError(f"Training normalization statistics not found: {p}\n"
                                f"Make sure training was completed with the updated training script.")
    st = json.loads(p.read_text())
    mean, std = float(st["mean"]), float(st["std"])
    print(f"✓ Loaded training normalization statistics:\n  Mean: {mean:.4f}\n  Std: {std:.4f}\n  Source: {p}")
    return mean, std


def binarize_prediction(pred, threshold: float = 0.5):
    return (np.asarray(pred) > threshold).astype(np.uint8)


# ------------------------------------------------------------------------------ metrics
def _host(a):
    return a.detach().float().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)


def _dev(a):
    if isinstance(a, torch.Tensor):
        t = a if a.is_cuda else a.cuda()
    else:
        t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()
    return t.float().contiguous()


def threshold_counts(pred, true, thresholds) -> np.ndarray:
    """(T, 4) int64 [tp, fp, fn, tn] of (pred > t) vs (true > 0.5) for every t — one GPU pass."""
    thr = np.asarray(thresholds, dtype=np.float64)
    order = np.argsort(thr, kind="stable")
    p, t = _dev(pred), _dev(true)
    T = len(thr)
    hist = torch.zeros(2 * (T + 1), dtype=torch.int64, device=p.device)
    ops.threshold_hist(p, t, thr[order], hist)
    h = hist.cpu().numpy().reshape(2, T + 1)
    # suffix sums: count of pixels with j > k, i.e. pred > thr_sorted[k]
    above = np.cumsum(h[:, ::-1], axis=1)[:, ::-1][:, 1:]          # (2, T)
    pos, n = int(h[1].sum()), int(h.sum())
    out = np.zeros((T, 4), dtype=np.int64)
    for k, idx in enumerate(order):
        tp, fp = int(above[1, k]), int(above[0, k])
        out[idx] = (tp, fp, pos - tp, (n - pos) - fp)
    return out


def _metrics_from_row(c):
    tp, fp, fn, tn = (int(v) for v in c)
    if tp + fp == 0 and tp + fn == 0:
        return {"dice_score": 1.0, "jaccard_index": 1.0, "sensitivity": 1.0, "specificity": 1.0,
                "precision": 1.0, "f1_score": 1.0, "accuracy": 1.0, "tp": 0, "fp": 0, "fn": 0, "tn": tn}
    return metrics_from_counts(np.int64(tp), np.int64(fp), np.int64(fn), np.int64(tn))


def _dev_map(a, dev):
    t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.asarray(a, np.float32))
    t = t.to(dev, torch.float32).contiguous()
    if t.dim() != 2:
        t = t.reshape(t.shape[-2], t.shape[-1])
    return t


def calculate_boundary_metrics(pred, true, threshold: float = 0.5, spacing=(1.0, 1.0)) -> Dict[str, float]:
    """:788-844 on the GPU (adp_boundary_metrics: exact EDTs of ~pred_bin / ~true_bin with the given
    sampling, skimage-style surfaces, each distance map sampled at its own surface as the reference does,
    np.percentile(95) and mean of the samples)."""
    dev = torch.device("cuda", torch.cuda.current_device())
    p, t = _dev_map(pred, dev), _dev_map(true, dev)
    if p.shape != t.shape:
        raise ValueError("calculate_boundary_metrics: prediction and mask shapes differ")
    out = (C.c_double * 2)()
    ops.call("adp_boundary_metrics", p.shape[0], p.shape[1], ops.ptr(p), ops.ptr(t), float(threshold),
             float(spacing[0]), float(spacing[1]), out, ops.stream_ptr())
    return {"hausdorff95": float(out[0]), "assd": float(out[1])}


def distance_transform_edt(mask, sampling=(1.0, 1.0)):
    """scipy.ndimage.distance_transform_edt(mask, sampling) on the GPU for a 2-D mask: distance of every
    pixel to the nearest zero of mask (device f64)."""
    dev = torch.device("cuda", torch.cuda.current_device())
    m = _dev_map(mask, dev)
    inv = (m == 0).to(torch.float32)
    out = torch.empty(m.shape, dtype=torch.float64, device=dev)
    ops.call("adp_distance_transform", m.shape[0], m.shape[1], ops.ptr(inv), 0.5, float(sampling[0]),
             float(sampling[1]), ops.ptr(out), ops.stream_ptr())
    return out


def calculate_auc_metrics(pred, true) -> Dict[str, float]:
    """:847-888 — roc_auc_score / average_precision_score of the flattened map (truth > 0.5 positive),
    computed on the GPU (adp_auc_metrics: radix sort + scans, exact pixel counts, ties grouped by score);
    NaN for a single-class mask."""
    dev = torch.device("cuda", torch.cuda.current_device())
    p = (pred if isinstance(pred, torch.Tensor) else torch.from_numpy(np.asarray(pred, np.float32)))
    t = (true if isinstance(true, torch.Tensor) else torch.from_numpy(np.asarray(true, np.float32)))
    p = p.to(dev, torch.float32).contiguous().reshape(-1)
    t = t.to(dev, torch.float32).contiguous().reshape(-1)
    if p.numel() != t.numel() or p.numel() == 0:
        raise ValueError("calculate_auc_metrics: prediction and mask sizes differ")
    out = torch.empty(2, dtype=torch.float64, device=dev)
    ops.call("adp_auc_metrics", p.numel(), ops.ptr(p), ops.ptr(t), ops.ptr(out), ops.stream_ptr())
    roc, ap = out.cpu().tolist()
    return {"roc_auc": float(roc), "pr_auc": float(ap)}


def optimize_threshold_f1_slide_level(predictions, ground_truths, tile_paths, threshold_range=None):
    """:891-939 — slide-macro F1 per threshold; all thresholds of a tile counted in one GPU pass."""
    if threshold_range is None:
        threshold_range = np.arange(0.1, 0.95, 0.05)
    print("Optimizing threshold using slide-level F1 scores...")
    thr = list(threshold_range)
    slide_of = [extract_slide_id(p) for p in tile_paths]
    per_tile = [threshold_counts(p, t, thr) for p, t in zip(predictions, ground_truths)]
    best_threshold, best_mean_f1, f1_scores = 0.5, -1.0, []
    for k, threshold in enumerate(thr):
        slide_f1 = defaultdict(list)
        for sid, c in zip(slide_of, per_tile):
            slide_f1[sid].append(_metrics_from_row(c[k])["f1_score"])
        slide_macro_f1 = np.mean([np.mean(v) for v in slide_f1.values()])
        f1_scores.append(slide_macro_f1)
        if slide_macro_f1 > best_mean_f1:
            best_mean_f1, best_threshold = slide_macro_f1, threshold
        print(f"  Threshold {threshold:.2f}: Slide-Macro F1 = {slide_macro_f1:.4f}")
    print(f"✓ Optimal threshold: {best_threshold:.2f} (Slide-Macro F1 = {best_mean_f1:.4f})")
    return best_threshold, np.array(f1_scores)


def optimize_threshold_f1(predictions, ground_truths, threshold_range=None):
    """:942-980 — tile-level mean F1 per threshold."""
    if threshold_range is None:
        threshold_range = np.arange(0.1, 0.95, 0.05)
    print("Optimizing threshold on validation set (tile-level)...")
    thr = list(threshold_range)
    per_tile = [threshold_counts(p, t, thr) for p, t in zip(predictions, ground_truths)]
    f1_scores = []
    for k, threshold in enumerate(thr):
        mean_f1 = np.mean([_metrics_from_row(c[k])["f1_score"] for c in per_tile])
        f1_scores.append(mean_f1)
        print(f"  Threshold {threshold:.2f}: F1 = {mean_f1:.4f}")
    f1_scores = np.array(f1_scores)
    i = int(np.argmax(f1_scores))
    optimal = threshold_range[i]
    print(f"✓ Optimal threshold: {optimal:.2f} (F1 = {f1_scores[i]:.4f})")
    return optimal, f1_scores


def bootstrap_confidence_interval(data, statistic_func=np.mean, n_bootstrap: int = 10000, alpha: float = 0.05,
                                  seed: int = 42):
    """:983-1009 (same RandomState stream)."""
    rng = np.random.RandomState(seed)
    n = len(data)
    stats = np.asarray([statistic_func(rng.choice(data, size=n, replace=True)) for _ in range(n_bootstrap)])
    lo, hi = np.percentile(stats, [100 * alpha / 2, 100 * (1 - alpha / 2)])
    return float(statistic_func(data)), float(lo), float(hi)


def safe_bootstrap_ci(data, func=np.mean):
    """:1012-1018"""
    valid = data[np.isfinite(data)]
    if len(valid) == 0:
        return np.nan, (np.nan, np.nan)
    point, lo, hi = bootstrap_confidence_interval(valid, func)
    return point, (lo, hi)


# ------------------------------------------------------------------------------ images / data
def read_image_gray(path: str) -> np.ndarray:
    """:1356-1383 — TIFFs keep their bit depth; RGB -> BT.601 gray."""
    from PIL import Image
    p = Path(path)
    with Image.open(p) as im:
        if p.suffix.lower() in {".tif", ".tiff"}:
            arr = np.asarray(im)
            if arr.ndim == 3 and arr.shape[-1] in (3, 4):
                arr = np.asarray(im.convert("RGB").convert("L"))
            return arr.astype(np.float32)
        return np.asarray(im.convert("L"), np.float32)


def read_mask(path: str) -> np.ndarray:
    from PIL import Image
    with Image.open(path) as im:
        m = np.asarray(im)
    return m.squeeze() if m.ndim == 3 else m


def load_validation_data(val_root: str) -> List[Tuple[str, str]]:
    """:1386-1443"""
    val_root = Path(val_root)
    images_dir, masks_dir = val_root / "images", val_root / "masks"
    if not images_dir.exists() or not masks_dir.exists():
        raise FileNotFoundError(f"Image/mask dirs not found:\n  {images_dir}\n  {masks_dir}")
    img_exts = {".jpg", ".jpeg", ".png", ".tif", ".tiff"}
    mask_exts = {".tif", ".tiff", ".png", ".jpg", ".jpeg"}
    image_files = [p for p in images_dir.rglob("*") if p.suffix.lower() in img_exts]
    mask_files = [p for p in masks_dir.rglob("*") if p.suffix.lower() in mask_exts]
    if not image_files:
        raise FileNotFoundError(f"No image files under {images_dir} (looked for {sorted(img_exts)})")
    if not mask_files:
        raise FileNotFoundError(f"No mask files under  {masks_dir} (looked for {sorted(mask_exts)})")
    by_stem: Dict[str, Path] = {}
    for m in mask_files:
        by_stem.setdefault(m.stem, m)
        if m.stem.endswith("_mask"):
            by_stem.setdefault(m.stem[:-5], m)
    paired, missing = [], 0
    for img in sorted(image_files):
        m = by_stem.get(img.stem)
        if m is not None:
            paired.append((str(img), str(m)))
        else:
            missing += 1
    if not paired:
        raise FileNotFoundError("No paired image-mask files found.\n"
                                f"Sample images: {[p.name for p in image_files[:5]]}\n"
                                f"Sample masks:  {[p.name for p in mask_files[:5]]}\n"
                                "Ensure stems match (optionally with '_mask' on masks).")
    print(f"Found {len(paired)} pairs (images: {len(image_files)}, masks: {len(mask_files)}, unpaired images: {missing})")
    return paired


# ------------------------------------------------------------------------------ post-processing
def ellipse_rows(k):
    """cv2.getStructuringElement(MORPH_ELLIPSE, (k, k)) as row extents [j1, j2) (OpenCV's construction:
    r = c = k // 2, row i spans c +- round(c * sqrt((r^2 - (i - r)^2) / r^2)), round half to even)."""
    r = c = k // 2
    inv_r2 = 1.0 / (r * r) if r else 0.0
    lo, hi = [], []
    for i in range(k):
        dy = i - r
        dx = int(np.rint(c * math.sqrt((r * r - dy * dy) * inv_r2))) if abs(dy) <= r else -1
        lo.append(max(c - dx, 0) if dx >= 0 else 0)
        hi.append(min(c + dx + 1, k) if dx >= 0 else 0)
    return lo, hi


class BoundaryRefiner:
    """full_evaluation_enhanced.py:332-393 on the GPU (adp_boundary_refine): ellipse erode / dilate -> boundary
    band, bilateral filter (d, sigma_color, sigma_space) inside the band, morphological open + close with the
    ellipse. cv2 is absent here: the restated OpenCV semantics (header of csrc/refine.hip) are checked bit for
    bit against oracle/numpy_ref.boundary_refine; parity vs cv2 itself is unpinned."""

    def __init__(self, kernel_size: int = 5, bilateral_d: int = 5, bilateral_sigma_color: float = 50,
                 bilateral_sigma_space: float = 50):
        if not 1 <= kernel_size <= 31:
            raise ValueError("kernel_size must be in 1..31")
        self.kernel_size = kernel_size
        self.bilateral_d = bilateral_d
        self.sigma_color = bilateral_sigma_color
        self.sigma_space = bilateral_sigma_space
        self.rows = ellipse_rows(kernel_size)
        lo, hi = self.rows
        self.kernel = np.zeros((kernel_size, kernel_size), np.uint8)
        for i in range(kernel_size):
            self.kernel[i, lo[i]:hi[i]] = 1

    def refine_device(self, mask):
        """mask: (H, W) probabilities (device f32 tensor or host array) -> refined (H, W) device f32 tensor."""
        import ctypes as C

        from ._lib import call, ptr, stream_ptr
        m = torch.as_tensor(mask, dtype=torch.float32)
        m = (m if m.is_cuda else m.cuda()).contiguous()
        H, W = m.shape
        work = torch.empty(4 * H * W, dtype=torch.uint8, device=m.device)
        out = torch.empty_like(m)
        lo = (C.c_int * self.kernel_size)(*self.rows[0])
        hi = (C.c_int * self.kernel_size)(*self.rows[1])
        call("adp_boundary_refine", H, W, ptr(m), self.kernel_size, lo, hi, int(self.bilateral_d),
             float(self.sigma_color), float(self.sigma_space), ptr(work), ptr(out), stream_ptr())
        return out

    def refine(self, mask, image=None):
        """Binary prediction mask [0-1] -> refined mask [0-1] (host float32, as the reference returns);
        `image` is unused, as in the reference."""
        return self.refine_device(mask).cpu().numpy()


def _add_weighted(a, wa, b, wb):
    return np.clip(np.rint(a.astype(np.float64) * wa + b.astype(np.float64) * wb), 0, 255).astype(np.uint8)


def create_4panel_visualization(original, gt_mask, pred_mask, dice_score: float, output_path: str) -> None:
    """:1021-1107 as a 2x2 PNG mosaic (matplotlib is not installed: panels without titles; the Dice value
    is in the file name as in the reference's overlay naming)."""
    from PIL import Image
    original = np.asarray(original)
    if original.ndim == 2:
        gray = original.astype(np.uint8)
        rgb = np.stack([gray] * 3, axis=-1)
    else:
        rgb = original.astype(np.uint8)
        gray = (rgb[..., 0] * 0.299 + rgb[..., 1] * 0.587 + rgb[..., 2] * 0.114).round().astype(np.uint8)
    g3 = np.stack([gray] * 3, axis=-1)
    gt = np.asarray(gt_mask) > 0
    pb = _host(pred_mask) > 0.5
    yellow = np.zeros_like(g3)
    yellow[gt] = (255, 255, 0)
    magenta = np.zeros_like(g3)
    magenta[pb] = (255, 0, 255)
    disc = np.zeros_like(g3)
    disc[gt & pb] = (0, 255, 0)
    disc[~gt & pb] = (255, 0, 0)
    disc[gt & ~pb] = (0, 0, 255)
    top = np.concatenate([rgb, _add_weighted(g3, 0.6, yellow, 0.4)], axis=1)
    bot = np.concatenate([_add_weighted(g3, 0.6, magenta, 0.4), disc], axis=1)
    Image.fromarray(np.concatenate([top, bot], axis=0)).save(output_path)


def sample_tiles(predictions, ground_truths, tile_paths, n_positive: int = 120, n_negative: int = 30):
    """:1110-1141"""
    pos = [i for i, g in enumerate(ground_truths) if np.asarray(g).sum() > 0]
    neg = [i for i, g in enumerate(ground_truths) if np.asarray(g).sum() <= 0]
    print("[Sampling] Categorizing tiles as positive/negative...")
    print(f"[Sampling] Found {len(pos)} positive and {len(neg)} negative tiles")
    if len(pos) < n_positive:
        print(f"[WARN] Only {len(pos)} positive tiles available, sampling all")
        sp = pos
    else:
        sp = np.random.choice(pos, n_positive, replace=False).tolist()
    if len(neg) < n_negative:
        print(f"[WARN] Only {len(neg)} negative tiles available, sampling all")
        sn = neg
    else:
        sn = np.random.choice(neg, n_negative, replace=False).tolist()
    idx = sp + sn
    np.random.shuffle(idx)
    return idx


def categorize_by_dice(dice_score: float) -> str:
    """:1144-1153"""
    if dice_score < 0.25:
        return "poor"
    if dice_score < 0.50:
        return "medium"
    if dice_score < 0.75:
        return "good"
    return "excellent"


# ------------------------------------------------------------------------------ pipeline
def run_publication_evaluation(val_data_root: str, weights_path: str, output_dir: str, dataset_name: str = "test",
                               optimize_threshold: bool = True, save_visualizations: bool = True,
                               n_vis_samples: int = 20, use_tta: bool = False, tta_mode: str = "basic",
                               use_sliding_window: bool = False, overlap: float = 0.5, blend_mode: str = "gaussian",
                               use_boundary_refine: bool = False, refine_kernel: int = 5,
                               adaptive_threshold: bool = False, save_overlays: bool = False, n_positive: int = 120,
                               n_negative: int = 30, *, tile_size: int = 1024, dtype: str = "f32",
                               max_batch: int = 8) -> ComprehensiveMetrics:
    """:1446-1958 (same steps, prints and output files). tile_size / dtype / max_batch: this build."""
    import pandas as pd

    from .predictor import AdiposeUNet, SlidingWindowInference

    print(f"\n{'=' * 80}\nPUBLICATION-QUALITY EVALUATION: {dataset_name.upper()} DATASET\n{'=' * 80}")
    set_deterministic_seeds(1337)
    output_dir = Path(output_dir)
    output_dir.mkdir(parents=True, exist_ok=True)
    import sys
    print(f"Environment: Python {sys.version.split()[0]}, PyTorch {torch.__version__} (HIP engine)")
    checkpoint_dir = Path(weights_path).parent
    train_mean, train_std = load_training_stats(str(checkpoint_dir))
    paired = load_validation_data(val_data_root)
    n_files = len(paired)
    print("\nBuilding model...")
    ds = _detect_deep_supervision(checkpoint_dir)
    print("🔬 Detected deep supervision architecture (train_adipose_unet_3.py)" if ds
          else "📐 Using standard architecture (train_adipose_unet_2.py)")
    model = AdiposeUNet(tile_size=tile_size, dtype=dtype, max_batch=max_batch)
    model.build_model(init_nb=44, dropout_rate=0.3, use_deep_supervision=ds)
    print("Loading trained model...")
    model.load_weights(weights_path)
    print("✓ Model loaded successfully")
    sliding = SlidingWindowInference(tile_size=tile_size, overlap=overlap, blend_mode=blend_mode) \
        if use_sliding_window else None
    if sliding is not None:
        print("✓ Sliding window inference enabled")
    refiner = BoundaryRefiner(kernel_size=refine_kernel, bilateral_d=5, bilateral_sigma_color=50,
                              bilateral_sigma_space=50) if use_boundary_refine else None
    if refiner is not None:
        print(f"✓ Boundary refinement enabled (kernel={refine_kernel})")

    print(f"\nRunning inference on {n_files} samples...")
    preds, trues, images, paths = [], [], [], []
    t0 = time.time()
    for i, (img_path, mask_path) in enumerate(paired):
        image = read_image_gray(img_path)
        true_mask = (read_mask(mask_path) > 0).astype(np.uint8)
        if sliding is not None:
            pred = sliding.predict_with_sliding_window(image, model, train_mean, train_std, use_tta=use_tta,
                                                       tta_mode=tta_mode)
        else:
            pred, _ = model.predict(image, train_mean, train_std, use_tta=use_tta, tta_mode=tta_mode)
        pred = np.asarray(pred, np.float32)
        if refiner is not None:
            pred = refiner.refine(pred, image)
        preds.append(pred)
        trues.append(true_mask)
        images.append(image)
        paths.append(img_path)
        if (i + 1) % 50 == 0:
            el = time.time() - t0
            rate = (i + 1) / el
            print(f"  Processed {i + 1}/{n_files} samples | Rate: {rate:.1f}/s | "
                  f"ETA: {(n_files - i - 1) / rate / 60 if rate > 0 else 0:.1f}min")
    print(f"✓ Inference completed in {(time.time() - t0) / 60:.1f} minutes")

    if optimize_threshold:
        print(f"\nOptimizing threshold on {dataset_name} set...")
        if adaptive_threshold:
            print("Using adaptive two-stage threshold optimization...\nStage 1: Coarse grid search...")
            coarse, _ = optimize_threshold_f1_slide_level(preds, trues, paths, np.arange(0.1, 1.0, 0.1))
            print(f"Stage 2: Fine search around {coarse:.2f}...")
            lo, hi = max(0.1, coarse - 0.1), min(0.9, coarse + 0.1)
            optimal_threshold, _ = optimize_threshold_f1_slide_level(preds, trues, paths, np.arange(lo, hi + 0.01, 0.01))
            print(f"✓ Adaptive optimization complete: {optimal_threshold:.3f}")
        else:
            optimal_threshold, _ = optimize_threshold_f1_slide_level(preds, trues, paths)
    else:
        optimal_threshold = 0.5
        print(f"Using fixed threshold: {optimal_threshold}")

    print("\nGrouping tiles by slide for slide-level analysis...")
    slides = defaultdict(list)
    for i, p in enumerate(paths):
        slides[extract_slide_id(p)].append(i)
    n_slides = len(slides)
    print(f"✓ Grouped {n_files} tiles into {n_slides} slides")
    print(f"\nCalculating slide-level metrics with threshold {optimal_threshold:.2f}...")
    keys = ["dice_scores", "jaccard_indices", "sensitivities", "specificities", "precisions", "f1_scores",
            "accuracies", "roc_aucs", "pr_aucs", "hausdorff95s", "assds"]
    sm = {k: [] for k in keys}
    for sid, idxs in slides.items():
        tm = [calculate_pixel_metrics(preds[i], trues[i], optimal_threshold) for i in idxs]
        bm = [calculate_boundary_metrics(preds[i], trues[i], optimal_threshold) for i in idxs]
        am = [calculate_auc_metrics(preds[i], trues[i]) for i in idxs]
        for k, mk in (("dice_scores", "dice_score"), ("jaccard_indices", "jaccard_index"),
                      ("sensitivities", "sensitivity"), ("specificities", "specificity"),
                      ("precisions", "precision"), ("f1_scores", "f1_score"), ("accuracies", "accuracy")):
            sm[k].append(np.mean([m[mk] for m in tm]))
        vr = [m["roc_auc"] for m in am if np.isfinite(m["roc_auc"])]
        vp = [m["pr_auc"] for m in am if np.isfinite(m["pr_auc"])]
        sm["roc_aucs"].append(np.mean(vr) if vr else np.nan)
        sm["pr_aucs"].append(np.mean(vp) if vp else np.nan)
        vh = [m["hausdorff95"] for m in bm if np.isfinite(m["hausdorff95"])]
        va = [m["assd"] for m in bm if np.isfinite(m["assd"])]
        sm["hausdorff95s"].append(np.mean(vh) if vh else np.nan)
        sm["assds"].append(np.mean(va) if va else np.nan)
    sm = {k: np.array(v) for k, v in sm.items()}
    print(f"✓ Calculated slide-level metrics for {n_slides} slides")
    print("\nCalculating bootstrap confidence intervals (n=10000)...")
    ci = {k: safe_bootstrap_ci(sm[k]) for k in keys}
    print("✓ Bootstrap confidence intervals calculated")
    res = ComprehensiveMetrics(
        dice_score=ci["dice_scores"][0], dice_ci=ci["dice_scores"][1],
        jaccard_index=ci["jaccard_indices"][0], jaccard_ci=ci["jaccard_indices"][1],
        sensitivity=ci["sensitivities"][0], sensitivity_ci=ci["sensitivities"][1],
        specificity=ci["specificities"][0], specificity_ci=ci["specificities"][1],
        precision=ci["precisions"][0], precision_ci=ci["precisions"][1],
        f1_score=ci["f1_scores"][0], f1_ci=ci["f1_scores"][1],
        accuracy=ci["accuracies"][0], accuracy_ci=ci["accuracies"][1],
        roc_auc=ci["roc_aucs"][0], roc_auc_ci=ci["roc_aucs"][1],
        pr_auc=ci["pr_aucs"][0], pr_auc_ci=ci["pr_aucs"][1],
        hausdorff95=ci["hausdorff95s"][0], hausdorff95_ci=ci["hausdorff95s"][1],
        assd=ci["assds"][0], assd_ci=ci["assds"][1],
        n_slides=n_slides, n_tiles=n_files, optimal_threshold=optimal_threshold)
    names = ["Dice Score", "Jaccard Index (IoU)", "Sensitivity (Recall)", "Specificity", "Precision", "F1 Score",
             "Accuracy", "ROC AUC", "PR AUC", "Hausdorff95", "ASSD"]
    df = pd.DataFrame({"Metric": names, "Mean": [ci[k][0] for k in keys],
                       "CI_Lower": [ci[k][1][0] for k in keys], "CI_Upper": [ci[k][1][1] for k in keys],
                       "N_Slides": [n_slides] * 11, "N_Tiles": [n_files] * 11})
    df["Mean_CI"] = df.apply(lambda r: f"{r['Mean']:.4f} [{r['CI_Lower']:.4f}, {r['CI_Upper']:.4f}]", axis=1)
    table = output_dir / f"{dataset_name}_comprehensive_results.csv"
    df.to_csv(table, index=False)
    print(f"✓ Saved results table: {table}")

    if save_overlays:
        print("\nGenerating 4-panel overlay visualizations...")
        idxs = sample_tiles(preds, trues, paths, n_positive=n_positive, n_negative=n_negative)
        od = output_dir / "overlays"
        counts = {b: 0 for b in ("poor", "medium", "good", "excellent")}
        for b in counts:
            (od / b).mkdir(parents=True, exist_ok=True)
        dices = []
        for i, idx in enumerate(idxs):
            dice = calculate_pixel_metrics(preds[idx], trues[idx], optimal_threshold)["dice_score"]
            dices.append(dice)
            b = categorize_by_dice(dice)
            counts[b] += 1
            from PIL import Image
            with Image.open(paths[idx]) as im:
                rgb = np.asarray(im.convert("RGB"))
            create_4panel_visualization(rgb, trues[idx], preds[idx], dice,
                                        str(od / b / f"{b}_{i + 1:03d}_{Path(paths[idx]).stem}_dice_{dice:.3f}.png"))
        with open(od / "summary.txt", "w") as f:
            f.write(f"OVERLAY VISUALIZATION SUMMARY: {dataset_name.upper()}\n{'=' * 80}\n\n"
                    f"Total samples: {len(idxs)}\nPositive tiles: {n_positive}\nNegative tiles: {n_negative}\n"
                    f"Threshold: {optimal_threshold:.3f}\n\n")
            if dices:
                f.write(f"DICE SCORE STATISTICS:\n{'-' * 40}\nMean Dice: {np.mean(dices):.4f}\n"
                        f"Median Dice: {np.median(dices):.4f}\nStd Dice: {np.std(dices):.4f}\n"
                        f"Min Dice: {np.min(dices):.4f}\nMax Dice: {np.max(dices):.4f}\n\n")
            f.write(f"BUCKET DISTRIBUTION:\n{'-' * 40}\n" + "".join(f"{k}: {v}\n" for k, v in counts.items()))
        print(f"✓ Saved {len(idxs)} overlay visualizations to: {od}")
    elif save_visualizations:
        n_viz = min(n_vis_samples, n_files)
        print(f"\nCreating sample visualizations (n={n_viz})...")
        vd = output_dir / "visualizations"
        vd.mkdir(exist_ok=True)
        for i, idx in enumerate(np.linspace(0, n_files - 1, n_viz, dtype=int)):
            dice = calculate_pixel_metrics(preds[idx], trues[idx], optimal_threshold)["dice_score"]
            create_4panel_visualization(images[idx], trues[idx], preds[idx], dice,
                                        str(vd / f"{dataset_name}_sample_{i + 1:02d}_{Path(paths[idx]).stem}.png"))
        print(f"✓ Saved visualizations to: {vd}")

    print(f"\n{'=' * 80}\nPUBLICATION-QUALITY RESULTS SUMMARY: {dataset_name.upper()}\n{'=' * 80}")
    print(f"Evaluation Date: {datetime.now().strftime('%Y-%m-%d %H:%M:%S')}")
    print(f"Dataset: {n_slides} slides, {n_files} tiles\nOptimal Threshold: {optimal_threshold:.3f}")
    print("Bootstrap Samples: 10,000\n")
    print(f"{'Metric':<20} {'Mean (95% CI)':<30} {'Range':<25}\n{'-' * 75}")
    for name, k in (("Dice Score", "dice_scores"), ("Jaccard (IoU)", "jaccard_indices"),
                    ("Sensitivity", "sensitivities"), ("Specificity", "specificities"), ("Precision", "precisions"),
                    ("F1 Score", "f1_scores"), ("Accuracy", "accuracies")):
        m, (lo, hi) = ci[k]
        print(f"{name:<20} {f'{m:.4f} [{lo:.4f}, {hi:.4f}]':<30} "
              f"{f'[{np.min(sm[k]):.4f}, {np.max(sm[k]):.4f}]':<25}")
    print(f"\n✓ All results saved to: {output_dir}\n✓ Results table: {table}\n{'=' * 80}\n")
    return res
