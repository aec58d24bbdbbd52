"""Training-time augmentation + normalisation on the GPU (src/utils/data.py:13-264, 398-429; the
TileDataset feed of train_adipose_unet_v3.py:568-607).

Same names, arguments and RandomState call order as the reference (``augment_pair_light / _moderate /
_heavy(image, mask, rng)``), so a seeded RandomState yields the same augmentation parameters as the
reference. The host only draws the parameters; the pixel work is done by the adp_aug_* kernels on f32
(H, W) device planes (numpy float32 evaluation order where the reference is numpy; OpenCV semantics
where it calls cv2 -- see csrc/augment.hip). Inputs may be numpy arrays or torch tensors; outputs are
float32 device tensors. The two random fields of elastic_transform and the noise of
random_gaussian_noise are drawn on the host (they consume the RandomState stream), moved to the device
and used there.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import ops
from ._lib import call, ptr, stream_ptr

DEV = "cuda"


def _dev(a):
    t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))
    if not t.is_cuda:
        t = t.to(DEV)
    return t.float().contiguous()


def gaussian_taps(sigma):
    """cv2.getGaussianKernel for ksize = round(8 sigma + 1) | 1 (f32 taps, radius)."""
    n = int(round(sigma * 4 * 2 + 1)) | 1
    x = np.arange(n, dtype=np.float64) - (n - 1) * 0.5
    t = np.exp(-0.5 / (sigma * sigma) * x * x)
    return (t / t.sum()).astype(np.float32), (n - 1) // 2


def _blur(src, sigma):
    taps, r = gaussian_taps(sigma)
    w = torch.from_numpy(taps).to(src.device)
    H, W = src.shape
    tmp, out = torch.empty_like(src), torch.empty_like(src)
    call("adp_aug_blur", 1 if src.dtype == torch.float64 else 0, H, W, ptr(src), ptr(tmp), ptr(out), ptr(w), r,
         stream_ptr())
    return out


# ------------------------------------------------------------------------ data.py:13-145 (GPU)
def random_rotation_90(image, mask, rng=np.random):
    k = rng.randint(0, 4)
    if k == 0:
        return image, mask
    return _geom(image, k, 0, 0), _geom(mask, k, 0, 0)


def _geom(x, k, flr, fud):
    H, W = x.shape
    out = torch.empty((W, H) if k & 1 else (H, W), dtype=torch.float32, device=x.device)
    call("adp_aug_geom", H, W, ptr(x), ptr(out), k, flr, fud, stream_ptr())
    return out


def random_flip(image, mask, rng=np.random):
    if rng.random() > 0.5:
        image, mask = _geom(image, 0, 1, 0), _geom(mask, 0, 1, 0)
    if rng.random() > 0.5:
        image, mask = _geom(image, 0, 0, 1), _geom(mask, 0, 0, 1)
    return image, mask


def _photo(image, mode, f, m=0.0):
    out = torch.empty_like(image)
    call("adp_aug_photometric", image.numel(), ptr(image), ptr(out), mode, float(np.float32(f)), float(m), stream_ptr())
    return out


def random_brightness(image, factor_range=(0.7, 1.3), rng=np.random):
    return _photo(image, 0, rng.uniform(*factor_range))


def random_contrast(image, factor_range=(0.7, 1.3), rng=np.random):
    s = torch.zeros(1, dtype=torch.float64, device=image.device)
    call("adp_aug_sum", image.numel(), ptr(image), ptr(s), stream_ptr())
    mean = np.float32(s.item() / image.numel())          # image.mean() (float32 result)
    return _photo(image, 1, rng.uniform(*factor_range), mean)


def random_gamma(image, gamma_range=(0.7, 1.3), rng=np.random):
    return _photo(image, 2, rng.uniform(*gamma_range))


def random_gaussian_blur(image, sigma_range=(0, 1.5), prob=0.3, rng=np.random):
    if rng.random() > prob:
        return image
    sigma = rng.uniform(*sigma_range)
    if sigma < 0.1:
        return image
    return _blur(image, sigma)


def random_gaussian_noise(image, std_range=(0, 10), prob=0.3, rng=np.random):
    if rng.random() > prob:
        return image
    std = rng.uniform(*std_range)
    noise = torch.from_numpy(rng.normal(0, std, tuple(image.shape))).to(image.device)
    out = torch.empty_like(image)
    call("adp_aug_noise", image.numel(), ptr(image), ptr(noise), ptr(out), stream_ptr())
    return out


def random_scale(image, mask, scale_range=(0.85, 1.15), prob=0.5, rng=np.random):
    if rng.random() > prob:
        return image, mask
    scale = rng.uniform(*scale_range)
    h, w = image.shape
    new_h, new_w = int(h * scale), int(w * scale)
    oi, om = torch.empty_like(image), torch.empty_like(mask)
    call("adp_aug_scale", h, w, new_h, new_w, ptr(image), ptr(oi), 0, stream_ptr())
    call("adp_aug_scale", h, w, new_h, new_w, ptr(mask), ptr(om), 1, stream_ptr())
    return oi, om


def elastic_transform(image, mask, alpha=10, sigma=3, rng=np.random):
    shape = tuple(image.shape)
    fields = []
    for _ in range(2):   # dx then dy, each GaussianBlur(rand*2-1) (f64); * alpha inside the remap kernel
        r = torch.from_numpy(rng.rand(*shape) * 2 - 1).to(image.device)
        fields.append(_blur(r, sigma))
    dx, dy = fields
    oi, om = torch.empty_like(image), torch.empty_like(mask)
    call("adp_aug_remap", shape[0], shape[1], ptr(image), ptr(mask), ptr(dx), ptr(dy), C.c_double(alpha), ptr(oi),
         ptr(om), stream_ptr())
    return oi, om


# ------------------------------------------------------------------------ pipelines (:148-262)
def augment_pair_heavy(image, mask, rng=np.random):
    image, mask = _dev(image), _dev(mask)
    image, mask = random_rotation_90(image, mask, rng)
    image, mask = random_flip(image, mask, rng)
    image, mask = random_scale(image, mask, scale_range=(0.9, 1.1), prob=0.5, rng=rng)
    if rng.random() > 0.7:
        image, mask = elastic_transform(image, mask, alpha=15, sigma=3, rng=rng)
    if rng.random() > 0.3:
        image = random_brightness(image, factor_range=(0.8, 1.2), rng=rng)
    if rng.random() > 0.3:
        image = random_contrast(image, factor_range=(0.8, 1.2), rng=rng)
    if rng.random() > 0.3:
        image = random_gamma(image, gamma_range=(0.8, 1.2), rng=rng)
    image = random_gaussian_blur(image, sigma_range=(0, 1.0), prob=0.2, rng=rng)
    image = random_gaussian_noise(image, std_range=(0, 5), prob=0.2, rng=rng)
    return image, mask


def augment_pair_moderate(image, mask, rng=np.random):
    image, mask = _dev(image), _dev(mask)
    image, mask = random_rotation_90(image, mask, rng)
    image, mask = random_flip(image, mask, rng)
    image, mask = random_scale(image, mask, scale_range=(0.95, 1.05), prob=0.3, rng=rng)
    if rng.random() > 0.85:
        image, mask = elastic_transform(image, mask, alpha=8, sigma=3, rng=rng)
    if rng.random() > 0.5:
        image = random_brightness(image, factor_range=(0.9, 1.1), rng=rng)
    if rng.random() > 0.5:
        image = random_contrast(image, factor_range=(0.9, 1.1), rng=rng)
    image = random_gaussian_blur(image, sigma_range=(0, 0.8), prob=0.15, rng=rng)
    return image, mask


def augment_pair_light(image, mask, rng=np.random):
    image, mask = _dev(image), _dev(mask)
    image, mask = random_rotation_90(image, mask, rng)
    image, mask = random_flip(image, mask, rng)
    if rng.random() > 0.7:
        image = random_brightness(image, factor_range=(0.95, 1.05), rng=rng)
    return image, mask


def augment_pair_tta_style(image, mask, rng=np.random):
    """:264-339 -- one of the 8 TTA dihedral transforms, then conservative scale / photometric / blur."""
    image, mask = _dev(image), _dev(mask)
    t = rng.randint(0, 8)
    if t >= 4:                                   # horizontal flip first, then rotate (t - 4) * 90
        image, mask = _geom(image, 0, 1, 0), _geom(mask, 0, 1, 0)
    if t % 4:
        image, mask = _geom(image, t % 4, 0, 0), _geom(mask, t % 4, 0, 0)
    if rng.random() > 0.7:
        image, mask = random_scale(image, mask, scale_range=(0.95, 1.05), prob=1.0, rng=rng)
    if rng.random() > 0.4:
        image = random_brightness(image, factor_range=(0.85, 1.15), rng=rng)
    if rng.random() > 0.4:
        image = random_contrast(image, factor_range=(0.85, 1.15), rng=rng)
    if rng.random() > 0.5:
        image = random_gamma(image, gamma_range=(0.85, 1.15), rng=rng)
    image = random_gaussian_blur(image, sigma_range=(0, 0.7), prob=0.15, rng=rng)
    return image, mask


PIPELINES = {"light": augment_pair_light, "moderate": augment_pair_moderate, "heavy": augment_pair_heavy,
             "tta-style": augment_pair_tta_style}


def select_augment_fn(level):
    """_select_augment_fn (train_adipose_unet_v3.py:1056-1067) -> (GPU pipeline or None, label)."""
    lvl = (level or "moderate").lower()
    if lvl == "light":
        return augment_pair_light, "light"
    if lvl == "heavy":
        return augment_pair_heavy, "heavy"
    if lvl in ("tta-style", "tta_style"):
        return augment_pair_tta_style, "tta-style"
    if lvl in ("none", "off", "disable"):
        return None, "none"
    return augment_pair_moderate, "moderate"

_work = {}


def normalize_percentile(image, p_low=1.0, p_high=99.0, out=None):
    """normalize_image(method='percentile') on the device (exact order statistics); returns float32."""
    image = _dev(image)
    dev = image.device
    w = _work.get(dev)
    if w is None:
        w = _work[dev] = torch.empty(64 + 4 * 2048 * 4, dtype=torch.uint8, device=dev)
    out = torch.empty_like(image) if out is None else out
    ops._check(out.numel() == image.numel() and out.dtype == torch.float32, "normalize_percentile: out")
    call("adp_percentile_normalize", image.numel(), ptr(image), ptr(out), C.c_double(p_low), C.c_double(p_high),
         ptr(w), None, stream_ptr())
    return out


def normalize_zscore(image, mean, std):
    """(image - mean) / (std + 1e-10) in float32 (TileDataset zscore, train_adipose_unet_v3.py:589-590)."""
    image = _dev(image)
    return _photo_raw(image, 3, np.float32(std + 1e-10), np.float32(mean))


def _photo_raw(image, mode, f, m):
    out = torch.empty_like(image)
    call("adp_aug_photometric", image.numel(), ptr(image), ptr(out), mode, float(f), float(m), stream_ptr())
    return out
