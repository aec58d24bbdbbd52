"""Host-side data feed: synthetic histology tiles, the reference's on-disk tile format, and the
reference's normalisations.

  * TileDataset (train_adipose_unet_v3.py:510-623): pairs <stem>.jpg images with <stem>.tif masks,
    grayscale decode (cv2.IMREAD_GRAYSCALE equivalent), optional augmentation, per-tile percentile
    normalisation (default, :591-593) or dataset z-score (:589-590); the last batch is padded by
    repeating its last tile (:600-602).
  * compute_mean_std (:1125-1133) for normalization_stats.json.
  * synthetic tiles (seed 865 from seed.csv): blurred-noise background (mean ~201,
    std ~25) with adipocyte-like ellipses (bright lumen, dark rim); mask = ellipse interiors.

cv2/tifffile are not available on this image: JPEG decoding uses PIL (ITU-R 601 luma, the same
weights cv2 uses for IMREAD_GRAYSCALE); masks use PIL-readable TIFF.
"""
from __future__ import annotations

import os
from pathlib import Path

import numpy as np

SEED = 865


def load_seed(path=None):
    """src/utils/seed_utils.py: first integer of seed.csv (865)."""
    if path and os.path.exists(path):
        with open(path) as f:
            for tok in f.read().replace(",", " ").split():
                if tok.strip().lstrip("-").isdigit():
                    return int(tok)
    return SEED


# ------------------------------------------------------------------------------ synthetic data
def synthetic_tile(rng, size=1024, channels=3, n_cells=None):
    """One uint8 histology-like tile (H,W,C) and its {0,1} float32 mask (H,W)."""
    from scipy import ndimage

    h = w = size
    noise = rng.normal(0.0, 1.0, (h // 4 + 2, w // 4 + 2)).astype(np.float32)
    bg = ndimage.gaussian_filter(noise, 2.0)
    bg = ndimage.zoom(bg, 4, order=1)[:h, :w]
    bg = 201.0 + 25.0 * bg / (bg.std() + 1e-6)
    mask = np.zeros((h, w), np.float32)
    yy, xx = np.mgrid[0:h, 0:w]
    n_cells = n_cells or rng.integers(max(4, size // 128), max(8, size // 48))
    img = bg.copy()
    for _ in range(int(n_cells)):
        cy, cx = rng.uniform(0, h), rng.uniform(0, w)
        ry, rx = rng.uniform(0.03, 0.09) * size, rng.uniform(0.03, 0.09) * size
        th = rng.uniform(0, np.pi)
        c, s = np.cos(th), np.sin(th)
        y0, y1 = int(max(0, cy - 1.2 * max(ry, rx))), int(min(h, cy + 1.2 * max(ry, rx) + 1))
        x0, x1 = int(max(0, cx - 1.2 * max(ry, rx))), int(min(w, cx + 1.2 * max(ry, rx) + 1))
        if y1 <= y0 or x1 <= x0:
            continue
        dy, dx = yy[y0:y1, x0:x1] - cy, xx[y0:y1, x0:x1] - cx
        r = ((dy * c + dx * s) / ry) ** 2 + ((-dy * s + dx * c) / rx) ** 2
        inside = r < 1.0
        rim = (r >= 1.0) & (r < 1.35)
        mask[y0:y1, x0:x1][inside] = 1.0
        img[y0:y1, x0:x1][inside] = 235.0 + 8.0 * rng.normal(size=int(inside.sum()))
        img[y0:y1, x0:x1][rim] = 120.0 + 15.0 * rng.normal(size=int(rim.sum()))
    img = np.clip(img, 0, 255)
    if channels == 1:
        return img.astype(np.uint8), mask
    tint = np.array([1.0, 0.86, 0.93], np.float32)[:channels]
    rgb = np.clip(img[..., None] * tint + rng.normal(0, 3, (h, w, channels)), 0, 255)
    return rgb.astype(np.uint8), mask


def synthetic_batch(n, size, channels=3, seed=SEED):
    rng = np.random.default_rng(seed)
    xs, ys = zip(*(synthetic_tile(rng, size, channels) for _ in range(n)))
    return np.stack(xs), np.stack(ys)


def _smooth_field(gen, size, cells, device):
    """A smooth random field in [-1, 1]-ish: a (cells+1)^2 grid of N(0,1) draws, bicubically upsampled."""
    import torch
    import torch.nn.functional as F

    g = torch.randn(1, 1, cells + 1, cells + 1, generator=gen).to(device)
    return F.interpolate(g, size=(size, size), mode="bicubic", align_corners=True)[0, 0]


def synthetic_tile_hard(gen, size=1024, channels=3, device="cpu"):
    """A harder synthetic histology tile than synthetic_tile (whose ellipse task saturates at Dice 0.998):
    packed, touching adipocytes -- a power diagram of ~300-900 cells per 1024^2 whose neighbours share 1-3 px
    membranes, many of them torn -- beside stroma regions (textured, with nuclei), bright NON-fat distractors
    (vessel-like lumens, a fifth of the non-stroma cells, whose walls are only ~1 px thicker than a membrane) and
    stain noise (per-tile H&E tint, low-frequency illumination, a sigma 0.8-2 blur, pixel noise). The mask is the fat-cell interiors (a torn membrane between two fat cells counts
    as fat). Random draws come from the CPU torch.Generator `gen` (reproducible per seed); the arithmetic runs
    on `device` (a 1024^2 tile takes milliseconds on the GPU). Returns (uint8 (S,S,C), float32 {0,1} (S,S))."""
    import torch
    import torch.nn.functional as F

    S = size
    sc = S / 1024.0
    u = lambda a, b, n=(): (a + (b - a) * torch.rand(n, generator=gen)).to(device)   # noqa: E731
    n = max(8, int((300 + 600 * torch.rand((), generator=gen).item()) * sc * sc))
    seeds = u(-0.04 * S, 1.04 * S, (n, 2))
    spacing = S / (n ** 0.5)
    rad = u(0.0, 0.45 * spacing, (n,))            # additive power weights: cell-size variation
    # cell kinds from a smooth tissue field: stroma (~25 %), distractor lumens (~6 %), fat (the rest)
    tissue = _smooth_field(gen, S, 4, device)
    sy = seeds[:, 0].clamp(0, S - 1).long()
    sx = seeds[:, 1].clamp(0, S - 1).long()
    tv = tissue[sy, sx]
    stroma = tv < torch.quantile(tissue.flatten()[:: max(1, S * S // 65536)], 0.3)
    lumen = (~stroma) & (u(0, 1, (n,)) < 0.2)
    fat = ~(stroma | lumen)
    # nearest two cells of every pixel (power distance), in row chunks
    ys = torch.arange(S, device=device, dtype=torch.float32)
    xs = torch.arange(S, device=device, dtype=torch.float32)
    i1 = torch.empty(S, S, dtype=torch.long, device=device)
    i2 = torch.empty(S, S, dtype=torch.long, device=device)
    bis = torch.empty(S, S, device=device)       # distance to the bisector of the two nearest cells
    rows = max(1, (1 << 22) // (S * n))
    for y0 in range(0, S, rows):
        yy = ys[y0:y0 + rows, None, None]
        d = (yy - seeds[:, 0]) ** 2 + (xs[None, :, None] - seeds[:, 1]) ** 2 - rad ** 2
        dv, di = torch.topk(d, 2, dim=2, largest=False)
        s1, s2 = seeds[di[..., 0]], seeds[di[..., 1]]
        i1[y0:y0 + rows] = di[..., 0]
        bis[y0:y0 + rows] = (dv[..., 1] - dv[..., 0]) / (2.0 * (s1 - s2).norm(dim=-1) + 1e-6)
        i2[y0:y0 + rows] = di[..., 1]   # (second-nearest cell: the torn-membrane rule)
    half = float(u(0.5, 1.5))                      # membrane half-width (px)
    wall = torch.where(lumen[i1], 2.0 + float(u(0, 1)), half)   # (lumen walls: only ~1 px thicker)
    torn = _smooth_field(gen, S, int(8 * max(1.0, sc)), device) > 0.7
    memb = (bis < wall) & ~(torn & fat[i1] & fat[i2]) & ~(stroma[i1] & stroma[i2])   # (stroma: no membranes)
    mask = (fat[i1] & ~memb).float()
    # intensities (gray, before the tint)
    noise = lambda s: torch.randn(S, S, generator=gen).to(device) * s   # noqa: E731
    img = torch.full((S, S), 232.0, device=device) + noise(6.0) + 6.0 * _smooth_field(gen, S, 12, device)
    img = torch.where(lumen[i1], 228.0 + noise(8.0), img)
    tex = _smooth_field(gen, S, int(48 * max(1.0, sc)), device)
    img = torch.where(stroma[i1], 188.0 + 24.0 * tex + noise(14.0), img)
    img = torch.where(memb, float(u(140.0, 190.0)) + noise(18.0), img)
    # nuclei: dark dots in the stroma and on some membranes
    nn_ = int(400 * sc * sc)
    ny, nx, nr = u(0, S, (nn_,)), u(0, S, (nn_,)), u(1.5, 4.0, (nn_,))
    yi, xi = ny.long().clamp(0, S - 1), nx.long().clamp(0, S - 1)
    ok = stroma[i1[yi, xi]] | (bis[yi, xi] < 3.0)
    ny, nx, nr = ny[ok], nx[ok], nr[ok]
    nuc = torch.zeros(S, S, dtype=torch.bool, device=device)
    if len(ny):
        rows = max(1, (1 << 22) // (S * len(ny)))
        for y0 in range(0, S, rows):
            d = (ys[y0:y0 + rows, None, None] - ny) ** 2 + (xs[None, :, None] - nx) ** 2 - nr ** 2
            nuc[y0:y0 + rows] = (d < 0).any(dim=2)
    img = torch.where(nuc, 85.0 + noise(12.0), img)
    # blur, illumination, stain tint, pixel noise
    sig = float(u(0.8, 2.0))
    k = torch.arange(-4, 5, device=device, dtype=torch.float32)
    k = torch.exp(-k * k / (2 * sig * sig))
    k = k / k.sum()
    im = F.conv2d(F.pad(img[None, None], (4, 4, 0, 0), mode="replicate"), k.view(1, 1, 1, 9))
    im = F.conv2d(F.pad(im, (0, 0, 4, 4), mode="replicate"), k.view(1, 1, 9, 1))[0, 0]
    im = im * (1.0 + 0.08 * _smooth_field(gen, S, 3, device))
    base = torch.tensor([1.0, 0.86, 0.93], device=device)[:channels]
    tint = base * (1.0 + u(-0.07, 0.07, (channels,)))
    pink = torch.tensor([1.04, 0.90, 0.97], device=device)[:channels]
    rgb = im[..., None] * torch.where(stroma[i1][..., None], tint * pink, tint)
    rgb = rgb + torch.randn(S, S, channels, generator=gen).to(device) * 7.0
    return rgb.clamp(0, 255).to(torch.uint8), mask


def synthetic_stream_hard(seed, n, size, channels=3, device="cpu"):
    """n tiles of synthetic_tile_hard from one seeded generator: (uint8 (n,S,S,C), float32 (n,S,S))."""
    import torch

    gen = torch.Generator().manual_seed(int(seed))
    xs, ys = zip(*(synthetic_tile_hard(gen, size, channels, device) for _ in range(n)))
    return torch.stack(xs), torch.stack(ys)


def to_gray(rgb):
    """cv2.COLOR_RGB2GRAY / IMREAD_GRAYSCALE weights (ITU-R BT.601)."""
    rgb = np.asarray(rgb, np.float32)
    return rgb[..., 0] * 0.299 + rgb[..., 1] * 0.587 + rgb[..., 2] * 0.114


# ------------------------------------------------------------------------------ normalisation
def normalize_image(image, method="percentile", p_low=1, p_high=99, mean=None, std=None):
    """src/utils/data.py:398-429"""
    if method == "percentile":
        plow, phigh = np.percentile(image, (p_low, p_high))
        scale = max(phigh - plow, 1e-3)
        return np.clip((image - plow) / scale, 0, 1)
    if method == "minmax":
        imin, imax = image.min(), image.max()
        return (image - imin) / max(imax - imin, 1e-3)
    if method == "zscore":
        return (image - image.mean()) / (image.std() + 1e-10)
    if method == "zscore_dataset":
        if mean is None or std is None:
            raise ValueError("Dataset mean and std required for zscore_dataset method")
        return (image - mean) / (std + 1e-10)
    raise ValueError(f"Unknown normalization method: {method}")


# ------------------------------------------------------------------------------ file format
def read_gray(path):
    """cv2.imread(path, IMREAD_GRAYSCALE) equivalent -> float32."""
    from PIL import Image

    with Image.open(path) as im:
        if im.mode in ("I;16", "I;16B", "I", "F"):
            return np.asarray(im, np.float32)
        return np.asarray(im.convert("L"), np.float32)


def read_mask(path):
    from PIL import Image

    with Image.open(path) as im:
        m = np.asarray(im).astype(np.float32)
    return m.squeeze() if m.ndim == 3 else m


def write_mask(path, arr):
    from PIL import Image

    Image.fromarray(np.asarray(arr)).save(path)


def compute_mean_std(image_paths, max_n=None):
    """train_adipose_unet_v3.py:1125-1133 (float64 accumulate over all pixels)."""
    s, s2, n = 0.0, 0.0, 0
    for i, p in enumerate(image_paths):
        if max_n and i >= max_n:
            break
        v = read_gray(p).astype(np.float64).reshape(-1)
        s += v.sum()
        s2 += (v * v).sum()
        n += v.size
    mean = s / n
    return float(mean), float(np.sqrt(max(s2 / n - mean * mean, 0.0)) + 1e-10)


class TileDataset:
    """train_adipose_unet_v3.py:510-623 (generator semantics; batches are numpy float32)."""

    def __init__(self, images_dir, masks_dir, batch_size, augment=True, cache_size=100, mean=None, std=None,
                 normalization_method="zscore", percentile_low=1.0, percentile_high=99.0, augment_fn=None,
                 augment_level="moderate", seed=None, device=None):
        self.images_dir, self.masks_dir = Path(images_dir), Path(masks_dir)
        self.batch_size = batch_size
        self.augment, self.augment_fn = augment, augment_fn
        self.cache_size = cache_size
        self.mean, self.std = mean, std
        self.normalization_method = normalization_method
        self.percentile_low, self.percentile_high = percentile_low, percentile_high
        image_files = sorted(self.images_dir.glob("*.jpg"))
        mask_files = {p.stem: p for p in self.masks_dir.glob("*.tif")}
        self.pairs = [(p, mask_files[p.stem]) for p in image_files if p.stem in mask_files]
        self.cache = {}
        self.seed = seed
        # device feed: augmentation (adipose_amd.augment pipelines) and normalisation run on the GPU and
        # batches are device tensors; the host only decodes tiles and draws the random parameters
        self.device = device

    def __len__(self):
        return len(self.pairs)

    def load_pair(self, img_path, mask_path):
        key = img_path.stem
        if key in self.cache:
            return self.cache[key]
        img = read_gray(img_path)
        mask = read_mask(mask_path)
        if len(self.cache) < self.cache_size:
            self.cache[key] = (img.copy(), mask.copy())
        return img, mask

    def _norm_dev(self, img):
        from . import augment as GA
        if self.normalization_method == "zscore":
            return GA.normalize_zscore(img, self.mean, self.std)
        if self.normalization_method == "percentile":
            return GA.normalize_percentile(img, self.percentile_low, self.percentile_high)
        raise ValueError(f"Unknown normalization method: {self.normalization_method}")

    def _norm(self, img):
        if self.normalization_method == "zscore":
            return (img - self.mean) / (self.std + 1e-10)
        if self.normalization_method == "percentile":
            return normalize_image(img, "percentile", self.percentile_low, self.percentile_high)
        raise ValueError(f"Unknown normalization method: {self.normalization_method}")

    def generator(self, shard=0, num_shards=1):
        """Endless batches; with num_shards>1 each DP rank reads a disjoint slice of each epoch order."""
        rng = np.random.RandomState(self.seed)
        idx = np.arange(len(self.pairs))
        while True:
            rng.shuffle(idx)
            mine = idx[shard::num_shards]
            for i in range(0, len(mine), self.batch_size):
                imgs, masks = [], []
                for j in mine[i:i + self.batch_size]:
                    img, mask = self.load_pair(*self.pairs[j])
                    if self.device is not None:
                        from .augment import _dev
                        img, mask = _dev(img), _dev(mask)
                    if self.augment and self.augment_fn is not None:
                        img, mask = self.augment_fn(img, mask, rng)
                    imgs.append(self._norm_dev(img) if self.device is not None else self._norm(img))
                    masks.append(mask)
                while len(imgs) < self.batch_size:
                    imgs.append(imgs[-1])
                    masks.append(masks[-1])
                if self.device is not None:
                    import torch
                    yield torch.stack(imgs), torch.stack(masks)
                else:
                    yield np.array(imgs, np.float32), np.array(masks, np.float32)


def write_synthetic_build(root, n_train=8, n_val=4, size=1024, seed=SEED):
    """Materialise a reference-format build directory (dataset/{train,val}/{images,masks}) with
    synthetic tiles named like build_dataset.py's '{base}_r{r}_c{c}.jpg' (:1531-1532)."""
    from PIL import Image

    rng = np.random.default_rng(seed)
    root = Path(root)
    for split, n in (("train", n_train), ("val", n_val)):
        (root / "dataset" / split / "images").mkdir(parents=True, exist_ok=True)
        (root / "dataset" / split / "masks").mkdir(parents=True, exist_ok=True)
        for i in range(n):
            img, mask = synthetic_tile(rng, size, 3)
            stem = f"synthetic_slide{i // 4}_r{i % 2}_c{(i // 2) % 2}"
            Image.fromarray(img).save(root / "dataset" / split / "images" / f"{stem}.jpg", quality=100)
            Image.fromarray(mask.astype(np.uint8)).save(root / "dataset" / split / "masks" / f"{stem}.tif")
    return root
