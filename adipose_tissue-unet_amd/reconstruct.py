"""Full-slide reconstruction from pre-tiled overlapping tiles (Segmentation/reconstruct_full_images.py).

Same functions, arguments, return values and output tree as the reference:
  * parse_tile_filename / group_tiles_by_slide / get_source_image_dimensions /
    infer_full_image_dimensions / get_full_image_dimensions / find_missing_tiles /
    create_expected_grid                                          reconstruct_full_images.py:114-327
  * reconstruct_slide                                             :334-417
  * create_overlay / create_4panel_comparison                     :424-537
  * create_reconstruction_log                                     :544-579
  * reconstruct_all_slides                                        :586-866  (CLI: cli/reconstruct_full_images.py)

MI355X-first differences (same results): tile images are decoded on the host, uploaded once and run
through the HIP engine in batches of tiles x TTA views (one forward per batch; the reference runs one
Keras predict per tile and view); the prediction, ground-truth and the three RGB planes are blended
on the GPU (adp_blend_accum / adp_blend_finalize, the GaussianBlender / LinearBlender arithmetic of
full_evaluation_enhanced.py:115-204 in f32, tile by tile in the reference's order). With a
torch.distributed process group the tiles are split into contiguous runs per rank and the blend
accumulators are SUM-reduced (RCCL) before the division. Files: cv2 / tifffile are absent, so tiles
and masks are read with PIL (BT.601 grayscale, the weights cv2.IMREAD_GRAYSCALE uses) and the TIFF
outputs are written by PIL with LZW compression.
"""
from __future__ import annotations

import json
import math
import warnings
from collections import defaultdict
from datetime import datetime
from pathlib import Path
from typing import Dict, List, Optional, Set, Tuple

import numpy as np
import torch

from . import ops
from .evaluation import (BoundaryRefiner, _add_weighted, calculate_pixel_metrics, load_training_stats,
                         set_deterministic_seeds)
from .predictor import (TTA_VIEWS, AdiposeUNet, BandCanvas, GaussianBlender, LinearBlender, TestTimeAugmentation,
                        band_rows)

__all__ = ["parse_tile_filename", "group_tiles_by_slide", "get_source_image_dimensions",
           "infer_full_image_dimensions", "get_full_image_dimensions", "find_missing_tiles",
           "create_expected_grid", "reconstruct_slide", "create_overlay", "create_4panel_comparison",
           "create_reconstruction_log", "reconstruct_all_slides"]


# ------------------------------------------------------------------------------ tile grid
def parse_tile_filename(filename: str) -> Tuple[str, int, int]:
    """:114-146 — "<slide>_r<row>_c<col>.<ext>" -> (slide, row, col); ValueError otherwise."""
    parts = Path(filename).stem.split("_")
    if len(parts) >= 2 and parts[-2].startswith("r") and parts[-1].startswith("c"):
        try:
            return "_".join(parts[:-2]), int(parts[-2][1:]), int(parts[-1][1:])
        except (ValueError, IndexError):
            pass
    raise ValueError(f"Cannot parse tile position from filename: {filename}")


def group_tiles_by_slide(images_dir: Path, masks_dir: Optional[Path] = None) -> Dict[str, Dict]:
    """:149-201 — sorted *.jpg tiles grouped by slide; masks (*.tif) matched by stem."""
    slides = defaultdict(lambda: {"tiles": [], "positions": set()})
    masks = {}
    if masks_dir and Path(masks_dir).exists():
        masks = {p.stem: p for p in Path(masks_dir).glob("*.tif")}
    for img in sorted(Path(images_dir).glob("*.jpg")):
        try:
            sid, r, c = parse_tile_filename(img.name)
        except ValueError as e:
            warnings.warn(f"Skipping file {img.name}: {e}")
            continue
        slides[sid]["tiles"].append((r, c, img, masks.get(img.stem)))
        slides[sid]["positions"].add((r, c))
    for info in slides.values():
        if info["positions"]:
            rows = [r for r, _ in info["positions"]]
            cols = [c for _, c in info["positions"]]
            info["row_range"] = (min(rows), max(rows))
            info["col_range"] = (min(cols), max(cols))
    return dict(slides)


def get_source_image_dimensions(slide_id: str, data_root: Optional[str] = None) -> Optional[Tuple[int, int]]:
    """:204-237 — (H, W) of ~/Data_for_ML/Meat_Luci_Tulane/Pseudocolored/**/<slide>.jpg, else None."""
    base = Path.home() / "Data_for_ML" / "Meat_Luci_Tulane" / "Pseudocolored"
    matches = list(base.rglob(f"{slide_id}.jpg")) if base.exists() else []
    if not matches:
        return None
    print(f"  ✓ Found source image: {matches[0]}")
    try:
        from PIL import Image
        with Image.open(matches[0]) as im:
            w, h = im.size
        return (h, w)
    except Exception as e:  # noqa: BLE001 (the reference warns and falls back)
        warnings.warn(f"Failed to load source image {matches[0]}: {e}")
        return None


def infer_full_image_dimensions(tile_positions: Set[Tuple[int, int]], tile_size: int,
                                stride: int) -> Tuple[int, int]:
    """:240-271"""
    if not tile_positions:
        return (0, 0)
    return (max(r for r, _ in tile_positions) * stride + tile_size,
            max(c for _, c in tile_positions) * stride + tile_size)


def get_full_image_dimensions(slide_id: str, tile_positions: Set[Tuple[int, int]], tile_size: int, stride: int,
                              data_root: Optional[str] = None) -> Tuple[int, int]:
    """:274-298"""
    dims = get_source_image_dimensions(slide_id, data_root)
    if dims is not None:
        print(f"  ✓ Using actual source image dimensions: {dims[1]}x{dims[0]}")
        return dims
    print("  ⚠️  Source image not found, inferring dimensions from tiles")
    return infer_full_image_dimensions(tile_positions, tile_size, stride)


def find_missing_tiles(expected_positions: Set[Tuple[int, int]],
                       found_positions: Set[Tuple[int, int]]) -> Set[Tuple[int, int]]:
    """:301-313"""
    return expected_positions - found_positions


def create_expected_grid(row_range: Tuple[int, int], col_range: Tuple[int, int]) -> Set[Tuple[int, int]]:
    """:316-327"""
    return {(r, c) for r in range(row_range[0], row_range[1] + 1) for c in range(col_range[0], col_range[1] + 1)}


# ------------------------------------------------------------------------------ reconstruction
def _read_tile(path):
    """cv2.imread(IMREAD_GRAYSCALE) -> f32 gray and cv2.imread(IMREAD_COLOR) + BGR2RGB -> uint8 RGB."""
    from PIL import Image
    with Image.open(path) as im:
        rgb = np.asarray(im.convert("RGB"))
        gray = np.asarray(im.convert("L"), np.float32)
    return gray, rgb


def _read_gt(path):
    """:386-393 — squeeze, /255 only when the mask is not already in [0, 1]."""
    from PIL import Image
    with Image.open(path) as im:
        g = np.asarray(im).astype(np.float32)
    if g.ndim == 3:
        g = g.squeeze()
    if g.max() > 1.0:
        g = g / 255.0
    return g


class _Canvas:
    """Device blend accumulators of one output plane (GaussianBlender / LinearBlender.reconstruct), held as a row
    band (predictor.BandCanvas): with a process group, rank 0 holds the frame and the other ranks the band of their
    tiles, added into rank 0's frame by result()."""

    def __init__(self, blender, shape, dev, bands=None, rank=0):
        self.blender, self.dev, self.bands = blender, dev, bands
        self.c = BandCanvas(shape, (0, shape[0]) if bands is None else bands[rank], dev)

    def add(self, tile, y, x):
        T = tile.shape[-1]
        if tile.shape[-2] != T:
            raise ValueError("blend tiles must be square")
        self.c.add(tile, self.blender.device_weights(self.dev, T, T), y, x)

    def result(self, group=None):
        """The blended plane (on rank 0 with a process group; None on the other ranks)."""
        if group is not None and not self.c.reduce_to_root(group, self.bands):
            return None
        return self.c.finalize(self.blender.floor)


def _shard(items, group, rank=None):
    if group is None:
        return 0, len(items)
    import torch.distributed as dist
    r, n = dist.get_rank(group) if rank is None else rank, dist.get_world_size(group)
    per = math.ceil(len(items) / n)
    return min(r * per, len(items)), min((r + 1) * per, len(items))


def reconstruct_slide(model, tiles_info: List[Tuple], full_shape: Tuple[int, int], tile_size: int, stride: int,
                      mean: float, std: float, blender, boundary_refiner: Optional[BoundaryRefiner] = None,
                      use_tta: bool = False, tta_mode: str = "basic", process_group=None,
                      return_device: bool = False):
    """:334-417 -> (full_image_rgb (H,W,3), full_pred (H,W), full_gt (H,W) or None), f32 in [0, 1].

    Tile k sits at (min(row*stride, H-T), min(col*stride, W-T)). As in the reference, the GT tiles
    are blended against the first len(gt_tiles) positions (zip), so a slide with some masks missing
    pairs them with the leading positions. ``model`` is any predictor with predict_single (the
    reference's duck type); HIP predictors (predict_views) run tiles x TTA views batched."""
    dev = torch.device("cuda", torch.cuda.current_device())
    H, W = int(full_shape[0]), int(full_shape[1])
    positions = [(min(r * stride, H - tile_size), min(c * stride, W - tile_size)) for r, c, _, _ in tiles_info]
    views = TTA_VIEWS[(tta_mode or "basic").lower() if (tta_mode or "basic").lower() in TTA_VIEWS else "basic"] \
        if use_tta else [0]
    lo, hi = _shard(tiles_info, process_group)
    # GT tiles pair with positions in order of appearance (zip over the GT list)
    gt_rank = []
    n_gt = 0
    for _, _, _, m in tiles_info:
        gt_rank.append(n_gt if m is not None else -1)
        n_gt += m is not None
    # row bands of every rank (rank 0: the frame): its tiles' rows, and the rows of the positions its GT tiles go to
    bands = gt_bands = None
    rank = 0
    if process_group is not None:
        import torch.distributed as dist
        rank, n = dist.get_rank(process_group), dist.get_world_size(process_group)
        bands, gt_bands = [(0, H)], [(0, H)]
        for q in range(1, n):
            a, b = _shard(tiles_info, process_group, q)
            bands.append(band_rows(positions[a:b], tile_size))
            gt_bands.append(band_rows([positions[gt_rank[i]] for i in range(a, b) if gt_rank[i] >= 0], tile_size))
    pred_c = _Canvas(blender, (H, W), dev, bands, rank)
    rgb_c = [_Canvas(blender, (H, W), dev, bands, rank) for _ in range(3)]
    gt_c = _Canvas(blender, (H, W), dev, gt_bands, rank)
    batched = hasattr(model, "predict_views")
    per = max(1, getattr(model, "max_batch", 8) // len(views)) if batched else 1
    for i0 in range(lo, hi, per):
        idx = list(range(i0, min(i0 + per, hi)))
        grays, rgbs = zip(*(_read_tile(tiles_info[i][2]) for i in idx))
        if batched:
            g_dev = [torch.from_numpy(g).to(dev) for g in grays]
            probs = model.predict_views(g_dev, mean, std, views)
        elif use_tta:
            tta = TestTimeAugmentation(mode=tta_mode)
            probs = [tta.predict_with_tta(model, g, mean, std) for g in grays]
        else:
            probs = [model.predict_single(g, mean, std) for g in grays]
        for k, i in enumerate(idx):
            p = probs[k]
            if boundary_refiner is not None:
                p = boundary_refiner.refine(p.cpu().numpy() if isinstance(p, torch.Tensor) else p, grays[k])
            if not isinstance(p, torch.Tensor):
                p = torch.from_numpy(np.ascontiguousarray(p, dtype=np.float32)).to(dev)
            y, x = positions[i]
            pred_c.add(p, y, x)
            rgb = torch.from_numpy(np.array(rgbs[k], copy=True)).to(dev).float() / 255.0
            for ch in range(3):
                rgb_c[ch].add(rgb[..., ch].contiguous(), y, x)
            m = tiles_info[i][3]
            if m is not None:
                gy, gx = positions[gt_rank[i]]
                gt_c.add(torch.from_numpy(np.ascontiguousarray(_read_gt(m), dtype=np.float32)).to(dev), gy, gx)
    full_pred = pred_c.result(process_group)
    rgbs_ = [c.result(process_group) for c in rgb_c]
    full_gt = gt_c.result(process_group) if n_gt else None
    if full_pred is None:   # (a rank > 0: the planes live on rank 0)
        return None, None, None
    full_rgb = torch.stack(rgbs_, dim=-1)
    if return_device:
        return full_rgb, full_pred, full_gt
    return (full_rgb.cpu().numpy(), full_pred.cpu().numpy(), None if full_gt is None else full_gt.cpu().numpy())


# ------------------------------------------------------------------------------ visualisation
def create_overlay(image_rgb: np.ndarray, mask: np.ndarray, color: Tuple[int, int, int] = (255, 0, 255),
                   alpha: float = 0.4) -> np.ndarray:
    """:424-453 — uint8 RGB; cv2.addWeighted(img, 0.6, colour_mask, 0.4, 0) with saturate-rounding
    (alpha is unused by the reference's blend, which is fixed at 0.6 / 0.4)."""
    image_rgb = np.asarray(image_rgb)
    img = (image_rgb * 255).astype(np.uint8) if image_rgb.max() <= 1.0 else image_rgb.astype(np.uint8)
    cm = np.zeros_like(img)
    cm[np.asarray(mask) > 0.5] = color
    return _add_weighted(img, 0.6, cm, 0.4)


def create_4panel_comparison(original_rgb: np.ndarray, gt_mask: np.ndarray, pred_mask: np.ndarray, slide_id: str,
                             dice_score: float) -> np.ndarray:
    """:456-537 — original | GT overlay (yellow) / prediction overlay (magenta) | discrepancy
    (TP green, FP red, FN blue) as one uint8 RGB mosaic (panel titles are not rendered)."""
    o = np.asarray(original_rgb)
    orig = (o * 255).astype(np.uint8) if o.max() <= 1.0 else o.astype(np.uint8)
    g = np.asarray(gt_mask) > 0.5
    p = np.asarray(pred_mask) > 0.5
    disc = np.zeros(g.shape + (3,), np.uint8)
    disc[g & p] = (0, 255, 0)
    disc[~g & p] = (255, 0, 0)
    disc[g & ~p] = (0, 0, 255)
    top = np.concatenate([orig, create_overlay(original_rgb, gt_mask, (255, 255, 0))], axis=1)
    bot = np.concatenate([create_overlay(original_rgb, pred_mask, (255, 0, 255)), disc], axis=1)
    return np.concatenate([top, bot], axis=0)


def _save_tiff(path, arr):
    from PIL import Image
    Image.fromarray(arr).save(str(path), compression="tiff_lzw")


def _save_png(path, arr):
    from PIL import Image
    Image.fromarray(arr).save(str(path))


# ------------------------------------------------------------------------------ log + driver
def create_reconstruction_log(args, output_dir: Path, slide_results: List[Dict]) -> Path:
    """:544-579"""
    log = {
        "reconstruction_info": {"timestamp": datetime.now().isoformat(),
                                "script_version": "Full Image Reconstruction v1.0",
                                "output_directory": str(output_dir)},
        "configuration": {"weights_path": args.weights, "data_root": args.data_root, "tile_size": args.tile_size,
                          "stride": args.stride, "threshold": args.threshold, "blend_mode": args.blend_mode,
                          "use_tta": args.use_tta, "tta_mode": args.tta_mode if args.use_tta else None,
                          "boundary_refine": args.boundary_refine,
                          "refine_kernel": args.refine_kernel if args.boundary_refine else None},
        "slides_processed": len(slide_results),
        "slide_results": slide_results,
        "summary_statistics": {
            "mean_dice": float(np.mean([r["metrics"]["dice_score"] for r in slide_results]))
            if all(r["metrics"] for r in slide_results) else None,
            "mean_coverage": float(np.mean([r["reconstruction"]["coverage_ratio"] for r in slide_results])),
            "total_tiles_used": sum(r["reconstruction"]["tiles_used"] for r in slide_results),
            "total_tiles_missing": sum(r["reconstruction"]["tiles_missing"] for r in slide_results)},
    }
    path = Path(output_dir) / "reconstruction_log.json"
    path.write_text(json.dumps(log, indent=2, default=float))
    return path


def reconstruct_all_slides(args, model=None, process_group=None):
    """:586-866 — per slide: coverage check, dimensions, reconstruction, TIFF / PNG / metrics outputs.
    ``model`` overrides building AdiposeUNet from args.weights (tests, custom predictors)."""
    print(f"\n{'=' * 80}\nFULL IMAGE RECONSTRUCTION FROM OVERLAPPING TILES\n{'=' * 80}")
    set_deterministic_seeds(1337)
    data_root = Path(args.data_root)
    images_dir, masks_dir = data_root / "images", data_root / "masks"
    output_dir = Path(args.output_dir)
    if args.max_tiles:
        output_dir = output_dir.parent / f"{output_dir.name}_{args.max_tiles}x{args.max_tiles}"
    if not images_dir.exists():
        raise FileNotFoundError(f"Images directory not found: {images_dir}")
    rank0 = process_group is None or torch.distributed.get_rank(process_group) == 0
    if rank0:
        for sub in ("masks", "overlays", "comparisons", "metrics"):
            (output_dir / sub).mkdir(parents=True, exist_ok=True)
    train_mean, train_std = load_training_stats(str(Path(args.weights).parent))
    if model is None:
        model = AdiposeUNet(tile_size=args.tile_size, dtype=getattr(args, "dtype", "f32"),
                            max_batch=getattr(args, "batch", 8))
        model.build_model()
        model.load_weights(args.weights)
    blender = GaussianBlender(tile_size=args.tile_size, sigma_factor=0.25) if args.blend_mode == "gaussian" \
        else LinearBlender()
    refiner = BoundaryRefiner(kernel_size=args.refine_kernel, bilateral_d=5, bilateral_sigma_color=50,
                              bilateral_sigma_space=50) if args.boundary_refine else None
    slides = group_tiles_by_slide(images_dir, masks_dir)
    print(f"✓ Found {len(slides)} slide(s)")
    results = []
    for slide_id, info in slides.items():
        tiles_info, positions = info["tiles"], info["positions"]
        if args.max_tiles:
            tiles_info = [t for t in tiles_info if t[0] < args.max_tiles and t[1] < args.max_tiles]
            positions = {(r, c) for r, c in positions if r < args.max_tiles and c < args.max_tiles}
            row_range = col_range = (0, args.max_tiles - 1)
        else:
            row_range, col_range = info["row_range"], info["col_range"]
        expected = create_expected_grid(row_range, col_range)
        missing = find_missing_tiles(expected, positions)
        coverage = len(positions) / len(expected)
        print(f"\nProcessing: {slide_id}\n  Tiles found: {len(tiles_info)}\n  Coverage: {coverage:.1%}")
        if coverage < args.min_coverage:
            print(f"  ⚠️  Skipping (coverage {coverage:.1%} < {args.min_coverage:.1%})")
            continue
        if args.max_tiles:
            side = (args.max_tiles - 1) * args.stride + args.tile_size
            full_shape = (side, side)
        else:
            full_shape = get_full_image_dimensions(slide_id, positions, args.tile_size, args.stride, args.data_root)
        full_rgb, full_pred, full_gt = reconstruct_slide(
            model, tiles_info, full_shape, args.tile_size, args.stride, train_mean, train_std, blender, refiner,
            args.use_tta, args.tta_mode, process_group=process_group)
        if not rank0:
            continue
        slide_dir = output_dir / slide_id
        slide_dir.mkdir(parents=True, exist_ok=True)
        _save_tiff(slide_dir / "original_image.tif", (full_rgb * 255).astype(np.uint8))
        _save_tiff(slide_dir / "prediction_mask.tif", (full_pred * 255).astype(np.uint8))
        metrics = {}
        if full_gt is not None:
            _save_tiff(slide_dir / "ground_truth_mask.tif", (full_gt * 255).astype(np.uint8))
            metrics = calculate_pixel_metrics(full_pred, full_gt, args.threshold)
            print(f"  Dice: {metrics['dice_score']:.4f}\n  IoU: {metrics['jaccard_index']:.4f}")
            _save_png(slide_dir / "gt_overlay.png", create_overlay(full_rgb, full_gt, (255, 255, 0)))
            _save_png(slide_dir / "pred_overlay.png", create_overlay(full_rgb, full_pred, (255, 0, 255)))
            _save_png(slide_dir / "comparison_4panel.png",
                      create_4panel_comparison(full_rgb, full_gt, full_pred, slide_id, metrics["dice_score"]))
            with open(slide_dir / "metrics.txt", "w") as f:
                f.write(f"Full Image Reconstruction Metrics\n{'=' * 60}\n\n")
                f.write(f"Slide: {slide_id}\nImage Size: {full_shape[1]} x {full_shape[0]} pixels\n")
                f.write(f"Tiles Used: {len(tiles_info)}\nCoverage: {coverage:.1%}\n\n")
                f.write(f"Reconstruction Settings:\n  Blend Mode: {args.blend_mode}\n")
                f.write(f"  TTA: {'Yes (' + args.tta_mode + ')' if args.use_tta else 'No'}\n")
                f.write(f"  Boundary Refinement: {'Yes' if args.boundary_refine else 'No'}\n")
                f.write(f"  Threshold: {args.threshold}\n\nPerformance Metrics:\n")
                for k, name in (("dice_score", "Dice Score:    "), ("jaccard_index", "IoU (Jaccard): "),
                                ("sensitivity", "Sensitivity:   "), ("specificity", "Specificity:   "),
                                ("precision", "Precision:     "), ("f1_score", "F1-Score:      ")):
                    f.write(f"  {name} {metrics[k]:.4f}\n")
        if args.save_metrics:
            res = {"slide_id": slide_id,
                   "reconstruction": {"tiles_used": len(tiles_info), "tiles_missing": len(missing),
                                      "coverage_ratio": coverage, "blend_mode": args.blend_mode,
                                      "tta_enabled": args.use_tta,
                                      "tta_mode": args.tta_mode if args.use_tta else None,
                                      "boundary_refined": args.boundary_refine},
                   "dimensions": {"width": full_shape[1], "height": full_shape[0],
                                  "tiles_rows": info["row_range"][1] - info["row_range"][0] + 1,
                                  "tiles_cols": info["col_range"][1] - info["col_range"][0] + 1},
                   "metrics": metrics if full_gt is not None else None}
            results.append(res)
            mp = output_dir / "metrics" / f"{slide_id}_metrics.json"
            mp.parent.mkdir(parents=True, exist_ok=True)
            mp.write_text(json.dumps(res, indent=2, default=float))
    if results and rank0:
        rows = [{"slide_id": r["slide_id"], "dice_score": r["metrics"]["dice_score"],
                 "jaccard_iou": r["metrics"]["jaccard_index"], "sensitivity": r["metrics"]["sensitivity"],
                 "specificity": r["metrics"]["specificity"], "precision": r["metrics"]["precision"],
                 "tiles_used": r["reconstruction"]["tiles_used"],
                 "tiles_missing": r["reconstruction"]["tiles_missing"],
                 "coverage": r["reconstruction"]["coverage_ratio"]} for r in results if r["metrics"]]
        if rows:
            import pandas as pd
            df = pd.DataFrame(rows)
            df.to_csv(output_dir / "metrics" / "summary.csv", index=False)
            print(f"\nMean Dice: {df['dice_score'].mean():.4f}\nMean IoU: {df['jaccard_iou'].mean():.4f}")
        create_reconstruction_log(args, output_dir, results)
    print(f"\n✅ Reconstruction complete!\n   Output directory: {output_dir}")
    return output_dir
