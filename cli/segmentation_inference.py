#!/usr/bin/env python3
"""Drop-in CLI for Segmentation/segmentation_inference.py (flags and defaults of :325-348, flow of
:307-488) on the HIP engine.

Same behaviour as the reference: weights from a file or a checkpoint directory (find_weights_file
:252-285, genuine `.weights.h5` first, then an earlier build's `.weights.safetensors`), z-score stats from `normalization_stats.json` next to the
weights (defaults 0/1 with a warning, :232-249), images of the wrong size are skipped with a warning
(:441-444), `masks/{stem}_mask.tif` (uint8 0/1), optional `probabilities/{stem}_prob.tif` (uint8
prob*255) and `overlays/{stem}_overlay.png`; returns 0/1. All TTA views of a tile run as one batched
forward on the GPU. Extra flags of this build: --tile (the reference hard-codes 1024), --dtype
(f32 = the reference's numerics, bf16 = throughput), --batch (tiles x views per forward).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

COLORS = {"cyan": (0, 255, 255), "yellow": (255, 255, 0), "magenta": (255, 0, 255), "green": (0, 255, 0),
          "red": (255, 0, 0)}
IMAGE_EXTS = {".jpg", ".jpeg", ".png", ".tif", ".tiff"}


def load_normalization_stats(checkpoint_dir):
    """segmentation_inference.py:232-249"""
    p = Path(checkpoint_dir) / "normalization_stats.json"
    if not p.exists():
        print(f"⚠️  Warning: {p} not found, using default normalization")
        return 0.0, 1.0
    with open(p) as f:
        st = json.load(f)
    mean, std = float(st["mean"]), float(st["std"])
    print(f"✓ Loaded normalization stats: mean={mean:.4f}, std={std:.4f}")
    return mean, std


def create_overlay_visualization(image, mask, color=(0, 255, 255)):
    """segmentation_inference.py:288-304: 0.6*image + 0.4*(image with mask pixels painted), rounded as
    cv2.addWeighted does (saturate_cast of the rounded sum)."""
    import numpy as np

    img = np.asarray(image)
    rgb = np.repeat(img.astype(np.uint8)[..., None], 3, axis=-1) if img.ndim == 2 else img.astype(np.uint8)
    over = rgb.copy()
    over[np.asarray(mask) > 0] = color
    out = rgb.astype(np.float64) * 0.6 + over.astype(np.float64) * 0.4
    return np.clip(np.rint(out), 0, 255).astype(np.uint8)


def build_parser():
    p = argparse.ArgumentParser(description="Run segmentation inference on a folder of images (MI355X HIP engine)")
    p.add_argument("--images-dir", type=str, required=True, help="Directory containing input images")
    p.add_argument("--output-dir", type=str, required=True, help="Directory to save predictions")
    p.add_argument("--weights", type=str, required=True, help="Path to model weights file or checkpoint directory")
    p.add_argument("--threshold", type=float, default=0.5, help="Binarization threshold (0-1, default: 0.5)")
    p.add_argument("--use-tta", action="store_true", default=False, help="Use Test Time Augmentation")
    p.add_argument("--tta-mode", type=str, default="basic", choices=["minimal", "basic", "full"])
    p.add_argument("--save-overlays", action="store_true", default=False)
    p.add_argument("--overlay-color", type=str, default="cyan", choices=list(COLORS))
    p.add_argument("--save-probability", action="store_true", default=False)
    # this build
    p.add_argument("--tile", type=int, default=1024, help="tile size the network is built for (reference: 1024)")
    p.add_argument("--dtype", type=str, default="f32", choices=["f32", "bf16"])
    p.add_argument("--batch", type=int, default=8, help="tiles x TTA views per batched forward")
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)
    images_dir, output_dir = Path(args.images_dir), Path(args.output_dir)
    if not images_dir.exists():
        print(f"❌ Error: Images directory not found: {images_dir}")
        return 1
    masks_dir = output_dir / "masks"
    masks_dir.mkdir(parents=True, exist_ok=True)
    overlays_dir = output_dir / "overlays"
    prob_dir = output_dir / "probabilities"
    if args.save_overlays:
        overlays_dir.mkdir(parents=True, exist_ok=True)
    if args.save_probability:
        prob_dir.mkdir(parents=True, exist_ok=True)

    print(f"\n{'=' * 80}\nADIPOSE TISSUE SEGMENTATION - INFERENCE\n{'=' * 80}")
    print(f"Images: {images_dir}\nOutput: {output_dir}\nThreshold: {args.threshold:.2f}")
    print(f"TTA: {'Enabled (' + args.tta_mode + ')' if args.use_tta else 'Disabled'}\n{'=' * 80}\n")

    import numpy as np

    import _adipose_pkg  # noqa: F401
    from adipose_amd.checkpoint import resolve_weights_file
    from adipose_amd.data import read_gray, write_mask
    from adipose_amd.predictor import AdiposeUNet, TestTimeAugmentation

    print("Loading model...")
    try:
        weights_file, checkpoint_dir = resolve_weights_file(args.weights)
    except FileNotFoundError as e:
        print(f"❌ {e}")
        return 1
    if weights_file.lower().endswith(".onnx"):
        print("❌ ONNX weights are not supported by the HIP engine (export the Keras-named weights instead)")
        return 1
    model = AdiposeUNet(tile_size=args.tile, dtype=args.dtype, max_batch=args.batch)
    model.build_model()
    model.load_weights(weights_file)
    mean, std = load_normalization_stats(checkpoint_dir)
    tta = None
    if args.use_tta:
        tta = TestTimeAugmentation(mode=args.tta_mode)
        print(f"✓ TTA enabled: {args.tta_mode} mode ({len(tta.transforms)} augmentations)")
    color = COLORS[args.overlay_color]

    image_files = [f for f in images_dir.iterdir() if f.suffix.lower() in IMAGE_EXTS and f.is_file()]
    if not image_files:
        print(f"❌ Error: No images found in {images_dir}\n   Looking for: {IMAGE_EXTS}")
        return 1
    print(f"\nFound {len(image_files)} images\nProcessing...\n")
    t0 = time.time()
    for img_path in image_files:
        try:
            image = read_gray(img_path)
        except Exception:  # cv2.imread returns None on unreadable files (:437-439)
            print(f"⚠️  Warning: Failed to load {img_path.name}, skipping")
            continue
        if image.shape != (args.tile, args.tile):
            print(f"⚠️  Warning: {img_path.name} is {image.shape}, expected ({args.tile}, {args.tile}), skipping")
            continue
        image = image.astype(np.float32)
        pred = tta.predict_with_tta(model, image, mean, std) if tta is not None else model.predict_single(image, mean, std)
        if args.save_probability:
            write_mask(prob_dir / f"{img_path.stem}_prob.tif", (pred * 255).astype(np.uint8))
        binary = (pred > args.threshold).astype(np.uint8)
        write_mask(masks_dir / f"{img_path.stem}_mask.tif", binary)
        if args.save_overlays:
            from PIL import Image
            Image.fromarray(create_overlay_visualization(image, binary, color)).save(
                overlays_dir / f"{img_path.stem}_overlay.png")
    elapsed = time.time() - t0
    print(f"\n{'=' * 80}\nINFERENCE COMPLETE\n{'=' * 80}")
    print(f"Processed: {len(image_files)} images")
    print(f"Time: {elapsed:.1f}s ({elapsed / len(image_files):.2f}s per image)")
    print(f"\nOutput saved to:\n  Masks: {masks_dir}")
    if args.save_overlays:
        print(f"  Overlays: {overlays_dir}")
    if args.save_probability:
        print(f"  Probabilities: {prob_dir}")
    print(f"{'=' * 80}\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
