#!/usr/bin/env python3
"""Drop-in CLI for Segmentation/full_evaluation_enhanced.py (flags and defaults of :1989-2036, flow of
main() :1961-2215) on the HIP engine: weights resolution (:401-490), output folder naming
{dataset}_{source}_{enhancements} under {checkpoint}/evaluation/ (:2053-2101), adaptive threshold implies
optimisation (:2104), returns 0/1. Extra flags of this build: --tile, --dtype, --batch."""
import argparse
import os
import sys
from pathlib import Path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build_parser():
    p = argparse.ArgumentParser(description="Publication-Quality Full Evaluation for Adipose U-Net (MI355X HIP engine)")
    p.add_argument("--weights", type=str, required=True)
    p.add_argument("--test-dataset", type=str, required=True)
    p.add_argument("--output", type=str, default="")
    p.add_argument("--ema", action="store_true", default=False)
    p.add_argument("--optimize-threshold", action="store_true")
    p.add_argument("--no-visualizations", action="store_true")
    p.add_argument("--n-vis-samples", type=int, default=10)
    p.add_argument("--use-tta", action="store_true", default=False)
    p.add_argument("--tta-mode", type=str, default="basic", choices=["minimal", "basic", "full"])
    p.add_argument("--sliding-window", action="store_true", default=False)
    p.add_argument("--overlap", type=float, default=0.5)
    p.add_argument("--blend-mode", type=str, default="gaussian", choices=["gaussian", "linear", "none"])
    p.add_argument("--boundary-refine", action="store_true", default=False)
    p.add_argument("--refine-kernel", type=int, default=5)
    p.add_argument("--adaptive-threshold", action="store_true", default=False)
    p.add_argument("--save-overlays", action="store_true", default=False)
    p.add_argument("--n-positive", type=int, default=120)
    p.add_argument("--n-negative", type=int, default=30)
    # this build
    p.add_argument("--tile", type=int, default=1024, help="tile size the network is built for (reference: 1024)")
    p.add_argument("--dtype", type=str, default="f32", choices=["f32", "bf16"])
    p.add_argument("--batch", type=int, default=8, help="tiles x TTA views per batched forward")
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)
    import _adipose_pkg  # noqa: F401
    from adipose_amd.evaluation import resolve_weights_path, run_publication_evaluation

    try:
        weights_path, checkpoint_dir = resolve_weights_path(args.weights, use_ema=args.ema)
    except (ValueError, FileNotFoundError) as e:
        print(e)
        return 1
    ds_path = Path(args.test_dataset)
    if not ds_path.exists():
        print(f"❌ Test dataset not found: {ds_path}")
        return 1
    if not ds_path.is_dir():
        print(f"❌ Test dataset path must be a directory: {ds_path}")
        return 1
    dataset_name = ds_path.name
    source = "stain" if "stain" in ds_path.parent.name.lower() else "original"
    suf = []
    if args.ema:
        suf.append("ema")
    if args.use_tta:
        suf.append(f"tta_{args.tta_mode}")
    if args.sliding_window:
        s = f"sw_{args.blend_mode}"
        if args.overlap != 0.5:
            s += f"_o{int(args.overlap * 100)}"
        suf.append(s)
    if args.boundary_refine:
        suf.append("refine" + (f"{args.refine_kernel}" if args.refine_kernel != 5 else ""))
    if args.adaptive_threshold:
        suf.append("adaptive")
    folder = f"{dataset_name}_{source}" + (f"_{'_'.join(suf)}" if suf else "")
    output_dir = Path(args.output) if args.output else Path(checkpoint_dir) / "evaluation" / folder
    opt_thresh = args.optimize_threshold or args.adaptive_threshold
    print(f"\n{'=' * 80}\nPUBLICATION-QUALITY EVALUATION PIPELINE\n{'=' * 80}")
    print(f"Weights:       {weights_path}\nCheckpoint:    {checkpoint_dir}\nTest Dataset:  {ds_path}")
    print(f"Dataset Name:  {dataset_name}\nData Source:   {source}\nOutput Dir:    {output_dir}\n{'=' * 80}")
    if not (ds_path / "images").exists() or not (ds_path / "masks").exists():
        print(f"❌ Dataset structure invalid. Expected:\n   {ds_path}/images/\n   {ds_path}/masks/")
        return 1
    try:
        r = run_publication_evaluation(
            val_data_root=str(ds_path), weights_path=weights_path, output_dir=str(output_dir),
            dataset_name=dataset_name, optimize_threshold=opt_thresh, save_visualizations=not args.no_visualizations,
            n_vis_samples=args.n_vis_samples, use_tta=args.use_tta, tta_mode=args.tta_mode,
            use_sliding_window=args.sliding_window, overlap=args.overlap, blend_mode=args.blend_mode,
            use_boundary_refine=args.boundary_refine, refine_kernel=args.refine_kernel,
            adaptive_threshold=args.adaptive_threshold, save_overlays=args.save_overlays,
            n_positive=args.n_positive, n_negative=args.n_negative, tile_size=args.tile, dtype=args.dtype,
            max_batch=args.batch)
    except Exception as e:  # noqa: BLE001 (reference prints the failure and returns 1, :2201-2215)
        import traceback
        print(f"\n{'=' * 80}\n❌ EVALUATION FAILED\n{'=' * 80}\nError: {e}")
        traceback.print_exc()
        return 1
    print(f"\n{'=' * 80}\nEVALUATION COMPLETE: {dataset_name.upper()}\n{'=' * 80}")
    print(f"  Dice Score:      {r.dice_score:.4f} (95% CI: [{r.dice_ci[0]:.4f}, {r.dice_ci[1]:.4f}])")
    print(f"  Jaccard (IoU):   {r.jaccard_index:.4f} (95% CI: [{r.jaccard_ci[0]:.4f}, {r.jaccard_ci[1]:.4f}])")
    print(f"  Precision:       {r.precision:.4f}\n  Sensitivity:     {r.sensitivity:.4f}")
    print(f"  Specificity:     {r.specificity:.4f}\n  Optimal Thresh:  {r.optimal_threshold:.3f}")
    print(f"  Slides:          {r.n_slides}\n  Tiles:           {r.n_tiles}\n\n📂 Results saved to: {output_dir}\n{'=' * 80}\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
