#!/usr/bin/env python3
"""Drop-in CLI for Segmentation/reconstruct_full_images.py (flags and defaults of :873-931, main() :934-953,
returns 0/1) on the HIP engine. Extra flags of this build: --dtype (f32 = the reference's numerics, bf16),
--batch (tiles x TTA views per forward). Launched with torch.distributed.run (WORLD_SIZE > 1), each rank
predicts a contiguous run of every slide's tiles and the blend accumulators are SUM-reduced over RCCL."""
import argparse
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Reconstruct full images from overlapping tiles",
                                formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--weights", type=str, required=True, help="Path to trained model weights")
    p.add_argument("--data-root", type=str, required=True,
                   help="Path to dataset directory (contains images/ and masks/)")
    p.add_argument("--output-dir", type=str, required=True, help="Output directory for reconstructed images")
    p.add_argument("--tile-size", type=int, default=1024, help="Tile size (default: 1024)")
    p.add_argument("--stride", type=int, default=512, help="Stride between tiles (default: 512 for 50%% overlap)")
    p.add_argument("--threshold", type=float, default=0.5, help="Threshold for binary masks (default: 0.5)")
    p.add_argument("--blend-mode", type=str, default="gaussian", choices=["gaussian", "linear"])
    p.add_argument("--use-tta", action="store_true", default=False, help="Enable Test Time Augmentation")
    p.add_argument("--tta-mode", type=str, default="basic", choices=["minimal", "basic", "full"])
    p.add_argument("--boundary-refine", action="store_true", default=False, help="Enable boundary refinement")
    p.add_argument("--refine-kernel", type=int, default=5)
    p.add_argument("--save-masks", action="store_true", default=True)
    p.add_argument("--save-overlays", action="store_true", default=False)
    p.add_argument("--save-comparisons", action="store_true", default=False)
    p.add_argument("--save-metrics", action="store_true", default=False)
    p.add_argument("--min-coverage", type=float, default=0.90)
    p.add_argument("--max-tiles", type=int, default=None)
    p.add_argument("--dtype", type=str, default="f32", choices=["f32", "bf16"])
    p.add_argument("--batch", type=int, default=8)
    return p.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    group = None
    try:
        import torch
        import _adipose_pkg  # noqa: F401
        from adipose_amd.reconstruct import reconstruct_all_slides
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            import torch.distributed as dist
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
            dist.init_process_group("nccl")
            group = dist.group.WORLD
        reconstruct_all_slides(args, process_group=group)
        return 0
    except Exception as e:  # noqa: BLE001 (:949-953)
        print(f"\n❌ Reconstruction failed: {e}")
        traceback.print_exc()
        return 1
    finally:
        if group is not None:
            import torch.distributed as dist
            dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
