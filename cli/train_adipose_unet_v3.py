#!/usr/bin/env python3
"""Drop-in CLI for Segmentation/train_adipose_unet_v3.py (flags and defaults of :1458-1630) on the HIP
engine. Extra flags of this build: --tile, --dtype, --steps-per-epoch, --validation-steps, --seed,
--build-timestamp."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    p = argparse.ArgumentParser(description="Train adipose U-Net v3 (MI355X HIP engine)")
    p.add_argument("--data-root", type=str, default="/home/luci/adipose_tissue-unet/data/Meat_Luci_Tulane")
    p.add_argument("--pretrained-weights", type=str, default="checkpoints/unet_1024_dilation/weights_loss_val.weights.h5")
    p.add_argument("--batch-size", type=int, default=2)
    p.add_argument("--epochs-phase1", type=int, default=75)
    p.add_argument("--epochs-phase2", type=int, default=150)
    p.add_argument("--normalization-method", type=str, default="percentile", choices=["percentile", "zscore"])
    p.add_argument("--percentile-low", type=float, default=1.0)
    p.add_argument("--percentile-high", type=float, default=99.0)
    p.add_argument("--augmentation-level", type=str, default="moderate")
    p.add_argument("--checkpoint-suffix", type=str, default="")
    p.add_argument("--use-deep-supervision", action="store_true", default=True)
    p.add_argument("--no-deep-supervision", action="store_false", dest="use_deep_supervision")
    p.add_argument("--use-hard-mining", action="store_true", default=True)
    p.add_argument("--no-hard-mining", action="store_false", dest="use_hard_mining")
    p.add_argument("--hard-example-ratio", type=float, default=0.7)
    p.add_argument("--ema-decay", type=float, default=0.995)
    p.add_argument("--optimizer", type=str, default="adam", choices=["adam", "adamw"])
    p.add_argument("--label-smoothing", action="store_true", default=False)
    p.add_argument("--no-label-smoothing", action="store_false", dest="label_smoothing")
    p.add_argument("--label-smooth-epsilon-pos", type=float, default=0.03)
    p.add_argument("--label-smooth-epsilon-neg", type=float, default=0.07)
    p.add_argument("--use-cosine-schedule", action="store_true", default=True)
    p.add_argument("--no-cosine-schedule", action="store_false", dest="use_cosine_schedule")
    p.add_argument("--warmup-epochs-phase1", type=int, default=5)
    p.add_argument("--warmup-epochs-phase2", type=int, default=3)
    p.add_argument("--ds-weight-main", type=float, default=1.0)
    p.add_argument("--ds-weight-aux1", type=float, default=0.4)
    p.add_argument("--ds-weight-aux2", type=float, default=0.3)
    # this build
    p.add_argument("--tile", type=int, default=1024)
    p.add_argument("--dtype", type=str, default="f32", choices=["f32", "bf16"])
    p.add_argument("--steps-per-epoch", type=int, default=None)
    p.add_argument("--validation-steps", type=int, default=None)
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--build-timestamp", type=str, default=None)
    args = p.parse_args(argv)

    import _adipose_pkg  # noqa: F401
    from adipose_amd.training import train_model
    try:
        train_model(args.data_root, args.pretrained_weights, batch_size=args.batch_size,
                    epochs_phase1=args.epochs_phase1, epochs_phase2=args.epochs_phase2,
                    normalization_method=args.normalization_method, percentile_low=args.percentile_low,
                    percentile_high=args.percentile_high, build_timestamp=args.build_timestamp,
                    augmentation_level=args.augmentation_level, checkpoint_suffix=args.checkpoint_suffix,
                    use_deep_supervision=args.use_deep_supervision, use_hard_mining=args.use_hard_mining,
                    hard_example_ratio=args.hard_example_ratio, ema_decay=args.ema_decay,
                    optimizer_type=args.optimizer, use_label_smoothing=args.label_smoothing,
                    epsilon_pos=args.label_smooth_epsilon_pos, epsilon_neg=args.label_smooth_epsilon_neg,
                    use_cosine_schedule=args.use_cosine_schedule, warmup_epochs_phase1=args.warmup_epochs_phase1,
                    warmup_epochs_phase2=args.warmup_epochs_phase2, ds_weight_main=args.ds_weight_main,
                    ds_weight_aux1=args.ds_weight_aux1, ds_weight_aux2=args.ds_weight_aux2, tile=args.tile,
                    dtype=args.dtype, steps_per_epoch=args.steps_per_epoch, validation_steps=args.validation_steps,
                    seed=args.seed)
    except FileNotFoundError as e:
        print(f"Error: {e}")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
