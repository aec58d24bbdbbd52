"""Training surface of Segmentation/train_adipose_unet_v3.py on the HIP engine (SURVEY.md §8b seam 2).

* ``AdiposeUNetV3`` (train_adipose_unet_v3.py:628-922): checkpoint directory naming, ``build_model``,
  ``freeze_encoder_layers`` / ``unfreeze_encoder``, ``compile_model`` (loss selection, deep-supervision
  weights, Adam / AdamW), ``load_pretrained_weights``, ``save_weights_modern``; ``.net`` is a
  ``KerasLikeNet`` exposing the tf.keras.Model members the reference calls (fit / evaluate / predict,
  get/set/save/load_weights, count_params, trainable_weights, layers[i].trainable, optimizer.lr).
* Callbacks with the reference's semantics: ``CosineAnnealingWithWarmup`` (:368-407), ``EMACallback``
  (:410-505, per-epoch EMA of the weights), and the Keras ones the driver uses (ModelCheckpoint,
  EarlyStopping, CSVLogger, ReduceLROnPlateau).
* ``train_model`` (:1072-1441): the two-phase schedule (frozen encoder lr 1e-4 + EMA 0.999 unsaved, then
  all layers lr 1e-5 + EMA(--ema-decay) saved on the best monitor), normalization_stats.json,
  training_settings.log, phase*_best / phase*_final weights.

Every step runs on the GPU through ``trainer.Trainer`` (HIP kernels); this module is host control flow.
Weight files are genuine Keras 2.13 ``*.weights.h5`` files under the reference's names (checkpoint.py /
h5io.py: a pure-Python HDF5 writer, h5py is not installed on this image).
"""
from __future__ import annotations

import csv
import json
import math
import os
import platform
import sys
import time
from collections import OrderedDict
from datetime import datetime
from pathlib import Path

import numpy as np
import torch

from . import checkpoint as ckpt
from .nets import AdiposeV3Net
from .trainer import LossConfig, Trainer, cosine_warmup_lr

# freeze_encoder_layers (train_adipose_unet_v3.py:760-772); pooling layers carry no weights
ENCODER_LAYERS = ["down1_conv1", "down1_conv2", "down1_pool", "down2_conv1", "down2_conv2", "down2_pool",
                  "down3_conv1", "down3_conv2", "down3_pool"]


def weights_path(path):
    """Reference weight-file name -> the file this build writes/reads: the same name (genuine
    ``*.weights.h5``); a ``*.weights.h5`` that does not exist but has a ``*.weights.safetensors``
    sibling (an earlier build of this engine) resolves to the sibling."""
    p = str(path)
    if p.endswith(".weights.h5") and not os.path.exists(p):
        alt = p[: -len(".weights.h5")] + ".weights.safetensors"
        if os.path.exists(alt):
            return alt
    return p


# ----------------------------------------------------------------------------- model facade
class _Layer:
    def __init__(self, name):
        self.name = name
        self.trainable = True


class _Optimizer:
    """Holds the learning rate the LR callbacks set (K.set_value(model.optimizer.lr, v))."""

    def __init__(self, kind, lr):
        self.name = kind
        self.lr = float(lr)

    @property
    def learning_rate(self):
        return self.lr

    @learning_rate.setter
    def learning_rate(self, v):
        self.lr = float(v)


class History:
    def __init__(self):
        self.history = OrderedDict()
        self.epoch = []


def _labels(y):
    return y["main_out"] if isinstance(y, dict) else y


class KerasLikeNet:
    """The tf.keras.Model members train_adipose_unet_v3.py / full_evaluation_enhanced.py use."""

    def __init__(self, engine, name="adipose_unet_v3"):
        self.engine = engine
        self.name = name
        names = list(engine.layers)
        for extra in ("down1_pool", "down2_pool", "down3_pool"):
            if extra not in names:
                names.append(extra)
        self.layers = [_Layer(n) for n in names]
        self.optimizer = None
        self.trainer = None
        self.stop_training = False
        self.ds = getattr(engine, "ds", True)

    # -- compile / step
    def compile(self, *, optimizer_type="adam", lr=1e-4, loss_cfg=None):
        """Keras re-compile semantics: a fresh optimizer (new moments), trainable flags read now."""
        self.trainer = Trainer(self.engine, loss_cfg or LossConfig(), optimizer=optimizer_type, lr=lr)
        frozen = [l.name for l in self.layers if not l.trainable and l.name in self.engine.layers]
        self.trainer.set_frozen(frozen)
        self.optimizer = _Optimizer(optimizer_type, lr)

    def _require_compiled(self):
        if self.trainer is None:
            raise RuntimeError("You must compile your model before training/testing. Use `model.compile(...)`.")

    def _dev(self, a):
        if isinstance(a, torch.Tensor):   # device feed (TileDataset(device=...)): no host round trip
            return a.to(self.engine.device, torch.float32).contiguous()
        return torch.as_tensor(np.asarray(a, np.float32)).to(self.engine.device)

    def _metrics(self):
        m = self.trainer.read_metrics()
        if self.ds:
            return m
        return {"loss": m["loss"], "dice_coef": m["main_out_dice_coef"],
                "binary_accuracy": m["main_out_binary_accuracy"]}

    def train_on_batch(self, x, y):
        self._require_compiled()
        self.trainer.train_step(self._dev(x), self._dev(_labels(y)), lr=self.optimizer.lr)
        return self._metrics()

    def test_on_batch(self, x, y):
        self._require_compiled()
        self.trainer.eval_step(self._dev(x), self._dev(_labels(y)))
        return self._metrics()

    def evaluate(self, data, steps=None, verbose=0, return_dict=True):
        it = iter(data)
        sums, n = OrderedDict(), 0
        while steps is None or n < steps:
            try:
                x, y = next(it)
            except StopIteration:
                break
            for k, v in self.test_on_batch(x, y).items():
                sums[k] = sums.get(k, 0.0) + v
            n += 1
        return OrderedDict((k, v / max(n, 1)) for k, v in sums.items())

    def fit(self, x, steps_per_epoch=None, epochs=1, validation_data=None, validation_steps=None, callbacks=None,
            verbose=1, initial_epoch=0):
        """Keras fit over an endless generator of (x, y) batches: per-epoch means of the per-batch
        metrics (Keras Mean), 'val_' metrics from ``validation_steps`` batches, callback protocol."""
        self._require_compiled()
        callbacks = list(callbacks or [])
        for cb in callbacks:
            cb.set_model(self)
        hist = History()
        it = iter(x)
        self.stop_training = False
        for cb in callbacks:
            cb.on_train_begin({})
        for epoch in range(initial_epoch, epochs):
            for cb in callbacks:
                cb.on_epoch_begin(epoch, {})
            t0 = time.time()
            sums, n = OrderedDict(), 0
            while steps_per_epoch is None or n < steps_per_epoch:
                try:
                    xb, yb = next(it)
                except StopIteration:
                    break
                for k, v in self.train_on_batch(xb, yb).items():
                    sums[k] = sums.get(k, 0.0) + v
                n += 1
            logs = OrderedDict((k, v / max(n, 1)) for k, v in sums.items())
            if validation_data is not None:
                for k, v in self.evaluate(validation_data, validation_steps).items():
                    logs["val_" + k] = v
            if verbose:
                msg = " - ".join(f"{k}: {v:.4f}" for k, v in logs.items())
                print(f"Epoch {epoch + 1}/{epochs} - {time.time() - t0:.0f}s - {msg}", flush=True)
            for k, v in logs.items():
                hist.history.setdefault(k, []).append(v)
            hist.epoch.append(epoch)
            for cb in callbacks:
                cb.on_epoch_end(epoch, logs)
            if self.stop_training:
                break
        for cb in callbacks:
            cb.on_train_end({})
        return hist

    def predict(self, x, batch_size=None, verbose=0):
        """x: (B,S,S) normalised -> main probability map(s) (B,S,S) numpy."""
        xs = np.asarray(x, np.float32)
        net = self.engine
        out = []
        from . import ops
        for i in range(0, len(xs), net.B):
            chunk = xs[i:i + net.B]
            n = len(chunk)
            a = net.acts(net.B)
            pad = np.concatenate([chunk, np.repeat(chunk[-1:], net.B - n, 0)]) if n < net.B else chunk
            ops.prep_input(self._dev(pad), a["x"], mean=0.0, std=1.0)
            outs = net.forward(net.B, train=False)
            out.append(outs["main_out"].cpu().numpy()[:n])
        return np.concatenate(out)

    # -- weights (Keras flat-list order: layers in model order, [kernel, bias, ...] each)
    def get_weights(self):
        return [a for arrs in self.engine.get_weights().values() for a in arrs]

    def set_weights(self, weights):
        it = iter(weights)
        wd = OrderedDict()
        for name in self.engine.layers:
            wd[name] = [next(it) for _ in self.engine._slots(name)]
        self.engine.set_weights(wd)

    def save_weights(self, filepath, overwrite=True):
        p = weights_path(filepath)
        ckpt.save_weights(self.engine, p)
        return p

    def load_weights(self, filepath, by_name=False, skip_mismatch=False):
        ckpt.load_weights(self.engine, weights_path(filepath), by_name=by_name, skip_mismatch=skip_mismatch)

    def count_params(self):
        return self.engine.count_params()

    def _weights_of(self, trainable):
        out = []
        for l in self.layers:
            if l.name in self.engine.layers and l.trainable == trainable:
                out += self.engine.get_layer_weights(l.name)
        return out

    @property
    def trainable_weights(self):
        return self._weights_of(True)

    @property
    def non_trainable_weights(self):
        return self._weights_of(False)

    def summary(self, print_fn=print):
        print_fn(f'Model: "{self.name}"')
        for l in self.layers:
            if l.name in self.engine.layers:
                ks = [tuple(np.shape(a)) for a in self.engine.get_layer_weights(l.name)]
                print_fn(f"  {l.name:<14} {str(ks):<48} trainable={l.trainable}")
        print_fn(f"Total params: {self.count_params():,}")


# -------------------------------------------------------------------------------- callbacks
class Callback:
    def __init__(self):
        self.model = None

    def set_model(self, model):
        self.model = model

    def on_train_begin(self, logs=None):
        pass

    def on_train_end(self, logs=None):
        pass

    def on_epoch_begin(self, epoch, logs=None):
        pass

    def on_epoch_end(self, epoch, logs=None):
        pass


def _better(mode, a, b):
    return a > b if mode == "max" else a < b


class ModelCheckpoint(Callback):
    def __init__(self, filepath, monitor="val_loss", mode="auto", save_best_only=False, save_weights_only=True,
                 verbose=0):
        super().__init__()
        self.filepath, self.monitor, self.verbose = str(filepath), monitor, verbose
        self.mode = mode if mode in ("min", "max") else ("max" if "acc" in monitor or "dice" in monitor else "min")
        self.save_best_only = save_best_only
        self.best = -np.inf if self.mode == "max" else np.inf

    def on_epoch_end(self, epoch, logs=None):
        v = (logs or {}).get(self.monitor)
        if self.save_best_only:
            if v is None or not _better(self.mode, v, self.best):
                return
            if self.verbose:
                print(f"\nEpoch {epoch + 1}: {self.monitor} improved from {self.best:.5f} to {v:.5f}, "
                      f"saving model to {weights_path(self.filepath)}")
            self.best = v
        self.model.save_weights(self.filepath.format(epoch=epoch + 1, **(logs or {})))


class EarlyStopping(Callback):
    def __init__(self, monitor="val_loss", mode="auto", patience=0, restore_best_weights=False, verbose=0,
                 min_delta=0.0):
        super().__init__()
        self.monitor, self.patience, self.verbose = monitor, patience, verbose
        self.mode = mode if mode in ("min", "max") else "min"
        self.restore_best_weights, self.min_delta = restore_best_weights, abs(min_delta)
        self.wait, self.best, self.best_weights, self.stopped_epoch = 0, None, None, 0

    def on_train_begin(self, logs=None):
        self.wait = 0
        self.best = -np.inf if self.mode == "max" else np.inf

    def on_epoch_end(self, epoch, logs=None):
        v = (logs or {}).get(self.monitor)
        if v is None:
            return
        delta = self.min_delta if self.mode == "max" else -self.min_delta
        if _better(self.mode, v - delta, self.best):
            self.best, self.wait = v, 0
            if self.restore_best_weights:
                self.best_weights = self.model.get_weights()
            return
        self.wait += 1
        if self.wait >= self.patience:
            self.stopped_epoch = epoch
            self.model.stop_training = True
            if self.restore_best_weights and self.best_weights is not None:
                self.model.set_weights(self.best_weights)
            if self.verbose:
                print(f"Epoch {epoch + 1}: early stopping")


class CSVLogger(Callback):
    """Keras CSVLogger: header 'epoch,<sorted metric keys>', one row per epoch."""

    def __init__(self, filename, separator=",", append=False):
        super().__init__()
        self.filename, self.sep, self.append = str(filename), separator, append
        self.keys = None

    def on_train_begin(self, logs=None):
        if not self.append and os.path.exists(self.filename):
            os.remove(self.filename)
        self.keys = None

    def on_epoch_end(self, epoch, logs=None):
        logs = logs or {}
        new = not os.path.exists(self.filename)
        if self.keys is None:
            self.keys = sorted(logs.keys())
        with open(self.filename, "a", newline="") as f:
            w = csv.writer(f, delimiter=self.sep)
            if new:
                w.writerow(["epoch"] + self.keys)
            w.writerow([epoch] + [logs.get(k, "NA") for k in self.keys])


class ReduceLROnPlateau(Callback):
    def __init__(self, monitor="val_loss", mode="auto", factor=0.1, patience=10, min_lr=0.0, verbose=0):
        super().__init__()
        self.monitor, self.factor, self.patience, self.min_lr, self.verbose = monitor, factor, patience, min_lr, verbose
        self.mode = mode if mode in ("min", "max") else "min"
        self.best, self.wait = None, 0

    def on_train_begin(self, logs=None):
        self.best = -np.inf if self.mode == "max" else np.inf
        self.wait = 0

    def on_epoch_end(self, epoch, logs=None):
        v = (logs or {}).get(self.monitor)
        if v is None:
            return
        if _better(self.mode, v, self.best):
            self.best, self.wait = v, 0
            return
        self.wait += 1
        if self.wait >= self.patience:
            old = self.model.optimizer.lr
            new = max(old * self.factor, self.min_lr)
            if new < old:
                self.model.optimizer.lr = new
                if self.verbose:
                    print(f"Epoch {epoch + 1}: ReduceLROnPlateau reducing learning rate to {new:.2e}")
            self.wait = 0


class CosineAnnealingWithWarmup(Callback):
    """train_adipose_unet_v3.py:368-407 (per-epoch LR: linear warmup, then cosine to min_lr)."""

    def __init__(self, max_lr, min_lr, warmup_epochs, total_epochs, verbose=1):
        super().__init__()
        self.max_lr, self.min_lr = max_lr, min_lr
        self.warmup_epochs, self.total_epochs, self.verbose = warmup_epochs, total_epochs, verbose
        self.current_epoch = 0

    def on_epoch_begin(self, epoch, logs=None):
        self.current_epoch = epoch
        lr = cosine_warmup_lr(epoch, self.max_lr, self.min_lr, self.warmup_epochs, self.total_epochs)
        self.model.optimizer.lr = lr
        if self.verbose and epoch % 5 == 0:
            print(f"\nEpoch {epoch + 1}: Learning rate = {lr:.2e}")


class EMACallback(Callback):
    """train_adipose_unet_v3.py:410-505: per-EPOCH EMA of the weights (ema = d*ema + (1-d)*w), optional
    best-snapshot save on a monitor, save at train end if no best snapshot was written."""

    def __init__(self, decay=0.995, save_ema_weights=True, checkpoint_dir=None, monitor=None, mode="max",
                 save_best_only=False):
        super().__init__()
        self.decay, self.save_ema_weights = decay, save_ema_weights
        self.checkpoint_dir = Path(checkpoint_dir) if checkpoint_dir else None
        self.ema_weights = None
        self.monitor, self.mode, self.save_best_only = monitor, mode.lower(), save_best_only
        if self.mode not in ("min", "max"):
            raise ValueError("EMACallback mode must be 'min' or 'max'")
        self.best = -np.inf if self.mode == "max" else np.inf
        self._best_saved = False

    def on_epoch_end(self, epoch, logs=None):
        cur = self.model.get_weights()
        if self.ema_weights is None:
            self.ema_weights = [w.copy() for w in cur]
        else:
            self.ema_weights = [self.decay * e + (1 - self.decay) * c for e, c in zip(self.ema_weights, cur)]
        if self.save_best_only and self.save_ema_weights and self.monitor:
            v = (logs or {}).get(self.monitor)
            if v is not None and _better(self.mode, v, self.best):
                self.best = v
                self._best_saved = True
                self._save(best_snapshot=True)

    def on_train_end(self, logs=None):
        if self.save_ema_weights and self.ema_weights and self.checkpoint_dir and not self._best_saved:
            self._save()

    def _save(self, best_snapshot=False):
        if not self.checkpoint_dir:
            return
        cur = self.model.get_weights()
        self.model.set_weights(self.ema_weights)
        p = self.model.save_weights(str(self.checkpoint_dir / "weights_ema.weights.h5"))
        self.model.set_weights(cur)
        print(f"\nSaved EMA weights to: {p}" + ("  (best EMA snapshot)" if best_snapshot else ""))


# ------------------------------------------------------------------------------- the model
class AdiposeUNetV3:
    """train_adipose_unet_v3.py:628-922 on the HIP engine. ``batch_size``/``tile`` fix the engine's
    buffers (the reference hard-codes 1024); ``dtype`` is the compute dtype (the reference is fp32)."""

    def __init__(self, checkpoint_name, freeze_encoder=True, build_timestamp=None, use_deep_supervision=True, *,
                 batch_size=2, tile=1024, dtype="f32", device="cuda", root="."):
        self.checkpoint_name = checkpoint_name
        self.freeze_encoder = freeze_encoder
        self.use_deep_supervision = use_deep_supervision
        self.batch_size, self.tile, self.dtype, self.device = batch_size, tile, dtype, device
        self.net = None
        timestamp = build_timestamp or datetime.now().strftime("%Y%m%d_%H%M%S")
        self.checkpoint_dir = Path(root) / "checkpoints" / "segmentation" / f"{timestamp}_{checkpoint_name}_1024_finetune_v3"
        self.checkpoint_dir.mkdir(parents=True, exist_ok=True)
        print(f"Checkpoint directory: {self.checkpoint_dir}")

    def build_model(self, init_nb=44, dropout_rate=0.3):
        engine = AdiposeV3Net(self.batch_size, self.tile, dtype=self.dtype, device=self.device, init_nb=init_nb,
                              dropout_rate=dropout_rate, deep_supervision=self.use_deep_supervision)
        self.net = KerasLikeNet(engine)
        if self.freeze_encoder:
            self.freeze_encoder_layers()
        return self.net

    def freeze_encoder_layers(self):
        for layer in self.net.layers:
            if layer.name in ENCODER_LAYERS:
                layer.trainable = False
        print(f"Frozen {len(ENCODER_LAYERS)} encoder layers for transfer learning")

    def unfreeze_encoder(self):
        for layer in self.net.layers:
            layer.trainable = True
        print("Unfrozen all layers for fine-tuning")

    def compile_model(self, lr=1e-4, use_hard_mining=True, hard_example_ratio=0.7, optimizer_type="adam",
                      use_label_smoothing=False, epsilon_pos=0.03, epsilon_neg=0.07, ds_weight_main=1.0,
                      ds_weight_aux1=0.4, ds_weight_aux2=0.3):
        cfg = LossConfig(use_hard_mining=use_hard_mining, hard_example_ratio=hard_example_ratio,
                         use_label_smoothing=use_label_smoothing, epsilon_pos=epsilon_pos, epsilon_neg=epsilon_neg,
                         ds_weight_main=ds_weight_main, ds_weight_aux1=ds_weight_aux1, ds_weight_aux2=ds_weight_aux2)
        opt = "adamw" if optimizer_type.lower() == "adamw" else "adam"
        self.net.compile(optimizer_type=opt, lr=lr, loss_cfg=cfg)
        print(f"Using {opt.upper()} optimizer (lr={lr}); hard mining={use_hard_mining} "
              f"(ratio={hard_example_ratio}); label smoothing={use_label_smoothing}")

    def load_pretrained_weights(self, h5_path):
        """By name with skipped mismatches under deep supervision (aux heads stay initialised), else strict
        with a by-name fallback (train_adipose_unet_v3.py:881-916)."""
        path = weights_path(h5_path)
        if self.use_deep_supervision:
            try:
                self.net.load_weights(path, by_name=True, skip_mismatch=True)
                print(f"Loaded pretrained weights from {path} (by name, skipped aux heads)")
            except Exception as e:  # the reference warns and trains from scratch
                print(f"Warning: Partial weight loading failed: {e}\nTraining from scratch!")
        else:
            try:
                self.net.load_weights(path)
                print(f"Loaded weights from {path} (strict topology match)")
            except Exception as e:
                print(f"Strict load failed: {e}")
                self.net.load_weights(path, by_name=True, skip_mismatch=True)
                print(f"Loaded weights from {path} by layer name (skipped mismatches)")

    def save_weights_modern(self, suffix="finetuned"):
        p = self.net.save_weights(str(self.checkpoint_dir / f"weights_{suffix}.weights.h5"))
        print(f"Saved modern weights to {p}")
        return p


# ------------------------------------------------------------------------------ the driver
def capture_system_info():
    info = {"python": sys.version.split()[0], "platform": platform.platform(), "torch": torch.__version__,
            "hip": getattr(torch.version, "hip", None)}
    if torch.cuda.is_available():
        info["device"] = torch.cuda.get_device_name(0)
        info["device_count"] = torch.cuda.device_count()
    return info


def log_training_settings(checkpoint_dir, command_line_args, data_config, model_config, training_config):
    """training_settings.log (train_adipose_unet_v3.py:984-1053): the run's settings as JSON sections."""
    p = Path(checkpoint_dir) / "training_settings.log"
    with open(p, "w") as f:
        f.write(f"Training settings - {datetime.now().isoformat()}\n")
        for title, d in (("SYSTEM", capture_system_info()), ("COMMAND LINE", command_line_args),
                         ("DATA", data_config), ("MODEL", model_config), ("TRAINING", training_config)):
            f.write(f"\n[{title}]\n{json.dumps(d, indent=2, default=str)}\n")
    return p


def train_model(data_root, pretrained_weights, batch_size=2, epochs_phase1=75, epochs_phase2=150,
                normalization_method="percentile", percentile_low=1.0, percentile_high=99.0, build_timestamp=None,
                augmentation_level="moderate", checkpoint_suffix="", use_deep_supervision=True, use_hard_mining=True,
                hard_example_ratio=0.7, ema_decay=0.995, optimizer_type="adam", use_label_smoothing=False,
                epsilon_pos=0.03, epsilon_neg=0.07, use_cosine_schedule=True, warmup_epochs_phase1=5,
                warmup_epochs_phase2=3, ds_weight_main=1.0, ds_weight_aux1=0.4, ds_weight_aux2=0.3, *,
                tile=1024, dtype="f32", steps_per_epoch=None, validation_steps=None, root=".", seed=None):
    """Two-phase fine-tuning (train_adipose_unet_v3.py:1072-1441)."""
    from .data import TileDataset, compute_mean_std

    data_root = Path(data_root)
    tr_img, tr_msk = data_root / "dataset" / "train" / "images", data_root / "dataset" / "train" / "masks"
    va_img, va_msk = data_root / "dataset" / "val" / "images", data_root / "dataset" / "val" / "masks"
    for p in (tr_img, tr_msk, va_img, va_msk):
        if not p.exists():
            raise FileNotFoundError(f"Training data not found: {p}")
    train_paths = sorted(tr_img.glob("*.jpg"))
    train_mean, train_std = compute_mean_std(train_paths)
    name = "adipose_v3" + (f"_{checkpoint_suffix}" if checkpoint_suffix else "")
    model = AdiposeUNetV3(name, freeze_encoder=True, build_timestamp=build_timestamp,
                          use_deep_supervision=use_deep_supervision, batch_size=batch_size, tile=tile, dtype=dtype,
                          root=root)
    model.build_model()
    compile_kw = dict(use_hard_mining=use_hard_mining, hard_example_ratio=hard_example_ratio,
                      optimizer_type=optimizer_type, use_label_smoothing=use_label_smoothing, epsilon_pos=epsilon_pos,
                      epsilon_neg=epsilon_neg, ds_weight_main=ds_weight_main, ds_weight_aux1=ds_weight_aux1,
                      ds_weight_aux2=ds_weight_aux2)
    model.compile_model(lr=1e-4, **compile_kw)
    if pretrained_weights and Path(weights_path(pretrained_weights)).exists():
        model.load_pretrained_weights(pretrained_weights)
    else:
        print(f"Pretrained weights not found: {pretrained_weights}; training from scratch")
    norm = {"mean": float(train_mean), "std": float(train_std), "normalization_method": normalization_method,
            "dataset_path": str(data_root), "num_training_images": len(train_paths),
            "build_timestamp": build_timestamp, "version": "3.0"}
    with open(model.checkpoint_dir / "normalization_stats.json", "w") as f:
        json.dump(norm, f, indent=2)
    # the reference's pipelines (_select_augment_fn, :1056-1067) on the GPU; feed batches stay in HBM
    from .augment import select_augment_fn
    augment_fn, augment_label = select_augment_fn(augmentation_level)
    ds_kw = dict(mean=train_mean, std=train_std, normalization_method=normalization_method,
                 percentile_low=percentile_low, percentile_high=percentile_high, seed=seed,
                 device=model.net.engine.device)
    train_ds = TileDataset(tr_img, tr_msk, batch_size, augment=augment_fn is not None, augment_fn=augment_fn,
                           augment_level=augment_label, **ds_kw)
    val_ds = TileDataset(va_img, va_msk, batch_size, augment=False, **ds_kw)
    spe = steps_per_epoch or max(1, len(train_ds) // batch_size)
    vst = validation_steps or max(1, len(val_ds) // batch_size)
    log_training_settings(
        model.checkpoint_dir,
        {"data_root": str(data_root), "pretrained_weights": pretrained_weights, "batch_size": batch_size,
         "use_deep_supervision": use_deep_supervision, "use_hard_mining": use_hard_mining,
         "hard_example_ratio": hard_example_ratio, "ema_decay": ema_decay, "optimizer": optimizer_type},
        {"train_images_count": len(train_ds), "validation_images_count": len(val_ds),
         "normalization_mean": train_mean, "normalization_std": train_std, "augmentation_type": augmentation_level},
        {"architecture": "U-Net V3 with deep supervision", "deep_supervision": use_deep_supervision,
         "total_parameters": model.net.count_params(),
         "trainable_parameters": int(sum(np.size(w) for w in model.net.trainable_weights)),
         "non_trainable_parameters": int(sum(np.size(w) for w in model.net.non_trainable_weights))},
        {"total_epochs": epochs_phase1 + epochs_phase2, "batch_size": batch_size, "hard_mining": use_hard_mining,
         "ema_decay": ema_decay, "optimizer": optimizer_type, "compute_dtype": dtype})
    monitor = "val_main_out_dice_coef" if use_deep_supervision else "val_dice_coef"
    cdir = model.checkpoint_dir

    def phase_callbacks(phase, ema, max_lr, min_lr, warmup, epochs):
        cbs = [ModelCheckpoint(cdir / f"phase{phase}_best.weights.h5", monitor=monitor, mode="max", save_best_only=True,
                               verbose=1),
               EarlyStopping(monitor=monitor, mode="max", patience=15, verbose=1), ema,
               CSVLogger(cdir / f"phase{phase}_training.log")]
        if use_cosine_schedule:
            cbs.append(CosineAnnealingWithWarmup(max_lr, min_lr, warmup, epochs))
        else:
            cbs.append(ReduceLROnPlateau(monitor=monitor, mode="max", factor=0.5, patience=5, min_lr=min_lr, verbose=1))
        return cbs

    # phase 1: frozen encoder
    h1 = model.net.fit(train_ds.generator(), steps_per_epoch=spe, epochs=epochs_phase1,
                       validation_data=val_ds.generator(), validation_steps=vst,
                       callbacks=phase_callbacks(1, EMACallback(decay=0.999, save_ema_weights=False, checkpoint_dir=cdir),
                                                 1e-4, 1e-7, warmup_epochs_phase1, epochs_phase1))
    model.save_weights_modern("phase1_final")
    best1 = Path(weights_path(cdir / "phase1_best.weights.h5"))
    if best1.exists():
        model.net.load_weights(str(best1))
    # phase 2: everything trainable, fresh optimizer
    model.unfreeze_encoder()
    model.compile_model(lr=1e-5, **compile_kw)
    ema2 = EMACallback(decay=ema_decay, save_ema_weights=True, checkpoint_dir=cdir, monitor=monitor, mode="max",
                       save_best_only=True)
    h2 = model.net.fit(train_ds.generator(), steps_per_epoch=spe, epochs=epochs_phase2,
                       validation_data=val_ds.generator(), validation_steps=vst,
                       callbacks=phase_callbacks(2, ema2, 1e-5, 1e-8, warmup_epochs_phase2, epochs_phase2))
    model.save_weights_modern("phase2_final")
    return model, h1, h2
