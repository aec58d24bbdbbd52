"""Host logic of the training surface (training.py) against the reference's formulas:
CosineAnnealingWithWarmup (train_adipose_unet_v3.py:393-404), per-epoch EMA (:446-505),
Keras ModelCheckpoint(save_best_only) / EarlyStopping(patience) / CSVLogger as the driver uses them
(:1266-1300), and the weight-file name resolution (genuine .weights.h5, earlier .weights.safetensors)."""
import csv
import math

import numpy as np

from adipose_amd import training as T


class FakeModel:
    def __init__(self, weights):
        self.w = [np.array(a, np.float64) for a in weights]
        self.optimizer = T._Optimizer("adam", 1e-4)
        self.stop_training = False
        self.saved = []

    def get_weights(self):
        return [a.copy() for a in self.w]

    def set_weights(self, ws):
        self.w = [np.array(a) for a in ws]

    def save_weights(self, path):
        self.saved.append((str(path), [a.copy() for a in self.w]))
        return T.weights_path(path)


def test_cosine_warmup_schedule():
    m = FakeModel([np.zeros(1)])
    cb = T.CosineAnnealingWithWarmup(1e-4, 1e-7, 5, 75, verbose=0)
    cb.set_model(m)
    for e, want in [(0, 2e-5), (4, 1e-4), (5, 1e-4),
                    (40, 1e-7 + 0.5 * (1e-4 - 1e-7) * (1 + math.cos(math.pi * 35 / 70))),
                    (74, 1e-7 + 0.5 * (1e-4 - 1e-7) * (1 + math.cos(math.pi * 69 / 70)))]:
        cb.on_epoch_begin(e)
        assert abs(m.optimizer.lr - want) < 1e-15, (e, m.optimizer.lr, want)


def test_ema_per_epoch_and_best_snapshot(tmp_path):
    m = FakeModel([np.ones(3), np.full(2, 4.0)])
    cb = T.EMACallback(decay=0.9, save_ema_weights=True, checkpoint_dir=tmp_path, monitor="val_main_out_dice_coef",
                       mode="max", save_best_only=True)
    cb.set_model(m)
    seq = [(1.0, 0.5), (3.0, 0.4), (5.0, 0.7)]
    ema = None
    for e, (wv, dice) in enumerate(seq):
        m.w = [np.full(3, wv), np.full(2, 4.0 * wv)]
        cb.on_epoch_end(e, {"val_main_out_dice_coef": dice})
        cur = [np.full(3, wv), np.full(2, 4.0 * wv)]
        ema = cur if ema is None else [0.9 * a + 0.1 * c for a, c in zip(ema, cur)]
        for a, b in zip(cb.ema_weights, ema):
            np.testing.assert_allclose(a, b)
    # best snapshots at epochs 0 and 2 only, saved as the EMA weights, model weights restored after
    assert len(m.saved) == 2 and all(p.endswith("weights_ema.weights.h5") for p, _ in m.saved)
    np.testing.assert_allclose(m.saved[-1][1][0], ema[0])
    np.testing.assert_allclose(m.w[0], np.full(3, 5.0))
    cb.on_train_end()
    assert len(m.saved) == 2           # a best snapshot exists -> no extra save at train end


def test_checkpoint_best_only_and_early_stopping(tmp_path):
    m = FakeModel([np.zeros(1)])
    ck = T.ModelCheckpoint(tmp_path / "phase1_best.weights.h5", monitor="val_dice", mode="max", save_best_only=True)
    es = T.EarlyStopping(monitor="val_dice", mode="max", patience=2)
    log = T.CSVLogger(tmp_path / "phase1_training.log")
    for cb in (ck, es, log):
        cb.set_model(m)
        cb.on_train_begin()
    vals = [0.1, 0.3, 0.2, 0.25, 0.9]
    for e, v in enumerate(vals):
        for cb in (ck, es, log):
            cb.on_epoch_end(e, {"val_dice": v, "loss": 1.0 - v})
        if m.stop_training:
            break
    assert len(m.saved) == 2           # improvements at epochs 0 and 1 only
    assert m.stop_training and es.stopped_epoch == 3
    rows = list(csv.reader(open(tmp_path / "phase1_training.log")))
    assert rows[0] == ["epoch", "loss", "val_dice"] and len(rows) == 5


def test_weights_path_mapping():
    assert T.weights_path("a/phase1_best.weights.h5") == "a/phase1_best.weights.h5"
    assert T.weights_path("x.weights.safetensors") == "x.weights.safetensors"
