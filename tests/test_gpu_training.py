"""End-to-end two-phase driver (train_adipose_unet_v3.py:1072-1441) on a small synthetic build:
phase 1 keeps the encoder frozen, phase 2 trains it, and the run leaves the reference's artefacts
(normalization_stats.json, training_settings.log, phase*_training.log, phase*_best / phase*_final /
weights_ema weight files) in the checkpoint directory; the drop-in CLI runs the same driver."""
import json

import numpy as np
import pytest

from adipose_amd import training as T
from adipose_amd.data import write_synthetic_build

pytestmark = pytest.mark.gpu


def test_phase1_freezes_encoder(tmp_path):
    build = write_synthetic_build(tmp_path / "build", n_train=4, n_val=2, size=64, seed=3)
    m = T.AdiposeUNetV3("t", freeze_encoder=True, build_timestamp="20260101_000000", batch_size=2, tile=64,
                        root=tmp_path)
    m.build_model()
    m.compile_model(lr=1e-3)
    before = {n: [a.copy() for a in m.net.engine.get_layer_weights(n)] for n in ("down1_conv1", "up1_conv1")}
    from adipose_amd.data import TileDataset
    ds = TileDataset(build / "dataset" / "train" / "images", build / "dataset" / "train" / "masks", 2,
                     augment=False, mean=200.0, std=25.0, normalization_method="zscore", seed=1)
    h = m.net.fit(ds.generator(), steps_per_epoch=2, epochs=1, verbose=0)
    assert np.isfinite(h.history["loss"][0])
    after = {n: m.net.engine.get_layer_weights(n) for n in before}
    assert all(np.array_equal(a, b) for a, b in zip(before["down1_conv1"], after["down1_conv1"]))
    assert not np.array_equal(before["up1_conv1"][0], after["up1_conv1"][0])


def test_two_phase_driver_and_cli(tmp_path):
    build = write_synthetic_build(tmp_path / "build", n_train=4, n_val=2, size=64, seed=4)
    import os

    from cli.train_adipose_unet_v3 import main
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        rc = main(["--data-root", str(build), "--pretrained-weights", "", "--epochs-phase1", "2", "--epochs-phase2",
                   "2", "--tile", "64", "--steps-per-epoch", "2", "--validation-steps", "1", "--seed", "1",
                   "--build-timestamp", "20260101_000000", "--warmup-epochs-phase1", "1",
                   "--warmup-epochs-phase2", "1"])
    finally:
        os.chdir(cwd)
    assert rc == 0
    cdir = tmp_path / "checkpoints" / "segmentation" / "20260101_000000_adipose_v3_1024_finetune_v3"
    names = {p.name for p in cdir.iterdir()}
    for f in ["normalization_stats.json", "training_settings.log", "phase1_training.log", "phase2_training.log",
              "phase1_best.weights.h5", "weights_phase1_final.weights.h5",
              "phase2_best.weights.h5", "weights_phase2_final.weights.h5",
              "weights_ema.weights.h5"]:
        assert f in names, (f, sorted(names))
    st = json.load(open(cdir / "normalization_stats.json"))
    assert st["normalization_method"] == "percentile" and st["num_training_images"] == 4
