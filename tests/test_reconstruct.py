"""Full-slide reconstruction (adipose_amd.reconstruct vs Segmentation/reconstruct_full_images.py).

Golden vectors: tests/golden/reconstruct.npz, produced by the reference's own functions
(tests/golden/make_reconstruct_golden.py): filename parsing, slide grouping / missing tiles / inferred
dimensions, and reconstruct_slide outputs (RGB, prediction, GT) for Gaussian and linear blending, with
and without TTA, on two synthetic slides (one with a missing tile, masks missing for two tiles, 0/1
masks and clamped edge positions). The tile decode is pinned by construction (the generator served
the reference the PIL decode of the same tiles); cv2's own JPEG / grayscale decode is parity unpinned.
"""
import argparse
import json
import os
from pathlib import Path

import numpy as np
import pytest

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "reconstruct.npz"))
T, STRIDE = 64, 32


class FakePredictor:
    """Same deterministic predictor the golden generator used (make_golden.fake_predictor)."""

    def predict_single(self, image, mean, std):
        h, w = image.shape
        yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
        z = (image - mean) / (std + 1e-10)
        return (1.0 / (1.0 + np.exp(-(0.03 * yy - 0.05 * xx + 0.7 * z + 0.001 * yy * xx / h)))).astype(np.float32)


def write_dataset(root):
    """Tiles (lossless PNG content under the reference's *.jpg names) and masks (*.tif) from the golden."""
    from PIL import Image
    img_dir, msk_dir = Path(root) / "images", Path(root) / "masks"
    img_dir.mkdir(parents=True)
    msk_dir.mkdir(parents=True)
    for k in GOLD.files:
        if k.startswith("tile_"):
            Image.fromarray(GOLD[k]).save(img_dir / f"{k[5:]}.jpg", format="PNG")
        elif k.startswith("mask_"):
            Image.fromarray(GOLD[k]).save(msk_dir / f"{k[5:]}.tif", format="TIFF")
    return img_dir, msk_dir


def test_parse_tile_filename_golden():
    from adipose_amd.reconstruct import parse_tile_filename
    for name, want in zip(GOLD["parse_names"], GOLD["parse_out"]):
        try:
            s, r, c = parse_tile_filename(str(name))
            got = f"{s}|{r}|{c}"
        except ValueError:
            got = "ValueError"
        assert got == want, name


def test_grouping_missing_and_dimensions_golden(tmp_path):
    from adipose_amd import reconstruct as R
    img_dir, msk_dir = write_dataset(tmp_path)
    slides = R.group_tiles_by_slide(img_dir, msk_dir)
    assert list(slides) == ["slideA", "slide_B x"]
    for k, sid in enumerate(slides):
        info = slides[sid]
        got = [f"{r}|{c}|{Path(i).name}|{Path(m).name if m else ''}" for r, c, i, m in info["tiles"]]
        assert got == list(GOLD[f"group_{k}_tiles"])
        assert [*info["row_range"], *info["col_range"]] == list(GOLD[f"group_{k}_ranges"])
        exp = R.create_expected_grid(info["row_range"], info["col_range"])
        miss = sorted(R.find_missing_tiles(exp, info["positions"]))
        assert [list(m) for m in miss] == GOLD[f"group_{k}_missing"].reshape(-1, 2).tolist()
        assert list(R.infer_full_image_dimensions(info["positions"], T, STRIDE)) == list(GOLD[f"group_{k}_inferred"])
    assert R.get_source_image_dimensions("no-such-slide-xyz") is None
    with pytest.raises(ValueError):
        R.parse_tile_filename("nope.jpg")


def test_create_overlay_and_panel():
    from adipose_amd.reconstruct import create_4panel_comparison, create_overlay
    rgb = np.full((4, 4, 3), 0.5, np.float32)
    m = np.zeros((4, 4), np.float32)
    m[0, 0] = 1.0
    ov = create_overlay(rgb, m, (255, 0, 255))
    # uint8(0.5 * 255) = 127; 0.6 * 127 + 0.4 * 255 = 178.2 -> 178; 0.6 * 127 = 76.2 -> 76
    assert ov.dtype == np.uint8 and tuple(ov[0, 0]) == (178, 76, 178) and tuple(ov[1, 1]) == (76, 76, 76)
    p = create_4panel_comparison(rgb, m, 1 - m, "s", 0.0)
    assert p.shape == (8, 8, 3) and tuple(p[4 + 0, 4 + 0]) == (0, 0, 255) and tuple(p[4 + 1, 4 + 1]) == (255, 0, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["gaussian", "linear"])
@pytest.mark.parametrize("tta", [None, "basic"])
def test_reconstruct_slide_golden(tmp_path, mode, tta):
    from adipose_amd import reconstruct as R
    from adipose_amd.predictor import GaussianBlender, LinearBlender
    img_dir, msk_dir = write_dataset(tmp_path)
    slides = R.group_tiles_by_slide(img_dir, msk_dir)
    for k, sid in enumerate(slides):
        shape = tuple(int(v) for v in GOLD[f"group_{k}_shape"])
        blender = GaussianBlender(tile_size=T, sigma_factor=0.25) if mode == "gaussian" else LinearBlender()
        rgb, pred, gt = R.reconstruct_slide(FakePredictor(), slides[sid]["tiles"], shape, T, STRIDE, 120.0, 40.0,
                                            blender, None, tta is not None, tta or "basic")
        key = f"rec_{k}_{mode}_{tta or 'none'}"
        np.testing.assert_allclose(pred, GOLD[key + "_pred"], rtol=0, atol=2e-6)
        np.testing.assert_allclose(rgb, GOLD[key + "_rgb"], rtol=0, atol=2e-6)
        np.testing.assert_allclose(gt, GOLD[key + "_gt"], rtol=0, atol=2e-6)


@pytest.mark.gpu
def test_reconstruct_slide_hip_batched_matches_per_tile(tmp_path):
    """The HIP predictor's batched tiles x views path gives the same slide as the reference's per-tile
    loop over the same predictor (predict_single / per-view TTA)."""
    from adipose_amd import reconstruct as R
    from adipose_amd.predictor import AdiposeUNet, GaussianBlender
    from oracle import torch_ref as TR
    img_dir, msk_dir = write_dataset(tmp_path)
    slides = R.group_tiles_by_slide(img_dir, msk_dir)
    m = AdiposeUNet(tile_size=T, dtype="f32", max_batch=8)
    m.build_model()
    m.net.set_weights(TR.adipose_v3_keras_weights(seed=5, deep_supervision=False))

    class PerTile:
        def predict_single(self, image, mean, std):
            return m.predict_single(image, mean, std)

    info = slides["slide_B x"]
    shape = tuple(int(v) for v in GOLD["group_1_shape"])
    for tta in (False, True):
        a = R.reconstruct_slide(m, info["tiles"], shape, T, STRIDE, 120.0, 40.0, GaussianBlender(T), None, tta, "full")
        b = R.reconstruct_slide(PerTile(), info["tiles"], shape, T, STRIDE, 120.0, 40.0, GaussianBlender(T), None,
                                tta, "full")
        for x, y in zip(a, b):
            np.testing.assert_allclose(x, y, rtol=0, atol=1e-5)


@pytest.mark.gpu
def test_reconstruct_all_slides_outputs(tmp_path):
    from PIL import Image
    from adipose_amd import reconstruct as R
    write_dataset(tmp_path / "data")
    ck = tmp_path / "ckpt"
    ck.mkdir()
    (ck / "normalization_stats.json").write_text(json.dumps({"mean": 120.0, "std": 40.0}))
    args = argparse.Namespace(weights=str(ck / "w.weights.h5"), data_root=str(tmp_path / "data"),
                              output_dir=str(tmp_path / "out"), tile_size=T, stride=STRIDE, threshold=0.5,
                              blend_mode="gaussian", use_tta=False, tta_mode="basic", boundary_refine=False,
                              refine_kernel=5, save_metrics=True, min_coverage=0.9, max_tiles=None)
    out = R.reconstruct_all_slides(args, model=FakePredictor())
    # slide_B x has 11 / 12 tiles (coverage 0.917 >= 0.9); its source image is absent -> inferred 128 x 160
    for sid in ("slideA", "slide_B x"):
        d = out / sid
        for f in ("original_image.tif", "prediction_mask.tif", "ground_truth_mask.tif", "gt_overlay.png",
                  "pred_overlay.png", "comparison_4panel.png", "metrics.txt"):
            assert (d / f).exists(), (sid, f)
        assert (out / "metrics" / f"{sid}_metrics.json").exists()
    with Image.open(out / "slideA" / "prediction_mask.tif") as im:
        got = np.asarray(im)
    np.testing.assert_array_equal(got, (GOLD["rec_0_gaussian_none_pred"] * 255).astype(np.uint8))
    log = json.loads((out / "reconstruction_log.json").read_text())
    assert log["slides_processed"] == 2 and log["summary_statistics"]["total_tiles_missing"] == 1
    assert (out / "metrics" / "summary.csv").read_text().splitlines()[0].startswith("slide_id,dice_score")
    args.min_coverage = 0.95
    args.output_dir = str(tmp_path / "out2")
    R.reconstruct_all_slides(args, model=FakePredictor())
    assert not (tmp_path / "out2" / "slide_B x").exists()


def test_cli_flags_and_missing_data_root(tmp_path):
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "recon_cli", os.path.join(os.path.dirname(os.path.dirname(__file__)), "cli", "reconstruct_full_images.py"))
    cli = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cli)
    a = cli.parse_args(["--weights", "w.h5", "--data-root", "d", "--output-dir", "o"])
    assert (a.tile_size, a.stride, a.threshold, a.blend_mode, a.tta_mode, a.refine_kernel, a.min_coverage,
            a.max_tiles, a.use_tta, a.save_metrics) == (1024, 512, 0.5, "gaussian", "basic", 5, 0.9, None, False, False)
    # images/ missing -> FileNotFoundError inside, main() returns 1 (:946-953)
    assert cli.main(["--weights", str(tmp_path / "w.h5"), "--data-root", str(tmp_path / "none"),
                     "--output-dir", str(tmp_path / "o")]) == 1
