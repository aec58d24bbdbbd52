"""Pin the oracle (oracle/numpy_ref.py) to golden vectors produced by the reference's own code
(tests/golden/make_golden.py). Runs on CPU."""
import os

import numpy as np
import pytest

from oracle import numpy_ref as O

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def test_pixel_metrics_golden():
    d = load("pixel_metrics.npz")
    keys = [str(k) for k in d["keys"]]
    for a in range(d["preds"].shape[0]):
        for b, th in enumerate(d["thresholds"]):
            m = O.calculate_pixel_metrics(d["preds"][a], d["trues"][a], float(th))
            got = np.array([m[k] for k in keys], np.float64)
            np.testing.assert_allclose(got, d["metrics"][a, b], rtol=0, atol=1e-12)


def test_pixel_metrics_known_answers():
    # both empty -> all 1.0 (full_evaluation_enhanced.py:737-752)
    m = O.calculate_pixel_metrics(np.zeros((8, 8)), np.zeros((8, 8)))
    assert m["dice_score"] == 1.0 and m["tn"] == 64
    # 4x4 hand case: tp=3, fp=1, fn=1 -> dice 6/8, IoU 3/5
    pred = np.zeros((4, 4)); pred[0, :3] = 0.9; pred[1, 0] = 0.9
    true = np.zeros((4, 4)); true[0, :2] = 1; true[1, :2] = 1
    m = O.calculate_pixel_metrics(pred, true)
    assert (m["tp"], m["fp"], m["fn"], m["tn"]) == (3, 1, 1, 11)
    assert abs(m["dice_score"] - 0.75) < 1e-9 and abs(m["jaccard_index"] - 0.6) < 1e-9


def test_sliding_window_positions_golden():
    d = load("sw_positions.npz")
    for key in d.files:
        shape, ov = key.split("_")
        h, w = (int(v) for v in shape.split("x"))
        got = np.array(O.tile_positions((h, w), 1024, float(ov)), np.int64).reshape(-1, 2)
        np.testing.assert_array_equal(got, d[key])
    assert len(d["8192x8192_0.75"]) == 841  # config 4: 29 x 29 tiles


def test_gaussian_blend_golden():
    d = load("blend.npz")
    wm = O.gaussian_weight_map(1024)
    np.testing.assert_array_equal(wm[448:512, 0:64], d["weight_crop"])
    np.testing.assert_array_equal(wm[512], d["weight_row512"])
    assert abs(wm.astype(np.float64).sum() - float(d["weight_sum"])) < 1e-6
    tiles = list(d["tiles"])
    pos = [tuple(p) for p in d["tile_positions"]]
    np.testing.assert_array_equal(O.gaussian_reconstruct(tiles, pos, d["gauss_128"].shape, O.gaussian_weight_map(128)),
                                  d["gauss_128"])
    np.testing.assert_array_equal(O.linear_reconstruct(tiles, pos, d["linear"].shape), d["linear"])


def _fake_predict(image, mean, std):
    h, w = image.shape
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    z = (image - mean) / (std + 1e-10)
    return (1.0 / (1.0 + np.exp(-(0.03 * yy - 0.05 * xx + 0.7 * z + 0.001 * yy * xx / h)))).astype(np.float32)


@pytest.mark.parametrize("mode", ["minimal", "basic", "full"])
def test_tta_golden(mode):
    d = load("tta.npz")
    got = O.tta_predict(_fake_predict, d["image"], 120.0, 40.0, mode)
    np.testing.assert_array_equal(got, d[mode])


def test_threshold_search_golden():
    d = load("threshold.npz")
    pm = load("pixel_metrics.npz")
    preds, trues = list(pm["preds"][:12]), list(pm["trues"][:12])
    t, f1 = O.optimize_threshold_f1(preds, trues)
    assert abs(t - float(d["t_best"])) < 1e-12
    np.testing.assert_allclose(f1, d["f1"], atol=1e-12)
    t2, f1s = O.optimize_threshold_f1_slide_level(preds, trues, [str(p) for p in d["paths"]])
    assert abs(t2 - float(d["t_best_slide"])) < 1e-12
    np.testing.assert_allclose(f1s, d["f1_slide"], atol=1e-12)
    extra = ["6 BEEF Shoulder -1_grid_5x5_r1_c2_r0_c1.jpg", "plain.jpg", "x_c3.jpg"]
    ids = [O.extract_slide_id(p) for p in [str(p) for p in d["paths"]] + extra]
    assert ids == [str(s) for s in d["slide_ids"]]


def test_percentile_normalisation_golden():
    d = load("normalize.npz")
    for im, ref in zip(d["images"], d["percentile"]):
        np.testing.assert_allclose(O.normalize_percentile(im), ref, rtol=0, atol=1e-6)
