"""Evaluation surface (full_evaluation_enhanced.py) on the HIP engine.

CPU: host logic of the evaluation module — slide ids (reference golden), dice buckets, bootstrap CI,
weights resolution, image/mask pairing, boundary (EDT) metrics on known answers, AUC edge cases.
GPU: the one-pass threshold histogram (adp_threshold_hist) against per-threshold oracle counts
(calculate_pixel_metrics, :721-785) including float32 values that straddle float64 thresholds, the
threshold searches against the reference's golden curve (:891-980), and the drop-in evaluation
pipeline end to end against the CPU oracle network.
Boundary metrics rely on skimage.binary_erosion, which is absent here: restated with scipy (cross
footprint, border_value=1) and checked on known answers only — parity unpinned.
"""
import json
import os

import numpy as np
import pytest

from adipose_amd import evaluation as E
from oracle import numpy_ref as NR

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


# ------------------------------------------------------------------------------ CPU: host logic
def test_extract_slide_id_golden():
    d = golden("threshold.npz")
    extra = ["6 BEEF Shoulder -1_grid_5x5_r1_c2_r0_c1.jpg", "plain.jpg", "x_c3.jpg"]
    ids = [E.extract_slide_id(p) for p in [str(p) for p in d["paths"]] + extra]
    assert ids == [str(s) for s in d["slide_ids"]]


def test_categorize_by_dice_buckets():
    assert [E.categorize_by_dice(v) for v in (0.0, 0.2499, 0.25, 0.4999, 0.5, 0.7499, 0.75, 1.0)] == \
        ["poor", "poor", "medium", "medium", "good", "good", "excellent", "excellent"]


def test_bootstrap_ci_seeded_stream():
    data = np.random.default_rng(0).random(37)
    p, lo, hi = E.bootstrap_confidence_interval(data, n_bootstrap=500)
    rng = np.random.RandomState(42)
    stats = [np.mean(rng.choice(data, size=37, replace=True)) for _ in range(500)]
    assert p == float(np.mean(data))
    assert (lo, hi) == tuple(float(v) for v in np.percentile(stats, [2.5, 97.5]))
    pt, ci = E.safe_bootstrap_ci(np.array([np.nan, np.inf]))
    assert np.isnan(pt) and np.isnan(ci[0]) and np.isnan(ci[1])


def test_resolve_weights_path(tmp_path):
    d = tmp_path / "20260101_000000_adipose_v3"
    d.mkdir()
    with pytest.raises(ValueError):
        E.resolve_weights_path("")
    with pytest.raises(FileNotFoundError):
        E.resolve_weights_path(str(d))
    (d / "phase2_best.weights.safetensors").write_bytes(b"")
    (d / "weights_ema.weights.h5").write_bytes(b"")
    w, c = E.resolve_weights_path(str(d))
    assert w.endswith("phase2_best.weights.safetensors") and c == str(d)
    (d / "phase2_best.weights.h5").write_bytes(b"")
    assert E.resolve_weights_path(str(d))[0].endswith("phase2_best.weights.h5")
    w, _ = E.resolve_weights_path(str(d), use_ema=True)
    assert w.endswith("weights_ema.weights.h5")
    (d / "weights_best_overall.weights.safetensors").write_bytes(b"")
    assert E.resolve_weights_path(str(d))[0].endswith("weights_best_overall.weights.safetensors")
    root = tmp_path / "checkpoints"
    root.mkdir()
    with pytest.raises(ValueError):
        E.resolve_weights_path(str(root))


def test_detect_deep_supervision(tmp_path):
    assert E._detect_deep_supervision(tmp_path) is False
    (tmp_path / "training_settings.log").write_text("lr: 1e-4\nuse_deep_supervision: True\n")
    assert E._detect_deep_supervision(tmp_path) is True


def test_load_validation_data_pairs_by_stem(tmp_path):
    from PIL import Image
    (tmp_path / "images").mkdir()
    (tmp_path / "masks").mkdir()
    z = np.zeros((8, 8), np.uint8)
    for s in ("a_r0_c0", "a_r0_c1", "b_r1_c0"):
        Image.fromarray(z).save(tmp_path / "images" / f"{s}.jpg")
    Image.fromarray(z).save(tmp_path / "masks" / "a_r0_c0.tif")
    Image.fromarray(z).save(tmp_path / "masks" / "b_r1_c0_mask.png")
    pairs = E.load_validation_data(str(tmp_path))
    assert [(os.path.basename(a), os.path.basename(b)) for a, b in pairs] == \
        [("a_r0_c0.jpg", "a_r0_c0.tif"), ("b_r1_c0.jpg", "b_r1_c0_mask.png")]
    with pytest.raises(FileNotFoundError):
        E.load_validation_data(str(tmp_path / "missing"))


@pytest.mark.gpu
def test_boundary_metrics_known_answers():
    t = np.zeros((32, 32), np.float32)
    t[8:20, 8:20] = 1
    assert E.calculate_boundary_metrics(t, t) == {"hausdorff95": 0.0, "assd": 0.0}
    assert E.calculate_boundary_metrics(np.zeros_like(t), np.zeros_like(t)) == {"hausdorff95": 0.0, "assd": 0.0}
    assert E.calculate_boundary_metrics(np.zeros_like(t), t)["hausdorff95"] == float("inf")
    # reference quirk (:815-828): each surface is sampled in the EDT of its OWN complement, where it is 0,
    # so any pair of non-empty masks with surfaces scores 0 — reproduced as-is
    p = np.zeros_like(t)
    p[8:20, 10:22] = 1
    assert E.calculate_boundary_metrics(p, t) == {"hausdorff95": 0.0, "assd": 0.0}
    # an all-foreground mask has no surface (pixels outside the image count as set, skimage semantics)
    full = np.ones_like(t)
    assert E.calculate_boundary_metrics(full, full) == {"hausdorff95": float("inf"), "assd": float("inf")}


@pytest.mark.gpu
def test_auc_metrics_edge_cases():
    rng = np.random.default_rng(0)
    t = (rng.random((16, 16)) > 0.5).astype(np.float32)
    m = E.calculate_auc_metrics(t, t)
    assert m["roc_auc"] == 1.0 and m["pr_auc"] == 1.0
    m = E.calculate_auc_metrics(rng.random((16, 16)), np.zeros((16, 16)))
    assert np.isnan(m["roc_auc"]) and np.isnan(m["pr_auc"])


@pytest.mark.gpu
@pytest.mark.parametrize("shape,levels", [((64, 64), 0), ((256, 256), 17), ((1024, 1024), 0), ((1024, 1024), 255),
                                          ((3, 1000), 3)])
def test_auc_metrics_vs_sklearn(shape, levels):
    """GPU ROC AUC / average precision (adp_auc_metrics) vs the reference's scikit-learn calls
    (full_evaluation_enhanced.py:873-876) on continuous scores and on quantised scores (ties)."""
    from sklearn.metrics import average_precision_score, roc_auc_score
    rng = np.random.default_rng(sum(shape) + levels)
    y = (rng.random(shape) > 0.7).astype(np.float32)
    p = np.clip(0.35 * y + 0.65 * rng.random(shape), 0, 1).astype(np.float32)
    if levels:
        p = (np.round(p * levels) / levels).astype(np.float32)
    m = E.calculate_auc_metrics(p, y)
    yt, pf = (y > 0.5).astype(int).ravel(), p.ravel()
    assert abs(m["roc_auc"] - roc_auc_score(yt, pf)) <= 1e-9
    assert abs(m["pr_auc"] - average_precision_score(yt, pf)) <= 1e-9


def test_oracle_boundary_refiner_fixed_points_and_ellipse():
    """The cv2 restatement the GPU refiner is checked against: getStructuringElement(MORPH_ELLIPSE) rows for
    5 x 5 and 7 x 7 (OpenCV's published masks), constant maps are fixed points, output in [0, 1]."""
    lo, hi = NR.cv_ellipse_rows(5)
    assert list(zip(lo, hi)) == [(2, 3), (0, 5), (0, 5), (0, 5), (2, 3)]
    lo, hi = NR.cv_ellipse_rows(7)
    assert list(zip(lo, hi)) == [(3, 4), (1, 6), (0, 7), (0, 7), (0, 7), (1, 6), (3, 4)]
    assert E.ellipse_rows(9) == NR.cv_ellipse_rows(9)
    z = np.zeros((24, 24), np.float32)
    assert np.array_equal(NR.boundary_refine(z), z)
    o = np.ones((24, 24), np.float32)
    assert np.array_equal(NR.boundary_refine(o), o)
    m = np.zeros((24, 24), np.float32)
    m[6:18, 6:18] = 1
    out = NR.boundary_refine(m)
    assert out.dtype == np.float32 and out.shape == m.shape and out.min() >= 0 and out.max() <= 1


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,k,d,seed", [(64, 64, 5, 5, 0), (100, 37, 7, 9, 1), (256, 256, 5, 5, 2), (33, 65, 3, 3, 3)])
def test_gpu_boundary_refiner_vs_oracle(H, W, k, d, seed):
    """adp_boundary_refine (csrc/refine.hip) bit for bit against the numpy restatement of the cv2 calls on
    smoothed random probability maps (soft edges, so the bilateral filter acts inside the band)."""
    from scipy import ndimage
    rng = np.random.default_rng(seed)
    m = ndimage.gaussian_filter(rng.random((H, W)), 3)
    m = np.clip((m - m.mean()) * 8 + 0.5, 0, 1).astype(np.float32)
    r = E.BoundaryRefiner(kernel_size=k, bilateral_d=d)
    got = r.refine(m)
    ref = NR.boundary_refine(m, kernel_size=k, d=d)
    assert got.dtype == np.float32
    np.testing.assert_array_equal(got, ref)
    for c in (np.zeros((H, W), np.float32), np.ones((H, W), np.float32)):
        np.testing.assert_array_equal(r.refine(c), c)


def test_eval_cli_flags():
    from cli.full_evaluation_enhanced import build_parser
    a = build_parser().parse_args(["--weights", "w", "--test-dataset", "d"])
    assert (a.n_vis_samples, a.tta_mode, a.overlap, a.blend_mode, a.refine_kernel, a.n_positive, a.n_negative) == \
        (10, "basic", 0.5, "gaussian", 5, 120, 30)
    assert not (a.ema or a.use_tta or a.sliding_window or a.boundary_refine or a.adaptive_threshold)


# ------------------------------------------------------------------------------ GPU
def _oracle_counts(pred, true, thresholds):
    out = []
    for th in thresholds:
        pb, tb = pred > th, true > 0.5
        tp = int(np.sum(pb & tb))
        fp = int(np.sum(pb & ~tb))
        fn = int(np.sum(~pb & tb))
        out.append((tp, fp, fn, int(pb.size) - tp - fp - fn))
    return np.array(out, np.int64)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(1, 1), (37, 53), (256, 256), (1024, 1024)])
def test_threshold_hist_vs_oracle(shape):
    rng = np.random.default_rng(shape[0] * 7 + shape[1])
    thr = np.arange(0.1, 0.95, 0.05)
    pred = rng.random(shape).astype(np.float32)
    # values sitting exactly on float32(threshold): compared in float64 as numpy does
    flat = pred.reshape(-1)
    flat[: min(flat.size, len(thr))] = thr[: min(flat.size, len(thr))].astype(np.float32)
    if flat.size > 40:
        flat[20:24] = (0.0, 1.0, np.nextafter(np.float32(0.5), np.float32(1)), np.float32(0.5))
    true = (rng.random(shape) > 0.6).astype(np.float32)
    got = E.threshold_counts(pred, true, thr)
    np.testing.assert_array_equal(got, _oracle_counts(pred, true, thr))
    # unsorted thresholds come back in caller order
    perm = rng.permutation(len(thr))
    np.testing.assert_array_equal(E.threshold_counts(pred, true, thr[perm]), _oracle_counts(pred, true, thr[perm]))


@pytest.mark.gpu
def test_threshold_counts_empty_truth_and_metrics_row():
    pred = np.full((17, 19), 0.3, np.float32)
    true = np.zeros_like(pred)
    c = E.threshold_counts(pred, true, [0.2, 0.5])
    assert c.tolist() == [[0, 17 * 19, 0, 0], [0, 0, 0, 17 * 19]]
    for k, th in enumerate((0.2, 0.5)):
        ref = NR.calculate_pixel_metrics(pred, true, th)
        got = E._metrics_from_row(c[k])
        for key in ("dice_score", "jaccard_index", "precision", "sensitivity", "specificity", "accuracy"):
            assert abs(got[key] - ref[key]) < 1e-15, key


@pytest.mark.gpu
def test_threshold_search_golden_on_gpu():
    d = golden("threshold.npz")
    pm = golden("pixel_metrics.npz")
    preds, trues = list(pm["preds"][:12]), list(pm["trues"][:12])
    t, f1 = E.optimize_threshold_f1(preds, trues)
    assert abs(t - float(d["t_best"])) < 1e-12
    np.testing.assert_allclose(f1, d["f1"], rtol=0, atol=1e-12)
    t2, f1s = E.optimize_threshold_f1_slide_level(preds, trues, [str(p) for p in d["paths"]])
    assert abs(t2 - float(d["t_best_slide"])) < 1e-12
    np.testing.assert_allclose(f1s, d["f1_slide"], rtol=0, atol=1e-12)
    # fine adaptive grid (stage 2 of :1676-1690) against the oracle search
    grid = np.arange(0.3, 0.51, 0.01)
    ta, fa = E.optimize_threshold_f1_slide_level(preds, trues, [str(p) for p in d["paths"]], grid)
    to, fo = NR.optimize_threshold_f1_slide_level(preds, trues, [str(p) for p in d["paths"]], grid)
    assert ta == to
    np.testing.assert_allclose(fa, fo, rtol=0, atol=1e-12)


def _write_eval_fixture(tmp_path, S=64, n=5):
    """checkpoint dir (weights + normalization_stats.json + training_settings.log) and images/masks."""
    from PIL import Image

    from adipose_amd.checkpoint import save_weights
    from adipose_amd.nets import AdiposeV3Net
    from oracle import torch_ref as R
    w = R.adipose_v3_keras_weights(seed=865, deep_supervision=False)
    ck = tmp_path / "ckpt"
    ck.mkdir()
    net = AdiposeV3Net(1, S, dtype="f32", device="cuda", deep_supervision=False)
    net.set_weights(w)
    save_weights(net, str(ck / "phase2_best.weights.h5"))
    (ck / "normalization_stats.json").write_text(json.dumps({"mean": 127.0, "std": 50.0}))
    (ck / "training_settings.log").write_text("use_deep_supervision: False\n")
    ds = tmp_path / "val"
    (ds / "images").mkdir(parents=True)
    (ds / "masks").mkdir()
    rng = np.random.default_rng(11)
    names = []
    for i in range(n):
        img = (rng.random((S, S)) * 255).astype(np.uint8)
        m = (rng.random((S, S)) > 0.5).astype(np.uint8)
        name = f"slide{i % 2}_r{i}_c0"
        Image.fromarray(img).save(ds / "images" / f"{name}.png")
        Image.fromarray(m).save(ds / "masks" / f"{name}.tif")
        names.append(name)
    return ck, ds, w


@pytest.mark.gpu
def test_publication_evaluation_vs_oracle(tmp_path):
    import torch

    from cli.full_evaluation_enhanced import main
    from oracle import torch_ref as R
    ck, ds, w = _write_eval_fixture(tmp_path)
    res = E.run_publication_evaluation(str(ds), str(ck / "phase2_best.weights.h5"), str(tmp_path / "out"),
                                       dataset_name="val", optimize_threshold=False, save_visualizations=True,
                                       n_vis_samples=2, use_tta=True, tta_mode="basic", tile_size=64)
    assert (tmp_path / "out" / "val_comprehensive_results.csv").exists()
    assert len(list((tmp_path / "out" / "visualizations").glob("*.png"))) == 2

    def f(image, mean, std):
        x = torch.from_numpy(((image - np.float32(mean)) / np.float32(std + 1e-10)).astype(np.float32))[None]
        return R.adipose_v3_forward(x, w, deep_supervision=False)["main_out"][0].numpy()
    by = {}
    for img_p, m_p in E.load_validation_data(str(ds)):
        ref = NR.tta_predict(f, E.read_image_gray(img_p), 127.0, 50.0, "basic")
        true = (E.read_mask(m_p) > 0).astype(np.uint8)
        by.setdefault(E.extract_slide_id(img_p), []).append(NR.calculate_pixel_metrics(ref, true, 0.5)["dice_score"])
    dice_ref = float(np.mean([np.mean(v) for v in by.values()]))
    assert res.n_slides == 2 and res.n_tiles == 5
    assert abs(res.dice_score - dice_ref) < 1e-4
    # the drop-in CLI over the same checkpoint directory (weights resolution + output folder naming)
    rc = main(["--weights", str(ck), "--test-dataset", str(ds), "--tile", "64", "--optimize-threshold",
               "--no-visualizations", "--sliding-window", "--overlap", "0.25"])
    assert rc == 0
    assert (ck / "evaluation" / "val_original_sw_gaussian_o25" / "val_comprehensive_results.csv").exists()



@pytest.mark.gpu
@pytest.mark.parametrize("shape,spacing", [((64, 64), (1.0, 1.0)), ((200, 136), (1.0, 1.0)), ((96, 80), (0.5, 2.0)),
                                           ((1024, 1024), (1.0, 1.0))])
def test_distance_transform_vs_scipy(shape, spacing):
    """GPU exact EDT (adp_distance_transform) vs scipy.ndimage.distance_transform_edt on sparse random
    masks (large, non-trivial distances) with isotropic and anisotropic sampling."""
    from scipy import ndimage
    rng = np.random.default_rng(shape[0] + shape[1])
    m = rng.random(shape) > 0.003   # few zeros -> long distances
    m[rng.integers(0, shape[0]), rng.integers(0, shape[1])] = False
    got = E.distance_transform_edt(m, sampling=spacing).cpu().numpy()
    ref = ndimage.distance_transform_edt(m, sampling=spacing)
    assert np.abs(got - ref).max() <= 1e-9 * max(1.0, ref.max())


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_boundary_metrics_vs_oracle(seed):
    """calculate_boundary_metrics on the GPU vs the line-for-line scipy restatement of :788-844."""
    from oracle import numpy_ref as NR
    rng = np.random.default_rng(seed)
    H, W = 128, 96
    yy, xx = np.mgrid[0:H, 0:W]
    t = (((yy - 60) ** 2 + (xx - 40) ** 2) < 900).astype(np.float32)
    p = np.clip(t * 0.8 + rng.random((H, W)) * 0.4 - 0.1, 0, 1).astype(np.float32)
    if seed == 3:
        t[:] = 1.0   # full mask: no surface -> inf
    for thr in (0.3, 0.5, 0.7):
        got = E.calculate_boundary_metrics(p, t, thr, spacing=(1.0, 1.5))
        ref = NR.boundary_metrics(p, t, thr, spacing=(1.0, 1.5))
        for k in ("hausdorff95", "assd"):
            assert got[k] == ref[k] or abs(got[k] - ref[k]) <= 1e-9, (k, got, ref)
