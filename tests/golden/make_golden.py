"""Generate golden vectors by running the REFERENCE's own numpy code paths (build container only).

The reference evaluation module (Segmentation/full_evaluation_enhanced.py) imports TensorFlow, cv2,
tifffile, skimage and seaborn at module level; none is installed here (ordinary ImportError, not a
permission denial — SURVEY.md §8c). Only numpy/scipy code paths are exercised below, so those imports
are satisfied with inert placeholder modules whose attributes are never called by the functions used:
  calculate_pixel_metrics, SlidingWindowInference.extract_tile_positions, GaussianBlender,
  LinearBlender, TestTimeAugmentation (driven by a deterministic fake predictor),
  optimize_threshold_f1(_slide_level), extract_slide_id;
and src/utils/data.py:normalize_image. Outputs go to tests/golden/*.npz (data only — no reference
source is stored). Usage:  python tests/golden/make_golden.py [/root/reference]
"""
import importlib.abc
import importlib.machinery
import io
import contextlib
import os
import sys
import types

import numpy as np

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
STUB_ROOTS = ("tensorflow", "cv2", "tifffile", "skimage", "seaborn", "keras")


class _Anything:
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return _Anything()

    def __getattr__(self, name):
        return _Anything()


class _StubModule(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return _Anything()


class _StubFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, fullname, path, target=None):
        if fullname.split(".")[0] in STUB_ROOTS:
            return importlib.machinery.ModuleSpec(fullname, self, is_package=True)
        return None

    def create_module(self, spec):
        m = _StubModule(spec.name)
        m.__path__ = []
        return m

    def exec_module(self, module):
        pass


def load_reference():
    sys.meta_path.insert(0, _StubFinder())
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, "Segmentation"))
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    sys.dont_write_bytecode = True
    import full_evaluation_enhanced as fe  # noqa: E402
    from src.utils import data as du  # noqa: E402
    return fe, du


def fake_predictor():
    """Asymmetric deterministic predictor: p = sigmoid of a function of (y, x, intensity)."""
    class P:
        def predict_single(self, image, mean, std):
            h, w = image.shape
            yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
            z = (image - mean) / (std + 1e-10)
            return (1.0 / (1.0 + np.exp(-(0.03 * yy - 0.05 * xx + 0.7 * z + 0.001 * yy * xx / h)))).astype(np.float32)
    return P()


def main():
    fe, du = load_reference()
    quiet = contextlib.redirect_stdout(io.StringIO())
    rng = np.random.default_rng(865)
    g = {}

    # (i) pixel metrics
    preds, trues = [], []
    for i in range(12):
        p = rng.random((64, 64)).astype(np.float32)
        t = (rng.random((64, 64)) > 0.55).astype(np.float32)
        preds.append(p)
        trues.append(t)
    preds.append(np.zeros((64, 64), np.float32)); trues.append(np.zeros((64, 64), np.float32))   # both empty
    preds.append(np.ones((64, 64), np.float32)); trues.append(np.ones((64, 64), np.float32))     # all positive
    preds.append(np.full((64, 64), 0.9, np.float32)); trues.append(np.zeros((64, 64), np.float32))  # all FP
    preds.append(np.zeros((64, 64), np.float32)); trues.append(np.ones((64, 64), np.float32))    # all FN
    keys = ["dice_score", "jaccard_index", "sensitivity", "specificity", "precision", "f1_score", "accuracy",
            "tp", "fp", "fn", "tn"]
    ths = [0.3, 0.5, 0.7]
    met = np.zeros((len(preds), len(ths), len(keys)), np.float64)
    for a, (p, t) in enumerate(zip(preds, trues)):
        for b, th in enumerate(ths):
            m = fe.calculate_pixel_metrics(p, t, th)
            met[a, b] = [m[k] for k in keys]
    np.savez_compressed(os.path.join(OUT, "pixel_metrics.npz"), preds=np.stack(preds), trues=np.stack(trues),
                        thresholds=np.array(ths), keys=np.array(keys), metrics=met)

    # (ii) sliding-window positions
    shapes = [(1024, 1024), (1500, 2100), (8192, 8192), (1024, 3000), (2048, 1100)]
    overlaps = [0.0, 0.25, 0.5, 0.75, 0.9]
    pos = {}
    with quiet:
        for sh in shapes:
            for ov in overlaps:
                sw = fe.SlidingWindowInference(tile_size=1024, overlap=ov, blend_mode="gaussian" if ov != 0.25 else "linear")
                pos[f"{sh[0]}x{sh[1]}_{ov}"] = np.array(sw.extract_tile_positions(sh), np.int64).reshape(-1, 2)
    np.savez_compressed(os.path.join(OUT, "sw_positions.npz"), **pos)

    # (iii) Gaussian weight map (T=1024) and (v) blends of synthetic tiles
    gb = fe.GaussianBlender(1024)
    wm = gb.weight_map
    blend = {"weight_sum": np.float64(wm.astype(np.float64).sum()), "weight_crop": wm[448:512, 0:64].copy(),
             "weight_corner": wm[0, 0], "weight_center": wm[512, 512], "weight_row512": wm[512].copy()}
    with quiet:
        sw = fe.SlidingWindowInference(tile_size=128, overlap=0.5)
        H, W = 256, 320
        ps_ = sw.extract_tile_positions((H, W))
        tiles = [rng.random((128, 128)).astype(np.float32) for _ in ps_]
        blend["tile_positions"] = np.array(ps_)
        blend["tiles"] = np.stack(tiles)
        blend["gauss_128"] = fe.GaussianBlender(128).reconstruct(tiles, ps_, (H, W))
        blend["linear"] = fe.LinearBlender().reconstruct(tiles, ps_, (H, W))
    np.savez_compressed(os.path.join(OUT, "blend.npz"), **blend)

    # (iv) TTA with a deterministic fake predictor (both reference TTA classes)
    img = (rng.random((96, 96)) * 255).astype(np.float32)
    tta = {"image": img}
    P = fake_predictor()
    with quiet:
        for mode in ("minimal", "basic", "full"):
            pred, _ = fe.TestTimeAugmentation(mode).predict_with_tta(P, img, 120.0, 40.0)
            tta[mode] = pred
    np.savez_compressed(os.path.join(OUT, "tta.npz"), **tta)

    # (vi) threshold search + slide ids
    paths = [f"slideA_grid_5x5_r{i % 3}_c{i}.jpg" if i < 7 else f"slide B_r{i}_c{i % 2}.jpg" for i in range(12)]
    with quiet:
        t_best, f1 = fe.optimize_threshold_f1(preds[:12], trues[:12])
        t_best_s, f1_s = fe.optimize_threshold_f1_slide_level(preds[:12], trues[:12], paths)
    ids = [fe.extract_slide_id(p) for p in paths + ["6 BEEF Shoulder -1_grid_5x5_r1_c2_r0_c1.jpg", "plain.jpg",
                                                     "x_c3.jpg"]]
    np.savez_compressed(os.path.join(OUT, "threshold.npz"), t_best=t_best, f1=f1, t_best_slide=t_best_s,
                        f1_slide=f1_s, paths=np.array(paths), slide_ids=np.array(ids))

    # percentile normalisation (TileDataset default, train_adipose_unet_v3.py:591-593)
    imgs = np.stack([(rng.random((128, 128)) * 255).astype(np.float32) for _ in range(3)])
    imgs[2, :10] = 0.0
    normed = np.stack([np.asarray(du.normalize_image(im, method="percentile", p_low=1.0, p_high=99.0), np.float32)
                       for im in imgs])
    np.savez_compressed(os.path.join(OUT, "normalize.npz"), images=imgs, percentile=normed)
    print("golden vectors written to", OUT)


if __name__ == "__main__":
    main()
