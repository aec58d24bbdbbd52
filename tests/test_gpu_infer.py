"""Inference-path parity on the GPU: TTA view transforms / merge, Gaussian & linear blending, the
sliding window and pixel metrics — against the reference's golden vectors (bit-exact where the
reference arithmetic is exact) and against the CPU oracle network."""
import os

import numpy as np
import pytest
import torch

from adipose_amd import metrics as M
from adipose_amd import ops
from adipose_amd.nets import AdiposeV3Net
from adipose_amd.predictor import (TTA_VIEWS, GaussianBlender, HipUnetPredictor, LinearBlender,
                                   SlidingWindowInference, TestTimeAugmentation)
from oracle import numpy_ref as NR
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def fake_predict(image, mean, std):
    h, w = image.shape
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    z = (image - mean) / (std + 1e-10)
    return (1.0 / (1.0 + np.exp(-(0.03 * yy - 0.05 * xx + 0.7 * z + 0.001 * yy * xx / h)))).astype(np.float32)


@pytest.mark.parametrize("mode", ["minimal", "basic", "full"])
def test_tta_merge_matches_reference_golden(mode):
    """Per-view predictions of the reference's fake predictor -> GPU inverse transform + mean must be
    bit-identical to the reference TestTimeAugmentation output."""
    d = golden("tta.npz")
    img = d["image"]
    views = TTA_VIEWS[mode]
    per_view = np.stack([fake_predict(NR.TTA_TRANSFORMS[v][0](img).copy(), 120.0, 40.0) for v in views])
    out = torch.empty(img.shape, dtype=torch.float32, device=DEV)
    ops.tta_merge(torch.from_numpy(per_view).to(DEV), views, out)
    np.testing.assert_array_equal(out.cpu().numpy(), d[mode])


@pytest.mark.parametrize("view", range(8))
def test_prep_input_view_transform(view):
    """adp_prep_input(view) == (aug_v(image) - mean)/(std + 1e-10) exactly (f32)."""
    rng = np.random.default_rng(view)
    img = (rng.random((40, 40)) * 255).astype(np.float32)
    dst = torch.zeros((1, 40, 40, 8), dtype=torch.float32, device=DEV)
    ops.prep_input(torch.from_numpy(img).to(DEV)[None], dst, mean=120.5, std=33.25, view=view)
    ref = (NR.TTA_TRANSFORMS[view][0](img) - np.float32(120.5)) / np.float32(33.25 + 1e-10)
    np.testing.assert_array_equal(dst[0, :, :, 0].cpu().numpy(), ref.astype(np.float32))
    assert dst[..., 1:].abs().max().item() == 0.0


def test_prep_input_strided_window():
    rng = np.random.default_rng(1)
    img = (rng.random((100, 130)) * 255).astype(np.float32)
    dimg = torch.from_numpy(img).to(DEV)
    dst = torch.zeros((1, 32, 32, 8), dtype=torch.float32, device=DEV)
    ops.prep_input(dimg[20:52, 70:102][None], dst, mean=0.0, std=1.0)
    np.testing.assert_array_equal(dst[0, :, :, 0].cpu().numpy(), img[20:52, 70:102] / np.float32(1 + 1e-10))


def test_blenders_match_reference_golden():
    d = golden("blend.npz")
    tiles = list(d["tiles"])
    pos = [tuple(int(v) for v in p) for p in d["tile_positions"]]
    g = GaussianBlender(128).reconstruct(tiles, pos, d["gauss_128"].shape)
    np.testing.assert_array_equal(g, d["gauss_128"])
    lin = LinearBlender().reconstruct(tiles, pos, d["linear"].shape)
    np.testing.assert_array_equal(lin, d["linear"])
    np.testing.assert_array_equal(GaussianBlender(1024).weight_map[448:512, 0:64], d["weight_crop"])


def test_sliding_window_positions_golden():
    d = golden("sw_positions.npz")
    for key in d.files:
        shape, ov = key.split("_")
        h, w = (int(v) for v in shape.split("x"))
        sw = SlidingWindowInference(1024, float(ov), verbose=False)
        np.testing.assert_array_equal(np.array(sw.extract_tile_positions((h, w))).reshape(-1, 2), d[key])


def test_pixel_metrics_gpu_golden():
    d = golden("pixel_metrics.npz")
    keys = [str(k) for k in d["keys"]]
    for a in range(d["preds"].shape[0]):
        for b, th in enumerate(d["thresholds"]):
            m = M.calculate_pixel_metrics(d["preds"][a], d["trues"][a], float(th))
            np.testing.assert_allclose([m[k] for k in keys], d["metrics"][a, b], rtol=0, atol=1e-12)


@pytest.fixture(scope="module")
def small_predictor():
    w = R.adipose_v3_keras_weights(seed=865, deep_supervision=False)
    net = AdiposeV3Net(1, 64, dtype="f32", device=DEV, deep_supervision=False)
    net.set_weights(w)
    return HipUnetPredictor(net, max_batch=8), w


def oracle_predict_single(w):
    def f(image, mean, std):
        x = torch.from_numpy(((image - np.float32(mean)) / np.float32(std + 1e-10)).astype(np.float32))[None]
        return R.adipose_v3_forward(x, w, deep_supervision=False)["main_out"][0].numpy()
    return f


@pytest.mark.parametrize("mode", ["minimal", "basic", "full"])
def test_tta_network_vs_oracle(small_predictor, mode):
    pred, w = small_predictor
    rng = np.random.default_rng(5)
    img = (rng.random((64, 64)) * 255).astype(np.float32)
    got = TestTimeAugmentation(mode).predict_with_tta(pred, img, 127.0, 50.0)
    ref = NR.tta_predict(oracle_predict_single(w), img, 127.0, 50.0, mode)
    assert np.abs(got - ref).max() < 1e-4
    # batched GPU TTA == per-view GPU loop (reference host semantics) on the same predictor
    class Loop:
        def predict_single(self, image, mean, std):
            return pred.predict_single(np.ascontiguousarray(image), mean, std)
    loop = TestTimeAugmentation(mode).predict_with_tta(Loop(), img, 127.0, 50.0)
    assert np.abs(got - loop).max() < 1e-5


def test_sliding_window_network_vs_oracle(small_predictor):
    pred, w = small_predictor
    rng = np.random.default_rng(6)
    img = (rng.random((160, 224)) * 255).astype(np.float32)
    sw = SlidingWindowInference(64, 0.5, "gaussian", verbose=False)
    got = sw.predict_with_sliding_window(img, pred, 127.0, 50.0, use_tta=True, tta_mode="basic")
    f = oracle_predict_single(w)
    pos = NR.tile_positions(img.shape, 64, 0.5)
    tiles = [NR.tta_predict(f, img[y:y + 64, x:x + 64], 127.0, 50.0, "basic") for y, x in pos]
    ref = NR.gaussian_reconstruct(tiles, pos, img.shape, NR.gaussian_weight_map(64))
    assert np.abs(got - ref).max() < 1e-4
    # Dice/IoU of the thresholded maps agree within 1e-4 (north-star acceptance)
    truth = (ref > 0.5).astype(np.float32)
    a, b = M.calculate_pixel_metrics(got, truth), NR.calculate_pixel_metrics(ref, truth)
    assert abs(a["dice_score"] - b["dice_score"]) < 1e-4 and abs(a["jaccard_index"] - b["jaccard_index"]) < 1e-4


def test_loss_surface_vs_oracle():
    g = torch.Generator().manual_seed(2)
    p = torch.rand(2, 32, 48, generator=g)
    y = (torch.rand(2, 32, 48, generator=g) > 0.5).float()
    tol = 1e-5
    assert abs(M.dice_coef(y, p) - R.dice_coef(y, p).item()) < tol
    assert abs(M.combined_loss_standard(y, p) - R.combined_loss_standard(y, p).item()) < tol
    assert abs(M.online_hard_example_mining_loss(y, p) - R.ohem_loss(y, p).item()) < tol
    assert abs(M.combined_loss_with_label_smoothing(y, p) - R.combined_loss_with_label_smoothing(y, p).item()) < tol
    assert abs(M.online_hard_example_mining_loss_with_smoothing(y, p) - R.ohem_loss_with_smoothing(y, p).item()) < tol
    inter = (y * p).sum()
    jac = ((inter + 1e-7) / ((y + p).sum() - inter + 1e-7)).item()
    assert abs(M.jaccard_coef(y, p) - jac) < tol
    pi = torch.round(torch.clamp(p, 0, 1))
    inter_i = (y * pi).sum()
    jac_i = ((inter_i + 1e-7) / ((y + p).sum() - inter_i + 1e-7)).item()
    assert abs(M.jaccard_coef_int(y, p) - jac_i) < tol
    assert abs(M.binary_accuracy(y, p) - R.binary_accuracy(y, p).item()) < 1e-7
