"""Handle-level C ABI (adp_create / adp_set_param / adp_forward / adp_destroy; csrc/engine.cpp): the native
adipose_v3 inference engine against the Python schedule (nets.AdiposeV3Net through HipUnetPredictor)
and the CPU oracle, on the same Keras weights (predict_single segmentation_inference.py:153-158, TTA
:181-229)."""
import numpy as np
import pytest
import torch

from oracle import numpy_ref as NR
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu
S = 64


@pytest.fixture(scope="module")
def weights():
    return R.adipose_v3_keras_weights(seed=865, deep_supervision=True)


def oracle_predict(w):
    def f(image, mean, std):
        x = torch.from_numpy(((image - np.float32(mean)) / np.float32(std + 1e-10)).astype(np.float32))[None]
        return R.adipose_v3_forward(x, w, deep_supervision=True)["main_out"][0].numpy()
    return f


def test_engine_params_round_trip_and_errors(weights):
    from adipose_amd._lib import AdpError
    from adipose_amd.engine import NativeAdiposeV3
    eng = NativeAdiposeV3(tile=S, max_batch=4, dtype="f32")
    names = eng.layer_names()
    assert names[0] == "down1_conv1" and "dilate6" in names and names[-1] == "output_softmax"
    assert set(names) == set(weights)
    eng.set_weights(weights)
    got = eng.get_weights()
    for k in names:
        for a, b in zip(weights[k], got[k]):
            np.testing.assert_array_equal(np.asarray(a, np.float32).ravel(), b)
    with pytest.raises(AdpError):
        eng.predict_batch(np.zeros((1, S + 8, S + 8), np.float32), 0.0, 1.0)
    bad = {"down1_conv1": [np.zeros(5, np.float32), np.zeros(44, np.float32)]}
    with pytest.raises(AdpError):
        eng.set_weights(bad)
    eng.close()


@pytest.mark.parametrize("tta", [None, "minimal", "basic", "full"])
def test_engine_f32_vs_python_and_oracle(weights, tta):
    from adipose_amd.engine import NativeAdiposeV3
    from adipose_amd.nets import AdiposeV3Net
    from adipose_amd.predictor import TTA_VIEWS, HipUnetPredictor
    rng = np.random.default_rng(3)
    imgs = (rng.random((3, S, S)) * 255).astype(np.float32)
    eng = NativeAdiposeV3(tile=S, max_batch=8, dtype="f32")
    eng.set_weights(weights)
    got = eng.predict_batch(imgs, 127.0, 50.0, tta_mode=tta).cpu().numpy()
    net = AdiposeV3Net(1, S, dtype="f32", device="cuda", deep_supervision=True)
    net.set_weights(weights)
    pred = HipUnetPredictor(net, max_batch=8)
    views = TTA_VIEWS[tta] if tta else [0]
    ref = pred.predict_views(list(imgs), 127.0, 50.0, views).cpu().numpy()
    assert np.abs(got - ref).max() <= 1e-5, np.abs(got - ref).max()
    f = oracle_predict(weights)
    for i in range(3):
        o = NR.tta_predict(f, imgs[i], 127.0, 50.0, tta) if tta else f(imgs[i], 127.0, 50.0)
        assert np.abs(got[i] - o).max() <= 1e-4
    eng.close()


def test_engine_bf16_matches_python_bf16_predictor(weights):
    from adipose_amd.engine import NativeAdiposeV3
    from adipose_amd.predictor import AdiposeUNet
    rng = np.random.default_rng(4)
    imgs = (rng.random((5, S, S)) * 255).astype(np.float32)
    eng = NativeAdiposeV3(tile=S, max_batch=4, dtype="bf16")
    eng.set_weights(weights)
    got = eng.predict_batch(imgs, 127.0, 50.0, tta_mode="basic").cpu().numpy()
    m = AdiposeUNet(tile_size=S, dtype="bf16", max_batch=4)
    m.build_model(use_deep_supervision=True)
    m.net.set_weights(weights)
    ref = np.stack([m.predict(im, 127.0, 50.0, use_tta=True, tta_mode="basic")[0] for im in imgs])
    assert np.abs(got - ref).max() <= 1e-5, np.abs(got - ref).max()
    f32 = NativeAdiposeV3(tile=S, max_batch=4, dtype="f32")
    f32.set_weights(weights)
    exact = f32.predict_batch(imgs, 127.0, 50.0, tta_mode="basic").cpu().numpy()
    assert np.abs(got - exact).max() <= 2e-2
    eng.close()
    f32.close()
