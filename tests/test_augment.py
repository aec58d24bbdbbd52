"""Training-time augmentation (src/utils/data.py:13-264) and percentile normalisation (:398-429).

CPU: the oracle restatement (oracle/augment_ref.py) against golden vectors generated from the
reference's own functions (tests/golden/make_augment_golden.py): pixel-exact for the numpy functions and
the light pipeline, and the exact random-draw sequence (cv2 calls + next RandomState value) of the
moderate / heavy pipelines. GPU: the adp_aug_* / adp_percentile_normalize kernels through
adipose_amd.augment against the oracle on the same seeds. The cv2 operations (resize, GaussianBlur,
remap) are restated from OpenCV's documented semantics: parity unpinned (cv2 is not installed).
"""
import os

import numpy as np
import pytest
import torch

from oracle import augment_ref as A

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden():
    return np.load(os.path.join(G, "augment.npz"), allow_pickle=False)


class RecordingCv2(A.Cv2Restated):
    def __init__(self):
        self.calls = []

    def GaussianBlur(self, src, ksize, sigma):
        self.calls.append(repr(("GaussianBlur", float(sigma), tuple(np.shape(src)))))
        return np.array(src, copy=True)

    def resize(self, src, dsize, interpolation):
        self.calls.append(repr(("resize", tuple(int(v) for v in dsize), int(interpolation))))
        return np.zeros((dsize[1], dsize[0]), dtype=np.asarray(src).dtype)

    def remap(self, src, map1, map2, interpolation, borderMode=None, borderValue=0):
        self.calls.append(repr(("remap", tuple(np.shape(map1)), int(interpolation))))
        return np.array(src, copy=True)


# ------------------------------------------------------------------------------ CPU: oracle vs reference
def test_numpy_functions_match_reference():
    d = golden()
    img, mask = d["image"], d["mask"]
    for s in range(6):
        r = np.random.RandomState(100 + s)
        a, b = A.random_rotation_90(img, mask, r)
        a, b = A.random_flip(a, b, r)
        np.testing.assert_array_equal(a, d[f"geom_{s}_img"])
        np.testing.assert_array_equal(b, d[f"geom_{s}_mask"])
        np.testing.assert_array_equal(A.random_brightness(img, (0.7, 1.3), r), d[f"bright_{s}"])
        np.testing.assert_array_equal(A.random_contrast(img, (0.7, 1.3), r), d[f"contrast_{s}"])
        np.testing.assert_array_equal(A.random_gamma(img, (0.7, 1.3), r), d[f"gamma_{s}"])
        np.testing.assert_array_equal(A.random_gaussian_noise(img, (0, 10), 1.0, r), d[f"noise_{s}"])
        assert r.random() == float(d[f"next_{s}"])
        r = np.random.RandomState(200 + s)
        li, lm = A.augment_pair_light(img, mask, r)
        np.testing.assert_array_equal(li, d[f"light_{s}_img"])
        np.testing.assert_array_equal(lm, d[f"light_{s}_mask"])
        assert r.random() == float(d[f"light_{s}_next"])


@pytest.mark.parametrize("name", ["moderate", "heavy", "tta_style"])
def test_pipeline_draw_sequence_matches_reference(name):
    d = golden()
    fn = getattr(A, f"augment_pair_{name}")
    for s in range(40):
        cv = RecordingCv2()
        r = np.random.RandomState(1000 + s)
        fn(d["image"], d["mask"], r, cv2=cv)
        assert cv.calls == [str(c) for c in d[f"{name}_{s}_calls"]], s
        assert r.random() == float(d[f"{name}_{s}_next"]), s


def test_percentile_numpy123_semantics():
    d = np.load(os.path.join(G, "normalize.npz"), allow_pickle=False)
    for im, ref in zip(d["images"], d["percentile"]):
        np.testing.assert_allclose(A.normalize_percentile_np123(im), ref, rtol=0, atol=1e-6)


def test_cv2_restatements_basic_properties():
    rng = np.random.default_rng(0)
    x = rng.random((20, 30)).astype(np.float32) * 255
    # identity resize, reflect-101 blur of a constant, zero-displacement remap
    np.testing.assert_array_equal(A.CV2.resize(x, (30, 20), 1), x)
    np.testing.assert_array_equal(A.CV2.resize(x, (30, 20), 0), x)
    c = np.full((9, 11), 7.0, np.float32)
    np.testing.assert_allclose(A.CV2.GaussianBlur(c, (0, 0), 1.3), c, rtol=1e-6)
    yy, xx = np.mgrid[0:20, 0:30].astype(np.float32)
    np.testing.assert_array_equal(A.CV2.remap(x, xx, yy, 1), x)
    np.testing.assert_array_equal(A.CV2.remap(x, xx, yy, 0), x)
    w, r = A.gaussian_taps(0.8)
    assert len(w) == 2 * r + 1 == 7 and abs(float(w.sum()) - 1) < 1e-6   # round(8*0.8+1)|1 = 7


# ------------------------------------------------------------------------------ GPU
def _gpu_aug():
    from adipose_amd import augment as GA
    return GA


def _np(t):
    return t.detach().cpu().numpy()


@pytest.mark.gpu
def test_gpu_light_pipeline_bit_exact():
    GA = _gpu_aug()
    d = golden()
    for s in range(6):
        r = np.random.RandomState(200 + s)
        gi, gm = GA.augment_pair_light(d["image"], d["mask"], r)
        np.testing.assert_array_equal(_np(gi), d[f"light_{s}_img"])
        np.testing.assert_array_equal(_np(gm), d[f"light_{s}_mask"])
        assert r.random() == float(d[f"light_{s}_next"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["moderate", "heavy", "tta_style"])
def test_gpu_pipelines_vs_oracle(name):
    """Same seeds -> same draws (next RandomState value), image within 1e-3 of the oracle on the 0-255
    scale (contrast's mean is an f64 device sum vs numpy's f32 pairwise sum), masks identical."""
    GA = _gpu_aug()
    d = golden()
    rng = np.random.RandomState(5)
    img = (rng.rand(96, 128) * 255).astype(np.float32)
    mask = (rng.rand(96, 128) > 0.5).astype(np.float32)
    for s in range(40):
        r1, r2 = np.random.RandomState(1000 + s), np.random.RandomState(1000 + s)
        gi, gm = getattr(GA, f"augment_pair_{name}")(img, mask, r1)
        oi, om = getattr(A, f"augment_pair_{name}")(img, mask, r2)
        assert r1.random() == r2.random(), s
        assert np.abs(_np(gi) - oi).max() <= 1e-3, (s, np.abs(_np(gi) - oi).max())
        mism = np.mean(_np(gm) != om)
        assert mism == 0.0, (s, mism)
    _ = d


@pytest.mark.gpu
@pytest.mark.parametrize("shape,new", [((64, 80), (70, 88)), ((64, 80), (60, 75)), ((33, 47), (33, 47))])
def test_gpu_scale_vs_oracle(shape, new):
    GA = _gpu_aug()
    rng = np.random.default_rng(1)
    x = (rng.random(shape) * 255).astype(np.float32)
    m = (rng.random(shape) > 0.5).astype(np.float32)
    H, W = shape
    scale_is_up = new[0] >= H
    xs = A.CV2.resize(x, (new[1], new[0]), 1)
    ms = A.CV2.resize(m, (new[1], new[0]), 0)
    if scale_is_up:
        y0, x0 = (new[0] - H) // 2, (new[1] - W) // 2
        ref_i, ref_m = xs[y0:y0 + H, x0:x0 + W], ms[y0:y0 + H, x0:x0 + W]
    else:
        ph, pw = (H - new[0]) // 2, (W - new[1]) // 2
        pad = ((ph, H - new[0] - ph), (pw, W - new[1] - pw))
        ref_i, ref_m = np.pad(xs, pad, mode="reflect"), np.pad(ms, pad, mode="constant")
    from adipose_amd._lib import call, ptr, stream_ptr
    xi, xm = GA._dev(x), GA._dev(m)
    oi, om = torch.empty_like(xi), torch.empty_like(xm)
    call("adp_aug_scale", H, W, new[0], new[1], ptr(xi), ptr(oi), 0, stream_ptr())
    call("adp_aug_scale", H, W, new[0], new[1], ptr(xm), ptr(om), 1, stream_ptr())
    assert np.abs(_np(oi) - ref_i).max() <= 1e-3
    np.testing.assert_array_equal(_np(om), ref_m)


@pytest.mark.gpu
@pytest.mark.parametrize("sigma,dt", [(0.5, np.float32), (1.0, np.float32), (3.0, np.float64)])
def test_gpu_blur_vs_oracle(sigma, dt):
    GA = _gpu_aug()
    x = np.random.default_rng(2).random((40, 56)).astype(dt) * 255
    got = _np(GA._blur(torch.from_numpy(x).cuda(), sigma))
    ref = A.CV2.GaussianBlur(x, (0, 0), sigma)
    assert got.dtype == ref.dtype
    assert np.abs(got - ref).max() <= (1e-3 if dt == np.float32 else 1e-9)


@pytest.mark.gpu
def test_gpu_elastic_vs_oracle():
    GA = _gpu_aug()
    rng = np.random.RandomState(3)
    img = (rng.rand(50, 70) * 255).astype(np.float32)
    mask = (rng.rand(50, 70) > 0.5).astype(np.float32)
    r1, r2 = np.random.RandomState(9), np.random.RandomState(9)
    gi, gm = GA.elastic_transform(GA._dev(img), GA._dev(mask), alpha=15, sigma=3, rng=r1)
    oi, om = A.elastic_transform(img, mask, 15, 3, r2)
    assert r1.random() == r2.random()
    assert np.abs(_np(gi) - oi).max() <= 1e-3
    assert np.mean(_np(gm) != om) <= 1e-3    # rounding of maps that land exactly on .5 may differ


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["random", "ties", "const", "small", "large"])
def test_gpu_percentile_normalize_exact(case):
    GA = _gpu_aug()
    rng = np.random.default_rng(7)
    if case == "random":
        x = (rng.random((128, 128)) * 255).astype(np.float32)
    elif case == "ties":
        x = rng.integers(0, 6, (100, 77)).astype(np.float32) * 17.0
    elif case == "const":
        x = np.full((31, 33), 42.0, np.float32)
    elif case == "small":
        x = np.array([[3.0, -1.0, 2.5]], np.float32)
    else:
        x = (rng.standard_normal((1024, 1024)) * 40 + 200).astype(np.float32)
    got = _np(GA.normalize_percentile(x))
    np.testing.assert_array_equal(got, A.normalize_percentile_np123(x))


@pytest.mark.gpu
def test_gpu_zscore_and_tile_feed(tmp_path):
    """GPU feed of TileDataset: per-tile augmentation + normalisation on the device, batches as device
    tensors; with a seeded RandomState it equals the oracle pipeline + numpy normalisation."""
    GA = _gpu_aug()
    x = (np.random.default_rng(4).random((32, 40)) * 255).astype(np.float32)
    np.testing.assert_array_equal(_np(GA.normalize_zscore(x, 123.4, 56.7)),
                                  ((x - np.float32(123.4)) / np.float32(56.7 + 1e-10)).astype(np.float32))
    from adipose_amd.data import TileDataset, write_synthetic_build
    build = write_synthetic_build(tmp_path / "b", n_train=3, n_val=1, size=64, seed=2)
    kw = dict(normalization_method="percentile", seed=11)
    gds = TileDataset(build / "dataset" / "train" / "images", build / "dataset" / "train" / "masks", 2,
                      augment=True, augment_fn=GA.augment_pair_moderate, device="cuda", **kw)
    xb, yb = next(gds.generator())
    assert isinstance(xb, torch.Tensor) and xb.is_cuda and tuple(xb.shape) == (2, 64, 64)
    # host replay with the same seed: shuffle, load, oracle augmentation, numpy-1.23 percentile
    rng = np.random.RandomState(11)
    idx = np.arange(len(gds.pairs))
    rng.shuffle(idx)
    for b, j in enumerate(idx[:2]):
        img, mask = gds.load_pair(*gds.pairs[j])
        oi, om = A.augment_pair_moderate(img, mask, rng)
        assert np.abs(_np(xb[b]) - A.normalize_percentile_np123(oi)).max() <= 1e-4
        np.testing.assert_array_equal(_np(yb[b]), om)
