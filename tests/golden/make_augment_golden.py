"""Golden vectors for the training-time augmentations (src/utils/data.py:13-264), generated HERE from the
reference's own functions (cv2 is absent: it is replaced by a recording stub, see below). Data only is
written (tests/golden/augment.npz); no reference source is stored. Usage:
    python tests/golden/make_augment_golden.py [/root/reference]

  * numpy-only functions, pixel-exact: random_rotation_90, random_flip, random_brightness,
    random_contrast, random_gamma, random_gaussian_noise, and the whole augment_pair_light pipeline;
  * moderate / heavy pipelines: the sequence of cv2 calls they make (function, sigma / dsize / maps'
    shape) and the next value of the RandomState after the pipeline, per seed -- i.e. the order and
    number of random draws, which pins the host-side parameter stream of the GPU pipeline. The cv2 stub
    returns shape-correct placeholders (GaussianBlur: its input, resize: zeros of dsize, remap: its
    input), so the pixels of those two pipelines are NOT pinned here.
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402  (stub importer for tensorflow / cv2 / tifffile / skimage / seaborn)

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
CALLS = []


def recording_cv2():
    m = types.ModuleType("cv2")
    m.INTER_LINEAR, m.INTER_NEAREST, m.BORDER_REFLECT, m.BORDER_CONSTANT = 1, 0, 2, 0

    def GaussianBlur(src, ksize, sigma):
        CALLS.append(("GaussianBlur", float(sigma), tuple(np.shape(src))))
        return np.array(src, copy=True)

    def resize(src, dsize, interpolation=None):
        CALLS.append(("resize", tuple(int(v) for v in dsize), int(interpolation)))
        return np.zeros((dsize[1], dsize[0]), dtype=np.asarray(src).dtype)

    def remap(src, map1, map2, interpolation, borderMode=None, borderValue=None):
        CALLS.append(("remap", tuple(np.shape(map1)), int(interpolation)))
        return np.array(src, copy=True)

    m.GaussianBlur, m.resize, m.remap = GaussianBlur, resize, remap
    return m


def main():
    make_golden.REF = REF
    sys.modules["cv2"] = recording_cv2()
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    from src.utils import data as du  # noqa: E402

    out = {}
    base = np.random.RandomState(7)
    img = (base.rand(48, 64) * 255).astype(np.float32)
    mask = (base.rand(48, 64) > 0.6).astype(np.float32)
    out["image"], out["mask"] = img, mask
    for s in range(6):
        r = np.random.RandomState(100 + s)
        a, b = du.random_rotation_90(img, mask, r)
        a, b = du.random_flip(a, b, r)
        out[f"geom_{s}_img"], out[f"geom_{s}_mask"] = np.ascontiguousarray(a), np.ascontiguousarray(b)
        out[f"bright_{s}"] = np.asarray(du.random_brightness(img, (0.7, 1.3), r))
        out[f"contrast_{s}"] = np.asarray(du.random_contrast(img, (0.7, 1.3), r))
        out[f"gamma_{s}"] = np.asarray(du.random_gamma(img, (0.7, 1.3), r))
        out[f"noise_{s}"] = np.asarray(du.random_gaussian_noise(img, (0, 10), 1.0, r))
        out[f"next_{s}"] = np.float64(r.random())
        r = np.random.RandomState(200 + s)
        li, lm = du.augment_pair_light(img, mask, r)
        out[f"light_{s}_img"], out[f"light_{s}_mask"], out[f"light_{s}_next"] = li, lm, np.float64(r.random())
    # draw sequences of the moderate / heavy pipelines
    for name in ("moderate", "heavy", "tta_style"):
        fn = getattr(du, f"augment_pair_{name}")
        for s in range(40):
            CALLS.clear()
            r = np.random.RandomState(1000 + s)
            fn(img, mask, r)
            out[f"{name}_{s}_next"] = np.float64(r.random())
            out[f"{name}_{s}_calls"] = np.array([repr(c) for c in CALLS])
    np.savez_compressed(os.path.join(HERE, "augment.npz"), **out)
    print("wrote", os.path.join(HERE, "augment.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
