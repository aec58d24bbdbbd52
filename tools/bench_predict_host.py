#!/usr/bin/env python3
"""PCIe-inclusive rate of the drop-in predictor boundary: AdiposeUNet.predict_single(image, mean, std) and
predict(..., use_tta=True, tta_mode='full') with host numpy in / host numpy out, one 1024^2 tile per call as
the reference's callers issue them (segmentation_inference.py:153-158, full_evaluation_enhanced.py:1323-1353).
Random Keras-default weights (seed 865), bf16 inference layout. Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import _adipose_pkg  # noqa: F401
    from adipose_amd.predictor import AdiposeUNet
    m = AdiposeUNet(tile_size=1024, dtype="bf16", device="cuda")
    m.build_model()
    rng = np.random.default_rng(865)
    imgs = [rng.uniform(0, 255, (1024, 1024)).astype(np.float32) for _ in range(4)]
    res = {}
    for name, fn, n in (("predict_single", lambda im: m.predict_single(im, 200.0, 25.0), 40),
                        ("predict_tta_full", lambda im: m.predict(im, 200.0, 25.0, use_tta=True, tta_mode="full")[0], 10)):
        for i in range(3):
            fn(imgs[i % 4])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            out = fn(imgs[i % 4])
        t1 = time.perf_counter()
        assert out.shape == (1024, 1024) and out.dtype == np.float32
        res[name] = {"calls": n, "ms_per_call": round((t1 - t0) / n * 1e3, 3), "tiles_per_s": round(n / (t1 - t0), 2)}
    print(json.dumps({"boundary": "AdiposeUNet host numpy in/out, 1024^2, bf16, 1 GPU, PCIe-inclusive", **res}))


if __name__ == "__main__":
    main()
