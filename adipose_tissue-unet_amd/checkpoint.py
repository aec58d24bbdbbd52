"""Weight files.

Reference: Keras 2.13 ``save_weights`` to ``*.weights.h5`` (weights-only HDF5; per layer
``layers/<layer_name>/vars/{0: kernel HWIO, 1: bias}``), e.g. train_adipose_unet_v3.py:918-922,
loaded by full_evaluation_enhanced.py:1266-1301. h5py is not installed on this image, so weights are
stored with the same names and slot order in a safetensors container (``*.weights.safetensors``);
genuine ``.weights.h5`` files are read when h5py is importable. Tensor name:
``layers/<layer_name>/vars/<slot>``; metadata carries the preset and topology.
"""
from __future__ import annotations

import json
import os

import numpy as np

SUFFIX = ".weights.safetensors"


def _name(layer, i):
    return f"layers/{layer}/vars/{i}"


def save_weights(net, path, weights=None):
    from safetensors.numpy import save_file

    wd = weights if weights is not None else net.get_weights()
    tensors = {}
    for layer, arrs in wd.items():
        for i, a in enumerate(arrs):
            tensors[_name(layer, i)] = np.ascontiguousarray(np.asarray(a, np.float32))
    meta = {"format": "adipose_amd/keras-weights", "preset": getattr(net, "preset", ""),
            "layers": json.dumps(list(wd.keys()))}
    save_file(tensors, path, metadata=meta)
    return path


def read_weights(path):
    """-> OrderedDict layer -> [arrays] from a .weights.safetensors (or .weights.h5 if h5py exists)."""
    from collections import OrderedDict

    if path.endswith(".h5"):
        try:
            import h5py  # noqa: F401
        except ImportError as e:
            raise RuntimeError(f"{path}: reading Keras HDF5 weights needs h5py, which is not installed; "
                               f"convert to {SUFFIX}") from e
        return _read_h5(path)
    from safetensors import safe_open

    out = OrderedDict()
    with safe_open(path, framework="numpy") as f:
        meta = f.metadata() or {}
        order = json.loads(meta.get("layers", "[]"))
        keys = list(f.keys())
        layers = order or sorted({k.split("/")[1] for k in keys})
        for layer in layers:
            arrs = []
            i = 0
            while _name(layer, i) in keys:
                arrs.append(f.get_tensor(_name(layer, i)))
                i += 1
            out[layer] = arrs
    return out


def _read_h5(path):
    import h5py
    from collections import OrderedDict

    out = OrderedDict()
    with h5py.File(path, "r") as f:
        root = f["layers"] if "layers" in f else f
        for layer in root:
            g = root[layer]
            if "vars" in g:
                v = g["vars"]
                out[layer] = [np.asarray(v[str(i)]) for i in range(len(v))]
    return out


def load_weights(net, path, by_name=True, skip_mismatch=False):
    wd = read_weights(path)
    for layer, arrs in wd.items():
        if layer not in net.layers:
            if by_name:
                continue
            raise KeyError(f"unknown layer {layer}")
        try:
            net.set_layer_weights(layer, arrs)
        except ValueError:
            if not skip_mismatch:
                raise
    return net


def resolve_weights_file(path):
    """Directory -> best candidate file (segmentation_inference.py:252-285 order, our suffix first)."""
    if os.path.isfile(path):
        return path, os.path.dirname(path)
    names = ["weights_best_overall", "phase2_best", "phase1_best", "best_model", "model_best", "weights_best",
             "weights_ema"]
    for n in names:
        for suf in (SUFFIX, ".weights.h5"):
            p = os.path.join(path, n + suf)
            if os.path.exists(p):
                return p, path
    if os.path.isdir(path):
        for f in sorted(os.listdir(path)):
            if f.endswith(SUFFIX) or f.endswith(".h5"):
                return os.path.join(path, f), path
    raise FileNotFoundError(f"No weights files found in {path}")
