"""Weight files.

Reference: Keras 2.13 ``save_weights`` to ``*.weights.h5`` (weights-only HDF5, saving_lib layout
``/layers/<layer_name>/vars/{0: kernel HWIO, 1: bias}``), e.g. train_adipose_unet_v3.py:918-922, loaded by
full_evaluation_enhanced.py:1266-1301; legacy hdf5_format ``*.h5`` files (``layer_names`` /
``weight_names`` attributes) for the v2 pretrained weights (train_adipose_unet_v3.py:881-916).
h5py is not installed on this image: both layouts are read and written by h5io.py (a pure-Python HDF5
subset pinned against libhdf5-written files), so this build writes genuine ``*.weights.h5`` files under
the reference's names. ``*.weights.safetensors`` (same ``layers/<name>/vars/<i>`` tensor names,
earlier builds of this engine) is still read and can still be written.
"""
from __future__ import annotations

import json
import os
from collections import OrderedDict

import numpy as np

from . import h5io

SUFFIX = ".weights.h5"                      # what this build writes (the reference's own suffix)
ALT_SUFFIXES = (".weights.h5", ".weights.safetensors")


def _name(layer, i):
    return f"layers/{layer}/vars/{i}"


def save_weights(net, path, weights=None):
    """``*.weights.h5`` -> Keras 2.13 layout; other ``*.h5`` -> legacy hdf5_format layout;
    ``*.safetensors`` -> safetensors with Keras tensor names."""
    wd = weights if weights is not None else net.get_weights()
    wd = OrderedDict((k, [np.ascontiguousarray(np.asarray(a, np.float32)) for a in v]) for k, v in wd.items())
    path = str(path)
    if path.endswith(".safetensors"):
        from safetensors.numpy import save_file
        tensors = {_name(layer, i): a for layer, arrs in wd.items() for i, a in enumerate(arrs)}
        meta = {"format": "adipose_amd/keras-weights", "preset": getattr(net, "preset", ""),
                "layers": json.dumps(list(wd.keys()))}
        save_file(tensors, path, metadata=meta)
        return path
    if path.endswith(".h5"):
        return h5io.write_keras_weights(path, wd, fmt="keras_v3" if path.endswith(".weights.h5") else "legacy")
    raise ValueError(f"{path}: weight files end in .weights.h5, .h5 or .safetensors")


def read_weights(path):
    """-> OrderedDict layer -> [arrays] (Keras slot order) from any of the supported weight files."""
    path = str(path)
    if path.endswith(".h5"):
        return h5io.read_keras_weights(path)[1]
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
        for suf in ALT_SUFFIXES:
            p = os.path.join(path, n + suf)
            if os.path.exists(p):
                return p, path
    if os.path.isdir(path):
        for f in sorted(os.listdir(path)):
            if f.endswith(".safetensors") or f.endswith(".h5"):
                return os.path.join(path, f), path
    raise FileNotFoundError(f"No weights files found in {path}")
