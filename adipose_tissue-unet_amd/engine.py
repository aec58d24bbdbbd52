"""ctypes face of the handle-level C ABI (include/adipose_hip.h: adp_create / adp_set_param /
adp_forward / adp_destroy; csrc/engine.cpp): the native adipose_v3 inference engine, exposed with the
predictor seam's method surface (segmentation_inference.py:153-158 predict_single, :181-229 TTA) so that
it can stand in for AdiposeUNet. This is also the binding a non-Python caller would write.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from ._lib import AdpError, call, lib, ptr, stream_ptr

ADP_PRESET_ADIPOSE_V3 = 0
DTYPES = {"f32": 0, "bf16": 1}
TTA_MODES = {None: 0, "none": 0, "minimal": 1, "basic": 2, "full": 3}


class AdpConfig(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("preset", "tile", "max_batch", "dtype", "deep_supervision", "init_nb")]


class NativeAdiposeV3:
    """One adp_handle: build (topology + buffers) at construction, Keras-layout weights, batched TTA."""

    def __init__(self, tile=1024, max_batch=8, dtype="f32", deep_supervision=True, init_nb=44, device=0):
        self.tile, self.max_batch, self.device = tile, max_batch, torch.device("cuda", device)
        cfg = AdpConfig(ADP_PRESET_ADIPOSE_V3, tile, max_batch, DTYPES[dtype], int(deep_supervision), init_nb)
        h = C.c_void_p()
        call("adp_create", C.byref(cfg), device, C.byref(h))
        self._h = h

    def close(self):
        if self._h:
            lib().adp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 (interpreter shutdown)
            pass

    def layer_names(self):
        out, i = [], 0
        while True:
            n = lib().adp_param_name(self._h, i)
            if n is None:
                return out
            out.append(n.decode())
            i += 1

    def set_weights(self, weights):
        """weights: {keras layer name: [kernel, bias]} (e.g. checkpoint.read_weights of a .weights.h5);
        layers the engine does not have are skipped, like load_weights(by_name=True)."""
        names = set(self.layer_names())
        for layer, arrs in weights.items():
            if layer not in names:
                continue
            for slot, a in enumerate(arrs[:2]):
                a = np.ascontiguousarray(np.asarray(a, np.float32))
                call("adp_set_param", self._h, layer.encode(), slot, a.ctypes.data, a.size)

    def get_weights(self):
        out = {}
        for layer in self.layer_names():
            arrs = []
            for slot in (0, 1):
                n = C.c_size_t()
                call("adp_param_size", self._h, layer.encode(), slot, C.byref(n))
                a = np.empty(n.value, np.float32)
                call("adp_get_param", self._h, layer.encode(), slot, a.ctypes.data, a.size)
                arrs.append(a)
            out[layer] = arrs
        return out

    def predict_batch(self, images, mean, std, tta_mode=None):
        """images: (n, S, S) f32 (host or device) raw gray -> (n, S, S) device f32 probabilities."""
        x = images if isinstance(images, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(images, np.float32))
        x = x.to(self.device, torch.float32).contiguous()
        if x.dim() == 2:
            x = x[None]
        if tuple(x.shape[1:]) != (self.tile, self.tile):
            raise AdpError(f"engine built for {self.tile}x{self.tile} tiles, got {tuple(x.shape[1:])}")
        out = torch.empty_like(x)
        call("adp_forward", self._h, ptr(x), x.shape[0], x.shape[1] * x.shape[2], float(mean), float(std),
             TTA_MODES[tta_mode], ptr(out), stream_ptr())
        return out

    def predict_single(self, image, mean, std):
        """segmentation_inference.py:153-158: new float32 numpy (S, S) array."""
        return self.predict_batch(image, mean, std)[0].cpu().numpy()
