"""ctypes face of the handle-level C ABI (include/adipose_hip.h: adp_create / adp_set_param /
adp_forward / adp_train_step / adp_set_comm / adp_destroy; csrc/engine.cpp): the native adipose_v3
engine, exposed with the predictor seam's method surface (segmentation_inference.py:153-158
predict_single, :181-229 TTA) so that it can stand in for AdiposeUNet, plus a native training step
(model.net.fit's step, train_adipose_unet_v3.py:1316-1324 with compile_model's losses :780-879). This is
also the binding a non-Python caller would write.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from ._lib import AdpError, call, lib, ptr, stream_ptr

ADP_PRESET_ADIPOSE_V3 = 0
ADP_PRESET_UNET_BN = 1
DTYPES = {"f32": 0, "bf16": 1}
TTA_MODES = {None: 0, "none": 0, "minimal": 1, "basic": 2, "full": 3}


class AdpConfig(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("preset", "tile", "max_batch", "dtype", "deep_supervision", "init_nb",
                                       "levels", "base", "in_ch")] + [("dropout_rate", C.c_float),
                                                                      ("seed", C.c_uint)]


class AdpTrainCfg(C.Structure):
    _fields_ = [("use_hard_mining", C.c_int), ("hard_example_ratio", C.c_float), ("use_label_smoothing", C.c_int),
                ("epsilon_pos", C.c_float), ("epsilon_neg", C.c_float), ("w_main", C.c_float),
                ("w_aux1", C.c_float), ("w_aux2", C.c_float), ("optimizer", C.c_int), ("beta1", C.c_float),
                ("beta2", C.c_float), ("eps", C.c_float), ("weight_decay", C.c_float), ("dropout_rate", C.c_float),
                ("freeze_encoder", C.c_int)]


METRIC_NAMES = ("loss", "main_out_loss", "aux_out1_loss", "aux_out2_loss", "main_out_dice_coef",
                "main_out_binary_accuracy")


def train_cfg(*, use_hard_mining=True, hard_example_ratio=0.7, use_label_smoothing=False, epsilon_pos=0.03,
              epsilon_neg=0.07, ds_weight_main=1.0, ds_weight_aux1=0.4, ds_weight_aux2=0.3, optimizer="adam",
              beta1=0.9, beta2=0.999, eps=1e-7, weight_decay=0.01, dropout_rate=0.3, freeze_encoder=False):
    """compile_model's defaults (train_adipose_unet_v3.py:780-879) as an adp_train_cfg."""
    return AdpTrainCfg(int(use_hard_mining), hard_example_ratio, int(use_label_smoothing), epsilon_pos, epsilon_neg,
                       ds_weight_main, ds_weight_aux1, ds_weight_aux2, 1 if optimizer.lower() == "adamw" else 0,
                       beta1, beta2, eps, weight_decay, dropout_rate, int(freeze_encoder))


def comm_unique_id():
    """128-byte RCCL unique id (rank 0 creates it and shares it, e.g. through torch.distributed)."""
    buf = (C.c_char * 128)()
    call("adp_comm_unique_id", buf)
    return bytes(buf)


def comm_init(nranks, uid, rank):
    buf = (C.c_char * 128).from_buffer_copy(uid)
    comm = C.c_void_p()
    call("adp_comm_init", nranks, buf, rank, C.byref(comm))
    return comm


def comm_destroy(comm):
    call("adp_comm_destroy", comm)


class NativeAdiposeV3:
    """One adp_handle: build (topology + buffers) at construction, Keras-layout weights, batched TTA."""

    in_ch = 1
    nslots = 2

    def __init__(self, tile=1024, max_batch=8, dtype="f32", deep_supervision=True, init_nb=44, device=0,
                 dropout_rate=0.3, seed=0):
        self.tile, self.max_batch, self.device = tile, max_batch, torch.device("cuda", device)
        cfg = AdpConfig(ADP_PRESET_ADIPOSE_V3, tile, max_batch, DTYPES[dtype], int(deep_supervision), init_nb,
                        0, 0, 0, float(dropout_rate), int(seed))
        self._create(cfg, device)

    def _create(self, cfg, device):
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
            for slot, a in enumerate(arrs[:self.nslots]):
                a = np.ascontiguousarray(np.asarray(a, np.float32))
                call("adp_set_param", self._h, layer.encode(), slot, a.ctypes.data, a.size)

    def _slots(self, layer):
        return (0, 1)

    def get_weights(self):
        out = {}
        for layer in self.layer_names():
            arrs = []
            for slot in self._slots(layer):
                n = C.c_size_t()
                call("adp_param_size", self._h, layer.encode(), slot, C.byref(n))
                a = np.empty(n.value, np.float32)
                call("adp_get_param", self._h, layer.encode(), slot, a.ctypes.data, a.size)
                arrs.append(a)
            out[layer] = arrs
        return out

    def _tiles(self, images):
        x = images if isinstance(images, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(images, np.float32))
        x = x.to(self.device, torch.float32).contiguous()
        shape = (self.tile, self.tile) if self.in_ch == 1 else (self.tile, self.tile, self.in_ch)
        if x.dim() == len(shape):
            x = x[None]
        if tuple(x.shape[1:]) != shape:
            raise AdpError(f"engine built for {shape} tiles, got {tuple(x.shape[1:])}")
        return x

    def get_grads(self):
        """The last train_step's gradients, {layer: [kernel grad, bias / gamma / beta grads ...]} (Keras layout)."""
        out = {}
        for layer in self.layer_names():
            arrs = []
            for slot in self._slots(layer):
                n = C.c_size_t()
                call("adp_param_size", self._h, layer.encode(), slot, C.byref(n))
                a = np.empty(n.value, np.float32)
                call("adp_get_grad", self._h, layer.encode(), slot, a.ctypes.data, a.size)
                arrs.append(a)
            out[layer] = arrs
        return out

    def predict_batch(self, images, mean, std, tta_mode=None):
        """images: (n, S, S) f32 raw gray (unet_bn: (n, S, S, in_ch)), host or device -> (n, S, S) device f32
        probabilities."""
        x = self._tiles(images)
        out = torch.empty((x.shape[0], self.tile, self.tile), dtype=torch.float32, device=self.device)
        call("adp_forward", self._h, ptr(x), x.shape[0], x[0].numel(), float(mean), float(std),
             TTA_MODES[tta_mode], ptr(out), stream_ptr())
        return out

    def predict_single(self, image, mean, std):
        """segmentation_inference.py:153-158: new float32 numpy (S, S) array."""
        return self.predict_batch(image, mean, std)[0].cpu().numpy()

    # ------------------------------------------------------------------------------ training
    def set_comm(self, comm):
        """Attach an RCCL communicator (comm_init) for data-parallel steps; None detaches."""
        call("adp_set_comm", self._h, comm)

    def train_step(self, x, y, lr, cfg=None):
        """One native training step: x (n, S, S) normalised images, y (n, S, S) labels (host or device).
        Returns the Keras per-batch metrics (METRIC_NAMES)."""
        cfg = cfg or train_cfg()
        xd = self._tiles(x)
        yt = y if isinstance(y, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(y, np.float32))
        yd = yt.to(self.device, torch.float32).contiguous()
        if yd.dim() == 2:
            yd = yd[None]
        if tuple(yd.shape) != (xd.shape[0], self.tile, self.tile):
            raise AdpError(f"labels {tuple(yd.shape)} do not match {xd.shape[0]} tiles of {self.tile}^2")
        m = (C.c_float * 6)()
        call("adp_train_step", self._h, ptr(xd), ptr(yd), xd.shape[0], C.byref(cfg), float(lr), m, stream_ptr())
        return dict(zip(METRIC_NAMES, (float(v) for v in m)))


class NativeUNetBN(NativeAdiposeV3):
    """The unet_bn preset behind the same handle ABI (BASELINE.json configs 2/3/5; nets.UNetBN is the Python
    schedule of the same network): Keras-style weights per layer ([kernel, gamma, beta] for the conv + BatchNorm
    layers, as nets.UNetBN.get_weights returns them, plus slots 3 / 4 = moving mean / variance; [kernel, bias]
    for the ConvTranspose layers (torch (Cin, Cout, 2, 2) layout) and the head)."""

    nslots = 3

    def __init__(self, tile=1024, max_batch=4, dtype="bf16", levels=5, base=64, in_ch=3, device=0, seed=0):
        self.tile, self.max_batch, self.device = tile, max_batch, torch.device("cuda", device)
        self.in_ch = in_ch
        cfg = AdpConfig(ADP_PRESET_UNET_BN, tile, max_batch, DTYPES[dtype], 0, 0, levels, base, in_ch, 0.0, int(seed))
        self._create(cfg, device)

    def _slots(self, layer):
        return (0, 1, 2) if ("_conv" in layer) else (0, 1)

    def set_running_stats(self, layer, mean, var):
        """Set the moving mean / variance (slots 3, 4) of a conv + BatchNorm layer (e.g. from a checkpoint)."""
        for slot, a in ((3, mean), (4, var)):
            a = np.ascontiguousarray(np.asarray(a, np.float32))
            call("adp_set_param", self._h, layer.encode(), slot, a.ctypes.data, a.size)

    def running_stats(self, layer):
        """(moving mean, moving variance) of a conv + BatchNorm layer (slots 3, 4)."""
        out = []
        for slot in (3, 4):
            n = C.c_size_t()
            call("adp_param_size", self._h, layer.encode(), slot, C.byref(n))
            a = np.empty(n.value, np.float32)
            call("adp_get_param", self._h, layer.encode(), slot, a.ctypes.data, a.size)
            out.append(a)
        return out
