"""ctypes binding of ``libadipose_hip.so`` (the C ABI declared in ``include/adipose_hip.h``).

The shared library is built in-tree (``adipose_tissue-unet_amd/libadipose_hip.so``) and is the ONLY
compute path of this package: there is no CPU or PyTorch fallback. ``lib()`` raises if the library
is missing, and every wrapped call raises ``AdpError`` with ``adp_last_error()`` when the C side
reports a failure.

``torch`` is imported first on purpose: torch ships its own ``libamdhip64.so.7`` and the dynamic
linker then resolves this library's ``libamdhip64.so.7`` dependency to that same runtime, so
device pointers and ``hipStream_t`` handles from torch are valid here.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ADP_LIB_PATH") or os.path.join(PKG_DIR, "libadipose_hip.so")  # override: A/B timing only

F32 = 0
BF16 = 1
FP8 = 2   # OCP e4m3fn (torch.float8_e4m3fn storage), forward launches only
ABI_VERSION = 21


class AdpError(RuntimeError):
    pass


class ConvDesc(C.Structure):
    _fields_ = [(n, C.c_int) for n in (
        "N", "Hs", "Ws", "CA_stride", "CB_stride", "upsample", "Ho", "Wo", "stride",
        "kh", "kw", "dil", "pad", "Nout", "relu")] + [
        ("dropout_rate", C.c_float), ("dropout_seed", C.c_uint),
        ("out_stride", C.c_int), ("out_mode", C.c_int), ("shuffle_c", C.c_int),
        ("out2_stride", C.c_int), ("split_c", C.c_int),
        ("mask_stride", C.c_int), ("mask_scale", C.c_float),
        ("mask2_stride", C.c_int), ("mask2_scale", C.c_float),
        ("accum_stride", C.c_int), ("bnr_stride", C.c_int), ("out_fp8", C.c_int), ("bn_defer_fold", C.c_int),
        ("CA_real", C.c_int), ("CB_real", C.c_int), ("Nout_real", C.c_int)]


class ConvIO(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in (
        "srcA", "srcB", "bn_scaleA", "bn_shiftA", "bn_scaleB", "bn_shiftB", "W", "bias",
        "out", "out2", "addend", "mask", "mask2", "accum", "bn_sum", "bn_sqsum",
        "bnr_z", "bnr_scale", "bnr_shift", "bnr_mean", "bnr_invstd", "bnr_dgamma", "bnr_dbeta", "w_scale",
        "act_outA")]


class BnBwdArgs(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in (
        "dA", "z", "scale", "shift", "mean", "invstd", "gamma", "dgamma", "dbeta")] + [("count", C.c_float)]


_P = C.c_void_p
_I = C.c_int
_F = C.c_float
_S = C.c_size_t

# name -> argtypes (restype is always c_int)
_SIGS = {
    "adp_abi_version": [],
    "adp_set_option": [C.c_char_p, _I],
    "adp_timing": [_I],
    "adp_timing_filter": [C.c_char_p],
    "adp_timing_read": [_I, C.c_char_p, _I, C.POINTER(C.c_float), C.POINTER(C.c_int)],
    "adp_conv_fwd": [_I, C.POINTER(ConvDesc), C.POINTER(ConvIO), _P],
    "adp_conv_wgrad": [_I, C.POINTER(ConvDesc), C.POINTER(ConvIO), _P, _I, _P, _P, _P],
    "adp_conv_wgrad_bn": [_I, C.POINTER(ConvDesc), C.POINTER(ConvIO), C.POINTER(BnBwdArgs), _P, _I, _P, _P, _P],
    "adp_pack_weights": [_I, _I, _I, _I, _I, _P, _I, _P, _I, _I, _P],
    "adp_maxpool2_fwd": [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P],
    "adp_maxpool2_fwd_fp8": [_I, _I, _I, _I, _I, _P, _P, _P],
    "adp_pack_weights_fp8": [_I, _P, _I, _P, _I, _P, _P],
    "adp_bn_apply_fp8": [_I, _S, _I, _P, _P, _P, _P, _P],
    "adp_vec_mul": [_S, _P, _P, _P, _P],
    "adp_scale_rows": [_I, _I, _I, _P, _I, _P, _I, _P, _I, _P],
    "adp_maxpool2_bwd": [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _F, _P, _P],
    "adp_maxpool2_bwd_bnr": [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "adp_upsample2_bwd": [_I, _I, _I, _I, _I, _P, _P, _P, _F, _P, _P],
    "adp_ew_add_mask": [_I, _S, _P, _P, _P, _F, _P, _P],
    "adp_cast": [_I, _I, _S, _P, _P, _P],
    "adp_fill_f32": [_S, _F, _P, _P],
    "adp_sum_bf16": [_I, _P, _S, _P, _P],
    "adp_bn_finalize": [_I, _F, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P, _P],
    "adp_bn_finalize_fold": [_I, _F, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P, _P],
    "adp_bn_fold_reset": [_P],
    "adp_wgrad_defer": [_I, _P],
    "adp_wgrad_flush": [_P],
    "adp_wgrad_release": [_P],
    "adp_get_option": [C.c_char_p],
    "adp_wgrad_arena_chunks": [_P],
    "adp_debug_grad_flat": [_P, _I, _P, _S],
    "adp_bn_apply": [_I, _S, _I, _P, _P, _P, _P, _P],
    "adp_bn_bwd_reduce":[_I, _S, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "adp_bn_bwd_apply": [_I, _S, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _F, _P, _P],
    "adp_bn_bwd_apply_head": [_I, _S, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _F, _P, _P],
    "adp_head_softmax2_fwd": [_I, _S, _I, _I, _P, _P, _P, _P, _P, _P, _P],
    "adp_head_softmax2_bwd": [_I, _S, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _F, _P, _P, _P, _P],
    "adp_head_sigmoid_fwd": [_I, _S, _I, _I, _P, _P, _P, _P, _P, _P, _P],
    "adp_head_sigmoid_bwd": [_I, _S, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _F, _P, _P, _P, _P],
    "adp_resize_bilinear_fwd": [_I, _I, _I, _I, _I, _P, _P, _P],
    "adp_resize_bilinear_bwd": [_I, _I, _I, _I, _I, _P, _P, _P],
    "adp_loss_rows": [_I, _I, _I, _P, _P, _I, _F, _F, _P, _P, _P],
    "adp_loss_select": [_I, _I, _I, _P, _I, _F, _F, _F, _P, _P, _P],
    "adp_loss_grad": [_I, _I, _I, _P, _P, _I, _F, _F, _P, _P, _F, _I, _P, _P],
    "adp_pixel_counts": [_S, _P, _P, _F, _P, _P],
    "adp_threshold_hist": [_S, _P, _P, _I, C.POINTER(C.c_double), _P, _P],
    "adp_aug_geom": [_I, _I, _P, _P, _I, _I, _I, _P],
    "adp_aug_photometric": [_S, _P, _P, _I, _F, _F, _P],
    "adp_aug_noise": [_S, _P, _P, _P, _P],
    "adp_aug_sum": [_S, _P, _P, _P],
    "adp_aug_blur": [_I, _I, _I, _P, _P, _P, _P, _I, _P],
    "adp_aug_scale": [_I, _I, _I, _I, _P, _P, _I, _P],
    "adp_aug_remap": [_I, _I, _P, _P, _P, _P, C.c_double, _P, _P, _P],
    "adp_percentile_normalize": [_S, _P, _P, C.c_double, C.c_double, _P, _P, _P],
    "adp_create": [_P, _I, _P],
    "adp_destroy": [_P],
    "adp_param_size": [_P, C.c_char_p, _I, C.POINTER(C.c_size_t)],
    "adp_set_param": [_P, C.c_char_p, _I, _P, _S],
    "adp_get_param": [_P, C.c_char_p, _I, _P, _S],
    "adp_get_grad": [_P, C.c_char_p, _I, _P, _S],
    "adp_forward": [_P, _P, _I, C.c_longlong, _F, _F, _I, _P, _P],
    "adp_train_step": [_P, _P, _P, _I, _P, _F, _P, _P],
    "adp_auc_metrics": [_S, _P, _P, _P, _P],
    "adp_border_weight": [_I, _I, _I, _I, _P, _P, _P, _P, _P],
    "adp_weighted_loss_stats": [_S, _P, _P, _P, _P, _P, _P],
    "adp_weighted_loss_grad": [_S, _P, _P, _P, _P, _P, _F, _F, _P, _P],
    "adp_value_stats": [_S, _P, _P, _P, _P],
    "adp_onehot_counts": [_I, _I, _P, _P, _P, _P],
    "adp_boundary_refine": [_I, _I, _P, _I, C.POINTER(C.c_int), C.POINTER(C.c_int), _I, _F, _F, _P, _P, _P],
    "adp_pack_weights_batch": [_I, _I, _P, _P],
    "adp_bn_apply_maxpool2": [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P],
    "adp_head_sigmoid_bwd_bnr": [_I, _S, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "adp_distance_transform": [_I, _I, _P, _F, C.c_double, C.c_double, _P, _P],
    "adp_boundary_metrics": [_I, _I, _P, _P, _F, C.c_double, C.c_double, _P, _P],
    "adp_set_comm": [_P, _P],
    "adp_comm_unique_id": [_P],
    "adp_comm_init": [_I, _P, _I, _P],
    "adp_comm_destroy": [_P],
    "adp_adam": [_S, _P, _P, _P, _P, _F, _F, _F, _F, _I, _F, _F, _P],
    "adp_ema": [_S, _P, _P, _F, _P],
    "adp_prep_input": [_I, _I, _I, _I, _I, _P, C.c_longlong, C.c_longlong, _F, _F, _I, _I, _P, _P],
    "adp_tta_merge": [_I, _I, _I, C.POINTER(C.c_int), _P, _P, _P],
    "adp_blend_accum": [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P],
    "adp_blend_finalize": [_S, _P, _P, _F, _P, _P],
}

_lib = None
CSRC = os.path.join(PKG_DIR, "csrc")


def exported_symbols():
    return ["adp_last_error", "adp_last_kernel", "adp_param_name", "adp_source_hash"] + list(_SIGS)


def source_hash():
    """sha256 of the sources the Makefile hashes into the library's build record (same files, same order),
    or None when the sources are not beside the package."""
    import hashlib
    import re
    mk = os.path.join(CSRC, "Makefile")
    if not os.path.exists(mk):
        return None
    text = open(mk).read()
    srcs = re.search(r"^SRCS = (.*)$", text, re.M).group(1).split()
    hashed = re.search(r"^HASHED = (.*)$", text, re.M).group(1).split()
    files = [f for h in hashed for f in (srcs if h == "$(SRCS)" else [h])]
    h = hashlib.sha256()
    for f in files:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def lib():
    """Load (once) and return the CDLL. Raises if the HIP extension has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise AdpError(
                f"libadipose_hip.so not found at {LIB_PATH}; run __graft_entry__.build() "
                "(make -C adipose_tissue-unet_amd/csrc). There is no CPU fallback.")
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        L.adp_last_error.restype = C.c_char_p
        L.adp_last_error.argtypes = []
        L.adp_last_kernel.restype = C.c_char_p
        L.adp_last_kernel.argtypes = []
        L.adp_param_name.restype = C.c_char_p
        L.adp_param_name.argtypes = [C.c_void_p, C.c_int]
        L.adp_source_hash.restype = C.c_char_p
        L.adp_source_hash.argtypes = []
        for name, args in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = C.c_int
            fn.argtypes = args
        if L.adp_abi_version() != ABI_VERSION:
            raise AdpError(f"{LIB_PATH}: ABI version {L.adp_abi_version()} != {ABI_VERSION}; rebuild the library")
        # the build record ties the binary to the sources beside it (a stale library is refused)
        want = source_hash()
        got = L.adp_source_hash().decode()
        if want is not None and got != want and not os.environ.get("ADP_LIB_PATH"):
            raise AdpError(f"{LIB_PATH} was built from other sources (record {got[:16]}, tree {want[:16]}); "
                           "rebuild it: make -C adipose_tissue-unet_amd/csrc")
        _lib = L
    return _lib


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise AdpError(f"{name} failed ({rc}): {lib().adp_last_error().decode()}")
    return rc


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def ptr(t):
    """Device pointer of a tensor (or None -> NULL)."""
    if t is None:
        return None
    return C.c_void_p(t.data_ptr())
