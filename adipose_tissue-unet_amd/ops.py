"""Thin, shape-checked Python wrappers over the libadipose_hip C ABI.

Tensors are torch device tensors used purely as memory (no torch compute runs on the hot path);
every function here validates operand shapes on the host before launching, then calls exactly one
C-ABI entry point on the current torch stream.

Activation tensors are NHWC ``(N, H, W, Cs)`` with ``Cs % 8 == 0``; packed GEMM weights are
``(Npad, Kpad)`` (see include/adipose_hip.h).
"""
from __future__ import annotations

import ctypes as C

import torch

from ._lib import BF16, F32, FP8, AdpError, BnBwdArgs, ConvDesc, ConvIO, call, lib, ptr, stream_ptr

FP8_DTYPE = torch.float8_e4m3fn   # storage dtype of the fp8 (OCP e4m3fn) inference tensors


def round_up(x, m):
    return (x + m - 1) // m * m


class LaunchTimer:
    """Optional per-launch timing of the conv kernels (bench.py roofline leg).

    The library brackets the MAIN kernel of every adp_conv_fwd / adp_conv_wgrad(_bn) call with a HIP
    event pair on the launch stream (adp_timing): the statistic folds, split reduces, bias sums and
    BatchNorm applies a call may launch around it are outside the pair, so each timing is exactly one
    kernel of rocprofv3's list, under the name the library reports for it (adp_last_kernel). The wrapper
    records, per call and in the same order, the launch dtype and its algorithmic FLOPs and bytes."""

    NAME_LEN = 160

    def __init__(self, only=None):
        """only: a kernel name (as adp_last_kernel reports it): record that kernel's launches alone
        (adp_timing_filter), so the other launches of a timed region carry no event pair."""
        self.recs = []
        self.only = only

    def wrap(self, dcode, flops, fn, nbytes=0.0):
        fn()
        if self.only is None or lib().adp_last_kernel().decode() == self.only:
            self.recs.append((dcode, flops, nbytes))

    def summary(self):
        """(kernel name, dtype code) -> (launches, total flops, total ms, total algorithmic bytes)
        (synchronises; ends the library's recording)."""
        torch.cuda.synchronize()
        n = C.c_int(0)
        call("adp_timing_read", 0, None, 0, None, C.byref(n))
        cnt = n.value
        names = C.create_string_buffer(max(1, cnt) * self.NAME_LEN)
        ms = (C.c_float * max(1, cnt))()
        call("adp_timing_read", cnt, names, self.NAME_LEN, ms, C.byref(n))
        call("adp_timing", 2)
        _check(cnt == len(self.recs), f"LaunchTimer: {cnt} timed kernels for {len(self.recs)} conv calls")
        out = {}
        raw = names.raw
        for i, (dcode, f, nb) in enumerate(self.recs):
            name = raw[i * self.NAME_LEN:(i + 1) * self.NAME_LEN].split(b"\0", 1)[0].decode()
            _check(ms[i] >= 0, f"LaunchTimer: {name} has no end mark")
            k = (name, dcode)
            c, fl, t, b = out.get(k, (0, 0.0, 0.0, 0.0))
            out[k] = (c + 1, fl + f, t + ms[i], b + nb)
        return out


_timer = None


def set_launch_timer(t):
    """Start (t = a LaunchTimer) or stop (None) recording; the record is read by t.summary()."""
    global _timer
    _timer = t
    if t is not None:
        call("adp_timing_filter", t.only.encode() if t.only else None)
        call("adp_timing", 1)
    else:
        call("adp_timing", 0)
        call("adp_timing_filter", None)


def _timed(dcode, flops, fn, nbytes=0.0):
    if _timer is None:
        fn()
    else:
        _timer.wrap(dcode, flops, fn, nbytes)


def set_option(name, value):
    """Set a kernel-selection option of the native library (adp_set_option; see include/adipose_hip.h).
    value=None restores the built-in default."""
    call("adp_set_option", name.encode(), -(2 ** 31) if value is None else int(value))


def dtype_code(t):
    if t.dtype == torch.bfloat16:
        return BF16
    if t.dtype == torch.float32:
        return F32
    if t.dtype == FP8_DTYPE:
        return FP8
    raise AdpError(f"unsupported dtype {t.dtype}")


def _check(cond, msg):
    if not cond:
        raise AdpError(msg)


def _act(t, name):
    _check(t is not None and t.dim() == 4 and t.is_contiguous() and t.shape[3] % 8 == 0,
           f"{name}: expected contiguous NHWC tensor with C%8==0, got "
           f"{None if t is None else (tuple(t.shape), t.is_contiguous())}")
    _check(t.is_cuda, f"{name}: must be a device tensor")


def conv_geometry(Hs, Ws, *, up=False, stride=1, kh=3, kw=3, dil=1, pad=None, transpose_fwd=False):
    """Output grid of a gather-conv launch (None pad -> 'same' for odd kernels)."""
    if pad is None:
        pad = dil * (kh // 2)
    Hv, Wv = Hs * (2 if up else 1), Ws * (2 if up else 1)
    Ho = (Hv + 2 * pad - dil * (kh - 1) - 1) // stride + 1
    Wo = (Wv + 2 * pad - dil * (kw - 1) - 1) // stride + 1
    return Ho, Wo, pad


def _desc_io(srcA, W, srcB, bnA, bnB, bias, up, stride, kh, kw, dil, pad, Ho, Wo, nout):
    _act(srcA, "srcA")
    N, Hs, Ws, CA = srcA.shape
    CB = 0
    if srcB is not None:
        _act(srcB, "srcB")
        _check(tuple(srcB.shape[:3]) == (N, Hs, Ws) and srcB.dtype == srcA.dtype, "srcB shape/dtype mismatch")
        CB = srcB.shape[3]
    Ho_, Wo_, pad = conv_geometry(Hs, Ws, up=up, stride=stride, kh=kh, kw=kw, dil=dil, pad=pad)
    Ho = Ho_ if Ho is None else Ho
    Wo = Wo_ if Wo is None else Wo
    K = kh * kw * (CA + CB)
    Kpad = round_up(K, 32)
    _check(W.dtype == srcA.dtype and W.is_contiguous() and W.dim() == 2, "W dtype/layout mismatch")
    _check(W.shape[1] == Kpad and W.shape[0] >= round_up(nout, 64),
           f"W shape {tuple(W.shape)} != (>= {round_up(nout, 64)}, {Kpad})")
    d = ConvDesc()
    d.N, d.Hs, d.Ws, d.CA_stride, d.CB_stride = N, Hs, Ws, CA, CB
    d.upsample = 1 if up else 0
    d.Ho, d.Wo, d.stride = Ho, Wo, stride
    d.kh, d.kw, d.dil, d.pad = kh, kw, dil, pad
    d.Nout = nout
    d.mask_scale = 1.0
    d.mask2_scale = 1.0
    io = ConvIO()
    io.srcA, io.srcB = ptr(srcA), ptr(srcB)
    if bnA is not None:
        _check(bnA[0].numel() >= CA and bnA[1].numel() >= CA, "bnA vectors too short")
        io.bn_scaleA, io.bn_shiftA = ptr(bnA[0]), ptr(bnA[1])
    if bnB is not None:
        _check(bnB[0].numel() >= CB and bnB[1].numel() >= CB, "bnB vectors too short")
        io.bn_scaleB, io.bn_shiftB = ptr(bnB[0]), ptr(bnB[1])
    io.W = ptr(W)
    if bias is not None:
        _check(bias.dtype == torch.float32, "bias must be f32")
        io.bias = ptr(bias)
    return d, io, N, Ho, Wo


def conv_fwd(srcA, W, nout, *, out=None, srcB=None, bnA=None, bnB=None, bias=None, up=False, stride=1,
             kh=3, kw=3, dil=1, pad=None, Ho=None, Wo=None, relu=False, dropout_rate=0.0, dropout_seed=0,
             out_mode=0, shuffle_c=0, out2=None, split_c=0, addend=None, mask=None, mask_scale=1.0,
             mask2=None, mask2_scale=1.0, accum=None, bn_stats=None, bn_reduce=None, w_scale=None,
             defer_fold=False, act_out=None, real=None):
    """Implicit-GEMM conv forward-shaped launch (conv, conv dgrad, convT fwd/dgrad).

    real=(CA_real, CB_real, Nout_real) (optional hints, adp_conv_desc v19): the unpadded channel counts of the
    sources and of the GEMM columns whose pad weight columns / rows are zeros (every packed layer's are); the
    f32 tap kernel then skips the products with those zero weights (44-channel layers in 64-channel strides).

    bnA=(scale, shift) with act_out (one source): srcA is read pre-BatchNorm, relu(srcA*scale+shift) is what the
    conv multiplies and is also stored to act_out (adp_conv_io.act_outA: one launch on the persistent halo forward,
    else bn_apply + the launch; bit-identical to bn_apply(srcA) -> act_out, conv_fwd(act_out)).

    bn_reduce=(z, scale, shift, mean, invstd, dgamma, dbeta): fuse the BatchNorm-backward reduction
    (bn_bwd_reduce) of the layer whose activation relu(z*scale+shift) `out` is the gradient of.
    fp8 launches (srcA/W torch.float8_e4m3fn): w_scale (f32, per GEMM column, from pack_weights_fp8) is
    required; `out` may be bf16 or fp8.
    defer_fold (with bn_stats): leave the statistics in the library's accumulator replicas; the next call
    on the stream must be bn_finalize(..., fold=True) on the same two vectors."""
    d, io, N, Ho, Wo = _desc_io(srcA, W, srcB, bnA, bnB, bias, up, stride, kh, kw, dil, pad, Ho, Wo, nout)
    d.relu = 1 if relu else 0
    if real is not None:
        ca, cb, nr = (int(v) for v in real)
        _check(0 <= ca <= d.CA_stride and 0 <= cb <= d.CB_stride and 0 <= nr <= nout, "real channel counts out of range")
        d.CA_real, d.CB_real, d.Nout_real = ca, cb, nr
    d.dropout_rate = float(dropout_rate)
    d.dropout_seed = int(dropout_seed) & 0xFFFFFFFF
    d.out_mode = out_mode
    if out_mode == 1:
        _check(shuffle_c > 0 and nout % shuffle_c == 0, "pixel-shuffle needs nout % shuffle_c == 0")
        _check(out is not None and tuple(out.shape[:3]) == (N, 2 * Ho, 2 * Wo) and out.shape[3] >= shuffle_c,
               "convT output shape mismatch")
        d.shuffle_c = shuffle_c
    elif out_mode == 2:
        _check(out2 is not None and 0 < split_c < nout, "split store needs out2 and 0<split_c<nout")
        _act(out2, "out2")
        _check(tuple(out2.shape[:3]) == (N, Ho, Wo) and out2.shape[3] >= nout - split_c, "out2 shape mismatch")
        d.out2_stride, d.split_c = out2.shape[3], split_c
        io.out2 = ptr(out2)
        if mask2 is not None:
            _check(tuple(mask2.shape[:3]) == (N, Ho, Wo), "mask2 shape mismatch")
            d.mask2_stride, d.mask2_scale = mask2.shape[3], float(mask2_scale)
            io.mask2 = ptr(mask2)
    if out is not None:
        _act(out, "out")
        if srcA.dtype == FP8_DTYPE:
            _check(out.dtype in (FP8_DTYPE, torch.bfloat16), "fp8 launch: out must be bf16 or fp8")
            _check(w_scale is not None and w_scale.dtype == torch.float32 and w_scale.numel() >= nout,
                   "fp8 launch needs w_scale (f32, >= nout entries)")
            d.out_fp8 = 1 if out.dtype == FP8_DTYPE else 0
            io.w_scale = ptr(w_scale)
        elif out.dtype == FP8_DTYPE:   # a bf16 input layer storing its fp8 operand (UNetBN.forward_fp8)
            _check(srcA.dtype == torch.bfloat16, "fp8 output needs a bf16 (input layer) or fp8 launch")
            d.out_fp8 = 1
        else:
            _check(out.dtype == srcA.dtype, "out dtype mismatch")
        if out_mode != 1:
            _check(tuple(out.shape[:3]) == (N, Ho, Wo), f"out shape {tuple(out.shape)} != {(N, Ho, Wo)}")
            _check(out.shape[3] >= (split_c if out_mode == 2 else nout), "out has too few channels")
        d.out_stride = out.shape[3]
        io.out = ptr(out)
    else:
        _check(out_mode == 2, "out may only be omitted for a split store")
    if addend is not None:
        _check(addend.shape == out.shape and addend.dtype == out.dtype, "addend must match out")
        io.addend = ptr(addend)
    if mask is not None:
        _check(tuple(mask.shape[:3]) == (N, Ho, Wo) and mask.dtype == srcA.dtype, "mask shape mismatch")
        d.mask_stride, d.mask_scale = mask.shape[3], float(mask_scale)
        io.mask = ptr(mask)
    if accum is not None:
        _check(accum.dtype == torch.float32 and tuple(accum.shape[:3]) == (N, Ho, Wo), "accum must be f32 NHWC")
        d.accum_stride = accum.shape[3]
        io.accum = ptr(accum)
    if bn_stats is not None:
        io.bn_sum, io.bn_sqsum = ptr(bn_stats[0]), ptr(bn_stats[1])
        d.bn_defer_fold = 1 if defer_fold else 0
    if bn_reduce is not None:
        z, sc, sh, mu, ist, dg, dbt = bn_reduce
        _check(out_mode == 0 and out is not None and z.shape == out.shape and z.dtype == out.dtype,
               "bn_reduce needs a plain store with z shaped like out")
        d.bnr_stride = z.shape[3]
        io.bnr_z, io.bnr_scale, io.bnr_shift, io.bnr_mean = ptr(z), ptr(sc), ptr(sh), ptr(mu)
        io.bnr_invstd, io.bnr_dgamma, io.bnr_dbeta = ptr(ist), ptr(dg), ptr(dbt)
    if act_out is not None:
        _check(bnA is not None and srcB is None, "act_out needs bnA and one source")
        _check(act_out.shape == srcA.shape and act_out.dtype == srcA.dtype and act_out.is_contiguous() and
               act_out.data_ptr() != srcA.data_ptr(), "act_out must be a separate tensor shaped like srcA")
        io.act_outA = ptr(act_out)
    dc = dtype_code(srcA)
    flops = 2.0 * N * Ho * Wo * nout * kh * kw * (d.CA_stride + d.CB_stride)
    # algorithmic bytes: every operand read once, every output written once
    nbytes = _nbytes(srcA) + _nbytes(srcB) + _nbytes(W) + _nbytes(out) + _nbytes(out2) + _nbytes(addend) + \
        _nbytes(mask) + _nbytes(mask2) + 2 * _nbytes(accum) + (_nbytes(bn_reduce[0]) if bn_reduce else 0) + \
        _nbytes(act_out)
    _timed(dc, flops,
           lambda: call("adp_conv_fwd", dc, C.byref(d), C.byref(io), stream_ptr()), nbytes)
    return out


def _nbytes(t):
    return 0 if t is None else t.numel() * t.element_size()


def conv_wgrad(srcA, dY, dW, nout, *, dB=None, srcB=None, bnA=None, bnB=None, up=False, stride=1, kh=3, kw=3,
               dil=1, pad=None, Ho=None, Wo=None, shuffle_c=0, bn_apply=None, real=None):
    """dW (+)= X_tap^T dY (f32 accumulators, caller zeroes). shuffle_c>0: dY is a ConvT output.
    real=(CA_real, CB_real, Nout_real): optional hints as in conv_fwd (the pad channels of the sources and of dY are
    zeros); the f32 halo weight gradient then runs chunks of <= 16 real channels on fewer waves.
    bn_apply=(dA, z, scale, shift, mean, invstd, gamma, dgamma, dbeta, count): dY is first computed as
    bn_bwd_apply(dA, z, ...) and stored (adp_conv_wgrad_bn: fused into the weight-gradient launch where the
    halo kernel takes the shape, bit-identical to bn_bwd_apply + conv_wgrad). With bn_apply, dY may be None
    (and dB None) when nothing reads dz: the fused forms then store nothing (the input layer, which has no
    data gradient)."""
    Wdummy = torch.empty(0)
    _act(srcA, "srcA")
    _check(dY is not None or (bn_apply is not None and dB is None), "dY is None only with bn_apply and no dB")
    dYs = dY if dY is not None else bn_apply[0]   # (its shape stands for dz's)
    _act(dYs, "dY")
    N, Hs, Ws, CA = srcA.shape
    CB = 0 if srcB is None else srcB.shape[3]
    K = kh * kw * (CA + CB)
    Kpad = round_up(K, 32)
    _check(dW.dtype == torch.float32 and dW.is_contiguous() and dW.dim() == 2, "dW must be f32 2-D")
    _check(dW.shape[1] == Kpad and dW.shape[0] >= nout, f"dW shape {tuple(dW.shape)} != (>={nout}, {Kpad})")
    _check(nout % 8 == 0, "wgrad needs nout % 8 == 0")
    d = ConvDesc()
    io = ConvIO()
    Ho_, Wo_, pad = conv_geometry(Hs, Ws, up=up, stride=stride, kh=kh, kw=kw, dil=dil, pad=pad)
    Ho = Ho_ if Ho is None else Ho
    Wo = Wo_ if Wo is None else Wo
    d.N, d.Hs, d.Ws, d.CA_stride, d.CB_stride = N, Hs, Ws, CA, CB
    d.upsample = 1 if up else 0
    d.Ho, d.Wo, d.stride, d.kh, d.kw, d.dil, d.pad = Ho, Wo, stride, kh, kw, dil, pad
    d.Nout = nout
    if real is not None:
        ca, cb, nr = (int(v) for v in real)
        _check(0 <= ca <= CA and 0 <= cb <= CB and 0 <= nr <= nout, "real channel counts out of range")
        d.CA_real, d.CB_real, d.Nout_real = ca, cb, nr
    if shuffle_c:
        d.out_mode, d.shuffle_c = 1, shuffle_c
        _check(tuple(dYs.shape[:3]) == (N, 2 * Ho, 2 * Wo), "convT dY shape mismatch")
    else:
        _check(tuple(dYs.shape[:3]) == (N, Ho, Wo) and dYs.shape[3] >= nout, "dY shape mismatch")
    io.srcA, io.srcB = ptr(srcA), ptr(srcB)
    if bnA is not None:
        io.bn_scaleA, io.bn_shiftA = ptr(bnA[0]), ptr(bnA[1])
    if bnB is not None:
        io.bn_scaleB, io.bn_shiftB = ptr(bnB[0]), ptr(bnB[1])
    if dB is not None:
        _check(dB.dtype == torch.float32, "dB must be f32")
    del Wdummy
    dc = dtype_code(srcA)
    flops = 2.0 * N * Ho * Wo * nout * K
    # algorithmic bytes: sources and dY read once, dW (f32) accumulated once
    nbytes = _nbytes(srcA) + _nbytes(srcB) + _nbytes(dY) + 4.0 * nout * Kpad
    if bn_apply is not None:
        dA, z, sc, sh, mu, ist, gam, dg, dbt, count = bn_apply
        _check(not shuffle_c and dA.shape == z.shape == dYs.shape and dYs.shape[3] == nout and
               dA.dtype == z.dtype == dYs.dtype, "bn_apply: dA, z, dY of one [N, Ho, Wo, nout] shape")
        bn = BnBwdArgs(ptr(dA), ptr(z), ptr(sc), ptr(sh), ptr(mu), ptr(ist), ptr(gam), ptr(dg), ptr(dbt),
                       float(count))
        _timed(dc, flops,
               lambda: call("adp_conv_wgrad_bn", dc, C.byref(d), C.byref(io), C.byref(bn), ptr(dY),
                            int(dYs.shape[3]), ptr(dW), ptr(dB), stream_ptr()), nbytes + 2 * _nbytes(dA))
        return
    _timed(dc, flops,
           lambda: call("adp_conv_wgrad", dc, C.byref(d), C.byref(io), ptr(dY), int(dY.shape[3]), ptr(dW),
                        ptr(dB), stream_ptr()), nbytes)


def pack_weights(src, dst, mode, *, taps=1, cin_s=0, nout=0):
    """mode 0: cast/copy [Npad][Kpad]; mode 1: conv dgrad flip+transpose; mode 2: convT transpose."""
    _check(src.dtype == torch.float32 and src.dim() == 2 and dst.dim() == 2, "pack_weights: bad tensors")
    if mode == 0:
        _check(dst.shape == src.shape, "pack mode 0 needs equal shapes")
    else:
        _check(dst.shape[0] >= cin_s and dst.shape[1] >= taps * nout and src.shape[0] >= nout
               and src.shape[1] >= taps * cin_s, "pack_weights: shape mismatch")
    call("adp_pack_weights", dtype_code(dst), mode, taps, cin_s, nout, ptr(src), int(src.shape[1]), ptr(dst),
         int(dst.shape[0]), int(dst.shape[1]), stream_ptr())


class PackJob(C.Structure):
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("taps", C.c_int), ("Cin_s", C.c_int), ("Nout", C.c_int),
                ("src_kpad", C.c_int), ("dst_rows", C.c_int), ("dst_kpad", C.c_int)]


PACK_MAX_JOBS = 24


def pack_weights_batch(jobs):
    """Data-gradient repack (pack_weights modes 1/2) of many layers in one launch per 24 layers:
    jobs = [(src f32 [Npad][Kpad], dst [dNpad][dKpad], taps, cin_s, nout)], dst all of one dtype."""
    for i in range(0, len(jobs), PACK_MAX_JOBS):
        chunk = jobs[i:i + PACK_MAX_JOBS]
        arr = (PackJob * len(chunk))()
        dc = None
        for k, (src, dst, taps, cin_s, nout) in enumerate(chunk):
            _check(src.dtype == torch.float32 and src.dim() == 2 and dst.dim() == 2 and dst.is_contiguous(),
                   "pack_weights_batch: bad tensors")
            _check(dst.shape[0] >= cin_s and dst.shape[1] >= taps * nout and src.shape[0] >= nout
                   and src.shape[1] >= taps * cin_s, "pack_weights_batch: shape mismatch")
            _check(dc is None or dtype_code(dst) == dc, "pack_weights_batch: one destination dtype")
            dc = dtype_code(dst)
            arr[k] = PackJob(ptr(src), ptr(dst), taps, cin_s, nout, int(src.shape[1]), int(dst.shape[0]),
                             int(dst.shape[1]))
        call("adp_pack_weights_batch", dc, len(chunk), arr, stream_ptr())


def pack_weights_fp8(src, dst, scale):
    """Forward-layout fp8 weights + per-row dequantisation scale (adp_pack_weights_fp8)."""
    _check(src.dtype == torch.float32 and src.dim() == 2 and dst.dtype == FP8_DTYPE and dst.dim() == 2
           and dst.shape[0] == src.shape[0] and dst.shape[1] >= src.shape[1] and dst.shape[1] % 8 == 0,
           "pack_weights_fp8: bad tensors")
    _check(scale.dtype == torch.float32 and scale.numel() >= src.shape[0], "pack_weights_fp8: scale size")
    call("adp_pack_weights_fp8", int(src.shape[0]), ptr(src), int(src.shape[1]), ptr(dst), int(dst.shape[1]),
         ptr(scale), stream_ptr())


def vec_mul(a, b, out):
    """out = a * b on f32 vectors (adp_vec_mul)."""
    _check(a.dtype == b.dtype == out.dtype == torch.float32 and a.numel() <= b.numel() and a.numel() <= out.numel(),
           "vec_mul: f32 vectors, b and out at least as long as a")
    call("adp_vec_mul", a.numel(), ptr(a), ptr(b), ptr(out), stream_ptr())
    return out


def scale_rows(src, scale, dst):
    """dst = src * scale[:, None] (rows past scale's length: 0) cast to dst's dtype (adp_scale_rows)."""
    _check(src.dtype == torch.float32 and src.dim() == 2 and dst.dim() == 2 and dst.shape == src.shape and
           scale.dtype == torch.float32 and dst.is_contiguous() and src.stride(1) == 1, "scale_rows: bad tensors")
    call("adp_scale_rows", dtype_code(dst), int(src.shape[0]), int(src.shape[1]), ptr(src), int(src.stride(0)),
         ptr(scale), int(scale.numel()), ptr(dst), int(dst.shape[1]), stream_ptr())
    return dst


def bn_apply_fp8(z, scale, shift, out):
    _check(out.shape == z.shape and out.dtype == FP8_DTYPE, "bn_apply_fp8 shapes")
    Cs = z.shape[-1]
    call("adp_bn_apply_fp8", dtype_code(z), z.numel() // Cs, Cs, ptr(z), ptr(scale), ptr(shift), ptr(out),
         stream_ptr())
    return out


def bn_apply_maxpool2(z, scale, shift, act, pool):
    """act = relu(z * scale + shift) and pool = 2x2 max-pool of act, one pass (adp_bn_apply_maxpool2)."""
    _act(z, "z")
    N, H, W, Cs = z.shape
    _check(act.shape == z.shape and act.dtype == z.dtype, "bn_apply_maxpool2: act shape")
    _check(tuple(pool.shape) == (N, H // 2, W // 2, Cs) and pool.dtype == z.dtype, "bn_apply_maxpool2: pool shape")
    call("adp_bn_apply_maxpool2", dtype_code(z), N, H, W, Cs, ptr(z), ptr(scale), ptr(shift), ptr(act), ptr(pool),
         stream_ptr())
    return act


def maxpool2_fwd(src, dst, bn=None):
    _act(src, "src")
    _act(dst, "dst")
    N, H, W, Cs = src.shape
    if dst.dtype == FP8_DTYPE:
        _check(tuple(dst.shape) == (N, H // 2, W // 2, Cs) and bn is None, "maxpool fp8 dst shape")
        call("adp_maxpool2_fwd_fp8", dtype_code(src), N, H, W, Cs, ptr(src), ptr(dst), stream_ptr())
        return dst
    _check(tuple(dst.shape) == (N, H // 2, W // 2, Cs) and dst.dtype == src.dtype, "maxpool dst shape")
    call("adp_maxpool2_fwd", dtype_code(src), N, H, W, Cs, ptr(src), ptr(bn[0]) if bn else None,
         ptr(bn[1]) if bn else None, ptr(dst), stream_ptr())
    return dst


def maxpool2_bwd(src, dpool, dsrc, *, bn=None, addend=None, mask=None, mask_scale=1.0, bn_reduce=None,
                 argmax_from_z=True):
    """bn_reduce=(z, scale, shift, mean, invstd, dgamma, dbeta): fused BatchNorm-backward reduction of
    the layer whose activation src = relu(z*scale+shift) is (adp_maxpool2_bwd_bnr; needs addend, no
    bn/mask). argmax_from_z: the kernel recomputes src from z instead of reading it (bit-identical when
    src was stored by bn_apply / bn_apply_maxpool2 with the same scale/shift; src then only gives the
    shape)."""
    _act(src, "src")
    N, H, W, Cs = src.shape
    _check(tuple(dpool.shape) == (N, H // 2, W // 2, Cs), "dpool shape")
    _check(dsrc.shape == src.shape, "dsrc shape")
    for t in (addend, mask):
        _check(t is None or t.shape == src.shape, "addend/mask shape")
    if bn_reduce is not None:
        z, sc, sh, mean, inv, dg, db = bn_reduce
        _check(bn is None and mask is None and addend is not None and z.shape == src.shape and z.dtype == src.dtype,
               "maxpool2_bwd bn_reduce: needs addend, z like src, no bn/mask")
        call("adp_maxpool2_bwd_bnr", dtype_code(src), N, H, W, Cs, None if argmax_from_z else ptr(src), ptr(dpool),
             ptr(addend), ptr(dsrc),
             ptr(z), ptr(sc), ptr(sh), ptr(mean), ptr(inv), ptr(dg), ptr(db), stream_ptr())
        return dsrc
    call("adp_maxpool2_bwd", dtype_code(src), N, H, W, Cs, ptr(src), ptr(bn[0]) if bn else None,
         ptr(bn[1]) if bn else None, ptr(dpool), ptr(addend), ptr(mask), float(mask_scale), ptr(dsrc), stream_ptr())
    return dsrc


def upsample2_bwd(dup, dsrc, *, addend=None, mask=None, mask_scale=1.0):
    _act(dup, "dup")
    _act(dsrc, "dsrc")
    N, Hs, Ws, Cs = dsrc.shape
    _check(tuple(dup.shape) == (N, 2 * Hs, 2 * Ws, Cs), "upsample grad shapes")
    for t in (addend, mask):
        _check(t is None or t.shape == dsrc.shape, "addend/mask shape")
    call("adp_upsample2_bwd", dtype_code(dup), N, Hs, Ws, Cs, ptr(dup), ptr(addend), ptr(mask), float(mask_scale),
         ptr(dsrc), stream_ptr())
    return dsrc


def add_mask(a, out, *, b=None, mask=None, mask_scale=1.0):
    _check(out.shape == a.shape and a.numel() % 8 == 0, "add_mask shapes")
    for t in (b, mask):
        _check(t is None or t.shape == a.shape, "add_mask operand shape")
    call("adp_ew_add_mask", dtype_code(a), a.numel(), ptr(a), ptr(b), ptr(mask), float(mask_scale), ptr(out),
         stream_ptr())
    return out


def cast(src, dst):
    _check(src.numel() == dst.numel(), "cast sizes")
    call("adp_cast", dtype_code(src), dtype_code(dst), src.numel(), ptr(src), ptr(dst), stream_ptr())
    return dst


def sum_bf16(srcs, out):
    """out = bf16(sum(srcs)) (f32 sum in list order): adp_sum_bf16."""
    import ctypes
    _check(1 <= len(srcs) <= 8, "sum_bf16: 1..8 sources")
    _check(out.dtype == torch.bfloat16 and all(t.dtype == torch.bfloat16 and t.shape == out.shape and t.is_contiguous()
                                                for t in srcs), "sum_bf16: same-shape contiguous bf16 maps")
    arr = (ctypes.c_void_p * len(srcs))(*[ptr(t) for t in srcs])
    call("adp_sum_bf16", len(srcs), ctypes.cast(arr, ctypes.c_void_p).value, out.numel(), ptr(out), stream_ptr())
    return out


def fill(dst, value):
    _check(dst.dtype == torch.float32, "fill is f32")
    call("adp_fill_f32", dst.numel(), float(value), ptr(dst), stream_ptr())


def wgrad_defer(on=True):
    """adp_wgrad_defer on the current stream: the deterministic weight / bias gradient reductions of the following
    conv_wgrad launches are recorded, not launched; dW / dB are final only after wgrad_flush()."""
    call("adp_wgrad_defer", 1 if on else 0, stream_ptr())


def wgrad_flush():
    """adp_wgrad_flush: every recorded reduction of the current stream in one launch; ends the deferral."""
    call("adp_wgrad_flush", stream_ptr())


def get_option(name):
    """adp_get_option: the value set for `name`, None when unset (the built-in default applies)."""
    from . import _lib
    v = int(_lib.lib().adp_get_option(name.encode()))
    return None if v == -(2 ** 31) else v


def wgrad_release(stream=None):
    """adp_wgrad_release: free the deferral arena of (current device, stream) and forget the stream (synchronises it;
    AdpError with reductions pending). stream: a torch.cuda.Stream, default the current one."""
    call("adp_wgrad_release", stream_ptr() if stream is None else stream.cuda_stream)


def wgrad_arena_chunks(stream=None):
    """The number of deferral-arena chunks of (current device, stream) (adp_wgrad_arena_chunks; test hook)."""
    from . import _lib
    return int(_lib.lib().adp_wgrad_arena_chunks(stream_ptr() if stream is None else stream.cuda_stream))


def bn_fold_reset():
    """Drop a deferred BatchNorm fold left pending by a failed step and re-zero the accumulator replicas
    (adp_bn_fold_reset, stream-ordered; a no-op when nothing is pending)."""
    call("adp_bn_fold_reset", stream_ptr())


def bn_finalize(count, ssum, ssq, gamma, beta, eps, momentum, scale, shift, mean, invstd, rmean=None, rvar=None,
                fold=False):
    """fold=True: first add the statistics the previous conv_fwd(..., defer_fold=True) left in the
    accumulator replicas into ssum / ssq (adp_bn_finalize_fold: one launch for fold + finalize)."""
    C_ = gamma.numel()
    if fold:
        _check(count > 0, "bn_finalize(fold=True) is the training form")
        call("adp_bn_finalize_fold", C_, float(count), ptr(ssum), ptr(ssq), ptr(gamma), ptr(beta), float(eps),
             float(momentum), ptr(scale), ptr(shift), ptr(mean), ptr(invstd), ptr(rmean), ptr(rvar), stream_ptr())
        return
    call("adp_bn_finalize", C_, float(count), ptr(ssum), ptr(ssq), ptr(gamma), ptr(beta), float(eps),
         float(momentum), ptr(scale), ptr(shift), ptr(mean), ptr(invstd), ptr(rmean), ptr(rvar), stream_ptr())


def bn_apply(z, scale, shift, out):
    _check(out.shape == z.shape and out.dtype == z.dtype, "bn_apply shapes")
    Cs = z.shape[-1]
    call("adp_bn_apply", dtype_code(z), z.numel() // Cs, Cs, ptr(z), ptr(scale), ptr(shift), ptr(out), stream_ptr())
    return out


def bn_bwd_reduce(dA, z, scale, shift, mean, invstd, dgamma, dbeta):
    _check(dA.shape == z.shape, "bn bwd shapes")
    Cs = z.shape[-1]
    M = z.numel() // Cs
    call("adp_bn_bwd_reduce", dtype_code(z), M, Cs, ptr(dA), ptr(z), ptr(scale), ptr(shift), ptr(mean),
         ptr(invstd), ptr(dgamma), ptr(dbeta), stream_ptr())


def bn_bwd_apply(dA, z, scale, shift, mean, invstd, gamma, dgamma, dbeta, count, dz):
    _check(dA.shape == z.shape == dz.shape, "bn bwd shapes")
    Cs = z.shape[-1]
    M = z.numel() // Cs
    call("adp_bn_bwd_apply", dtype_code(z), M, Cs, ptr(dA), ptr(z), ptr(scale), ptr(shift), ptr(mean),
         ptr(invstd), ptr(gamma), ptr(dgamma), ptr(dbeta), float(count), ptr(dz), stream_ptr())


def bn_bwd_apply_head(W, p, dp, z, scale, shift, mean, invstd, gamma, dgamma, dbeta, count, dz, *, cin):
    """adp_bn_bwd_apply with dA = dp*p*(1-p)*W[c] recomputed from the sigmoid head (the dx the fused head
    backward would have stored: it then runs with dx=None)."""
    _check(z.shape == dz.shape, "bn bwd shapes")
    Cs = z.shape[-1]
    M = z.numel() // Cs
    _check(p.numel() == M and dp.numel() == M and W.numel() == cin and cin <= Cs, "head grad sizes")
    call("adp_bn_bwd_apply_head", dtype_code(z), M, Cs, cin, ptr(W), ptr(p), ptr(dp), ptr(z), ptr(scale),
         ptr(shift), ptr(mean), ptr(invstd), ptr(gamma), ptr(dgamma), ptr(dbeta), float(count), ptr(dz),
         stream_ptr())


def head_fwd(x, W, b, p, *, cin, softmax2, bn=None):
    _act(x, "x")
    Cs = x.shape[-1]
    M = x.numel() // Cs
    _check(p.numel() == M and p.dtype == torch.float32, "head output size")
    _check(W.numel() == (2 if softmax2 else 1) * cin and cin <= Cs, "head weight size")
    name = "adp_head_softmax2_fwd" if softmax2 else "adp_head_sigmoid_fwd"
    call(name, dtype_code(x), M, Cs, cin, ptr(x), ptr(W), ptr(b), ptr(bn[0]) if bn else None,
         ptr(bn[1]) if bn else None, ptr(p), stream_ptr())
    return p


def head_bwd(x, W, p, dp, dW, db, *, cin, softmax2, dx=None, bn=None, addend=None, mask=None, mask_scale=1.0,
             bn_reduce=None):
    """bn_reduce=(mean, invstd, dgamma, dbeta): x is the pre-BN map z of the layer under the head (bn its
    scale/shift); that layer's BatchNorm-backward reduction over dx is fused (adp_head_sigmoid_bwd_bnr)."""
    _act(x, "x")
    if bn_reduce is not None:
        _check(not softmax2 and bn is not None and addend is None and mask is None,
               "head_bwd bn_reduce: sigmoid head and bn only")
        Cs = x.shape[-1]
        M = x.numel() // Cs
        _check(p.numel() == M and dp.numel() == M and (dx is None or dx.shape == x.shape), "head grad sizes")
        mean, invstd, dg, dbeta = bn_reduce
        call("adp_head_sigmoid_bwd_bnr", dtype_code(x), M, Cs, cin, ptr(x), ptr(W), ptr(bn[0]), ptr(bn[1]),
             ptr(mean), ptr(invstd), ptr(p), ptr(dp), ptr(dx), ptr(dW), ptr(db), ptr(dg), ptr(dbeta), stream_ptr())
        return
    Cs = x.shape[-1]
    M = x.numel() // Cs
    _check(p.numel() == M and dp.numel() == M, "head grad sizes")
    for t in (dx, addend, mask):
        _check(t is None or t.shape == x.shape, "head dx/addend/mask shape")
    name = "adp_head_softmax2_bwd" if softmax2 else "adp_head_sigmoid_bwd"
    call(name, dtype_code(x), M, Cs, cin, ptr(x), ptr(W), ptr(bn[0]) if bn else None, ptr(bn[1]) if bn else None,
         ptr(p), ptr(dp), ptr(addend), ptr(mask), float(mask_scale), ptr(dx), ptr(dW), ptr(db), stream_ptr())


def resize_bilinear_fwd(src, dst):
    N, Hs, Ws = src.shape
    _, Ho, Wo = dst.shape
    _check(dst.shape[0] == N and src.dtype == dst.dtype == torch.float32, "resize shapes")
    call("adp_resize_bilinear_fwd", N, Hs, Ws, Ho, Wo, ptr(src), ptr(dst), stream_ptr())
    return dst


def resize_bilinear_bwd(dout, dsrc):
    N, Ho, Wo = dout.shape
    _, Hs, Ws = dsrc.shape
    call("adp_resize_bilinear_bwd", N, Hs, Ws, Ho, Wo, ptr(dout), ptr(dsrc), stream_ptr())
    return dsrc


def loss_rows(p, y, row_bce, stats, *, smooth=False, eps_pos=0.03, eps_neg=0.07):
    N, H, W = p.shape
    _check(y.shape == p.shape and row_bce.numel() == N * H and stats.dtype == torch.float64, "loss_rows shapes")
    call("adp_loss_rows", N, H, W, ptr(p), ptr(y), int(smooth), float(eps_pos), float(eps_neg), ptr(row_bce),
         ptr(stats), stream_ptr())


def loss_select(row_bce, row_coef, out, *, N, H, W, ohem, keep_ratio, weight, norm_rows):
    call("adp_loss_select", N, H, W, ptr(row_bce), int(ohem), float(keep_ratio), float(weight), float(norm_rows),
         ptr(row_coef), ptr(out), stream_ptr())


def loss_grad(p, y, row_coef, stats, dp, *, weight, smooth=False, eps_pos=0.03, eps_neg=0.07, accumulate=False):
    N, H, W = p.shape
    call("adp_loss_grad", N, H, W, ptr(p), ptr(y), int(smooth), float(eps_pos), float(eps_neg), ptr(row_coef),
         ptr(stats), float(weight), int(accumulate), ptr(dp), stream_ptr())


def pixel_counts(pred, truth, thr, counts):
    _check(pred.numel() == truth.numel() and counts.dtype == torch.int64 and counts.numel() >= 4, "counts")
    call("adp_pixel_counts", pred.numel(), ptr(pred), ptr(truth), float(thr), ptr(counts), stream_ptr())


def threshold_hist(pred, truth, thresholds, hist):
    """hist (int64, 2*(T+1), caller zeroes) (+)= pixel histogram of #{t: pred > t} split by truth > 0.5."""
    T = len(thresholds)
    _check(pred.numel() == truth.numel() and pred.dtype == truth.dtype == torch.float32, "threshold_hist inputs")
    _check(hist.dtype == torch.int64 and hist.numel() >= 2 * (T + 1), "threshold_hist: hist size")
    arr = (C.c_double * T)(*[float(t) for t in thresholds])
    call("adp_threshold_hist", pred.numel(), ptr(pred), ptr(truth), T, arr, ptr(hist), stream_ptr())


def adam(param, grad, m, v, *, lr, beta1, beta2, eps, step, weight_decay=0.0, grad_scale=1.0):
    n = param.numel()
    _check(grad.numel() == n and m.numel() == n and v.numel() == n, "adam sizes")
    call("adp_adam", n, ptr(param), ptr(grad), ptr(m), ptr(v), float(lr), float(beta1), float(beta2), float(eps),
         int(step), float(weight_decay), float(grad_scale), stream_ptr())


def ema(ema_buf, param, decay):
    call("adp_ema", param.numel(), ptr(ema_buf), ptr(param), float(decay), stream_ptr())


def prep_input(src, dst, *, mean, std, view=0):
    """src f32 (N,H,W) or (N,H,W,C) raw intensities -> dst NHWC normalised (pad channels zero).
    ``src`` may be a strided window of a larger image (e.g. img[y:y+T, x:x+T]): rows are read in
    place with the parent's row stride."""
    if src.dim() == 3:
        N, H, W = src.shape
        Cin = 1
        rs, ims = src.stride(1), src.stride(0)
        _check(src.stride(2) == 1, "prep src rows must be contiguous")
    else:
        N, H, W, Cin = src.shape
        _check(src.stride(3) == 1 and src.stride(2) == Cin, "prep src pixels must be contiguous")
        rs, ims = src.stride(1) // Cin, src.stride(0)
    _check(src.dtype == torch.float32 and src.is_cuda, "prep src must be a device f32 tensor")
    _check(tuple(dst.shape[:3]) == (N, H, W) and dst.shape[3] >= Cin, "prep dst shape")
    call("adp_prep_input", dtype_code(dst), N, H, W, Cin, ptr(src), int(rs), int(ims), float(mean), float(std),
         int(view), int(dst.shape[3]), ptr(dst), stream_ptr())
    return dst


def tta_merge(probs, views, out):
    nv, H, W = probs.shape
    arr = (C.c_int * 8)(*list(views) + [0] * (8 - len(views)))
    call("adp_tta_merge", H, W, nv, arr, ptr(probs), ptr(out), stream_ptr())
    return out


def blend_accum(tile, weight, acc, wsum, y0, x0):
    H, W = acc.shape
    T = tile.shape[-1]
    _check(y0 + T <= H and x0 + T <= W, "tile outside the canvas")
    call("adp_blend_accum", H, W, T, int(y0), int(x0), ptr(tile), ptr(weight), ptr(acc), ptr(wsum), stream_ptr())


def blend_finalize(acc, wsum, out, floor_=1e-8):
    call("adp_blend_finalize", acc.numel(), ptr(acc), ptr(wsum), float(floor_), ptr(out), stream_ptr())
    return out
