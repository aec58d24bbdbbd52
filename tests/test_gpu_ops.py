"""Kernel-level parity: every libadipose_hip op vs the CPU fp32 oracle (oracle/torch_ref.py).

f32 launches run the exact-f32 MFMA path: tolerance 1e-4 relative to the output scale.
bf16 launches are compared with the oracle evaluated on bf16-rounded operands (f32 accumulate):
tolerance 2e-2 relative to the output scale.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from adipose_amd import _lib, ops
from adipose_amd.nets import Dense, Head
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def nhwc_pad(x, cs, dt):
    """logical NHWC CPU tensor -> device tensor with channel stride cs (zero pad)."""
    N, H, W, C = x.shape
    out = torch.zeros((N, H, W, cs), dtype=dt, device=DEV)
    out[..., :C] = x.to(DEV, dt)
    return out


@pytest.fixture(autouse=True)
def _no_split_k():
    """The kernel-level tests here compare kernel forms bit for bit on small problems, which the tap64 launcher's
    split-K (round 6) would otherwise take: it is off in this module except where a test turns it on
    (test_tap64_split_k); the network and config tests run with the default."""
    from adipose_amd import ops
    ops.set_option("tap64_ksplit", 0)
    yield
    ops.set_option("tap64_ksplit", None)


def relerr(a, b):
    a = a.float().cpu()
    b = b.float().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-6)


def rb(t, dt):
    return t.to(dt).float() if dt == torch.bfloat16 else t


TOL = {torch.float32: 1e-4, torch.bfloat16: 2e-2}
DTS = [torch.float32, torch.bfloat16]

CONV_CASES = [
    # name, N, S, cin_parts, cout, dil, up
    ("first", 2, 16, [1], 44, 1, False),
    # one 8-channel source (network input): bf16 launches take the register-resident cin8 kernel
    ("first3_64", 2, 16, [3], 64, 1, False),
    ("first3_ragged_dil2", 1, 13, [3], 64, 2, False),
    ("first1_24", 3, 10, [1], 24, 1, False),
    ("plain", 2, 16, [44], 88, 2, False),
    ("dil8", 1, 32, [88], 176, 8, False),
    ("dil32", 1, 16, [64], 64, 32, False),
    ("up", 2, 8, [88], 44, 1, True),
    ("concat", 2, 16, [44, 44], 44, 1, False),
    ("wide", 1, 16, [176], 352, 4, False),
    # channel strides % 64 == 0 -> bf16 launches take the 8-phase tap64 kernel (ragged M, partial N tile)
    ("c64", 2, 24, [64], 64, 1, False),
    ("c128_320", 1, 20, [128], 320, 2, False),
    ("concat64", 2, 16, [64, 64], 128, 1, False),
    # 3x3 stride-1 layers with <= 128 output channels and 8x32-divisible images -> halo kernel (bf16)
    ("halo64", 2, 32, [64], 64, 1, False),
    ("halo_cat", 1, 32, [64, 64], 128, 1, False),
    ("halo_n96", 1, 64, [128], 96, 1, False),
    ("halo_c64_n128", 1, 32, [64], 128, 1, False),
]


def make_case(N, S, cin_parts, cout, dil, up, seed=0):
    g = torch.Generator().manual_seed(seed)
    xs = [torch.randn(N, S, S, c, generator=g) for c in cin_parts]
    cin = sum(cin_parts)
    kern = torch.randn(3, 3, cin, cout, generator=g) * (1.0 / np.sqrt(9 * cin))
    bias = torch.randn(cout, generator=g) * 0.1
    layer = Dense("t", cin_parts, cout, dil=dil, up=up)
    return xs, kern, bias, layer


def oracle_fwd(xs, kern, bias, dil, up, relu=True):
    x = torch.cat(xs, -1)
    if up:
        x = R.upsample_nearest2(x)
    return R.conv2d_same(x, kern, bias, dilation=dil, relu=relu)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("case", CONV_CASES, ids=[c[0] for c in CONV_CASES])
def test_conv_fwd(case, dt):
    _, N, S, parts, cout, dil, up = case
    xs, kern, bias, l = make_case(N, S, parts, cout, dil, up)
    Wp = torch.from_numpy(l.keras_to_packed(kern.numpy())).to(DEV)
    W = Wp.to(dt).contiguous()
    b = torch.zeros(l.cout_s, device=DEV)
    b[:cout] = bias.to(DEV)
    srcs = [nhwc_pad(x, cs, dt) for x, cs in zip(xs, l.cin_s)]
    So = S * 2 if up else S
    out = torch.zeros((N, So, So, l.cout_s), dtype=dt, device=DEV)
    ops.conv_fwd(srcs[0], W, l.Nout, out=out, srcB=srcs[1] if len(srcs) > 1 else None, bias=b, up=up, dil=dil,
                 relu=True)
    torch.cuda.synchronize()
    ref = oracle_fwd([rb(x, dt) for x in xs], rb(kern, dt), bias, dil, up)
    assert relerr(out[..., :cout], ref) < TOL[dt]
    if l.cout_s > cout:
        assert out[..., cout:].abs().max().item() == 0.0  # pad channels stay zero


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("case", CONV_CASES, ids=[c[0] for c in CONV_CASES])
def test_conv_grads(case, dt):
    """wgrad (+bias grad) and dgrad vs autograd of the oracle conv (pre-activation)."""
    _, N, S, parts, cout, dil, up = case
    xs, kern, bias, l = make_case(N, S, parts, cout, dil, up, seed=1)
    xs = [rb(x, dt) for x in xs]
    kern = rb(kern, dt)
    So = S * 2 if up else S
    g = torch.Generator().manual_seed(5)
    dZ = rb(torch.randn(N, So, So, cout, generator=g), dt)
    xr = [x.clone().requires_grad_(True) for x in xs]
    kr = kern.clone().requires_grad_(True)
    br = bias.clone().requires_grad_(True)
    y = oracle_fwd(xr, kr, br, dil, up, relu=False)
    (y * dZ).sum().backward()
    # device
    srcs = [nhwc_pad(x, cs, dt) for x, cs in zip(xs, l.cin_s)]
    dZd = nhwc_pad(dZ, l.cout_s, dt)
    dW = torch.zeros((l.Npad, l.Kpad), device=DEV)
    dB = torch.zeros(l.cout_s, device=DEV)
    ops.conv_wgrad(srcs[0], dZd, dW, l.Nout, dB=dB, srcB=srcs[1] if len(srcs) > 1 else None, up=up, dil=dil)
    Wmaster = torch.from_numpy(l.keras_to_packed(kern.numpy())).to(DEV)
    Wd = torch.zeros((l.dNpad, l.dKpad), dtype=dt, device=DEV)
    ops.pack_weights(Wmaster, Wd, 1, taps=9, cin_s=l.Cin_s, nout=l.cout_s)
    Hs = S * 2 if up else S
    dX = torch.zeros((N, Hs, Hs, l.Cin_s), dtype=dt, device=DEV)
    ops.conv_fwd(dZd, Wd, l.Cin_s, out=dX, dil=dil)
    torch.cuda.synchronize()
    dW_k = torch.from_numpy(l.packed_to_keras(dW.cpu().numpy()))
    tol = 1e-4 if dt == torch.float32 else 2e-2
    assert relerr(dW_k, kr.grad) < tol
    assert relerr(dB[:cout], br.grad) < tol
    # data gradient: for the upsample layer compare on the upsampled grid (kernel output before 2x2 sum)
    xcat = torch.cat(xs, -1)
    if up:
        xu = R.upsample_nearest2(xcat).clone().requires_grad_(True)
        (R.conv2d_same(xu, kern, bias, dilation=dil, relu=False) * dZ).sum().backward()
        ref_dx = xu.grad
    else:
        ref_dx = torch.cat([x.grad for x in xr], -1)
    got = torch.cat([dX[..., sum(l.cin_s[:i]): sum(l.cin_s[:i]) + c] for i, c in enumerate(parts)], -1)
    assert relerr(got, ref_dx) < tol


@pytest.mark.parametrize("cfg", [2, 3, 4, 5], ids=["256x256", "256x128", "512x64", "256x64"])
def test_tap64_configs(cfg):
    """Each forced tile configuration of the tap64 kernel: output and fused BatchNorm statistics vs the
    oracle on a ragged pixel count (M = 529) and a partial N tile (Nout = 192)."""
    N, S, cin, cout = 1, 23, 128, 192
    xs, kern, bias, l = make_case(N, S, [cin], cout, 1, False, seed=7)
    dt = torch.bfloat16
    W = torch.from_numpy(l.keras_to_packed(kern.numpy())).to(DEV).to(dt).contiguous()
    b = bias.to(DEV)
    x = nhwc_pad(xs[0], l.Cin_s, dt)
    out = torch.zeros((N, S, S, l.cout_s), dtype=dt, device=DEV)
    st = torch.zeros(2, l.cout_s, device=DEV)
    ops.set_option("fwd_tap64", cfg)
    try:
        ops.conv_fwd(x, W, l.Nout, out=out, bias=b, relu=True, bn_stats=(st[0], st[1]))
        torch.cuda.synchronize()
    finally:
        ops.set_option("fwd_tap64", 1)
    ref = oracle_fwd([rb(xs[0], dt)], rb(kern, dt), bias, 1, False)
    assert relerr(out[..., :cout], ref) < 2e-2
    rs = ref.reshape(-1, cout)
    assert relerr(st[0, :cout], rs.sum(0)) < 2e-2
    assert relerr(st[1, :cout], (rs * rs).sum(0)) < 2e-2


@pytest.mark.parametrize("claim", [0, 1, 2], ids=["static", "claimed", "claimed_full"])
@pytest.mark.parametrize("wide", [0, 1, 2], ids=["st8", "st16", "st16_lines"])
@pytest.mark.parametrize("tile", [256, 128], ids=["256x256x2", "256x128x3"])
@pytest.mark.parametrize("grid", [None, 3, 7], ids=["chip_grid", "3_blocks", "7_blocks"])
@pytest.mark.parametrize("mode", ["plain", "one_chunk", "concat", "split"])
def test_tap64p_halo_matches(mode, grid, tile, wide, claim):
    """Halo form of the persistent 256x256 forward (A operand read from a 10x34 halo moved into LDS once per
    64-channel chunk, chunk-major K stream, next chunk's halo issued one group per step) vs a float64
    reference convolution of the same bf16 operands, and vs the gathered form (tap64p_halo=0) to within the
    bf16 rounding of a different f32 summation order; BatchNorm sums to 1e-4. Ragged N tile (320), 1-3
    input chunks from one or two sources, split store; 3 / 7-block grids walk many patches per block."""
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(12)
    N, H, W_ = 2, 32, 64
    parts = {"plain": [128], "one_chunk": [64], "concat": [64, 128], "split": [128, 64]}[mode]
    nout = {"plain": 320, "one_chunk": 256, "concat": 256, "split": 256}[mode]
    if tile == 128:
        nout = {"plain": 192, "one_chunk": 128, "concat": 128, "split": 256}[mode]
    cin = sum(parts)
    srcs = [torch.randn(N, H, W_, c, generator=g).to(DEV, dt) for c in parts]
    Wt = (torch.randn(((nout + 63) // 64) * 64, 9 * cin, generator=g) * 0.03).to(DEV, dt)
    bias = torch.randn(nout, generator=g).to(DEV)
    x = torch.cat([t.double() for t in srcs], -1).permute(0, 3, 1, 2)
    wk = Wt[:nout].double().view(nout, 3, 3, cin).permute(0, 3, 1, 2)
    ref = F.conv2d(x, wk, padding=1).permute(0, 2, 3, 1) + bias.double()
    relu = mode != "split"
    if relu:
        ref = ref.clamp_min(0.0)
    res = []
    for halo in (1, 0):
        outs = [torch.zeros(N, H, W_, nout, dtype=dt, device=DEV)]
        kw = dict(srcB=srcs[1] if len(srcs) > 1 else None, bias=bias, relu=relu)
        if mode == "split":
            outs = [torch.zeros(N, H, W_, 128, dtype=dt, device=DEV), torch.zeros(N, H, W_, nout - 128, dtype=dt, device=DEV)]
            kw.update(out_mode=2, out2=outs[1], split_c=128)
        st = torch.zeros(2, nout, device=DEV)
        ops.set_option("fwd_tap64", 2 if tile == 256 else 3)   # the 256x256 / 256x128 configuration
        ops.set_option("fwd_halo", 0)   # (the <= 128-output halo kernels would take the narrow shapes)
        ops.set_option("tap64p_halo", halo)
        ops.set_option("fwd_w4", 0)   # (the four-wave form takes the Nout % 256 == 0 shapes: its own test)
        ops.set_option("tap64p_wide", wide)
        ops.set_option("tap64p_claim", min(claim, 1))
        ops.set_option("claim_full", 1 if claim == 2 else 0)   # (every tile claimed: the 3 / 7-block grids)
        if grid:
            ops.set_option("tap64_persist_grid", grid)
        try:
            ops.conv_fwd(srcs[0], Wt, nout, out=outs[0], bn_stats=(st[0], st[1]), **kw)
            torch.cuda.synchronize()
            kname = _lib.lib().adp_last_kernel().decode()
        finally:
            for o_ in ("fwd_tap64", "fwd_halo", "tap64p_halo", "tap64_persist_grid", "fwd_w4", "tap64p_wide", "tap64p_claim",
                       "claim_full"):
                ops.set_option(o_, None)
        assert kname.startswith("igemm_fwd_tap64p_kernel<256, %d, %d, false, %s, false" % (
            tile, 2 if tile == 256 else 3, "true" if halo else "false")), kname
        res.append((torch.cat(outs, -1).double(), st.double()))
    (yh, sh_), (yg, sg) = res
    assert (yh - ref).abs().max().item() < 0.02 * ref.abs().max().item()
    assert (yh - yg).abs().max().item() <= 0.01 * ref.abs().max().item()
    torch.testing.assert_close(sh_, sg, rtol=1e-4, atol=1e-2)
    rf = ref.reshape(-1, nout)
    torch.testing.assert_close(sh_[0], rf.sum(0), rtol=2e-3, atol=1.0)


@pytest.mark.parametrize("claim", [0, 1], ids=["static", "claimed"])
@pytest.mark.parametrize("grid", [None, 3, 7], ids=["chip_grid", "3_blocks", "7_blocks"])
@pytest.mark.parametrize("mode", ["plain", "concat", "up", "split", "n352"])
def test_tap64p_f32_halo(mode, grid, claim):
    """f32 halo form of the persistent forward (igemm_fwd_tap64p_kernel<256, 128, 3, ..., F32>: 32-channel K steps,
    eight exact v_mfma_f32_16x16x4_f32 per 16x16 block and step) vs a float64 convolution of the same f32 operands
    (<= 1e-5 of the largest element: only the f32 accumulation differs) and vs the non-persistent f32 tap64 kernel
    (option tap64p_f32=0) to the same bound; BatchNorm sums to f32 order. adipose_v3's f32 channel strides (96 /
    192 / 352: a ragged last N tile), two sources, the nearest-x2 upsample gather, a split store."""
    dt = torch.float32
    g = torch.Generator().manual_seed(21)
    N, H, W_ = 2, 32, 64
    parts, nout, up = {"plain": ([96], 96, 1), "concat": ([64, 128], 192, 1), "up": ([192], 96, 2),
                       "split": ([96, 96], 192, 1), "n352": ([352], 352, 1)}[mode]
    Hs, Ws = H // up, W_ // up
    cin = sum(parts)
    srcs = [torch.randn(N, Hs, Ws, c, generator=g).to(DEV, dt) for c in parts]
    Wt = (torch.randn(((nout + 63) // 64) * 64, 9 * cin, generator=g) * 0.03).to(DEV, dt)
    bias = torch.randn(nout, generator=g).to(DEV)
    x = torch.cat([t.double() for t in srcs], -1).permute(0, 3, 1, 2)
    if up == 2:
        x = x.repeat_interleave(2, 2).repeat_interleave(2, 3)
    wk = Wt[:nout].double().view(nout, 3, 3, cin).permute(0, 3, 1, 2)
    ref = F.conv2d(x, wk, padding=1).permute(0, 2, 3, 1) + bias.double()
    relu = mode != "split"
    if relu:
        ref = ref.clamp_min(0.0)
    res = []
    for persist in (1, 0):
        outs = [torch.zeros(N, H, W_, nout, dtype=dt, device=DEV)]
        kw = dict(srcB=srcs[1] if len(srcs) > 1 else None, bias=bias, relu=relu, up=up == 2)
        if mode == "split":
            outs = [torch.zeros(N, H, W_, 96, dtype=dt, device=DEV), torch.zeros(N, H, W_, nout - 96, dtype=dt, device=DEV)]
            kw.update(out_mode=2, out2=outs[1], split_c=96)
        st = torch.zeros(2, nout, device=DEV)
        ops.set_option("tap64p_f32", persist)
        ops.set_option("tap64p_claim", claim)
        ops.set_option("fwd_tap64", 3)   # the 256x128 tile (these small launches would score 256x64 higher)
        if grid:
            ops.set_option("tap64_persist_grid", grid)
        try:
            ops.conv_fwd(srcs[0], Wt, nout, out=outs[0], bn_stats=(st[0], st[1]), **kw)
            torch.cuda.synchronize()
            kname = _lib.lib().adp_last_kernel().decode()
        finally:
            for o_ in ("tap64p_f32", "tap64p_claim", "tap64_persist_grid", "fwd_tap64"):
                ops.set_option(o_, None)
        if persist:
            assert kname == "igemm_fwd_tap64p_kernel<256, 128, 3, false, true, false, false, true, -1>", kname
        else:
            assert kname.startswith("igemm_fwd_tap64_kernel<4, 2, 64"), kname
        res.append((torch.cat(outs, -1).double(), st.double()))
    (yp, sp), (yt, stt) = res
    scale = ref.abs().max().item()
    assert (yp - ref).abs().max().item() < 1e-5 * scale
    assert (yp - yt).abs().max().item() < 1e-5 * scale
    rf = ref.reshape(-1, nout)
    torch.testing.assert_close(sp[0], rf.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(sp[1], (rf * rf).sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(sp, stt, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("persist", [1, 0], ids=["tap64p", "tap64"])
@pytest.mark.parametrize("nout", [96, 192, 352])
def test_f32_column_skip_bit_identical(nout, persist):
    """f32 256x128 tiles (option f32_skip, default on): the waves sharing a SIMD take the two column halves and a
    wave skips the MFMAs of 32-column groups wholly past Nout. Every stored column keeps its K order, so the output
    and the BatchNorm sums are bit-identical to the unskipped launch (f32_skip=0)."""
    dt = torch.float32
    g = torch.Generator().manual_seed(nout)
    N, H, W_, cin = 2, 24, 64, 96
    x = torch.randn(N, H, W_, cin, generator=g).to(DEV, dt)
    Wt = (torch.randn(((nout + 63) // 64) * 64, 9 * cin, generator=g) * 0.03).to(DEV, dt)
    bias = torch.randn(nout, generator=g).to(DEV)
    res = []
    for skip in (1, 0):
        out = torch.zeros(N, H, W_, nout, dtype=dt, device=DEV)
        st = torch.zeros(2, nout, device=DEV)
        for o_, v in (("f32_skip", skip), ("tap64p_f32", persist), ("fwd_tap64", 3)):
            ops.set_option(o_, v)
        try:
            ops.conv_fwd(x, Wt, nout, out=out, bias=bias, relu=True, bn_stats=(st[0], st[1]))
            torch.cuda.synchronize()
            kname = _lib.lib().adp_last_kernel().decode()
        finally:
            for o_ in ("f32_skip", "tap64p_f32", "fwd_tap64"):
                ops.set_option(o_, None)
        assert kname.startswith("igemm_fwd_tap64p_kernel<256, 128, 3" if persist else "igemm_fwd_tap64_kernel<4, 2, 64"), kname
        res.append((out, st))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])
    xd = x.double().permute(0, 3, 1, 2)
    ref = (F.conv2d(xd, Wt[:nout].double().view(nout, 3, 3, cin).permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
           + bias.double()).clamp_min(0.0)
    assert (res[0][0].double() - ref).abs().max().item() < 1e-5 * ref.abs().max().item()


@pytest.mark.parametrize("form", ["halo256", "halo128", "gather_dil2", "convt"])
def test_tap64p_claim_counters_reset(form):
    """Dynamic tile claiming (option tap64p_claim): every launch takes its tiles from a counter slot of the
    library's ring (adp::claim_slot, 64 slots) and the last block to finish re-zeroes it. 150 launches -- more
    than two turns of the ring, grids of 256 / 7 / 1 blocks, several N columns -- must all equal the static
    launch bit for bit: a slot left non-zero would make a later launch skip tiles (stale output rows)."""
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(31)
    N, H, W_ = 2, 32, 64
    kw = {}
    if form == "convt":
        cin, cs = 128, 64
        x = torch.randn(N, H, W_, cin, generator=g).to(DEV, dt)
        Wt = (torch.randn(4 * cs, cin, generator=g) * 0.05).to(DEV, dt)
        nout, oshape = 4 * cs, (N, 2 * H, 2 * W_, cs)
        kw.update(bias=torch.randn(cs, generator=g).to(DEV), kh=1, kw=1, pad=0, out_mode=1, shuffle_c=cs)
        opts = dict(fwd_tap64=2, tap64p_cfg=3)
    else:
        cin, nout = 128, 512
        x = torch.randn(N, H, W_, cin, generator=g).to(DEV, dt)
        Wt = (torch.randn(nout, 9 * cin, generator=g) * 0.03).to(DEV, dt)
        oshape = (N, H, W_, nout)
        kw.update(bias=torch.randn(nout, generator=g).to(DEV), relu=True)
        opts = dict(fwd_tap64=2 if form != "halo128" else 3, fwd_halo=0, fwd_w4=0)
        if form == "gather_dil2":
            kw.update(dil=2, pad=2)
    outs = []
    try:
        for k_, v_ in opts.items():
            ops.set_option(k_, v_)
        for i in range(150):
            claim = 0 if i == 0 else 1
            ops.set_option("tap64p_claim", claim)
            ops.set_option("tap64_persist_grid", (None, 7, 1)[i % 3] if i else None)
            o = torch.full(oshape, float("nan"), dtype=dt, device=DEV)
            ops.conv_fwd(x, Wt, nout, out=o, **kw)
            outs.append(o)
        torch.cuda.synchronize()
        kname = _lib.lib().adp_last_kernel().decode()
    finally:
        for k_ in list(opts) + ["tap64p_claim", "tap64_persist_grid"]:
            ops.set_option(k_, None)
    assert kname.startswith("igemm_fwd_tap64p_kernel"), kname
    for i, o in enumerate(outs[1:], 1):
        assert torch.equal(o, outs[0]), (i, torch.isnan(o.float()).sum().item())


@pytest.mark.parametrize("grid", [None, 3, 7], ids=["chip_grid", "3_blocks", "7_blocks"])
@pytest.mark.parametrize("mode", ["one_chunk", "concat", "ragged_n", "split", "up2"])
def test_tap64p_wreg_matches_dma(mode, grid):
    """The 256x256 halo kernel with its weights and halo groups staged through registers (ds_write into the
    free stage, option tap64p_wreg=1) against the LDS-DMA form (tap64p_wreg=0, the default): the same K
    order and fragments, so the stored outputs are identical and the BatchNorm sums agree to f32 order."""
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(17)
    N, H, W_ = 2, 32, 64
    parts = {"one_chunk": [64], "concat": [64, 128], "ragged_n": [128], "split": [128, 64], "up2": [192]}[mode]
    nout = {"ragged_n": 320}.get(mode, 256)
    up = mode == "up2"
    cin = sum(parts)
    srcs = [torch.randn(N, H // (2 if up else 1), W_ // (2 if up else 1), c, generator=g).to(DEV, dt) for c in parts]
    Wt = (torch.randn(((nout + 63) // 64) * 64, 9 * cin, generator=g) * 0.03).to(DEV, dt)
    bias = torch.randn(nout, generator=g).to(DEV)
    res = []
    for wreg in (1, 0):
        outs = [torch.zeros(N, H, W_, nout, dtype=dt, device=DEV)]
        kw = dict(srcB=srcs[1] if len(srcs) > 1 else None, bias=bias, relu=mode != "split", up=up)
        if mode == "split":
            outs = [torch.zeros(N, H, W_, 128, dtype=dt, device=DEV), torch.zeros(N, H, W_, nout - 128, dtype=dt, device=DEV)]
            kw.update(out_mode=2, out2=outs[1], split_c=128)
        st = torch.zeros(2, nout, device=DEV)
        opts = dict(fwd_tap64=2, fwd_halo=0, fwd_w4=0, tap64p_wreg=wreg)
        if grid:
            opts["tap64_persist_grid"] = grid
        for k_, v_ in opts.items():
            ops.set_option(k_, v_)
        try:
            ops.conv_fwd(srcs[0], Wt, nout, out=outs[0], bn_stats=(st[0], st[1]), **kw)
            torch.cuda.synchronize()
            kname = _lib.lib().adp_last_kernel().decode()
        finally:
            for k_ in opts:
                ops.set_option(k_, None)
        # (the DMA arm: the default line-ordered-epilogue instance, EPIC = 3 with static tile lists, 2 with claiming)
        assert kname in (("igemm_fwd_tap64p_kernel<256, 256, 2, false, true, false, true, false, -1>",) if wreg else
                         ("igemm_fwd_tap64p_kernel<256, 256, 2, false, true, false, false, false, 4>",
                          "igemm_fwd_tap64p_kernel<256, 256, 2, false, true, false, false, false, 3>",
                          "igemm_fwd_tap64p_kernel<256, 256, 2, false, true, false, false, false, 2>")), kname
        res.append((torch.cat(outs, -1), st.double()))
    (y1, s1), (y0, s0) = res
    assert torch.equal(y1, y0), (y1.double() - y0.double()).abs().max().item()
    torch.testing.assert_close(s1, s0, rtol=1e-5, atol=1e-3)


W4_CASES = [
    # name, source channels, Nout, up, relu + bias, BatchNorm sums
    ("one_chunk_stats", [64], 256, 1, False, True),
    ("concat_relu", [64, 128], 256, 1, True, False),
    ("wide_stats", [256], 512, 1, False, True),
    ("up2_concat_stats", [128, 128], 256, 2, False, True),
    ("n1024_relu_stats", [128], 1024, 1, True, True),
]


@pytest.mark.parametrize("grid", [None, 3, 7], ids=["chip_grid", "3_blocks", "7_blocks"])
@pytest.mark.parametrize("case", W4_CASES, ids=[c[0] for c in W4_CASES])
def test_fwd_w4_matches(case, grid):
    """Four-wave direct-weight forward (conv_fwd_w4.hip: one wave per SIMD, 128x128 per wave, weights loaded
    straight into registers, halo through registers into LDS once per chunk) vs a float64 reference convolution
    of the same bf16 operands, and vs the 8-wave LDS-DMA halo kernel (fwd_w4=0): the same chunk / tap / 32-deep
    MFMA order, so the stored outputs are identical; the BatchNorm sums (a different order of f32 additions)
    to 1e-5. Upsample x2 folded into the gather, two sources, 1-4 N tiles, 3 / 7-block grids."""
    name, parts, nout, up, relu, stats = case
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(21)
    N, H, W_ = 2, 32, 64
    cin = sum(parts)
    srcs = [torch.randn(N, H // up, W_ // up, c, generator=g).to(DEV, dt) for c in parts]
    Wt = (torch.randn(nout, 9 * cin, generator=g) * 0.03).to(DEV, dt)
    bias = torch.randn(nout, generator=g).to(DEV) if relu else None
    x = torch.cat([t.double() for t in srcs], -1).permute(0, 3, 1, 2)
    if up == 2:
        x = x.repeat_interleave(2, 2).repeat_interleave(2, 3)
    wk = Wt.double().view(nout, 3, 3, cin).permute(0, 3, 1, 2)
    ref = F.conv2d(x, wk, padding=1).permute(0, 2, 3, 1)
    if relu:
        ref = (ref + bias.double()).clamp_min(0.0)
    res = []
    for w4 in (1, 0):
        out = torch.zeros(N, H, W_, nout, dtype=dt, device=DEV)
        st = torch.zeros(2, nout, device=DEV)
        kw = dict(srcB=srcs[1] if len(srcs) > 1 else None, bias=bias, relu=relu, up=up == 2)
        if stats:
            kw["bn_stats"] = (st[0], st[1])
        ops.set_option("fwd_tap64", 2)   # the 256x256 configuration
        ops.set_option("fwd_halo", 0)
        ops.set_option("fwd_w4", w4)
        if grid:
            ops.set_option("tap64_persist_grid", grid)
            ops.set_option("fwd_w4_grid", grid)
        try:
            ops.conv_fwd(srcs[0], Wt, nout, out=out, **kw)
            torch.cuda.synchronize()
            kname = _lib.lib().adp_last_kernel().decode()
        finally:
            for o_ in ("fwd_tap64", "fwd_halo", "fwd_w4", "tap64_persist_grid", "fwd_w4_grid"):
                ops.set_option(o_, None)
        want = ("igemm_fwd_w4_kernel<%s" % ("true" if stats else "false") if w4 else
                "igemm_fwd_tap64p_kernel<256, 256, 2, false, true, false")
        assert kname.startswith(want), kname
        res.append((out.double(), st.double()))
    (y4, s4), (y8, s8) = res
    assert (y4 - ref).abs().max().item() < 0.02 * ref.abs().max().item()
    assert torch.equal(y4, y8), (y4 - y8).abs().max().item()
    if stats:
        torch.testing.assert_close(s4, s8, rtol=1e-5, atol=1e-3)
        rf = ref.reshape(-1, nout)
        torch.testing.assert_close(s4[0], rf.sum(0), rtol=2e-3, atol=1.0)


@pytest.mark.parametrize("cin,cout", [(64, 64), (128, 128), (128, 64)])
def test_halop_relu_dropout_epilogue(cin, cout):
    """Persistent halo kernel with the ReLU + dropout epilogue (EPI 5, adipose_v3 up*_conv3 in training):
    the same stateless dropout mask as the non-persistent halo kernel (option halo_persist=0), kept values
    = relu(conv + b) / (1 - rate) within bf16 rounding of the no-dropout launch."""
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(43)
    N, H, W_, rate = 2, 16, 64, 0.3
    x = torch.randn(N, H, W_, cin, generator=g).to(DEV, dt)
    Wt = (torch.randn(cout, 9 * cin, generator=g) * 0.05).to(DEV, dt)
    b = torch.randn(cout, generator=g).to(DEV) * 0.1
    res = {}
    for persist in (1, 0):
        for drop in (rate, 0.0):
            out = torch.zeros(N, H, W_, cout, dtype=dt, device=DEV)
            ops.set_option("halo_persist", persist)
            try:
                ops.conv_fwd(x, Wt, cout, out=out, bias=b, relu=True, dropout_rate=drop, dropout_seed=1234)
                torch.cuda.synchronize()
                kname = _lib.lib().adp_last_kernel().decode()
            finally:
                ops.set_option("halo_persist", None)
            assert kname.startswith("igemm_fwd_halop_kernel") == bool(persist), kname
            if persist and drop:
                assert kname.split(", ")[3:5] == ["false", "5"], kname
            res[(persist, drop)] = out.double()
    yp, yn, y0 = res[(1, rate)], res[(0, rate)], res[(1, 0.0)]
    pos = y0 > 1e-2 * y0.abs().max()        # clearly positive before dropout: kept or dropped, never ReLU-zeroed
    kept_p, kept_n = (yp != 0) & pos, (yn != 0) & pos
    assert torch.equal(kept_p, kept_n)      # the same dropout mask
    frac = kept_p.sum().item() / pos.sum().item()
    assert abs(frac - (1 - rate)) < 0.02, frac
    ks = 1.0 / (1.0 - rate)
    assert ((yp - y0 * ks).abs() - 2 ** -6 * (y0 * ks).abs())[kept_p].max().item() < 1e-3
    assert ((yp - yn).abs() - 2 ** -7 * yn.abs()).max().item() < 1e-2


@pytest.mark.parametrize("mode", ["mask", "addend_mask", "split_masks", "split_mask2", "two_chunks", "addend_only"])
def test_halop_mask_addend_epilogue(mode):
    """Persistent halo kernel with the addend / ReLU-backward-mask epilogue (EPI 4: the adipose_v3 data
    gradients, out = (acc + addend) * (mask > 0 ? scale : 0), mask2 on a split store's second part) vs a
    float64 reference and vs the non-persistent halo kernel (option halo_persist=0)."""
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(41)
    N, H, W_ = 2, 16, 64
    cin = 128 if mode == "two_chunks" else 64
    nout = 128 if mode.startswith("split") else 64
    x = torch.randn(N, H, W_, cin, generator=g).to(DEV, dt)
    Wt = (torch.randn(nout, 9 * cin, generator=g) * 0.05).to(DEV, dt)
    mk = torch.randn(N, H, W_, nout, generator=g).to(DEV, dt)
    ad = torch.randn(N, H, W_, nout, generator=g).to(DEV, dt) if "addend" in mode else None
    xd = x.double().permute(0, 3, 1, 2)
    wk = Wt.double().view(nout, 3, 3, cin).permute(0, 3, 1, 2)
    ref = F.conv2d(xd, wk, padding=1).permute(0, 2, 3, 1)
    if ad is not None:
        ref = ref + ad.double()
    sc1, sc2 = 1.25, 0.5
    if mode != "addend_only":
        scale = torch.full((nout,), sc1, dtype=torch.float64, device=DEV)
        if mode.startswith("split"):
            scale[64:] = sc2
        keep = mk.double() > 0
        if mode == "split_mask2":   # no mask on the first part
            scale[:64] = 1.0
            keep[..., :64] = True
        ref = torch.where(keep, ref * scale, torch.zeros_like(ref))
    res = []
    for persist in (1, 0):
        kw = dict(addend=ad)
        if mode.startswith("split"):
            o1 = torch.zeros(N, H, W_, 64, dtype=dt, device=DEV)
            o2 = torch.zeros(N, H, W_, 64, dtype=dt, device=DEV)
            kw.update(out_mode=2, out2=o2, split_c=64, mask=mk[..., :64].contiguous(), mask_scale=sc1,
                      mask2=mk[..., 64:].contiguous(), mask2_scale=sc2, addend=None)
            if mode == "split_mask2":
                kw.update(mask=None)
            outs = [o1, o2]
        else:
            outs = [torch.zeros(N, H, W_, nout, dtype=dt, device=DEV)]
            if mode != "addend_only":
                kw.update(mask=mk, mask_scale=sc1)
        ops.set_option("halo_persist", persist)
        try:
            ops.conv_fwd(x, Wt, nout, out=outs[0], **kw)
            torch.cuda.synchronize()
            kname = _lib.lib().adp_last_kernel().decode()
        finally:
            ops.set_option("halo_persist", None)
        assert kname.startswith("igemm_fwd_halop_kernel") == bool(persist), kname
        if persist:
            assert kname.split(", ")[3:5] == ["false", "4"], kname
        res.append(torch.cat(outs, -1).double())
    tol = 2 ** -7 * ref.abs() + 1e-3 * ref.abs().max()
    assert ((res[0] - ref).abs() - tol).max().item() < 0, (res[0] - ref).abs().max().item()
    assert ((res[0] - res[1]).abs() - tol).max().item() < 0


@pytest.mark.parametrize("form", ["halop_1ch", "halop_2ch", "tap64p_256", "tap64p_128", "w4_256"])
@pytest.mark.parametrize("grid", [None, 3], ids=["chip_grid", "3_blocks"])
def test_upsample_gather_halo_forms(form, grid):
    """Nearest-x2 upsample folded into the halo gathers of the persistent forward kernels (adipose_v3's
    UpSampling2D + 3x3 conv, train_adipose_unet_v3.py:691-692): halop (one / two 64-channel chunks) and the
    256x256 / 256x128 halo forms of tap64p, vs a float64 convolution of the upsampled bf16 operands and
    vs the non-persistent tap64 kernel's gather (different f32 summation order: within bf16 rounding);
    BatchNorm sums to 1e-4."""
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(13)
    N, Hs, Ws = 2, 16, 32
    cin, nout, kern = {"halop_1ch": (64, 64, "igemm_fwd_halop_kernel<false, 1, 64"),
                       "halop_2ch": (128, 64, "igemm_fwd_halop_kernel<false, 2, 32"),
                       "tap64p_256": (128, 256, "igemm_fwd_tap64p_kernel<256, 256, 2, false, true, false"),
                       "tap64p_128": (192, 128, "igemm_fwd_tap64p_kernel<256, 128, 3, false, true, false, false"),
                       "w4_256": (128, 256, "igemm_fwd_w4_kernel<true")}[form]
    x = torch.randn(N, Hs, Ws, cin, generator=g).to(DEV, dt)
    Wt = (torch.randn(nout, 9 * cin, generator=g) * 0.03).to(DEV, dt)
    bias = torch.randn(nout, generator=g).to(DEV)
    xu = x.double().repeat_interleave(2, 1).repeat_interleave(2, 2).permute(0, 3, 1, 2)
    wk = Wt.double().view(nout, 3, 3, cin).permute(0, 3, 1, 2)
    ref = (F.conv2d(xu, wk, padding=1).permute(0, 2, 3, 1) + bias.double()).clamp_min(0.0)
    res = []
    for persist in (1, 0):
        out = torch.zeros(N, 2 * Hs, 2 * Ws, nout, dtype=dt, device=DEV)
        st = torch.zeros(2, nout, device=DEV)
        opts = {"halo_persist": persist, "tap64_persist": persist}
        if form.startswith("tap64p"):   # the 256x256 / 256x128 configuration (small M picks narrow tiles)
            opts.update(fwd_halo=0, fwd_tap64=2 if form == "tap64p_256" else 3, fwd_w4=0)
        if form == "w4_256":
            opts.update(fwd_halo=0, fwd_tap64=2, fwd_w4=1)
        if grid:
            opts.update(tap64_persist_grid=grid, halo_persist_grid=grid, fwd_w4_grid=grid)
        for k_, v_ in opts.items():
            ops.set_option(k_, v_)
        try:
            ops.conv_fwd(x, Wt, nout, out=out, bias=bias, relu=True, up=True, bn_stats=(st[0], st[1]))
            torch.cuda.synchronize()
            kname = _lib.lib().adp_last_kernel().decode()
        finally:
            for k_ in opts:
                ops.set_option(k_, None)
        res.append((out.double(), st.double(), kname))
    (yp, sp, kp), (yn, sn, kn) = res
    assert kp.startswith(kern), kp
    assert not kn.startswith("igemm_fwd_halop") and not kn.startswith("igemm_fwd_tap64p") and "w4" not in kn, kn
    assert (yp - ref).abs().max().item() < 0.02 * ref.abs().max().item()
    assert (yp - yn).abs().max().item() <= 0.01 * ref.abs().max().item()
    torch.testing.assert_close(sp, sn, rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("claim", [0, 1], ids=["static", "claimed"])
@pytest.mark.parametrize("wide", [0, 1], ids=["st8", "st16"])
@pytest.mark.parametrize("cfg", [1, 2, 3], ids=["256x256x2", "256x128x3", "128x256x3"])
@pytest.mark.parametrize("grid", [None, 3], ids=["chip_grid", "3_blocks"])
@pytest.mark.parametrize("mode", ["plain", "concat", "convt_shuffle", "split", "convt_dgrad", "bnr", "dilated"])
def test_tap64_persistent_matches(mode, grid, cfg, wide, claim):
    """Persistent tap64 kernel (conv_fwd_tap64p.hip: one K-step stream over the block's tiles through an
    NST-stage LDS ring, register epilogue with 8-B buffer stores, or with 16-B stores of channel pairs joined
    by permlane16_swap: option tap64p_wide) in its three tile / ring forms vs the
    non-persistent kernel on the same launch: bit-identical outputs and equal BatchNorm sums (statistics,
    or the fused BatchNorm-backward reduction for bnr); a 3-block grid makes every block walk many tiles
    (ragged last M tile, partial N tile), so the cross-tile prefetch and the counted vmcnt waits are
    exercised. claimed: the persistent blocks take their tiles from an atomic counter (option tap64p_claim),
    which changes which block computes a tile, not how: still bit-identical."""
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(11)
    kw = {}
    bnr = None
    if mode in ("plain", "concat", "split", "bnr", "dilated"):
        N, S = 2, 23
        parts = [128] if mode in ("plain", "bnr", "dilated") else [64, 128]
        cin = sum(parts)
        nout = 320 if mode in ("plain", "bnr", "dilated") else 256
        srcs = [torch.randn(N, S, S, c, generator=g).to(DEV, dt) for c in parts]
        W = (torch.randn(((nout + 63) // 64) * 64, 9 * cin, generator=g) * 0.03).to(DEV, dt)
        args = (srcs[0], W, nout)
        if len(srcs) > 1:
            kw["srcB"] = srcs[1]
        outs = [torch.zeros(N, S, S, nout, dtype=dt, device=DEV)]
        if mode == "split":
            outs = [torch.zeros(N, S, S, 128, dtype=dt, device=DEV), torch.zeros(N, S, S, 128, dtype=dt, device=DEV)]
            kw.update(out_mode=2, out2=outs[1], split_c=128)
        elif mode == "bnr":   # data gradient with the fused BatchNorm-backward reduction of the layer below
            z = torch.randn(N, S, S, nout, generator=g).to(DEV, dt)
            vec = [(torch.rand(nout, generator=g) + 0.5).to(DEV) for _ in range(4)]
            bnr = (z, vec[0], vec[1] - 1.0, vec[2] - 1.0, vec[3])
        else:   # dilated: the adipose_v3 bottleneck's 'same' 3x3 with dilation 4 (gather form, not halo)
            kw.update(bias=torch.randn(nout, generator=g).to(DEV), relu=mode in ("plain", "dilated"))
            if mode == "dilated":
                kw.update(dil=4, pad=4)
        stats_c = nout
    elif mode == "convt_shuffle":   # ConvTranspose 2x2/s2 forward: 1x1 GEMM + pixel-shuffle store
        N, S, cin, cs = 2, 19, 128, 64
        x = torch.randn(N, S, S, cin, generator=g).to(DEV, dt)
        W = (torch.randn(4 * cs, cin, generator=g) * 0.05).to(DEV, dt)
        args = (x, W, 4 * cs)
        outs = [torch.zeros(N, 2 * S, 2 * S, cs, dtype=dt, device=DEV)]
        kw.update(bias=torch.randn(cs, generator=g).to(DEV), kh=1, kw=1, pad=0, out_mode=1, shuffle_c=cs)
        stats_c = cs
    else:   # ConvTranspose data gradient: stride-2 4-tap gather over the 2x-resolution gradient
        N, S, cin, cs = 2, 21, 256, 64
        dt_ = torch.randn(N, 2 * S, 2 * S, cs, generator=g).to(DEV, dt)
        W = (torch.randn(cin, 4 * cs, generator=g) * 0.05).to(DEV, dt)
        args = (dt_, W, cin)
        outs = [torch.zeros(N, S, S, cin, dtype=dt, device=DEV)]
        kw.update(kh=2, kw=2, dil=1, pad=0, stride=2, Ho=S, Wo=S)
        stats_c = cin
    res = []
    for persist in (0, 1):
        for o in outs:
            o.zero_()
        st = torch.zeros(2, stats_c, device=DEV)
        ops.set_option("tap64_persist", persist)
        ops.set_option("fwd_tap64", 2)   # the 256x256 configuration (small problems would pick narrower tiles)
        ops.set_option("tap64p_cfg", cfg)
        ops.set_option("tap64p_wide", wide)
        ops.set_option("tap64p_claim", claim)
        if grid:
            ops.set_option("tap64_persist_grid", grid)
        try:
            if bnr is not None:
                ops.conv_fwd(*args, out=outs[0], bn_reduce=bnr + (st[1], st[0]), **kw)
            else:
                ops.conv_fwd(*args, out=outs[0], bn_stats=(st[0], st[1]), **kw)
            torch.cuda.synchronize()
            kname = _lib.lib().adp_last_kernel().decode()
        finally:
            for o_ in ("tap64_persist", "fwd_tap64", "tap64_persist_grid", "tap64p_cfg", "tap64p_wide", "tap64p_claim"):
                ops.set_option(o_, None)
        res.append(([o.clone() for o in outs], st.clone(), kname))
    assert res[0][2].startswith("igemm_fwd_tap64_kernel") and res[1][2].startswith("igemm_fwd_tap64p_kernel"), \
        (res[0][2], res[1][2])
    for a_, b_ in zip(res[0][0], res[1][0]):
        assert torch.equal(a_, b_)
    assert relerr(res[1][1], res[0][1]) < 1e-5


@pytest.mark.parametrize("cfg", [2, 3, 4], ids=["256x256", "256x128", "512x64"])
@pytest.mark.parametrize("mode", ["plain", "concat", "bnr", "convt_dgrad", "f32"])
def test_tap64_kpipe_matches(mode, cfg):
    """Non-persistent tap64 kernel with the software-pipelined K loop (option tap64_kpipe=1: the barrier in
    the middle of the previous step, the refill of step t + 2 issued there, B half 0 of the next step
    preloaded behind the fourth MFMA cluster) against the default loop: bit-identical outputs and equal
    BatchNorm sums (statistics or the fused BN-backward reduction); bf16 and exact-f32 forms."""
    g = torch.Generator().manual_seed(23)
    dt = torch.float32 if mode == "f32" else torch.bfloat16
    kw, bnr = {}, None
    if mode != "convt_dgrad":
        N, S = 2, 23
        parts = [64, 128] if mode == "concat" else ([64] if mode == "f32" else [128])
        cin = sum(parts)
        nout = 256 if mode != "plain" else 320
        srcs = [torch.randn(N, S, S, c, generator=g).to(DEV, dt) for c in parts]
        W = (torch.randn(((nout + 63) // 64) * 64, 9 * cin, generator=g) * 0.03).to(DEV, dt)
        args = (srcs[0], W, nout)
        if len(srcs) > 1:
            kw["srcB"] = srcs[1]
        out_shape = (N, S, S, nout)
        if mode == "bnr":
            z = torch.randn(N, S, S, nout, generator=g).to(DEV, dt)
            vec = [(torch.rand(nout, generator=g) + 0.5).to(DEV) for _ in range(4)]
            bnr = (z, vec[0], vec[1] - 1.0, vec[2] - 1.0, vec[3])
        else:
            kw.update(bias=torch.randn(nout, generator=g).to(DEV), relu=True)
        stats_c = nout
    else:   # ConvTranspose data gradient: stride-2 4-tap gather over the 2x-resolution gradient
        N, S, cin, cs = 2, 21, 256, 64
        dt_ = torch.randn(N, 2 * S, 2 * S, cs, generator=g).to(DEV, dt)
        W = (torch.randn(cin, 4 * cs, generator=g) * 0.05).to(DEV, dt)
        args = (dt_, W, cin)
        out_shape = (N, S, S, cin)
        kw.update(kh=2, kw=2, dil=1, pad=0, stride=2, Ho=S, Wo=S)
        stats_c = cin
    res = []
    for kp in (1, 0):
        out = torch.zeros(out_shape, dtype=dt, device=DEV)
        st = torch.zeros(2, stats_c, device=DEV)
        opts = dict(tap64_persist=0, fwd_tap64=cfg, fwd_halo=0, tap64_kpipe=kp)
        for k_, v_ in opts.items():
            ops.set_option(k_, v_)
        try:
            if bnr is not None:
                ops.conv_fwd(*args, out=out, bn_reduce=bnr + (st[1], st[0]), **kw)
            else:
                ops.conv_fwd(*args, out=out, bn_stats=(st[0], st[1]), **kw)
            torch.cuda.synchronize()
            kname = _lib.lib().adp_last_kernel().decode()
        finally:
            for k_ in opts:
                ops.set_option(k_, None)
        assert kname.startswith("igemm_fwd_tap64_kernel<"), kname
        res.append((out.clone(), st.clone()))
    assert torch.equal(res[0][0], res[1][0]), (res[0][0].double() - res[1][0].double()).abs().max().item()
    assert relerr(res[0][1], res[1][1]) < 1e-5


def test_halo_fused_epilogues():
    """Halo kernel (conv_fwd_halo.hip): fused BatchNorm statistics of a forward launch vs the oracle,
    and the fused BatchNorm-backward reduction of a data-gradient launch vs adp_bn_bwd_reduce run on
    the same stored gradient."""
    dt = torch.bfloat16
    N, S, cin, cout = 2, 32, 64, 64
    xs, kern, bias, l = make_case(N, S, [cin], cout, 1, False, seed=21)
    W = torch.from_numpy(l.keras_to_packed(kern.numpy())).to(DEV).to(dt).contiguous()
    x = nhwc_pad(xs[0], l.Cin_s, dt)
    out = torch.zeros((N, S, S, l.cout_s), dtype=dt, device=DEV)
    st = torch.zeros(2, l.cout_s, device=DEV)
    ops.conv_fwd(x, W, l.Nout, out=out, bias=bias.to(DEV), relu=True, bn_stats=(st[0], st[1]))
    from adipose_amd import _lib
    assert "halo" in _lib.lib().adp_last_kernel().decode()
    ref = oracle_fwd([rb(xs[0], dt)], rb(kern, dt), bias, 1, False).reshape(-1, cout)
    assert relerr(st[0, :cout], ref.sum(0)) < 2e-2 and relerr(st[1, :cout], (ref * ref).sum(0)) < 2e-2
    # data gradient with the fused reduction; z/scale/shift/mean/invstd of a synthetic BN layer
    g = torch.Generator().manual_seed(22)
    dZ = nhwc_pad(torch.randn(N, S, S, cout, generator=g), l.cout_s, dt)
    Wd = torch.zeros((l.dNpad, l.dKpad), dtype=dt, device=DEV)
    ops.pack_weights(torch.from_numpy(l.keras_to_packed(kern.numpy())).to(DEV), Wd, 1, taps=9, cin_s=l.Cin_s,
                     nout=l.cout_s)
    z = nhwc_pad(torch.randn(N, S, S, cin, generator=g), l.Cin_s, dt)
    sc, sh = (torch.rand(l.Cin_s, generator=g) + 0.5).to(DEV), (torch.randn(l.Cin_s, generator=g) * 0.2).to(DEV)
    mu, ist = (torch.randn(l.Cin_s, generator=g) * 0.1).to(DEV), (torch.rand(l.Cin_s, generator=g) + 0.5).to(DEV)
    dA = torch.zeros((N, S, S, l.Cin_s), dtype=dt, device=DEV)
    dg, db = torch.zeros(l.Cin_s, device=DEV), torch.zeros(l.Cin_s, device=DEV)
    ops.conv_fwd(dZ, Wd, l.Cin_s, out=dA, bn_reduce=(z, sc, sh, mu, ist, dg, db))
    assert "halo" in _lib.lib().adp_last_kernel().decode()
    dg2, db2 = torch.zeros_like(dg), torch.zeros_like(db)
    ops.bn_bwd_reduce(dA, z, sc, sh, mu, ist, dg2, db2)
    torch.cuda.synchronize()
    assert relerr(db, db2) < 1e-4 and relerr(dg, dg2) < 1e-4


@pytest.mark.parametrize("S,N", [(32, 2), (64, 3)])
def test_persistent_halo_split_and_stats(S, N):
    """Persistent halo kernel, 128 output channels in two halves: split store (out_mode 2, split_c 64)
    equals the plain store sliced, BatchNorm statistics of both halves, vs the oracle."""
    from adipose_amd import _lib
    dt = torch.bfloat16
    xs, kern, bias, l = make_case(N, S, [64], 128, 1, False, seed=31)
    W = torch.from_numpy(l.keras_to_packed(kern.numpy())).to(DEV).to(dt).contiguous()
    x = nhwc_pad(xs[0], l.Cin_s, dt)
    # BatchNorm statistics of the pre-activation output (the unet_bn form: no ReLU on the conv)
    out = torch.zeros((N, S, S, 128), dtype=dt, device=DEV)
    st = torch.zeros(2, 128, device=DEV)
    ops.conv_fwd(x, W, 128, out=out, bias=bias.to(DEV), bn_stats=(st[0], st[1]))
    assert _lib.lib().adp_last_kernel().decode().startswith("igemm_fwd_halop_kernel")
    ref = oracle_fwd([rb(xs[0], dt)], rb(kern, dt), bias, 1, False, relu=False)
    assert relerr(out, ref) < TOL[dt]
    r2 = ref.reshape(-1, 128)
    assert relerr(st[0], r2.sum(0)) < 2e-2 and relerr(st[1], (r2 * r2).sum(0)) < 2e-2
    # ReLU epilogue, plain and split store
    out = torch.zeros((N, S, S, 128), dtype=dt, device=DEV)
    ops.conv_fwd(x, W, 128, out=out, bias=bias.to(DEV), relu=True)
    assert _lib.lib().adp_last_kernel().decode().startswith("igemm_fwd_halop_kernel")
    assert relerr(out, oracle_fwd([rb(xs[0], dt)], rb(kern, dt), bias, 1, False)) < TOL[dt]
    o1 = torch.zeros((N, S, S, 64), dtype=dt, device=DEV)
    o2 = torch.zeros((N, S, S, 72), dtype=dt, device=DEV)   # wider stride than the 64 channels stored
    ops.conv_fwd(x, W, 128, out=o1, bias=bias.to(DEV), relu=True, out_mode=2, out2=o2, split_c=64)
    assert _lib.lib().adp_last_kernel().decode().startswith("igemm_fwd_halop_kernel")
    torch.cuda.synchronize()
    assert torch.equal(o1, out[..., :64]) and torch.equal(o2[..., :64], out[..., 64:])
    assert o2[..., 64:].abs().max().item() == 0.0


@pytest.mark.parametrize("epi", ["stats", "relu"])
@pytest.mark.parametrize("grid", [None, 3], ids=["chip_grid", "3_blocks"])
@pytest.mark.parametrize("parts,cout,split", [([64], 64, False), ([64], 128, True), ([64, 64], 128, False),
                                              ([128], 64, False)])
def test_halop_pipelined_epilogue_matches(parts, cout, split, grid, epi):
    """Persistent halo kernel with the epilogue of tile k between the MFMAs of tile k+1 (halop_pipe=2)
    vs the tile-serial form: bit-identical outputs (plain or split store) and equal BatchNorm sums; a
    3-block grid gives every block many tiles, so the carried accumulators and the last tile's epilogue
    after the loop are exercised."""
    from adipose_amd import _lib
    dt = torch.bfloat16
    N, S = 2, 64
    g = torch.Generator().manual_seed(53)
    xs = [torch.randn(N, S, S, c, generator=g).to(DEV, dt) for c in parts]
    cin = sum(parts)
    W = (torch.randn(cout, 9 * cin, generator=g) * 0.03).to(DEV, dt)
    bias = torch.randn(cout, generator=g).to(DEV)
    res = []
    for pipe in (0, 1):
        ops.set_option("halop_pipe", 2 * pipe)   # 2: every (non-BNR) form pipelined
        ops.set_option("halop_swp", 0)           # (the two-chunk forms' default software-pipelined loop replaces it)
        if grid:
            ops.set_option("halo_persist_grid", grid)
        try:
            st = torch.zeros(2, cout, device=DEV)
            kw = dict(srcB=xs[1] if len(xs) > 1 else None, bias=bias, relu=epi == "relu",
                      bn_stats=(st[0], st[1]) if epi == "stats" else None)
            if split:
                o1 = torch.zeros(N, S, S, 64, dtype=dt, device=DEV)
                o2 = torch.zeros(N, S, S, cout - 64, dtype=dt, device=DEV)
                ops.conv_fwd(xs[0], W, cout, out=o1, out_mode=2, out2=o2, split_c=64, **kw)
                outs = [o1, o2]
            else:
                o = torch.zeros(N, S, S, cout, dtype=dt, device=DEV)
                ops.conv_fwd(xs[0], W, cout, out=o, **kw)
                outs = [o]
            torch.cuda.synchronize()
            kname = _lib.lib().adp_last_kernel().decode()
        finally:
            ops.set_option("halop_pipe", None)
            ops.set_option("halop_swp", None)
            ops.set_option("halo_persist_grid", None)
        # igemm_fwd_halop_kernel<BNR, NCH, BN, PIPE, EPI>
        assert kname.startswith("igemm_fwd_halop_kernel") and kname.split(", ")[3] == ("true" if pipe else "false"), kname
        res.append((outs, st))
    for a_, b_ in zip(res[0][0], res[1][0]):
        assert torch.equal(a_, b_)
    if epi == "stats":
        assert relerr(res[1][1], res[0][1]) < 1e-5


@pytest.mark.parametrize("epi", ["stats", "relu", "plain", "mask"])
@pytest.mark.parametrize("grid", [None, 3], ids=["chip_grid", "3_blocks"])
@pytest.mark.parametrize("parts,cout,split,S", [([64], 64, False, 64), ([64], 128, True, 64), ([64], 64, False, 96),
                                                ([64, 64], 128, False, 64), ([128], 64, False, 64)])
def test_halop_swp_matches(parts, cout, split, S, grid, epi):
    """Persistent halo kernel with the software-pipelined K loop (halop_swp=1: the LDS fragments of step s + 1 read
    before the MFMAs of step s) vs the default forms (the pipelined epilogue on the one-chunk layers): the same K
    order, so outputs are bit-identical and the BatchNorm sums equal; one and two input chunks, plain / split stores,
    statistics, ReLU, the mask epilogue."""
    from adipose_amd import _lib
    dt = torch.bfloat16
    N = 2
    g = torch.Generator().manual_seed(57)
    xs = [torch.randn(N, S, S, c, generator=g).to(DEV, dt) for c in parts]
    cin = sum(parts)
    W = (torch.randn(cout, 9 * cin, generator=g) * 0.03).to(DEV, dt)
    bias = torch.randn(cout, generator=g).to(DEV)
    mask = (torch.rand(N, S, S, cout, generator=g) > 0.3).to(DEV, dt) if epi == "mask" else None
    res = []
    for swp in (0, 1):
        ops.set_option("halop_swp", swp)   # (default 2: the two-chunk forms only)
        if grid:
            ops.set_option("halo_persist_grid", grid)
        try:
            st = torch.zeros(2, cout, device=DEV)
            kw = dict(srcB=xs[1] if len(xs) > 1 else None, bias=bias, relu=epi == "relu",
                      bn_stats=(st[0], st[1]) if epi == "stats" else None)
            if mask is not None:
                kw.update(mask=mask, mask_scale=2.0)
            if split:
                o1 = torch.zeros(N, S, S, 64, dtype=dt, device=DEV)
                o2 = torch.zeros(N, S, S, cout - 64, dtype=dt, device=DEV)
                ops.conv_fwd(xs[0], W, cout, out=o1, out_mode=2, out2=o2, split_c=64, **kw)
                outs = [o1, o2]
            else:
                o = torch.zeros(N, S, S, cout, dtype=dt, device=DEV)
                ops.conv_fwd(xs[0], W, cout, out=o, **kw)
                outs = [o]
            torch.cuda.synchronize()
            kname = _lib.lib().adp_last_kernel().decode()
        finally:
            for o_ in ("halop_swp", "halo_persist_grid"):
                ops.set_option(o_, None)
        if epi == "mask" and not kname.startswith("igemm_fwd_halop_kernel"):
            pytest.skip(f"this mask launch is not a persistent halo one ({kname})")
        assert kname.startswith("igemm_fwd_halop_kernel") and kname.endswith(", true>") == bool(swp), kname
        res.append((outs, st))
    for a_, b_ in zip(res[0][0], res[1][0]):
        assert torch.equal(a_, b_)
    if epi == "stats":
        assert relerr(res[1][1], res[0][1]) < 1e-6


@pytest.mark.parametrize("C,cout,S,grid,opt", [(64, 64, 64, None, None), (64, 64, 96, 100, None),
                                               (128, 128, 64, None, None), (128, 128, 32, 96, None),
                                               (64, 96, 64, None, None), (64, 64, 64, None, "halop_bnl"),
                                               (256, 128, 32, None, None)])
def test_conv_bn_on_load_with_act_out(C, cout, S, grid, opt):
    """adp_conv_io.act_outA (round 5): conv_fwd(z, bnA=(scale, shift), act_out=act) with BatchNorm statistics equals
    bn_apply(z) -> act followed by conv_fwd(act) bit for bit: output, statistics and the stored activation. 64 -> 64
    launches take the persistent halo forward's EPI 6 (one launch; also a static grid that does not divide the
    patch count); 128-channel sources, 64 -> 96 outputs, option halop_bnl = 0 and a 256-channel source take the
    library's two-launch fallback. Out-of-image halo pixels must stay 0 (relu(0 * scale + shift) would not be)."""
    from adipose_amd import _lib
    dt = torch.bfloat16
    N = 2
    g = torch.Generator().manual_seed(61)
    z = (torch.randn(N, S, S, C, generator=g) * 2).to(DEV, dt)
    sc = (torch.rand(C, generator=g) + 0.5).to(DEV)
    sh = (torch.randn(C, generator=g) * 0.5 + 0.3).to(DEV)   # (mostly positive: a zero halo would show)
    W = (torch.randn(ops.round_up(cout, 64), 9 * C, generator=g) * 0.03).to(DEV, dt)
    act_ref = torch.zeros_like(z)
    o_ref = torch.zeros(N, S, S, cout, dtype=dt, device=DEV)
    st_ref = torch.zeros(2, cout, device=DEV)
    ops.bn_apply(z, sc, sh, act_ref)
    ops.conv_fwd(act_ref, W, cout, out=o_ref, bn_stats=(st_ref[0], st_ref[1]))
    act = torch.full_like(z, 7.0)
    o = torch.zeros_like(o_ref)
    st = torch.zeros_like(st_ref)
    if grid:
        ops.set_option("halo_persist_grid", grid)
    if opt:
        ops.set_option(opt, 0)
    try:
        ops.conv_fwd(z, W, cout, out=o, bnA=(sc, sh), act_out=act, bn_stats=(st[0], st[1]))
        kname = _lib.lib().adp_last_kernel().decode()
        torch.cuda.synchronize()
    finally:
        ops.set_option("halo_persist_grid", None)
        if opt:
            ops.set_option(opt, None)
    fused = C == 64 and cout == 64 and not opt
    assert (", 6, " in kname) == fused, kname
    assert torch.equal(act, act_ref)
    assert torch.equal(o, o_ref), (o.float() - o_ref.float()).abs().max().item()
    assert torch.equal(st, st_ref), relerr(st, st_ref)


@pytest.mark.parametrize("N,H,W,cin,cout,cfg", [(2, 32, 32, 256, 256, 2), (1, 24, 40, 256, 192, 2),
                                                (2, 16, 64, 128, 128, 5), (1, 32, 32, 512, 256, 2)])
def test_tap64_bnr_lds_epilogue(N, H, W, cin, cout, cfg):
    """The tap64 data gradient's LDS-staged BN-backward-reduction epilogue (option tap64_bnr_lds: z by LDS-DMA, dA
    staged as bf16) against the row-serial epilogue: the stored gradient bit for bit and the same dgamma / dbeta sums
    (same values, same order); ragged pixel counts (M not a multiple of the 256-row tile) and a 192-wide N tile."""
    from adipose_amd import _lib
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(71)
    x = torch.randn(N, H, W, cin, generator=g).to(DEV, dt)
    z = (torch.randn(N, H, W, cout, generator=g) * 2).to(DEV, dt)
    W_ = (torch.randn(ops.round_up(cout, 64), 9 * cin, generator=g) * 0.03).to(DEV, dt)
    vec = lambda: (torch.rand(cout, generator=g) + 0.5).to(DEV)   # noqa: E731
    sc, sh, mu, ist = vec(), vec() - 1.0, vec() - 1.0, vec()
    res = []
    for lds in (0, 1):
        o = torch.zeros(N, H, W, cout, dtype=dt, device=DEV)
        dg, db = torch.zeros(cout, device=DEV), torch.zeros(cout, device=DEV)
        ops.set_option("tap64_bnr_lds", lds)
        ops.set_option("fwd_tap64", cfg)
        ops.set_option("fwd_halo", 0)
        try:
            ops.conv_fwd(x, W_, cout, out=o, bn_reduce=(z, sc, sh, mu, ist, dg, db))
            kname = _lib.lib().adp_last_kernel().decode()
            torch.cuda.synchronize()
        finally:
            for k in ("tap64_bnr_lds", "fwd_tap64", "fwd_halo"):
                ops.set_option(k, None)
        assert kname.startswith("igemm_fwd_tap64_kernel<") and ", true, true," in kname, kname
        res.append((o, dg, db))
    (o0, g0, b0), (o1, g1, b1) = res
    assert torch.equal(o0, o1)
    assert torch.equal(g0, g1) and torch.equal(b0, b1), (relerr(g1, g0), relerr(b1, b0))
    assert g0.abs().sum().item() > 0


@pytest.mark.parametrize("dt,N,H,W,cin,cout,mask,add,stats", [
    ("bf16", 2, 32, 32, 192, 192, True, True, False), ("bf16", 1, 24, 40, 128, 96, True, False, True),
    ("bf16", 2, 16, 32, 256, 256, False, True, False), ("f32", 2, 32, 32, 64, 64, True, False, False),
    ("f32", 1, 24, 40, 96, 96, True, True, True)])
def test_tap64_mask_lds_epilogue(dt, N, H, W, cin, cout, mask, add, stats):
    """The tap64 kernel's LDS-staged mask / addend epilogue (option tap64_mask_lds: the rows come in by LDS-DMA) against
    the row-serial epilogue, bf16 and f32: the stored output bit for bit and the same BatchNorm sums; ragged pixel
    counts and N tiles wider than Nout."""
    from adipose_amd import _lib
    tdt = torch.bfloat16 if dt == "bf16" else torch.float32
    g = torch.Generator().manual_seed(73)
    x = torch.randn(N, H, W, cin, generator=g).to(DEV, tdt)
    W_ = (torch.randn(ops.round_up(cout, 64), ops.round_up(9 * cin, 32), generator=g) * 0.03).to(DEV, tdt)
    mk = (torch.rand(N, H, W, cout, generator=g) > 0.4).to(DEV, tdt) if mask else None
    ad = torch.randn(N, H, W, cout, generator=g).to(DEV, tdt) if add else None
    res = []
    for lds in (0, 1):
        o = torch.zeros(N, H, W, cout, dtype=tdt, device=DEV)
        st = torch.zeros(2, cout, device=DEV)
        ops.set_option("tap64_mask_lds", lds)
        ops.set_option("fwd_halo", 0)
        ops.set_option("tap64_persist", 0)
        try:
            ops.conv_fwd(x, W_, cout, out=o, mask=mk, mask_scale=2.0, addend=ad,
                         bn_stats=(st[0], st[1]) if stats else None)
            kname = _lib.lib().adp_last_kernel().decode()
            torch.cuda.synchronize()
        finally:
            for k in ("tap64_mask_lds", "fwd_halo", "tap64_persist"):
                ops.set_option(k, None)
        assert kname.startswith("igemm_fwd_tap64_kernel<"), kname
        res.append((o, st))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])


ZTAIL_CASES = [
    # name, real channels of the sources (stride 64 each), Nout (stride), real Nout, up, epilogue, expected ZT
    ("1src_both", [44], 64, 44, False, "relu_stats", 3),
    ("2src_both_mask_add", [44, 44], 64, 44, False, "mask_add", 3),
    ("1src_ntail", [64], 64, 44, False, "relu_stats", 2),
    ("1src_ktail", [44], 64, 64, False, "relu_stats", 1),
    ("1src_up2_both", [44], 64, 44, True, "relu_stats", 3),
    ("1src_n40_k8", [8], 64, 40, False, "relu_stats", 3),
    ("1src_ktail_n128", [44], 128, 0, False, "relu_stats", 1),       # (256x128 tile: the K tail only)
    ("2src_ktail_n128_mask", [44, 40], 128, 0, False, "mask_add", 1),
]


@pytest.mark.parametrize("case", ZTAIL_CASES, ids=[c[0] for c in ZTAIL_CASES])
def test_f32_zero_tail_forms(case):
    """f32 tap kernel, zero-tail forms (KP 4-6; adp_conv_desc CA_real / CB_real / Nout_real, ABI v19): sources of
    64-channel stride with <= 48 real channels skip the upper 16 channels of every odd K step, Nout 64 with <= 48 real
    columns the MFMA group 48-63 -- the skipped weights are the pad zeros of every packed layer. Output and BatchNorm
    sums bit-identical to the launch without the hints (ragged pixel count, bias, ReLU, mask, addend, upsample)."""
    from adipose_amd import _lib
    name, reals, nout, nreal, up, epi, zt = case
    g = torch.Generator().manual_seed(97)
    N, H, W = 2, 24, 40
    Hs, Ws = (H // 2, W // 2) if up else (H, W)
    xs = []
    for r in reals:
        x = torch.zeros(N, Hs, Ws, 64)
        x[..., :r] = torch.randn(N, Hs, Ws, r, generator=g)
        xs.append(x.to(DEV))
    cin_s = 64 * len(reals)
    nr = nreal or nout
    Wt = torch.zeros(nout, ops.round_up(9 * cin_s, 32))
    for t in range(9):
        for p, r in enumerate(reals):
            Wt[:nr, t * cin_s + 64 * p: t * cin_s + 64 * p + r] = torch.randn(nr, r, generator=g) * 0.05
    Wt = Wt.to(DEV)
    bias = torch.zeros(nout)
    bias[:nr] = torch.randn(nr, generator=g) * 0.1
    bias = bias.to(DEV)
    mk = (torch.rand(N, H, W, nout, generator=g) > 0.4).float().to(DEV) if epi == "mask_add" else None
    ad = torch.randn(N, H, W, nout, generator=g).to(DEV) if epi == "mask_add" else None
    res = []
    for hint in (False, True):
        o = torch.zeros(N, H, W, nout, device=DEV)
        st = torch.zeros(2, nout, device=DEV)
        ops.set_option("fwd_halo", 0)
        ops.set_option("tap64_persist", 0)
        ops.set_option("tap64p_f32", 0)
        ops.set_option("fwd_tap64", 3 if nout == 128 else 1)   # (Nout 128: the 256x128 tile, not two 64-wide ones)
        try:
            real = (reals[0], reals[1] if len(reals) > 1 else 0, nreal) if hint else None
            if epi == "mask_add":
                ops.conv_fwd(xs[0], Wt, nout, out=o, srcB=xs[1] if len(xs) > 1 else None, up=up, mask=mk,
                             mask_scale=2.0, addend=ad, real=real)
            else:
                ops.conv_fwd(xs[0], Wt, nout, out=o, srcB=xs[1] if len(xs) > 1 else None, up=up, bias=bias,
                             relu=True, bn_stats=(st[0], st[1]), real=real)
            kname = _lib.lib().adp_last_kernel().decode()
            torch.cuda.synchronize()
        finally:
            for k in ("fwd_halo", "tap64_persist", "tap64p_f32", "fwd_tap64"):
                ops.set_option(k, None)
        assert kname.startswith(f"igemm_fwd_tap64_kernel<4, {nout // 64}, 64,"), kname
        assert kname.endswith(f", {zt + 3}>" if hint else ", -1>"), kname
        res.append((o, st))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])
    if epi != "mask_add" and nr < nout:   # (the zero weight rows: zero pad channels; an addend's pad channels pass through)
        assert res[1][0][..., nr:].abs().max().item() == 0


@pytest.mark.parametrize("reals,nout,nreal", [([44], 64, 44), ([44, 44], 64, 44), ([40], 64, 64), ([12], 64, 20),
                                               ([44], 128, 100), ([44], 128, 88), ([64, 44], 192, 136),
                                               ([64, 44], 64, 40)],
                         ids=["1src_44", "2src_44_44", "1src_40_n64", "1src_12_n20", "1src_44_n128_100",
                              "1src_44_n128_88_row_tail", "2src_64_44_n192_136_12_combos", "2src_64_44_n40_tap_split"])
def test_f32_halo_wgrad_zero_tails(reals, nout, nreal):
    """f32 halo weight gradient with the real-channel hints (option wgrad_f32_zt): an input chunk with <= 16 real
    channels runs its useful 16 x 16 blocks one per wave on fewer waves and gets fewer blocks; and the bias gradient
    summed in the same pass (option wgrad_f32_bias: per-block rows + the fixed-order slab reduce) instead of the
    channel-sum launch. Round 6: row tails (an output block with <= 2 real 16-row blocks on 2 rb waves), tables of
    up to 40 combinations (12 here) with greedily balanced block counts, and the T3 tap split of a 3-row-block output
    block (44 and 40 real outputs: waves 4-7 share row block 2 by taps).
    The weight gradient equals the unhinted launch's to the f32 atomics' order, the pad rows and
    columns stay exactly zero, both match a float64 reference; the bias gradient to 1e-6 of the channel sum's."""
    from adipose_amd._lib import lib
    g = torch.Generator().manual_seed(101)
    N, S = 2, 64
    xs = []
    for r in reals:
        x = torch.zeros(N, S, S, 64)
        x[..., :r] = torch.randn(N, S, S, r, generator=g)
        xs.append(x.to(DEV))
    dy = torch.zeros(N, S, S, nout)
    dy[..., :nreal] = torch.randn(N, S, S, nreal, generator=g)
    dy = dy.to(DEV)
    cin_s = 64 * len(reals)
    res = []
    for hint in (False, True):
        dW = torch.zeros(nout, ops.round_up(9 * cin_s, 32), device=DEV)
        dB = torch.zeros(nout, device=DEV)
        ops.set_option("wgrad_f32_bias", 1 if hint else 0)
        try:
            ops.conv_wgrad(xs[0], dy, dW, nout, dB=dB, srcB=xs[1] if len(xs) > 1 else None,
                           real=(reals[0], reals[1] if len(reals) > 1 else 0, nreal) if hint else None)
            torch.cuda.synchronize()
            kname = lib().adp_last_kernel().decode()
        finally:
            ops.set_option("wgrad_f32_bias", None)
        assert kname.startswith("igemm_wgrad_halo_f32_kernel<"), kname
        res.append((dW.cpu(), dB.cpu()))
    # float64 reference: dW[n][t * cin_s + c] = sum_pixels dY[p][n] * X[p + off_t][c]
    x = torch.cat(xs, -1).cpu().double().permute(0, 3, 1, 2)
    xp = F.pad(x, (1, 1, 1, 1))
    d64 = dy.cpu().double().reshape(-1, nout)
    ref = torch.zeros(nout, 9 * cin_s, dtype=torch.float64)
    for t in range(9):
        ty, tx = t // 3, t % 3
        patch = xp[:, :, ty:ty + S, tx:tx + S].permute(0, 2, 3, 1).reshape(-1, cin_s)
        ref[:, t * cin_s:(t + 1) * cin_s] = d64.T @ patch
    for w_, b_ in res:
        assert relerr(w_[:, :9 * cin_s], ref) < 1e-5
        assert relerr(b_, d64.sum(0)) < 1e-5
    assert relerr(res[1][0], res[0][0]) < 1e-6
    assert relerr(res[1][1], res[0][1]) < 1e-6
    if nreal < nout:
        assert res[1][0][nreal:].abs().max().item() == 0 and res[1][1][nreal:].abs().max().item() == 0
    pad_cols = [t * cin_s + 64 * p + c for t in range(9) for p, r in enumerate(reals) for c in range(r, 64)]
    assert res[1][0][:, pad_cols].abs().max().item() == 0


HALOP_WIDE_CASES = [
    # name, source channels, Nout, epilogue, split, up
    ("1ch_stats", [64], 64, "stats", False, 1),
    ("1ch_relu_stats", [64], 64, "relu_stats", False, 1),
    ("1ch_plain_n48", [64], 48, "plain", False, 1),
    ("1ch_split128", [64], 128, "relu", True, 1),
    ("1ch_up2_stats", [64], 64, "stats", False, 2),
    ("2ch_stats", [64, 64], 128, "stats", False, 1),
    ("2ch_relu_n64", [128], 64, "relu", False, 1),
    ("2ch_split", [128], 128, "plain", True, 1),
    ("1ch_mask", [64], 64, "mask", False, 1),
    ("2ch_mask_split", [128], 128, "mask", True, 1),
    ("1ch_dropout", [64], 64, "dropout", False, 1),
]


@pytest.mark.parametrize("grid", [None, 3], ids=["chip_grid", "3_blocks"])
@pytest.mark.parametrize("case", HALOP_WIDE_CASES, ids=[c[0] for c in HALOP_WIDE_CASES])
def test_halop_wide_store_matches(case, grid):
    """Persistent halo kernel with 16-B epilogue stores (halop_wide=2: channel quads of two 16-channel groups
    joined by permlane16_swap; by default the tile-serial forms only) vs the 8-B quad stores (halop_wide=0): the same values in
    every channel of the outputs (plain, split, ragged N = 48 against a 64-wide block), and BatchNorm sums
    to f32 order, for every epilogue form (statistics, ReLU, ReLU-backward mask + addend, dropout), the
    pipelined one-chunk and the two-chunk forms, an upsampled source; a 3-block grid walks many tiles."""
    name, parts, nout, epi, split, up = case
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(61)
    N, S = 2, 32
    xs = [torch.randn(N, S // up, S // up, c, generator=g).to(DEV, dt) for c in parts]
    cin = sum(parts)
    W = (torch.randn(((nout + 63) // 64) * 64, 9 * cin, generator=g) * 0.03).to(DEV, dt)
    bias = torch.randn(nout, generator=g).to(DEV)
    mk = torch.randn(N, S, S, nout, generator=g).to(DEV, dt)
    ad = torch.randn(N, S, S, nout, generator=g).to(DEV, dt)
    res = []
    for wide in (1, 0):
        ops.set_option("halop_wide", 2 * wide)   # 2: every (non-BNR) form, the pipelined ones included
        if grid:
            ops.set_option("halo_persist_grid", grid)
        try:
            st = torch.zeros(2, nout, device=DEV)
            kw = dict(srcB=xs[1] if len(xs) > 1 else None, up=up == 2)
            if epi in ("stats", "relu", "relu_stats", "plain", "dropout"):
                kw.update(bias=bias, relu=epi in ("relu", "relu_stats", "dropout"))
            if epi in ("stats", "relu_stats"):
                kw.update(bn_stats=(st[0], st[1]))
            if epi == "dropout":
                kw.update(dropout_rate=0.3, dropout_seed=77)
            if split:
                o1 = torch.full((N, S, S, 64), 7.0, dtype=dt, device=DEV)
                o2 = torch.full((N, S, S, nout - 64 + 8), 7.0, dtype=dt, device=DEV)   # wider stride than stored
                if epi == "mask":
                    kw.update(mask=mk[..., :64].contiguous(), mask_scale=1.5, mask2=mk[..., 64:].contiguous(),
                              mask2_scale=0.5)
                ops.conv_fwd(xs[0], W, nout, out=o1, out_mode=2, out2=o2, split_c=64, **kw)
                outs = [o1, o2]
            else:
                o = torch.full((N, S, S, 64 if nout < 64 else nout), 7.0, dtype=dt, device=DEV)
                if epi == "mask":
                    kw.update(mask=mk, mask_scale=1.5, addend=ad)
                ops.conv_fwd(xs[0], W, nout, out=o, **kw)
                outs = [o]
            torch.cuda.synchronize()
            kname = _lib.lib().adp_last_kernel().decode()
        finally:
            ops.set_option("halop_wide", None)
            ops.set_option("halo_persist_grid", None)
        # igemm_fwd_halop_kernel<BNR, NCH, BN, PIPE, EPI, WIDE, DYN>
        assert kname.startswith("igemm_fwd_halop_kernel") and kname.split(", ")[5] == ("true" if wide else "false"), kname
        res.append(([t.clone() for t in outs], st.clone()))
    for a_, b_ in zip(res[0][0], res[1][0]):
        assert torch.equal(a_, b_), (a_.double() - b_.double()).abs().max().item()
    if nout < 64:   # the pad channels of the 64-stride output: untouched by either form
        assert (res[0][0][0][..., nout:] == 7.0).all()
    torch.testing.assert_close(res[0][1], res[1][1], rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("parts,cout", [([128], 64), ([64, 64], 64), ([128], 128), ([64, 64], 128)])
@pytest.mark.parametrize("S,N", [(32, 2), (64, 1)])
def test_persistent_halo_two_chunks(parts, cout, S, N):
    """Persistent halo kernel with two 64-channel input chunks (one or two sources) in 32-wide output
    blocks: output + BatchNorm statistics vs the oracle and vs the one-tile halo kernel
    (halo_persist2=0); split store for 128 outputs; data gradient with the fused BN-backward reduction."""
    from adipose_amd import _lib
    dt = torch.bfloat16
    xs, kern, bias, l = make_case(N, S, parts, cout, 1, False, seed=41)
    W = torch.from_numpy(l.keras_to_packed(kern.numpy())).to(DEV).to(dt).contiguous()
    xd = [x.to(DEV, dt).contiguous() for x in xs]
    srcB = xd[1] if len(xd) > 1 else None
    out = torch.zeros((N, S, S, cout), dtype=dt, device=DEV)
    st = torch.zeros(2, cout, device=DEV)
    ops.conv_fwd(xd[0], W, cout, out=out, srcB=srcB, bias=bias.to(DEV), relu=True, bn_stats=(st[0], st[1]))
    assert _lib.lib().adp_last_kernel().decode().startswith("igemm_fwd_halop_kernel<false, 2, 32")
    ref = oracle_fwd([rb(x, dt) for x in xs], rb(kern, dt), bias, 1, False)
    assert relerr(out, ref) < TOL[dt]
    r2 = ref.reshape(-1, cout)
    assert relerr(st[0], r2.sum(0)) < 2e-2 and relerr(st[1], (r2 * r2).sum(0)) < 2e-2
    old = torch.zeros_like(out)
    ops.set_option("halo_persist2", 0)
    try:
        ops.conv_fwd(xd[0], W, cout, out=old, srcB=srcB, bias=bias.to(DEV), relu=True)
        assert "halop" not in _lib.lib().adp_last_kernel().decode()
    finally:
        ops.set_option("halo_persist2", None)
    torch.cuda.synchronize()
    assert (out.float() - old.float()).abs().max().item() <= 2 ** -6 * out.float().abs().max().item()
    if cout == 128:
        o1 = torch.zeros((N, S, S, 64), dtype=dt, device=DEV)
        o2 = torch.zeros((N, S, S, 72), dtype=dt, device=DEV)
        ops.conv_fwd(xd[0], W, 128, out=o1, srcB=srcB, bias=bias.to(DEV), relu=True, out_mode=2, out2=o2,
                     split_c=64)
        assert _lib.lib().adp_last_kernel().decode().startswith("igemm_fwd_halop_kernel")
        torch.cuda.synchronize()
        assert torch.equal(o1, out[..., :64]) and torch.equal(o2[..., :64], out[..., 64:])
    if len(parts) == 1:
        # data gradient of a 64 -> 128 conv: dY has 128 channels (two chunks), dX 64 / 128 channels
        g = torch.Generator().manual_seed(42)
        dZ = torch.randn(N, S, S, 128, generator=g).to(DEV, dt)
        Wd = (torch.randn(cout, 9 * 128, generator=g) * 0.03).to(DEV, dt)
        z = torch.randn(N, S, S, cout, generator=g).to(DEV, dt)
        sc, sh = (torch.rand(cout, generator=g) + 0.5).to(DEV), (torch.randn(cout, generator=g) * 0.2).to(DEV)
        mu, ist = (torch.randn(cout, generator=g) * 0.1).to(DEV), (torch.rand(cout, generator=g) + 0.5).to(DEV)
        dA = torch.zeros((N, S, S, cout), dtype=dt, device=DEV)
        dg, db = torch.zeros(cout, device=DEV), torch.zeros(cout, device=DEV)
        ops.conv_fwd(dZ, Wd, cout, out=dA, bn_reduce=(z, sc, sh, mu, ist, dg, db))
        assert _lib.lib().adp_last_kernel().decode().startswith("igemm_fwd_halop_kernel<true, 2, 32")
        dg2, db2 = torch.zeros_like(dg), torch.zeros_like(db)
        ops.bn_bwd_reduce(dA, z, sc, sh, mu, ist, dg2, db2)
        ref = torch.zeros_like(dA)
        ops.set_option("halo_persist2", 0)
        try:
            ops.conv_fwd(dZ, Wd, cout, out=ref)
        finally:
            ops.set_option("halo_persist2", None)
        torch.cuda.synchronize()
        assert relerr(db, db2) < 1e-4 and relerr(dg, dg2) < 1e-4
        assert relerr(dA, ref) < 1e-2


@pytest.mark.parametrize("cfg", [2, 3, 4], ids=["256x256", "128x256", "64x256"])
@pytest.mark.parametrize("cout", [64, 192])
@pytest.mark.parametrize("S", [23, 64], ids=["ragged", "rowaligned"])
def test_wgrad_tap64_configs(cfg, cout, S):
    """Each forced tile configuration of the tap64 weight-gradient kernel vs autograd of the oracle
    conv: a ragged pixel count (S = 23: M = 1058, general gather path) and row-aligned images
    (S = 64: Wo % 64 == 0, the scalar stage-origin gather path)."""
    N, cin = 2, 128
    xs, kern, bias, l = make_case(N, S, [cin], cout, 1, False, seed=11)
    dt = torch.bfloat16
    x = rb(xs[0], dt)
    g = torch.Generator().manual_seed(12)
    dZ = rb(torch.randn(N, S, S, cout, generator=g), dt)
    kr = rb(kern, dt).clone().requires_grad_(True)
    (R.conv2d_same(x, kr, None, relu=False) * dZ).sum().backward()
    dW = torch.zeros((l.Npad, l.Kpad), device=DEV)
    ops.set_option("wgrad_tap64", cfg)
    try:
        ops.conv_wgrad(nhwc_pad(x, l.Cin_s, dt), nhwc_pad(dZ, l.cout_s, dt), dW, l.Nout)
        torch.cuda.synchronize()
    finally:
        ops.set_option("wgrad_tap64", 1)
    assert relerr(torch.from_numpy(l.packed_to_keras(dW.cpu().numpy())), kr.grad) < 2e-2


WF32_CASES = [
    # name, N, H, W, CA, CB, Nout, k, dil, up, shuffle_c (ConvT 1x1 with pixel-shuffled dY)
    ("plain_n96", 2, 24, 40, 64, 0, 96, 3, 1, False, 0),
    ("concat_n64", 1, 20, 36, 32, 64, 64, 3, 1, False, 0),
    ("dil4_n48", 2, 16, 16, 96, 0, 48, 3, 4, False, 0),
    ("up2_n128", 2, 12, 20, 64, 0, 128, 3, 1, True, 0),
    ("wide_n256", 1, 16, 32, 128, 0, 256, 3, 1, False, 0),
    ("ragged_n40", 1, 13, 23, 32, 0, 40, 3, 1, False, 0),
    ("convt_c32", 2, 8, 16, 64, 0, 128, 1, 1, False, 32),
]


@pytest.mark.parametrize("case", WF32_CASES, ids=[c[0] for c in WF32_CASES])
def test_wgrad_f32_lds_kernel(case):
    """f32 weight gradient on the LDS-DMA kernel (opt-in, conv_wgrad_f32.hip: 32-pixel stages, exact
    v_mfma_f32_16x16x4_f32, per-split slabs / atomics) vs the register-staged f32 kernel (option
    wgrad_f32=0) on the same operands to 1e-5, and vs a float64 autograd of the convolution; the bias
    gradient (channel-sum launch) to 1e-5. Plain / concat / dilated / upsample-gather / 1-4 N tiles / ragged
    pixel count and N / ConvT pixel-shuffle dY."""
    name, N, H, W_, CA, CB, nout, k, dil, up, shuf = case
    g = torch.Generator().manual_seed(41)
    Hs, Ws = (H // 2, W_ // 2) if up else (H, W_)
    xa = torch.randn(N, Hs, Ws, CA, generator=g)
    xb = torch.randn(N, Hs, Ws, CB, generator=g) if CB else None
    if shuf:
        dY = torch.randn(N, 2 * H, 2 * W_, shuf, generator=g)
    else:   # (channel stride a multiple of 8)
        dY = torch.zeros(N, H, W_, (nout + 7) // 8 * 8)
        dY[..., :nout] = torch.randn(N, H, W_, nout, generator=g)
    kw = dict(srcB=xb.to(DEV) if CB else None, up=up, dil=dil, kh=k, kw=k)
    if shuf:
        kw.update(pad=0, shuffle_c=shuf)
    res = []
    for f32k in (1, 0):
        K = k * k * (CA + CB)
        dW = torch.zeros(nout, (K + 31) // 32 * 32, device=DEV)
        dB = torch.zeros(shuf if shuf else nout, device=DEV)
        ops.set_option("wgrad_f32", f32k)
        ops.set_option("wgrad_f32_halo", 0)   # (the persistent halo form has its own test)
        try:
            ops.conv_wgrad(xa.to(DEV), dY.to(DEV), dW, nout, dB=dB, **kw)
            torch.cuda.synchronize()
            kname = _lib.lib().adp_last_kernel().decode()
        finally:
            ops.set_option("wgrad_f32", None)
            ops.set_option("wgrad_f32_halo", None)
        assert kname.startswith("igemm_wgrad_f32_kernel") == bool(f32k), kname
        res.append((dW.cpu().double(), dB.cpu().double()))
    (w1, b1), (w0, b0) = res
    assert relerr(w1, w0) < 1e-5, relerr(w1, w0)
    assert relerr(b1, b0) < 1e-5
    if not shuf:   # float64 autograd: dW[n][tap * Cin + c]
        x = torch.cat([xa, xb], -1) if CB else xa
        x = x.double().permute(0, 3, 1, 2)
        if up:
            x = x.repeat_interleave(2, 2).repeat_interleave(2, 3)
        wt = torch.zeros(nout, CA + CB, k, k, dtype=torch.float64, requires_grad=True)
        y = F.conv2d(x, wt, padding=dil * (k // 2), dilation=dil)
        (y * dY[..., :nout].double().permute(0, 3, 1, 2)).sum().backward()
        ref = wt.grad.permute(0, 2, 3, 1).reshape(nout, -1)
        assert relerr(w1[:, :ref.shape[1]], ref) < 1e-5, relerr(w1[:, :ref.shape[1]], ref)


@pytest.mark.parametrize("N,H,W,cin", [(2, 32, 64, 3), (1, 16, 96, 1), (3, 8, 32, 8)])
def test_wgrad_input_layer_cin8(N, H, W, cin):
    """Input-layer weight gradient (one 8-channel source, 64 outputs): the persistent cin8 kernel vs
    autograd of the oracle conv and vs the generic LDS-DMA kernel (option wgrad_cin8=0)."""
    from adipose_amd import _lib
    cout = 64
    _, kern, bias, l = make_case(N, H, [cin], cout, 1, False, seed=51)
    assert l.Cin_s == 8
    g = torch.Generator().manual_seed(52)
    dt = torch.bfloat16
    x = rb(torch.randn(N, H, W, cin, generator=g), dt)
    dZ = rb(torch.randn(N, H, W, cout, generator=g), dt)
    kr = rb(kern, dt).clone().requires_grad_(True)
    (R.conv2d_same(x, kr, None, relu=False) * dZ).sum().backward()
    xd, dzd = nhwc_pad(x, l.Cin_s, dt), nhwc_pad(dZ, l.cout_s, dt)
    dW = torch.zeros((l.Npad, l.Kpad), device=DEV)
    ops.conv_wgrad(xd, dzd, dW, l.Nout)
    assert _lib.lib().adp_last_kernel().decode().startswith("igemm_wgrad_cin8_kernel")
    ref = torch.zeros_like(dW)
    ops.set_option("wgrad_cin8", 0)
    try:
        ops.conv_wgrad(xd, dzd, ref, l.Nout)
        torch.cuda.synchronize()
    finally:
        ops.set_option("wgrad_cin8", None)
    assert relerr(torch.from_numpy(l.packed_to_keras(dW.cpu().numpy())), kr.grad) < 2e-2
    assert relerr(dW.cpu(), ref.cpu()) < 1e-4
    assert dW[:, 72:].abs().max().item() == 0.0


@pytest.mark.parametrize("N,H,W,parts,cout,dtn,fused", [
    (2, 64, 64, [64], 64, "bf16", True), (1, 32, 96, [64], 64, "bf16", True),
    (2, 32, 64, [64, 64], 64, "bf16", True), (1, 32, 32, [128], 128, "bf16", True),
    (1, 16, 64, [64], 128, "bf16", True), (2, 16, 64, [128, 64], 128, "bf16", False),
    (1, 16, 32, [64], 64, "f32", False)])
@pytest.mark.parametrize("maxch", [None, 2], ids=["default", "maxch2"])
def test_wgrad_bn_apply_fused(N, H, W, parts, cout, dtn, fused, maxch):
    """adp_conv_wgrad_bn (BatchNorm-backward apply computed inside the halo weight-gradient kernel, dz
    stored for the data gradient) == adp_bn_bwd_apply + adp_conv_wgrad: dz bit for bit, dW to f32
    summation order; shapes the fused kernel does not take run the two launches. By default only
    single-chunk layers take the fused kernel (wgrad_bna_maxch=1, step A/B in profiles/r03_bna_maxch_ab.txt);
    option wgrad_bna_maxch=2 keeps the two-chunk form reachable."""
    from adipose_amd import _lib
    dt = torch.bfloat16 if dtn == "bf16" else torch.float32
    g = torch.Generator().manual_seed(31)
    xs = [(torch.randn(N, H, W, c, generator=g)).to(DEV, dt) for c in parts]
    z = (torch.randn(N, H, W, cout, generator=g) * 2).to(DEV, dt)
    dA = torch.randn(N, H, W, cout, generator=g).to(DEV, dt)
    vec = lambda: (torch.rand(cout, generator=g) + 0.5).to(DEV)   # noqa: E731
    sc, sh, mu, ist, gam = vec(), vec() - 1.0, vec() - 1.0, vec(), vec()
    dg, db = torch.randn(cout, generator=g).to(DEV), torch.randn(cout, generator=g).to(DEV)
    count = N * H * W
    K = 9 * sum(parts)
    srcB = xs[1] if len(xs) > 1 else None
    dz1, dz2 = torch.full_like(z, 7.0), torch.full_like(z, 7.0)
    dW1 = torch.zeros((cout, K), device=DEV)
    dW2 = torch.zeros_like(dW1)
    ops.bn_bwd_apply(dA, z, sc, sh, mu, ist, gam, dg, db, count, dz1)
    ops.conv_wgrad(xs[0], dz1, dW1, cout, srcB=srcB)
    ops.set_option("wgrad_bna_maxch", maxch)
    try:
        ops.conv_wgrad(xs[0], dz2, dW2, cout, srcB=srcB, bn_apply=(dA, z, sc, sh, mu, ist, gam, dg, db, count))
        kname = _lib.lib().adp_last_kernel().decode()
        torch.cuda.synchronize()
    finally:
        ops.set_option("wgrad_bna_maxch", None)
    fused = fused and (maxch == 2 or sum(parts) == 64)
    assert kname.startswith("igemm_wgrad_halop_kernel<8, true") == fused, kname
    assert torch.equal(dz1, dz2)
    assert relerr(dW2.cpu(), dW1.cpu()) < 1e-5


@pytest.mark.parametrize("N,H,W,grid", [(2, 64, 64, None), (1, 32, 96, None), (3, 16, 32, 5), (2, 64, 64, 7)])
@pytest.mark.parametrize("opt", [None, "wgrad_cin8_bna", "wgrad_bna"])
def test_wgrad_bn_apply_input_layer_no_dz(N, H, W, grid, opt):
    """adp_conv_wgrad_bn with dY = NULL (nothing reads dz): on the input layer (one 8-channel source, 64
    outputs) the persistent input-layer kernel computes dz = bn_bwd_apply(dA, z) from dA (LDS-DMA) and z
    (registers) in its stage images and stores none; dW equals adp_bn_bwd_apply + adp_conv_wgrad to f32
    summation order. Options wgrad_cin8_bna=0 / wgrad_bna=0 take the two-launch form through library scratch;
    small grids (5 / 7 blocks) walk many patches per block, an odd count exercising the unrolled tail."""
    from adipose_amd import _lib
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(37)
    cout = 64
    x = torch.randn(N, H, W, 8, generator=g).to(DEV, dt)
    z = (torch.randn(N, H, W, cout, generator=g) * 2).to(DEV, dt)
    dA = torch.randn(N, H, W, cout, generator=g).to(DEV, dt)
    vec = lambda: (torch.rand(cout, generator=g) + 0.5).to(DEV)   # noqa: E731
    sc, sh, mu, ist, gam = vec(), vec() - 1.0, vec() - 1.0, vec(), vec()
    dg, db = torch.randn(cout, generator=g).to(DEV), torch.randn(cout, generator=g).to(DEV)
    count = N * H * W
    dz1 = torch.full_like(z, 7.0)
    dW1 = torch.zeros((cout, 96), device=DEV)   # Kpad = 72 rounded to 32
    dW2 = torch.zeros_like(dW1)
    ops.bn_bwd_apply(dA, z, sc, sh, mu, ist, gam, dg, db, count, dz1)
    ops.conv_wgrad(x, dz1, dW1, cout)
    assert _lib.lib().adp_last_kernel().decode() == "igemm_wgrad_cin8_kernel<false>"
    if opt:
        ops.set_option(opt, 0)
    if grid:
        ops.set_option("wgrad_cin8_grid", grid)
    try:
        ops.conv_wgrad(x, None, dW2, cout, bn_apply=(dA, z, sc, sh, mu, ist, gam, dg, db, count))
        kname = _lib.lib().adp_last_kernel().decode()
        torch.cuda.synchronize()
    finally:
        for o_ in (opt, "wgrad_cin8_grid"):
            if o_:
                ops.set_option(o_, None)
    assert kname == "igemm_wgrad_cin8_kernel<%s>" % ("false" if opt else "true"), kname
    assert relerr(dW2.cpu(), dW1.cpu()) < 1e-5
    if grid is None and opt is None:   # a halo-kernel layer with dY = NULL: fused, dz not stored
        xs = torch.randn(N, H, W, 64, generator=g).to(DEV, dt)
        dW3 = torch.zeros((cout, 9 * 64), device=DEV)
        dW4 = torch.zeros_like(dW3)
        ops.conv_wgrad(xs, dz1, dW3, cout)
        ops.conv_wgrad(xs, None, dW4, cout, bn_apply=(dA, z, sc, sh, mu, ist, gam, dg, db, count))
        assert _lib.lib().adp_last_kernel().decode().startswith("igemm_wgrad_halop_kernel<8, true")
        torch.cuda.synchronize()
        assert relerr(dW4.cpu(), dW3.cpu()) < 1e-5


@pytest.mark.parametrize("opt", ["wgrad_tap64", "wgrad_halop", "wgrad_bna"])
def test_wgrad_bn_apply_with_kernel_options_off(opt):
    """adp_conv_wgrad_bn with the halo weight-gradient kernel switched off (wgrad_tap64 = 0 is a documented
    'off' value): the library must run the BatchNorm-backward apply itself before the fallback kernel, so dz
    and dW equal the two-launch form (the fused form used to fall through to a kernel reading an
    uncomputed dY)."""
    N, H, W, cout = 2, 32, 64, 64
    g = torch.Generator().manual_seed(41)
    x = torch.randn(N, H, W, 64, generator=g).to(DEV, torch.bfloat16)
    z = (torch.randn(N, H, W, cout, generator=g) * 2).to(DEV, torch.bfloat16)
    dA = torch.randn(N, H, W, cout, generator=g).to(DEV, torch.bfloat16)
    vec = lambda: (torch.rand(cout, generator=g) + 0.5).to(DEV)   # noqa: E731
    sc, sh, mu, ist, gam = vec(), vec() - 1.0, vec() - 1.0, vec(), vec()
    dg, db = torch.randn(cout, generator=g).to(DEV), torch.randn(cout, generator=g).to(DEV)
    count = N * H * W
    dz1, dz2 = torch.full_like(z, 7.0), torch.full_like(z, 7.0)
    dW1 = torch.zeros((cout, 9 * 64), device=DEV)
    dW2 = torch.zeros_like(dW1)
    ops.bn_bwd_apply(dA, z, sc, sh, mu, ist, gam, dg, db, count, dz1)
    ops.conv_wgrad(x, dz1, dW1, cout)
    ops.set_option(opt, 0)
    try:
        ops.conv_wgrad(x, dz2, dW2, cout, bn_apply=(dA, z, sc, sh, mu, ist, gam, dg, db, count))
        torch.cuda.synchronize()
    finally:
        ops.set_option(opt, None)
    assert torch.equal(dz1, dz2)
    assert relerr(dW2.cpu(), dW1.cpu()) < 1e-5


@pytest.mark.parametrize("N,H,W,parts,cout", [(2, 64, 64, [64], 64), (1, 32, 96, [64], 64), (3, 16, 32, [64], 64),
                                               (2, 32, 64, [64, 64], 64), (1, 32, 32, [128], 128),
                                               (2, 16, 64, [128, 64], 128)])
def test_wgrad_persistent_halo(N, H, W, parts, cout):
    """Persistent halo weight-gradient kernel (3x3, 64-channel input chunks from one or two sources,
    64-wide output blocks) vs autograd of the oracle conv, and vs the tap64 / glds kernels on the same
    operands (option wgrad_halop=0)."""
    from adipose_amd import _lib
    cin = sum(parts)
    _, kern, bias, l = make_case(N, H, parts, cout, 1, False, seed=21)
    g = torch.Generator().manual_seed(22)
    dt = torch.bfloat16
    xs = [rb(torch.randn(N, H, W, c, generator=g), dt) for c in parts]
    dZ = rb(torch.randn(N, H, W, cout, generator=g), dt)
    kr = rb(kern, dt).clone().requires_grad_(True)
    (R.conv2d_same(torch.cat(xs, -1), kr, None, relu=False) * dZ).sum().backward()
    xd = [x.to(DEV, dt).contiguous() for x in xs]
    dzd = nhwc_pad(dZ, l.cout_s, dt)
    srcB = xd[1] if len(xd) > 1 else None
    dW = torch.zeros((l.Npad, l.Kpad), device=DEV)
    try:
        ops.conv_wgrad(xd[0], dzd, dW, l.Nout, srcB=srcB)
        # default: the tap-pair form (round 6)
        assert _lib.lib().adp_last_kernel().decode() == "igemm_wgrad_halopair_kernel<6, 0>"
        torch.cuda.synchronize()
        dW2 = torch.zeros_like(dW)   # fixed-order slab reduce (option wgrad_det): a second run gives the same bits
        ops.conv_wgrad(xd[0], dzd, dW2, l.Nout, srcB=srcB)
        torch.cuda.synchronize()
        assert torch.equal(dW, dW2)
        ops.set_option("wgrad_halop_pair", 0)   # the one-tap-per-wave forms: the row-pipelined one (round 5) ...
        dWpf = torch.zeros_like(dW)
        ops.conv_wgrad(xd[0], dzd, dWpf, l.Nout, srcB=srcB)
        assert _lib.lib().adp_last_kernel().decode() == "igemm_wgrad_halop_kernel<8, false, 4, false, true>"
        ops.set_option("wgrad_halop_pf", 0)   # ... and the unpipelined row loop: the same per-block sums
        dWn = torch.zeros_like(dW)
        ops.conv_wgrad(xd[0], dzd, dWn, l.Nout, srcB=srcB)
        assert _lib.lib().adp_last_kernel().decode() == "igemm_wgrad_halop_kernel<8, false, 4, false, false>"
        ops.set_option("wgrad_halop_pf", None)
        ops.set_option("wgrad_halop_spread", 8)   # next patch's loads over all 8 patch rows
        dWp8 = torch.zeros_like(dW)
        ops.conv_wgrad(xd[0], dzd, dWp8, l.Nout, srcB=srcB)
        assert _lib.lib().adp_last_kernel().decode() == "igemm_wgrad_halop_kernel<8, false, 8, false, true>"
        ops.set_option("wgrad_halop_pf", 0)
        dWs = torch.zeros_like(dW)
        ops.conv_wgrad(xd[0], dzd, dWs, l.Nout, srcB=srcB)
        assert _lib.lib().adp_last_kernel().decode() == "igemm_wgrad_halop_kernel<8, false, 8, true, false>"
        ops.set_option("wgrad_halop_pf", None)
        ops.set_option("wgrad_halop_waves", 9)   # one wave per tap
        dW9 = torch.zeros_like(dW)
        ops.conv_wgrad(xd[0], dzd, dW9, l.Nout, srcB=srcB)
        ref = torch.zeros_like(dW)
        ops.set_option("wgrad_halop", 0)
        ops.conv_wgrad(xd[0], dzd, ref, l.Nout, srcB=srcB)
        torch.cuda.synchronize()
    finally:
        ops.set_option("wgrad_halop", None)
        ops.set_option("wgrad_halop_waves", None)
        ops.set_option("wgrad_halop_spread", None)
        ops.set_option("wgrad_halop_pf", None)
        ops.set_option("wgrad_halop_pair", None)
    assert relerr(torch.from_numpy(l.packed_to_keras(dW.cpu().numpy())), kr.grad) < 2e-2
    assert torch.equal(dWpf, dWn) and torch.equal(dWpf, dWp8)   # (same per-block sums, same fixed-order reduce)
    # the tap-pair form sums the even and the odd patch rows separately, then adds the two: another f32 order
    assert relerr(dW.cpu(), dWpf.cpu()) < 1e-5
    assert relerr(dW.cpu(), ref.cpu()) < 1e-4 and relerr(dW9.cpu(), ref.cpu()) < 1e-4
    assert relerr(dWs.cpu(), ref.cpu()) < 1e-4


def test_wgrad_defer_arena_release():
    """adp_wgrad_release (ABI 20, round-5 ADVICE): deferral arenas are per (device, stream); a stream that deferred holds
    an arena until released, release frees it (and refuses while reductions are pending), a second stream gets its own,
    and a deferral after a release allocates again and still gives the immediate-mode bits."""
    N, H, W, cout = 2, 64, 64, 64
    _, kern, bias, l = make_case(N, H, [64], cout, 1, False, seed=25)
    g = torch.Generator().manual_seed(26)
    x = torch.randn(N, H, W, 64, generator=g).to(DEV, torch.bfloat16)
    dz = nhwc_pad(rb(torch.randn(N, H, W, cout, generator=g), torch.bfloat16), l.cout_s, torch.bfloat16)
    ref = torch.zeros((l.Npad, l.Kpad), device=DEV)
    ops.conv_wgrad(x, dz, ref, l.Nout)
    torch.cuda.synchronize()
    side = torch.cuda.Stream(device=DEV)
    outs = []
    for st in (torch.cuda.current_stream(), side, torch.cuda.current_stream()):
        with torch.cuda.stream(st):
            d = torch.zeros_like(ref)
            ops.wgrad_defer(True)
            ops.conv_wgrad(x, dz, d, l.Nout)
            with pytest.raises(ops.AdpError):
                ops.wgrad_release()   # reductions pending
            ops.wgrad_flush()
            assert ops.wgrad_arena_chunks() >= 1
            outs.append(d)
    torch.cuda.synchronize()
    assert ops.wgrad_arena_chunks(side) >= 1
    ops.wgrad_release(side)
    assert ops.wgrad_arena_chunks(side) == 0
    ops.wgrad_release()
    assert ops.wgrad_arena_chunks() == 0
    for d in outs:
        assert torch.equal(d, ref)


def test_wgrad_deferred_reductions():
    """adp_wgrad_defer / adp_wgrad_flush: between them the slab reductions of the deterministic weight-gradient
    launches are only recorded (dW untouched), the flush runs them all in one batched launch with the arithmetic of
    the per-launch reduce (bit-identical dW), a gradient accumulated twice into one buffer keeps both terms (the
    second segment goes to a table launched after the first), and ending a deferral with reductions pending is an
    error. Covers the halo kernel's slabs, the tap64 kernel's split slabs (wgrad_halop = 0) and bias sums."""
    from adipose_amd import _lib
    N, H, W, cout = 2, 64, 64, 64
    _, kern, bias, l = make_case(N, H, [64], cout, 1, False, seed=23)
    g = torch.Generator().manual_seed(24)
    x = torch.randn(N, H, W, 64, generator=g).to(DEV, torch.bfloat16)
    dz = nhwc_pad(rb(torch.randn(N, H, W, cout, generator=g), torch.bfloat16), l.cout_s, torch.bfloat16)
    z = lambda: torch.zeros((l.Npad, l.Kpad), device=DEV)   # noqa: E731

    def run(dst, opt=None, dB=None):
        if opt:
            ops.set_option(opt, 0)
        try:
            ops.conv_wgrad(x, dz, dst, l.Nout, dB=dB)
        finally:
            if opt:
                ops.set_option(opt, None)
    # immediate: halo slabs, twice into one buffer; tap64 split slabs; bias sums
    ref_h, ref_h2, ref_t = z(), z(), z()
    ref_b = torch.zeros(l.Npad, device=DEV)
    run(ref_h)
    run(ref_h2)
    run(ref_h2)
    run(ref_t, "wgrad_halop", dB=ref_b)
    torch.cuda.synchronize()
    d_h, d_h2, d_t = z(), z(), z()
    d_b = torch.zeros(l.Npad, device=DEV)
    ops.wgrad_defer(True)
    try:
        run(d_h)
        assert _lib.lib().adp_last_kernel().decode() == "igemm_wgrad_halopair_kernel<6, 0>"
        run(d_h2)
        run(d_h2)
        run(d_t, "wgrad_halop", dB=d_b)
        assert _lib.lib().adp_last_kernel().decode().startswith("igemm_wgrad_tap64_kernel")
        torch.cuda.synchronize()
        untouched = [bool((t == 0).all()) for t in (d_h, d_h2, d_t, d_b)]
        with pytest.raises(ops.AdpError):
            ops.wgrad_defer(False)   # reductions pending
    finally:
        ops.wgrad_flush()
    torch.cuda.synchronize()
    assert untouched == [True] * 4
    assert torch.equal(d_h, ref_h) and torch.equal(d_h2, ref_h2) and torch.equal(d_t, ref_t)
    assert torch.equal(d_b, ref_b)
    assert relerr(ref_h2.cpu(), 2 * ref_h.cpu()) < 1e-6 and relerr(ref_t.cpu(), ref_h.cpu()) < 1e-4
    # after the flush the stream launches its reductions at once again
    d = z()
    run(d)
    torch.cuda.synchronize()
    assert torch.equal(d, ref_h)


F32_HALO_WGRAD_CASES = [
    # name, N, H, W (output grid), source channel strides, Nout, up
    ("c64_64", 2, 32, 64, [64], 64, False),
    ("c96_96_ragged_n", 1, 16, 64, [96], 96, False),
    ("concat_64_64", 2, 16, 32, [64, 64], 64, False),
    ("up2_96_64", 2, 32, 64, [96], 64, True),
    ("up2_352_192", 1, 16, 32, [352], 192, True),
    ("c192_352", 1, 8, 32, [192], 352, False),
]


@pytest.mark.parametrize("case", F32_HALO_WGRAD_CASES, ids=[c[0] for c in F32_HALO_WGRAD_CASES])
def test_wgrad_f32_halo(case):
    """Persistent halo form of the f32 weight gradient (igemm_wgrad_halo_f32_kernel: 32-channel input chunks,
    64-wide output blocks, 4 x 32 patches, exact v_mfma_f32_16x16x4_f32) vs autograd of the fp32 oracle conv
    (<= 1e-4 of the largest element) and vs the register-staged f32 kernel (option wgrad_f32_halo=0) on the
    same operands: adipose_v3's f32 channel strides (64 / 96 / 192 / 352: Nout not a multiple of 64 leaves a
    part-empty output block), a concat input, the nearest-x2 input gather of the up*_conv1 layers."""
    name, N, H, W_, parts, cout, up = case
    g = torch.Generator().manual_seed(61)
    Hs, Ws = (H // 2, W_ // 2) if up else (H, W_)
    xs = [torch.randn(N, Hs, Ws, c, generator=g) for c in parts]
    dZ = torch.randn(N, H, W_, cout, generator=g)
    cin = sum(parts)
    kern = (torch.randn(3, 3, cin, cout, generator=g) * 0.05).requires_grad_(True)
    x = torch.cat(xs, -1)
    if up:
        x = R.upsample_nearest2(x)
    (R.conv2d_same(x, kern, None, relu=False) * dZ).sum().backward()
    xd = [t.to(DEV).contiguous() for t in xs]
    dzd = torch.zeros(N, H, W_, cout, device=DEV)   # (the network's dZ stride: cout_s)
    dzd[..., :cout] = dZ.to(DEV)
    K = 9 * cin
    res = []
    for halo in (1, 0):
        dW = torch.zeros(((cout + 63) // 64 * 64, K), device=DEV)
        ops.set_option("wgrad_f32_halo", halo)
        try:
            ops.conv_wgrad(xd[0], dzd, dW, cout, srcB=xd[1] if len(xd) > 1 else None, up=up)
            torch.cuda.synchronize()
            kname = _lib.lib().adp_last_kernel().decode()
        finally:
            ops.set_option("wgrad_f32_halo", None)
        res.append((dW[:cout].cpu(), kname))
    assert res[0][1].startswith("igemm_wgrad_halo_f32_kernel<"), res[0][1]
    assert not res[1][1].startswith("igemm_wgrad_halo_f32_kernel"), res[1][1]
    # packed [n][tap * Cin + c] -> Keras (ky, kx, c, n)
    got = res[0][0].view(cout, 3, 3, cin).permute(1, 2, 3, 0)
    assert relerr(got, kern.grad) < 1e-4, relerr(got, kern.grad)
    assert relerr(res[0][0], res[1][0]) < 1e-5


@pytest.mark.parametrize("shape", [(2, 64, 96, 44, 64), (1, 40, 56, 48, 64), (2, 32, 32, 64, 64)],
                         ids=["n2_64x96_44of64", "ragged_40x56_48", "n2_32x32_64"])
def test_wgrad_f32_input_layer(shape):
    """f32 weight gradient of the one-real-channel input layer (wgrad_in1_f32_kernel: adipose_v3's down1_conv1, the
    gray tile in an 8-channel stride): dW at columns 8 t and dB against a float64 reference (1e-5 of the largest
    element), against the generic register-staged kernel (option wgrad_f32_in1=0, 1e-5), pad columns exactly zero,
    and two runs bit-identical (per-block slabs summed in a fixed order)."""
    from adipose_amd._lib import lib
    N, H, W_, nreal, nst = shape
    g = torch.Generator().manual_seed(131)
    x = torch.zeros(N, H, W_, 8)
    x[..., 0] = torch.randn(N, H, W_, generator=g)
    dy = torch.zeros(N, H, W_, nst)
    dy[..., :nreal] = torch.randn(N, H, W_, nreal, generator=g)
    xd, dyd = x.to(DEV), dy.to(DEV)

    def run(on):
        dW = torch.zeros(nst, 96, device=DEV)
        dB = torch.zeros(nst, device=DEV)
        ops.set_option("wgrad_f32_in1", on)
        try:
            ops.conv_wgrad(xd, dyd, dW, nst, dB=dB, real=(1, 0, nreal))
            torch.cuda.synchronize()
            kn = lib().adp_last_kernel().decode()
        finally:
            ops.set_option("wgrad_f32_in1", None)
        return dW.cpu(), dB.cpu(), kn

    w1, b1, k1 = run(1)
    w1b, b1b, _ = run(1)
    w0, b0, k0 = run(0)
    assert k1 == "wgrad_in1_f32_kernel" and k0 != k1, (k1, k0)
    assert torch.equal(w1, w1b) and torch.equal(b1, b1b)
    xp = F.pad(x[..., 0].double(), (1, 1, 1, 1))
    d64 = dy.double().reshape(-1, nst)
    ref = torch.zeros(nst, 96, dtype=torch.float64)
    for t in range(9):
        ty, tx = t // 3, t % 3
        ref[:, 8 * t] = d64.T @ xp[:, ty:ty + H, tx:tx + W_].reshape(-1)
    assert relerr(w1, ref) < 1e-5 and relerr(b1, d64.sum(0)) < 1e-5
    assert relerr(w1, w0) < 1e-5 and relerr(b1, b0) < 1e-5
    pad = [c for c in range(96) if c % 8 or c >= 72]
    assert w1[:, pad].abs().max().item() == 0


F32_DIL_WGRAD_CASES = [
    # name, dilation, N, H, W, Cin, Nout: sub-lattices of Wo / d >= 32 columns (SPLIT 1) and narrower (2, 4, 8 segments)
    ("d2_64_64", 2, 1, 32, 64, 64, 64),
    ("d4_96_96_ragged_n", 4, 2, 16, 128, 96, 96),
    ("d8_split2", 8, 1, 32, 128, 64, 64),
    ("d16_split4", 16, 1, 128, 128, 64, 64),
    ("d16_split8", 16, 1, 64, 64, 32, 96),
    ("d32_352_352_bottleneck", 32, 2, 128, 128, 352, 352),
]


@pytest.mark.parametrize("case", F32_DIL_WGRAD_CASES, ids=[c[0] for c in F32_DIL_WGRAD_CASES])
def test_wgrad_f32_halo_dilated(case):
    """Dilated halo form of the f32 weight gradient (igemm_wgrad_halo_f32_dil_kernel<SPLIT>: sub-lattice patches,
    work ranges across combinations, the bias gradient in the same pass) vs autograd of the fp32 oracle conv at the
    same dilation (<= 1e-4 of the largest element) and vs the register-staged f32 kernel (option wgrad_f32_dil=0)
    on the same operands (<= 1e-5): adipose_v3's bottleneck dilations 2 .. 32, the last at its real 128^2 x 352
    shape."""
    name, dil, N, H, W_, cin, cout = case
    g = torch.Generator().manual_seed(67)
    x = torch.randn(N, H, W_, cin, generator=g)
    dZ = torch.randn(N, H, W_, cout, generator=g)
    kern = (torch.randn(3, 3, cin, cout, generator=g) * 0.05).requires_grad_(True)
    (R.conv2d_same(x, kern, None, dilation=dil, relu=False) * dZ).sum().backward()
    xd = x.to(DEV).contiguous()
    dzd = dZ.to(DEV).contiguous()
    K = 9 * cin
    res = []
    for on in (1, 0):
        dW = torch.zeros(((cout + 63) // 64 * 64, K), device=DEV)
        dB = torch.zeros(cout, device=DEV)
        ops.set_option("wgrad_f32_dil", on)
        try:
            ops.conv_wgrad(xd, dzd, dW, cout, dB=dB, dil=dil)
            torch.cuda.synchronize()
            kname = _lib.lib().adp_last_kernel().decode()
        finally:
            ops.set_option("wgrad_f32_dil", None)
        res.append((dW[:cout].cpu(), dB.cpu(), kname))
    assert res[0][2].startswith("igemm_wgrad_halo_f32_dil_kernel<"), res[0][2]
    assert not res[1][2].startswith("igemm_wgrad_halo_f32_dil_kernel"), res[1][2]
    got = res[0][0].view(cout, 3, 3, cin).permute(1, 2, 3, 0)
    assert relerr(got, kern.grad) < 1e-4, relerr(got, kern.grad)
    assert relerr(res[0][0], res[1][0]) < 1e-5
    assert relerr(res[0][1], dZ.sum((0, 1, 2))) < 1e-5 and relerr(res[0][1], res[1][1]) < 1e-5


CLAIM_HALO_CASES = [
    # name, source channels, Nout, forward kwargs kind
    ("fwd_1ch_relu", [64], 64, "relu"),
    ("fwd_1ch_128", [64], 128, "plain"),
    ("fwd_2ch_stats", [64, 64], 128, "stats"),
    ("fwd_2ch_bnr", [128], 64, "bnr"),
    ("fwd_1ch_mask", [64], 64, "mask"),
    ("fwd_2ch_split", [128], 128, "split"),
    ("fwd_1ch_up2", [64], 64, "up"),
    ("wgrad_1ch", [64], 64, "wgrad"),
    ("wgrad_2src", [64, 64], 128, "wgrad"),
    ("wgrad_bna", [64], 64, "wgrad_bna"),
]


@pytest.mark.parametrize("grid", [None, 7, 1], ids=["chip_grid", "7_blocks", "1_block"])
@pytest.mark.parametrize("case", CLAIM_HALO_CASES, ids=[c[0] for c in CLAIM_HALO_CASES])
def test_halo_kernels_claimed_match_static(case, grid):
    """Dynamic tile claiming in the persistent halo kernels (options halop_claim, wgrad_halop_claim): the tiles a
    block takes change, their arithmetic does not. Forward forms (plain / ReLU / statistics / BN-backward
    reduction / mask / split / upsample gather): stored outputs bit-identical to the static lists, BatchNorm sums
    to f32 order; weight gradient (plain, two sources, fused BN apply): dW to f32 order (per-block f32 atomics),
    dz bit-identical. Each claimed launch runs three times (the counter slot re-zeroed by its last block), then twice
    with every super-tile claimed (option claim_full, one-patch claims so that the 1 / 7-block grids take it)."""
    name, parts, cout, kind = case
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(51)
    N, H, W_ = 2, 64, 64
    up = kind == "up"
    Hs, Ws = (H // 2, W_ // 2) if up else (H, W_)
    srcs = [torch.randn(N, Hs, Ws, c, generator=g).to(DEV, dt) for c in parts]
    cin = sum(parts)
    vec = lambda n: (torch.rand(n, generator=g) + 0.5).to(DEV)   # noqa: E731
    wopt = "wgrad_halop_claim" if kind.startswith("wgrad") else "halop_claim"

    def run():
        if kind.startswith("wgrad"):
            dZ = torch.randn(N, H, W_, cout, generator=torch.Generator().manual_seed(5)).to(DEV, dt)
            dW = torch.zeros((cout, 9 * cin), device=DEV)
            if kind == "wgrad_bna":
                gg = torch.Generator().manual_seed(6)
                z = (torch.randn(N, H, W_, cout, generator=gg) * 2).to(DEV, dt)
                v = [(torch.rand(cout, generator=gg) + 0.5).to(DEV) for _ in range(7)]
                dz = torch.zeros_like(z)
                ops.conv_wgrad(srcs[0], dz, dW, cout, bn_apply=(dZ, z, v[0], v[1] - 1.0, v[2] - 1.0, v[3], v[4], v[5],
                                                                 v[6], N * H * W_))
                return [dz], [dW]
            ops.conv_wgrad(srcs[0], dZ, dW, cout, srcB=srcs[1] if len(srcs) > 1 else None)
            return [], [dW]
        gw = torch.Generator().manual_seed(7)
        Wt = (torch.randn(cout, 9 * cin, generator=gw) * 0.03).to(DEV, dt)
        out = torch.zeros(N, H, W_, cout, dtype=dt, device=DEV)
        st = torch.zeros(2, cout, device=DEV)
        kw = dict(srcB=srcs[1] if len(srcs) > 1 else None, up=up)
        outs = [out]
        if kind == "bnr":
            z = torch.randn(N, H, W_, cout, generator=gw).to(DEV, dt)
            v = [(torch.rand(cout, generator=gw) + 0.5).to(DEV) for _ in range(4)]
            ops.conv_fwd(srcs[0], Wt, cout, out=out, bn_reduce=(z, v[0], v[1] - 1.0, v[2] - 1.0, v[3], st[1], st[0]), **kw)
        elif kind == "mask":
            m = torch.randn(N, H, W_, cout, generator=gw).to(DEV, dt)
            ops.conv_fwd(srcs[0], Wt, cout, out=out, mask=m, **kw)
        elif kind == "split":
            o2 = torch.zeros(N, H, W_, cout - 64, dtype=dt, device=DEV)
            out = torch.zeros(N, H, W_, 64, dtype=dt, device=DEV)
            outs = [out, o2]
            ops.conv_fwd(srcs[0], Wt, cout, out=out, out_mode=2, out2=o2, split_c=64, **kw)
        else:
            b = torch.randn(cout, generator=gw).to(DEV)
            ops.conv_fwd(srcs[0], Wt, cout, out=out, bias=b, relu=kind in ("relu", "up"),
                         bn_stats=(st[0], st[1]) if kind == "stats" else None, **kw)
        return outs, [st]

    res = []
    try:
        if grid:
            ops.set_option("halo_persist_grid", grid)
            ops.set_option("wgrad_halop_grid", grid)
        for claim in (0, 1, 1, 1, 2, 2):
            ops.set_option(wopt, min(claim, 1))
            if claim == 2:
                ops.set_option("claim_full", 1)
                ops.set_option(wopt + "_chunk", 1)
            ex, fl = run()
            torch.cuda.synchronize()
            res.append((ex, fl, _lib.lib().adp_last_kernel().decode()))
    finally:
        for o_ in ("halo_persist_grid", "wgrad_halop_grid", wopt, "claim_full", wopt + "_chunk"):
            ops.set_option(o_, None)
    k0 = res[0][2]
    assert k0.startswith("igemm_wgrad_halop" if kind.startswith("wgrad") else "igemm_fwd_halop_kernel"), k0
    for ex, fl, kn in res[1:]:
        if not kind.startswith("wgrad") and kind != "bnr":
            assert kn.split("<")[1].rstrip(">").split(", ")[6] == "true", kn   # the claimed form ran (DYN)
        for a_, b_ in zip(ex, res[0][0]):
            assert torch.equal(a_, b_)
        for a_, b_ in zip(fl, res[0][1]):
            assert relerr(a_, b_) < 1e-5


@pytest.mark.parametrize("N,Hs,Ws,parts,cout", [(2, 8, 16, [64], 64), (1, 16, 32, [128], 128), (2, 8, 32, [192], 192)])
def test_wgrad_persistent_halo_upsample(N, Hs, Ws, parts, cout):
    """Halo weight gradient with the nearest-x2 upsample folded into its input gather (adipose_v3's
    UpSampling2D + conv, train_adipose_unet_v3.py:691-692) vs autograd of the oracle conv on the upsampled
    input, and vs the tap64 / glds kernels (option wgrad_halop=0)."""
    from adipose_amd import _lib
    cin = sum(parts)
    _, kern, bias, l = make_case(N, 2 * Hs, parts, cout, 1, False, seed=23)
    g = torch.Generator().manual_seed(24)
    dt = torch.bfloat16
    x = rb(torch.randn(N, Hs, Ws, cin, generator=g), dt)
    xu = x.repeat_interleave(2, 1).repeat_interleave(2, 2)
    dZ = rb(torch.randn(N, 2 * Hs, 2 * Ws, cout, generator=g), dt)
    kr = rb(kern, dt).clone().requires_grad_(True)
    (R.conv2d_same(xu, kr, None, relu=False) * dZ).sum().backward()
    xd = x.to(DEV, dt).contiguous()
    dzd = nhwc_pad(dZ, l.cout_s, dt)
    dW = torch.zeros((l.Npad, l.Kpad), device=DEV)
    ref = torch.zeros_like(dW)
    try:
        ops.conv_wgrad(xd, dzd, dW, l.Nout, up=True)
        kname = _lib.lib().adp_last_kernel().decode()
        ops.set_option("wgrad_halop", 0)
        ops.conv_wgrad(xd, dzd, ref, l.Nout, up=True)
        torch.cuda.synchronize()
    finally:
        ops.set_option("wgrad_halop", None)
    assert kname == "igemm_wgrad_halopair_kernel<6, 0>", kname
    assert relerr(torch.from_numpy(l.packed_to_keras(dW.cpu().numpy())), kr.grad) < 2e-2
    assert relerr(dW.cpu(), ref.cpu()) < 1e-4


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("S", [8, 64])
def test_conv_transpose(dt, S):
    N, cin, cout = 2, 128, 64
    g = torch.Generator().manual_seed(3)
    x = rb(torch.randn(N, S, S, cin, generator=g), dt)
    k = rb(torch.randn(cin, cout, 2, 2, generator=g) * 0.1, dt)
    b = torch.randn(cout, generator=g) * 0.1
    l = Dense("t", [cin], cout, transpose=True, relu=False)
    xr = x.clone().requires_grad_(True)
    kr = k.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    y = F.conv_transpose2d(xr.permute(0, 3, 1, 2), kr, br, stride=2).permute(0, 2, 3, 1)
    dY = rb(torch.randn(y.shape, generator=g), dt)
    (y * dY).sum().backward()
    Wm = torch.from_numpy(l.keras_to_packed(k.numpy())).to(DEV)
    bd = b.to(DEV)
    xd = nhwc_pad(x, l.Cin_s, dt)
    out = torch.zeros((N, 2 * S, 2 * S, l.cout_s), dtype=dt, device=DEV)
    ops.conv_fwd(xd, Wm.to(dt).contiguous(), l.Nout, out=out, bias=bd, kh=1, kw=1, pad=0, out_mode=1,
                 shuffle_c=l.cout_s)
    dYd = nhwc_pad(dY, l.cout_s, dt)
    dW = torch.zeros((l.Npad, l.Kpad), device=DEV)
    dB = torch.zeros(l.cout_s, device=DEV)
    ops.conv_wgrad(xd, dYd, dW, l.Nout, dB=dB, kh=1, kw=1, pad=0, shuffle_c=l.cout_s)
    Wd = torch.zeros((l.dNpad, l.dKpad), dtype=dt, device=DEV)
    ops.pack_weights(Wm, Wd, 2, taps=1, cin_s=l.Cin_s, nout=l.Nout)
    dX = torch.zeros((N, S, S, l.Cin_s), dtype=dt, device=DEV)
    ops.conv_fwd(dYd, Wd, l.Cin_s, out=dX, kh=2, kw=2, pad=0, stride=2, Ho=S, Wo=S)
    torch.cuda.synchronize()
    tol = 1e-4 if dt == torch.float32 else 2e-2
    assert relerr(out, y.detach()) < tol
    assert relerr(torch.from_numpy(l.packed_to_keras(dW.cpu().numpy())), kr.grad) < tol
    assert relerr(dB, br.grad) < tol
    assert relerr(dX, xr.grad) < tol


def test_sum_bf16_matches_accumulate():
    """adp_sum_bf16 (the bottleneck Add as one pass) == an f32 accumulator zeroed, += each bf16 map in
    order, cast to bf16 (the accumulate-epilogue path): bit for bit."""
    g = torch.Generator().manual_seed(5)
    maps = [(torch.randn(2, 16, 16, 384, generator=g) * (k + 1)).to(DEV, torch.bfloat16) for k in range(6)]
    acc = torch.zeros(maps[0].shape, device=DEV)
    for m in maps:
        acc += m.float()
    out = torch.full_like(maps[0], 7.0)
    ops.sum_bf16(maps, out)
    torch.cuda.synchronize()
    assert torch.equal(out, acc.to(torch.bfloat16))
    one = torch.empty_like(out)
    ops.sum_bf16(maps[:1], one)
    assert torch.equal(one, maps[0])


@pytest.mark.parametrize("dt", DTS)
def test_pool_upsample(dt):
    g = torch.Generator().manual_seed(7)
    x = rb(torch.relu(torch.randn(2, 16, 16, 48, generator=g)), dt)
    xd = x.to(DEV, dt).contiguous()
    p = torch.zeros((2, 8, 8, 48), dtype=dt, device=DEV)
    ops.maxpool2_fwd(xd, p)
    xr = x.clone().requires_grad_(True)
    pr = R.maxpool2(xr)
    dp = rb(torch.randn(pr.shape, generator=g), dt)
    (pr * dp).sum().backward()
    add = rb(torch.randn(x.shape, generator=g), dt)
    dx = torch.zeros_like(xd)
    ops.maxpool2_bwd(xd, dp.to(DEV, dt).contiguous(), dx, addend=add.to(DEV, dt).contiguous(), mask=xd)
    torch.cuda.synchronize()
    assert relerr(p, pr.detach()) < 1e-6
    ref = (xr.grad + add) * (x > 0).float()
    assert relerr(dx, ref) < (1e-6 if dt == torch.float32 else 1e-2)
    # nearest-upsample gradient = 2x2 sum
    du = rb(torch.randn(2, 16, 16, 48, generator=g), dt)
    ds = torch.zeros((2, 8, 8, 48), dtype=dt, device=DEV)
    ops.upsample2_bwd(du.to(DEV, dt).contiguous(), ds)
    torch.cuda.synchronize()
    ref = du.reshape(2, 8, 2, 8, 2, 48).sum((2, 4))
    assert relerr(ds, ref) < (1e-6 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("S,cout", [(32, 64), (19, 48)])
def test_cin8_input_layer_bn_stats(S, cout):
    """bf16 input-layer launch (adp_conv_fwd -> igemm_fwd_cin8_kernel): output vs the oracle on
    bf16-rounded operands, BatchNorm sums of the stored values vs a host reduction of the same
    (pre-rounding) values, pad channels untouched."""
    from adipose_amd._lib import lib
    xs, kern, bias, l = make_case(2, S, [3], cout, 1, False, seed=3)
    W = torch.from_numpy(l.keras_to_packed(kern.numpy())).to(DEV).to(torch.bfloat16).contiguous()
    b = torch.zeros(l.cout_s, device=DEV)
    b[:cout] = bias.to(DEV)
    src = nhwc_pad(xs[0], l.cin_s[0], torch.bfloat16)
    out = torch.zeros((2, S, S, l.cout_s), dtype=torch.bfloat16, device=DEV)
    s1 = torch.zeros(l.cout_s, device=DEV)
    s2 = torch.zeros(l.cout_s, device=DEV)
    ops.conv_fwd(src, W, l.Nout, out=out, bias=b, relu=False, bn_stats=(s1, s2))
    torch.cuda.synchronize()
    assert lib().adp_last_kernel().decode().startswith("igemm_fwd_cin8")
    ref = oracle_fwd([rb(xs[0], torch.bfloat16)], rb(kern, torch.bfloat16), bias, 1, False, relu=False)
    assert relerr(out[..., :cout], ref) < TOL[torch.bfloat16]
    if l.cout_s > cout:
        assert out[..., cout:].abs().max().item() == 0.0
    r = ref.reshape(-1, cout).double()
    assert bool(((s1[:cout].cpu().double() - r.sum(0)).abs() <= 1e-2 * r.abs().sum(0) + 1e-3).all())
    assert bool(((s2[:cout].cpu().double() - (r * r).sum(0)).abs() <= 1e-2 * (r * r).sum(0) + 1e-3).all())


@pytest.mark.parametrize("N,S,cin,cout,dil,hint", [(2, 32, 1, 44, 1, True), (2, 32, 3, 64, 1, True),
                                                     (3, 13, 3, 24, 2, False), (1, 19, 1, 44, 1, False)])
def test_cin8_f32_input_layer(N, S, cin, cout, dil, hint):
    """f32 input-layer launch (igemm_fwd_cin8_f32_kernel: exact f32 MFMA, one channel quad per tap when the caller says
    CA_real <= 4, else two) vs the f64 oracle at the f32 gate, BatchNorm sums vs a host reduction, pad channels stored
    as zeros; and within f32 rounding of the generic register-staged kernel it replaces (option fwd_cin8_f32=0).
    Ragged images leave partial 16-pixel groups."""
    from adipose_amd._lib import lib
    xs, kern, bias, l = make_case(N, S, [cin], cout, dil, False, seed=17)
    W = torch.from_numpy(l.keras_to_packed(kern.numpy())).to(DEV).float().contiguous()
    b = torch.zeros(l.cout_s, device=DEV)
    b[:cout] = bias.to(DEV)
    src = nhwc_pad(xs[0], l.cin_s[0], torch.float32)
    res = {}
    for on in (1, 0):
        ops.set_option("fwd_cin8_f32", on)
        try:
            out = torch.full((N, S, S, l.cout_s), 7.0, device=DEV)
            s1 = torch.zeros(l.cout_s, device=DEV)
            s2 = torch.zeros(l.cout_s, device=DEV)
            ops.conv_fwd(src, W, l.Nout, out=out, bias=b, relu=True, dil=dil, bn_stats=(s1, s2),
                         real=(cin, 0, cout) if hint else None)
            torch.cuda.synchronize()
            res[on] = (out.clone(), s1.clone(), s2.clone(), lib().adp_last_kernel().decode())
        finally:
            ops.set_option("fwd_cin8_f32", None)
    out, s1, s2, kname = res[1]
    assert kname == f"igemm_fwd_cin8_f32_kernel<{1 if hint and cin <= 4 else 2}, 4>", kname
    assert not res[0][3].startswith("igemm_fwd_cin8_f32"), res[0][3]
    ref = oracle_fwd([xs[0]], kern, bias, dil, False, relu=True)
    assert relerr(out[..., :cout], ref) < TOL[torch.float32]
    assert relerr(out, res[0][0]) < 1e-6
    if l.cout_s > cout:
        assert out[..., cout:].abs().max().item() == 0.0
    r = ref.reshape(-1, cout).double()
    assert bool(((s1[:cout].cpu().double() - r.sum(0)).abs() <= 1e-4 * r.abs().sum(0) + 1e-4).all())
    assert bool(((s2[:cout].cpu().double() - (r * r).sum(0)).abs() <= 1e-4 * (r * r).sum(0) + 1e-4).all())


@pytest.mark.parametrize("N,S,cin,cout,dil,relu", [(2, 32, 3, 64, 1, True), (3, 13, 1, 44, 2, False),
                                                     (1, 10, 3, 24, 1, True), (5, 8, 3, 64, 1, False)])
def test_cin8_pipelined_matches_plain(N, S, cin, cout, dil, relu):
    """The pipelined branch-free input-layer kernel (igemm_fwd_cin8p_kernel, buffer accesses with
    out-of-range padding / tail offsets) against the plain one (option cin8_pf=0; with 16-B stores of
    permlane16_swap-joined quads, and with 8-B stores, cin8_wide=0): same MFMA order, so the
    stored outputs are bit-identical; BatchNorm sums equal up to the order of the per-wave atomics; pad
    channels stored as zeros. Ragged images (13x13, 10x10, 8x8) leave partial 16-pixel groups."""
    from adipose_amd._lib import lib
    xs, kern, bias, l = make_case(N, S, [cin], cout, dil, False, seed=11)
    W = torch.from_numpy(l.keras_to_packed(kern.numpy())).to(DEV).to(torch.bfloat16).contiguous()
    b = torch.zeros(l.cout_s, device=DEV)
    b[:cout] = bias.to(DEV)
    src = nhwc_pad(xs[0], l.cin_s[0], torch.bfloat16)
    res = {}
    for pf in (1, 0, "narrow"):   # "narrow": the plain form with 8-B stores (option cin8_wide=0)
        ops.set_option("cin8_pf", 1 if pf == 1 else 0)
        ops.set_option("cin8_wide", 0 if pf == "narrow" else 1)
        try:
            out = torch.full((N, S, S, l.cout_s), 7.0, dtype=torch.bfloat16, device=DEV)
            s1 = torch.zeros(l.cout_s, device=DEV)
            s2 = torch.zeros(l.cout_s, device=DEV)
            ops.conv_fwd(src, W, l.Nout, out=out, bias=b, relu=relu, dil=dil, bn_stats=(s1, s2))
            torch.cuda.synchronize()
            res[pf] = (out.clone(), s1.clone(), s2.clone(), lib().adp_last_kernel().decode())
        finally:
            ops.set_option("cin8_pf", None)
            ops.set_option("cin8_wide", None)
    assert res[1][3].startswith("igemm_fwd_cin8p_kernel") and res[0][3].startswith("igemm_fwd_cin8_kernel")
    assert torch.equal(res[1][0], res[0][0]) and torch.equal(res["narrow"][0], res[0][0])
    for k in (1, 2):
        assert torch.allclose(res["narrow"][k], res[0][k], rtol=1e-5, atol=1e-3)
    if l.cout_s > cout:   # (pad channels: zero weight rows, zero bias -> stored zeros, as the plain form)
        assert res[1][0][..., cout:].abs().max().item() == 0.0
    ref = oracle_fwd([rb(xs[0], torch.bfloat16)], rb(kern, torch.bfloat16), bias, dil, False, relu=relu)
    assert relerr(res[1][0][..., :cout], ref) < TOL[torch.bfloat16]
    for k in (1, 2):
        assert torch.allclose(res[1][k], res[0][k], rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("C", [64, 128, 1024, 48])
def test_pool_bwd_fused_bn_reduce(dt, C):
    """adp_maxpool2_bwd_bnr == adp_maxpool2_bwd(addend) followed by adp_bn_bwd_reduce: identical dsrc,
    dgamma/dbeta equal up to f32 summation order (and to the CPU oracle of the BN-backward sums)."""
    g = torch.Generator().manual_seed(C)
    N, H = 2, 12
    z = rb(torch.randn(N, H, H, C, generator=g), dt).to(DEV, dt).contiguous()
    sc = (torch.rand(C, generator=g) + 0.5).to(DEV)
    sh = (torch.randn(C, generator=g) * 0.3).to(DEV)
    mu = (torch.randn(C, generator=g) * 0.1).to(DEV)
    ist = (torch.rand(C, generator=g) + 0.5).to(DEV)
    a = torch.zeros_like(z)
    ops.bn_apply(z, sc, sh, a)
    dp = rb(torch.randn(N, H // 2, H // 2, C, generator=g), dt).to(DEV, dt).contiguous()
    add = rb(torch.randn(N, H, H, C, generator=g), dt).to(DEV, dt).contiguous()
    d1, d2, d3 = torch.zeros_like(z), torch.zeros_like(z), torch.zeros_like(z)
    dg1, db1, dg2, db2, dg3, db3 = (torch.zeros(C, device=DEV) for _ in range(6))
    ops.maxpool2_bwd(a, dp, d1, addend=add)
    ops.bn_bwd_reduce(d1, z, sc, sh, mu, ist, dg1, db1)
    ops.maxpool2_bwd(a, dp, d2, addend=add, bn_reduce=(z, sc, sh, mu, ist, dg2, db2), argmax_from_z=False)
    ops.maxpool2_bwd(a, dp, d3, addend=add, bn_reduce=(z, sc, sh, mu, ist, dg3, db3))   # argmax from z
    torch.cuda.synchronize()
    assert torch.equal(d1, d2) and torch.equal(d1, d3)
    assert torch.equal(dg2, dg3) and torch.equal(db2, db3)
    zf, df = z.float().cpu(), d1.float().cpu()
    db = torch.where(zf * sc.cpu() + sh.cpu() > 0, df, torch.zeros_like(df))
    ref_b = db.sum((0, 1, 2))
    ref_g = (db * (zf - mu.cpu()) * ist.cpu()).sum((0, 1, 2))
    for got, ref in ((db2, ref_b), (dg2, ref_g), (db1, ref_b), (dg1, ref_g)):
        assert (got.cpu() - ref).abs().max().item() <= 1e-4 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("softmax2", [True, False])
def test_heads(dt, softmax2):
    g = torch.Generator().manual_seed(11)
    cin, cs = 44, 48
    nout = 2 if softmax2 else 1
    x = rb(torch.relu(torch.randn(2, 8, 8, cin, generator=g)), dt)
    k = torch.randn(1, 1, cin, nout, generator=g) * 0.3
    b = torch.randn(nout, generator=g) * 0.1
    h = Head("h", cin, nout)
    Wd = torch.from_numpy(h.keras_to_packed(k.numpy())).to(DEV)
    xd = nhwc_pad(x, cs, dt)
    p = torch.zeros((2, 8, 8), device=DEV)
    ops.head_fwd(xd, Wd, b.to(DEV), p, cin=cin, softmax2=softmax2)
    xr = x.clone().requires_grad_(True)
    kr = k.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    z = R.conv1x1(xr, kr, br)
    pr = torch.softmax(z, -1)[..., 1] if softmax2 else torch.sigmoid(z)[..., 0]
    dp = torch.randn(pr.shape, generator=g)
    (pr * dp).sum().backward()
    dW = torch.zeros_like(Wd)
    dB = torch.zeros(nout, device=DEV)
    dx = torch.zeros_like(xd)
    ops.head_bwd(xd, Wd, p, dp.to(DEV), dW, dB, cin=cin, softmax2=softmax2, dx=dx)
    torch.cuda.synchronize()
    assert relerr(p, pr.detach()) < 1e-5
    assert relerr(torch.from_numpy(h.packed_to_keras(dW.cpu().numpy())), kr.grad) < 1e-4
    assert relerr(dB, br.grad) < 1e-4
    assert relerr(dx[..., :cin], xr.grad) < (1e-5 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("scale", [2, 4])
def test_resize_bilinear(scale):
    g = torch.Generator().manual_seed(13)
    s = torch.rand(2, 16, 16, generator=g)
    sr = s.clone().requires_grad_(True)
    o = R.resize_bilinear_half_pixel(sr[..., None], (16 * scale, 16 * scale))[..., 0]
    do = torch.randn(o.shape, generator=g)
    (o * do).sum().backward()
    od = torch.zeros(o.shape, device=DEV)
    ops.resize_bilinear_fwd(s.to(DEV), od)
    dsd = torch.zeros(s.shape, device=DEV)
    ops.resize_bilinear_bwd(do.to(DEV), dsd)
    torch.cuda.synchronize()
    assert relerr(od, o.detach()) < 1e-6
    assert relerr(dsd, sr.grad) < 1e-5


@pytest.mark.parametrize("ohem,smooth", [(True, False), (False, False), (True, True), (False, True)])
def test_loss_value_and_grad(ohem, smooth):
    g = torch.Generator().manual_seed(17)
    N, H, W = 2, 64, 64
    p = torch.rand(N, H, W, generator=g)
    p[0, 0, :4] = torch.tensor([0.0, 1.0, 1e-9, 1 - 1e-9])   # clip edges
    y = (torch.rand(N, H, W, generator=g) > 0.6).float()
    pr = p.clone().requires_grad_(True)
    if ohem:
        L = R.ohem_loss_with_smoothing(y, pr) if smooth else R.ohem_loss(y, pr)
    else:
        L = R.combined_loss_with_label_smoothing(y, pr) if smooth else R.combined_loss_standard(y, pr)
    L.backward()
    pd, yd = p.to(DEV), y.to(DEV)
    rows = torch.zeros(N * H, device=DEV)
    stats = torch.zeros(8, dtype=torch.float64, device=DEV)
    coef = torch.zeros(N * H, device=DEV)
    out = torch.zeros(1, dtype=torch.float64, device=DEV)
    ops.loss_rows(pd, yd, rows, stats, smooth=smooth)
    k = int(np.float32(H) * np.float32(0.7)) if ohem else H
    ops.loss_select(rows, coef, out, N=N, H=H, W=W, ohem=ohem, keep_ratio=0.7, weight=1.0, norm_rows=N * k)
    dp = torch.zeros_like(pd)
    ops.loss_grad(pd, yd, coef, stats, dp, weight=1.0, smooth=smooth)
    torch.cuda.synchronize()
    st = stats.cpu().numpy()
    dice = 1.0 - (2 * st[0] + 1) / (st[1] + st[2] + 1)
    val = out.item() + dice
    assert abs(val - L.item()) < 1e-5 * max(1.0, abs(L.item()))
    assert relerr(dp, pr.grad) < 1e-4
    # dice_coef / binary accuracy stats
    assert abs((2 * st[3] + 1) / (st[4] + st[5] + 1) - R.dice_coef(y, p).item()) < 1e-6
    assert abs(st[6] / (N * H * W) - R.binary_accuracy(y, p).item()) < 1e-6


def test_adam_matches_keras():
    g = torch.Generator().manual_seed(19)
    w = torch.randn(1000, generator=g)
    grads = [torch.randn(1000, generator=g) for _ in range(3)]
    ref = R.KerasAdam([w.clone()], lr=1e-3, weight_decay=0.01)
    wd, m, v = w.to(DEV), torch.zeros(1000, device=DEV), torch.zeros(1000, device=DEV)
    for t, gr in enumerate(grads, 1):
        ref.step([gr])
        ops.adam(wd, gr.to(DEV), m, v, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-7, step=t, weight_decay=0.01)
    torch.cuda.synchronize()
    assert relerr(wd, ref.p[0]) < 1e-6


def test_pixel_counts_and_blend():
    g = torch.Generator().manual_seed(23)
    pred = torch.rand(64, 64, generator=g)
    true = (torch.rand(64, 64, generator=g) > 0.5).float()
    c = torch.zeros(4, dtype=torch.int64, device=DEV)
    ops.pixel_counts(pred.to(DEV), true.to(DEV), 0.5, c)
    pb, tb = pred > 0.5, true > 0.5
    ref = [int((pb & tb).sum()), int((pb & ~tb).sum()), int((~pb & tb).sum()), int((~pb & ~tb).sum())]
    assert c.cpu().tolist() == ref


def test_pack_weights_batch_matches_per_layer():
    """Batched LDS-tiled data-gradient repack (adp_pack_weights_batch) == per-layer adp_pack_weights
    (modes 1 and 2) for ragged shapes, both destination dtypes, several layers in one launch."""
    g = torch.Generator().manual_seed(71)
    shapes = [(9, 64, 64), (9, 48, 88), (1, 128, 256), (9, 176, 352), (9, 8, 64), (1, 64, 512)]
    for dt in (torch.float32, torch.bfloat16):
        jobs, refs = [], []
        for taps, cin_s, nout in shapes:
            Kpad, Npad = (taps * cin_s + 31) // 32 * 32, (nout + 63) // 64 * 64
            src = torch.randn(Npad, Kpad, generator=g).to(DEV)
            rows, dkp = (cin_s + 63) // 64 * 64 + 64, (taps * nout + 31) // 32 * 32
            ref = torch.full((rows, dkp), 7.0, device=DEV).to(dt)
            ops.pack_weights(src, ref, 1 if taps == 9 else 2, taps=taps, cin_s=cin_s, nout=nout)
            got = torch.full((rows, dkp), 7.0, device=DEV).to(dt)
            jobs.append((src, got, taps, cin_s, nout))
            refs.append(ref)
        ops.pack_weights_batch(jobs)
        torch.cuda.synchronize()
        for (_, got, *_), ref in zip(jobs, refs):
            assert torch.equal(got, ref)


@pytest.mark.parametrize("dt", DTS)
def test_bn_apply_maxpool_fused(dt):
    """adp_bn_apply_maxpool2 == adp_bn_apply followed by adp_maxpool2_fwd, bit for bit."""
    g = torch.Generator().manual_seed(81)
    z = (torch.randn(2, 32, 48, 64, generator=g) * 2).to(DEV, dt)
    sc = (torch.rand(64, generator=g) + 0.5).to(DEV)
    sh = (torch.randn(64, generator=g) * 0.5).to(DEV)
    a1, a2 = torch.empty_like(z), torch.empty_like(z)
    p1 = torch.empty((2, 16, 24, 64), dtype=dt, device=DEV)
    p2 = torch.empty_like(p1)
    ops.bn_apply(z, sc, sh, a1)
    ops.maxpool2_fwd(a1, p1)
    ops.bn_apply_maxpool2(z, sc, sh, a2, p2)
    torch.cuda.synchronize()
    assert torch.equal(a1, a2) and torch.equal(p1, p2)


@pytest.mark.parametrize("dt", DTS)
def test_head_bn_on_load_and_fused_bn_reduce(dt):
    """unet_bn head with dec0_conv2's BatchNorm applied on load (forward) and its BatchNorm-backward
    reduction fused (adp_head_sigmoid_bwd_bnr) == adp_bn_apply + plain head + adp_bn_bwd_reduce: p, dx and
    dW bit for bit (same rounding of the activation), dgamma/dbeta to f32 summation-order tolerance."""
    g = torch.Generator().manual_seed(83)
    M, Cs, cin = 3 * 40 * 64, 64, 48
    z = (torch.randn(3, 40, 64, Cs, generator=g) * 2).to(DEV, dt)
    sc = (torch.rand(Cs, generator=g) + 0.5).to(DEV)
    sh = (torch.randn(Cs, generator=g) * 0.5).to(DEV)
    mean = (torch.randn(Cs, generator=g) * 0.1).to(DEV)
    inv = (torch.rand(Cs, generator=g) + 0.5).to(DEV)
    W = (torch.randn(cin, generator=g) * 0.2).to(DEV)
    b = torch.tensor([0.1], device=DEV)
    dp = torch.randn(M, generator=g).to(DEV)
    act = torch.empty_like(z)
    ops.bn_apply(z, sc, sh, act)
    p1, p2 = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    ops.head_fwd(act, W, b, p1, cin=cin, softmax2=False)
    ops.head_fwd(z, W, b, p2, cin=cin, softmax2=False, bn=(sc, sh))
    dx1, dx2 = torch.empty_like(z), torch.empty_like(z)
    gw1, gw2 = torch.zeros(cin, device=DEV), torch.zeros(cin, device=DEV)
    gb1, gb2 = torch.zeros(1, device=DEV), torch.zeros(1, device=DEV)
    dg1, dg2, db1, db2 = (torch.zeros(Cs, device=DEV) for _ in range(4))
    ops.head_bwd(act, W, p1, dp, gw1, gb1, cin=cin, softmax2=False, dx=dx1)
    ops.bn_bwd_reduce(dx1, z, sc, sh, mean, inv, dg1, db1)
    ops.head_bwd(z, W, p1, dp, gw2, gb2, cin=cin, softmax2=False, dx=dx2, bn=(sc, sh),
                 bn_reduce=(mean, inv, dg2, db2))
    torch.cuda.synchronize()
    assert torch.equal(p1, p2) and torch.equal(dx1, dx2)
    torch.testing.assert_close(gw2, gw1, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gb2, gb1, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(dg2, dg1, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(db2, db1, rtol=1e-4, atol=1e-3)
    # the compile-time form (round 6, option head_bwd_fast) against the run-time-flag form: dx bit for bit, the sums
    # (per-block f64 replicas; the two forms may be resident with different block counts) to f32 rounding
    outs = []
    for fast in (1, 0):
        dx3 = torch.empty_like(z)
        gw3, gb3 = torch.zeros(cin, device=DEV), torch.zeros(1, device=DEV)
        dg3, db3 = torch.zeros(Cs, device=DEV), torch.zeros(Cs, device=DEV)
        ops.set_option("head_bwd_fast", fast)
        try:
            ops.head_bwd(z, W, p1, dp, gw3, gb3, cin=cin, softmax2=False, dx=dx3, bn=(sc, sh),
                         bn_reduce=(mean, inv, dg3, db3))
            torch.cuda.synchronize()
        finally:
            ops.set_option("head_bwd_fast", None)
        outs.append((dx3, gw3, gb3, dg3, db3))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][0], dx2)
    for u, v in zip(outs[0][1:], outs[1][1:]):
        torch.testing.assert_close(u, v, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("dt", DTS)
def test_bn_bwd_apply_head_recompute(dt):
    """adp_bn_bwd_apply_head (dA recomputed from the sigmoid head) == adp_head_sigmoid_bwd_bnr's stored dx
    fed to adp_bn_bwd_apply, bit for bit; the fused head backward with dx=None leaves the same sums."""
    g = torch.Generator().manual_seed(84)
    Cs, cin = 64, 48
    shape = (2, 24, 96, Cs)
    M = shape[0] * shape[1] * shape[2]
    z = (torch.randn(*shape, generator=g) * 2).to(DEV, dt)
    sc = (torch.rand(Cs, generator=g) + 0.5).to(DEV)
    sh = (torch.randn(Cs, generator=g) * 0.5).to(DEV)
    mean = (torch.randn(Cs, generator=g) * 0.1).to(DEV)
    inv = (torch.rand(Cs, generator=g) + 0.5).to(DEV)
    gam = (torch.rand(Cs, generator=g) + 0.5).to(DEV)
    W = (torch.randn(cin, generator=g) * 0.2).to(DEV)
    b = torch.tensor([0.1], device=DEV)
    dp = torch.randn(M, generator=g).to(DEV)
    p = torch.empty(M, device=DEV)
    ops.head_fwd(z, W, b, p, cin=cin, softmax2=False, bn=(sc, sh))
    dx = torch.empty_like(z)
    gw1, gw2 = torch.zeros(cin, device=DEV), torch.zeros(cin, device=DEV)
    gb1, gb2 = torch.zeros(1, device=DEV), torch.zeros(1, device=DEV)
    dg1, dg2, db1, db2 = (torch.zeros(Cs, device=DEV) for _ in range(4))
    ops.head_bwd(z, W, p, dp, gw1, gb1, cin=cin, softmax2=False, dx=dx, bn=(sc, sh), bn_reduce=(mean, inv, dg1, db1))
    ops.head_bwd(z, W, p, dp, gw2, gb2, cin=cin, softmax2=False, dx=None, bn=(sc, sh), bn_reduce=(mean, inv, dg2, db2))
    dz1, dz2 = torch.empty_like(z), torch.empty_like(z)
    ops.bn_bwd_apply(dx, z, sc, sh, mean, inv, gam, dg1, db1, M, dz1)
    ops.bn_bwd_apply_head(W, p, dp, z, sc, sh, mean, inv, gam, dg1, db1, M, dz2, cin=cin)
    torch.cuda.synchronize()
    assert torch.equal(dz1, dz2)
    torch.testing.assert_close(gw2, gw1, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gb2, gb1, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(dg2, dg1, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(db2, db1, rtol=1e-4, atol=1e-3)


def test_deferred_bn_fold_is_guarded():
    """A conv launch with bn_defer_fold leaves its BatchNorm sums in the library's accumulator replicas: until
    the matching adp_bn_finalize_fold (same channel count, sum vector, stream) runs, every other launch that
    uses the replicas must fail loudly instead of mixing its sums in, and the matching finalize
    then gives the statistics of the non-deferred form."""
    g = torch.Generator().manual_seed(5)
    N, H, C = 2, 16, 64
    x = torch.randn(N, H, 32, 64, generator=g).to(DEV, torch.bfloat16)
    W = (torch.randn(64, 9 * 64, generator=g) * 0.05).to(DEV, torch.bfloat16)
    out = torch.zeros(N, H, 32, C, device=DEV, dtype=torch.bfloat16)
    gamma, beta = torch.ones(C, device=DEV), torch.zeros(C, device=DEV)
    vec = lambda: torch.zeros(C, device=DEV)   # noqa: E731
    sc, sh, mu, ist = vec(), vec(), vec(), vec()
    # reference: statistics folded by the conv launch itself
    s_ref, q_ref = vec(), vec()
    ops.conv_fwd(x, W, C, out=out, bn_stats=(s_ref, q_ref))
    s0, q0 = vec(), vec()
    ops.conv_fwd(x, W, C, out=out, bn_stats=(s0, q0), defer_fold=True)
    z = out.clone()
    with pytest.raises(ops.AdpError):   # another statistics launch while the fold is pending
        ops.conv_fwd(x, W, C, out=out, bn_stats=(vec(), vec()))
    with pytest.raises(ops.AdpError):   # a BN-backward reduction while the fold is pending
        ops.bn_bwd_reduce(z, z, sc, sh, mu, ist, vec(), vec())
    with pytest.raises(ops.AdpError):   # a finalize for another sum vector
        ops.bn_finalize(N * H * 32, vec(), q0, gamma, beta, 1e-5, 0.1, sc, sh, mu, ist, fold=True)
    ops.bn_finalize(N * H * 32, s0, q0, gamma, beta, 1e-5, 0.1, sc, sh, mu, ist, fold=True)
    torch.cuda.synchronize()
    torch.testing.assert_close(s0, s_ref, rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(q0, q_ref, rtol=1e-5, atol=1e-3)
    with pytest.raises(ops.AdpError):   # nothing pending any more
        ops.bn_finalize(N * H * 32, s0, q0, gamma, beta, 1e-5, 0.1, sc, sh, mu, ist, fold=True)
    ops.conv_fwd(x, W, C, out=out, bn_stats=(vec(), vec()))   # the replicas are usable again
    torch.cuda.synchronize()
    # a deferred fold that never reaches its finalize (an error between the two): adp_bn_fold_reset drops the
    # record and re-zeroes the replicas, so the next statistics launch runs and its sums are not polluted
    ops.conv_fwd(x, W, C, out=out, bn_stats=(vec(), vec()), defer_fold=True)
    with pytest.raises(ops.AdpError):
        ops.conv_fwd(x, W, C, out=out, bn_stats=(vec(), vec()))
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):   # a reset on another stream leaves the pending fold alone (not its caller's)
        ops.bn_fold_reset()
    with pytest.raises(ops.AdpError):
        ops.conv_fwd(x, W, C, out=out, bn_stats=(vec(), vec()))
    ops.bn_fold_reset()
    ops.bn_fold_reset()   # nothing pending: a no-op
    s1, q1 = vec(), vec()
    ops.conv_fwd(x, W, C, out=out, bn_stats=(s1, q1))
    torch.cuda.synchronize()
    torch.testing.assert_close(s1, s_ref, rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(q1, q_ref, rtol=1e-5, atol=1e-3)


F32_TAP_CASES = [
    # name, N, S, cin_parts, cout, dil, up, mode
    ("plain_relu_bias", 2, 24, [64], 96, 1, False, "plain"),
    ("dil4_concat", 1, 20, [32, 64], 64, 4, False, "plain"),
    ("up_stats", 2, 8, [96], 64, 1, True, "stats"),
    ("addend_mask", 2, 16, [64], 64, 2, False, "addmask"),
    ("split_mask2", 1, 16, [64], 96, 1, False, "split"),
    ("bnr", 2, 16, [192], 64, 1, False, "bnr"),
    ("convt", 2, 8, [128], 64, 1, False, "convt"),
]


@pytest.mark.parametrize("case", F32_TAP_CASES, ids=[c[0] for c in F32_TAP_CASES])
def test_f32_tap_kernel_matches_generic(case):
    """The f32 form of the LDS-DMA tap kernel (32-channel K steps, exact v_mfma_f32_16x16x4_f32; every 32-channel
    K step inside one tap) against the register-staged f32 kernel (option f32_tap=0) on the same operands, for
    each epilogue mode it takes: bias + ReLU, BatchNorm statistics, addend + mask, channel-split store with mask2,
    the fused BatchNorm-backward reduction, and the ConvTranspose pixel-shuffle store."""
    name, N, S, parts, cout, dil, up, mode = case
    g = torch.Generator().manual_seed(len(name))
    dt = torch.float32
    l = Dense("t", parts, cout, dil=dil, up=up, transpose=mode == "convt", cpad=32)
    srcs = [torch.randn(N, S, S, cs, generator=g).to(DEV) for cs in l.cin_s]
    W = (torch.randn(l.Npad, l.Kpad, generator=g) * (1.0 / np.sqrt(l.K))).to(DEV)
    So = 2 * S if up else S
    bias = torch.randn(l.cout_s, generator=g).to(DEV)
    res = []
    for tap in (1, 0):
        ops.set_option("f32_tap", tap)
        try:
            kw = {}
            if mode == "convt":
                out = torch.zeros(N, 2 * S, 2 * S, l.cout_s, device=DEV)
                ops.conv_fwd(srcs[0], W, l.Nout, out=out, bias=bias, kh=1, kw=1, pad=0, out_mode=1, shuffle_c=l.cout_s)
                extra = ()
            else:
                out = torch.zeros(N, So, So, l.cout_s, device=DEV)
                if mode == "plain":
                    kw = dict(bias=torch.linspace(-0.5, 0.5, l.cout_s, device=DEV), relu=True)
                if mode == "stats":
                    s1, s2 = torch.zeros(l.cout_s, device=DEV), torch.zeros(l.cout_s, device=DEV)
                    kw = dict(bn_stats=(s1, s2))
                if mode == "addmask":
                    ga = torch.Generator().manual_seed(3)
                    kw = dict(addend=torch.randn(out.shape, generator=ga).to(DEV),
                              mask=torch.randn(out.shape, generator=ga).to(DEV), mask_scale=1.4)
                if mode == "bnr":
                    gz = torch.Generator().manual_seed(4)
                    z = torch.randn(out.shape, generator=gz).to(DEV)
                    vec = lambda: (torch.rand(l.cout_s, generator=gz) + 0.5).to(DEV)   # noqa: E731
                    dg, db = torch.zeros(l.cout_s, device=DEV), torch.zeros(l.cout_s, device=DEV)
                    kw = dict(bn_reduce=(z, vec(), vec() - 1.0, vec() - 1.0, vec(), dg, db))
                if mode == "split":
                    c0 = 64
                    out = torch.zeros(N, So, So, c0, device=DEV)
                    out2 = torch.zeros(N, So, So, l.cout_s - c0, device=DEV)
                    m2 = torch.randn(out2.shape, generator=torch.Generator().manual_seed(6)).to(DEV)
                    kw = dict(out_mode=2, out2=out2, split_c=c0, mask2=m2, mask2_scale=0.7)
                ops.conv_fwd(srcs[0], W, l.Nout, out=out, srcB=srcs[1] if len(srcs) > 1 else None, up=up, dil=dil,
                             **kw)
                extra = tuple(v for k, v in kw.items() if k in ("out2",)) + \
                    (kw["bn_stats"] if "bn_stats" in kw else ()) + ((kw["bn_reduce"][5], kw["bn_reduce"][6])
                                                                  if "bn_reduce" in kw else ())
            torch.cuda.synchronize()
            kname = _lib.lib().adp_last_kernel().decode()
        finally:
            ops.set_option("f32_tap", None)
        assert kname.startswith("igemm_fwd_tap64_kernel") == bool(tap) and kname.endswith("true, -1>") == bool(tap), kname
        res.append([out.clone()] + [e.clone() for e in extra])
    for a, b in zip(*res):
        assert relerr(a, b) < 1e-5, (name, relerr(a, b))


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("epi", ["bias_relu", "mask_addend", "accum", "stats", "bnr"])
@pytest.mark.parametrize("dil", [1, 4])
@pytest.mark.parametrize("hw", [32, 64])
def test_tap64_split_k(dt, epi, dil, hw):
    """Split-K on the tap64 kernel (round 6, option tap64_ksplit): a launch whose tiles fill under a
    quarter of the CUs -- the 32^2 bottleneck of BASELINE configs[0] (adipose_v3 at 256^2: M = 2048) -- runs several
    blocks per tile over contiguous K ranges; the tile's last block sums the partials in split order and runs the
    epilogue. Against the oracle conv (plain product) and against the unsplit launch (every epilogue: bias + ReLU,
    mask + addend, f32 accumulate, BatchNorm statistics, the BN-backward reduction), and two runs give the same bits.
    hw 64: the f32 64^2 x 192 layers of configs[0] -- 96 tiles, more than one 64-counter claim slot held before the
    slots grew to 512 counters."""
    if dt == "f32" and epi == "bnr":
        pytest.skip("the BN-backward reduction epilogue is a bf16 data-gradient form")
    if hw == 64 and dt == "bf16":
        pytest.skip("the 96-tile case is an f32 shape")
    torch_dt = torch.float32 if dt == "f32" else torch.bfloat16
    N, H, W_ = 2, hw, hw
    cin = cout = (352 if hw == 32 else 192) if dt == "f32" else 384
    g = torch.Generator().manual_seed(71)
    x = torch.randn(N, H, W_, cin, generator=g)
    Wm = torch.randn(cout, 9 * cin, generator=g) * (1.0 / math.sqrt(9 * cin))
    npad = (cout + 63) // 64 * 64   # (the packed layout's rows: a multiple of 64, the pad rows zero)
    xd, Wd = x.to(DEV, torch_dt), torch.cat([Wm, torch.zeros(npad - cout, 9 * cin)]).to(DEV, torch_dt)
    bias = torch.randn(cout, generator=g).to(DEV)
    mask = torch.randn(N, H, W_, cout, generator=g).to(DEV, torch_dt)
    addend = torch.randn(N, H, W_, cout, generator=g).to(DEV, torch_dt)
    z = torch.randn(N, H, W_, cout, generator=g).to(DEV, torch.bfloat16)
    vec = [(torch.rand(cout, generator=g) + 0.5).to(DEV) for _ in range(4)]

    def run(split):
        ops.set_option("tap64_ksplit", split)   # (the module fixture turns it off around every test)
        try:
            out = torch.zeros(N, H, W_, cout, dtype=torch_dt, device=DEV)
            side = [torch.zeros(cout, device=DEV), torch.zeros(cout, device=DEV)]
            acc = torch.ones(N, H, W_, cout, device=DEV)
            kw = dict(out=out, dil=dil)
            if epi == "bias_relu":
                ops.conv_fwd(xd, Wd, cout, bias=bias, relu=True, **kw)
            elif epi == "mask_addend":
                ops.conv_fwd(xd, Wd, cout, mask=mask, addend=addend, **kw)
            elif epi == "accum":
                ops.conv_fwd(xd, Wd, cout, accum=acc, **kw)
            elif epi == "stats":
                ops.conv_fwd(xd, Wd, cout, bias=bias, bn_stats=(side[0], side[1]), **kw)
            else:
                ops.conv_fwd(xd, Wd, cout, bn_reduce=(z, vec[0], vec[1] - 1.0, vec[2] - 1.0, vec[3], side[1], side[0]),
                             **kw)
            ks = ops.get_option("tap64_ksplit_last")
            kn = _lib.lib().adp_last_kernel().decode()
            torch.cuda.synchronize()
            return out.float().cpu(), acc.cpu(), [t.cpu() for t in side], ks, kn
        finally:
            ops.set_option("tap64_ksplit", 0)

    from adipose_amd import _lib
    o1, a1, s1, ks1, kn1 = run(1)
    o1b, a1b, s1b, _, _ = run(1)
    o0, a0, s0, ks0, kn0 = run(0)
    assert kn1.startswith("igemm_fwd_tap64_kernel") and kn0 == kn1, (kn0, kn1)
    assert ks1 >= 2 and ks0 == 0, (ks1, ks0)
    assert torch.equal(o1, o1b) and torch.equal(a1, a1b) and all(torch.equal(p, q) for p, q in zip(s1, s1b))
    tol = 1e-5 if dt == "f32" else 2e-2   # (bf16: the stored outputs round the two f32 sums; a flip is one bf16 ulp)
    assert relerr(o1, o0) < tol and relerr(a1, a0) < tol   # (bf16 accum: the rounded output is what it adds)
    for p, q in zip(s1, s0):
        assert relerr(p, q) < (1e-5 if dt == "f32" else 1e-2)
    if epi == "bias_relu" and dt == "f32":   # the oracle: 'same' dilated conv of the packed weights
        wk = Wm.view(cout, 3, 3, cin).permute(0, 3, 1, 2)
        ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), wk, bias.cpu(), padding=dil, dilation=dil).relu()
        assert relerr(o1, ref.permute(0, 2, 3, 1)) < 1e-4
