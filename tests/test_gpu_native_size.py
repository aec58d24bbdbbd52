"""adipose_v3 at the reference's own tile size, and its dilated bottleneck with taps inside the image.

The reference hard-codes S = 1024 (Segmentation/train_adipose_unet_v3.py:664-665), so its bottleneck runs at
128^2 with dilations 2, 4, 8, 16, 32 (:681-688). At S <= 256 every off-centre tap of the dilation-32 conv falls
in the zero padding, so only these tests check a dilation-16/32 gather whose taps land inside the image:

  * op level: forward, data gradient (plain and with the network's addend + ReLU-mask epilogue) and weight
    gradient of a 352 -> 352 dilated 3x3 conv at S = 48 (d = 16), 96 (d = 32) and the bottleneck's own
    B = 2 x 128^2 (d = 16, 32), f32 and bf16, against the CPU fp32 oracle (oracle/torch_ref.py). The bf16 launches
    at 128^2 are checked to run on the kernel forms the 1024^2 network routes the bottleneck to (the persistent
    gather-form forward, tap64 data and weight gradients), the f32 ones on the f32 tap kernel.
  * network: adipose_v3 f32, S = 1024, B = 1 (one reference training tile, OHEM + deep supervision loss):
    forward <= 1e-4 and Dice / IoU of the thresholded maps <= 1e-4 vs the fp32 oracle, per-layer gradients
    <= 1e-3 relative vs the same oracle evaluated in float64. (At 1024^2 a bias gradient is a sum over 2^20 pixels
    with cancellation: the fp32 CPU oracle's own up1_conv3 bias gradient is 2.8e-3 off its float64 value, so the
    gradients are gated against the float64 evaluation, and the fp32 oracle's own error is reported beside.)
    The same step in bf16 with the report-style gates of tests/test_gpu_network.py.

The network oracle is parity unpinned vs TF 2.13."""
import numpy as np
import pytest
import torch

from adipose_amd import _lib, ops
from adipose_amd.data import synthetic_batch, to_gray
from adipose_amd.metrics import calculate_pixel_metrics
from adipose_amd.nets import AdiposeV3Net, Dense
from adipose_amd.trainer import LossConfig, Trainer
from oracle import numpy_ref as NR
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def cos(a, b):
    a, b = torch.as_tensor(a).flatten().double(), torch.as_tensor(b).flatten().double()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


def relerr(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-12)


def nhwc_pad(x, cs, dt):
    N, H, W, C = x.shape
    out = torch.zeros((N, H, W, cs), dtype=dt, device=DEV)
    out[..., :C] = x.to(DEV, dt)
    return out


def rb(t, dt):
    return t.to(dt).float() if dt == torch.bfloat16 else t


def kname():
    return _lib.lib().adp_last_kernel().decode()


# ------------------------------------------------------------------------------ dilated bottleneck ops
DIL_CASES = [
    # N, S, dil: every case has off-centre taps inside the image (S > dil)
    (1, 48, 16),
    (1, 96, 32),
    (2, 128, 16),    # the 1024^2 network's bottleneck, B = 2 as the reference trains
    (2, 128, 32),
]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("case", DIL_CASES, ids=[f"S{c[1]}_d{c[2]}" for c in DIL_CASES])
def test_dilated_bottleneck_taps_inside(case, dt):
    N, S, dil = case
    C = 352
    cpad = 32 if dt == torch.float32 else 64          # the network's channel granule per dtype (nets.py)
    l = Dense("dilate", [C], C, dil=dil, cpad=cpad)
    g = torch.Generator().manual_seed(100 + dil + S)
    x = rb(torch.randn(N, S, S, C, generator=g), dt)
    kern = rb(torch.randn(3, 3, C, C, generator=g) * (1.0 / np.sqrt(9 * C)), dt)
    bias = torch.randn(C, generator=g) * 0.1
    dZ = rb(torch.randn(N, S, S, C, generator=g), dt)
    addend = rb(torch.randn(N, S, S, C, generator=g), dt)
    mask_src = torch.randn(N, S, S, C, generator=g).clamp_min(0.0)     # a ReLU output: mask = (m > 0)
    tol = 1e-4 if dt == torch.float32 else 2e-2
    names = {}

    # the oracle's taps at distance dil must reach real pixels: guard the premise of the test
    assert S > dil

    # forward (bias + ReLU)
    xr = x.clone().requires_grad_(True)
    kr = kern.clone().requires_grad_(True)
    br = bias.clone().requires_grad_(True)
    y = R.conv2d_same(xr, kr, br, dilation=dil, relu=False)
    (y * dZ).sum().backward()
    ref_fwd = y.detach().clamp_min(0.0)
    W = torch.from_numpy(l.keras_to_packed(kern.numpy())).to(DEV).to(dt).contiguous()
    b = torch.zeros(l.cout_s, device=DEV)
    b[:C] = bias.to(DEV)
    xd = nhwc_pad(x, l.Cin_s, dt)
    out = torch.zeros((N, S, S, l.cout_s), dtype=dt, device=DEV)
    ops.conv_fwd(xd, W, l.Nout, out=out, bias=b, dil=dil, relu=True)
    torch.cuda.synchronize()
    names["fwd"] = kname()
    assert relerr(out[..., :C].float(), ref_fwd) < tol, ("fwd", relerr(out[..., :C].float(), ref_fwd))
    assert out[..., C:].abs().max().item() == 0.0 if l.cout_s > C else True

    # an off-centre-only check: the same conv with the centre tap zeroed still matches (so the inside taps
    # carry real weight, not just the centre)
    k_off = kern.clone()
    k_off[1, 1] = 0.0
    W_off = torch.from_numpy(l.keras_to_packed(k_off.numpy())).to(DEV).to(dt).contiguous()
    out_off = torch.zeros_like(out)
    ops.conv_fwd(xd, W_off, l.Nout, out=out_off, dil=dil, relu=False)
    torch.cuda.synchronize()
    ref_off = R.conv2d_same(x, k_off, None, dilation=dil, relu=False)
    assert ref_off.abs().max().item() > 0.1
    assert relerr(out_off[..., :C].float(), ref_off) < tol

    # weight + bias gradient
    dZd = nhwc_pad(dZ, l.cout_s, dt)
    dW = torch.zeros((l.Npad, l.Kpad), device=DEV)
    dB = torch.zeros(l.cout_s, device=DEV)
    ops.conv_wgrad(xd, dZd, dW, l.Nout, dB=dB, dil=dil)
    torch.cuda.synchronize()
    names["wgrad"] = kname()
    dW_k = torch.from_numpy(l.packed_to_keras(dW.cpu().numpy()))
    assert relerr(dW_k, kr.grad) < tol, ("wgrad", relerr(dW_k, kr.grad))
    assert relerr(dB[:C], br.grad) < tol

    # data gradient, plain
    Wm = torch.from_numpy(l.keras_to_packed(kern.numpy())).to(DEV)
    Wd = torch.zeros((l.dNpad, l.dKpad), dtype=dt, device=DEV)
    ops.pack_weights(Wm, Wd, 1, taps=9, cin_s=l.Cin_s, nout=l.cout_s)
    dX = torch.zeros((N, S, S, l.Cin_s), dtype=dt, device=DEV)
    ops.conv_fwd(dZd, Wd, l.Cin_s, out=dX, dil=dil)
    torch.cuda.synchronize()
    names["dgrad"] = kname()
    assert relerr(dX[..., :C].float(), xr.grad) < tol, ("dgrad", relerr(dX[..., :C].float(), xr.grad))

    # data gradient with the bottleneck's epilogue: dX = (conv(dZ) + addend) * (m > 0)  (nets.AdiposeV3Net)
    add_d = nhwc_pad(addend, l.Cin_s, dt)
    mask_d = nhwc_pad(mask_src, l.Cin_s, dt)
    dX2 = torch.zeros_like(dX)
    ops.conv_fwd(dZd, Wd, l.Cin_s, out=dX2, dil=dil, addend=add_d, mask=mask_d)
    torch.cuda.synchronize()
    names["dgrad_addend_mask"] = kname()
    ref2 = (xr.grad + addend) * (rb(mask_src, dt) > 0).float()
    assert relerr(dX2[..., :C].float(), ref2) < tol, ("dgrad+epi", relerr(dX2[..., :C].float(), ref2))

    print(f"S={S} d={dil} {dt}: {names}")
    if N == 2 and S == 128:
        # the kernel forms the 1024^2 network's bottleneck runs on (tools/launch_map.py)
        if dt == torch.bfloat16:
            assert names["fwd"].startswith("igemm_fwd_tap64p_kernel"), names
            assert names["dgrad_addend_mask"].startswith("igemm_fwd_tap64_kernel"), names
            assert names["wgrad"].startswith("igemm_wgrad_tap64_kernel"), names
        else:
            assert "tap64" in names["fwd"] and "tap64" in names["dgrad_addend_mask"], names


# ----------------------------------------------------------------------- network at the native size
@pytest.fixture(scope="module")
def native_case():
    """One 1024^2 reference training tile: synthetic histology (seed 865), BT.601 gray, z-scored, the
    reference topology's weights as oracle/torch_ref.adipose_v3_keras_weights draws them (glorot-uniform kernels,
    N(0, 0.01) biases -- non-zero, so the bias paths are exercised, where Keras would start from zeros), oracle
    forward + OHEM/DS loss
    gradients on the CPU in f32."""
    B, S = 1, 1024
    xs, ys = synthetic_batch(B, S, channels=3, seed=865)
    g = to_gray(xs).astype(np.float32)
    x = torch.from_numpy((g - g.mean()) / (g.std() + 1e-10))
    y = torch.from_numpy(ys.astype(np.float32))
    w = R.adipose_v3_keras_weights(seed=865)
    W = {k: [torch.tensor(v[0], requires_grad=True), torch.tensor(v[1], requires_grad=True)] for k, v in w.items()}
    ref = R.adipose_v3_forward(x, W)
    loss = R.ds_total_loss(y, ref)
    loss.backward()
    W64 = {k: [torch.tensor(v[0], dtype=torch.float64, requires_grad=True),
               torch.tensor(v[1], dtype=torch.float64, requires_grad=True)] for k, v in w.items()}
    R.ds_total_loss(y.double(), R.adipose_v3_forward(x.double(), W64)).backward()
    return dict(B=B, S=S, x=x, y=y, ys=ys, w=w, W=W, W64=W64, ref={k: v.detach() for k, v in ref.items()},
                loss=loss.item())


def run_native(case, dtype):
    B, S = case["B"], case["S"]
    net = AdiposeV3Net(B, S, dtype=dtype, device=DEV)
    net.set_weights(case["w"])
    tr = Trainer(net, LossConfig())          # reference defaults: OHEM main + 0.4 / 0.3 deep supervision
    ops.prep_input(case["x"].to(DEV), net.acts(B)["x"], mean=0.0, std=1.0)
    outs = net.forward(B, train=False)       # dropout off: TF's RNG stream is not reproducible (§8a7)
    grads = tr.loss_and_grads(outs, case["y"].to(DEV))
    ops.fill(net.ps.grad, 0.0)
    net.backward(grads)
    torch.cuda.synchronize()
    outs = {k: v.float().cpu() for k, v in outs.items()}
    layer_grads = {n: net.get_layer_grads(n) for n in case["W"]}
    met = tr.read_metrics()
    del net, tr
    torch.cuda.empty_cache()
    return outs, layer_grads, met


def test_adipose_v3_1024_f32_vs_oracle(native_case):
    c = native_case
    outs, lg, met = run_native(c, "f32")
    for k in ("main_out", "aux_out1", "aux_out2"):
        err = (outs[k] - c["ref"][k]).abs().max().item()
        assert err < 1e-4, (k, err)
    assert abs(met["loss"] - c["loss"]) < 1e-4 * max(1.0, abs(c["loss"]))
    bad, report = [], []
    for name, (k, b) in c["W64"].items():
        gk, gb = lg[name]
        rk, rbb = relerr(gk, k.grad), relerr(gb, b.grad)
        k32, b32 = c["W"][name]
        report.append((name, rk, rbb, relerr(k32.grad, k.grad), relerr(b32.grad, b.grad)))
        if not (rk < 1e-3 and rbb < 1e-3):
            bad.append(report[-1])
    print("layer, GPU f32 vs f64 (kernel, bias), CPU f32 oracle vs f64 (kernel, bias):")
    for r in report:
        print("  %-14s %.2e %.2e   %.2e %.2e" % r)
    assert not bad, bad
    pg, pr = outs["main_out"][0].numpy(), c["ref"]["main_out"][0].numpy()
    for truth in (c["ys"][0].astype(np.float32), (pr > 0.5).astype(np.float32)):
        mg, mr = calculate_pixel_metrics(pg, truth), NR.calculate_pixel_metrics(pr, truth)
        assert abs(mg["dice_score"] - mr["dice_score"]) <= 1e-4, (mg["dice_score"], mr["dice_score"])
        assert abs(mg["jaccard_index"] - mr["jaccard_index"]) <= 1e-4


def test_adipose_v3_1024_bf16_vs_oracle(native_case):
    """bf16 is a reported precision: forward within 2e-2, per-layer gradient cosine >= 0.99,
    the same gates tests/test_gpu_network.py applies at 64^2 / 128^2."""
    c = native_case
    outs, lg, met = run_native(c, "bf16")
    for k in ("main_out", "aux_out1", "aux_out2"):
        d = (outs[k] - c["ref"][k]).abs()
        assert d.max().item() < 2e-2 and d.mean().item() < 2e-3, (k, d.max().item(), d.mean().item())
    assert abs(met["loss"] - c["loss"]) < 2e-2 * max(1.0, abs(c["loss"]))
    bad = [(n, cos(lg[n][0], k.grad)) for n, (k, _) in c["W"].items() if cos(lg[n][0], k.grad) <= 0.99]
    assert not bad, bad
    pg, pr = outs["main_out"][0].numpy(), c["ref"]["main_out"][0].numpy()
    truth = c["ys"][0].astype(np.float32)
    assert abs(calculate_pixel_metrics(pg, truth)["dice_score"]
               - NR.calculate_pixel_metrics(pr, truth)["dice_score"]) <= 1e-2
