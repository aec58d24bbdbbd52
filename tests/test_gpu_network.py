"""Whole-network parity of the HIP engine against the CPU fp32 oracle (oracle/torch_ref.py).

adipose_v3 (reference topology, train_adipose_unet_v3.py:660-758) and unet_bn (north-star preset)
on identical weights and seeded inputs:
  * f32: forward probabilities within 1e-4 abs; per-layer parameter gradients of the reference loss
    (OHEM main + 0.4/0.3 aux BCE+Dice, dropout off) within 1e-3 relative; Dice/IoU of the thresholded
    predictions within 1e-4 (BASELINE.json north_star acceptance).
  * bf16: reported-only precision — forward within 2e-2 abs, gradients cosine >= 0.99.
"""
import numpy as np
import pytest
import torch

from adipose_amd import ops
from adipose_amd.nets import AdiposeV3Net, UNetBN
from adipose_amd.trainer import LossConfig, Trainer
from oracle import numpy_ref as NR
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def synth_batch(B, S, C=None, seed=3):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn((B, S, S) if C is None else (B, S, S, C), generator=g)
    yy, xx = torch.meshgrid(torch.arange(S), torch.arange(S), indexing="ij")
    y = torch.zeros(B, S, S)
    for b in range(B):
        cy, cx = torch.randint(0, S, (2,), generator=g)
        y[b] = (((yy - cy) ** 2 + (xx - cx) ** 2) < (S / 3) ** 2).float()
    return x, y


def cos(a, b):
    a, b = a.flatten().double(), b.flatten().double()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


@pytest.fixture(scope="module")
def adipose_weights():
    return R.adipose_v3_keras_weights(seed=865)


def build_adipose(dtype, weights, B=2, S=64, cpad=None):
    net = AdiposeV3Net(B, S, dtype=dtype, device=DEV, cpad=cpad)
    net.set_weights(weights)
    return net


# bf16 default: channels stored 64-granular (44 -> 64, 88 -> 128, ...: tap64 / halo kernels);
# cpad=8 keeps the 48/88/176/352 strides of the generic LDS-DMA kernels
@pytest.mark.parametrize("dtype,cpad,S", [("f32", None, 64), ("bf16", None, 64), ("bf16", None, 128),
                                          ("bf16", 8, 64), ("bf16", (8, 8, 64, 64), 64)])
def test_adipose_forward(dtype, cpad, S, adipose_weights):
    B = 2
    x, _ = synth_batch(B, S)
    net = build_adipose(dtype, adipose_weights, B, S, cpad)
    a = net.acts(B)
    ops.prep_input(x.to(DEV), a["x"], mean=0.0, std=1.0)
    outs = net.forward(B, train=False)
    ref = R.adipose_v3_forward(x, adipose_weights)
    tol = 1e-4 if dtype == "f32" else 2e-2
    for k in ("main_out", "aux_out1", "aux_out2"):
        err = (outs[k].cpu() - ref[k]).abs().max().item()
        assert err < tol, (k, err)
    if dtype == "f32":
        # thresholded Dice/IoU parity (calculate_pixel_metrics, full_evaluation_enhanced.py:721-785)
        for b in range(B):
            truth = (ref["main_out"][b] > 0.5).numpy().astype(np.float32)
            m_gpu = NR.calculate_pixel_metrics(outs["main_out"][b].cpu().numpy(), truth)
            m_ref = NR.calculate_pixel_metrics(ref["main_out"][b].numpy(), truth)
            assert abs(m_gpu["dice_score"] - m_ref["dice_score"]) < 1e-4
            assert abs(m_gpu["jaccard_index"] - m_ref["jaccard_index"]) < 1e-4


@pytest.mark.parametrize("dtype,cpad,S,hard_mining", [("f32", None, 64, True), ("f32", None, 64, False),
                                                      ("bf16", None, 64, True), ("bf16", None, 64, False),
                                                      ("bf16", None, 128, True), ("bf16", 8, 64, True),
                                                      ("bf16", (8, 8, 64, 64), 64, True)])
def test_adipose_grads(dtype, cpad, S, hard_mining, adipose_weights):
    B = 2
    x, y = synth_batch(B, S, seed=4)
    net = build_adipose(dtype, adipose_weights, B, S, cpad)
    tr = Trainer(net, LossConfig(use_hard_mining=hard_mining))
    a = net.acts(B)
    ops.prep_input(x.to(DEV), a["x"], mean=0.0, std=1.0)
    outs = net.forward(B, train=False)
    grads = tr.loss_and_grads(outs, y.to(DEV))
    ops.fill(net.ps.grad, 0.0)
    net.backward(grads)
    torch.cuda.synchronize()
    # oracle
    W = {k: [torch.tensor(v[0], requires_grad=True), torch.tensor(v[1], requires_grad=True)]
         for k, v in adipose_weights.items()}
    ref_out = R.adipose_v3_forward(x, {k: v for k, v in W.items()})
    loss = R.ds_total_loss(y, ref_out, use_hard_mining=hard_mining)
    loss.backward()
    met = tr.read_metrics()
    assert abs(met["loss"] - loss.item()) < (1e-4 if dtype == "f32" else 2e-2) * max(1, abs(loss.item()))
    for name, (k, b) in W.items():
        gk, gb = net.get_layer_grads(name)
        if dtype == "f32":
            rk = (torch.as_tensor(gk) - k.grad).abs().max().item() / max(k.grad.abs().max().item(), 1e-12)
            rb = (torch.as_tensor(gb) - b.grad).abs().max().item() / max(b.grad.abs().max().item(), 1e-12)
            assert rk < 1e-3 and rb < 1e-3, (name, rk, rb)
        else:
            assert cos(torch.as_tensor(gk), k.grad) > 0.99, name


def test_adipose_f32_zero_tail_skip_is_exact(adipose_weights):
    """f32 adipose_v3 (44-channel level-0 layers in 64-channel strides): the tap kernel's zero-tail forms (option
    f32_ztail, default on; the real channel counts passed by nets.py) skip the products with the zero pad weights --
    forward probabilities bit-identical to the launches that multiply them, parameter gradients to the f32 weight-
    gradient atomics' run-to-run order (each zero-tail launch is bit-exact: test_gpu_ops.py::test_f32_zero_tail_forms)."""
    from adipose_amd import _lib
    B, S = 2, 64
    x, y = synth_batch(B, S, seed=4)
    res = []
    for zt in (0, 1):
        ops.set_option("f32_ztail", zt)
        ops.set_option("wgrad_f32_zt", zt)
        try:
            net = build_adipose("f32", adipose_weights, B, S)
            tr = Trainer(net, LossConfig(use_hard_mining=True))
            a = net.acts(B)
            ops.prep_input(x.to(DEV), a["x"], mean=0.0, std=1.0)
            outs = net.forward(B, train=False)
            grads = tr.loss_and_grads(outs, y.to(DEV))
            ops.fill(net.ps.grad, 0.0)
            net.backward(grads)
            torch.cuda.synchronize()
        finally:
            ops.set_option("f32_ztail", None)
            ops.set_option("wgrad_f32_zt", None)
        o = outs if isinstance(outs, dict) else dict(enumerate(outs))
        res.append(({k: v.clone() for k, v in o.items() if torch.is_tensor(v)},
                    {n: net.get_layer_grads(n) for n in adipose_weights}))
    assert res[0][0].keys() == res[1][0].keys() and res[0][0]
    for k in res[0][0]:
        assert torch.equal(res[0][0][k], res[1][0][k]), k
    # the f32 weight gradients add per-block partials with f32 atomics in the order blocks finish (4-7e-7 between
    # identical runs, profiles/r04e_f32_step_determinism.txt): gradients to 1e-5 of each layer's largest element
    for n in adipose_weights:
        for g0, g1 in zip(res[0][1][n], res[1][1][n]):
            g0, g1 = torch.as_tensor(g0), torch.as_tensor(g1)
            assert (g0 - g1).abs().max().item() <= 1e-5 * max(g0.abs().max().item(), 1e-12), n


def test_adipose_frozen_encoder_grads(adipose_weights):
    """Phase 1: encoder frozen -> encoder grads exactly zero, decoder grads unchanged."""
    B, S = 2, 64
    x, y = synth_batch(B, S, seed=6)
    net = build_adipose("f32", adipose_weights, B, S)
    tr = Trainer(net, LossConfig())
    a = net.acts(B)
    ops.prep_input(x.to(DEV), a["x"], mean=0.0, std=1.0)
    outs = net.forward(B, train=False)
    grads = tr.loss_and_grads(outs, y.to(DEV))
    ops.fill(net.ps.grad, 0.0)
    net.backward(grads)
    full = {n: net.get_layer_grads(n) for n in ("up1_conv2", "dilate1", "down1_conv1")}
    tr.set_frozen(AdiposeV3Net.ENCODER)
    outs = net.forward(B, train=False)
    grads = tr.loss_and_grads(outs, y.to(DEV))
    ops.fill(net.ps.grad, 0.0)
    net.backward(grads)
    assert np.abs(net.get_layer_grads("down1_conv1")[0]).max() == 0.0
    for n in ("up1_conv2", "dilate1"):
        np.testing.assert_allclose(net.get_layer_grads(n)[0], full[n][0], rtol=1e-5, atol=1e-9)


def test_adipose_train_step_adam(adipose_weights):
    """Two full train steps (f32, dropout off) vs oracle autograd + Keras Adam."""
    B, S = 2, 32
    x, y = synth_batch(B, S, seed=8)
    net = build_adipose("f32", adipose_weights, B, S)
    net.dropout_rate = 0.0
    tr = Trainer(net, LossConfig(), lr=1e-3)
    W = {k: [torch.tensor(v[0], requires_grad=True), torch.tensor(v[1], requires_grad=True)]
         for k, v in adipose_weights.items()}
    params = [p for v in W.values() for p in v]
    opt = R.KerasAdam(params, lr=1e-3)
    for _ in range(2):
        tr.train_step(x.to(DEV), y.to(DEV))
        for p in params:
            p.grad = None
        R.ds_total_loss(y, R.adipose_v3_forward(x, W)).backward()
        opt.step([p.grad for p in params])
    torch.cuda.synchronize()
    for name, (k, b) in W.items():
        gk, gb = net.get_layer_weights(name)
        assert (torch.as_tensor(gk) - k.detach()).abs().max().item() < 1e-4, name


# f32 parity needs inputs whose BatchNorm pre-activations all keep a margin from the ReLU kink: the GPU
# sums BatchNorm statistics in a run-dependent order, so an element within float rounding of 0 takes
# either subgradient, and BatchNorm-backward spreads that one element over its whole channel (data seed
# 9 has one at 1.1e-6 and failed 1 run in 6). Seed 33 keeps every element >= 1.8e-5 away.
F32_SEED, F32_MARGIN = 33, 1e-5


def _unet_bn_case(dtype, base, S, L=3, B=2):
    w = R.unet_bn_keras_weights(levels=L, base=base, in_ch=3, seed=5)
    x, y = synth_batch(B, S, C=3, seed=F32_SEED if dtype == "f32" else 9)
    W = {k: [torch.tensor(v, requires_grad=True) for v in vs] for k, vs in w.items()}
    rec = []
    p = R.unet_bn_forward(x, W, levels=L, record=rec)
    p.retain_grad()
    loss = R.combined_loss_standard(y, p)
    loss.backward()
    if dtype == "f32":
        m = min(r["margin"] for r in rec)
        assert m >= F32_MARGIN, f"ill-conditioned f32 case: a BatchNorm pre-activation {m:.2e} from the ReLU kink"
    return w, x, y, W, p, loss, rec


def _unet_bn_step(net, tr, x, y, B, *, backward=True):
    a = net.acts(B)
    ops.prep_input(x.to(DEV), a["x"], mean=0.0, std=1.0)
    outs = net.forward(B, train=True)
    grads = tr.loss_and_grads(outs, y.to(DEV))
    if backward:
        ops.fill(net.ps.grad, 0.0)
        net.backward(grads)
    torch.cuda.synchronize()
    return outs, grads


def _grad_errors(net, W, dtype):
    bad = []
    for name, ts in W.items():
        got = net.get_layer_grads(name)
        for si, (gi, t) in enumerate(zip(got, ts)):
            if dtype == "f32":
                r = (torch.as_tensor(gi) - t.grad).abs().max().item() / max(t.grad.abs().max().item(), 1e-12)
                if r >= 2e-3:
                    bad.append((name, si, r))
            else:
                c = cos(torch.as_tensor(gi), t.grad)
                if c <= 0.95:  # bf16 dz storage through BN bwd
                    bad.append((name, si, c))
    return bad


@pytest.mark.parametrize("dtype,base,S", [("f32", 16, 32), ("bf16", 16, 32), ("bf16", 64, 32), ("bf16", 64, 128)])
def test_unet_bn_forward_and_grads(dtype, base, S):
    """base 64 puts every layer but the input conv on the tap64 kernels (fwd, dgrad, wgrad, ConvT,
    concat); S = 128 makes the two upper levels row-aligned (Wo % 64 == 0) for the wgrad gather."""
    B, L = 2, 3
    w, x, y, W, p, loss, _ = _unet_bn_case(dtype, base, S, L, B)
    net = UNetBN(B, S, levels=L, base=base, in_ch=3, dtype=dtype, device=DEV)
    net.set_weights(w)
    tr = Trainer(net, LossConfig(use_hard_mining=False))
    outs, grads = _unet_bn_step(net, tr, x, y, B)
    tol = 1e-4 if dtype == "f32" else 3e-2
    assert (outs["main_out"].cpu() - p.detach()).abs().max().item() < tol
    bad = _grad_errors(net, W, dtype)
    if bad:  # localise: is the loss gradient dL/dp already off, or only the backward pass?
        dp_err = (grads["main_out"].cpu() - p.grad).abs().max().item() / p.grad.abs().max().item()
        met = tr.read_metrics()
        bad.insert(0, ("dL/dp", dp_err, "loss", met["loss"], loss.item()))
    assert not bad, bad


@pytest.mark.parametrize("flag", ["fuse_head_bn", "head_recompute_dA", "fuse_bn_fold", "fuse_bn_wgrad",
                                  "pool_argmax_from_z", "fuse_bn_load"])
def test_unet_bn_fallback_paths_match_default(flag):
    """The alternate schedules nets.UNetBN keeps for A/B runs (each fusion flag off, and the pool backward's
    argmax read from the stored activation instead of recomputed from z) give the default path's outputs and
    gradients (bf16, base 64, so every fused kernel form is the one the bench runs). Since round 4 the BatchNorm
    sums are deterministic (f64 replicas fed fixed-order f32 partials, csrc/common.h) and every fused form computes
    the same f32 partials as its unfused pair, so the outputs are bit-identical (measured: max difference 0 for
    every flag, profiles/r04c_gates.log; round 3 allowed 1.5e-2 and gradient cosines down to 0.98, when f32
    atomics in run order made even two runs of one path differ). Weight gradients within 1e-5 (the fused and unfused
    weight-gradient kernels may sum a block's pixels in another order). Round 5 adds the BatchNorm-ReLU applied on
    load by conv2 of levels 0-1 (fuse_bn_load); the second-stream weight gradients are in the determinism test."""
    B, L, S = 2, 3, 64
    w = R.unet_bn_keras_weights(levels=L, base=64, in_ch=3, seed=5)
    x, y = synth_batch(B, S, C=3, seed=9)
    res = []
    for off in (False, True):
        net = UNetBN(B, S, levels=L, base=64, in_ch=3, dtype="bf16", device=DEV)
        net.set_weights(w)
        if off:
            setattr(net, flag, False)
        tr = Trainer(net, LossConfig(use_hard_mining=False))
        outs, _ = _unet_bn_step(net, tr, x, y, B)
        res.append((outs["main_out"].cpu().clone(), {n: net.get_layer_grads(n) for n in w}))
    (p0, g0), (p1, g1) = res
    d = (p0 - p1).abs()
    cs = {n: min(cos(torch.as_tensor(a), torch.as_tensor(b)) for a, b in zip(g0[n], g1[n])) for n in w}
    print(f"[gate] fallback {flag}: output max {d.max().item():.3e} mean {d.mean().item():.3e}, lowest gradient "
          f"cosine {min(cs.values()):.6f} ({min(cs, key=cs.get)})")
    assert torch.equal(p0, p1), (d.max().item(), d.mean().item())
    for n in w:
        for a, b in zip(g0[n], g1[n]):
            a, b = torch.as_tensor(a), torch.as_tensor(b)
            r = (a - b).abs().max().item() / max(a.abs().max().item(), 1e-30)
            assert r <= 1e-5, (flag, n, r)


@pytest.mark.parametrize("levels,S", [(3, 64), (5, 128)])
def test_unet_bn_bf16_runs_are_deterministic(levels, S):
    """Two identical bf16 training forward + backward passes give bit-identical outputs, BatchNorm statistics and
    data-gradient chains: since round 4 the BatchNorm sums (forward statistics in every conv epilogue and the
    fused BN-backward reductions) are f64 replicas fed f32 partials of a fixed order (csrc/common.h), where f32
    atomics in run-dependent order used to make runs differ by bf16 rounding flips (per-layer gradient cosines down
    to 0.9895: profiles/r03_bf16_bn_nondeterminism.txt). Since round 5 the weight gradients are bit-identical too:
    the halo / input-layer / tap64 weight-gradient kernels write per-block slabs that a fixed-order reduce adds into
    dW (option wgrad_det), where f32 atomics in the order blocks finished used to move the last bits. The third run launches every
    reduction at once (option wgrad_defer = 0) instead of batched at the end of the backward, the fourth puts the
    off-critical-path weight gradients on a second stream (UNetBN.wgrad_side): the same bits."""
    B = 2
    w = R.unet_bn_keras_weights(levels=levels, base=64, in_ch=3, seed=5)
    x, y = synth_batch(B, S, C=3, seed=9)
    net = UNetBN(B, S, levels=levels, base=64, in_ch=3, dtype="bf16", device=DEV)
    net.set_weights(w)
    tr = Trainer(net, LossConfig(use_hard_mining=False))
    runs = []
    for i in range(4):
        ops.set_option("wgrad_defer", 0 if i == 2 else None)
        net.wgrad_side = i == 3
        try:
            outs, _ = _unet_bn_step(net, tr, x, y, B)
        finally:
            ops.set_option("wgrad_defer", None)
            net.wgrad_side = False
        runs.append((outs["main_out"].clone(), {n: [torch.as_tensor(g).clone() for g in net.get_layer_grads(n)]
                                                for n in w}))
    p0, g0 = runs[0]
    for p1, g1 in runs[1:]:
        assert torch.equal(p0, p1), (p0 - p1).abs().max().item()
        for n in w:
            for a, b in zip(g0[n], g1[n]):
                assert torch.equal(a, b), (n, (a - b).abs().max().item() / max(a.abs().max().item(), 1e-30))


def test_unet_bn_repeated_steps_and_double_backward():
    """The per-step statistic arena (BatchNorm sums zeroed once per training forward, the ConvTranspose
    bias-gradient sums once per backward) must not carry anything over: a second training forward +
    backward on the same buffers gives the oracle's gradients again, the running statistics follow
    two momentum updates (PyTorch semantics: unbiased batch variance), and a second backward after
    one forward reproduces the first."""
    B, L, base, S = 2, 3, 16, 32
    w, x, y, W, p, loss, rec = _unet_bn_case("f32", base, S, L, B)
    net = UNetBN(B, S, levels=L, base=base, in_ch=3, dtype="f32", device=DEV)
    net.set_weights(w)
    tr = Trainer(net, LossConfig(use_hard_mining=False))
    for step in range(2):
        outs, _ = _unet_bn_step(net, tr, x, y, B)
        assert (outs["main_out"].cpu() - p.detach()).abs().max().item() < 1e-4, step
        assert not _grad_errors(net, W, "f32"), (step, _grad_errors(net, W, "f32"))
    first = {n: net.get_layer_grads(n) for n in W}
    # double backward after one training forward (loss gradients of the same outputs)
    outs, grads = _unet_bn_step(net, tr, x, y, B, backward=False)
    for _ in range(2):
        ops.fill(net.ps.grad, 0.0)
        net.backward(grads)
        torch.cuda.synchronize()
        for n in W:
            for g1, g0 in zip(net.get_layer_grads(n), first[n]):
                np.testing.assert_allclose(g1, g0, rtol=0, atol=1e-5 * max(np.abs(g0).max(), 1e-12))
    # running statistics after three training forwards: r <- (1 - m) r + m * batch_stat
    mom = net.bn_momentum
    names = [n for n, l in net.layers.items() if getattr(l, "bn", False)]
    assert len(names) == len(rec)
    for n, r in zip(names, rec):
        rm, rv = net.running[n]
        c = r["mean"].numel()
        em, ev = torch.zeros(c), torch.ones(c)
        for _ in range(3):
            em = (1 - mom) * em + mom * r["mean"]
            ev = (1 - mom) * ev + mom * r["var_unbiased"]
        np.testing.assert_allclose(rm[:c].cpu().numpy(), em.numpy(), rtol=1e-4, atol=1e-5, err_msg=n)
        np.testing.assert_allclose(rv[:c].cpu().numpy(), ev.numpy(), rtol=1e-4, atol=1e-5, err_msg=n)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_unet_bn_eval_bn_folded(dtype):
    """Eval forward with each conv's BatchNorm folded in (forward weights scaled per output channel by the BN
    scale with adp_scale_rows, BN shift as the bias, ReLU and the activation store in the conv epilogue; no z, no
    apply pass, the encoder pools from the stored activation) against the unfolded schedule (z, then the BN
    apply), after a few training steps so the running statistics are not the initial ones: f32 to 1e-5, bf16 to
    the storage rounding of z the folded form skips."""
    B, L, S = 2, 3, 64
    w = R.unet_bn_keras_weights(levels=L, base=32, in_ch=3, seed=7)
    x, y = synth_batch(B, S, C=3, seed=13)
    net = UNetBN(B, S, levels=L, base=32, in_ch=3, dtype=dtype, device=DEV)
    net.set_weights(w)
    tr = Trainer(net, LossConfig(use_hard_mining=False))
    for _ in range(3):
        tr.train_step(x.to(DEV), y.to(DEV))
    outs = {}
    for fold in (False, True):
        net.fuse_eval_bn = fold
        ops.prep_input(x.to(DEV), net.acts(B)["x"], mean=0.0, std=1.0)
        outs[fold] = net.forward(B, train=False)["main_out"].cpu().clone()
    net.fuse_eval_bn = True
    d = (outs[True] - outs[False]).abs()
    if dtype == "f32":
        assert d.max().item() < 1e-5, d.max().item()
    else:
        assert d.max().item() < 2e-2 and d.mean().item() < 2e-3, (d.max().item(), d.mean().item())
