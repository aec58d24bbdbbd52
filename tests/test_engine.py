"""Handle-level C ABI (adp_create / adp_set_param / adp_forward / adp_destroy; csrc/engine.cpp): the native
adipose_v3 inference engine against the Python schedule (nets.AdiposeV3Net through HipUnetPredictor)
and the CPU oracle, on the same Keras weights (predict_single segmentation_inference.py:153-158, TTA
:181-229)."""
import numpy as np
import pytest
import torch

from oracle import numpy_ref as NR
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu
S = 64


@pytest.fixture(scope="module")
def weights():
    return R.adipose_v3_keras_weights(seed=865, deep_supervision=True)


def oracle_predict(w):
    def f(image, mean, std):
        x = torch.from_numpy(((image - np.float32(mean)) / np.float32(std + 1e-10)).astype(np.float32))[None]
        return R.adipose_v3_forward(x, w, deep_supervision=True)["main_out"][0].numpy()
    return f


def test_engine_params_round_trip_and_errors(weights):
    from adipose_amd._lib import AdpError
    from adipose_amd.engine import NativeAdiposeV3
    eng = NativeAdiposeV3(tile=S, max_batch=4, dtype="f32")
    names = eng.layer_names()
    assert names[0] == "down1_conv1" and "dilate6" in names and names[-1] == "output_softmax"
    assert set(names) == set(weights)
    eng.set_weights(weights)
    got = eng.get_weights()
    for k in names:
        for a, b in zip(weights[k], got[k]):
            np.testing.assert_array_equal(np.asarray(a, np.float32).ravel(), b)
    with pytest.raises(AdpError):
        eng.predict_batch(np.zeros((1, S + 8, S + 8), np.float32), 0.0, 1.0)
    bad = {"down1_conv1": [np.zeros(5, np.float32), np.zeros(44, np.float32)]}
    with pytest.raises(AdpError):
        eng.set_weights(bad)
    eng.close()


@pytest.mark.parametrize("tta", [None, "minimal", "basic", "full"])
def test_engine_f32_vs_python_and_oracle(weights, tta):
    from adipose_amd.engine import NativeAdiposeV3
    from adipose_amd.nets import AdiposeV3Net
    from adipose_amd.predictor import TTA_VIEWS, HipUnetPredictor
    rng = np.random.default_rng(3)
    imgs = (rng.random((3, S, S)) * 255).astype(np.float32)
    eng = NativeAdiposeV3(tile=S, max_batch=8, dtype="f32")
    eng.set_weights(weights)
    got = eng.predict_batch(imgs, 127.0, 50.0, tta_mode=tta).cpu().numpy()
    net = AdiposeV3Net(1, S, dtype="f32", device="cuda", deep_supervision=True)
    net.set_weights(weights)
    pred = HipUnetPredictor(net, max_batch=8)
    views = TTA_VIEWS[tta] if tta else [0]
    ref = pred.predict_views(list(imgs), 127.0, 50.0, views).cpu().numpy()
    assert np.abs(got - ref).max() <= 1e-5, np.abs(got - ref).max()
    f = oracle_predict(weights)
    for i in range(3):
        o = NR.tta_predict(f, imgs[i], 127.0, 50.0, tta) if tta else f(imgs[i], 127.0, 50.0)
        assert np.abs(got[i] - o).max() <= 1e-4
    eng.close()


def test_engine_bf16_matches_python_bf16_predictor(weights):
    from adipose_amd.engine import NativeAdiposeV3
    from adipose_amd.predictor import AdiposeUNet
    rng = np.random.default_rng(4)
    imgs = (rng.random((5, S, S)) * 255).astype(np.float32)
    eng = NativeAdiposeV3(tile=S, max_batch=4, dtype="bf16")
    eng.set_weights(weights)
    got = eng.predict_batch(imgs, 127.0, 50.0, tta_mode="basic").cpu().numpy()
    m = AdiposeUNet(tile_size=S, dtype="bf16", max_batch=4)
    m.build_model(use_deep_supervision=True)
    m.net.set_weights(weights)
    ref = np.stack([m.predict(im, 127.0, 50.0, use_tta=True, tta_mode="basic")[0] for im in imgs])
    assert np.abs(got - ref).max() <= 1e-5, np.abs(got - ref).max()
    f32 = NativeAdiposeV3(tile=S, max_batch=4, dtype="f32")
    f32.set_weights(weights)
    exact = f32.predict_batch(imgs, 127.0, 50.0, tta_mode="basic").cpu().numpy()
    assert np.abs(got - exact).max() <= 2e-2
    eng.close()
    f32.close()


def _train_data(seed, B=2):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((B, S, S)).astype(np.float32)
    yy, xx = np.mgrid[0:S, 0:S]
    y = np.stack([((yy - 20 - 8 * b) ** 2 + (xx - 30) ** 2 < 300).astype(np.float32) for b in range(B)])
    return x, y


def _python_trainer(weights, dtype, cpad=None, lr=1e-3, freeze=False):
    from adipose_amd.nets import AdiposeV3Net
    from adipose_amd.trainer import LossConfig, Trainer
    net = AdiposeV3Net(2, S, dtype=dtype, device="cuda", deep_supervision=True, cpad=cpad)
    net.set_weights(weights)
    tr = Trainer(net, LossConfig(), optimizer="adam", lr=lr)
    if freeze:
        tr.set_frozen(net.ENCODER)
    return net, tr


def _compare_weights(a, b, lr, steps):
    n_big, n_all, worst, per = 0, 0, 0.0, []
    for k in a:
        for i, (u, v) in enumerate(zip(a[k], b[k])):
            d = np.abs(np.asarray(u, np.float32).ravel() - np.asarray(v, np.float32).ravel())
            nb = int((d > 1e-6).sum())
            n_big += nb
            n_all += d.size
            worst = max(worst, float(d.max()))
            if nb:
                per.append((k, i, nb, d.size, float(d.max())))
    # Adam's first steps move every weight by ~lr * sign(g): a gradient that is zero up to rounding may
    # take either sign in two f32 atomic summation orders, so a few elements may differ by <= 2 lr (measured:
    # up to 0.17 % of the weights by more than 1e-6, all in layers with many near-zero gradients). A wrong or
    # missing gradient term moves most of its layer's weights by ~lr: every layer is bounded on its own (10 % of
    # its elements, at least 4), so one bad layer fails even when it is small against the whole net
    assert worst <= 2 * lr * steps + 1e-6 and n_big <= 3e-3 * n_all, (worst, n_big, n_all, per[:8])
    bad = [p for p in per if p[2] > max(4, 0.1 * p[3])]
    assert not bad, bad


@pytest.mark.parametrize("freeze", [False, True])
def test_native_train_step_matches_python_f32(weights, freeze):
    """adp_train_step (csrc/engine.cpp) vs the Python schedule (trainer.Trainer over nets.AdiposeV3Net):
    OHEM main + BCE-Dice aux losses with dropout 0.3, Adam; per-step Keras metrics and the weights after
    two steps; frozen encoder = no encoder update."""
    from adipose_amd.engine import NativeAdiposeV3, train_cfg
    lr = 1e-3
    x, y = _train_data(7)
    net, tr = _python_trainer(weights, "f32", lr=lr, freeze=freeze)
    eng = NativeAdiposeV3(tile=S, max_batch=2, dtype="f32")
    eng.set_weights(weights)
    cfg = train_cfg(freeze_encoder=freeze)
    xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    for step in range(2):
        tr.train_step(xd, yd)
        ref = tr.read_metrics()
        got = eng.train_step(x, y, lr, cfg)
        for k, v in got.items():
            assert abs(v - ref[k]) <= 2e-5 * max(1.0, abs(ref[k])), (step, k, v, ref[k])
    w_eng, w_py = eng.get_weights(), net.get_weights()
    _compare_weights(w_eng, w_py, lr, 2)
    if freeze:
        for k in net.ENCODER:
            np.testing.assert_array_equal(w_eng[k][0], np.asarray(weights[k][0], np.float32).ravel())
    # inference after training uses the trained weights (adp_forward)
    from adipose_amd.predictor import HipUnetPredictor
    p_eng = eng.predict_batch(x * 50 + 127, 127.0, 50.0).cpu().numpy()
    p_py = HipUnetPredictor(net, max_batch=2).predict_views(list(x * 50 + 127), 127.0, 50.0, [0]).cpu().numpy()
    assert np.abs(p_eng - p_py).max() <= 1e-4
    eng.close()


def test_native_train_step_bf16_and_comm(weights):
    """bf16 native step vs the Python bf16 schedule on the same channel layout; then the same step through
    a one-rank RCCL communicator (adp_comm_unique_id / adp_comm_init / adp_set_comm: the gradient and loss
    all-reduces run) equals the step without one."""
    from adipose_amd.engine import NativeAdiposeV3, comm_destroy, comm_init, comm_unique_id, train_cfg
    lr = 1e-3
    x, y = _train_data(8)
    net, tr = _python_trainer(weights, "bf16", cpad=(64, 64, 64, 64), lr=lr)
    eng = NativeAdiposeV3(tile=S, max_batch=2, dtype="bf16")
    eng.set_weights(weights)
    tr.train_step(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda())
    ref = tr.read_metrics()
    got = eng.train_step(x, y, lr, train_cfg())
    for k, v in got.items():
        assert abs(v - ref[k]) <= 1e-3 * max(1.0, abs(ref[k])), (k, v, ref[k])
    a = NativeAdiposeV3(tile=S, max_batch=2, dtype="f32")
    b = NativeAdiposeV3(tile=S, max_batch=2, dtype="f32")
    a.set_weights(weights)
    b.set_weights(weights)
    comm = comm_init(1, comm_unique_id(), 0)
    b.set_comm(comm)
    cfg = train_cfg(dropout_rate=0.0)
    ma, mb = a.train_step(x, y, lr, cfg), b.train_step(x, y, lr, cfg)
    for k in ma:
        assert abs(ma[k] - mb[k]) <= 1e-6 * max(1.0, abs(ma[k])), k
    _compare_weights(a.get_weights(), b.get_weights(), lr, 1)
    b.set_comm(None)
    comm_destroy(comm)
    for e in (eng, a, b):
        e.close()


# ------------------------------------------------------------------------------ unet_bn behind the handle
def _bn_case(L=3, S_=64, B=2, seed=5):
    w = R.unet_bn_keras_weights(levels=L, base=64, in_ch=3, seed=seed)
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((B, S_, S_, 3)).astype(np.float32)
    yy, xx = np.mgrid[0:S_, 0:S_]
    y = np.stack([((yy - 20 - 8 * b) ** 2 + (xx - 30) ** 2 < 300).astype(np.float32) for b in range(B)])
    return w, x, y


def _compare_grads(a, b, dtype, what, after_step=False, same_schedule=False):
    """Per-layer gradients of two runs of the same step. Two schedules (native vs Python) sum in different orders,
    so they differ by f32 rounding, and where a pre-activation within rounding of the ReLU kink takes the other
    subgradient, by that element spread over its channel through the BatchNorm backward, whose mean subtraction
    cancels (measured up to ~3e-2 of a layer's largest gradient in the first layer at cosine 0.999996; bf16 adds its
    storage rounding). One schedule twice (same_schedule): activations, BatchNorm sums and data gradients are
    bit-identical since round 4, only the weight gradients' f32 atomic order differs. A wrong or missing term moves a whole layer: the direction (cosine) and the largest
    element error catch it."""
    bad = []
    for n in a:
        for si, (u, v) in enumerate(zip(a[n], b[n])):
            u, v = np.asarray(u, np.float64).ravel(), np.asarray(v, np.float64).ravel()
            c = float(u @ v / (np.linalg.norm(u) * np.linalg.norm(v) + 1e-30))
            r = float(np.abs(u - v).max() / max(np.abs(v).max(), 1e-12))
            # (after_step: the gradients of a second step, on weights that already differ where Adam's first
            # step took a rounding-level gradient's sign: measured cosine 0.99967, largest element 3.5e-2)
            cmin, rmax = (0.999, 0.1) if after_step else (0.9999, 5e-2)
            if same_schedule:   # one schedule twice: only the weight gradients' f32 atomic order differs (<= 7e-7
                cmin, rmax = 0.9999999, 1e-5   # measured, profiles/r04e_f32_step_determinism.txt)
            if (dtype == "f32" and (c < cmin or r > rmax)) or (dtype == "bf16" and c < 0.99):
                bad.append((n, si, round(c, 6), round(r, 5)))
    assert not bad, (what, bad)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_native_unet_bn_train_step_matches_python(dtype):
    """unet_bn through adp_create -> adp_train_step -> adp_get_grad / adp_get_param (csrc/engine.cpp) vs the
    Python schedule (nets.UNetBN + trainer.Trainer) on the same weights and tiles: per-step Keras metrics,
    per-layer gradients of the first step, weights after two Adam steps, BatchNorm running statistics, and the
    eval forward (adp_forward) after training."""
    from adipose_amd import ops
    from adipose_amd.engine import NativeUNetBN, train_cfg
    from adipose_amd.nets import UNetBN
    from adipose_amd.trainer import LossConfig, Trainer
    L, S_, B, lr = 3, 64, 2, 1e-3
    w, x, y = _bn_case(L, S_, B)
    net = UNetBN(B, S_, levels=L, base=64, in_ch=3, dtype=dtype, device="cuda")
    net.set_weights(w)
    tr = Trainer(net, LossConfig(use_hard_mining=False), lr=lr)
    eng = NativeUNetBN(tile=S_, max_batch=B, dtype=dtype, levels=L)
    assert eng.layer_names() == list(net.layers)
    eng.set_weights(w)
    got0 = eng.get_weights()
    for k in w:
        for a, b in zip(w[k], got0[k]):
            np.testing.assert_array_equal(np.asarray(a, np.float32).ravel(), b)
    cfg = train_cfg(use_hard_mining=False)
    xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    for step in range(2):
        # (step 2 runs on weights that already differ where Adam's first step took a rounding-level gradient's
        # sign: f32 metrics to 1e-4 there)
        tol = (2e-5 if step == 0 else 1e-4) if dtype == "f32" else 3e-3
        tr.train_step(xd, yd)
        ref = tr.read_metrics()
        got = eng.train_step(x, y, lr, cfg)
        for k in ("loss", "main_out_loss", "main_out_dice_coef", "main_out_binary_accuracy"):
            t_k = tol
            if k == "main_out_binary_accuracy" and step > 0:
                # (a count metric: one pixel at the 0.5 threshold is 1 / (B S^2) = 1.2e-4 here; on step-2 weights
                # that differ at the rounding level a few pixels may sit on the other side of it)
                t_k = max(tol, 8.0 / (B * S_ * S_))
            assert abs(got[k] - ref[k]) <= t_k * max(1.0, abs(ref[k])), (step, k, got[k], ref[k])
        if step == 0:
            _compare_grads(eng.get_grads(), {n: net.get_layer_grads(n) for n in net.layers}, dtype, "step-1 grads")
    w_eng = eng.get_weights()
    w_py = {n: net.get_layer_weights(n) for n in net.layers}
    worst = max(float(np.abs(np.asarray(u, np.float32).ravel() - np.asarray(v, np.float32).ravel()).max())
                for k in w_py for u, v in zip(w_eng[k], w_py[k]))
    assert worst <= 2 * lr * 2 + 1e-6, worst   # Adam moves a weight by <= ~lr per step
    for n, l in net.layers.items():
        if getattr(l, "bn", False):
            rm, rv = eng.running_stats(n)
            # (the second step's batch statistics come from weights that differ by <= 2 lr in a few elements)
            at = 2e-3 if dtype == "f32" else 2e-2
            np.testing.assert_allclose(rm, net.running[n][0][:l.cout].cpu().numpy(), rtol=1e-2, atol=at, err_msg=n)
            np.testing.assert_allclose(rv, net.running[n][1][:l.cout].cpu().numpy(), rtol=1e-2, atol=at, err_msg=n)
    # eval forward (running statistics) of the trained handle vs the Python network
    p_eng = eng.predict_batch(x, 0.0, 1.0).cpu().numpy()
    ops.prep_input(xd, net.acts(B)["x"], mean=0.0, std=1.0)
    p_py = net.forward(B, train=False)["main_out"].cpu().numpy()
    assert np.abs(p_eng - p_py).max() <= (1e-3 if dtype == "f32" else 2e-2), np.abs(p_eng - p_py).max()
    eng.close()


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_native_unet_bn_eval_matches_python(dtype):
    """adp_forward of the unet_bn handle vs nets.UNetBN.forward(train=False) on the same weights and running
    statistics: both fold the eval BatchNorm into the conv weights (adp_scale_rows) and epilogues, the level-0
    activation is materialised by its folded conv and the head reads it without BatchNorm-on-load; the eval
    path has no atomics, so the two schedules give the same probabilities."""
    from adipose_amd import ops
    from adipose_amd.engine import NativeUNetBN
    from adipose_amd.nets import UNetBN
    L, S_, B = 3, 64, 2
    w, x, _ = _bn_case(L, S_, B, seed=9)
    rng = np.random.default_rng(9)
    net = UNetBN(B, S_, levels=L, base=64, in_ch=3, dtype=dtype, device="cuda")
    net.set_weights(w)
    eng = NativeUNetBN(tile=S_, max_batch=B, dtype=dtype, levels=L)
    eng.set_weights(w)
    for n, l in net.layers.items():
        if getattr(l, "bn", False):
            rm = rng.normal(0, 0.2, l.cout).astype(np.float32)
            rv = rng.uniform(0.5, 1.5, l.cout).astype(np.float32)
            net.running[n][0][:l.cout].copy_(torch.from_numpy(rm))
            net.running[n][1][:l.cout].copy_(torch.from_numpy(rv))
            eng.set_running_stats(n, rm, rv)
            got = eng.running_stats(n)
            np.testing.assert_array_equal(got[0], rm)
            np.testing.assert_array_equal(got[1], rv)
    p_eng = eng.predict_batch(x, 0.0, 1.0).cpu().numpy()
    xd = torch.from_numpy(x).cuda()
    ops.prep_input(xd, net.acts(B)["x"], mean=0.0, std=1.0)
    p_py = net.forward(B, train=False)["main_out"].cpu().numpy()
    assert np.abs(p_eng - p_py).max() <= 1e-6, np.abs(p_eng - p_py).max()
    eng.close()


def test_native_unet_bn_bucketed_comm_and_errors():
    """The bucketed, stream-overlapped gradient all-reduce (one-rank RCCL communicator) leaves the unet_bn step
    unchanged (metrics, per-layer gradients); bad parameter names / slots, a gradient read of a running
    statistic and a frozen-encoder request are rejected."""
    from adipose_amd._lib import AdpError, call
    from adipose_amd.engine import NativeUNetBN, comm_destroy, comm_init, comm_unique_id, train_cfg
    L, S_, B, lr = 3, 64, 2, 1e-3
    w, x, y = _bn_case(L, S_, B, seed=6)
    a = NativeUNetBN(tile=S_, max_batch=B, dtype="f32", levels=L)
    b = NativeUNetBN(tile=S_, max_batch=B, dtype="f32", levels=L)
    a.set_weights(w)
    b.set_weights(w)
    with pytest.raises(AdpError):   # no step yet
        call("adp_get_grad", a._h, b"head", 1, np.zeros(1, np.float32).ctypes.data, 1)
    comm = comm_init(1, comm_unique_id(), 0)
    b.set_comm(comm)
    cfg = train_cfg(use_hard_mining=False)
    for step in range(2):
        if step:   # Adam's first step moves a weight by ~lr * sign(g), and a rounding-level gradient takes either
            # sign in two runs (f32 atomic order), so the second step starts both handles from a's weights:
            # the comparison is then of the step itself, not of Adam's amplified rounding (measured: per-layer
            # gradient cosines down to 0.9908 otherwise)
            b.set_weights(a.get_weights())
        ma, mb = a.train_step(x, y, lr, cfg), b.train_step(x, y, lr, cfg)
        for k in ma:
            assert abs(ma[k] - mb[k]) <= 2e-5 * max(1.0, abs(ma[k])), (step, k)
        _compare_grads(b.get_grads(), a.get_grads(), "f32", f"step {step} grads", same_schedule=True)
    b.set_comm(None)
    comm_destroy(comm)
    with pytest.raises(AdpError):
        a.train_step(x, y, lr, train_cfg(use_hard_mining=False, freeze_encoder=True))
    with pytest.raises(AdpError):
        a.set_weights({"enc0_conv1": [np.zeros(7, np.float32)]})
    with pytest.raises(AdpError):
        call("adp_set_param", a._h, b"head", 2, np.zeros(1, np.float32).ctypes.data, 1)
    with pytest.raises(AdpError):
        call("adp_get_grad", a._h, b"enc0_conv1", 3, np.zeros(64, np.float32).ctypes.data, 64)
    a.close()
    b.close()


@pytest.mark.parametrize("preset", ["adipose_v3", "unet_bn"])
def test_bucket_allreduce_reads_final_gradients(weights, preset):
    """The native step's overlapped bucket all-reduce (engine.cpp dp_launch) may only start once every gradient
    of its bucket is written. With a one-rank communicator the in-place SUM changes nothing, so the test takes a
    snapshot of each bucket on the communication stream at the moment its all-reduce is issued (option
    dp_snapshot, adp_debug_grad_flat) and requires it to equal the final gradient buffer element for element: a
    gradient written after its bucket started would differ (frozen-encoder step included)."""
    from adipose_amd import ops
    from adipose_amd._lib import AdpError, call
    from adipose_amd.engine import NativeAdiposeV3, NativeUNetBN, comm_destroy, comm_init, comm_unique_id, train_cfg
    if preset == "adipose_v3":
        e = NativeAdiposeV3(tile=S, max_batch=2, dtype="bf16")
        e.set_weights(weights)
        x, y = _train_data(11)
        cfgs = [train_cfg(), train_cfg(freeze_encoder=True)]
    else:
        w, x, y = _bn_case(3, S, 2, seed=7)
        e = NativeUNetBN(tile=S, max_batch=2, dtype="bf16", levels=3)
        e.set_weights(w)
        cfgs = [train_cfg(use_hard_mining=False)]
    comm = comm_init(1, comm_unique_id(), 0)
    e.set_comm(comm)
    ops.set_option("dp_snapshot", 1)
    try:
        for cfg in cfgs:
            e.train_step(x, y, 1e-3, cfg)
            with pytest.raises(AdpError) as err:   # a size query: the message names the flat size
                call("adp_debug_grad_flat", e._h, 0, None, 0)
            n = int(str(err.value).rsplit(" ", 1)[-1])
            g = np.zeros(n, np.float32)
            snap = np.zeros(n, np.float32)
            call("adp_debug_grad_flat", e._h, 0, g.ctypes.data, n)
            call("adp_debug_grad_flat", e._h, 1, snap.ctypes.data, n)
            assert np.abs(g).max() > 0
            diff = np.flatnonzero(g != snap)
            assert diff.size == 0, (preset, diff.size, diff[:8])
    finally:
        ops.set_option("dp_snapshot", 0)
        e.set_comm(None)
        comm_destroy(comm)
        e.close()


def test_c_client_trains_both_presets():
    """The plain C caller (tests/c_abi/abi_client.c, built next to the library) drives both presets on device 0
    with its own HIP device buffers: adp_create -> adp_set_param (every layer / slot) -> four adp_train_step
    (finite metrics, falling loss) -> adp_get_grad -> adp_forward (probabilities in [0, 1]) -> a rejected
    TTA mode -> adp_destroy."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    client = os.path.join(root, "adipose_tissue-unet_amd", "abi_client")
    assert os.path.exists(client), "abi_client is built with the library (make -C adipose_tissue-unet_amd/csrc)"
    r = subprocess.run([client, "gpu"], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gpu: 0 failed" in r.stdout, r.stdout
