"""The product data-parallel paths at world size 2 on the GPU.

Two ranks are spawned as fresh processes (no GPU state inherited), both on cuda:0, joined by a gloo
process group (the collectives run on CUDA tensors through gloo; RCCL is the same torch.distributed API).

* Trainer.train_step with B=2 per rank vs a single-process B=4 step on the same tiles: the batch-global Dice
  sums (train_adipose_unet_v3.py:217-225) are all-reduced before the loss gradient, the OHEM row terms are
  normalised by the global row count, and the gradients are SUM-all-reduced in buckets from the backward's
  ready hooks (trainer.GradBuckets). Per-layer gradients must match the single-device ones to f32 tolerance
  and the post-Adam weights to Adam's sign tolerance (dropout off: its stateless mask is keyed by the
  rank-local element index).
* SlidingWindowInference(process_group=...) on a small image at world 2 and 4: tile rows sharded over the ranks,
  each rank > 0 blending into a row band of the frame only, the bands added into rank 0's frame (BandCanvas),
  equal to the one-process output (full_evaluation_enhanced.py:286-329)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
import _adipose_pkg  # noqa: E402,F401

pytestmark = pytest.mark.gpu
WORLD, B_LOCAL, S, LR = 2, 2, 64, 1e-3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    finally:
        dist.destroy_process_group()


def run_ranks(fn, world=WORLD):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, res = q.get(timeout=100)
            out[r] = res
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return out


def _data():
    from adipose_amd.data import synthetic_batch, to_gray
    xs, ys = synthetic_batch(WORLD * B_LOCAL, S, channels=3, seed=865)
    x = to_gray(xs).astype(np.float32)
    x = (x - x.mean()) / (x.std() + 1e-10)
    return x, ys.astype(np.float32)


def _net(batch):
    from adipose_amd.nets import AdiposeV3Net
    from oracle import torch_ref as R
    net = AdiposeV3Net(batch, S, dtype="f32", device="cuda", seed=865)
    net.set_weights(R.adipose_v3_keras_weights(seed=865))
    net.dropout_rate = 0.0
    return net


def _snapshot(net):
    names = list(net.layers)
    return {"grads": {n: [a.copy() for a in net.get_layer_grads(n)] for n in names},
            "weights": {n: [a.copy() for a in net.get_layer_weights(n)] for n in names}}


def _train_fn(rank, world, overlap=True):
    from adipose_amd.trainer import LossConfig, Trainer
    x, y = _data()
    sl = slice(rank * B_LOCAL, (rank + 1) * B_LOCAL)
    net = _net(B_LOCAL)
    tr = Trainer(net, LossConfig(), lr=LR, distributed=True, bucket_bytes=1 << 20,   # several buckets
                 overlap_allreduce=overlap)
    assert tr.buckets is not None and len(tr.buckets.buckets) > 2
    tr.train_step(torch.from_numpy(x[sl]).cuda(), torch.from_numpy(y[sl]).cuda())
    met = tr.read_metrics()
    torch.cuda.synchronize()
    out = _snapshot(net)
    out["metrics"] = met
    return out


def _train_after_fn(rank, world):
    return _train_fn(rank, world, overlap=False)


@pytest.mark.parametrize("fn", [_train_fn, _train_after_fn], ids=["overlap", "after_backward"])
def test_dp_train_step_world2_matches_single_device_batch(fn):
    from adipose_amd.trainer import LossConfig, Trainer
    res = run_ranks(fn)
    x, y = _data()
    net = _net(WORLD * B_LOCAL)
    tr = Trainer(net, LossConfig(), lr=LR)
    tr.train_step(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda())
    met = tr.read_metrics()
    torch.cuda.synchronize()
    ref = _snapshot(net)
    for r in range(WORLD):
        for k in ("loss", "main_out_dice_coef", "main_out_binary_accuracy"):
            assert abs(res[r]["metrics"][k] - met[k]) < 2e-5 * max(1.0, abs(met[k])), (r, k, res[r]["metrics"][k], met[k])
        for n, gs in ref["grads"].items():
            for si, g in enumerate(gs):
                got = res[r]["grads"][n][si]
                err = np.abs(got - g).max() / max(np.abs(g).max(), 1e-12)
                assert err < 1e-4, (r, n, si, err)
        for n, ws in ref["weights"].items():
            for si, w in enumerate(ws):
                d = np.abs(res[r]["weights"][n][si] - w)
                # Adam's first step moves every weight by ~lr * sign(g): a sign flip of a near-zero gradient
                # component is the only way two f32 summation orders can differ by more than rounding
                assert d.max() <= 2.05 * LR, (r, n, si, d.max())
                assert (d > 1e-6).mean() < 1e-3, (r, n, si, (d > 1e-6).mean())


def _sw_image():
    rng = np.random.default_rng(17)
    return (rng.random((320, 288)) * 255).astype(np.float32)


def _sw_predictor():
    from adipose_amd.nets import AdiposeV3Net
    from adipose_amd.predictor import HipUnetPredictor
    from oracle import torch_ref as R
    net = AdiposeV3Net(1, 64, dtype="f32", device="cuda", deep_supervision=False)
    net.set_weights(R.adipose_v3_keras_weights(seed=865, deep_supervision=False))
    return HipUnetPredictor(net, max_batch=8)


def _sw_fn(rank, world):
    import torch.distributed as dist

    from adipose_amd import predictor as P
    sw = P.SlidingWindowInference(64, 0.5, "gaussian", process_group=dist.group.WORLD, verbose=False)
    pos = sw.extract_tile_positions((320, 288))
    rows = []   # the canvas rows this rank allocates (BandCanvas.__init__)
    orig = P.BandCanvas.__init__

    def spy(self, shape, band, device):
        orig(self, shape, band, device)
        rows.append(self.y1 - self.y0)
    P.BandCanvas.__init__ = spy
    try:
        out = sw.predict_with_sliding_window(_sw_image(), _sw_predictor(), 127.0, 50.0, use_tta=True,
                                             tta_mode="basic")
    finally:
        P.BandCanvas.__init__ = orig
    # broadcast=True: every rank returns rank 0's map (round 6, opt-in)
    outb = sw.predict_with_sliding_window(_sw_image(), _sw_predictor(), 127.0, 50.0, use_tta=True, tta_mode="basic",
                                          broadcast=True)
    return {"out": out, "outb": outb, "mine": len(sw.shard(pos)), "all": len(pos), "rows": rows}


@pytest.mark.parametrize("world", [2, 4])
def test_dp_sliding_window_bands_match_one_rank(world):
    from adipose_amd.predictor import SlidingWindowInference
    res = run_ranks(_sw_fn, world)
    sw = SlidingWindowInference(64, 0.5, "gaussian", verbose=False)
    ref = sw.predict_with_sliding_window(_sw_image(), _sw_predictor(), 127.0, 50.0, use_tta=True, tta_mode="basic")
    assert sum(res[r]["mine"] for r in range(world)) == res[0]["all"] and min(res[r]["mine"] for r in range(world)) > 0
    # the bands are summed in a different association (rank partial sums), so allow f32 rounding
    np.testing.assert_allclose(res[0]["out"], ref, rtol=0, atol=2e-6)
    assert res[0]["rows"] == [320]
    for r in range(world):
        np.testing.assert_array_equal(res[r]["outb"], res[0]["out"])
    for r in range(1, world):
        assert res[r]["out"] is None   # (the frame lives on rank 0)
        assert len(res[r]["rows"]) == 1 and res[r]["rows"][0] < 320, res[r]["rows"]   # a band, not the frame
