"""Data-parallel paths at world_size 2 over gloo on the CPU.

* GradBuckets (trainer.py): reverse-order bucketing of the flat gradient buffer, async SUM all-reduce
  launched from the per-layer ready hooks, and finish() reducing whatever a hook did not launch.
* DP loss decomposition: with the Dice sums all-reduced and every row coefficient normalised by
  dp_row_normaliser (the global kept-row count), the per-rank gradients of the OHEM + Dice loss are
  exactly the single-device full-batch gradient (what Trainer.loss_and_grads / adp_loss_grad compute
  on the GPU). Checked against autograd of the oracle (oracle/torch_ref.py) on the whole batch.
* SlidingWindowInference.shard (predictor.py): rank shards are disjoint, contiguous and cover every
  tile position (full_evaluation_enhanced.py:232-245 positions).
Rendezvous on 127.0.0.1.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = fn(rank, world)
        # plain numpy copies: torch's fd-sharing of queued tensors dies with the child process
        q.put((rank, {k: (v.numpy().copy() if torch.is_tensor(v) else v) for k, v in res.items()}))
    finally:
        dist.destroy_process_group()


def run_ranks(fn, world=WORLD):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        # drain the results before joining: a child blocks in put() while the pipe is full
        for _ in range(world):
            r, res = q.get(timeout=180)   # a rank that died never answers: fail instead of hanging
            out[r] = res
    finally:
        for p in procs:
            p.join(60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return out


# ------------------------------------------------------------------------------- grad buckets
def _buckets_fn(rank, world, overlap=True):
    import _adipose_pkg  # noqa: F401
    from adipose_amd.nets import ParamStore
    from adipose_amd.trainer import GradBuckets

    class Net:
        pass

    net = Net()
    net.ps = ParamStore()
    sizes = {"l0": (300, 7), "l1": (64,), "l2": (1000, 3), "l3": (17,), "l4": (4000,), "l5": (256, 9)}
    for name, shp in sizes.items():
        net.ps.add(name + "/W", shp)
        net.ps.add(name + "/b", (shp[-1],))
    net.ps.allocate("cpu")
    g = torch.Generator().manual_seed(100 + rank)
    net.ps.grad.copy_(torch.randn(net.ps.total, generator=g))
    before = net.ps.grad.clone()
    gb = GradBuckets(net, bucket_bytes=16 << 10, overlap=overlap)    # small buckets -> several launches
    gb.begin()
    for name in reversed(list(sizes)):
        if name != "l2":                              # l2's hook never fires: finish() must cover it
            gb.ready(name)
    launched_before_finish = sum(gb.launched)
    gb.finish()
    return {"before": before, "after": net.ps.grad.clone(), "nbuckets": len(gb.buckets),
            "launched_before_finish": launched_before_finish, "launches": gb.launches}


def _buckets_after_fn(rank, world):
    return _buckets_fn(rank, world, overlap=False)


@pytest.mark.parametrize("fn", [_buckets_fn, _buckets_after_fn], ids=["overlap", "after_backward"])
def test_grad_buckets_sum_allreduce(fn):
    """Bucketed SUM all-reduce: launched from the backward's ready-hooks (overlap) or all at finish()
    (GradBuckets(overlap=False), bench.py --allreduce after): the same sums either way."""
    res = run_ranks(fn)
    total = sum(res[r]["before"] for r in range(WORLD))
    assert res[0]["nbuckets"] > 2
    if fn is _buckets_after_fn:
        assert res[0]["launched_before_finish"] == 0
    else:
        assert res[0]["launched_before_finish"] > 0
        # ready buckets go out two at a time behind one flush (launch_group = 2), the rest at finish()
        assert res[0]["launches"] <= (res[0]["nbuckets"] + 1) // 2 + 1
    for r in range(WORLD):
        np.testing.assert_allclose(res[r]["after"], total, rtol=0, atol=1e-5)


# ------------------------------------------------------------------------- DP loss decomposition
def _loss_fn(rank, world):
    import _adipose_pkg  # noqa: F401
    from adipose_amd.trainer import dp_row_normaliser
    from oracle import torch_ref as R

    B, H, W, keep = 4, 16, 24, 0.7
    g = torch.Generator().manual_seed(7)               # identical full batch on every rank
    y = (torch.rand(B, H, W, generator=g) > 0.55).float()
    p_full = torch.rand(B, H, W, generator=g) * 0.98 + 0.01
    # single-device reference gradient of the whole batch
    pr = p_full.clone().requires_grad_(True)
    R.ohem_loss(y, pr, keep).backward()
    # this rank's shard
    bl = B // world
    ys = y[rank * bl:(rank + 1) * bl]
    ps = p_full[rank * bl:(rank + 1) * bl].clone().requires_grad_(True)
    k = int(np.float32(H) * np.float32(keep))
    rows = R.keras_bce_rows(ys, ps)
    bce = torch.topk(rows, k, dim=1).values.sum() / dp_row_normaliser(world, bl, k)
    pc = torch.clamp(ps, R.KEPS, 1.0 - R.KEPS)
    sums = torch.stack([(ys * pc).sum(), ys.sum(), pc.sum()]).detach().double()
    dist.all_reduce(sums)                              # batch-global Dice sums
    inter, sy, sp = sums.tolist()
    den = sy + sp + 1.0
    g_i, g_c = -2.0 / den, (2.0 * inter + 1.0) / den ** 2  # d(1 - Dice)/d pc = g_i * y + g_c
    (bce + ((g_i * ys + g_c) * pc).sum()).backward()
    parts = [torch.zeros_like(ps.grad) for _ in range(world)]
    dist.all_gather(parts, ps.grad)
    return {"dp": torch.cat(parts), "ref": pr.grad}


def test_dp_loss_gradient_matches_full_batch():
    res = run_ranks(_loss_fn)
    for r in range(WORLD):
        np.testing.assert_allclose(res[r]["dp"], res[r]["ref"], rtol=1e-5, atol=1e-8)


# ------------------------------------------------------------------------------ SW sharding
def _shard_fn(rank, world):
    import _adipose_pkg  # noqa: F401
    from adipose_amd.predictor import SlidingWindowInference

    sw = SlidingWindowInference(tile_size=1024, overlap=0.75, process_group=dist.group.WORLD, verbose=False)
    pos = sw.extract_tile_positions((3000, 2500))
    return {"all": pos, "mine": sw.shard(pos)}


def test_sliding_window_shards_cover_positions():
    res = run_ranks(_shard_fn)
    allpos = res[0]["all"]
    got = [p for r in range(WORLD) for p in res[r]["mine"]]
    assert got == list(allpos)                         # disjoint, contiguous, complete, in order
    assert all(len(res[r]["mine"]) > 0 for r in range(WORLD))


# ------------------------------------------------------------------------------- row-band reduce to rank 0
def _tile(y, x, T):
    g = torch.Generator().manual_seed(1000 * y + x)
    return torch.rand(T, T, generator=g)


def _accum(c, tile, w, y, x):
    """blend_accum's arithmetic (acc += w * p, wsum += w) on a CPU BandCanvas (the kernel needs a GPU)."""
    T = tile.shape[-1]
    c.acc[y - c.y0:y - c.y0 + T, x:x + T] += w * tile
    c.ws[y - c.y0:y - c.y0 + T, x:x + T] += w


def _band_fn(rank, world):
    import _adipose_pkg  # noqa: F401
    from adipose_amd.predictor import BandCanvas, GaussianBlender, SlidingWindowInference, band_rows

    H, W, T = 320, 288, 64
    sw = SlidingWindowInference(tile_size=T, overlap=0.5, process_group=dist.group.WORLD, verbose=False)
    pos = sw.extract_tile_positions((H, W))
    bands = [(0, H)] + [band_rows(sw.shard(pos, q), T) for q in range(1, world)]
    c = BandCanvas((H, W), bands[rank], "cpu")
    w = torch.from_numpy(GaussianBlender(T).weight_map)
    for y, x in sw.shard(pos):
        _accum(c, _tile(y, x, T), w, y, x)
    root = c.reduce_to_root(dist.group.WORLD, bands)
    return {"root": root, "rows": c.y1 - c.y0, "acc": c.acc.clone() if root else None,
            "ws": c.ws.clone() if root else None}


@pytest.mark.parametrize("world", [2, 4])
def test_band_reduce_to_root_matches_one_canvas(world):
    """predictor.BandCanvas: ranks > 0 hold only the rows of their tiles; rank 0 adds their bands in rank order and
    gets the one-canvas blend sums (full_evaluation_enhanced.py:286-329) within f32 rounding of the association."""
    import _adipose_pkg  # noqa: F401
    from adipose_amd.predictor import BandCanvas, GaussianBlender, SlidingWindowInference

    res = run_ranks(_band_fn, world)
    H, W, T = 320, 288, 64
    sw = SlidingWindowInference(tile_size=T, overlap=0.5, verbose=False)
    ref = BandCanvas((H, W), (0, H), "cpu")
    w = torch.from_numpy(GaussianBlender(T).weight_map)
    for y, x in sw.extract_tile_positions((H, W)):
        _accum(ref, _tile(y, x, T), w, y, x)
    assert res[0]["root"] and res[0]["rows"] == H
    np.testing.assert_allclose(res[0]["acc"], ref.acc.numpy(), rtol=0, atol=2e-6)
    np.testing.assert_allclose(res[0]["ws"], ref.ws.numpy(), rtol=0, atol=2e-6)
    for r in range(1, world):
        assert not res[r]["root"] and 0 < res[r]["rows"] < H


def _bcast_fn(rank, world):
    import _adipose_pkg  # noqa: F401
    from adipose_amd.predictor import _bcast_frame
    frame = torch.arange(12, dtype=torch.float32).reshape(3, 4) + 0.5 if rank == 0 else None
    return {"out": _bcast_frame(frame, (3, 4), "cpu", dist.group.WORLD)}


@pytest.mark.parametrize("world", [2, 4])
def test_sliding_window_broadcast_frame(world):
    """predict_with_sliding_window(broadcast=True): rank 0's finished map reaches every rank (predictor._bcast_frame)."""
    res = run_ranks(_bcast_fn, world)
    ref = torch.arange(12, dtype=torch.float32).reshape(3, 4) + 0.5
    for r in range(world):
        np.testing.assert_array_equal(np.asarray(res[r]["out"]), ref.numpy())
