"""CPU checks of the oracle's model.py restatement (oracle/torch_ref.py): the 'same' average pool with the
pad-excluding count against a brute-force window average, the (B, H)-as-spatial weight map, and the
weighted losses' known answers."""
import torch

from oracle import torch_ref as R


def brute_pool(y, k):
    B, H, W = y.shape
    r = k // 2
    out = torch.zeros_like(y)
    for b in range(B):
        for h in range(H):
            out[b, h] = y[max(0, b - r):b + r + 1, max(0, h - r):h + r + 1].mean((0, 1))
    return out


def test_avg_pool_same_excludes_padding():
    g = torch.Generator().manual_seed(0)
    for shape in ((3, 40, 30), (1, 25, 5), (30, 12, 2)):
        y = (torch.rand(*shape, generator=g) > 0.5).double()
        assert (R.avg_pool_same(y[None], 21)[0] - brute_pool(y, 21)).abs().max().item() < 1e-12


def test_border_weight_renormalised_mean_one():
    g = torch.Generator().manual_seed(1)
    y = (torch.rand(2, 64, 64, generator=g) > 0.97).double()
    w = R.border_weight(y)
    assert w.shape == (1, 2, 64, 64)
    assert abs(w.mean().item() - 1.0) < 1e-12
    assert len(torch.unique(w)) <= 2


def test_weighted_dice_perfect_prediction():
    y = torch.zeros(2, 32, 32, dtype=torch.float64)
    y[:, 8:20, 8:20] = 1.0
    assert abs(R.weighted_dice_loss(y, y.clone()).item()) < 1e-2   # only the +1 smoothing is left
    assert R.weighted_dice_loss(y, 1 - y).item() > 0.9
