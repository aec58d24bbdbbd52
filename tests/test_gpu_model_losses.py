"""The rest of the src/utils/model.py loss / metric surface on the GPU against the CPU restatement
(oracle/torch_ref.py): weighted_dice_loss / weighted_bce_dice_loss values and gradients (:103-153, with the
21x21 'same' pad-excluding average pool over (B, H) per W), weighted_dice_coeff / weighted_bce_loss with an
explicit weight, and the metric helpers (:21-91). TF is absent, so the restatement is parity unpinned vs
TF 2.13; the pooling itself is checked against a brute-force window average (test_oracle_model_surface.py)."""
import numpy as np
import pytest
import torch

from adipose_amd import metrics as M
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu


def blobs(B, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    yy, xx = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    y = torch.zeros(B, H, W)
    for b in range(B):
        for _ in range(3):
            cy, cx = torch.randint(0, H, (1,), generator=g).item(), torch.randint(0, W, (1,), generator=g).item()
            r = 4 + torch.randint(0, max(5, H // 4), (1,), generator=g).item()
            y[b] += (((yy - cy) ** 2 + (xx - cx) ** 2) < r * r).float()
    y = (y > 0).float()
    p = torch.sigmoid(torch.randn(B, H, W, generator=g) * 2 + (y - 0.5) * 2)
    return y, p


CASES = [(2, 64, 48, 1), (1, 40, 70, 2), (4, 96, 96, 3), (3, 24, 24, 4)]


@pytest.mark.parametrize("B,H,W,seed", CASES)
@pytest.mark.parametrize("bce", [True, False])
def test_weighted_losses_value_and_grad(B, H, W, seed, bce):
    y, p = blobs(B, H, W, seed)
    # edge values: exact 0.5 (logit 0: TF's max(-l, 0) subgradient), the clip bounds and beyond
    p[0, 0, :4] = torch.tensor([0.5, 0.0, 1.0, 1e-9])
    loss, dp = M.weighted_loss_and_grad(y, p, bce=bce)
    # the oracle runs in f32, the reference's dtype: clip(1.0) = 1 - 1e-7 rounds to 1 - 2^-23 there, which moves
    # the logit of a clipped element by 0.2 against f64 arithmetic
    pr = p.clone().requires_grad_(True)
    ref = (R.weighted_bce_dice_loss if bce else R.weighted_dice_loss)(y, pr)
    ref.backward()
    assert abs(loss - ref.item()) <= 1e-5 * max(1.0, abs(ref.item())), (loss, ref.item())
    g = dp.cpu()
    err = (g - pr.grad).abs().max().item() / pr.grad.abs().max().item()
    assert err < 1e-4, err


def test_weighted_losses_empty_and_full_masks():
    for fill in (0.0, 1.0):
        y = torch.full((2, 32, 32), fill)
        _, p = blobs(2, 32, 32, 7)
        for bce, f in ((True, R.weighted_bce_dice_loss), (False, R.weighted_dice_loss)):
            loss, _ = M.weighted_loss_and_grad(y, p, bce=bce)
            ref = f(y, p).item()
            assert abs(loss - ref) <= 1e-5 * max(1.0, abs(ref)), (fill, bce, loss, ref)


def test_border_weight_map():
    y, _ = blobs(3, 50, 40, 5)
    wt, wsum = M.border_weight(y)
    ref = R.border_weight(y.double())[0]   # renormalised
    raw = wt.cpu().double()
    assert set(np.unique(raw.numpy()).tolist()) <= {1.0, 3.0}
    assert wsum.item() == raw.sum().item()
    got = raw * (raw.numel() / wsum.item())
    np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=1e-6)


def test_weighted_coeff_and_bce_with_explicit_weight():
    y, p = blobs(2, 48, 48, 8)
    g = torch.Generator().manual_seed(9)
    w = 0.5 + torch.rand(2, 48, 48, generator=g)
    c = M.weighted_dice_coeff(y, p, w)
    b = M.weighted_bce_loss(y, p, w)
    assert abs(c - R.weighted_dice_coeff(y.double(), p.double(), w.double()).item()) < 1e-6
    assert abs(b - R.weighted_bce_loss(y.double(), p.double(), w.double()).item()) < 1e-5


@pytest.mark.parametrize("B,H,W", [(2, 16, 64), (3, 7, 130), (1, 5, 3)])
def test_metric_helpers(B, H, W):
    y, p = blobs(B, H, W, 11)
    y[0, 0] = 0.0          # an all-zero row: argmax = argmin = 0 (first occurrence)
    p[0, 1, 1:3] = p[0, 1].max() + 1   # a tie for the maximum
    ref = R.metric_helpers(y, p)
    got = {"mean_diff": M.mean_diff(y, p), "act_mean": M.act_mean(y, p), "act_min": M.act_min(y, p),
           "act_max": M.act_max(y, p), "act_std": M.act_std(y, p), "tru_pos": M.tru_pos(y, p),
           "fls_pos": M.fls_pos(y, p), "tru_neg": M.tru_neg(y, p), "fls_neg": M.fls_neg(y, p),
           "precision_onehot": M.precision_onehot(y, p), "recall_onehot": M.recall_onehot(y, p),
           "fmeasure_onehot": M.fmeasure_onehot(y, p)}
    for k, v in ref.items():
        if isinstance(v, int):
            assert got[k] == v, (k, got[k], v)
        else:
            assert abs(got[k] - v) <= 1e-6 * max(1.0, abs(v)), (k, got[k], v)
