"""Fused loss / PSNR kernel (dls_l1_mse_psnr) vs the reference's torch formulas
(loss_mse.py:33-44, metrics.py:12-19) in fp32 on the same device."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(2, 3, 3, 17, 23), (4, 3, 64, 64), (1, 3, 256, 256)])
@pytest.mark.parametrize("w", [(1.0, 1.0), (0.0, 0.05), (2.0, 0.0)])
def test_loss_and_grad_match_torch(gpu, shape, w):
    from my_depthsplat_amd.loss import l1_mse_loss
    g = torch.Generator(device=gpu).manual_seed(1)
    pred = (torch.rand(shape, generator=g, device=gpu) * 1.4 - 0.2).requires_grad_(True)
    tgt = torch.rand(shape, generator=g, device=gpu)
    tgt.view(-1)[:7] = pred.detach().view(-1)[:7]  # exact zeros of the difference (sign(0) = 0)
    w1, w2 = w
    ref = pred.detach().clone().requires_grad_(True)
    d = ref - tgt
    lr = w1 * d.abs().mean() + w2 * (d ** 2).mean()
    lr.backward()
    lh = l1_mse_loss(pred, tgt, w1, w2)
    (lh * 3.0).backward()
    torch.testing.assert_close(lh, lr.detach(), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(pred.grad, 3.0 * ref.grad, rtol=1e-5, atol=1e-9)


def test_psnr_matches_compute_psnr(gpu):
    from my_depthsplat_amd.loss import psnr
    g = torch.Generator(device=gpu).manual_seed(2)
    gt = torch.rand(5, 3, 40, 30, generator=g, device=gpu)
    pr = gt + 0.05 * torch.randn(gt.shape, generator=g, device=gpu)
    ref = -10 * ((gt.clip(0, 1) - pr.clip(0, 1)) ** 2).mean(dim=(1, 2, 3)).log10()
    torch.testing.assert_close(psnr(gt, pr), ref, rtol=1e-5, atol=1e-4)


def test_loss_is_deterministic(gpu):
    from my_depthsplat_amd.loss import l1_mse_loss
    g = torch.Generator(device=gpu).manual_seed(3)
    a = torch.rand(8, 3, 128, 128, generator=g, device=gpu)
    b = torch.rand(8, 3, 128, 128, generator=g, device=gpu)
    vals = {float(l1_mse_loss(a, b)) for _ in range(5)}
    assert len(vals) == 1
