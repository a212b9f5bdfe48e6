"""The step after the rasterizer: fused L1 + MSE loss with its gradient,
and per-image PSNR, in one pass over the rendered and target images (dls_l1_mse_psnr).

References: loss_mse.py:33-44 (MSE term, `weight * (delta ** 2).mean()`), metrics.py:12-19
(`compute_psnr`). The L1 term stands in for LPIPS in the config-C step (VGG weights are not
available offline); either weight may be 0.
"""
from __future__ import annotations

import torch

from . import _lib


def _run(pred: torch.Tensor, target: torch.Tensor, w_l1: float, w_mse: float, want_grad: bool, want_psnr: bool):
    lib = _lib.load()
    _lib.require_gpu(pred, target)
    if pred.shape != target.shape:
        raise ValueError(f"prediction {tuple(pred.shape)} and target {tuple(target.shape)} differ")
    if pred.dim() < 3:
        raise ValueError("expected images [..., C, H, W]")
    p = pred.detach().contiguous().float()
    t = target.detach().contiguous().float()
    n_img = p[..., 0, 0, 0].numel()
    per = p.numel() // max(n_img, 1)
    dev = p.device
    loss = torch.empty((), dtype=torch.float32, device=dev)
    grad = torch.empty_like(p) if want_grad else None
    psnr = torch.empty(n_img, dtype=torch.float32, device=dev) if want_psnr else None
    ws = torch.empty(lib.dls_loss_workspace_size(n_img, per), dtype=torch.uint8, device=dev)
    _lib.check(lib.dls_l1_mse_psnr(n_img, per, p.data_ptr(), t.data_ptr(), float(w_l1), float(w_mse), loss.data_ptr(),
                                   None if grad is None else grad.data_ptr(),
                                   None if psnr is None else psnr.data_ptr(), ws.data_ptr(),
                                   _lib.stream_of(dev)), "dls_l1_mse_psnr")
    return loss, grad, psnr


class _L1MSE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, w_l1, w_mse):
        loss, grad, _ = _run(pred, target, w_l1, w_mse, pred.requires_grad, False)
        ctx.save_for_backward(grad if grad is not None else torch.empty(0, device=pred.device))
        ctx.shape_dtype = (pred.shape, pred.dtype)
        return loss

    @staticmethod
    def backward(ctx, gout):
        (grad,) = ctx.saved_tensors
        shape, dtype = ctx.shape_dtype
        return (grad * gout).reshape(shape).to(dtype), None, None, None


def l1_mse_loss(prediction: torch.Tensor, target: torch.Tensor, w_l1: float = 1.0, w_mse: float = 1.0):
    """w_l1 * mean|p - t| + w_mse * mean (p - t)^2 as a 0-d tensor; differentiable in p."""
    return _L1MSE.apply(prediction, target, float(w_l1), float(w_mse))


def psnr(ground_truth: torch.Tensor, predicted: torch.Tensor) -> torch.Tensor:
    """compute_psnr (metrics.py:12-19) per image over the leading dims: [..., C, H, W] -> [...]."""
    _, _, out = _run(predicted, ground_truth, 0.0, 0.0, False, True)
    return out.reshape(predicted.shape[:-3])
