"""PSNR as defined by the reference (src/evaluation/metrics.py:12-19)."""
from __future__ import annotations

import torch


@torch.no_grad()
def compute_psnr(ground_truth: torch.Tensor, predicted: torch.Tensor) -> torch.Tensor:
    """[b, c, h, w] x2 -> [b]: clip both to [0, 1], -10 log10(mean squared error).
    Device tensors: one fused HIP pass (my_depthsplat_amd.loss.psnr); host tensors: torch."""
    if ground_truth.is_cuda:
        from .loss import psnr
        return psnr(ground_truth, predicted)
    gt = ground_truth.clip(min=0, max=1)
    pr = predicted.clip(min=0, max=1)
    mse = ((gt - pr) ** 2).flatten(1).mean(dim=1)
    return -10 * mse.log10()
