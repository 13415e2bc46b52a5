"""NMSELoss / NMSELossSplit (FullPrecision/metrics.py:5-39) with the split form on the engine.

Argument order and normalisation follow the reference exactly: ``NMSE_cuda(x_hat, x)``
normalises by the SECOND argument's power, ``NMSE_Split_cuda(x_hat, x)`` by the FIRST's
(run_validation passes the model output first).  The split form runs the HIP
``cet_nmse_split`` kernel for fp32 tensors on a HIP device.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .engine import nmse_split


def NMSE_cuda(x_hat, x):
    """metrics.py:5-9."""
    return torch.sum((x - x_hat) ** 2) / torch.sum(x ** 2)


class NMSELoss(nn.Module):
    """metrics.py:12-23."""

    def __init__(self, reduction="mean"):
        super().__init__()
        self.reduction = reduction

    def forward(self, x_hat, x):
        n = NMSE_cuda(x_hat, x)
        return torch.mean(n) if self.reduction == "mean" else torch.sum(n)


def NMSE_Split_cuda(x_hat, x):
    """metrics.py:26-30 → ``[pred_len]``: Σ_{b,f}(x-x̂)² / Σ_{b,f} x̂²  (HIP kernel)."""
    if not (x_hat.is_cuda and x.is_cuda):
        raise RuntimeError("NMSE_Split_cuda runs on the HIP device (no CPU fallback)")
    return nmse_split(x_hat.float().contiguous(), x.float().contiguous())


class NMSELossSplit(nn.Module):
    """metrics.py:33-39."""

    def __init__(self, reduction="mean"):
        super().__init__()
        self.reduction = reduction

    def forward(self, x_hat, x):
        return NMSE_Split_cuda(x_hat, x)
