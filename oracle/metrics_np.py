"""CPU ORACLE (test infrastructure only) — NMSE reductions of ``FullPrecision/metrics.py``."""
from __future__ import annotations

import numpy as np


def nmse(x_hat, x):
    """NMSE_cuda (metrics.py:5-9): ``Σ(x-x̂)² / Σx²`` (normalised by the SECOND argument)."""
    x_hat = np.asarray(x_hat, np.float64)
    x = np.asarray(x, np.float64)
    return np.sum((x - x_hat) ** 2) / np.sum(x ** 2)


def nmse_split(x_hat, x):
    """NMSE_Split_cuda (metrics.py:26-30): per prediction step, normalised by the FIRST argument.

    ``power = Σ_{b,f} x̂²``, ``mse = Σ_{b,f} (x - x̂)²`` over dims (0, 2) → ``[pred_len]``.
    """
    x_hat = np.asarray(x_hat, np.float64)
    x = np.asarray(x, np.float64)
    return np.sum((x - x_hat) ** 2, axis=(0, 2)) / np.sum(x_hat ** 2, axis=(0, 2))


def to_db(v):
    """``10·log10`` as the comparison plots do (makePlots.py:31)."""
    return 10.0 * np.log10(np.asarray(v, np.float64))
