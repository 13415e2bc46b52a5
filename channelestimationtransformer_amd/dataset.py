"""Channel tensors in the reference's layout, and a synthetic channel source.

Layout contract (``FullPrecision/dataset.py:20-51``): a complex channel
``H[B, T, Nr=2, Nt=4]`` becomes float32 ``[B, T, 16]`` with feature
``f = 2·(r·Nt + t) + {0: real, 1: imag}``.  ``channelnorm`` (``:77-88``) scales a
sample to unit mean power, ``noise`` (``:54-74``) adds complex AWGN of variance
``10^(-SNR/10)`` times the sample's mean power, and ``SeqData.__getitem__``
(``:124-152``) windows ``seq_len + pred_len`` slots: the model sees the *noisy*
first ``seq_len`` slots and is scored on the *clean* last ``pred_len``.

The reference's datasets (Sionna CDL-B pickles) are absent, so
:func:`synthetic_channels` draws a seeded sum-of-sinusoids (Jakes) Doppler
process per antenna pair instead.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np


def LoadBatch(H):
    """complex ``[M, T, Nr, Nt]`` → float32 torch ``[M, T, Nr·Nt·2]`` (dataset.py:20-44)."""
    import torch

    H = np.asarray(H)
    M, T, Nr, Nt = H.shape
    Hf = H.reshape(M, T, Nr * Nt)
    out = np.empty((M, T, Nr * Nt, 2), dtype=np.float64)
    out[..., 0] = Hf.real
    out[..., 1] = Hf.imag
    return torch.tensor(out.reshape(M, T, Nr * Nt * 2), dtype=torch.float32)


def load_batch_np(H: np.ndarray) -> np.ndarray:
    """numpy form of :func:`LoadBatch` (float32)."""
    M, T, Nr, Nt = H.shape
    Hf = H.reshape(M, T, Nr * Nt)
    out = np.empty((M, T, Nr * Nt, 2), dtype=np.float32)
    out[..., 0] = Hf.real
    out[..., 1] = Hf.imag
    return out.reshape(M, T, Nr * Nt * 2)


def real2complex(data: np.ndarray) -> np.ndarray:
    """Inverse of the interleave (dataset.py:47-51)."""
    B, P, N = data.shape
    d = np.asarray(data).reshape(B, P, N // 2, 2)
    return d[..., 0] + 1j * d[..., 1]


def channelnorm(H: np.ndarray) -> np.ndarray:
    """Unit mean power over the whole sample (dataset.py:77-88)."""
    return H / np.sqrt(np.mean(np.abs(H) ** 2))


def noise(H: np.ndarray, SNR: float, rng: np.random.Generator) -> np.ndarray:
    """Complex AWGN at ``SNR`` dB relative to the sample power (dataset.py:54-74)."""
    sigma = 10 ** (-SNR / 10)
    n = np.sqrt(sigma / 2) * (rng.standard_normal(H.shape) + 1j * rng.standard_normal(H.shape))
    return H + n * np.sqrt(np.mean(np.abs(H) ** 2))


def synthetic_channels(n: int, slots: int = 95, nr: int = 2, nt: int = 4, seed: int = 1234,
                       doppler: float = 0.02, paths: int = 16) -> np.ndarray:
    """Seeded Jakes process ``H[n, slots, nr, nt]`` (complex64), each sample unit power.

    ``H[s, t, r, a] = Σ_p g_p · exp(j(2π·doppler·cos(α_p)·t + φ_p)) / sqrt(paths)`` with
    per-(sample, antenna-pair) random arrival angles ``α``, phases ``φ`` and complex
    path gains ``g``; ``doppler`` is the normalised maximum Doppler ``f_D·T_slot``.
    """
    rng = np.random.default_rng(seed)
    t = np.arange(slots, dtype=np.float64)
    alpha = rng.uniform(0, 2 * np.pi, size=(n, nr, nt, paths))
    phi = rng.uniform(0, 2 * np.pi, size=(n, nr, nt, paths))
    g = (rng.standard_normal((n, nr, nt, paths)) + 1j * rng.standard_normal((n, nr, nt, paths))) / np.sqrt(2)
    ph = 2 * np.pi * doppler * np.cos(alpha)[..., None] * t + phi[..., None]  # [n,nr,nt,p,T]
    H = np.sum(g[..., None] * np.exp(1j * ph), axis=3) / np.sqrt(paths)     # [n,nr,nt,T]
    H = np.transpose(H, (0, 3, 1, 2))
    H = H / np.sqrt(np.mean(np.abs(H) ** 2, axis=(1, 2, 3), keepdims=True))
    return H.astype(np.complex64)


def make_batch(n: int, seq_len: int = 90, label_len: int = 10, pred_len: int = 5, snr: float = 20.0,
               seed: int = 1234, doppler: float = 0.02) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Synthetic ``(x_enc[n,seq_len,16], x_dec[n,label_len+pred_len,16], label[n,pred_len,16])``.

    Mirrors ``SeqData.__getitem__`` (dataset.py:137-150) with the window fixed at
    slot 0, and the caller-side decoder input of ``run_validation``
    (``QuantizationAwareTraining.py:103-114``): the last ``label_len`` encoder
    slots followed by ``pred_len`` zero slots.
    """
    rng = np.random.default_rng(seed + 1)
    H = synthetic_channels(n, seq_len + pred_len, seed=seed, doppler=doppler)
    Hn = np.stack([noise(channelnorm(h), snr, rng) for h in H]) if n else H
    x_enc = load_batch_np(Hn[:, :seq_len])
    label = load_batch_np(H[:, seq_len:seq_len + pred_len])
    x_dec = decoder_input(x_enc, seq_len, label_len, pred_len)
    return x_enc, x_dec, label


def decoder_input(x_enc: np.ndarray, seq_len: int, label_len: int, pred_len: int) -> np.ndarray:
    """``cat(x_enc[:, seq_len-label_len:seq_len], zeros[pred_len])`` (QuantizationAwareTraining.py:103-114)."""
    B, _, C = x_enc.shape
    return np.concatenate([x_enc[:, seq_len - label_len:seq_len],
                           np.zeros((B, pred_len, C), dtype=x_enc.dtype)], axis=1).astype(np.float32)
