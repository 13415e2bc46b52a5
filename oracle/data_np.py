"""CPU ORACLE (test infrastructure only) — the reference's per-sample data path.

Restates, in numpy float64:

* ``SeqData.__getitem__`` (FullPrecision/dataset.py:124-152): ``channelnorm`` over the whole
  sample (:77-88), complex AWGN ``sqrt(σ/2)·(re + j·im)·sqrt(mean|Hn|²)`` with σ = 10^(-SNR/10)
  (:54-74), the ``seq_len + pred_len`` window at ``start``; the model input is the noisy
  ``H_seq``, the target the clean ``H_pred``;
* ``LoadBatch`` (:20-44): feature ``2·(r·Nt + t) + {re, im}``;
* the callers' decoder input (QuantizationAwareTraining.py:97-114): the last ``label_len``
  encoder slots followed by ``pred_len`` zero slots;
* the seeded Jakes channel source that stands in for the absent CDL pickles (our own stand-in,
  no reference counterpart: ``out = Σ_p g·exp(j(2π·f_D·cos α·t + φ))/sqrt(P)``, unit power).

The random draws (``np.random.randint`` window start, the two ``torch.randn`` arrays) are
explicit inputs.  Pinned by tests/golden/data_seqdata.npz, produced by running the reference's
own ``SeqData.__getitem__`` and ``LoadBatch`` (tests/golden/make_data_golden.py).  Only tests
and bench's cpu_baseline may import this module.
"""
from __future__ import annotations

import numpy as np


def get_item(H, start, re, im, snr, seq_len, pred_len):
    """One ``SeqData.__getitem__`` (dataset.py:133-152) with explicit draws → (H_win, Hnoise_win, H_seq, H_pred)."""
    H = np.asarray(H, np.complex128)
    Hn = H / np.sqrt(np.mean(np.abs(H) ** 2))                                   # channelnorm
    sigma = 10 ** (-snr / 10)
    noise = np.sqrt(sigma / 2) * (np.asarray(re, np.float64) + 1j * np.asarray(im, np.float64))
    Hnoise = Hn + noise * np.sqrt(np.mean(np.abs(Hn) ** 2))                     # noise()
    L = seq_len + pred_len
    Hw, Hnw = Hn[start:start + L], Hnoise[start:start + L]
    return Hw, Hnw, Hnw[:seq_len], Hw[seq_len:]


def load_batch(H):
    """complex ``[M, T, Nr, Nt]`` → ``[M, T, 2·Nr·Nt]`` (dataset.py:37-44)."""
    H = np.asarray(H)
    M, T, Nr, Nt = H.shape
    out = np.empty((M, T, Nr * Nt, 2), np.float64)
    out[..., 0] = H.reshape(M, T, Nr * Nt).real
    out[..., 1] = H.reshape(M, T, Nr * Nt).imag
    return out.reshape(M, T, Nr * Nt * 2)


def decoder_input(x_enc, seq_len, label_len, pred_len):
    """``cat(x_enc[:, seq_len-label_len:seq_len], zeros)`` (QuantizationAwareTraining.py:101-114)."""
    B, _, C = x_enc.shape
    return np.concatenate([x_enc[:, seq_len - label_len:seq_len], np.zeros((B, pred_len, C))], axis=1)


def prepare_batch(dataset, idx, starts, re, im, snr, seq_len, label_len, pred_len):
    """A DataLoader batch of ``get_item`` + ``LoadBatch`` + decoder input → (x_enc, x_dec, label)."""
    seqs, preds = [], []
    for b, s in enumerate(idx):
        _, _, h_seq, h_pred = get_item(dataset[s], int(starts[b]), re[b], im[b], snr, seq_len, pred_len)
        seqs.append(h_seq)
        preds.append(h_pred)
    x_enc = load_batch(np.stack(seqs))
    label = load_batch(np.stack(preds))
    return x_enc, decoder_input(x_enc, seq_len, label_len, pred_len), label


def jakes(alpha, phi, gain, slots, doppler):
    """``out[s, t, e] = Σ_p gain·exp(j(2π·doppler·cos α·t + φ)) / sqrt(P)`` then unit mean power per sample.

    alpha, phi: ``[n, E, P]``; gain complex ``[n, E, P]`` → complex ``[n, slots, E]``.
    """
    alpha = np.asarray(alpha, np.float64)
    phi = np.asarray(phi, np.float64)
    gain = np.asarray(gain, np.complex128)
    t = np.arange(slots, dtype=np.float64)
    ph = 2 * np.pi * doppler * np.cos(alpha)[..., None] * t + phi[..., None]        # [n, E, P, T]
    H = np.sum(gain[..., None] * np.exp(1j * ph), axis=2) / np.sqrt(alpha.shape[-1])  # [n, E, T]
    H = np.transpose(H, (0, 2, 1))
    return H / np.sqrt(np.mean(np.abs(H) ** 2, axis=(1, 2), keepdims=True))
