"""Device channel pipeline: ``SeqData`` + ``LoadBatch`` + decoder input on the GPU.

``DeviceSeqData`` mirrors ``SeqData`` (FullPrecision/dataset.py:92-152): it holds the complex
channel dataset ``[N, slots, Nr, Nt]`` resident in HBM, and :meth:`DeviceSeqData.batch` turns B
sample indices into the model's ``(x_enc, x_dec, label)`` in one HIP launch
(``cet_prepare_batch``): window, ``channelnorm``, complex AWGN, ``LoadBatch`` interleave and the
callers' decoder input (QuantizationAwareTraining.py:97-114).

Randomness:

* default — device Philox4x32-10 keyed by ``(seed, counter)``: window starts and the noise
  normals are drawn inside the kernel, nothing crosses PCIe;
* :meth:`DeviceSeqData.reference_batch` — the reference's own protocol: ``np.random.randint``
  per sample from numpy's global RNG and the two ``torch.randn(*H.shape)`` arrays of ``noise``
  from torch's global generator, drawn on the host in ``__getitem__`` order and uploaded
  (parity mode).

:func:`synth_channels` builds the seeded Jakes stand-in for the absent CDL pickles on the device
(``cet_synth_channels``) from host-drawn parameters (the recipe of ``dataset.synthetic_channels``).
The product path has no CPU fallback: without the HIP library the import fails.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from ._lib import check, lib


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(device):
    import torch

    return torch.cuda.current_stream(device).cuda_stream


def synth_channels(n: int, slots: int = 100, nr: int = 2, nt: int = 4, seed: int = 1234, doppler: float = 0.02,
                   paths: int = 16, device=None):
    """Seeded Jakes channels on the device → complex64 tensor ``[n, slots, nr, nt]`` (unit power per sample)."""
    import torch

    device = device or torch.device("cuda", torch.cuda.current_device())
    rng = np.random.default_rng(seed)
    E = nr * nt
    alpha = rng.uniform(0, 2 * np.pi, size=(n, E, paths)).astype(np.float32)
    phi = rng.uniform(0, 2 * np.pi, size=(n, E, paths)).astype(np.float32)
    gain = ((rng.standard_normal((n, E, paths)) + 1j * rng.standard_normal((n, E, paths))) / np.sqrt(2)).astype(
        np.complex64)
    a = torch.from_numpy(alpha).to(device)
    p = torch.from_numpy(phi).to(device)
    g = torch.view_as_real(torch.from_numpy(gain)).contiguous().to(device)
    out = torch.empty(n, slots, nr, nt, dtype=torch.complex64, device=device)
    check(lib.cet_synth_channels(_ptr(a), _ptr(p), _ptr(g), n, slots, nr, nt, paths, float(doppler), _ptr(out),
                                 ctypes.c_void_p(_stream(device))), "cet_synth_channels")
    return out


def reference_draws(B: int, slots: int, nr: int, nt: int, length: int) -> Tuple[np.ndarray, np.ndarray]:
    """The draws B consecutive ``SeqData.__getitem__`` calls make from the global RNGs: the window
    start ``np.random.randint(0, slots - length + 1)`` (dataset.py:142) from numpy's legacy
    generator, and per sample the two ``torch.randn(*H.shape)`` arrays of ``noise`` (:65-66)
    → (starts [B] int32, noise [B, slots, nr, nt, 2] float32)."""
    import torch

    starts = np.empty(B, np.int32)
    noise = np.empty((B, slots, nr, nt, 2), np.float32)
    for b in range(B):
        starts[b] = np.random.randint(0, slots - length + 1)
        noise[b, ..., 0] = torch.randn(slots, nr, nt).numpy()
        noise[b, ..., 1] = torch.randn(slots, nr, nt).numpy()
    return starts, noise


class DeviceSeqData:
    """Device-resident ``SeqData(dataset, seq_len, pred_len, SNR)`` (FullPrecision/dataset.py:92-152).

    ``dataset`` — complex ``[N, slots, Nr, Nt]`` numpy array or torch tensor (moved to ``device``
    as complex64).  ``label_len`` sets the decoder input the callers build.
    """

    def __init__(self, dataset, seq_len: int, pred_len: int, SNR: float = 20, label_len: int = 10, device=None):
        import torch

        self.device = device or torch.device("cuda", torch.cuda.current_device())
        if not isinstance(dataset, torch.Tensor):
            dataset = torch.from_numpy(np.ascontiguousarray(np.asarray(dataset, np.complex64)))
        if dataset.dim() != 4 or not dataset.is_complex():
            raise ValueError("dataset must be complex [N, slots, Nr, Nt]")
        self.dataset = dataset.to(self.device, torch.complex64).contiguous()
        self.N, self.slots, self.nr, self.nt = self.dataset.shape
        self.seq_len, self.pred_len, self.label_len = seq_len, pred_len, label_len
        self.length = seq_len + pred_len
        self.SNR = SNR
        if self.slots < self.length:
            raise ValueError(f"samples have {self.slots} slots < seq_len + pred_len = {self.length}")

    def __len__(self) -> int:
        return self.N

    @property
    def features(self) -> int:
        return 2 * self.nr * self.nt

    def batch(self, idx=None, sample_base: int = 0, B: Optional[int] = None, starts=None, noise=None, seed: int = 0,
              counter: int = 0, snr: Optional[float] = None, out=None, stream: Optional[int] = None,
              return_starts: bool = False):
        """``(x_enc, x_dec, label)`` fp32 device tensors for samples ``idx`` (int32 device/host) or
        ``sample_base .. sample_base+B``; explicit ``starts`` [B] / ``noise`` [B, slots, Nr, Nt, 2]
        replace the device draws.  ``out`` may pass preallocated (x_enc, x_dec, label)."""
        import torch

        dev = self.device
        if idx is not None:
            idx = torch.as_tensor(idx, dtype=torch.int32).to(dev).contiguous()
            B = int(idx.numel())
        elif B is None:
            raise ValueError("give idx or B")
        if starts is not None:
            starts = torch.as_tensor(starts, dtype=torch.int32).to(dev).contiguous()
        if noise is not None:
            noise = torch.as_tensor(noise, dtype=torch.float32).to(dev).contiguous()
            if noise.numel() != B * self.slots * self.nr * self.nt * 2:
                raise ValueError("noise must be [B, slots, Nr, Nt, 2]")
        F = self.features
        if out is None:
            out = (torch.empty(B, self.seq_len, F, device=dev), torch.empty(B, self.label_len + self.pred_len, F, device=dev),
                   torch.empty(B, self.pred_len, F, device=dev))
        x_enc, x_dec, label = out
        st_out = torch.empty(B, dtype=torch.int32, device=dev) if return_starts else None
        if stream is None:
            stream = _stream(dev)
        check(lib.cet_prepare_batch(_ptr(torch.view_as_real(self.dataset)), self.N, self.slots, self.nr, self.nt,
                                    _ptr(idx), int(sample_base), _ptr(starts), _ptr(noise), int(seed) & (2 ** 64 - 1),
                                    int(counter) & (2 ** 64 - 1), B, self.seq_len, self.label_len, self.pred_len,
                                    float(self.SNR if snr is None else snr), _ptr(x_enc), _ptr(x_dec), _ptr(label),
                                    _ptr(st_out), ctypes.c_void_p(stream)), "cet_prepare_batch")
        return (x_enc, x_dec, label, st_out) if return_starts else (x_enc, x_dec, label)

    def reference_draws(self, B: int) -> Tuple[np.ndarray, np.ndarray]:
        """See :func:`reference_draws`."""
        return reference_draws(B, self.slots, self.nr, self.nt, self.length)

    def reference_batch(self, idx, **kw):
        """Parity mode: the reference's RNG protocol (global numpy + torch generators), device math."""
        idx = np.asarray(idx)
        starts, noise = self.reference_draws(len(idx))
        return self.batch(idx=idx, starts=starts, noise=noise, **kw)
