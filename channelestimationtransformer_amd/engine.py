"""Thin object wrapper over one C-ABI engine handle (include/cet.h).

torch is used only as plumbing: device buffers, the current HIP stream, and the
global CPU generator for the reference's ProbSparse RNG protocol.
"""
from __future__ import annotations

import ctypes
import json
from typing import Dict, List, Mapping, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import check, lib


def _stream_ptr(device) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream


class Engine:
    """Owns a ``cet_engine*``; weights by reference key name; forward on device tensors."""

    def __init__(self, handle: int, kind: str):
        self._h = ctypes.c_void_p(handle)
        self.kind = kind
        self._dbg = None

    @classmethod
    def informer(cls, cfg: "_lib.InformerConfig") -> "Engine":
        h = ctypes.c_void_p()
        check(lib.cet_create_informer(ctypes.byref(cfg), ctypes.byref(h)), "cet_create_informer")
        return cls(h.value, "informer")

    @classmethod
    def transformer(cls, cfg: "_lib.TransformerConfig") -> "Engine":
        h = ctypes.c_void_p()
        check(lib.cet_create_transformer(ctypes.byref(cfg), ctypes.byref(h)), "cet_create_transformer")
        return cls(h.value, "transformer")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.cet_destroy(h)
            self._h = ctypes.c_void_p()

    # ------------------------------------------------------------------ weights
    def load_state_dict(self, state: Mapping[str, object], strict: bool = False) -> List[str]:
        """Push every tensor of ``state`` (reference key names).  Unknown keys raise if strict."""
        unexpected = []
        for k, v in state.items():
            a = np.ascontiguousarray(_to_numpy(v), dtype=np.float32)
            rc = lib.cet_load_weight(self._h, k.encode(), a.ctypes.data_as(ctypes.c_void_p), a.size)
            if rc < 0:
                if strict or "size mismatch" in lib.cet_last_error().decode():
                    check(rc, f"load {k}")
                unexpected.append(k)
        return unexpected

    def missing(self) -> Tuple[int, str]:
        buf = ctypes.create_string_buffer(512)
        n = check(lib.cet_missing_weights(self._h, buf, 512), "cet_missing_weights")
        return n, buf.value.decode()

    # ------------------------------------------------------------------ ProbSparse sampling
    def prob_calls(self) -> List[Tuple[int, Tuple[int, int]]]:
        n = check(lib.cet_prob_calls(self._h, None, 0))
        arr = (ctypes.c_int * (3 * max(n, 1)))()
        check(lib.cet_prob_calls(self._h, arr, n))
        return [(arr[3 * i], (arr[3 * i + 1], arr[3 * i + 2])) for i in range(n)]

    def set_indices(self, idx: Sequence[np.ndarray]) -> None:
        for k, a in enumerate(idx):
            a = np.ascontiguousarray(a, dtype=np.int32)
            check(lib.cet_set_prob_indices(self._h, k, a.ctypes.data_as(ctypes.c_void_p), a.shape[0], a.shape[1]),
                  "cet_set_prob_indices")

    def native_draw(self) -> List[np.ndarray]:
        """Next forward's draws from the native sampler (advances it), split per call."""
        n = check(lib.cet_native_draw(self._h, None, 0), "cet_native_draw")
        buf = np.empty(max(n, 1), dtype=np.int32)
        check(lib.cet_native_draw(self._h, buf.ctypes.data_as(ctypes.c_void_p), n), "cet_native_draw")
        out, k = [], 0
        for _, (lq, u) in self.prob_calls():
            out.append(buf[k:k + lq * u].reshape(lq, u))
            k += lq * u
        return out

    def peek_draw(self) -> List[np.ndarray]:
        """The draws the next native forward will consume, without advancing the stream."""
        n = check(lib.cet_peek_draw(self._h, None, 0), "cet_peek_draw")
        buf = np.empty(max(n, 1), dtype=np.int32)
        check(lib.cet_peek_draw(self._h, buf.ctypes.data_as(ctypes.c_void_p), n), "cet_peek_draw")
        out, k = [], 0
        for _, (lq, u) in self.prob_calls():
            out.append(buf[k:k + lq * u].reshape(lq, u))
            k += lq * u
        return out

    def seed(self, seed: int) -> None:
        check(lib.cet_seed(self._h, ctypes.c_uint64(int(seed) & (2 ** 64 - 1))), "cet_seed")

    # ------------------------------------------------------------------ forward
    def forward(self, x_enc, x_dec, out, attns=None, stream: Optional[int] = None) -> None:
        """All arguments are contiguous float32 torch tensors on the same HIP device."""
        B = int(x_enc.shape[0])
        if stream is None:
            stream = _stream_ptr(x_enc.device)
        check(lib.cet_forward(self._h, ctypes.c_void_p(x_enc.data_ptr()), ctypes.c_void_p(x_dec.data_ptr()), B,
                              ctypes.c_void_p(out.data_ptr()),
                              ctypes.c_void_p(attns.data_ptr()) if attns is not None else None,
                              ctypes.c_void_p(stream)), "cet_forward")

    def forward_nmse(self, x_enc, x_dec, out, label, nmse_acc=None, nmse_sums=None, stream: Optional[int] = None):
        """Forward + NMSE_Split(out, label) in one launch (cet_forward_nmse): ``nmse_acc`` float32 [T] += the
        batch's ratio, ``nmse_sums`` float64 [2, T] = its raw sums (either may be None, not both)."""
        import torch

        B, T = int(x_enc.shape[0]), int(out.shape[1])
        if tuple(label.shape) != tuple(out.shape) or label.dtype != torch.float32 or not label.is_contiguous():
            raise ValueError("label must be a contiguous float32 tensor shaped like out")
        if nmse_acc is not None and (nmse_acc.dtype != torch.float32 or nmse_acc.numel() != T):
            raise ValueError(f"nmse_acc must be float32 [{T}]")
        if nmse_sums is not None and (nmse_sums.dtype != torch.float64 or nmse_sums.numel() != 2 * T
                                      or not nmse_sums.is_contiguous()):
            raise ValueError(f"nmse_sums must be a contiguous float64 [2, {T}]")
        if stream is None:
            stream = _stream_ptr(x_enc.device)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        check(lib.cet_forward_nmse(self._h, ptr(x_enc), ptr(x_dec), B, ptr(out), ptr(label), ptr(nmse_acc),
                                   ptr(nmse_sums), ctypes.c_void_p(stream)), "cet_forward_nmse")

    def bind_forward_nmse(self, x_enc, x_dec, out, label, nmse_sums, stream: Optional[int] = None):
        """A step function for a loop over fixed device buffers: ``step(k)`` runs ``forward_nmse`` with the
        raw sums going to ``nmse_sums[k]`` (float64 [steps, 2, T]), the argument checks and pointer
        conversions done once here instead of per step (the host cost of a step stays far below the
        kernel's even on a loaded host)."""
        import torch

        B, T = int(x_enc.shape[0]), int(out.shape[1])
        if tuple(label.shape) != tuple(out.shape) or label.dtype != torch.float32 or not label.is_contiguous():
            raise ValueError("label must be a contiguous float32 tensor shaped like out")
        if nmse_sums.dtype != torch.float64 or not nmse_sums.is_contiguous() or tuple(nmse_sums.shape[1:]) != (2, T):
            raise ValueError(f"nmse_sums must be a contiguous float64 [steps, 2, {T}]")
        for t in (x_enc, x_dec, out):
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError("x_enc, x_dec and out must be contiguous float32")
        if int(x_dec.shape[0]) != B or int(out.shape[0]) != B:
            raise ValueError("x_enc, x_dec and out must have the same batch size")
        dev = x_enc.device
        for t in (x_dec, out, label, nmse_sums):
            if t.device != dev or not t.is_cuda:
                raise ValueError(f"every tensor must be on the engine's device {dev}")
        if stream is None:
            stream = _stream_ptr(x_enc.device)
        f, h = lib.cet_forward_nmse, self._h
        args = [ctypes.c_void_p(t.data_ptr()) for t in (x_enc, x_dec)] + [B] + \
               [ctypes.c_void_p(t.data_ptr()) for t in (out, label)] + [None]
        s0, stride, n = nmse_sums.data_ptr(), 2 * T * 8, int(nmse_sums.shape[0])
        st = ctypes.c_void_p(stream)
        # the step keeps the engine and every bound tensor alive: the launch writes through raw pointers
        keep = (self, x_enc, x_dec, out, label, nmse_sums)

        def step(k: int) -> None:
            if not 0 <= k < n:
                raise IndexError(k)
            rc = f(h, *args, s0 + k * stride, st)
            if rc < 0:
                check(rc, "cet_forward_nmse")

        step.keepalive = keep
        return step

    def attns_floats(self) -> int:
        return check(lib.cet_attns_floats(self._h), "cet_attns_floats")

    def attns_layout(self) -> List[Tuple[int, int]]:
        n = check(lib.cet_attns_layout(self._h, None, None, 0))
        offs = (ctypes.c_int64 * max(n, 1))()
        lens = (ctypes.c_int * max(n, 1))()
        check(lib.cet_attns_layout(self._h, offs, lens, n))
        return [(offs[i], lens[i]) for i in range(n)]

    def set_stamps(self, buf) -> None:
        """Diagnostics: per-phase s_memtime stamps into an int64 device tensor of B·128 (or None)."""
        check(lib.cet_set_stamps(self._h, ctypes.c_void_p(buf.data_ptr()) if buf is not None else None))

    def set_sampler(self, on_host: bool) -> None:
        """Native ProbSparse draws on the host (True) or the device-resident sampler (False)."""
        check(lib.cet_set_sampler(self._h, int(bool(on_host))), "cet_set_sampler")

    def set_variant(self, variant: int) -> None:
        """Fused-kernel generation: 4, the only one kept (one sequence per workgroup; every precision policy
        and the diagnostic outputs); 1-3 and 5 are retired (CET_E_INVALID)."""
        check(lib.cet_set_variant(self._h, int(variant)), "cet_set_variant")

    PATHS = {0: None, 3: "layerwise", 4: "v4", 31: "layerwise-fused", 41: "v4-split"}

    def last_path(self):
        """The kernel path the last Informer forward took: "v4", "v4-split", "layerwise" (operator
        launches), "layerwise-fused" (the layer-wise forward in one launch) or None."""
        return self.PATHS[check(lib.cet_last_path(self._h), "cet_last_path")]

    def last_kernel(self) -> str:
        """The kernel instance the last forward launched, as rocprofv3 names it (include/cet.h
        cet_last_kernel), e.g. "cet::v4::informer_forward_v4<64, false, 0, false, 1, false, false, 0>" (C2; the fifth
        argument is the compile-time row shape: 0 generic, 1 C2, 2 the e_layers [4, 3] stack; the last, the
        decoder on the LDS-DMA weight feed)."""
        n = check(lib.cet_last_kernel(self._h, None, 0), "cet_last_kernel")
        buf = ctypes.create_string_buffer(n + 1)
        check(lib.cet_last_kernel(self._h, buf, n + 1), "cet_last_kernel")
        return buf.value.decode()

    PRECISIONS = {"auto": -1, "bf16": 0, "split-bf16": 1, "fp8": 2, "fp32-layerwise": 3, "mixed": 4}

    def set_precision(self, prec) -> None:
        """Dense-layer operand precision of the v4 kernel: "auto", "bf16", "split-bf16", "fp8" or "mixed" (a bf16
        encoder with a split-bf16 decoder; include/cet.h).
        Engines on the layer-wise path (shapes outside the fused kernels) report "fp32-layerwise"."""
        code = self.PRECISIONS[prec] if isinstance(prec, str) else int(prec)
        check(lib.cet_set_precision(self._h, code), "cet_set_precision")

    def precision(self) -> str:
        code = check(lib.cet_get_precision(self._h), "cet_get_precision")
        return {v: k for k, v in self.PRECISIONS.items()}[code]

    # ------------------------------------------------------------------ kernel timing
    def timing(self, enable, every: int = 1) -> None:
        """Bracket one forward kernel launch in every ``every`` with hipEvents (off: enable=False)."""
        check(lib.cet_timing(self._h, max(1, int(every)) if enable else 0), "cet_timing")

    def timing_read(self) -> Tuple[float, int]:
        """(summed kernel milliseconds, launches) since ``timing(True)``."""
        ms = ctypes.c_double()
        n = ctypes.c_int64()
        check(lib.cet_timing_read(self._h, ctypes.byref(ms), ctypes.byref(n)), "cet_timing_read")
        return ms.value, n.value

    # ------------------------------------------------------------------ debug dumps
    def debug_floats(self) -> int:
        return check(lib.cet_debug_floats(self._h), "cet_debug_floats")

    def debug_layout(self) -> dict:
        n = check(lib.cet_debug_layout(self._h, None, 0))
        buf = ctypes.create_string_buffer(n + 1)
        check(lib.cet_debug_layout(self._h, buf, n + 1))
        return json.loads(buf.value.decode())

    def set_debug(self, buf) -> None:
        self._dbg = buf
        check(lib.cet_set_debug(self._h, ctypes.c_void_p(buf.data_ptr()) if buf is not None else None))


def nmse_split(pred, label, out=None, accumulate: bool = False, stream: Optional[int] = None):
    """Device NMSE_Split_cuda(pred, label) → fp32 tensor [T] (FullPrecision/metrics.py:26-30)."""
    import torch

    if pred.dim() != 3 or tuple(label.shape) != tuple(pred.shape):
        raise ValueError(f"pred and label must both be [B, T, F]; got {tuple(pred.shape)} and {tuple(label.shape)}")
    for name, t in (("pred", pred), ("label", label)):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.device != pred.device or not t.is_cuda:
            raise ValueError(f"{name} must be a contiguous float32 tensor on the same HIP device")
    B, T, F = pred.shape
    if out is None:
        out = torch.zeros(T, dtype=torch.float32, device=pred.device)
    elif out.dtype != torch.float32 or out.numel() != T or out.device != pred.device or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous float32 tensor of {T} elements on {pred.device}")
    if stream is None:
        stream = _stream_ptr(pred.device)
    check(lib.cet_nmse_split(ctypes.c_void_p(pred.data_ptr()), ctypes.c_void_p(label.data_ptr()), B, T, F,
                             ctypes.c_void_p(out.data_ptr()), int(accumulate), ctypes.c_void_p(stream)),
          "cet_nmse_split")
    return out


def nmse_split_sums(pred, label, sums, out=None, accumulate: bool = False, stream: Optional[int] = None):
    """Raw fp64 NMSE_Split sums of one batch into ``sums`` (float64 [2, T]: Σ(x−x̂)², Σx̂² per step), and
    optionally the ratio into ``out`` as :func:`nmse_split` does."""
    import torch

    if pred.dim() != 3 or tuple(label.shape) != tuple(pred.shape):
        raise ValueError(f"pred and label must both be [B, T, F]; got {tuple(pred.shape)} and {tuple(label.shape)}")
    for name, t in (("pred", pred), ("label", label)):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.device != pred.device or not t.is_cuda:
            raise ValueError(f"{name} must be a contiguous float32 tensor on the same HIP device")
    B, T, F = pred.shape
    if sums.dtype != torch.float64 or sums.numel() != 2 * T or sums.device != pred.device or not sums.is_contiguous():
        raise ValueError(f"sums must be a contiguous float64 tensor of {2 * T} elements on {pred.device}")
    if out is not None and (out.dtype != torch.float32 or out.numel() != T or out.device != pred.device):
        raise ValueError(f"out must be a float32 tensor of {T} elements on {pred.device}")
    if stream is None:
        stream = _stream_ptr(pred.device)
    check(lib.cet_nmse_split_sums(ctypes.c_void_p(pred.data_ptr()), ctypes.c_void_p(label.data_ptr()), B, T, F,
                                  ctypes.c_void_p(out.data_ptr()) if out is not None else None, int(accumulate),
                                  ctypes.c_void_p(sums.data_ptr()), ctypes.c_void_p(stream)), "cet_nmse_split_sums")
    return sums


def _to_numpy(v):
    if isinstance(v, np.ndarray):
        return v
    try:
        import torch

        if isinstance(v, torch.Tensor):
            return v.detach().to("cpu", torch.float32).numpy()
    except ImportError:  # pragma: no cover
        pass
    return np.asarray(v)
