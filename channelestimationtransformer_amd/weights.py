"""Synthetic (seeded) weights and the reference's fixed sinusoid tables.

There is no trained checkpoint for the north-star config, so benchmarks, tests
and golden fixtures all use one deterministic recipe: walk a schema from
:mod:`.spec` in order and draw every tensor from ``numpy.random.default_rng(seed)``.
Linear/conv weights and biases are uniform in ``±1/sqrt(fan_in)`` (the torch
default scale), norms are ``1 + 0.1·N(0,1)`` / ``0.1·N(0,1)``, BatchNorm running
statistics are randomised so the eval-mode fold is exercised.  Positional
tables follow ``embed.py:8-27`` (Informer) / ``models/Transformer/embed.py:8-54``.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, Tuple

import numpy as np

from .spec import Entry


def sinusoid_table(n_pos: int, d_model: int) -> np.ndarray:
    """``pe[p, 2i] = sin(p·w_i)``, ``pe[p, 2i+1] = cos(p·w_i)``, ``w_i = exp(-2i·ln(1e4)/d)``.

    Computed in float32 with torch, in the same operation order as the reference
    (``embed.py:12-24``), so a freshly built reference module and this table agree.
    """
    import torch

    pe = torch.zeros(n_pos, d_model).float()
    position = torch.arange(0, n_pos).float().unsqueeze(1)
    div_term = (torch.arange(0, d_model, 2).float() * -(math.log(10000.0) / d_model)).exp()
    pe[:, 0::2] = torch.sin(position * div_term)
    pe[:, 1::2] = torch.cos(position * div_term)
    return pe.numpy()


def _fan_in(shape: Tuple[int, ...]) -> int:
    return int(np.prod(shape[1:])) if len(shape) > 1 else int(shape[0])


def synthetic_state_dict(spec: Iterable[Entry], seed: int = 0, lsq_bits: int = 8) -> Dict[str, np.ndarray]:
    """Deterministic state dict for ``spec`` (numpy arrays, float32 / int64); LSQ step sizes (if the
    schema has them) are the ``lsq_bits`` initialisation of LSQ.py:54-58."""
    spec = list(spec)
    shapes = {k: s for k, s, _ in spec}
    rng = np.random.default_rng(seed)
    out: Dict[str, np.ndarray] = {}
    for key, shape, kind in spec:
        if kind == "linear_w":
            b = 1.0 / math.sqrt(_fan_in(shape))
            v = rng.uniform(-b, b, size=shape)
        elif kind == "bias":
            wshape = shapes.get(key[: -len("bias")] + "weight", shape)
            b = 1.0 / math.sqrt(_fan_in(wshape))
            v = rng.uniform(-b, b, size=shape)
        elif kind in ("ln_w", "bn_w"):
            v = 1.0 + 0.1 * rng.standard_normal(shape)
        elif kind in ("ln_b", "bn_b", "bn_rm"):
            v = 0.1 * rng.standard_normal(shape)
        elif kind == "bn_rv":
            v = rng.uniform(0.5, 1.5, size=shape)
        elif kind == "bn_nbt":
            out[key] = np.zeros(shape, dtype=np.int64)
            continue
        elif kind == "pe":
            v = sinusoid_table(shape[1], shape[2])[None]
        elif kind == "fixed_emb":
            v = sinusoid_table(shape[0], shape[1])
        elif kind == "step":
            # filled by lsq_step_sizes() once the weights exist (LSQ.py:54-58)
            continue
        else:  # pragma: no cover - schema bug
            raise ValueError(f"unknown kind {kind} for {key}")
        out[key] = np.ascontiguousarray(v, dtype=np.float32)
    steps = [k for k, _, kind in spec if kind == "step"]
    if steps:
        out.update(lsq_step_sizes(out, steps, nbits=lsq_bits))
    return out


def lsq_step_sizes(state: Dict[str, np.ndarray], step_keys: Iterable[str], nbits: int) -> Dict[str, np.ndarray]:
    """LSQ initial step ``s = mean|w| / sqrt(Qp)``, ``Qp = 2^(b-1)-1`` (``LSQ.py:54-58,214-218``)."""
    import torch

    qp = 2 ** (nbits - 1) - 1
    res = {}
    for k in step_keys:
        w = torch.from_numpy(state[k[: -len("step_size")] + "weight"])
        res[k] = (w.abs().mean() / math.sqrt(qp)).numpy().astype(np.float32)
    return res
