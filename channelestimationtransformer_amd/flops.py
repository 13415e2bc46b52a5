"""Algorithmic work per channel sequence (the roofline numerators).

FLOPs count matmul/conv multiply-adds as 2 FLOPs, exactly the ops torch's
``FlopCounterMode`` counts on the reference forward (61.10 MFLOP for the
FullPrecision Informer C2, 88.47 MFLOP for the Transformer C3).  ProbSparse counts the
reference's own matmuls: the sampled ``Q·K_sample`` (L_Q·U·E per head), the reduced
``Q_reduce·Kᵀ`` (u·L_K·E) and ``attn·V`` (u·L_K·E) — attn.py:100, :112, :138.

HBM bytes per sequence: fp32 ``x_enc`` in + fp32 ``out``.  ``x_dec`` is read too
(the reference builds it on the host; the engine reads it as given).  Weights are read
once per launch from HBM and then hit L2/MALL, so they are not per-sequence traffic.
"""
from __future__ import annotations

import math
from typing import Sequence


def u_part(factor: int, L: int) -> int:
    return min(factor * int(math.ceil(math.log(L))), L)


def informer_flops(seq_len=90, label_len=10, pred_len=5, d_model=128, n_heads=8, e_layers: Sequence[int] = (4,),
                   d_layers=3, d_ff=64, attn="prob", factor=5, distil=True, c_in=16, c_out=16, stack=True) -> int:
    D, H = d_model, n_heads
    E = D // H
    f = 0
    f += 2 * seq_len * D * 3 * c_in                              # enc token conv
    S = 0
    for i, el in enumerate(e_layers):
        L = seq_len // (2 ** i) if stack else seq_len
        for l in range(el):
            f += 2 * L * D * D * 4                               # q, k, v, out projections
            f += 2 * L * D * d_ff * 2                            # FFN conv1 + conv2
            if attn == "prob":
                U, u = u_part(factor, L), u_part(factor, L)
                f += 2 * H * E * (L * U + u * L + u * L)
            else:
                f += 2 * H * E * (L * L + L * L)
            if distil and l < el - 1:
                f += 2 * L * D * 3 * D                           # distil conv
                L = (L - 1) // 2 + 1
        S += L
    Ld = label_len + pred_len
    f += 2 * Ld * D * 3 * c_in                                   # dec token conv
    for _ in range(d_layers):
        f += 2 * Ld * D * D * 4                                  # self q, k, v, out
        f += 2 * Ld * D * D * 2 + 2 * S * D * D * 2              # cross q, out | k, v over S rows
        f += 2 * Ld * D * d_ff * 2
        if attn == "prob":
            U, u = u_part(factor, Ld), u_part(factor, Ld)
            f += 2 * H * E * (Ld * U + u * Ld + u * Ld)
        else:
            f += 2 * H * E * (Ld * Ld * 2)
        f += 2 * H * E * (Ld * S * 2)                            # cross attention
    f += 2 * Ld * D * c_out                                      # projection (all Ld rows)
    return f


def transformer_flops(src_len=90, tgt_len=5, label_len=10, d_model=128, N=3, h=8, d_ff=64, c_in=16, c_out=16) -> int:
    D = d_model
    Ld = tgt_len + label_len
    f = 2 * src_len * D * 3 * c_in + 2 * Ld * D * 3 * c_in
    for _ in range(N):
        f += 2 * src_len * D * D * 4 + 2 * src_len * src_len * D * 2 + 2 * src_len * D * d_ff * 2
    for _ in range(N):
        f += 2 * Ld * D * D * 4 + 2 * Ld * Ld * D * 2                       # self
        f += 2 * Ld * D * D * 2 + 2 * src_len * D * D * 2 + 2 * Ld * src_len * D * 2   # cross
        f += 2 * Ld * D * d_ff * 2
    f += 2 * Ld * D * c_out
    return f


def io_bytes(seq_len=90, label_len=10, pred_len=5, c_in=16, c_out=16) -> int:
    """HBM bytes per sequence touched by one forward: x_enc + x_dec in, out written (fp32)."""
    return 4 * (seq_len * c_in + (label_len + pred_len) * c_in + pred_len * c_out)
