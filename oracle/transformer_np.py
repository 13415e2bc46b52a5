"""CPU ORACLE (test infrastructure only) — numpy restatement of the reference's
``models/Transformer`` inference forward.  Only tests / smoke / bench's
cpu_baseline import it; the product path never does.  Pinned by
``tests/golden/transformer_c3.npz`` (generated from the reference itself).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np

from .informer_np import conv1d_circular3, softmax


def layer_norm_unbiased(x, alpha, bias, eps=1e-6):
    """LayerNormalization (buildingblocks.py:23-30): ``alpha·(x-mean)/(std+eps)+bias``, unbiased std."""
    mu = x.mean(-1, keepdims=True)
    std = x.std(-1, ddof=1, keepdims=True)
    return alpha * (x - mu) / (std + eps) + bias


@dataclass
class TransformerConfig:
    src_vocab: int = 16
    tgt_vocab: int = 16
    src_seq_len: int = 90
    tgt_seq_len: int = 5      # = pred_len (model.py:169: Transformer(..., tgt_seq_len))
    label_len: int = 10
    d_model: int = 128
    N: int = 3
    h: int = 8
    d_ff: int = 64


class TransformerOracle:
    """Transformer.forward (models/Transformer/model.py:76-87)."""

    def __init__(self, cfg: TransformerConfig, state: Dict[str, np.ndarray], dtype=np.float64):
        self.cfg = cfg
        self.dt = dtype
        self.p = {k: np.asarray(v, np.float32).astype(dtype) for k, v in state.items()}

    def ln(self, prefix, x):
        return layer_norm_unbiased(x, self.p[f"{prefix}.alpha"], self.p[f"{prefix}.bias"])

    def mha(self, prefix, q, k, v):
        """MultiHeadAttentionBlock.forward (buildingblocks.py:152-192), mask=None."""
        p, h = self.p, self.cfg.h
        B, L, D = q.shape
        S = k.shape[1]
        dk = D // h
        Q = (q @ p[f"{prefix}.w_q.weight"].T).reshape(B, L, h, dk).transpose(0, 2, 1, 3)
        K = (k @ p[f"{prefix}.w_k.weight"].T).reshape(B, S, h, dk).transpose(0, 2, 1, 3)
        V = (v @ p[f"{prefix}.w_v.weight"].T).reshape(B, S, h, dk).transpose(0, 2, 1, 3)
        A = softmax(Q @ K.transpose(0, 1, 3, 2) / np.sqrt(dk), -1)
        x = (A @ V).transpose(0, 2, 1, 3).reshape(B, L, D)
        return x @ p[f"{prefix}.w_o.weight"].T

    def ffn(self, prefix, x):
        """FeedForwardBlock (buildingblocks.py:54-65): linear_2(relu(linear_1(x)))."""
        p = self.p
        y = np.maximum(x @ p[f"{prefix}.linear_1.weight"].T + p[f"{prefix}.linear_1.bias"], 0)
        return y @ p[f"{prefix}.linear_2.weight"].T + p[f"{prefix}.linear_2.bias"]

    def forward(self, enc_in, dec_in, acts: Optional[dict] = None):
        cfg, p = self.cfg, self.p
        acts = {} if acts is None else acts
        # encode (model.py:27-30): InputEmbeddings (embed.py:98-103) + PositionalEncoding (:50-54)
        x = conv1d_circular3(np.asarray(enc_in, self.dt), p["src_embed.tokenEmbedding.weight"],
                             p["src_embed.tokenEmbedding.bias"])
        x = x + p["src_pos.pe"][0, : x.shape[1]]
        acts["enc_emb"] = x
        for l in range(cfg.N):   # EncoderBlock (encoder.py:41-46), pre-LN residuals (buildingblocks.py:214-226)
            pre = f"encoder.layers.{l}"
            n0 = self.ln(f"{pre}.residual_connections.0.norm", x)
            x = x + self.mha(f"{pre}.self_attention_block", n0, n0, n0)
            x = x + self.ffn(f"{pre}.feed_forward_block", self.ln(f"{pre}.residual_connections.1.norm", x))
            acts[f"enc_layer{l}"] = x
        enc = self.ln("encoder.norm", x)
        acts["enc_out"] = enc
        # decode (model.py:32-41)
        y = conv1d_circular3(np.asarray(dec_in, self.dt), p["tgt_embed.tokenEmbedding.weight"],
                             p["tgt_embed.tokenEmbedding.bias"])
        y = y + p["tgt_pos.pe"][0, : y.shape[1]]
        acts["dec_emb"] = y
        for l in range(cfg.N):   # DecoderBlock (decoder.py:48-72), tgt_mask = src_mask = None
            pre = f"decoder.layers.{l}"
            n0 = self.ln(f"{pre}.residual_connections.0.norm", y)
            y = y + self.mha(f"{pre}.self_attention_block", n0, n0, n0)
            n1 = self.ln(f"{pre}.residual_connections.1.norm", y)
            y = y + self.mha(f"{pre}.cross_attention_block", n1, enc, enc)
            y = y + self.ffn(f"{pre}.feed_forward_block", self.ln(f"{pre}.residual_connections.2.norm", y))
            acts[f"dec_layer{l}"] = y
        y = self.ln("decoder.norm", y)
        acts["dec_out"] = y
        out = y @ p["projection_layer.proj.weight"].T + p["projection_layer.proj.bias"]
        acts["proj"] = out
        return out[:, -cfg.tgt_seq_len:]
