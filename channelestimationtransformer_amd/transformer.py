"""Drop-in ``Transformer`` / ``build_transformer`` (models/Transformer/model.py:13-174) on the engine.

``build_transformer(src_vocab, tgt_vocab, src_seq_len, tgt_seq_len, label_len, d_model=512,
N=8, h=8, dropout=0.1, d_ff=2048)`` and ``Transformer.forward(encoder_input, decoder_input)``
keep the reference's signatures and return value (a single tensor ``[B, tgt_seq_len, tgt_vocab]``,
``model.py:76-87``); the state_dict keys follow :func:`.spec.transformer_spec`.
"""
from __future__ import annotations

import torch

from . import spec as S
from ._lib import TransformerConfig
from .engine import Engine
from .informer import _EngineModule, build_param_tree
from .weights import synthetic_state_dict


class Transformer(_EngineModule):
    def __init__(self, src_vocab, tgt_vocab, src_seq_len, tgt_seq_len, label_len, d_model, N, h, d_ff):
        super().__init__()
        self.src_vocab, self.tgt_vocab = src_vocab, tgt_vocab
        self.src_seq_len, self.tgt_seq_len, self.label_len = src_seq_len, tgt_seq_len, label_len
        self.d_model, self.N, self.h, self.d_ff = d_model, N, h, d_ff
        self.pred_len = tgt_seq_len
        self.c_out = tgt_vocab
        entries = S.transformer_spec(src_vocab, tgt_vocab, src_seq_len, tgt_seq_len, label_len, d_model, N, h, d_ff)
        build_param_tree(self, entries, synthetic_state_dict(entries, seed=int(torch.initial_seed()) % (2 ** 32)))

    def config(self) -> TransformerConfig:
        c = TransformerConfig()
        c.src_vocab, c.tgt_vocab = self.src_vocab, self.tgt_vocab
        c.src_seq_len, c.tgt_seq_len, c.label_len = self.src_seq_len, self.tgt_seq_len, self.label_len
        c.d_model, c.N, c.h, c.d_ff = self.d_model, self.N, self.h, self.d_ff
        return c

    def _make_engine(self) -> Engine:
        return Engine.transformer(self.config())

    def forward(self, encoder_input, decoder_input):
        if self.training:
            raise RuntimeError("inference-only engine: call .eval() first")
        dev = encoder_input.device if encoder_input.is_cuda else torch.device("cuda", torch.cuda.current_device())
        eng = self.engine(dev)
        xe = encoder_input.to(dev, torch.float32).contiguous()
        xd = decoder_input.to(dev, torch.float32).contiguous()
        out = torch.empty(xe.shape[0], self.tgt_seq_len, self.tgt_vocab, device=dev, dtype=torch.float32)
        eng.forward(xe, xd, out)
        return out


def build_transformer(src_vocab_size: int, tgt_vocab_size: int, src_seq_len: int, tgt_seq_len: int,
                      label_len: int, d_model: int = 512, N: int = 8, h: int = 8, dropout: float = 0.1,
                      d_ff: int = 2048) -> Transformer:
    """models/Transformer/model.py:90-174 (dropout is inference-irrelevant and ignored)."""
    return Transformer(src_vocab_size, tgt_vocab_size, src_seq_len, tgt_seq_len, label_len, d_model, N, h, d_ff)
