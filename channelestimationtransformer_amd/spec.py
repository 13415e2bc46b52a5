"""State-dict schemas of the reference models.

The engine accepts reference checkpoints unchanged, so every model here exposes
exactly the reference's ``state_dict`` key names and shapes.  The schemas are
generated from the constructor arguments (no reference code is imported):

* ``InformerStack`` — ``FullPrecision/InformerModel/model.py:142-271`` with the
  sub-module naming of ``encoder.py:6-106``, ``decoder.py:6-56``,
  ``attn.py:178-209`` and ``embed.py:8-135``.
* ``Informer`` (single encoder) — ``FullPrecision/InformerModel/model.py:11-139``.
* ``InformerStack`` LSQ variant — ``models/InformerLSQ/model.py`` with
  ``LSQ.py:23-74,247-314`` (one extra ``step_size`` scalar per quantized module).
* ``Transformer`` — ``models/Transformer/model.py:90-174`` and the blocks of
  ``buildingblocks.py``, ``encoder.py``, ``decoder.py``, ``embed.py``.

Each entry is ``(key, shape, kind)`` where ``kind`` drives the synthetic
initialiser in :mod:`.weights` (``linear_w``, ``bias``, ``ln_w``, ``ln_b``,
``bn_w``, ``bn_b``, ``bn_rm``, ``bn_rv``, ``bn_nbt``, ``pe``, ``fixed_emb``,
``step``).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

Entry = Tuple[str, Tuple[int, ...], str]

# temporal tables of embed.py:130-159 (FixedEmbedding, embed="fixed")
_TEMPORAL = (("hour_embed", 24), ("weekday_embed", 7), ("day_embed", 32), ("month_embed", 13))


def _data_embedding(prefix: str, c_in: int, d_model: int, embed: str, freq: str,
                    pe_len: int = 5000) -> List[Entry]:
    """DataEmbedding (embed.py:118-135): token conv + positional buffer + temporal tables."""
    out: List[Entry] = [
        (f"{prefix}.value_embedding.tokenConv.weight", (d_model, c_in, 3), "linear_w"),
        (f"{prefix}.value_embedding.tokenConv.bias", (d_model,), "bias"),
        (f"{prefix}.position_embedding.pe", (1, pe_len, d_model), "pe"),
    ]
    if embed == "timeF":
        d_inp = {"h": 4, "t": 5, "s": 6, "m": 1, "a": 1, "w": 2, "d": 3, "b": 3}[freq]
        out += [(f"{prefix}.temporal_embedding.embed.weight", (d_model, d_inp), "linear_w"),
                (f"{prefix}.temporal_embedding.embed.bias", (d_model,), "bias")]
        return out
    kind = "fixed_emb" if embed == "fixed" else "linear_w"
    tables = list(_TEMPORAL)
    if freq == "t":
        tables = [("minute_embed", 4)] + tables
    for name, n in tables:
        sub = "emb.weight" if embed == "fixed" else "weight"
        out.append((f"{prefix}.temporal_embedding.{name}.{sub}", (n, d_model), kind))
    return out


def _attention_layer(prefix: str, d_model: int, n_heads: int, lsq: bool) -> List[Entry]:
    """AttentionLayer (attn.py:178-193): q/k/v/out projections with bias."""
    dk = d_model // n_heads
    out: List[Entry] = []
    for name, (o, i) in (("query_projection", (dk * n_heads, d_model)),
                         ("key_projection", (dk * n_heads, d_model)),
                         ("value_projection", (dk * n_heads, d_model)),
                         ("out_projection", (d_model, dk * n_heads))):
        out.append((f"{prefix}.{name}.weight", (o, i), "linear_w"))
        out.append((f"{prefix}.{name}.bias", (o,), "bias"))
        if lsq:
            out.append((f"{prefix}.{name}.step_size", (), "step"))
    return out


def _ffn(prefix: str, d_model: int, d_ff: int, lsq: bool) -> List[Entry]:
    out: List[Entry] = []
    for name, (o, i) in (("conv1", (d_ff, d_model)), ("conv2", (d_model, d_ff))):
        out.append((f"{prefix}.{name}.weight", (o, i, 1), "linear_w"))
        out.append((f"{prefix}.{name}.bias", (o,), "bias"))
        if lsq:
            out.append((f"{prefix}.{name}.step_size", (), "step"))
    return out


def _ln(prefix: str, d_model: int) -> List[Entry]:
    return [(f"{prefix}.weight", (d_model,), "ln_w"), (f"{prefix}.bias", (d_model,), "ln_b")]


def _encoder(prefix: str, n_layers: int, d_model: int, n_heads: int, d_ff: int,
             distil: bool, lsq: bool) -> List[Entry]:
    """Encoder (encoder.py:59-86) of EncoderLayer (:31-56) and ConvLayer (:6-28)."""
    out: List[Entry] = []
    for l in range(n_layers):
        p = f"{prefix}.attn_layers.{l}"
        out += _attention_layer(f"{p}.attention", d_model, n_heads, lsq)
        out += _ffn(p, d_model, d_ff, lsq)
        out += _ln(f"{p}.norm1", d_model) + _ln(f"{p}.norm2", d_model)
    if distil:
        for l in range(n_layers - 1):
            p = f"{prefix}.conv_layers.{l}"
            out.append((f"{p}.downConv.weight", (d_model, d_model, 3), "linear_w"))
            out.append((f"{p}.downConv.bias", (d_model,), "bias"))
            if lsq:
                out.append((f"{p}.downConv.step_size", (), "step"))
            out += [(f"{p}.norm.weight", (d_model,), "bn_w"), (f"{p}.norm.bias", (d_model,), "bn_b"),
                    (f"{p}.norm.running_mean", (d_model,), "bn_rm"),
                    (f"{p}.norm.running_var", (d_model,), "bn_rv"),
                    (f"{p}.norm.num_batches_tracked", (), "bn_nbt")]
    out += _ln(f"{prefix}.norm", d_model)
    return out


def _decoder(n_layers: int, d_model: int, n_heads: int, d_ff: int, lsq: bool) -> List[Entry]:
    """Decoder (decoder.py:43-56) of DecoderLayer (:6-40)."""
    out: List[Entry] = []
    for l in range(n_layers):
        p = f"decoder.layers.{l}"
        out += _attention_layer(f"{p}.self_attention", d_model, n_heads, lsq)
        out += _attention_layer(f"{p}.cross_attention", d_model, n_heads, lsq)
        out += _ffn(p, d_model, d_ff, lsq)
        out += _ln(f"{p}.norm1", d_model) + _ln(f"{p}.norm2", d_model) + _ln(f"{p}.norm3", d_model)
    out += _ln("decoder.norm", d_model)
    return out


def informer_stack_spec(enc_in: int, dec_in: int, c_out: int, d_model: int, n_heads: int,
                        e_layers: Sequence[int], d_layers: int, d_ff: int, embed: str = "fixed",
                        freq: str = "h", distil: bool = True, lsq: bool = False) -> List[Entry]:
    """Schema of ``InformerStack`` (model.py:142-245)."""
    out = _data_embedding("enc_embedding", enc_in, d_model, embed, freq)
    out += _data_embedding("dec_embedding", dec_in, d_model, embed, freq)
    for i, el in enumerate(e_layers):
        out += _encoder(f"encoder.encoders.{i}", el, d_model, n_heads, d_ff, distil, lsq)
    out += _decoder(d_layers, d_model, n_heads, d_ff, lsq)
    out += [("projection.weight", (c_out, d_model), "linear_w"), ("projection.bias", (c_out,), "bias")]
    return out


def informer_spec(enc_in: int, dec_in: int, c_out: int, d_model: int, n_heads: int,
                  e_layers: int, d_layers: int, d_ff: int, embed: str = "fixed", freq: str = "h",
                  distil: bool = True) -> List[Entry]:
    """Schema of the single-encoder ``Informer`` (model.py:11-113)."""
    out = _data_embedding("enc_embedding", enc_in, d_model, embed, freq)
    out += _data_embedding("dec_embedding", dec_in, d_model, embed, freq)
    out += _encoder("encoder", e_layers, d_model, n_heads, d_ff, distil, False)
    out += _decoder(d_layers, d_model, n_heads, d_ff, False)
    out += [("projection.weight", (c_out, d_model), "linear_w"), ("projection.bias", (c_out,), "bias")]
    return out


def transformer_spec(src_vocab: int, tgt_vocab: int, src_seq_len: int, tgt_seq_len: int,
                     label_len: int, d_model: int, N: int, h: int, d_ff: int) -> List[Entry]:
    """Schema of ``build_transformer`` (models/Transformer/model.py:90-174)."""
    out: List[Entry] = []

    def mha(p):
        return [(f"{p}.w_{n}.weight", (d_model, d_model), "linear_w") for n in "qkvo"]

    def ff(p):
        return [(f"{p}.linear_1.weight", (d_ff, d_model), "linear_w"), (f"{p}.linear_1.bias", (d_ff,), "bias"),
                (f"{p}.linear_2.weight", (d_model, d_ff), "linear_w"), (f"{p}.linear_2.bias", (d_model,), "bias")]

    def lnt(p):
        return [(f"{p}.alpha", (d_model,), "ln_w"), (f"{p}.bias", (d_model,), "ln_b")]

    for l in range(N):
        p = f"encoder.layers.{l}"
        out += mha(f"{p}.self_attention_block") + ff(f"{p}.feed_forward_block")
        for r in range(2):
            out += lnt(f"{p}.residual_connections.{r}.norm")
    out += lnt("encoder.norm")
    for l in range(N):
        p = f"decoder.layers.{l}"
        out += mha(f"{p}.self_attention_block") + mha(f"{p}.cross_attention_block")
        out += ff(f"{p}.feed_forward_block")
        for r in range(3):
            out += lnt(f"{p}.residual_connections.{r}.norm")
    out += lnt("decoder.norm")
    out += [("src_embed.tokenEmbedding.weight", (d_model, src_vocab, 3), "linear_w"),
            ("src_embed.tokenEmbedding.bias", (d_model,), "bias"),
            ("tgt_embed.tokenEmbedding.weight", (d_model, tgt_vocab, 3), "linear_w"),
            ("tgt_embed.tokenEmbedding.bias", (d_model,), "bias"),
            ("src_pos.pe", (1, src_seq_len, d_model), "pe"),
            ("tgt_pos.pe", (1, tgt_seq_len + label_len, d_model), "pe"),
            ("projection_layer.proj.weight", (tgt_vocab, d_model), "linear_w"),
            ("projection_layer.proj.bias", (tgt_vocab,), "bias")]
    return out
